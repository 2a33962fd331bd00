#!/bin/bash
# Profile the bench workload on one MI355X (run through gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats of bench.py itself (per-kernel durations)
#   2. --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (HBM traffic)
#   3. --pmc SQ issue counters (VALU busy / wait breakdown)
# then summarises into profiles/<round>_* via tools/pmc_summary.py.
#   tools/profile.sh <round> [preset]   (preset: a bench.py --preset, default cfg4)
# Each step has its own time limit and the chain stops at the first failure.
set -euo pipefail
ROUND=${1:-r1}
PRESET=${2:-cfg4}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$ROUND
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --preset $PRESET --steps 2 --warmup 1 --no-cpu --no-e2e --workdir /tmp/ghostm_prof_data"
ONE="$R/bench.py --preset $PRESET --steps 1 --warmup 0 --no-cpu --no-e2e --workdir /tmp/ghostm_prof_data"
mkdir -p /tmp/ghostm_prof_data

timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 $BENCH > "$OUT/bench_trace.log" 2>&1
echo "trace done"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
  -- python3 $ONE > "$OUT/bench_fetch.log" 2>&1
echo "fetch done"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run \
  -- python3 $ONE > "$OUT/bench_write.log" 2>&1
echo "write done"
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/sq" -o run \
  -- python3 $ONE > "$OUT/bench_sq.log" 2>&1
echo "sq done"
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/lds" -o run \
  -- python3 $ONE > "$OUT/bench_lds.log" 2>&1
echo "lds done"
NQ=$(python3 -c "import sys; sys.path.insert(0, '$R'); from ghostm_amd.workloads import WORKLOADS; print(WORKLOADS['$PRESET']['queries'])")
python3 "$R/tools/pmc_summary.py" --round "$ROUND" --prof "$OUT" --queries "$NQ" --preset "$PRESET"
cp "$R/profiles/${ROUND}_pmc.json" "$R/profiles/pmc_traffic_${PRESET}.json" "$OUT/" 2>/dev/null || true
