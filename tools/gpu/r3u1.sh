# K2 unit-pair profile words (k_score16f<32, true, true>): parity with the unit
# kernel forced everywhere, then a same-box A/B against the 16-bit rows (swar16)
# on cfg4 with the full-output pin, then a kernel trace of the default.
export TMPDIR=/tmp
mkdir -p gpurun_out/r3u1
R=$GRAFT_REPO_ROOT
GHOSTM_K2=unit timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r3u1/parity_unit.log 2>&1
rc=$?
echo "parity rc=$rc"
tail -3 gpurun_out/r3u1/parity_unit.log
[ $rc -eq 0 ] || exit $rc
mkdir -p /tmp/ghostm_ab_data
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --workdir /tmp/ghostm_ab_data \
    > gpurun_out/r3u1/unit$i.log 2>&1 || exit $?
  GHOSTM_K2=swar16 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e \
    --workdir /tmp/ghostm_ab_data > gpurun_out/r3u1/swar16_$i.log 2>&1 || exit $?
done
python3 - gpurun_out/r3u1 <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.log"))):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            st = {k: round(v * 1e3, 1) for k, v in d["stages_s_per_step"].items()}
            print(os.path.basename(f), round(d["ms_per_step"], 1), st, d.get("full_output_matches_reference"))
PY
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3u1/prof -o run -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --workdir /tmp/ghostm_ab_data \
  > $R/gpurun_out/r3u1/prof.log 2>&1 || exit $?
head -6 $R/gpurun_out/r3u1/prof/run_kernel_stats.csv | cut -c1-160
