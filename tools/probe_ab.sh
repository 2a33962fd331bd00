#!/bin/bash
# Same-box timing of bench.py with the current library (A) and a probe build
# (ghostm_amd/lib/libghostm_hip_<tag>.so) whose output is allowed to differ
# (timing probes of an instruction mix): exit status 1 (output mismatch) is
# accepted for the probe, anything else stops the script.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-probe}
N=${AB_ROUNDS:-2}
ARGS="--steps ${AB_STEPS:-3} --warmup 1 --no-cpu --no-e2e --workdir /tmp/ghostm_ab_data ${AB_ARGS:-}"
mkdir -p "$R/gpurun_out/ab" /tmp/ghostm_ab_data
for i in $(seq 1 "$N"); do
  timeout -k 10 200 python3 "$R/bench.py" $ARGS > "$R/gpurun_out/ab/A$i.log" 2>&1 || exit $?
  GHOSTM_LIB_PATH="$R/ghostm_amd/lib/libghostm_hip_$T.so" \
    timeout -k 10 200 python3 "$R/bench.py" $ARGS > "$R/gpurun_out/ab/${T}$i.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
python3 - "$R/gpurun_out/ab" <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.log"))):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            st = {k: round(v * 1e3, 1) for k, v in d["stages_s_per_step"].items()}
            print(os.path.basename(f), round(d["ms_per_step"], 1), st, d.get("full_output_matches_reference"))
PY
