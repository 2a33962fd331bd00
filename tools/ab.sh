#!/bin/bash
# Same-box A/B timing: bench.py with the current library (A) and with each
# alternate build ab_libs/libghostm_hip_<tag>.so (tools/altlib.sh) given as arguments
# (default: prev), alternating, N rounds (AB_ROUNDS, default 2). AB_ARGS adds
# bench options (e.g. "--queries 125000"). The data set is generated once.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${AB_ROUNDS:-2}
TAGS=${*:-prev}
ARGS="--steps ${AB_STEPS:-3} --warmup 1 --no-cpu --no-e2e --workdir /tmp/ghostm_ab_data ${AB_ARGS:-}"
mkdir -p "$R/gpurun_out/ab" /tmp/ghostm_ab_data
for i in $(seq 1 "$N"); do
  timeout -k 10 200 python3 "$R/bench.py" $ARGS > "$R/gpurun_out/ab/A$i.log" 2>&1
  for t in $TAGS; do
    GHOSTM_LIB_PATH="$R/ab_libs/libghostm_hip_$t.so" \
      timeout -k 10 200 python3 "$R/bench.py" $ARGS > "$R/gpurun_out/ab/${t}$i.log" 2>&1
  done
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
