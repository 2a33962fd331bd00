#!/bin/bash
# Same-box A/B timing: bench.py with the current library (A) and with each
# alternate build ghostm_amd/lib/libghostm_hip_<tag>.so given as arguments
# (default: prev), alternating, N rounds (AB_ROUNDS, default 2).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${AB_ROUNDS:-2}
TAGS=${*:-prev}
mkdir -p "$R/gpurun_out/ab"
for i in $(seq 1 "$N"); do
  timeout -k 10 200 python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/ab/A$i.log" 2>&1
  for t in $TAGS; do
    GHOSTM_LIB_PATH="$R/ghostm_amd/lib/libghostm_hip_$t.so" \
      timeout -k 10 200 python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/ab/${t}$i.log" 2>&1
  done
done
