#!/bin/bash
# Same-box A/B timing: bench.py with the current library (A) and with
# ghostm_amd/lib/libghostm_hip_prev.so (B), alternating, N rounds each.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${1:-2}
mkdir -p "$R/gpurun_out/ab"
for i in $(seq 1 "$N"); do
  timeout -k 10 200 python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/ab/A$i.log" 2>&1
  GHOSTM_LIB_PATH="$R/ghostm_amd/lib/libghostm_hip_prev.so" \
    timeout -k 10 200 python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/ab/B$i.log" 2>&1
done
