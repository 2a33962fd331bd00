#!/bin/bash
# Host-pipeline A/B on one box: bench.py with GHOSTM_TRACE=1 (host timeline per
# run on stderr) once per configuration. HS_CFGS = "name:ENV=v ENV2=v;name2:..."
# (a name with no settings runs the defaults); HS_ARGS adds bench options.
set -euo pipefail
mkdir -p gpurun_out/hs /tmp/hsd
IFS=';' read -ra LIST <<< "${HS_CFGS:-default:}"
for cfg in "${LIST[@]}"; do
  name=${cfg%%:*}
  envs=${cfg#*:}
  env $envs GHOSTM_TRACE=1 timeout -k 10 200 python3 bench.py --steps ${HS_STEPS:-3} --warmup 1 --no-cpu \
    --no-e2e --workdir /tmp/hsd ${HS_ARGS:-} > gpurun_out/hs/$name.json 2> gpurun_out/hs/$name.err
done
python3 - <<'PY'
import glob, json, os
for f in sorted(glob.glob("gpurun_out/hs/*.json")):
    try:
        d = json.load(open(f))
    except Exception:
        continue
    st = {k: round(v * 1e3, 1) for k, v in d["stages_s_per_step"].items()}
    print(os.path.basename(f), round(d["ms_per_step"], 1), st, d.get("full_output_matches_reference"))
PY
