# K2 unit kernel: END columns through the E floor (no H mask) vs the previous
# commit (prev lib) vs the 16-bit rows (swar16), same box, cfg4 with the pin.
export TMPDIR=/tmp
mkdir -p gpurun_out/r3u4 /tmp/ghostm_ab_data
R=$GRAFT_REPO_ROOT
GHOSTM_K2=unit timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r3u4/parity_unit.log 2>&1
rc=$?
echo "parity rc=$rc"; tail -2 gpurun_out/r3u4/parity_unit.log
[ $rc -eq 0 ] || exit $rc
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --workdir /tmp/ghostm_ab_data"
for i in 1 2; do
  timeout -k 10 300 $B > gpurun_out/r3u4/pf$i.log 2>&1 || exit $?
  GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_prev.so timeout -k 10 300 $B > gpurun_out/r3u4/prev$i.log 2>&1 || exit $?
  GHOSTM_K2=swar16 timeout -k 10 300 $B > gpurun_out/r3u4/swar16_$i.log 2>&1 || exit $?
done
python3 - gpurun_out/r3u4 <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.log"))):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            st = {k: round(v * 1e3, 1) for k, v in d["stages_s_per_step"].items()}
            print(os.path.basename(f), round(d["ms_per_step"], 1), st, d.get("full_output_matches_reference"))
PY
