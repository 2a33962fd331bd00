# K3 key DP by strip class: parity (every golden variant, forced kinds incl.
# k3_nostrips, scale pins), then same-box A/B strips on vs GHOSTM_K3_STRIPS=0 on cfg4
export TMPDIR=/tmp
O=gpurun_out/r3s1
mkdir -p $O /tmp/ghostm_ab_data
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_shards.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --workdir /tmp/ghostm_ab_data"
for i in 1 2 3; do
  timeout -k 10 300 $B > $O/strips$i.log 2>&1 || exit $?
  GHOSTM_K3_STRIPS=0 timeout -k 10 300 $B > $O/nostrips$i.log 2>&1 || exit $?
done
python3 - $O <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.log"))):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            st = {k: round(v * 1e3, 1) for k, v in d["stages_s_per_step"].items() if k in ("total", "traceback_device", "score_device")}
            print(os.path.basename(f), round(d["ms_per_step"], 1), st, d.get("full_output_matches_reference"))
PY
