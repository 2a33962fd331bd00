# K1 filter: LDS zeroing with 16-byte stores vs the previous commit (prev lib):
# K1 tests, then same-box A/B on cfg4 with the pin
export TMPDIR=/tmp
O=gpurun_out/r3k1c
mkdir -p $O /tmp/ghostm_ab_data
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "not unit_k2" > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --workdir /tmp/ghostm_ab_data"
for i in 1 2 3; do
  timeout -k 10 300 $B > $O/new$i.log 2>&1 || exit $?
  GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_prev.so timeout -k 10 300 $B > $O/prev$i.log 2>&1 || exit $?
done
python3 - $O <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.log"))):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            st = {k: round(v * 1e3, 1) for k, v in d["stages_s_per_step"].items() if k in ("total", "seed_device", "score_device")}
            print(os.path.basename(f), round(d["ms_per_step"], 1), st, d.get("full_output_matches_reference"))
PY
