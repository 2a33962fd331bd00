# K2 stream at low priority, K4/K3 stream at high priority (A), the plain second stream (v1), one stream (prev)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -k "not full" -x -q --timeout 300 --timeout-method thread > gpurun_out/r3v_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=2 bash tools/ab.sh prev v1 > gpurun_out/r3v_ab.log 2>&1
echo "ab rc=$?"
cat gpurun_out/r3v_ab.log
