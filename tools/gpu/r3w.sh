# K1 gather: every lane loads its list predecessor (no lane-0 branch, no DPP): parity, then A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -v -k "not full_workload" --timeout 300 --timeout-method thread > gpurun_out/r3w_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=2 bash tools/ab.sh prev > gpurun_out/r3w_ab.log 2>&1
echo "ab rc=$?"
cat gpurun_out/r3w_ab.log
