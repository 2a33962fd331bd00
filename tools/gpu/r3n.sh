# k_finalize over slot-indexed data: merge/K3 parity tests, then A/B (A = this build, prev = before)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -v --timeout 300 --timeout-method thread > gpurun_out/r3n_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
AB_ROUNDS=3 timeout -k 10 900 bash tools/ab.sh prev > gpurun_out/r3n_ab.txt 2>&1
echo "ab rc=$?"
