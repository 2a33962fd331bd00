# K3 key DP: the residue loaded one column ahead: parity, then A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_shards.py -q --timeout 300 --timeout-method thread > gpurun_out/r3zb_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=2 bash tools/ab.sh prev > gpurun_out/r3zb_ab.log 2>&1
echo "ab rc=$?"
cat gpurun_out/r3zb_ab.log
