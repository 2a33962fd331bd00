# persistent host worker pool for ParallelFor: parity, then A/B at the 125 K-query shard size and at cfg4
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3x_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=3 AB_STEPS=10 AB_ARGS="--queries 125000" bash tools/ab.sh prev > gpurun_out/r3x_ab125k.log 2>&1 || exit $?
mkdir -p gpurun_out/ab125k && mv gpurun_out/ab/*.log gpurun_out/ab125k/
AB_ROUNDS=2 bash tools/ab.sh prev > gpurun_out/r3x_ab.log 2>&1
echo "ab rc=$?"
cat gpurun_out/r3x_ab125k.log gpurun_out/r3x_ab.log
