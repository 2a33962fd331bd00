# new shard edge tests, then the 125k-query shard traces (host timeline + kernel trace)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_shards.py -v -k "rank_local" --timeout 300 --timeout-method thread > gpurun_out/r3k_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
bash tools/gpu/r3j.sh
