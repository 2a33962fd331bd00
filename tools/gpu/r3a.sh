# shard parity tests, then a 2-rank rehearsal of the N > 1 bench path (gloo, one GPU)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_shards.py -v --timeout 300 --timeout-method thread > gpurun_out/r3a_shards.log 2>&1
rc=$?
echo "pytest rc=$rc"
# 0 = passed, 1 = test failures: the GPU is fine; anything else (fault, abort, timeout) ends here
[ $rc -le 1 ] || exit $rc
GHOSTM_BENCH_BACKEND=gloo GHOSTM_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --queries 40000 --steps 3 --warmup 1 \
  --no-cpu > gpurun_out/r3a_bench2.json 2> gpurun_out/r3a_bench2.log
echo "bench rc=$?"
