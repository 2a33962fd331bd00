# 8-rank rehearsal of the driver N = 8 bench at full size with the unit K2 kernel (1 M cfg4 queries, gloo, every rank on GPU 0)
export TMPDIR=/tmp
mkdir -p gpurun_out
GHOSTM_BENCH_BACKEND=gloo GHOSTM_BENCH_DEVICE=0 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29513 bench.py --steps 3 --warmup 1 \
  > gpurun_out/r3u7_bench8_full.json 2> gpurun_out/r3u7_bench8_full.log
echo "rc=$?"
