# 8-rank rehearsal of the N > 1 bench path (gloo, every rank on GPU 0), then the 1-GPU headline bench
export TMPDIR=/tmp
mkdir -p gpurun_out
GHOSTM_BENCH_BACKEND=gloo GHOSTM_BENCH_DEVICE=0 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29512 bench.py --queries 40000 --steps 5 --warmup 1 \
  --no-cpu > gpurun_out/r3b_bench8.json 2> gpurun_out/r3b_bench8.log || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r3b_bench1.json 2> gpurun_out/r3b_bench1.log
