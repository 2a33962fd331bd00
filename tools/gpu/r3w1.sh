# the 8-GPU shard size on one GPU after the unit K2 / strip K3: host timeline (GHOSTM_TRACE) and a kernel trace
export TMPDIR=/tmp
mkdir -p gpurun_out/r3w1 /tmp/r3w1d
GHOSTM_TRACE=1 timeout -k 10 300 python3 bench.py --queries 125000 --steps 3 --warmup 1 --no-cpu --no-e2e \
  --workdir /tmp/r3w1d > gpurun_out/r3w1/bench125k.json 2> gpurun_out/r3w1/bench125k.err || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3w1/trace -o run \
  -- python3 $GRAFT_REPO_ROOT/bench.py --queries 125000 --steps 3 --warmup 1 --no-cpu --no-e2e --workdir /tmp/r3w1d \
  > $GRAFT_REPO_ROOT/gpurun_out/r3w1/trace.log 2>&1
echo "trace rc=$?"
