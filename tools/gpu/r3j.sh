# the 8-GPU shard size on one GPU: host timeline (GHOSTM_TRACE) and a kernel trace
export TMPDIR=/tmp
mkdir -p gpurun_out/r3j /tmp/r3jd
GHOSTM_TRACE=1 timeout -k 10 300 python3 bench.py --queries 125000 --steps 3 --warmup 1 --no-cpu --no-e2e \
  --workdir /tmp/r3jd > gpurun_out/r3j/bench125k.json 2> gpurun_out/r3j/bench125k.err || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3j/trace -o run \
  -- python3 $GRAFT_REPO_ROOT/bench.py --queries 125000 --steps 3 --warmup 1 --no-cpu --no-e2e --workdir /tmp/r3jd \
  > $GRAFT_REPO_ROOT/gpurun_out/r3j/trace.log 2>&1
echo "trace rc=$?"
