# cfg3 host timeline (GHOSTM_TRACE) and kernel trace: where a 100K-query step's time goes
export TMPDIR=/tmp
mkdir -p gpurun_out/r3w2 /tmp/r3w2d
GHOSTM_TRACE=1 timeout -k 10 300 python3 bench.py --preset cfg3 --steps 3 --warmup 1 --no-cpu --no-e2e \
  --workdir /tmp/r3w2d > gpurun_out/r3w2/bench.json 2> gpurun_out/r3w2/bench.err || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3w2/trace -o run \
  -- python3 $GRAFT_REPO_ROOT/bench.py --preset cfg3 --steps 3 --warmup 1 --no-cpu --no-e2e --workdir /tmp/r3w2d \
  > $GRAFT_REPO_ROOT/gpurun_out/r3w2/trace.log 2>&1
echo "trace rc=$?"
