# round 4: device timeline (kernels + copies) of cfg4 runs around the first timed run's K1a wait
export TMPDIR=/tmp
mkdir -p gpurun_out/r4v
GHOSTM_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r4v/prof -o tr -- python3 bench.py --preset cfg4 --steps 2 --warmup 1 --no-cpu --no-e2e --workdir /tmp/tr4v > gpurun_out/r4v/bench.json 2> gpurun_out/r4v/bench.log
echo rc=$?
find gpurun_out/r4v -name "*.csv" | head
