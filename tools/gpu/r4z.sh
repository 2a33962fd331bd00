# round 4: device/pinned allocations per run (cfg4 host timeline)
export TMPDIR=/tmp
mkdir -p gpurun_out/r4z
GHOSTM_TRACE=1 timeout -k 10 200 python3 bench.py --preset cfg4 --steps 2 --warmup 1 --no-cpu --no-e2e --workdir /tmp/tr4z > gpurun_out/r4z/b.json 2> gpurun_out/r4z/b.log || exit $?
awk '/seed /{s=$2} /k1_idle/{printf "%.1f ", $2-s}' gpurun_out/r4z/b.log; echo
