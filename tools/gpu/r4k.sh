export TMPDIR=/tmp
mkdir -p gpurun_out/r4k /tmp/k_cfg3 /tmp/k_cfg2
GHOSTM_DEBUG_TASKS=/tmp/t.bin timeout -k 10 200 python3 bench.py --preset cfg3 --steps 1 --warmup 0 --no-cpu --no-e2e --workdir /tmp/k_cfg3 > gpurun_out/r4k/cfg3.json 2> gpurun_out/r4k/cfg3.log; echo rc=$?
grep "k2 tasks" gpurun_out/r4k/cfg3.log
GHOSTM_DEBUG_TASKS=/tmp/t2.bin timeout -k 10 200 python3 bench.py --preset cfg2 --steps 1 --warmup 0 --no-cpu --no-e2e --workdir /tmp/k_cfg2 > gpurun_out/r4k/cfg2.json 2> gpurun_out/r4k/cfg2.log; echo rc=$?
grep "k2 tasks" gpurun_out/r4k/cfg2.log
