# round 4: end-to-end run-to-run variance: settle time between runs, and the
# output on /tmp (disk) against /dev/shm (memory)
export TMPDIR=/tmp
mkdir -p gpurun_out/r4n /tmp/e_cfg3
for settle in 0 1 3; do
  GHOSTM_BENCH_SETTLE_S=$settle GHOSTM_TRACE=1 timeout -k 10 300 python3 bench.py --preset cfg3 --steps 2 --warmup 1 --no-cpu --workdir /tmp/e_cfg3 > gpurun_out/r4n/s$settle.json 2> gpurun_out/r4n/s$settle.log || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print(sys.argv[1].split('/')[-1], 'e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e['runs_s']])" gpurun_out/r4n/s$settle.json
done
mkdir -p /dev/shm/e_cfg3
timeout -k 10 300 python3 bench.py --preset cfg3 --steps 2 --warmup 1 --no-cpu --workdir /dev/shm/e_cfg3 > gpurun_out/r4n/shm.json 2> gpurun_out/r4n/shm.log; rc=$?
rm -rf /dev/shm/e_cfg3
[ $rc -eq 0 ] || exit $rc
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print('shm e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e['runs_s']])" gpurun_out/r4n/shm.json
df -T /tmp | tail -1; cat /proc/sys/vm/dirty_ratio /proc/sys/vm/dirty_background_ratio /proc/sys/vm/dirty_bytes 2>/dev/null; cat /sys/fs/cgroup/memory.max 2>/dev/null
