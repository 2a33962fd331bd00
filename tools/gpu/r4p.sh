# round 4: is the e2e write stall CPU-quota throttling? cgroup cpu.stat around
# cfg3 benches at 16 (default), 12 and 8 host threads
export TMPDIR=/tmp
mkdir -p gpurun_out/r4p /tmp/e_cfg3
cat /sys/fs/cgroup/cpu.max
for t in 16 12 8; do
  before=$(grep -E "nr_throttled|throttled_usec" /sys/fs/cgroup/cpu.stat | tr '\n' ' ')
  GHOSTM_THREADS=$t timeout -k 10 300 python3 bench.py --preset cfg3 --steps 5 --warmup 1 --no-cpu --workdir /tmp/e_cfg3 > gpurun_out/r4p/t$t.json 2> gpurun_out/r4p/t$t.log || exit $?
  after=$(grep -E "nr_throttled|throttled_usec" /sys/fs/cgroup/cpu.stat | tr '\n' ' ')
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print(sys.argv[1].split('/')[-1], 'step', round(d['ms_per_step'],2), 'e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e['runs_s']])" gpurun_out/r4p/t$t.json
  echo "  before: $before"; echo "  after:  $after"
done
