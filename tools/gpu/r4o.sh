# round 4: the bench line of every preset (default steps, CPU baselines), then
# the cfg4 rocprofv3 kernel trace and PMC passes (profiles/r4o_*)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4o
for p in cfg4 cfg3 cfg5 cfg2; do
  timeout -k 10 600 python3 -u bench.py --preset $p > gpurun_out/r4o/bench_$p.json 2> gpurun_out/r4o/bench_$p.log || { echo "bench $p failed"; tail -5 gpurun_out/r4o/bench_$p.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; c=d['cpu_baseline']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms; K2 frac', round(d['roofline']['frac'],4), 'traffic', d['roofline']['traffic'], '; e2e', round(e['value']/1e6,1), '; cpu', round(c['value']), c['bit_identical_to_gpu_on_sample'], d['full_output_matches_reference'])" gpurun_out/r4o/bench_$p.json
done
bash tools/profile.sh r4o cfg4 > gpurun_out/r4o/prof.log 2>&1 || { echo "profile failed"; tail -5 gpurun_out/r4o/prof.log; exit 1; }
cp profiles/r4o_* profiles/pmc_traffic.json profiles/pmc_traffic_cfg4.json gpurun_out/r4o/
tail -1 gpurun_out/r4o/prof.log
