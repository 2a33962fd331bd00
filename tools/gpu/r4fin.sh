# round 4 final: GPU tests, the bench line of every preset (CPU baselines, e2e), cfg4 + cfg3 profiles
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=gpurun_out/r4fin
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for p in cfg4 cfg3 cfg5 cfg2; do
  timeout -k 10 600 python3 -u bench.py --preset $p > $O/bench_$p.json 2> $O/bench_$p.log || { echo "bench $p failed"; tail -5 $O/bench_$p.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; c=d['cpu_baseline']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms; K2 frac', round(d['roofline']['frac'],4), 'traffic', d['roofline']['traffic'], '; e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e.get('runs_s',[])], '; cpu', round(c['value']), c['bit_identical_to_gpu_on_sample'], d['full_output_matches_reference'])" $O/bench_$p.json
done
for p in cfg4 cfg3; do
  bash tools/profile.sh r4fin_$p $p > $O/prof_$p.log 2>&1 || { echo "profile $p failed"; tail -5 $O/prof_$p.log; exit 1; }
  tail -1 $O/prof_$p.log
done
cp profiles/r4fin_* profiles/pmc_traffic*.json $O/
