# round 6 zo: bench lines on the final library (CLI fast exit): bench lines for every config (CPU baselines
# included; counters from the hash-matched PMC summaries)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6zo
mkdir -p $O
cd $R
for p in cfg4 cfg3 cfg5 cfg2; do
  STEPS=10; [ $p = cfg4 ] && STEPS=5
  timeout -k 10 900 python3 -u bench.py --preset $p --steps $STEPS --warmup 2 --workdir /tmp/r6zo_$p > $O/bench_$p.json 2> $O/bench_$p.log || { echo "$p failed"; tail -5 $O/bench_$p.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d.get('cpu_baseline') or {}; s=d['stages_s_per_step']; print(sys.argv[2], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms; K1/K2/K3', round(1e3*s['seed_device'],2), round(1e3*s['score_device'],2), round(1e3*s['traceback_device'],2), '; K2 frac', round(d['roofline']['frac'],3), 'pmc', d['roofline']['pmc_source']['used'], '; e2e warm', round((d['value_end_to_end_warm'] or 0)/1e6,1), 'cold', round((d['value_end_to_end_cold'] or 0)/1e6,1), '; cpu', round(c.get('value',0)/1e3,1), 'K/s; matches', d.get('full_output_matches_reference'))" $O/bench_$p.json $p
done
echo done
