# round 4: cfg2 and cfg5 bench lines with their PMC summaries present (roofline traffic)
export TMPDIR=/tmp
O=gpurun_out/r4at
mkdir -p $O
for p in cfg2 cfg5; do
  timeout -k 10 600 python3 -u bench.py --preset $p > $O/bench_$p.json 2> $O/bench_$p.log || { echo "bench $p failed"; tail -5 $O/bench_$p.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms; traffic', d['roofline']['traffic'], '; e2e', round(e['value']/1e6,1), d['full_output_matches_reference'])" $O/bench_$p.json
done
