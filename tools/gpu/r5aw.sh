# round 5 final checkpoint: the whole GPU suite, then bench lines for every config
# (CPU baselines included) and the RCCL world-1 line
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5aw
mkdir -p $O
cd $R
GHOSTM_TEST_OUT=$O/rccl_world1.json timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for p in cfg4 cfg3 cfg5 cfg2; do
  STEPS=10; [ $p = cfg4 ] && STEPS=5
  timeout -k 10 600 python3 -u bench.py --preset $p --steps $STEPS --warmup 2 --workdir /tmp/r5aw_$p > $O/bench_$p.json 2> $O/bench_$p.log || { echo "$p failed"; tail -5 $O/bench_$p.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d.get('end_to_end') or {}; c=d.get('cpu_baseline') or {}; s=d['stages_s_per_step']; print(sys.argv[2], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms; K1/K2/K3', round(1e3*s['seed_device'],2), round(1e3*s['score_device'],2), round(1e3*s['traceback_device'],2), '; e2e', round(e.get('value',0)/1e6,1), '; cpu', round(c.get('value',0)/1e3,1), 'K/s; matches', d.get('full_output_matches_reference'))" $O/bench_$p.json $p
done
echo done
