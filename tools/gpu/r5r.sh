# round 5 bench lines: parity first (scale, parity, shards), then every config
# with the CPU baselines (cfg4, cfg3, cfg5, cfg2) and the cfg2 GPU-busy trace
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5r
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_shards.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for p in cfg4 cfg3 cfg5 cfg2; do
  STEPS=10; [ $p = cfg4 ] && STEPS=5
  timeout -k 10 600 python3 -u bench.py --preset $p --steps $STEPS --warmup 2 --workdir /tmp/r5r_$p > $O/bench_$p.json 2> $O/bench_$p.log || { echo "$p failed"; tail -5 $O/bench_$p.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d.get('end_to_end') or {}; c=d.get('cpu_baseline') or {}; print(sys.argv[2], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms; e2e', round(e.get('value',0)/1e6,1), '; cpu', round(c.get('value',0)/1e3,1), 'K/s', c.get('kind'), '; matches', d.get('full_output_matches_reference'))" $O/bench_$p.json $p
done
echo done
