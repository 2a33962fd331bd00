# round 4: K1 filter test by one ds_read2_b32 (guard word) against two reads (r2off); GPU tests
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4ap
mkdir -p $O
cd $R && timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for p in cfg4 cfg2; do
  GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_r2on.so timeout -k 10 300 python3 bench.py --preset $p --steps 3 --warmup 1 --no-cpu --no-e2e --workdir /tmp/ap_$p > $O/r2on_$p.json 2> $O/r2on_$p.log || { echo "r2on bench $p failed"; tail -5 $O/r2on_$p.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('r2on bench', sys.argv[2], round(d['ms_per_step'],1), 'ms, matches', d['full_output_matches_reference'], 'k1', round(d['roofline_k1']['ms_per_step'],2))" $O/r2on_$p.json $p
done
cd /tmp
for v in r2on cur r2on cur; do
  L=$R/ghostm_amd/lib/libghostm_hip_$v.so; [ $v = cur ] && L=$R/ghostm_amd/lib/libghostm_hip.so
  rm -rf $O/ab_$v
  GHOSTM_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ab_$v -o run -- python3 $R/tools/run_session.py --preset cfg4 --runs 2 --workdir /tmp/ap_cfg4 > $O/ab_$v.log 2>&1 || { echo "$v failed"; tail -5 $O/ab_$v.log; exit 1; }
  f=$(find $O/ab_$v -name "run_kernel_stats.csv" | head -1)
  echo -n "$v: "; python3 -c "
import csv,sys
t=0
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_seed' in r['Name'] or 'k_compact' in r['Name']:
        t+=float(r['TotalDurationNs'])
        if 'k_seed_filter' in r['Name']: print(r['Name'][27:60], round(float(r['AverageNs'])/1e6,3), end=' | ')
print('K1 kernels per run ms', round(t/2e6,2))
" $f
done
