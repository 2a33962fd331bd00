# round 4: K1 second-stage hashed filter over the queue (st2) against the current build, cfg4 (+ cfg3 parity)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4am
mkdir -p $O
for p in cfg4 cfg3; do
  GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_st2.so timeout -k 10 300 python3 bench.py --preset $p --steps 3 --warmup 1 --no-cpu --no-e2e --workdir /tmp/st2_$p > $O/st2_bench_$p.json 2> $O/st2_bench_$p.log || { echo "st2 bench $p failed"; tail -5 $O/st2_bench_$p.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('st2 bench', sys.argv[2], round(d['ms_per_step'],1), 'ms, matches', d['full_output_matches_reference'], 'k1', round(d['roofline_k1']['ms_per_step'],2))" $O/st2_bench_$p.json $p
done
cd /tmp
for v in cur st2 noalias cur st2 noalias; do
  L=$R/ghostm_amd/lib/libghostm_hip_$v.so; [ $v = cur ] && L=$R/ghostm_amd/lib/libghostm_hip.so
  rm -rf $O/ab_$v
  GHOSTM_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ab_$v -o run -- python3 $R/tools/run_session.py --preset cfg4 --runs 2 --workdir /tmp/st2_cfg4 > $O/ab_$v.log 2>&1 || { echo "$v failed"; tail -5 $O/ab_$v.log; exit 1; }
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
