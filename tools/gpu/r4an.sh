# round 4: K1 filter phases (cfg4): k_seed_filter builds that stop after phase N (GHOSTM_K1_STOP)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4an
mkdir -p $O
cd /tmp
for v in k1s1 k1s2 k1s3 k1s4 full; do
  L=$R/ghostm_amd/lib/libghostm_hip_$v.so; [ $v = full ] && L=$R/ghostm_amd/lib/libghostm_hip.so
  GHOSTM_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 $R/tools/run_session.py --preset cfg4 --runs 2 --workdir /tmp/k1ph > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  f=$(find $O/$v -name "run_kernel_stats.csv" | head -1)
  echo -n "$v: "; python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_seed_filter<512' in r['Name']: print(r['Calls'], 'calls, avg ms', round(float(r['AverageNs'])/1e6,3))
" $f
done
# cfg2 (one segment by default): a smaller tail splits it, so formatting overlaps K2
cd $R
for rep in 1 2; do
for t in 1048576 524288 262144; do
  GHOSTM_TAIL_CANDS=$t timeout -k 10 300 python3 bench.py --preset cfg2 --steps 10 --warmup 2 --no-cpu --no-e2e --workdir /tmp/tail_cfg2 > $O/cfg2_$t.$rep.json 2> $O/cfg2_$t.$rep.log || { echo "cfg2 $t failed"; tail -3 $O/cfg2_$t.$rep.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('cfg2', sys.argv[2], round(d['ms_per_step'],2), 'ms', d['config']['segments_per_rank_step'], d['full_output_matches_reference'])" $O/cfg2_$t.$rep.json $t
done
done
