# round 4: K1 filter phases (cfg4): k_seed_filter builds that stop after phase N (GHOSTM_K1_STOP)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4ad
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
