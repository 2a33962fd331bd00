# round 4: K1 list-byte fill by boundaries (cfg4): phase 0 and the whole filter, against the previous build
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4ai
mkdir -p $O
cd /tmp
for v in full ng pfng k1old full ng pfng k1old; do
  L=$R/ghostm_amd/lib/libghostm_hip_$v.so; [ $v = full ] && L=$R/ghostm_amd/lib/libghostm_hip.so
  rm -rf $O/$v
  GHOSTM_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 $R/tools/run_session.py --preset cfg4 --runs 2 --workdir /tmp/k1ph > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  f=$(find $O/$v -name "run_kernel_stats.csv" | head -1)
  echo -n "$v: "; python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_seed_filter<512' in r['Name']: print(r['Calls'], 'calls, avg ms', round(float(r['AverageNs'])/1e6,3), end=' ')
print()
" $f
  grep "^run" $O/$v.log | tr '\n' ' '; echo
done
