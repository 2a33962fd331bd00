# round 4: K1 variants (guards / prefetch) and the bank-private K3 scan table, cfg4
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4aj
mkdir -p $O
cd /tmp
stat() {  # $1 dir, $2 kernel name substring
  f=$(find $1 -name "run_kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r['Name']: print(r['Name'][:48], r['Calls'], 'calls, avg ms', round(float(r['AverageNs'])/1e6,3), end=' | ')
print()
" $f "$2"
}
cd $R && timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
# parity of the private-table scan on the full workload (bench checks the whole output against the pin)
cd $R && GHOSTM_K3_SCAN=priv timeout -k 10 300 python3 bench.py --preset cfg4 --steps 2 --warmup 1 --no-cpu --no-e2e --workdir /tmp/k1ph > $O/priv_bench.json 2> $O/priv_bench.log || { echo "priv bench failed"; tail -5 $O/priv_bench.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('priv bench', round(d['ms_per_step'],1), 'ms, matches', d['full_output_matches_reference'], 'tb', round(d['roofline_k3']['ms_per_step'],2))" $O/priv_bench.json
GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_a128.so timeout -k 10 300 python3 bench.py --preset cfg4 --steps 2 --warmup 1 --no-cpu --no-e2e --workdir /tmp/k1ph > $O/a128_bench.json 2> $O/a128_bench.log || { echo "a128 bench failed"; tail -5 $O/a128_bench.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('a128 bench', round(d['ms_per_step'],1), 'ms, matches', d['full_output_matches_reference'], 'k1', round(d['roofline_k1']['ms_per_step'],2))" $O/a128_bench.json
cd /tmp
for v in scan_base scan_priv scan_base scan_priv; do
  E=X=1; [ $v = scan_priv ] && E=GHOSTM_K3_SCAN=priv
  rm -rf $O/$v
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 $R/tools/run_session.py --preset cfg4 --runs 2 --workdir /tmp/k1ph > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  echo -n "$v: "; stat $O/$v k_tb_scan
done
for v in full ng f128 a128 a64 k1old full ng f128 a128 a64 k1old; do
  L=$R/ghostm_amd/lib/libghostm_hip_$v.so; [ $v = full ] && L=$R/ghostm_amd/lib/libghostm_hip.so
  rm -rf $O/$v
  GHOSTM_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 $R/tools/run_session.py --preset cfg4 --runs 2 --workdir /tmp/k1ph > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  echo -n "$v: "; stat $O/$v "k_seed_filter<512"
done
