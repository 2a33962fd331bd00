# round 5: K1 pass 1 with every lane loading its list predecessor
# (libghostm_hip_prevall, -DGHOSTM_K1_PREVALL=1): parity through that build,
# then cfg4 A/B against the default and the class-1 kernel time of both
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5aq
mkdir -p $O
cd $R
GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_prevall.so timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_ROUNDS=3 AB_STEPS=3 timeout -k 10 900 bash tools/ab.sh prevall > $O/ab.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
cd /tmp
ONE="$R/bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --workdir /tmp/ghostm_ab_data"
for v in new prevall; do
  LIB=""; [ $v = prevall ] && LIB="$R/ghostm_amd/lib/libghostm_hip_prevall.so"
  GHOSTM_LIB_PATH=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python3 $ONE > $O/trace_$v.log 2>&1 || { echo "trace $v failed"; tail -5 $O/trace_$v.log; exit 1; }
  python3 - $O $v <<'PY'
import csv, glob, sys
o, v = sys.argv[1], sys.argv[2]
for f in glob.glob(f"{o}/trace_{v}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "seed_filter" in r["Name"]:
            print(v, r["Name"][:48], "calls", r["Calls"], "avg us", round(float(r["AverageNs"]) / 1e3, 1))
PY
done
echo done
