# round 5: K1 pass 1 predecessor loads, list origins in the LDS table, queue slots by mbcnt, 24-bit bucket hash;
# the whole GPU suite, then cfg4 A/B against the round-start pass 1 and 2
# (libghostm_hip_old), without mbcnt (nomb) and with the 32-bit hash (nohash);
# K1 filter kernel times of the three
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5at
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_ROUNDS=2 AB_STEPS=3 timeout -k 10 900 bash tools/ab.sh old nomb nohash > $O/ab.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
cd /tmp
ONE="$R/bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --workdir /tmp/ghostm_ab_data"
for v in new old nomb nohash; do
  LIB=""; [ $v != new ] && LIB="$R/ghostm_amd/lib/libghostm_hip_$v.so"
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
