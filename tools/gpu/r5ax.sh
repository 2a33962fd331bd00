# round 5: cfg2 A/B of this round's K1 changes (libghostm_hip_old: lane-0
# predecessor loads, popcount slots, 32-bit hash) and the K1 kernel times
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ax
mkdir -p $O
cd $R
AB_ROUNDS=3 AB_STEPS=10 AB_ARGS="--preset cfg2" timeout -k 10 600 bash tools/ab.sh old > $O/ab.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
cd /tmp
ONE="$R/bench.py --preset cfg2 --steps 3 --warmup 1 --no-cpu --no-e2e --workdir /tmp/ghostm_ab_data"
for v in new old; do
  LIB=""; [ $v != new ] && LIB="$R/ghostm_amd/lib/libghostm_hip_$v.so"
  GHOSTM_LIB_PATH=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python3 $ONE > $O/trace_$v.log 2>&1 || { echo "trace $v failed"; tail -5 $O/trace_$v.log; exit 1; }
  python3 - $O $v <<'PY'
import csv, glob, sys
o, v = sys.argv[1], sys.argv[2]
for f in glob.glob(f"{o}/trace_{v}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "seed" in r["Name"]:
            print(v, r["Name"][:48], "calls", r["Calls"], "avg us", round(float(r["AverageNs"]) / 1e3, 1))
PY
done
echo done
