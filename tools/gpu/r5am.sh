# round 5: K1a reads a list's first position only for keys flagged in the
# low-keys bitmap; parity tests, cfg4 A/B against the unfiltered build
# (libghostm_hip_nolow), k_seed_lists duration and FETCH_SIZE for both
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5am
mkdir -p $O
cd $R
timeout -k 10 800 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_shards.py "tests/test_gpu_lds_poison.py::test_golden_variants_under_lds_poison[0xA5A5A5A5-kernels]" -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_ROUNDS=2 AB_STEPS=3 timeout -k 10 900 bash tools/ab.sh nolow > $O/ab.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
cd /tmp
ONE="$R/bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --workdir /tmp/ghostm_ab_data"
for v in new nolow; do
  LIB=""; [ $v = nolow ] && LIB="$R/ghostm_amd/lib/libghostm_hip_nolow.so"
  GHOSTM_LIB_PATH=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python3 $ONE > $O/trace_$v.log 2>&1 || { echo "trace $v failed"; tail -5 $O/trace_$v.log; exit 1; }
  GHOSTM_LIB_PATH=$LIB timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$v -o run -- python3 $ONE > $O/fetch_$v.log 2>&1 || { echo "fetch $v failed"; tail -5 $O/fetch_$v.log; exit 1; }
  python3 - $O $v <<'PY'
import csv, glob, sys
o, v = sys.argv[1], sys.argv[2]
for f in glob.glob(f"{o}/trace_{v}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "seed" in r["Name"] or "compact" in r["Name"] or "low_keys" in r["Name"]:
            print(v, r["Name"][:40], "calls", r["Calls"], "avg us", round(float(r["AverageNs"]) / 1e3, 1))
for f in glob.glob(f"{o}/fetch_{v}/**/*counter_collection.csv", recursive=True):
    agg = {}
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "seed_lists" in n or "low_keys" in n:
            k = n[:40]
            agg.setdefault(k, []).append(float(r["Counter_Value"]))
    for k, xs in agg.items():
        print(v, k, "FETCH_SIZE KB per launch", [round(x) for x in xs])
PY
done
echo done
