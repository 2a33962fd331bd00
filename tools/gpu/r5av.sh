# round 5: mbcnt queue slots + the 24-bit bucket hash (fixed: unsigned shift of
# the int-typed __umul24). Poison golden/kernels groups through the poison build
# with both (pboth), parity tests through libghostm_hip_mbhash, then cfg4 A/B:
# default against mbhash and hash alone
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5av
mkdir -p $O /tmp/r5av_data
cd $R
for g in golden kernels; do
  GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_pboth.so GHOSTM_LDS_POISON_PATTERN=0xA5A5A5A5 timeout -k 10 150 python3 tests/lds_poison_child.py $g /tmp/r5av_data > $O/poison_$g.out 2> $O/poison_$g.err || { echo "poison $g failed rc=$?"; tail -c 600 $O/poison_$g.out; tail -5 $O/poison_$g.err; exit 1; }
  echo "poison $g: $(tail -c 250 $O/poison_$g.out)"
done
GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_mbhash.so timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_ROUNDS=2 AB_STEPS=3 timeout -k 10 900 bash tools/ab.sh mbhash hash > $O/ab.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
cd /tmp
ONE="$R/bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --workdir /tmp/ghostm_ab_data"
for v in new mbhash; do
  LIB=""; [ $v != new ] && LIB="$R/ghostm_amd/lib/libghostm_hip_$v.so"
  GHOSTM_LIB_PATH=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python3 $ONE > $O/trace_$v.log 2>&1 || { echo "trace $v failed"; tail -5 $O/trace_$v.log; exit 1; }
  python3 - $O $v <<'PY'
import csv, glob, sys
o, v = sys.argv[1], sys.argv[2]
for f in glob.glob(f"{o}/trace_{v}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "seed_filter" in r["Name"] or "seed_hash" in r["Name"]:
            print(v, r["Name"][:48], "calls", r["Calls"], "avg us", round(float(r["AverageNs"]) / 1e3, 1))
PY
done
echo done
