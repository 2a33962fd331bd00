# round 6 m: K1 class-1 filter cost per phase: the library built to end after
# phase N (GHOSTM_K1_STOP=N, ab_libs/stopN; N=1 phase 0 list bytes, 2 pass 1
# gather + marks, 3 pass 2 filter + queue, 4 pass 3 table inserts) and the full
# kernel: kernel time and SQ_INSTS_VALU of k_seed_filter<512,...> per launch (cfg4,
# one session run)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6m
mkdir -p $O /tmp/r6m_data
cd /tmp
timeout -k 10 300 python3 $R/tools/run_session.py --preset cfg4 --runs 1 --workdir /tmp/r6m_data > $O/warm.log 2>&1 || { echo "data failed"; tail -5 $O/warm.log; exit 1; }
for v in stop1 stop2 stop3 stop4 full; do
  LIB=$R/ab_libs/libghostm_hip_$v.so; [ $v = full ] && LIB=$R/ghostm_amd/lib/libghostm_hip.so
  GHOSTM_LIB_PATH=$LIB timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python3 $R/tools/run_session.py --preset cfg4 --runs 2 --workdir /tmp/r6m_data > $O/trace_$v.log 2>&1 || { echo "trace $v failed"; tail -5 $O/trace_$v.log; exit 1; }
  GHOSTM_LIB_PATH=$LIB timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_$v -o run -- python3 $R/tools/run_session.py --preset cfg4 --runs 1 --workdir /tmp/r6m_data > $O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $O/pmc_$v.log; exit 1; }
  echo "$v done"
done
python3 - $O <<'PY'
import csv, glob, os, sys
O = sys.argv[1]
for v in ["stop1", "stop2", "stop3", "stop4", "full"]:
    st = [r for f in glob.glob(f"{O}/trace_{v}/**/*kernel_stats.csv", recursive=True) for r in csv.DictReader(open(f))]
    ms = [float(r["AverageNs"]) / 1e6 for r in st if "k_seed_filter<512u" in r["Name"]]
    vals = {}
    for f in glob.glob(f"{O}/pmc_{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_seed_filter<512u" in r["Kernel_Name"]:
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print(v, "ms/launch", [round(x, 3) for x in ms], {k: f"{sum(x)/len(x):.4g}" for k, x in vals.items()})
PY
echo done
