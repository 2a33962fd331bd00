# round 5: class-1 K1 filter time with the identity launch (every query a block,
# out-of-class blocks return) against the class-list launch (GHOSTM_K1_EARLY=0)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ao
mkdir -p $O /tmp/ghostm_ab_data
cd /tmp
ONE="$R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --workdir /tmp/ghostm_ab_data"
for v in early list early2 list2; do
  E=1; case $v in list*) E=0 ;; esac
  GHOSTM_K1_EARLY=$E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python3 $ONE > $O/trace_$v.log 2>&1 || { echo "trace $v failed"; tail -5 $O/trace_$v.log; exit 1; }
  python3 - $O $v <<'PY'
import csv, glob, json, sys
o, v = sys.argv[1], sys.argv[2]
for f in glob.glob(f"{o}/trace_{v}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "seed" in r["Name"] or "compact" in r["Name"]:
            print(v, r["Name"][:48], "calls", r["Calls"], "avg us", round(float(r["AverageNs"]) / 1e3, 1))
for line in open(f"{o}/trace_{v}.log"):
    if line.startswith("{"):
        d = json.loads(line)
        print(v, "ms/step", round(d["ms_per_step"], 1), "K1", round(d["stages_s_per_step"]["seed_device"] * 1e3, 2), "classes", d["roofline_k1"]["queries_per_class"])
PY
done
echo done
