# round 5: the one-time stall of a session's second run. Host timelines
# (GHOSTM_TRACE: "seed" -> "k1_idle" is the wait for the stream to drain before
# K1) of bench cfg4 with no settle after warmup: plain, with busy-waiting HSA
# signals, and with the K1 read-backs into pageable memory; then a kernel +
# memory-copy trace (no API trace) of three back-to-back runs
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5f
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
summ() {
python3 - "$1" "$2" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
runs, cur = [], {}
for l in open(sys.argv[2]):
    p = l.split()
    if len(p) >= 4 and p[0] == "trace":
        t, m = float(p[1]), p[3]
        if m == "run":
            cur = {"run": t}
            runs.append(cur)
        elif m in ("seed", "k1_idle", "run_end") and cur is not None and m not in cur:
            cur[m] = t
waits = [round(r["k1_idle"] - r["seed"], 2) for r in runs if "k1_idle" in r and "seed" in r]
print(sys.argv[1].split("/")[-1], "steps", [round(x, 1) for x in d["step_ms_rank0"]], "k1 waits per run", waits)
PY
}
cat /sys/fs/cgroup/cpu.max > $O/cgroup.txt 2>&1; nproc >> $O/cgroup.txt; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))" >> $O/cgroup.txt
echo "cpu.max $(cat /sys/fs/cgroup/cpu.max 2>/dev/null) nproc $(nproc)"
thr() { grep -E 'nr_throttled|throttled_usec' /sys/fs/cgroup/cpu.stat 2>/dev/null | tr '\n' ' '; echo; }
echo "before: $(thr)"
for v in plain nointr pageable; do
  ENVV=""
  [ $v = nointr ] && ENVV="HSA_ENABLE_INTERRUPT=0"
  [ $v = pageable ] && ENVV="GHOSTM_K1_PINNED=0"
  env $ENVV GHOSTM_TRACE=1 GHOSTM_BENCH_WARM_SETTLE_S=0 timeout -k 10 300 python3 -u bench.py --no-cpu --no-e2e --steps 4 --warmup 1 --workdir /tmp/r5f_cfg4 > $O/stall_$v.json 2> $O/stall_$v.log || { echo "stall $v failed"; tail -5 $O/stall_$v.log; exit 1; }
  summ $O/stall_$v.json $O/stall_$v.log
  echo "after $v: $(thr)"
done
GHOSTM_TRACE=1 timeout -k 10 300 python3 -u bench.py --preset cfg3 --no-cpu --steps 4 --warmup 1 --workdir /tmp/r5f_cfg3 > $O/cfg3_e2e_trace.json 2> $O/cfg3_e2e_trace.log || { echo "cfg3 trace failed"; tail -5 $O/cfg3_e2e_trace.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print('cfg3', round(d['ms_per_step'],2), 'ms; e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e['runs_s']])" $O/cfg3_e2e_trace.json
grep -E 'fmt_(wall|cpu)' $O/cfg3_e2e_trace.log | tail -9
echo "after cfg3: $(thr)"
GHOSTM_TRACE=1 timeout -k 10 300 python3 -u bench.py --preset cfg2 --no-cpu --no-e2e --steps 3 --warmup 1 --workdir /tmp/r5f_cfg2 > $O/cfg2_trace.json 2> $O/cfg2_trace.log || { echo "cfg2 trace failed"; tail -5 $O/cfg2_trace.log; exit 1; }
cd /tmp
GHOSTM_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/ktrace -o run -- python3 $R/tools/run_session.py --preset cfg4 --runs 3 --workdir /tmp/r5f_cfg4s > $O/ktrace.log 2>&1 || { echo "ktrace failed"; tail -5 $O/ktrace.log; exit 1; }
grep '^run ' $O/ktrace.log
echo done
