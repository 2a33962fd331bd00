# round 5: (1) parity after the head-segment cap; (2) the run-2 stall with idle
# probes at run start and after the carry reset (GHOSTM_TRACE marks run_idle,
# carry_idle, k1_idle) and this process's KFD counters after each run;
# (3) head cap A/B on cfg2, cfg3 (end to end) and cfg4
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity failed"; tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
ls /sys/class/kfd/kfd/proc 2>&1 | head -3 > $O/kfd_ls.txt
GHOSTM_TRACE=1 timeout -k 10 300 python3 -u tools/run_session.py --preset cfg4 --runs 4 --kfd --workdir /tmp/r5g_cfg4 > $O/probe.log 2> $O/probe_trace.log || { echo "probe failed"; tail -5 $O/probe.log $O/probe_trace.log; exit 1; }
grep -E '^(run|kfd)' $O/probe.log | cut -c1-400
python3 - $O/probe_trace.log <<'PY'
import sys
runs, cur = [], None
for l in open(sys.argv[1]):
    p = l.split()
    if len(p) >= 4 and p[0] == "trace":
        t, m = float(p[1]), p[3]
        if m == "run":
            cur = {}
            runs.append(cur)
        if cur is not None and m not in cur:
            cur[m] = t
for r in runs:
    print({k: r[k] for k in ("run_idle", "carry_idle", "seed", "k1_idle", "seed_done", "run_end") if k in r})
PY
for h in default 0; do
  ENVV=""
  [ $h = 0 ] && ENVV="GHOSTM_HEAD_CANDS=0"
  env $ENVV timeout -k 10 300 python3 -u bench.py --preset cfg2 --no-cpu --steps 10 --warmup 2 --workdir /tmp/r5g_cfg2 > $O/cfg2_head_$h.json 2> $O/cfg2_head_$h.log || { echo "cfg2 $h failed"; tail -5 $O/cfg2_head_$h.log; exit 1; }
  env $ENVV timeout -k 10 300 python3 -u bench.py --preset cfg3 --no-cpu --steps 6 --warmup 1 --workdir /tmp/r5g_cfg3 > $O/cfg3_head_$h.json 2> $O/cfg3_head_$h.log || { echo "cfg3 $h failed"; tail -5 $O/cfg3_head_$h.log; exit 1; }
  env $ENVV timeout -k 10 300 python3 -u bench.py --no-cpu --no-e2e --steps 3 --warmup 1 --workdir /tmp/r5g_cfg4 > $O/cfg4_head_$h.json 2> $O/cfg4_head_$h.log || { echo "cfg4 $h failed"; tail -5 $O/cfg4_head_$h.log; exit 1; }
  for c in cfg2 cfg3 cfg4; do
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d.get('end_to_end') or {}; s=d['stages_s_per_step']; print(sys.argv[2], 'head', sys.argv[3], round(d['ms_per_step'],3), 'ms', [round(x,2) for x in d['step_ms_rank0']], 'dev', round(1e3*(s['seed_device']+s['score_device']+s['traceback_device']),3), 'e2e', round(e.get('value',0)/1e6,1), [round(x*1e3,1) for x in e.get('runs_s',[])])" $O/${c}_head_$h.json $c $h
  done
done
echo done
