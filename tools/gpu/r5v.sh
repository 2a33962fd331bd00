# round 5: allocations after the first run (K2 task buffers now start each chunk
# at the same one): shard and cfg4 host timelines, parity
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5v
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity failed"; tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
GHOSTM_TRACE=1 timeout -k 10 300 python3 -u tools/run_session.py --preset cfg4 --queries 125000 --runs 4 --workdir /tmp/r5v_shard > $O/shard.log 2> $O/shard_trace.log || { echo "shard failed"; exit 1; }
grep '^run' $O/shard.log
GHOSTM_TRACE=1 timeout -k 10 300 python3 -u tools/run_session.py --preset cfg4 --runs 3 --workdir /tmp/r5v_cfg4 > $O/cfg4.log 2> $O/cfg4_trace.log || { echo "cfg4 failed"; exit 1; }
grep '^run' $O/cfg4.log
for f in shard cfg4; do
  python3 - $O/${f}_trace.log $f <<'PY'
import sys
runs, n = [], -1
for l in open(sys.argv[1]):
    p = l.split()
    if len(p) >= 4 and p[0] == "trace":
        if p[3] == "run":
            n += 1
            runs.append([])
        elif p[3] in ("pin_alloc", "dev_alloc", "dev_free", "dev_reuse") and n >= 0:
            runs[n].append((p[1], p[3], p[4]))
for k, r in enumerate(runs):
    print(sys.argv[2], "run", k, "allocations:", r[:12])
PY
done
echo done
