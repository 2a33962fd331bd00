# round 5: the 125 K-query shard (a rank's share of cfg4 at N = 8): per-step
# time with and without the head cap, and its GPU-busy trace
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5t
mkdir -p $O
cd $R
for v in head nohead head2 nohead2; do
  ENVV="GHOSTM_HEAD_CANDS=1048576"
  case $v in nohead*) ENVV="GHOSTM_HEAD_CANDS=0" ;; esac
  env $ENVV timeout -k 10 300 python3 -u bench.py --queries 125000 --no-cpu --no-e2e --steps 10 --warmup 2 --workdir /tmp/r5t_cfg4 > $O/shard_$v.json 2> $O/shard_$v.log || { echo "shard $v failed"; tail -5 $O/shard_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; print(sys.argv[2], round(d['ms_per_step'],2), 'ms; K1', round(1e3*s['seed_device'],2), 'K2', round(1e3*s['score_device'],2), 'K3', round(1e3*s['traceback_device'],2), 'segments', d['config'].get('segments_per_rank_step'))" $O/shard_$v.json $v
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/tools/run_session.py --preset cfg4 --queries 125000 --runs 5 --workdir /tmp/r5t_cfg4s > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
grep '^run' $O/trace.log
python3 $R/tools/gpu_busy.py $O/trace/run_kernel_trace.csv --chunks 1 --skip 1 --gaps 100 > $O/busy.txt
head -30 $O/busy.txt
echo done
