# round 5: host timeline of the 125 K-query shard's runs (the second run's
# 6 ms idle between a K2 and the next K4 in profiles/r5t)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5u
mkdir -p $O
cd $R
GHOSTM_TRACE=1 timeout -k 10 300 python3 -u tools/run_session.py --preset cfg4 --queries 125000 --runs 4 --workdir /tmp/r5u_cfg4 > $O/shard.log 2> $O/shard_trace.log || { echo "shard failed"; tail -5 $O/shard.log $O/shard_trace.log; exit 1; }
grep '^run' $O/shard.log
echo done
