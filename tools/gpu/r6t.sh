# round 6 t: the round-5 second-run stall: fresh processes with the run-start
# stream drains off (GHOSTM_RUN_SYNC=0) and on, four runs each (cfg4, first 125 K
# queries)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6t
mkdir -p $O
cd $R
timeout -k 10 300 python3 tools/run_session.py --preset cfg4 --queries 125000 --runs 1 --workdir /tmp/r6t > /dev/null 2>&1
for i in 1 2 3 4 5 6; do
  for s in 0 1; do
    echo "sync=$s proc $i: $(GHOSTM_RUN_SYNC=$s timeout -k 10 120 python3 tools/run_session.py --preset cfg4 --queries 125000 --runs 4 --workdir /tmp/r6t 2>&1 | grep -o 'run [0-9.]* ms' | tr '\n' ' ')"
  done
done | tee $O/stall.txt
echo done
