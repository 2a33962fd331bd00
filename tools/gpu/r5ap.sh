# round 5: the 125 K-query shard (per-rank work at N = 8): kernel-trace busy
# fraction and idle gaps per run, and a host timeline (GHOSTM_TRACE) of the same runs
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ap
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/tools/run_session.py --preset cfg4 --queries 125000 --runs 6 --workdir /tmp/r5ap > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
python3 $R/tools/gpu_busy.py $O/trace/run_kernel_trace.csv --chunks 1 --skip 1 --gaps 40 > $O/busy.txt
cat $O/busy.txt
GHOSTM_TRACE=1 timeout -k 10 300 python3 $R/tools/run_session.py --preset cfg4 --queries 125000 --runs 4 --workdir /tmp/r5ap > $O/host.log 2> $O/host_trace.txt || { echo "host trace failed"; tail -5 $O/host_trace.txt; exit 1; }
cat $O/host.log
echo done
