# round 5: (1) the run-2 stall, three fresh processes of bench cfg4 with one
# warmup run and no settle (stream drains at run start in the library);
# (2) cfg2 GPU busy per run from a kernel trace (tools/gpu_busy.py)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5o
mkdir -p $O
cd $R
for t in 1 2 3; do
  GHOSTM_BENCH_WARM_SETTLE_S=0 timeout -k 10 300 python3 -u bench.py --no-cpu --no-e2e --steps 2 --warmup 1 --workdir /tmp/r5o_cfg4 > $O/stall_$t.json 2> $O/stall_$t.log || { echo "stall $t failed"; tail -5 $O/stall_$t.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('trial', sys.argv[2], 'steps', [round(x,1) for x in d['step_ms_rank0']])" $O/stall_$t.json $t
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/cfg2trace -o run -- python3 $R/tools/run_session.py --preset cfg2 --runs 6 --workdir /tmp/r5o_cfg2 > $O/cfg2trace.log 2>&1 || { echo "cfg2 trace failed"; tail -5 $O/cfg2trace.log; exit 1; }
grep '^run' $O/cfg2trace.log
python3 $R/tools/gpu_busy.py $O/cfg2trace/run_kernel_trace.csv --chunks 1 --skip 1 --gaps 30 > $O/cfg2_busy.txt
head -40 $O/cfg2_busy.txt
echo done
