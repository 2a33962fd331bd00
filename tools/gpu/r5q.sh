# round 5: K1's host pass in parts with page-locked offsets, the first pair
# list built in parts: parity (scale, parity, shards), then cfg2/cfg4 lines and
# the cfg2 GPU-busy trace
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5q
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_shards.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u bench.py --preset cfg2 --no-cpu --steps 20 --warmup 2 --workdir /tmp/r5q_cfg2 > $O/cfg2.json 2> $O/cfg2.log || { echo "cfg2 failed"; tail -5 $O/cfg2.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; e=d['end_to_end']; print('cfg2', round(d['ms_per_step'],3), 'ms; K2', round(1e3*s['score_device'],3), 'e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e['runs_s']], 'matches', d.get('full_output_matches_reference'))" $O/cfg2.json
timeout -k 10 300 python3 -u bench.py --no-cpu --no-e2e --steps 3 --warmup 1 --workdir /tmp/r5q_cfg4 > $O/cfg4.json 2> $O/cfg4.log || { echo "cfg4 failed"; tail -5 $O/cfg4.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; print('cfg4', round(d['ms_per_step'],2), [round(x,1) for x in d['step_ms_rank0']], 'K1', round(1e3*s['seed_device'],2), 'matches', d.get('full_output_matches_reference'))" $O/cfg4.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/cfg2trace -o run -- python3 $R/tools/run_session.py --preset cfg2 --runs 6 --workdir /tmp/r5q_cfg2s > $O/cfg2trace.log 2>&1 || { echo "cfg2 trace failed"; tail -5 $O/cfg2trace.log; exit 1; }
python3 $R/tools/gpu_busy.py $O/cfg2trace/run_kernel_trace.csv --chunks 1 --skip 1 --gaps 30 > $O/cfg2_busy.txt
grep "^run" $O/cfg2_busy.txt
echo done
