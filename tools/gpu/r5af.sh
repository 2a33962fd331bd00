# round 5: query chunks also uploaded by their reading threads: tests, then end
# to end on cfg3, cfg2, cfg4 (create times) and a cfg2 create trace
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5af
mkdir -p $O
cd $R
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_shards.py tests/test_gpu_rccl.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for p in cfg3 cfg2 cfg3 cfg2; do
  timeout -k 10 300 python3 -u bench.py --preset $p --no-cpu --steps 4 --warmup 2 --workdir /tmp/r5af_$p > $O/$p.json 2> $O/$p.log || { echo "$p failed"; tail -5 $O/$p.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print(sys.argv[2], round(d['ms_per_step'],2), 'ms; e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e['runs_s']], 'create', [round(x*1e3,2) for x in e['create_s']], 'ok', e.get('output_files_match_reference'))" $O/$p.json $p
done
timeout -k 10 400 python3 -u bench.py --preset cfg4 --no-cpu --steps 1 --warmup 1 --workdir /tmp/r5af_cfg4 > $O/cfg4.json 2> $O/cfg4.log || { echo "cfg4 failed"; tail -5 $O/cfg4.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print('cfg4 e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e['runs_s']], 'create', [round(x*1e3,1) for x in e['create_s']])" $O/cfg4.json
GHOSTM_TRACE=1 timeout -k 10 400 python3 -u bench.py --preset cfg2 --no-cpu --steps 1 --warmup 1 --workdir /tmp/r5af_cfg2 > $O/cfg2_trace.json 2> $O/cfg2_trace.log || { echo "cfg2 trace failed"; exit 1; }
echo done
