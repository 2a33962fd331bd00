# round 5: DB chunks uploaded by their reading threads (create overlap): tests,
# then end to end on cfg3, cfg2 (twice) and cfg4 with create times
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ae
mkdir -p $O
cd $R
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_shards.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for p in cfg3 cfg2 cfg3 cfg2; do
  timeout -k 10 300 python3 -u bench.py --preset $p --no-cpu --steps 4 --warmup 2 --workdir /tmp/r5ae_$p > $O/$p.json 2> $O/$p.log || { echo "$p failed"; tail -5 $O/$p.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print(sys.argv[2], round(d['ms_per_step'],2), 'ms; e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e['runs_s']], 'create', [round(x*1e3,2) for x in e['create_s']], 'ok', e.get('output_files_match_reference'))" $O/$p.json $p
done
GHOSTM_TRACE=1 timeout -k 10 400 python3 -u bench.py --preset cfg4 --no-cpu --steps 1 --warmup 1 --workdir /tmp/r5ae_cfg4 > $O/cfg4.json 2> $O/cfg4.log || { echo "cfg4 failed"; tail -5 $O/cfg4.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print('cfg4 e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e['runs_s']], 'create', [round(x*1e3,1) for x in e['create_s']])" $O/cfg4.json
echo done
