# round 5: no head cap at >= 96 candidates per query; batch fast path; tests,
# shard / cfg4 / cfg3 lines
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5z
mkdir -p $O
cd $R
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_shards.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for t in 1 2; do
  timeout -k 10 300 python3 -u bench.py --queries 125000 --no-cpu --no-e2e --steps 10 --warmup 2 --workdir /tmp/r5z_shard > $O/shard_$t.json 2> $O/shard_$t.log || { echo "shard failed"; tail -5 $O/shard_$t.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; print('shard', round(d['ms_per_step'],3), 'ms; segments', d['config'].get('segments_per_rank_step'), 'K1', round(1e3*s['seed_device'],2), 'K3', round(1e3*s['traceback_device'],2))" $O/shard_$t.json
done
timeout -k 10 300 python3 -u bench.py --preset cfg3 --no-cpu --no-e2e --steps 10 --warmup 2 --workdir /tmp/r5z_cfg3 > $O/cfg3.json 2> $O/cfg3.log || { echo "cfg3 failed"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('cfg3', round(d['ms_per_step'],3), 'segments', d['config'].get('segments_per_rank_step'), 'matches', d.get('full_output_matches_reference'))" $O/cfg3.json
timeout -k 10 300 python3 -u bench.py --no-cpu --no-e2e --steps 3 --warmup 2 --workdir /tmp/r5z_cfg4 > $O/cfg4.json 2> $O/cfg4.log || { echo "cfg4 failed"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; print('cfg4', round(d['ms_per_step'],2), [round(x,1) for x in d['step_ms_rank0']], 'K1', round(1e3*s['seed_device'],2), 'matches', d.get('full_output_matches_reference'))" $O/cfg4.json
echo done
