# round 6 s: K2 consecutive tasks built in parts on host threads: K2/golden/
# segment/full-workload parity, then A/B (GHOSTM_K2_TASKS_PAR=0) on the 125 K
# query shard's workload, cfg4 and cfg3, alternating
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6s
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "golden or segment or full_workload" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in 1 0; do
    GHOSTM_K2_TASKS_PAR=$v timeout -k 10 300 python3 -u bench.py --queries 125000 --steps 10 --warmup 2 --no-cpu --no-e2e --workdir /tmp/r6s_shard > $O/shard_${v}_$i.json 2> $O/shard_${v}_$i.log || { echo "shard $v failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('shard par', sys.argv[2], round(d['ms_per_step'],2), [round(x,1) for x in d['step_ms_rank0']])" $O/shard_${v}_$i.json $v
    GHOSTM_K2_TASKS_PAR=$v timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --workdir /tmp/r6s_cfg4 > $O/cfg4_${v}_$i.json 2> $O/cfg4_${v}_$i.log || { echo "cfg4 $v failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('cfg4 par', sys.argv[2], round(d['ms_per_step'],2))" $O/cfg4_${v}_$i.json $v
    GHOSTM_K2_TASKS_PAR=$v timeout -k 10 300 python3 -u bench.py --preset cfg3 --steps 10 --warmup 2 --no-cpu --no-e2e --workdir /tmp/r6s_cfg3 > $O/cfg3_${v}_$i.json 2> $O/cfg3_${v}_$i.log || { echo "cfg3 $v failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('cfg3 par', sys.argv[2], round(d['ms_per_step'],2))" $O/cfg3_${v}_$i.json $v
  done
done
echo done
