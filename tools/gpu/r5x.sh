# round 5: K1 offsets and compaction on the device before the host count pass;
# forced-overflow tests; cfg2/cfg4/shard A/B (GHOSTM_K1_DEVOFF); cfg2 GPU busy
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5x
mkdir -p $O
cd $R
timeout -k 10 800 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_shards.py "tests/test_gpu_lds_poison.py::test_golden_variants_under_lds_poison[0xA5A5A5A5-kernels]" -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in on off on2 off2; do
  ENVV="GHOSTM_K1_DEVOFF=1"
  case $v in off*) ENVV="GHOSTM_K1_DEVOFF=0" ;; esac
  env $ENVV timeout -k 10 300 python3 -u bench.py --preset cfg2 --no-cpu --no-e2e --steps 20 --warmup 2 --workdir /tmp/r5x_cfg2 > $O/cfg2_$v.json 2> $O/cfg2_$v.log || { echo "cfg2 $v failed"; tail -5 $O/cfg2_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; print('cfg2', sys.argv[2], round(d['ms_per_step'],3), 'ms; K1', round(1e3*s['seed_device'],3), 'matches', d.get('full_output_matches_reference'))" $O/cfg2_$v.json $v
  env $ENVV timeout -k 10 300 python3 -u bench.py --queries 125000 --no-cpu --no-e2e --steps 10 --warmup 2 --workdir /tmp/r5x_shard > $O/shard_$v.json 2> $O/shard_$v.log || { echo "shard $v failed"; tail -5 $O/shard_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; print('shard', sys.argv[2], round(d['ms_per_step'],3), 'ms; K1', round(1e3*s['seed_device'],3))" $O/shard_$v.json $v
done
timeout -k 10 300 python3 -u bench.py --no-cpu --no-e2e --steps 3 --warmup 2 --workdir /tmp/r5x_cfg4 > $O/cfg4.json 2> $O/cfg4.log || { echo "cfg4 failed"; tail -5 $O/cfg4.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; print('cfg4', round(d['ms_per_step'],2), [round(x,1) for x in d['step_ms_rank0']], 'K1', round(1e3*s['seed_device'],2), 'matches', d.get('full_output_matches_reference'))" $O/cfg4.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/cfg2trace -o run -- python3 $R/tools/run_session.py --preset cfg2 --runs 6 --workdir /tmp/r5x_cfg2s > $O/cfg2trace.log 2>&1 || { echo "cfg2 trace failed"; tail -5 $O/cfg2trace.log; exit 1; }
python3 $R/tools/gpu_busy.py $O/cfg2trace/run_kernel_trace.csv --chunks 1 --skip 1 --gaps 30 > $O/cfg2_busy.txt
grep "^run" $O/cfg2_busy.txt
echo done
