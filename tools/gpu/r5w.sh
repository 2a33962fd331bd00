# round 5: next-segment K2 tasks built after the segment's K4/K3 are enqueued;
# head sizes on cfg2/cfg3; cfg2 GPU busy
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5w
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in def h131k h64k def2 h131k2 h64k2; do
  ENVV="GHOSTM_HEAD_CANDS_UNSET=1"
  case $v in h131k*) ENVV="GHOSTM_HEAD_CANDS=131072" ;; h64k*) ENVV="GHOSTM_HEAD_CANDS=65536" ;; esac
  env $ENVV timeout -k 10 300 python3 -u bench.py --preset cfg2 --no-cpu --no-e2e --steps 20 --warmup 2 --workdir /tmp/r5w_cfg2 > $O/cfg2_$v.json 2> $O/cfg2_$v.log || { echo "cfg2 $v failed"; tail -5 $O/cfg2_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('cfg2', sys.argv[2], round(d['ms_per_step'],3), 'ms; segments', d['config'].get('segments_per_rank_step'), 'matches', d.get('full_output_matches_reference'))" $O/cfg2_$v.json $v
done
for v in def h256k def2 h256k2; do
  ENVV="GHOSTM_HEAD_CANDS_UNSET=1"
  case $v in h256k*) ENVV="GHOSTM_HEAD_CANDS=262144" ;; esac
  env $ENVV timeout -k 10 300 python3 -u bench.py --preset cfg3 --no-cpu --no-e2e --steps 10 --warmup 2 --workdir /tmp/r5w_cfg3 > $O/cfg3_$v.json 2> $O/cfg3_$v.log || { echo "cfg3 $v failed"; tail -5 $O/cfg3_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('cfg3', sys.argv[2], round(d['ms_per_step'],3), 'ms; segments', d['config'].get('segments_per_rank_step'), 'matches', d.get('full_output_matches_reference'))" $O/cfg3_$v.json $v
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/cfg2trace -o run -- python3 $R/tools/run_session.py --preset cfg2 --runs 6 --workdir /tmp/r5w_cfg2s > $O/cfg2trace.log 2>&1 || { echo "cfg2 trace failed"; tail -5 $O/cfg2trace.log; exit 1; }
python3 $R/tools/gpu_busy.py $O/cfg2trace/run_kernel_trace.csv --chunks 1 --skip 1 --gaps 30 > $O/cfg2_busy.txt
grep "^run" $O/cfg2_busy.txt
echo done
