# round 5: tail floor capped at 16 K queries' worth of candidates: tests, then
# cfg5 (against the 1 M floor), cfg4, the shard, cfg3, cfg2
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ak
mkdir -p $O
cd $R
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  env $3 timeout -k 10 300 python3 -u bench.py $2 --no-cpu --no-e2e --warmup 2 --workdir /tmp/r5ak_$1 > $O/$1_$4.json 2> $O/$1_$4.log || { echo "$1 $4 failed"; tail -5 $O/$1_$4.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; print(sys.argv[2], round(d['ms_per_step'],2), 'ms; K3', round(1e3*s['traceback_device'],2), 'segments', d['config'].get('segments_per_rank_step'), 'matches', d.get('full_output_matches_reference'))" $O/$1_$4.json "$1 $4"
}
run cfg5 "--preset cfg5 --steps 6" "X=1" new
run cfg5 "--preset cfg5 --steps 6" "GHOSTM_TAIL_CANDS=1048576" old
run cfg5 "--preset cfg5 --steps 6" "X=1" new2
run cfg5 "--preset cfg5 --steps 6" "GHOSTM_TAIL_CANDS=1048576" old2
run cfg4 "--steps 3" "X=1" new
run shard "--queries 125000 --steps 10" "X=1" new
run cfg3 "--preset cfg3 --steps 10" "X=1" new
run cfg2 "--preset cfg2 --steps 10" "X=1" new
echo done
