# round 5: the whole GPU suite after the pair-table K2 default of 16 rows per
# lane, the device block cache and the run-start drains; then cfg2 and cfg4
# bench lines
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5l
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u bench.py --preset cfg2 --no-cpu --steps 20 --warmup 2 --workdir /tmp/r5l_cfg2 > $O/cfg2.json 2> $O/cfg2.log || { echo "cfg2 failed"; tail -5 $O/cfg2.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; r=d['roofline']; e=d['end_to_end']; print('cfg2', round(d['ms_per_step'],3), 'ms; K2', round(1e3*s['score_device'],3), 'ms, frac', round(r['frac'],3), 'e2e', round(e['value']/1e6,1), 'matches', d.get('full_output_matches_reference'))" $O/cfg2.json
timeout -k 10 300 python3 -u bench.py --no-cpu --no-e2e --steps 3 --warmup 1 --workdir /tmp/r5l_cfg4 > $O/cfg4.json 2> $O/cfg4.log || { echo "cfg4 failed"; tail -5 $O/cfg4.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('cfg4', round(d['ms_per_step'],2), d['step_ms_rank0'], 'matches', d.get('full_output_matches_reference'))" $O/cfg4.json
echo done
