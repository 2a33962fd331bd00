# round 5, first call: every GPU test (incl. the RCCL world-1 bench test and the
# LDS-poison runs), the cfg4 bench line, the cfg4 kernel trace, and a run
# without the warmup settle (per-step times show the one-time stall)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5a
mkdir -p $O
cd $R
GHOSTM_TEST_OUT=$O timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python3 -u bench.py --no-cpu > $O/bench_cfg4.json 2> $O/bench_cfg4.log || { echo "bench failed"; tail -5 $O/bench_cfg4.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; k3=d['roofline_k3']; print('cfg4', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms; K1', round(d['roofline_k1']['ms_per_step'],2), 'K3', round(k3['ms_per_step'],2), 'scan', round(k3['scan']['ms_per_step'],2), 'key', round(k3['key_dp']['ms_per_step'],2), 'k3 frac', round(k3['frac'],3), 'K2 frac', round(d['roofline']['frac'],4), '; e2e', round(e['value']/1e6,1), d['full_output_matches_reference'], [round(x) for x in d['step_ms_rank0']])" $O/bench_cfg4.json
GHOSTM_BENCH_WARM_SETTLE_S=0 timeout -k 10 300 python3 -u bench.py --no-cpu --no-e2e --steps 6 --warmup 1 --workdir /tmp/r5a_cfg4 > $O/bench_nosettle.json 2> $O/bench_nosettle.log || { echo "nosettle bench failed"; tail -5 $O/bench_nosettle.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('no settle', round(d['ms_per_step'],2), [round(x,1) for x in d['step_ms_rank0']])" $O/bench_nosettle.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --workdir /tmp/r5a_cfg4 > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
echo done
