# round 4: another box's cfg4 bench line (default settings), for the box-to-box spread
export TMPDIR=/tmp
O=gpurun_out/r4au
mkdir -p $O
timeout -k 10 600 python3 -u bench.py --preset cfg4 > $O/bench_cfg4.json 2> $O/bench_cfg4.log || { echo "bench failed"; tail -5 $O/bench_cfg4.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print(round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms; e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e['runs_s']], d['full_output_matches_reference'])" $O/bench_cfg4.json
