# round 4: host timelines of cfg4's end-to-end sessions (create -> file written)
export TMPDIR=/tmp
O=gpurun_out/r4ar
mkdir -p $O
GHOSTM_TRACE=1 timeout -k 10 400 python3 bench.py --preset cfg4 --steps 1 --warmup 1 --no-cpu --workdir /tmp/ar > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print(round(d['ms_per_step'],1), [round(x*1e3,1) for x in e['runs_s']])" $O/bench.json
