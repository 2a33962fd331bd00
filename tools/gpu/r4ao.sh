# round 4: GPU tests with the adaptive tail segment, then cfg2 / cfg3 / cfg4 step times
export TMPDIR=/tmp
O=gpurun_out/r4ao
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for p in cfg2 cfg3 cfg4; do
  timeout -k 10 300 python3 bench.py --preset $p --steps 5 --warmup 1 --no-cpu --no-e2e --workdir /tmp/ao_$p > $O/$p.json 2> $O/$p.log || { echo "$p failed"; tail -3 $O/$p.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), 'ms', d['config']['segments_per_rank_step'], 'segments', d['full_output_matches_reference'])" $O/$p.json $p
done
