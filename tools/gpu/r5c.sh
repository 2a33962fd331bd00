# round 5: host page-fault rates on the box, every GPU test (huge-page text
# buffers), cfg3/cfg2/cfg4 bench lines (end-to-end), and the one-time stall of a
# session's second run: host timelines without a profiler, plain and with
# HSA_ENABLE_INTERRUPT=0
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5c
mkdir -p $O
cd $R
g++ -O2 -pthread -o /tmp/pagefault tools/microbench/pagefault.cpp && timeout -k 10 120 /tmp/pagefault 64 > $O/pagefault.txt 2>&1 || { echo "pagefault failed"; exit 1; }
head -4 $O/pagefault.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for p in cfg3 cfg2 cfg4; do
  GHOSTM_TRACE=1 timeout -k 10 400 python3 -u bench.py --preset $p --no-cpu > $O/bench_$p.json 2> $O/bench_$p.log || { echo "bench $p failed"; tail -5 $O/bench_$p.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print(sys.argv[2], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms; e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e['runs_s']], d['full_output_matches_reference'], e.get('output_files_match_reference'))" $O/bench_$p.json $p
done
cd /tmp
GHOSTM_TRACE=1 timeout -k 10 300 python3 $R/tools/run_session.py --preset cfg4 --runs 3 --workdir /tmp/ghostm_bench_cfg4s > $O/stall_plain.log 2>&1 || { echo "stall plain failed"; tail -5 $O/stall_plain.log; exit 1; }
grep '^run ' $O/stall_plain.log
HSA_ENABLE_INTERRUPT=0 GHOSTM_TRACE=1 timeout -k 10 300 python3 $R/tools/run_session.py --preset cfg4 --runs 3 --workdir /tmp/ghostm_bench_cfg4s > $O/stall_nointr.log 2>&1 || { echo "stall nointr failed"; tail -5 $O/stall_nointr.log; exit 1; }
grep '^run ' $O/stall_nointr.log
echo done
