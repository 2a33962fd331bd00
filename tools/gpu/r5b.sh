# round 5: K1 pass-1 batch A/B (same box), a HIP runtime + kernel trace of a
# session run three times back to back (the one-time stall of the second run),
# and the cfg3 bench with host timelines (end-to-end breakdown)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b
mkdir -p $O
cd $R
AB_ROUNDS=2 timeout -k 10 700 bash tools/ab.sh k1batch k3rowoff > $O/ab.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt | tail -6
cd /tmp
GHOSTM_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/stall -o run -- python3 $R/tools/run_session.py --preset cfg4 --runs 3 --workdir /tmp/ghostm_ab_data > $O/stall.log 2>&1 || { echo "stall trace failed"; tail -20 $O/stall.log; exit 1; }
grep '^run ' $O/stall.log
cd $R
GHOSTM_TRACE=1 timeout -k 10 300 python3 -u bench.py --preset cfg3 --no-cpu --steps 5 > $O/bench_cfg3.json 2> $O/bench_cfg3.log || { echo "cfg3 bench failed"; tail -5 $O/bench_cfg3.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print('cfg3', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms; e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e['runs_s']], d['full_output_matches_reference'])" $O/bench_cfg3.json
echo done
