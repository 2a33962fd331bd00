# round 6 zk: the driver's round-end commands on the final tree: smoke(), then
# the default bench line (N = 1)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6zk
mkdir -p $O
cd $R
timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms; frac', round(r['frac'],3), 'traffic', r.get('traffic'), 'pmc', r['pmc_source']['used'], 'issue', round(r['issue_ceiling']['frac'],3), 'matches', d['full_output_matches_reference'])" $O/bench.json
echo done
