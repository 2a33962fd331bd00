# round 4: GPU tests after the loader changes (staged uploads, name tables,
# parallel query lengths), then end-to-end runs with host traces
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4m
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4m/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r4m/tests.log
[ $rc -eq 0 ] || exit $rc
for p in cfg3 cfg4 cfg2 cfg5; do
  mkdir -p /tmp/e_$p
  GHOSTM_TRACE=1 timeout -k 10 300 python3 bench.py --preset $p --steps 3 --warmup 1 --no-cpu --workdir /tmp/e_$p > gpurun_out/r4m/e2e_$p.json 2> gpurun_out/r4m/e2e_$p.log || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print(sys.argv[1].split('/')[-1], 'step', round(d['ms_per_step'],2), 'value', round(d['value']/1e6,1), 'e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e['runs_s']], e.get('output_files_match_reference'), d['full_output_matches_reference'])" gpurun_out/r4m/e2e_$p.json
done
