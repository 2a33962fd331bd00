# round 5: formatting buffers cached across sessions: tests, then end to end on
# cfg3/cfg2 with the cache on and off (GHOSTM_PART_CACHE_MB=0)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5y
mkdir -p $O
cd $R
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_shards.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for p in cfg3 cfg2; do
  for v in cache nocache cache2 nocache2; do
    ENVV="GHOSTM_PART_CACHE_MB=4096"
    case $v in nocache*) ENVV="GHOSTM_PART_CACHE_MB=0" ;; esac
    env $ENVV timeout -k 10 300 python3 -u bench.py --preset $p --no-cpu --steps 4 --warmup 2 --workdir /tmp/r5y_$p > $O/${p}_$v.json 2> $O/${p}_$v.log || { echo "$p $v failed"; tail -5 $O/${p}_$v.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],2), 'ms; e2e', round(e['value']/1e6,1), 'runs', [round(x*1e3,1) for x in e['runs_s']], 'create', [round(x*1e3,1) for x in e['create_s']], 'ok', e.get('output_files_match_reference'))" $O/${p}_$v.json $p $v
  done
done
echo done
