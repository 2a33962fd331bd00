# round 5: lazy file mappings (no MAP_POPULATE) and the word-wise query length:
# tests, then end to end with GHOSTM_MAP_POPULATE=0/1 on cfg2, cfg3, cfg4
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ag
mkdir -p $O
cd $R
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_shards.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for p in cfg2 cfg3; do
  for v in lazy pop lazy2 pop2; do
    ENVV="GHOSTM_MAP_POPULATE=0"; case $v in pop*) ENVV="GHOSTM_MAP_POPULATE=1" ;; esac
    env $ENVV timeout -k 10 300 python3 -u bench.py --preset $p --no-cpu --steps 2 --warmup 1 --workdir /tmp/r5ag_$p > $O/${p}_$v.json 2> $O/${p}_$v.log || { echo "$p $v failed"; tail -5 $O/${p}_$v.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print(sys.argv[2], sys.argv[3], 'e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e['runs_s']], 'create', [round(x*1e3,2) for x in e['create_s']], 'ok', e.get('output_files_match_reference'))" $O/${p}_$v.json $p $v
  done
done
for v in lazy pop; do
  ENVV="GHOSTM_MAP_POPULATE=0"; case $v in pop*) ENVV="GHOSTM_MAP_POPULATE=1" ;; esac
  env $ENVV timeout -k 10 400 python3 -u bench.py --preset cfg4 --no-cpu --steps 1 --warmup 1 --workdir /tmp/r5ag_cfg4 > $O/cfg4_$v.json 2> $O/cfg4_$v.log || { echo "cfg4 failed"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print('cfg4', sys.argv[2], 'e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e['runs_s']], 'create', [round(x*1e3,1) for x in e['create_s']])" $O/cfg4_$v.json $v
done
echo done
