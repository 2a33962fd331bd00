# round 5: (1) parity after the device block cache and the run-start drains;
# (2) end to end with the block cache on and off (GHOSTM_DEV_POOL_MB=0), cfg2
# and cfg3; (3) pair-table K2 with 16 against 32 rows per lane, alternating
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5k
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity failed"; tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for p in cfg2 cfg3; do
  for v in pool nopool pool2 nopool2; do
    ENVV="GHOSTM_DEV_POOL_MB=8192"
    case $v in nopool*) ENVV="GHOSTM_DEV_POOL_MB=0" ;; esac
    env $ENVV timeout -k 10 300 python3 -u bench.py --preset $p --no-cpu --steps 4 --warmup 1 --workdir /tmp/r5k_$p > $O/${p}_$v.json 2> $O/${p}_$v.log || { echo "$p $v failed"; tail -5 $O/${p}_$v.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],2), 'ms; e2e', round(e['value']/1e6,1), 'runs', [round(x*1e3,1) for x in e['runs_s']], 'create', [round(x*1e3,2) for x in e['create_s']], 'ok', e.get('output_files_match_reference'))" $O/${p}_$v.json $p $v
  done
done
for v in s32 s16 s32b s16b; do
  ENVV="GHOSTM_K2_PAIR_S=32"
  case $v in s16*) ENVV="GHOSTM_K2_PAIR_S=16" ;; esac
  env $ENVV timeout -k 10 300 python3 -u bench.py --preset cfg2 --no-cpu --no-e2e --steps 20 --warmup 2 --workdir /tmp/r5k_cfg2 > $O/cfg2_$v.json 2> $O/cfg2_$v.log || { echo "cfg2 $v failed"; tail -5 $O/cfg2_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],3), 'ms; K2', round(1e3*s['score_device'],3), 'ms, frac', round(r['frac'],3), 'matches', d.get('full_output_matches_reference'))" $O/cfg2_$v.json $v
done
echo done
