# round 5: tail floor 2 M (GHOSTM_TAIL_CANDS) against the default 1 M on cfg4 and cfg3
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5aj
mkdir -p $O
cd $R
for p in cfg4 cfg3; do
  STEPS=10; [ $p = cfg4 ] && STEPS=3
  for v in def t2m def2 t2m2; do
    ENVV="X=1"; case $v in t2m*) ENVV="GHOSTM_TAIL_CANDS=2097152" ;; esac
    env $ENVV timeout -k 10 300 python3 -u bench.py --preset $p --no-cpu --no-e2e --steps $STEPS --warmup 2 --workdir /tmp/r5aj_$p > $O/${p}_$v.json 2> $O/${p}_$v.log || { echo "$p $v failed"; tail -5 $O/${p}_$v.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],2), 'ms; K3', round(1e3*s['traceback_device'],2), 'segments', d['config'].get('segments_per_rank_step'), 'matches', d.get('full_output_matches_reference'))" $O/${p}_$v.json $p $v
  done
done
echo done
