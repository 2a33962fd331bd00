# round 5: (1) the run-2 stall with the run/chunk-start stream drains on and
# off (GHOSTM_RUN_SYNC=0), no trace, no settle; (2) pair-table K2 with the
# stride-27 table (two workgroups per CU) against the default, cfg2
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5j
mkdir -p $O
cd $R
for v in sync nosync sync2 nosync2; do
  ENVV="GHOSTM_RUN_SYNC=1"
  case $v in nosync*) ENVV="GHOSTM_RUN_SYNC=0" ;; esac
  env $ENVV GHOSTM_BENCH_WARM_SETTLE_S=0 timeout -k 10 300 python3 -u bench.py --no-cpu --no-e2e --steps 3 --warmup 1 --workdir /tmp/r5j_cfg4 > $O/cfg4_$v.json 2> $O/cfg4_$v.log || { echo "cfg4 $v failed"; tail -5 $O/cfg4_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'steps', [round(x,1) for x in d['step_ms_rank0']], 'matches', d.get('full_output_matches_reference'))" $O/cfg4_$v.json $v
done
for v in base st27_s32 st27_s16 st27_s8 st27_s8b base2; do
  ENVV="GHOSTM_K2_PAIR_S="
  case $v in
    st27_s32) ENVV="GHOSTM_K2_PAIR_STRIDE=27" ;;
    st27_s16) ENVV="GHOSTM_K2_PAIR_S=16 GHOSTM_K2_PAIR_STRIDE=27" ;;
    st27_s8) ENVV="GHOSTM_K2_PAIR_S=8 GHOSTM_K2_PAIR_STRIDE=27 GHOSTM_K2_PAIR_BLOCK=768" ;;
    st27_s8b) ENVV="GHOSTM_K2_PAIR_S=8 GHOSTM_K2_PAIR_STRIDE=27 GHOSTM_K2_PAIR_BLOCK=896" ;;
  esac
  env $ENVV timeout -k 10 300 python3 -u bench.py --preset cfg2 --no-cpu --no-e2e --steps 10 --warmup 2 --workdir /tmp/r5j_cfg2 > $O/cfg2_$v.json 2> $O/cfg2_$v.log || { echo "cfg2 $v failed"; tail -5 $O/cfg2_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],3), 'ms; K2', round(1e3*s['score_device'],3), 'ms, frac', round(r['frac'],3), 'matches', d.get('full_output_matches_reference'))" $O/cfg2_$v.json $v
done
echo done
