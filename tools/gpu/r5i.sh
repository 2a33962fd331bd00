# round 5: (1) pair-table K2 shape A/B on cfg2 (rows per lane S and workgroup
# size; GHOSTM_K2_PAIR_S / GHOSTM_K2_PAIR_BLOCK); (2) bench cfg4 timeline with
# the run-start idle probes and no settle (where the run-2 stall lands)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5i
mkdir -p $O
cd $R
for v in base s16 s16b s32b s8 base2; do
  ENVV="GHOSTM_K2_PAIR_S="
  case $v in
    s16) ENVV="GHOSTM_K2_PAIR_S=16" ;;
    s16b) ENVV="GHOSTM_K2_PAIR_S=16 GHOSTM_K2_PAIR_BLOCK=1024" ;;
    s32b) ENVV="GHOSTM_K2_PAIR_BLOCK=1024" ;;
    s8) ENVV="GHOSTM_K2_PAIR_S=8" ;;
  esac
  env $ENVV timeout -k 10 300 python3 -u bench.py --preset cfg2 --no-cpu --no-e2e --steps 10 --warmup 2 --workdir /tmp/r5i_cfg2 > $O/cfg2_$v.json 2> $O/cfg2_$v.log || { echo "cfg2 $v failed"; tail -5 $O/cfg2_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],3), 'ms; K2', round(1e3*s['score_device'],3), 'ms, frac', round(r['frac'],3), 'matches', d.get('full_output_matches_reference'))" $O/cfg2_$v.json $v
done
GHOSTM_TRACE=1 GHOSTM_BENCH_WARM_SETTLE_S=0 timeout -k 10 300 python3 -u bench.py --no-cpu --no-e2e --steps 2 --warmup 1 --workdir /tmp/r5i_cfg4 > $O/stall.json 2> $O/stall.log || { echo "stall failed"; tail -5 $O/stall.log; exit 1; }
python3 - $O/stall.log <<'PY'
import sys
runs, cur = [], None
for l in open(sys.argv[1]):
    p = l.split()
    if len(p) >= 4 and p[0] == "trace":
        t, m = float(p[1]), p[3]
        if m == "run":
            cur = {}
            runs.append(cur)
        if cur is not None and m not in cur:
            cur[m] = t
for r in runs:
    print({k: r[k] for k in ("run_idle", "carry_idle", "seed", "k1_idle", "seed_done", "run_end") if k in r})
PY
echo done
