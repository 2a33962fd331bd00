# round 5: the 125 K-query shard (N = 8's per-rank work): K3 longest-first
# (libghostm_hip_lpt.so) and the tail floor (GHOSTM_TAIL_CANDS) against the default
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ai
mkdir -p $O
cd $R
run() {
  env $2 timeout -k 10 300 python3 -u bench.py --queries 125000 --no-cpu --no-e2e --steps 10 --warmup 2 --workdir /tmp/r5ai_shard > $O/$1.json 2> $O/$1.log || { echo "$1 failed"; tail -5 $O/$1.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; print(sys.argv[2], round(d['ms_per_step'],3), 'ms; K1', round(1e3*s['seed_device'],2), 'K2', round(1e3*s['score_device'],2), 'K3', round(1e3*s['traceback_device'],2), 'segments', d['config'].get('segments_per_rank_step'))" $O/$1.json $1
}
run def "X=1"
run lpt "GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_lpt.so"
run tail512k "GHOSTM_TAIL_CANDS=524288"
run tail2m "GHOSTM_TAIL_CANDS=2097152"
run def2 "X=1"
run lpt2 "GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_lpt.so"
run tail512k2 "GHOSTM_TAIL_CANDS=524288"
run tail2m2 "GHOSTM_TAIL_CANDS=2097152"
echo done
