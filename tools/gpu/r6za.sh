# round 6 za: K2 restart levels and window-sorted lanes (k_score16f 16-bit rows): K2 parity
# (restart-level cases, every golden variant with the sparse and pair kernels
# forced, forced encodings, golden), then A/B against GHOSTM_K2_LEVELS=0 on cfg2
# and cfg3, alternating
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6za
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "restart_levels or sparse_rows or forced_score or matches_reference_golden or pair_k2" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in 1 0; do
    GHOSTM_K2_LEVELS=$v timeout -k 10 300 python3 -u bench.py --preset cfg2 --steps 20 --warmup 3 --no-cpu --no-e2e --workdir /tmp/r6za_cfg2 > $O/cfg2_${v}_$i.json 2> $O/cfg2_${v}_$i.log || { echo "cfg2 $v failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; print('cfg2 levels', sys.argv[2], round(d['ms_per_step'],3), 'K2', round(1e3*s['score_device'],3), 'frac', round(d['roofline']['frac'],3), d['full_output_matches_reference'])" $O/cfg2_${v}_$i.json $v
    GHOSTM_K2_LEVELS=$v timeout -k 10 300 python3 -u bench.py --preset cfg3 --steps 10 --warmup 2 --no-cpu --no-e2e --workdir /tmp/r6za_cfg3 > $O/cfg3_${v}_$i.json 2> $O/cfg3_${v}_$i.log || { echo "cfg3 $v failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; print('cfg3 levels', sys.argv[2], round(d['ms_per_step'],3), 'K2', round(1e3*s['score_device'],3), d['full_output_matches_reference'])" $O/cfg3_${v}_$i.json $v
  done
done
echo done
