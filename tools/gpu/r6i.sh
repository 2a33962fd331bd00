# round 6 i: the sparse rows K2 (k_score16f<16, true>, seven 27-row profiles per
# block): golden parity forced, poison, then cfg2 A/B against the pair kernel
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6i
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lds_poison.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "sparse or pair or poison" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for v in pair rows; do
    GHOSTM_K2_SPARSE=$v timeout -k 10 300 python3 -u bench.py --preset cfg2 --steps 10 --warmup 2 --no-cpu --no-e2e --workdir /tmp/r6i_cfg2 > $O/cfg2_${v}_$i.json 2> $O/cfg2_${v}_$i.log || { echo "bench $v failed"; tail -5 $O/cfg2_${v}_$i.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],3), 'K2', round(1e3*s['score_device'],3), 'frac', round(r['frac'],3), r['launches_per_step'], d['full_output_matches_reference'])" $O/cfg2_${v}_$i.json $v
  done
done
echo done
