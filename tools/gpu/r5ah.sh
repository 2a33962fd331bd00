# round 5: K1 slot of 512 candidates (fewer queries redone by the merge kernel):
# tests, then K1 times against the 256 build on cfg5, cfg4, cfg2
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ah
mkdir -p $O
cd $R
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for p in cfg5 cfg4 cfg2; do
  STEPS=6; [ $p = cfg4 ] && STEPS=3
  for v in s512 s256 s512b s256b; do
    LIB=""; case $v in s256*) LIB="GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_slot256.so" ;; esac
    env $LIB timeout -k 10 300 python3 -u bench.py --preset $p --no-cpu --no-e2e --steps $STEPS --warmup 2 --workdir /tmp/r5ah_$p > $O/${p}_$v.json 2> $O/${p}_$v.log || { echo "$p $v failed"; tail -5 $O/${p}_$v.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],2), 'ms; K1', round(1e3*s['seed_device'],3), 'matches', d.get('full_output_matches_reference'))" $O/${p}_$v.json $p $v
  done
done
echo done
