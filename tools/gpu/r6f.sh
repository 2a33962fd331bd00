# round 6 f: K1 wave scans (phase 0 and the emission): the K1 parity groups, then
# a same-box cfg4 A/B against the block scans (ab_libs/nowavescan), then the
# e2e host-thread A/B (r6e)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6f
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "k1 or probe or golden" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_ROUNDS=2 timeout -k 10 900 bash tools/ab.sh nowavescan > $O/ab.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
bash tools/gpu/r6e.sh
