# round 6 w: K1 emission look-ups queued and shared by the block: K1/golden/
# poison/full-workload parity, then a same-box cfg4 A/B against ab_libs/noemitq
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6w
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_lds_poison.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "k1 or probe or golden or poison or full_workload" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_ROUNDS=3 timeout -k 10 900 bash tools/ab.sh noemitq > $O/ab.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
echo done
