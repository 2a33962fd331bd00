# round 6 zf: K2's untested columns take their END test from the previous
# column's look-ahead (unit and restart-level kernels): K2 parity (golden,
# forced encodings, sparse rows, restart levels, LDS poison), then same-box A/B
# against ab_libs/prev (-DGHOSTM_K2_LAREUSE=0) at cfg4 and cfg2
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6zf
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lds_poison.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "restart_levels or sparse_rows or forced_score or matches_reference_golden or pair_k2 or poison" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_ROUNDS=3 timeout -k 10 900 bash tools/ab.sh prev > $O/ab_cfg4.txt 2>&1 || { echo "ab cfg4 failed"; tail -20 $O/ab_cfg4.txt; exit 1; }
cat $O/ab_cfg4.txt
rm -rf gpurun_out/ab
AB_ROUNDS=3 AB_STEPS=20 AB_ARGS="--preset cfg2" timeout -k 10 900 bash tools/ab.sh prev > $O/ab_cfg2.txt 2>&1 || { echo "ab cfg2 failed"; tail -20 $O/ab_cfg2.txt; exit 1; }
cat $O/ab_cfg2.txt
echo done
