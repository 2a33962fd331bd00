# round 5: the predecessor loads for classes 1-2 only (class 0 keeps the lane-0
# load and DPP: libghostm_hip_pc512): poison groups, parity, cfg2 and cfg4 A/B
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ay
mkdir -p $O /tmp/r5ay_data
cd $R
for g in golden kernels; do
  GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_ppc512.so GHOSTM_LDS_POISON_PATTERN=0xA5A5A5A5 timeout -k 10 150 python3 tests/lds_poison_child.py $g /tmp/r5ay_data > $O/poison_$g.out 2> $O/poison_$g.err || { echo "poison $g failed"; tail -c 600 $O/poison_$g.out; exit 1; }
  echo "poison $g: $(tail -c 120 $O/poison_$g.out)"
done
GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_pc512.so timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_ROUNDS=3 AB_STEPS=10 AB_ARGS="--preset cfg2" timeout -k 10 600 bash tools/ab.sh pc512 > $O/ab_cfg2.txt 2>&1 || { echo "ab cfg2 failed"; tail -20 $O/ab_cfg2.txt; exit 1; }
cat $O/ab_cfg2.txt
AB_ROUNDS=2 AB_STEPS=3 timeout -k 10 600 bash tools/ab.sh pc512 > $O/ab_cfg4.txt 2>&1 || { echo "ab cfg4 failed"; tail -20 $O/ab_cfg4.txt; exit 1; }
cat $O/ab_cfg4.txt
echo done
