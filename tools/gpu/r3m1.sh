# K4: a third k_merge_wave tier (groups of <= 256 keys, eight workgroups per CU):
# parity, then kernel traces of the new and the previous library (prev) on cfg4
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3m1
mkdir -p $O /tmp/ghostm_ab_data
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
cd /tmp
B="$R/bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --workdir /tmp/ghostm_ab_data"
for i in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new$i -o run -- python3 $B > $O/new$i.log 2>&1 || exit $?
  GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_prev.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $O/prev$i -o run -- python3 $B > $O/prev$i.log 2>&1 || exit $?
done
for f in $O/*/run_kernel_stats.csv; do echo $f; grep -h "k_merge_wave" $f | cut -c1-120; done
