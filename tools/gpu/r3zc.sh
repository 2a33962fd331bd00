# k_finalize: 32-bit slot math, one counter atomic per workgroup: parity, then A/B with a kernel trace of each
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_shards.py -q --timeout 300 --timeout-method thread > gpurun_out/r3zc_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
R=$GRAFT_REPO_ROOT
mkdir -p /tmp/ghostm_ab_data gpurun_out/r3zc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3zc/A -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --workdir /tmp/ghostm_ab_data > $R/gpurun_out/r3zc/A.log 2>&1 || exit $?
GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_prev.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3zc/prev -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --workdir /tmp/ghostm_ab_data > $R/gpurun_out/r3zc/prev.log 2>&1 || exit $?
grep -h "k_finalize\|k_records\|k_merge_wave" $R/gpurun_out/r3zc/*/run_kernel_stats.csv
