# round 4: bisect the syn_small/b20_t1 failure by library build (GHOSTM_LIB_PATH)
export TMPDIR=/tmp
mkdir -p gpurun_out/r4f
R=$GRAFT_REPO_ROOT
T="tests/test_gpu_parity.py::test_gpu_matches_reference_golden[syn_small/b20_t1]"
for i in 1 2 3; do
  timeout -k 10 120 python -m pytest "$T" -x -q --timeout 100 > gpurun_out/r4f/cur$i.log 2>&1; echo "current run $i -> rc=$?"
done
for v in noscan nok4 nopairs; do
  GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_$v.so timeout -k 10 120 python -m pytest "$T" -x -q --timeout 100 > gpurun_out/r4f/$v.log 2>&1; echo "$v -> rc=$?"
done
GHOSTM_K2_TASKS=consecutive GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_r3.so timeout -k 10 120 python -m pytest "$T" -x -q --timeout 100 > gpurun_out/r4f/r3.log 2>&1; echo "r3 kernels -> rc=$?"
GHOSTM_K2_TASKS=consecutive timeout -k 10 120 python -m pytest "$T" -x -q --timeout 100 > gpurun_out/r4f/cur_consec.log 2>&1; echo "current consecutive -> rc=$?"
grep -h "^E.*+ " gpurun_out/r4f/*.log
