# round 4: isolate the syn_small/b20_t1 parity failure by kernel variant
export TMPDIR=/tmp
mkdir -p gpurun_out/r4e
T="tests/test_gpu_parity.py::test_gpu_matches_reference_golden[syn_small/b20_t1]"
for v in "X=1" "GHOSTM_K2=swar16" "GHOSTM_K2=unit GHOSTM_K2_TASKS=consecutive" "GHOSTM_K2=unit GHOSTM_K2_TASKS=paired" "GHOSTM_K3_SCAN=f16frame" "GHOSTM_K4=thread" "GHOSTM_MERGE=host" "GHOSTM_K3_STRIPS=0"; do
  env $v timeout -k 10 120 python -m pytest "$T" -x -q --timeout 100 > gpurun_out/r4e/t.log 2>&1
  echo "$v -> rc=$?"
done
