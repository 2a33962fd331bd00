# full-size workloads: unsharded pins (incl. the cfg5 gap sweep) and the sharded cfg4 / cfg3 runs
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -v -k "full_workload" --timeout 400 --timeout-method thread > gpurun_out/r3o_tests.log 2>&1
echo "pytest rc=$?"
