# K1 variant: K1 parity tests, then same-box A/B against the previous build
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -v -k "k1 or classes or class3 or full_workload" --timeout 300 --timeout-method thread > gpurun_out/r3d_scale.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
AB_ROUNDS=3 timeout -k 10 900 bash tools/ab.sh prev > gpurun_out/r3d_ab.txt 2>&1
echo "ab rc=$?"
