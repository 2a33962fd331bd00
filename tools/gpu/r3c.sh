# K1 gather/filter rework: scale parity tests, then same-box A/B against the previous build
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -v --timeout 300 --timeout-method thread > gpurun_out/r3c_scale.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
AB_ROUNDS=2 timeout -k 10 700 bash tools/ab.sh prev > gpurun_out/r3c_ab.txt 2>&1
echo "ab rc=$?"
