# K1 emission without lookups for bins whose b + 1 cell the presence bitmap never saw: K1 parity, then A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -v -k "k1 or classes or class3 or full_workload or batch_cuts or golden" --timeout 300 --timeout-method thread > gpurun_out/r3l_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
AB_ROUNDS=3 timeout -k 10 900 bash tools/ab.sh prev > gpurun_out/r3l_ab.txt 2>&1
echo "ab rc=$?"
