# K2 on its own stream (overlapping the previous segment's K4/K3): the whole -m gpu suite, then A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3u_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
AB_ROUNDS=2 bash tools/ab.sh prev > gpurun_out/r3u_ab.log 2>&1
echo "ab rc=$?"
cat gpurun_out/r3u_ab.log
