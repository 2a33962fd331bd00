export TMPDIR=/tmp
mkdir -p gpurun_out/r4t
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4t/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r4t/tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu/r4q.sh
