# the whole -m gpu suite, then smoke()
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3h_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3h_smoke.log 2>&1
echo "smoke rc=$?"
