# final check of the session's tree: the whole -m gpu suite and smoke()
export TMPDIR=/tmp
O=gpurun_out/r3z1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke rc=$?"; tail -1 $O/smoke.log
