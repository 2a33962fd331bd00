# round 6 h: the whole GPU suite (checkpoint)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6h
mkdir -p $O
cd $R
rm -rf ab_libs
GHOSTM_TEST_OUT=$O/rccl_world1.json timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo done
