# round 6 p: final checkpoint part 1: the whole GPU suite, then the cfg4 profile
# (kernel stats + PMC, recorded with the library's source hash)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6p
mkdir -p $O
cd $R
GHOSTM_TEST_OUT=$O/rccl_world1.json timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd $R && timeout -k 10 900 bash tools/profile.sh r6p cfg4 > $O/profile_cfg4.log 2>&1 || { echo "profile failed"; tail -20 $O/profile_cfg4.log; exit 1; }
tail -2 $O/profile_cfg4.log
echo done
