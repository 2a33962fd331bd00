# round 6 zn: evidence on the final library (CLI fast exit): the whole GPU suite, then the
# cfg4/cfg3/cfg5/cfg2 profiles (kernel stats + PMC with the library's hash)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6zn
mkdir -p $O
cd $R
GHOSTM_TEST_OUT=$O/rccl_world1.json timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for p in cfg4 cfg3 cfg5 cfg2; do
  timeout -k 10 700 bash tools/profile.sh r6zn_$p $p > $O/profile_$p.log 2>&1 || { echo "profile $p failed"; tail -20 $O/profile_$p.log; exit 1; }
  echo "$p profiled"
done
echo done
