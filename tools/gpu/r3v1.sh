# closing set for the session: the whole -m gpu suite and smoke(), then rocprofv3
# stats + PMC (r3f), the cfg4 headline bench with CPU baselines, cfg3/cfg5/cfg2
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3v1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 1000 bash tools/profile.sh r3f > $O/profile.log 2>&1 || exit $?
cp $R/profiles/pmc_traffic.json $R/profiles/r3f_pmc.json $R/profiles/r3f_kernel_stats.csv $O/
cd $R
timeout -k 10 600 python bench.py > $O/bench_cfg4.json 2> $O/bench_cfg4.err || exit $?
for p in cfg3 cfg5 cfg2; do
  timeout -k 10 300 python bench.py --preset $p --no-cpu > $O/bench_$p.json 2> $O/bench_$p.err || exit $?
done
echo done
