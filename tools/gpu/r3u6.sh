# closing measurement after the unit K2 kernel: rocprofv3 stats + PMC, the cfg4 headline
# bench with CPU baselines, then cfg3 / cfg5 / cfg2 without
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3u6
timeout -k 10 1000 bash tools/profile.sh r3e > $R/gpurun_out/r3u6/profile.log 2>&1 || exit $?
cp $R/profiles/pmc_traffic.json $R/profiles/r3e_pmc.json $R/profiles/r3e_kernel_stats.csv $R/gpurun_out/r3u6/
cd $R
timeout -k 10 600 python bench.py > gpurun_out/r3u6/bench_cfg4.json 2> gpurun_out/r3u6/bench_cfg4.err || exit $?
for p in cfg3 cfg5 cfg2; do
  timeout -k 10 300 python bench.py --preset $p --no-cpu > gpurun_out/r3u6/bench_$p.json 2> gpurun_out/r3u6/bench_$p.err || exit $?
done
echo done
