# round 4: rocprofv3 kernel stats + PMC for cfg5 and cfg2 (final tree)
export TMPDIR=/tmp
O=gpurun_out/r4as
mkdir -p $O
for p in cfg5 cfg2; do
  bash tools/profile.sh r4as_$p $p > $O/prof_$p.log 2>&1 || { echo "profile $p failed"; tail -5 $O/prof_$p.log; exit 1; }
  tail -1 $O/prof_$p.log | cut -c1-200
done
cp profiles/r4as_* profiles/pmc_traffic_cfg5.json profiles/pmc_traffic_cfg2.json $O/ 2>/dev/null
echo done
