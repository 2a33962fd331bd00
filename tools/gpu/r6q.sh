# round 6 q: final checkpoint part 2: cfg3, cfg5 and cfg2 profiles (kernel stats +
# PMC with the library's source hash)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6q
mkdir -p $O
cd $R
for p in cfg3 cfg5 cfg2; do
  timeout -k 10 600 bash tools/profile.sh r6q_$p $p > $O/profile_$p.log 2>&1 || { echo "profile $p failed"; tail -20 $O/profile_$p.log; exit 1; }
  echo "$p profiled"
done
echo done
