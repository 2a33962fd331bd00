# round 5: cfg5 profile (K3 at 0.28 of the d3 peak against cfg4's 0.57)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 bash tools/profile.sh r5cfg5 cfg5 > gpurun_out/profile_r5_cfg5.log 2>&1 || { echo "cfg5 profile failed"; tail -20 gpurun_out/profile_r5_cfg5.log; exit 1; }
tail -2 gpurun_out/profile_r5_cfg5.log
echo done
