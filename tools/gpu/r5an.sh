# round 5: PMC profiles of the current code (cfg4 and cfg2) for the bench lines' traffic fields
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 bash tools/profile.sh r5an cfg4 > gpurun_out/r5an_cfg4.log 2>&1 || { echo "cfg4 profile failed"; tail -20 gpurun_out/r5an_cfg4.log; exit 1; }
tail -3 gpurun_out/r5an_cfg4.log
timeout -k 10 600 bash tools/profile.sh r5an_cfg2 cfg2 > gpurun_out/r5an_cfg2.log 2>&1 || { echo "cfg2 profile failed"; tail -20 gpurun_out/r5an_cfg2.log; exit 1; }
tail -3 gpurun_out/r5an_cfg2.log
echo done
