# round 5 profiles: tools/profile.sh (kernel trace + stats, FETCH/WRITE PMC
# passes, SQ issue and LDS passes) for cfg4 and cfg2
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 1000 bash tools/profile.sh r5 cfg4 > gpurun_out/profile_r5_cfg4.log 2>&1 || { echo "cfg4 profile failed"; tail -20 gpurun_out/profile_r5_cfg4.log; exit 1; }
tail -2 gpurun_out/profile_r5_cfg4.log
timeout -k 10 600 bash tools/profile.sh r5cfg2 cfg2 > gpurun_out/profile_r5_cfg2.log 2>&1 || { echo "cfg2 profile failed"; tail -20 gpurun_out/profile_r5_cfg2.log; exit 1; }
tail -2 gpurun_out/profile_r5_cfg2.log
echo done
