# round 4: how often syn_small -b 20 -t 1 -y 2 differs, and where (current build, r3 kernels)
export TMPDIR=/tmp
mkdir -p gpurun_out/r4g
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python3 tools/repeat_variant.py syn_small "-b 20 -t 1 -y 2" 20 > gpurun_out/r4g/cur.txt 2>&1; echo "cur rc=$?"; tail -30 gpurun_out/r4g/cur.txt
GHOSTM_K2_TASKS=consecutive GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_r3.so timeout -k 10 200 python3 tools/repeat_variant.py syn_small "-b 20 -t 1 -y 2" 20 > gpurun_out/r4g/r3.txt 2>&1; echo "r3 rc=$?"; tail -3 gpurun_out/r4g/r3.txt
GHOSTM_LIB_PATH=$R/ghostm_amd/lib/libghostm_hip_noscan.so timeout -k 10 200 python3 tools/repeat_variant.py syn_small "-b 20 -t 1 -y 2" 20 > gpurun_out/r4g/noscan.txt 2>&1; echo "noscan rc=$?"; tail -3 gpurun_out/r4g/noscan.txt
