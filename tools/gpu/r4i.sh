# round 4: dump the K2 tasks of the failing variant
export TMPDIR=/tmp
mkdir -p gpurun_out/r4i
rm -f gpurun_out/r4i/tasks.bin
GHOSTM_DEBUG_TASKS=$GRAFT_REPO_ROOT/gpurun_out/r4i/tasks.bin timeout -k 10 120 python3 tools/repeat_variant.py syn_small "-b 20 -t 1 -y 2" 1 > gpurun_out/r4i/run.txt 2>&1; echo "rc=$?"; tail -3 gpurun_out/r4i/run.txt
GHOSTM_K2_TASKS=consecutive timeout -k 10 120 python3 tools/repeat_variant.py syn_small "-b 20 -t 1 -y 2" 4 > gpurun_out/r4i/consec.txt 2>&1; echo "consec rc=$?"; tail -1 gpurun_out/r4i/consec.txt
GHOSTM_K2_TASKS=paired timeout -k 10 120 python3 tools/repeat_variant.py syn_small "-b 20 -t 1 -y 2" 4 > gpurun_out/r4i/paired.txt 2>&1; echo "paired rc=$?"; tail -1 gpurun_out/r4i/paired.txt
ls -la gpurun_out/r4i
