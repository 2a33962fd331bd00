# K3 scan variants, same-box A/B (A = 1024-thread blocks, 4-row prefetch; s4 = 768 threads; s8 = 768 threads, 8-row prefetch)
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_ROUNDS=3 timeout -k 10 1000 bash tools/ab.sh s4 s8 > gpurun_out/r3g_ab.txt 2>&1
echo "ab rc=$?"
