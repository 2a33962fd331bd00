# K1 micro-variants, same-box A/B (A = the previous build)
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_ROUNDS=3 timeout -k 10 1100 bash tools/ab.sh v1 v2 k1b > gpurun_out/r3e_ab.txt 2>&1
echo "ab rc=$?"
