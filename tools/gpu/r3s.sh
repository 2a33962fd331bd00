# cfg3 A/B: the current library (A) against the library before this session's K1 changes (orig)
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_ROUNDS=3 AB_STEPS=10 AB_ARGS="--preset cfg3" bash tools/ab.sh orig > gpurun_out/r3s_ab.log 2>&1
echo "ab rc=$?"
cat gpurun_out/r3s_ab.log
