# round 4: this build against the round-3 library on the same box (cfg2, cfg3, cfg4)
export TMPDIR=/tmp
mkdir -p gpurun_out/r4q
for p in cfg2 cfg3 cfg4; do
  AB_ROUNDS=2 AB_STEPS=5 AB_ARGS="--preset $p" timeout -k 10 500 bash tools/ab.sh r3 > gpurun_out/r4q/ab_$p.txt 2>&1 || exit $?
  rm -rf gpurun_out/ab_$p; mv gpurun_out/ab gpurun_out/r4q/ab_$p
  echo "== $p"; cat gpurun_out/r4q/ab_$p.txt
done
