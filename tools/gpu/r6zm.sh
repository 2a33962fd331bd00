# round 6 zm: `ghostm aln` leaves with _exit after its session (no HIP runtime
# teardown): cold processes on cfg3 and cfg4 data, alternating with
# GHOSTM_FAST_EXIT=0, files checked against each other
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6zm
mkdir -p $O
cd $R
for p in cfg3 cfg4; do
  timeout -k 10 300 python3 -u bench.py --preset $p --steps 1 --warmup 0 --no-cpu --no-e2e --workdir /tmp/r6zm_$p > $O/bench_$p.json 2> $O/bench_$p.log || { echo "bench failed"; exit 1; }
  D=/tmp/r6zm_$p
  for i in 1 2 3; do
    for v in 1 0; do
      sync; sleep 1
      s=$(date +%s.%N)
      GHOSTM_FAST_EXIT=$v timeout -k 10 120 ghostm_amd/bin/ghostm aln -i $D/q/q -d $D/db/db -o /tmp/r6zm_out_$v > /dev/null 2>&1 || { echo "aln failed"; exit 1; }
      e=$(date +%s.%N)
      echo "$p fast_exit=$v run $i: $(python3 -c "print(round(($e-$s)*1e3,1))") ms"
    done
    cmp /tmp/r6zm_out_1 /tmp/r6zm_out_0 || { echo "outputs differ"; exit 1; }
  done
done
echo done
