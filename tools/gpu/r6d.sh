# round 6 d: cfg3/cfg2 end-to-end runs at 16, 14 and 12 host threads, with the
# cgroup's throttling counters per run (is the formatting burst throttled?)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6d
mkdir -p $O
cd $R
cat /sys/fs/cgroup/cpu.max > $O/cpu.txt 2>&1; cat /sys/fs/cgroup/cpu.stat >> $O/cpu.txt 2>&1
for p in cfg3 cfg2; do
  for t in 16 14 12; do
    GHOSTM_THREADS=$t GHOSTM_TRACE=1 timeout -k 10 300 python3 -u tools/e2e_trace.py --preset $p --runs 5 --workdir /tmp/r6d_$p > $O/e2e_${p}_t$t.txt 2> $O/e2e_${p}_t${t}_trace.log || { echo "$p $t failed"; tail -5 $O/e2e_${p}_t${t}_trace.log; exit 1; }
    echo "$p threads $t"; cat $O/e2e_${p}_t$t.txt
  done
done
echo done
