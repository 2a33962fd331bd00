# round 6 e: end-to-end A/B of the host thread count (16 = default on the box,
# 14 leaves two CPUs to the main and writer threads), alternating, cfg2 and cfg3
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6e
mkdir -p $O
cd $R
for i in 1 2 3; do
  for p in cfg2 cfg3; do
    for t in 16 14; do
      GHOSTM_THREADS=$t timeout -k 10 300 python3 -u tools/e2e_trace.py --preset $p --runs 7 --settle 0.5 --workdir /tmp/r6e_$p > $O/e2e_${p}_t${t}_$i.txt 2> $O/e2e_${p}_t${t}_$i.log || { echo "$p $t failed"; tail -5 $O/e2e_${p}_t${t}_$i.log; exit 1; }
      echo "$p t$t round $i: $(python3 -c "
import re,sys,statistics
v=[float(m.group(1)) for m in re.finditer(r'total ([0-9.]+) ms', open(sys.argv[1]).read())]
print(sorted(v), 'median', statistics.median(v))" $O/e2e_${p}_t${t}_$i.txt)"
    done
  done
done
echo done
