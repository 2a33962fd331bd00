# round 6 c: end-to-end host timelines of cfg2 and cfg3 (GHOSTM_TRACE), the
# filesystem under /tmp, and a raw single-thread write rate of a 20 MB file there
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6c
mkdir -p $O
cd $R
df -T /tmp > $O/fs.txt 2>&1; nproc >> $O/fs.txt; cat /sys/fs/cgroup/cpu.max >> $O/fs.txt 2>&1
python3 - >> $O/fs.txt <<'PY'
import os, time
buf = os.urandom(1 << 20) * 20
for k in range(3):
    p = f"/tmp/wtest{k}"
    os.sync(); time.sleep(0.5)
    t = time.perf_counter()
    fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    for i in range(0, len(buf), 1 << 20):
        os.pwrite(fd, buf[i:i + (1 << 20)], i)
    os.close(fd)
    print(f"write 20 MB: {1e3 * (time.perf_counter() - t):.2f} ms")
    os.remove(p)
PY
for p in cfg2 cfg3; do
  GHOSTM_TRACE=1 timeout -k 10 300 python3 -u tools/e2e_trace.py --preset $p --runs 5 --workdir /tmp/r6c_$p > $O/e2e_$p.txt 2> $O/e2e_${p}_trace.log || { echo "$p failed"; tail -5 $O/e2e_${p}_trace.log; exit 1; }
  cat $O/e2e_$p.txt
done
cat $O/fs.txt
echo done
