# round 5: (1) is the run-2 stall tied to the output file? run_session with
# -o a file on /tmp, on /dev/shm, and /dev/null, timelines of 4 runs each;
# (2) PMC of cfg2 (pair-table K2) with tools/profile.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5h
mkdir -p $O
cd $R
summ() {
python3 - "$1" <<'PY'
import sys
runs, cur = [], None
for l in open(sys.argv[1]):
    p = l.split()
    if len(p) >= 4 and p[0] == "trace":
        t, m = float(p[1]), p[3]
        if m == "run":
            cur = {}
            runs.append(cur)
        if cur is not None and m not in cur:
            cur[m] = t
print(sys.argv[1].split("/")[-1], "k1 waits", [round(r["k1_idle"] - r["seed"], 2) for r in runs if "k1_idle" in r],
      "run ms", [round(r["run_end"], 1) for r in runs if "run_end" in r])
PY
}
for o in tmpfile shmfile devnull tmpfile2; do
  case $o in
    tmpfile|tmpfile2) OUTF=/tmp/r5h_out_$o ;;
    shmfile) OUTF=/dev/shm/r5h_out ;;
    devnull) OUTF=/dev/null ;;
  esac
  GHOSTM_TRACE=1 timeout -k 10 300 python3 -u tools/run_session.py --preset cfg4 --runs 4 --out $OUTF --workdir /tmp/r5h_cfg4 > $O/probe_$o.log 2> $O/probe_$o.trace || { echo "probe $o failed"; tail -5 $O/probe_$o.log $O/probe_$o.trace; exit 1; }
  summ $O/probe_$o.trace
  rm -f /dev/shm/r5h_out
done
timeout -k 10 1000 bash tools/profile.sh r5h cfg2 > $O/profile.log 2>&1 || { echo "profile failed"; tail -20 $O/profile.log; exit 1; }
tail -5 $O/profile.log
echo done
