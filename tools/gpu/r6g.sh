# round 6 g: K1 filter region in static LDS and the piece-streamed writer: K1,
# golden, streamed-output and poison groups; a same-box cfg4 A/B against the
# dynamic region (ab_libs/dynlds); then e2e with streamed pieces (4 per worker)
# against whole parts (GHOSTM_STREAM_PIECES=1), alternating
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_lds_poison.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "k1 or probe or golden or poison or streamed" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_ROUNDS=3 timeout -k 10 900 bash tools/ab.sh dynlds > $O/ab.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
for i in 1 2; do
  for p in cfg3 cfg2; do
    for sp in 4 1; do
      GHOSTM_STREAM_PIECES=$sp timeout -k 10 300 python3 -u tools/e2e_trace.py --preset $p --runs 7 --settle 0.5 --workdir /tmp/r6g_$p > $O/e2e_${p}_sp${sp}_$i.txt 2> $O/e2e_${p}_sp${sp}_$i.log || { echo "$p $sp failed"; tail -5 $O/e2e_${p}_sp${sp}_$i.log; exit 1; }
      echo "$p pieces/worker $sp round $i: $(python3 -c "
import re,sys,statistics
v=[float(m.group(1)) for m in re.finditer(r'total ([0-9.]+) ms', open(sys.argv[1]).read())]
print(sorted(v), 'median', statistics.median(v))" $O/e2e_${p}_sp${sp}_$i.txt)"
    done
  done
done
echo done
