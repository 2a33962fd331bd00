# round 6 l: host chunk copies dropped in the background after creation: the
# golden/streamed/shard groups, then cfg3/cfg2 e2e (traced)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6l
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_shards.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "golden or streamed or shard or world" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for p in cfg3 cfg2; do
  GHOSTM_TRACE=1 timeout -k 10 300 python3 -u tools/e2e_trace.py --preset $p --runs 7 --workdir /tmp/r6l_$p > $O/e2e_$p.txt 2> $O/e2e_${p}_trace.log || { echo "$p failed"; tail -5 $O/e2e_${p}_trace.log; exit 1; }
  cat $O/e2e_$p.txt
done
echo done
