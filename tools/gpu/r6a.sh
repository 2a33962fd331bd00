# round 6 a: the K1 probe-bound redo, the short-candidate-buffer compaction, the
# device-pool OOM retry; then the K1 groups (classes, overflow) and the poison groups
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6a
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "probe_bound or short_candidate or pool or overflow_redo or every_k1_class or syn_scale_runs" > $O/scale.log 2>&1 \
  || { echo "scale tests failed"; tail -40 $O/scale.log; exit 1; }
tail -1 $O/scale.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_lds_poison.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/poison.log 2>&1 \
  || { echo "poison tests failed"; tail -40 $O/poison.log; exit 1; }
tail -1 $O/poison.log
echo done
