# round 4: GPU tests (launcher/ok-flag/fixed gather/K4 stray-sid change), then the
# driver's N=8 command rehearsed on one GPU (gloo, every rank on device 0)
export TMPDIR=/tmp
mkdir -p gpurun_out/r4a
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4a/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r4a/tests.log
[ $rc -eq 0 ] || exit $rc
GHOSTM_BENCH_BACKEND=gloo GHOSTM_BENCH_DEVICE=0 timeout -k 10 600 python3 -u bench.py --gpus 8 --steps 2 --warmup 1 --no-cpu > gpurun_out/r4a/bench8.json 2> gpurun_out/r4a/bench8.log
rc=$?
echo "bench8 rc=$rc"; tail -5 gpurun_out/r4a/bench8.log
exit $rc
