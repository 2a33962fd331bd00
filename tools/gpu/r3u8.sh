# every golden variant with the unit K2 kernel forced, then the full-size 8-rank
# rehearsal of the driver's N = 8 bench (gloo, every rank on GPU 0)
export TMPDIR=/tmp
mkdir -p gpurun_out/r3u8
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "unit_k2 or forced" -v --timeout 120 \
  --timeout-method thread > gpurun_out/r3u8/unit_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r3u8/unit_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu/r3u7.sh
