# round 4: GPU tests, the N=8 command rehearsed on one GPU (gloo), then K2 task
# layouts A/B at cfg3 and cfg4 (unit kernel: paired vs consecutive tasks; 16-bit rows)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4b
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4b/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r4b/tests.log
[ $rc -eq 0 ] || exit $rc
GHOSTM_BENCH_BACKEND=gloo GHOSTM_BENCH_DEVICE=0 timeout -k 10 600 python3 -u bench.py --gpus 8 --steps 2 --warmup 1 --no-cpu > gpurun_out/r4b/bench8.json 2> gpurun_out/r4b/bench8.log
rc=$?
echo "bench8 rc=$rc"; tail -3 gpurun_out/r4b/bench8.log
[ $rc -eq 0 ] || exit $rc
for p in cfg3 cfg4; do
  mkdir -p /tmp/ab_$p
  for v in "swar16 x" "unit paired" "unit consecutive" "auto auto"; do
    set -- $v
    GHOSTM_K2=$([ $1 = auto ] && echo "" || echo $1) GHOSTM_K2_TASKS=$2 timeout -k 10 200 python3 bench.py --preset $p --steps 3 --warmup 1 --no-cpu --no-e2e --workdir /tmp/ab_$p > gpurun_out/r4b/ab_${p}_$1_$2.json 2>/dev/null || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['ms_per_step'],2), round(d['roofline']['avg_launch_ms'],3), round(d['roofline']['frac'],4), d['full_output_matches_reference'])" gpurun_out/r4b/ab_${p}_$1_$2.json
  done
done
# K3a scan: unpacked row offsets (this build) against the previous build
AB_ROUNDS=2 timeout -k 10 400 bash tools/ab.sh prev > gpurun_out/r4b/ab_scan.txt 2>&1 || exit $?
cat gpurun_out/r4b/ab_scan.txt
