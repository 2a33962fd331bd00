# round 4: GPU tests after the K2 kernel/task chooser, then K2 A/B at cfg3 and cfg4
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4j
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4j/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r4j/tests.log
[ $rc -eq 0 ] || exit $rc
for p in cfg3 cfg4; do
  mkdir -p /tmp/ab_$p
  for r in 1 2; do
  for v in "swar16 x" "unit consecutive" "auto auto"; do
    set -- $v
    E="GHOSTM_K2=$1 GHOSTM_K2_TASKS=$2"; [ $1 = auto ] && E="X=1"
    env $E timeout -k 10 200 python3 bench.py --preset $p --steps 5 --warmup 1 --no-cpu --no-e2e --workdir /tmp/ab_$p > gpurun_out/r4j/ab_${p}_$1_$2_$r.json 2>/dev/null || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], round(d['ms_per_step'],2), 'K2', round(d['roofline']['avg_launch_ms'],3), round(d['roofline']['frac'],4), 'unit', d['roofline']['kernel'][:28], d['full_output_matches_reference'])" gpurun_out/r4j/ab_${p}_$1_$2_$r.json
  done
  done
done
