# round 4: PMC HBM traffic for cfg3 and cfg5 (BASELINE config 3 asks for rocprof
# HBM GB/s), then the host timelines of the end-to-end runs (GHOSTM_TRACE)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4c
bash tools/profile.sh r4_cfg3 cfg3 > gpurun_out/r4c/prof_cfg3.log 2>&1 || { echo "profile cfg3 failed"; tail -5 gpurun_out/r4c/prof_cfg3.log; exit 1; }
tail -2 gpurun_out/r4c/prof_cfg3.log
bash tools/profile.sh r4_cfg5 cfg5 > gpurun_out/r4c/prof_cfg5.log 2>&1 || { echo "profile cfg5 failed"; tail -5 gpurun_out/r4c/prof_cfg5.log; exit 1; }
tail -2 gpurun_out/r4c/prof_cfg5.log
cp profiles/r4_cfg3_* profiles/r4_cfg5_* profiles/pmc_traffic_cfg3.json profiles/pmc_traffic_cfg5.json gpurun_out/r4c/ 2>/dev/null
for p in cfg3 cfg4; do
  mkdir -p /tmp/tr_$p
  GHOSTM_TRACE=1 timeout -k 10 300 python3 bench.py --preset $p --steps 2 --warmup 1 --no-cpu --workdir /tmp/tr_$p > gpurun_out/r4c/trace_$p.json 2> gpurun_out/r4c/trace_$p.log || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['ms_per_step'],2), d['end_to_end'])" gpurun_out/r4c/trace_$p.json
done
