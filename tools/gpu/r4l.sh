# round 4: GPU tests (lazy line-format caches), end-to-end tail-size sweep with
# host traces, then the VALU-by-waves microbenchmark
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4l
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4l/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r4l/tests.log
[ $rc -eq 0 ] || exit $rc
for p in cfg3 cfg4; do
  mkdir -p /tmp/e_$p
  for tail in 1048576 524288 262144; do
    GHOSTM_TAIL_CANDS=$tail GHOSTM_TRACE=1 timeout -k 10 300 python3 bench.py --preset $p --steps 3 --warmup 1 --no-cpu --workdir /tmp/e_$p > gpurun_out/r4l/e2e_${p}_$tail.json 2> gpurun_out/r4l/e2e_${p}_$tail.log || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print(sys.argv[1].split('/')[-1], 'step', round(d['ms_per_step'],2), 'e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e['runs_s']], e.get('output_files_match_reference'))" gpurun_out/r4l/e2e_${p}_$tail.json
  done
done
bash tools/gpu/r4d.sh
