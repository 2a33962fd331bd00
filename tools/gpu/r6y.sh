# round 6 y: the key DP's column-framed E chain (k_traceback_key FRAME): K3
# parity (scan modes incl. keyframe0, forced encodings, wide band, reference
# driver), then A/B against GHOSTM_K3_KEYFRAME=0 on cfg4 and cfg5, alternating
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6y
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "traceback or forced_score or reference_driver or default_encoding" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in 1 0; do
    GHOSTM_K3_KEYFRAME=$v timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --workdir /tmp/r6y_cfg4 > $O/cfg4_${v}_$i.json 2> $O/cfg4_${v}_$i.log || { echo "cfg4 $v failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['roofline_k3']; print('cfg4 frame', sys.argv[2], round(d['ms_per_step'],2), 'k3', round(k['ms_per_step'],2), 'key', round(k['key_dp']['ms_per_step'],2), 'scan', round(k['scan']['ms_per_step'],2), d['full_output_matches_reference'])" $O/cfg4_${v}_$i.json $v
    GHOSTM_K3_KEYFRAME=$v timeout -k 10 300 python3 -u bench.py --preset cfg5 --steps 5 --warmup 1 --no-cpu --no-e2e --workdir /tmp/r6y_cfg5 > $O/cfg5_${v}_$i.json 2> $O/cfg5_${v}_$i.log || { echo "cfg5 $v failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['roofline_k3']; print('cfg5 frame', sys.argv[2], round(d['ms_per_step'],2), 'k3', round(k['ms_per_step'],2), 'key', round(k['key_dp']['ms_per_step'],2), d['full_output_matches_reference'])" $O/cfg5_${v}_$i.json $v
  done
done
echo done
