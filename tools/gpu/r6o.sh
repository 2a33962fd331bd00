# round 6 o: K3 scan in query order (GHOSTM_K3_SCAN_ORDER=query, the order a
# per-query-profile scan needs) against the width order: golden parity with the
# knob, then cfg4 K3 scan time alternating
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6o
mkdir -p $O
cd $R
GHOSTM_K3_SCAN_ORDER=query timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "golden" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in width query; do
    GHOSTM_K3_SCAN_ORDER=$v timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --workdir /tmp/r6o_cfg4 > $O/cfg4_${v}_$i.json 2> $O/cfg4_${v}_$i.log || { echo "bench $v failed"; tail -5 $O/cfg4_${v}_$i.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline_k3']; print(sys.argv[2], round(d['ms_per_step'],1), 'K3', round(r['ms_per_step'],2), 'scan', round(r['scan']['ms_per_step'],2), 'tcups', round(r['scan']['tcups'],2), 'key', round(r['key_dp']['ms_per_step'],2), d['full_output_matches_reference'])" $O/cfg4_${v}_$i.json $v
  done
done
echo done
