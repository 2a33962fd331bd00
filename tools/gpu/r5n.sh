# round 5: the K3 scan at 16 rows per lane (GHOSTM_K3_SCAN_S=16): parity with
# it forced, then cfg4 and cfg2 K3 times against the default (32)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5n
mkdir -p $O
cd $R
GHOSTM_K3_SCAN_S=16 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/parity_s16.log 2>&1 || { echo "parity failed"; tail -40 $O/parity_s16.log; exit 1; }
tail -1 $O/parity_s16.log
for v in s32 s16 s32b s16b; do
  ENVV="GHOSTM_K3_SCAN_S=32"
  case $v in s16*) ENVV="GHOSTM_K3_SCAN_S=16" ;; esac
  env $ENVV timeout -k 10 300 python3 -u bench.py --no-cpu --no-e2e --steps 3 --warmup 1 --workdir /tmp/r5n_cfg4 > $O/cfg4_$v.json 2> $O/cfg4_$v.log || { echo "cfg4 $v failed"; tail -5 $O/cfg4_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; r=d['roofline_k3']; print(sys.argv[2], round(d['ms_per_step'],2), 'ms; K3', round(1e3*s['traceback_device'],2), 'scan', round(r['scan']['ms_per_step'],2) if 'ms_per_step' in r.get('scan',{}) else r.get('scan'), 'matches', d.get('full_output_matches_reference'))" $O/cfg4_$v.json $v
done
echo done
