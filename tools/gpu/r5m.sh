# round 5: class 1 of K1 at three widths (6/7/8 waves): the K1 class tests,
# parity, the LDS-poison K1 group, then cfg4 K1 time with the widths on and off
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5m
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py "tests/test_gpu_lds_poison.py::test_golden_variants_under_lds_poison[0xA5A5A5A5-kernels]" -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in sub nosub sub2 nosub2; do
  ENVV="GHOSTM_K1_SUB=1"
  case $v in nosub*) ENVV="GHOSTM_K1_SUB=0" ;; esac
  env $ENVV timeout -k 10 300 python3 -u bench.py --no-cpu --no-e2e --steps 3 --warmup 1 --workdir /tmp/r5m_cfg4 > $O/cfg4_$v.json 2> $O/cfg4_$v.log || { echo "cfg4 $v failed"; tail -5 $O/cfg4_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; print(sys.argv[2], round(d['ms_per_step'],2), 'ms; K1', round(1e3*s['seed_device'],2), 'ms; matches', d.get('full_output_matches_reference'))" $O/cfg4_$v.json $v
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- python3 $R/tools/run_session.py --preset cfg4 --runs 2 --workdir /tmp/r5m_cfg4s > $O/ktrace.log 2>&1 || { echo "ktrace failed"; tail -5 $O/ktrace.log; exit 1; }
grep -i "seed" $O/ktrace/run_kernel_stats.csv | cut -d, -f1-4
echo done
