# round 5: the formatter cursor fix (same-box A/B against the build before the
# host buffers), every GPU test with the pair-table K2 on by default for sparse
# segments, and the cfg2/cfg3/cfg4 bench lines (end to end)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5e
mkdir -p $O
cd $R
for k in 1 2; do
  for v in cur prevbuf; do
    L=$R/ghostm_amd/lib/libghostm_hip_$v.so; [ $v = cur ] && L=$R/ghostm_amd/lib/libghostm_hip.so
    GHOSTM_LIB_PATH=$L GHOSTM_TRACE=1 timeout -k 10 300 python3 -u bench.py --preset cfg3 --no-cpu --steps 6 --warmup 1 --workdir /tmp/r5e_cfg3 > $O/buf_${v}$k.json 2> $O/buf_${v}$k.log || { echo "buf $v failed"; tail -5 $O/buf_${v}$k.log; exit 1; }
    python3 -c "
import json,sys
d=json.load(open(sys.argv[1])); f=[]; b=None
for l in open(sys.argv[2]):
    p=l.split()
    if len(p)>=4 and p[0]=='trace' and p[3]=='fmt_begin': b=float(p[1])
    if len(p)>=4 and p[0]=='trace' and p[3]=='fmt_end' and b is not None: f.append(round(float(p[1])-b,2)); b=None
e=d['end_to_end']
print(sys.argv[3], round(d['ms_per_step'],2), 'ms; fmt ms (last e2e run)', f[-3:], 'e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e['runs_s']], d['full_output_matches_reference'])" $O/buf_${v}$k.json $O/buf_${v}$k.log $v
  done
done
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for p in cfg2 cfg3 cfg4; do
  timeout -k 10 400 python3 -u bench.py --preset $p --no-cpu > $O/bench_$p.json 2> $O/bench_$p.log || { echo "bench $p failed"; tail -5 $O/bench_$p.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; r=d['roofline']; print(sys.argv[2], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms; K2 frac', round(r['frac'],3), '; e2e', round(e['value']/1e6,1), [round(x*1e3,1) for x in e['runs_s']], d['full_output_matches_reference'], e.get('output_files_match_reference'), 'steps', [round(x,1) for x in d['step_ms_rank0']])" $O/bench_$p.json $p
done
echo done
