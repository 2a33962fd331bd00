# round 5: (1) same-box A/B of the formatter's host buffers (the build before
# host_buffers.h against the current one: cfg3 step and formatting times), (2)
# the sparse-segment pair-table K2's parity tests, (3) cfg2/cfg3 with it
# against the default kernels, (4) a cfg2 kernel trace with it
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5d
mkdir -p $O
cd $R
for k in 1 2; do
  for v in cur prevbuf; do
    L=$R/ghostm_amd/lib/libghostm_hip_$v.so; [ $v = cur ] && L=$R/ghostm_amd/lib/libghostm_hip.so
    GHOSTM_LIB_PATH=$L GHOSTM_TRACE=1 timeout -k 10 300 python3 -u bench.py --preset cfg3 --no-cpu --no-e2e --steps 6 --warmup 1 --workdir /tmp/r5d_cfg3 > $O/buf_${v}$k.json 2> $O/buf_${v}$k.log || { echo "buf $v failed"; tail -5 $O/buf_${v}$k.log; exit 1; }
    python3 -c "
import json,sys
d=json.load(open(sys.argv[1])); f=[]; b=None
for l in open(sys.argv[2]):
    p=l.split()
    if len(p)>=4 and p[0]=='trace' and p[3]=='fmt_begin': b=float(p[1])
    if len(p)>=4 and p[0]=='trace' and p[3]=='fmt_end' and b is not None: f.append(round(float(p[1])-b,2)); b=None
print(sys.argv[3], round(d['ms_per_step'],2), 'ms; fmt ms (last run)', f[-3:], d['full_output_matches_reference'])" $O/buf_${v}$k.json $O/buf_${v}$k.log $v
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread -k "pair or poison" > $O/tests_pair.log 2>&1 || { echo "pair tests failed"; tail -40 $O/tests_pair.log; exit 1; }
tail -1 $O/tests_pair.log
for p in cfg2 cfg3; do
  for v in default pair default pair; do
    if [ $v = pair ]; then export GHOSTM_K2=pair; else unset GHOSTM_K2; fi
    timeout -k 10 300 python3 -u bench.py --preset $p --no-cpu --no-e2e --steps 10 --warmup 2 --workdir /tmp/r5d_$p > $O/${p}_$v.json 2> $O/${p}_$v.log || { echo "bench $p $v failed"; tail -5 $O/${p}_$v.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], sys.argv[3], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],2), 'ms; K2', round(d['stages_s_per_step']['score_device']*1e3,2), 'ms frac', round(r['frac'],3), d['full_output_matches_reference'])" $O/${p}_$v.json $p $v
  done
done
unset GHOSTM_K2
cd /tmp
GHOSTM_K2=pair timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_cfg2 -o run -- python3 $R/bench.py --preset cfg2 --steps 3 --warmup 1 --no-cpu --no-e2e --workdir /tmp/r5d_cfg2 > $O/trace_cfg2.log 2>&1 || { echo "trace failed"; tail -5 $O/trace_cfg2.log; exit 1; }
echo done
