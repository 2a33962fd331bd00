# round 6 zi: the last segment's size against cfg3's end-to-end rate (its
# formatting and write are the run's tail): GHOSTM_TAIL_CANDS default / 500 K /
# 300 K, alternating, resident step and warm end to end
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6zi
mkdir -p $O
cd $R
for i in 1 2; do
  for v in def 500000 300000; do
    if [ $v = def ]; then unset GHOSTM_TAIL_CANDS; else export GHOSTM_TAIL_CANDS=$v; fi
    timeout -k 10 300 python3 -u bench.py --preset cfg3 --steps 10 --warmup 2 --no-cpu --workdir /tmp/r6zi_cfg3 > $O/cfg3_${v}_$i.json 2> $O/cfg3_${v}_$i.log || { echo "cfg3 $v failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print('cfg3 tail', sys.argv[2], round(d['ms_per_step'],2), 'e2e', round(d['value_end_to_end_warm']/1e6,1), [round(1e3*x,2) for x in e['runs_s']], d['full_output_matches_reference'])" $O/cfg3_${v}_$i.json $v
  done
done
unset GHOSTM_TAIL_CANDS
echo done
