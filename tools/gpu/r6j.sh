# round 6 j: sparse rows K2 profile slots per block (occupancy vs block fill), cfg2
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6j
mkdir -p $O
cd $R
for i in 1 2; do
  for v in pair 7 6 5 4; do
    if [ $v = pair ]; then E="GHOSTM_K2_SPARSE=pair"; else E="GHOSTM_K2_SPARSE=rows GHOSTM_K2_SPARSE_SLOTS=$v"; fi
    env $E timeout -k 10 300 python3 -u bench.py --preset cfg2 --steps 10 --warmup 2 --no-cpu --no-e2e --workdir /tmp/r6j_cfg2 > $O/cfg2_${v}_$i.json 2> $O/cfg2_${v}_$i.log || { echo "bench $v failed"; tail -5 $O/cfg2_${v}_$i.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],3), 'K2', round(1e3*s['score_device'],3), 'frac', round(r['frac'],3), d['full_output_matches_reference'])" $O/cfg2_${v}_$i.json $v
  done
done
echo done
