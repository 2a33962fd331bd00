# round 5: host timelines of end-to-end sessions (create: reads, uploads) for cfg4 and cfg3
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5ad
mkdir -p $O
cd $R
for p in cfg4 cfg3; do
  GHOSTM_TRACE=1 timeout -k 10 400 python3 -u bench.py --preset $p --no-cpu --steps 1 --warmup 1 --workdir /tmp/r5ad_$p > $O/$p.json 2> $O/$p.log || { echo "$p failed"; tail -5 $O/$p.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print(sys.argv[2], 'e2e', [round(x*1e3,1) for x in e['runs_s']], 'create', [round(x*1e3,1) for x in e['create_s']])" $O/$p.json $p
done
echo done
