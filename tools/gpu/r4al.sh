# round 4: segment tail size at cfg3 and at the 8-GPU shard size (125 K cfg4 queries), same box
export TMPDIR=/tmp
O=gpurun_out/r4al
mkdir -p $O
for rep in 1 2; do
for t in 1048576 524288 262144; do
  for p in cfg3 shard; do
    A="--preset cfg3"; [ $p = shard ] && A="--preset cfg4 --queries 125000"
    GHOSTM_TAIL_CANDS=$t timeout -k 10 300 python3 bench.py $A --steps 10 --warmup 2 --no-cpu --no-e2e --workdir /tmp/tail_$p > $O/${p}_$t.$rep.json 2> $O/${p}_$t.$rep.log || { echo "$p $t failed"; tail -3 $O/${p}_$t.$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],2), 'ms', d['full_output_matches_reference'])" $O/${p}_$t.$rep.json $p $t
  done
done
done
# the driver's N = 8 command rehearsed on one GPU (gloo, every rank on device 0), final build
GHOSTM_BENCH_BACKEND=gloo GHOSTM_BENCH_DEVICE=0 timeout -k 10 600 python3 -u bench.py --gpus 8 --steps 2 --warmup 1 --no-cpu > $O/bench8.json 2> $O/bench8.log || { echo "bench8 failed"; tail -5 $O/bench8.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench8 ranks', d.get('ranks'), 'matches', d['full_output_matches_reference'], 'gather', d.get('gather_check'), 'e2e files', d['end_to_end'].get('output_files_match_reference'))" $O/bench8.json
