# round 6 zl: the N > 1 path on the final library: bench.py --gpus 8 as eight
# ranks on the one GPU over gloo (full cfg4), then the 125 K-query shard (one
# rank's work at N = 8) beside cfg4 on the same box
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6zl
mkdir -p $O
cd $R
GHOSTM_BENCH_BACKEND=gloo GHOSTM_BENCH_DEVICE=0 timeout -k 10 900 python3 -u bench.py --gpus 8 --steps 3 --warmup 1 --no-cpu > $O/bench_8rank_gloo.json 2> $O/bench_8rank_gloo.log || { echo "8-rank failed"; tail -30 $O/bench_8rank_gloo.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ranks'], round(d['value']/1e6,1), round(d['ms_per_step'],1), d['full_output_matches_reference'], d['gather_check'], (d.get('end_to_end') or {}).get('output_files_match_reference'))" $O/bench_8rank_gloo.json
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --queries 125000 --steps 10 --warmup 2 --no-cpu --no-e2e --workdir /tmp/r6zl_shard > $O/shard_$i.json 2> $O/shard_$i.log || { echo "shard failed"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('shard', round(d['ms_per_step'],2), [round(x,1) for x in d['step_ms_rank0']])" $O/shard_$i.json
  timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --workdir /tmp/r6zl_cfg4 > $O/cfg4_$i.json 2> $O/cfg4_$i.log || { echo "cfg4 failed"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('cfg4', round(d['ms_per_step'],2))" $O/cfg4_$i.json
done
echo done
