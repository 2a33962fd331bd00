# round 6 x: the N > 1 path on this round's library: bench.py --gpus 8 as eight
# ranks on the one GPU over gloo (RCCL refuses two ranks on one device), full
# cfg4: shard sessions, the batch-plan all-gather, the record gather and the
# assembled file against the reference pin
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6x
mkdir -p $O
cd $R
GHOSTM_BENCH_BACKEND=gloo GHOSTM_BENCH_DEVICE=0 timeout -k 10 900 python3 -u bench.py --gpus 8 --steps 3 --warmup 1 --no-cpu > $O/bench_8rank_gloo.json 2> $O/bench_8rank_gloo.log || { echo "8-rank failed"; tail -30 $O/bench_8rank_gloo.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ranks'], d['n_gpus'], round(d['value']/1e6,1), round(d['ms_per_step'],1), d['full_output_matches_reference'], d['gather_check'], d['gather_fill'], (d.get('end_to_end') or {}).get('output_files_match_reference'))" $O/bench_8rank_gloo.json
echo done
