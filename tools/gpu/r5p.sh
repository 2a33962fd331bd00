# round 5: cfg2 host timeline (GHOSTM_TRACE) with the head cap and pair K2 at 16 rows
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5p
mkdir -p $O
cd $R
GHOSTM_TRACE=1 timeout -k 10 300 python3 -u bench.py --preset cfg2 --no-cpu --no-e2e --steps 4 --warmup 2 --workdir /tmp/r5p_cfg2 > $O/cfg2_trace.json 2> $O/cfg2_trace.log || { echo "cfg2 failed"; tail -5 $O/cfg2_trace.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('cfg2', round(d['ms_per_step'],3), d['step_ms_rank0'])" $O/cfg2_trace.json
echo done
