# round 6 b: cfg4 bench with the bounded K1 probes and the cold end-to-end leg
# (no CPU baseline), then the HEAD profile (kernel stats + PMC with the library hash)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6b
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u bench.py --steps 5 --warmup 2 --no-cpu --workdir /tmp/r6b_cfg4 > $O/bench_cfg4.json 2> $O/bench_cfg4.log || { echo "bench failed"; tail -20 $O/bench_cfg4.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_s_per_step']; print(round(d['value']/1e6,1), round(d['ms_per_step'],2), 'K1/K2/K3', round(1e3*s['seed_device'],2), round(1e3*s['score_device'],2), round(1e3*s['traceback_device'],2), 'warm', d['value_end_to_end_warm'], 'cold', d['value_end_to_end_cold'], d['end_to_end_cold'])" $O/bench_cfg4.json
timeout -k 10 1500 bash tools/profile.sh r6b cfg4 > $O/profile.log 2>&1 || { echo "profile failed"; tail -20 $O/profile.log; exit 1; }
tail -3 $O/profile.log
echo done
