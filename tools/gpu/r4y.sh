# round 4: is the one-time stall before an early K1 tied to time since create? (cfg4, pause after create)
export TMPDIR=/tmp
mkdir -p gpurun_out/r4y
for p in 0 0.05 0.2 1.0 0; do
  GHOSTM_BENCH_PAUSE_S=$p GHOSTM_TRACE=1 timeout -k 10 200 python3 bench.py --preset cfg4 --steps 3 --warmup 1 --no-cpu --no-e2e --workdir /tmp/tr4y > gpurun_out/r4y/p$p.json 2> gpurun_out/r4y/p$p.log || exit $?
  echo -n "pause $p: "; awk '/seed /{s=$2} /k1_idle/{printf "%.1f ", $2-s}' gpurun_out/r4y/p$p.log; python3 -c "import json,sys; print(round(json.load(open(sys.argv[1]))['ms_per_step'],1))" gpurun_out/r4y/p$p.json
done
