# round 4: cfg4 host timelines with a stream-idle probe before each K1 (4 timed runs)
export TMPDIR=/tmp
mkdir -p gpurun_out/r4w
for v in a b; do
  GHOSTM_TRACE=1 timeout -k 10 200 python3 bench.py --preset cfg4 --steps 4 --warmup 1 --no-cpu --no-e2e --workdir /tmp/tr4w > gpurun_out/r4w/$v.json 2> gpurun_out/r4w/$v.log || exit $?
  awk '/seed /{s=$2} /k1_idle/{i=$2} /k1a_enq/{t=$2} /k1a_done/{printf "idle %.1f wait %.1f | ", i-s, $2-t}' gpurun_out/r4w/$v.log; echo
done
