# round 4: the stall before the first timed run's K1 (cfg4) under variants: threads, pause after warmup
export TMPDIR=/tmp
mkdir -p gpurun_out/r4aa
run() { tag=$1; shift
  env "$@" GHOSTM_TRACE=1 timeout -k 10 200 python3 bench.py --preset cfg4 --steps 2 --warmup 1 --no-cpu --no-e2e --workdir /tmp/tr4aa > gpurun_out/r4aa/$tag.json 2> gpurun_out/r4aa/$tag.log || exit $?
  echo -n "$tag: "; awk '$4=="run"{r=$2} /seed /{s=$2; printf "[run->seed %.1f ", s-r} /k1_idle/{printf "idle %.1f] ", $2-s}' gpurun_out/r4aa/$tag.log; echo
}
run base1 X=1
run t8 GHOSTM_THREADS=8
run wp02 GHOSTM_BENCH_WARM_PAUSE_S=0.2
run wp1 GHOSTM_BENCH_WARM_PAUSE_S=1
run base2 X=1
