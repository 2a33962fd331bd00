# round 4: the stall before the first timed run's K1 (cfg4): selected hits staged through page-locked memory
export TMPDIR=/tmp
mkdir -p gpurun_out/r4ab
run() { tag=$1; shift
  env "$@" GHOSTM_TRACE=1 timeout -k 10 200 python3 bench.py --preset cfg4 --steps 2 --warmup 1 --no-cpu --no-e2e --workdir /tmp/tr4ab > gpurun_out/r4ab/$tag.json 2> gpurun_out/r4ab/$tag.log || exit $?
  echo -n "$tag: "; awk '$4=="run"{r=$2} /seed /{s=$2; printf "[run->seed %.1f ", s-r} /k1_idle/{printf "idle %.1f] ", $2-s}' gpurun_out/r4ab/$tag.log; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['ms_per_step'],1), d['full_output_matches_reference'])" gpurun_out/r4ab/$tag.json
}
run base1 X=1
run stage1 GHOSTM_HITS_STAGE=1
run base2 X=1
run stage2 GHOSTM_HITS_STAGE=1
