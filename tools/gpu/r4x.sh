# round 4: which commit brought the stall before the first timed run's K1 (cfg4, host timelines)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4x
for rep in 1 2; do
for v in r3 6c4030c 5c363b9 f8a4937 3b06ccc cur; do
  L=$R/ghostm_amd/lib/libghostm_hip_$v.so; [ $v = cur ] && L=$R/ghostm_amd/lib/libghostm_hip.so
  GHOSTM_LIB_PATH=$L GHOSTM_TRACE=1 timeout -k 10 200 python3 bench.py --preset cfg4 --steps 2 --warmup 1 --no-cpu --no-e2e --workdir /tmp/tr4x > gpurun_out/r4x/$v.$rep.json 2> gpurun_out/r4x/$v.$rep.log || exit $?
  echo -n "$v.$rep: "; awk '/seed /{s=$2} /k1a_done/{printf "%.1f ", $2-s}' gpurun_out/r4x/$v.$rep.log; echo
done
done
