# round 4: host timelines of cfg4 steps, this build and the round-3 library
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4u /tmp/tr4u
for v in cur r3; do
  L=$R/ghostm_amd/lib/libghostm_hip.so; [ $v = r3 ] && L=$R/ghostm_amd/lib/libghostm_hip_r3.so
  GHOSTM_LIB_PATH=$L GHOSTM_TRACE=1 timeout -k 10 200 python3 bench.py --preset cfg4 --steps 2 --warmup 1 --no-cpu --no-e2e --workdir /tmp/tr4u > gpurun_out/r4u/$v.json 2> gpurun_out/r4u/$v.log || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], round(d['ms_per_step'],2))" gpurun_out/r4u/$v.json
done
