# round 4: failure rate of syn_small -b 20 -t 1 -y 2 per build (10 runs each)
export TMPDIR=/tmp
mkdir -p gpurun_out/r4h
R=$GRAFT_REPO_ROOT
for v in cur nok2 nok4 nopairs noscan; do
  L=$R/ghostm_amd/lib/libghostm_hip_$v.so; [ $v = cur ] && L=$R/ghostm_amd/lib/libghostm_hip.so
  E=""; [ $v = nok2 ] && E="GHOSTM_K2_TASKS=consecutive"
  env $E GHOSTM_LIB_PATH=$L timeout -k 10 120 python3 tools/repeat_variant.py syn_small "-b 20 -t 1 -y 2" 10 > gpurun_out/r4h/$v.txt 2>&1
  echo "$v rc=$? $(tail -1 gpurun_out/r4h/$v.txt)"
done
GHOSTM_K2=swar16 timeout -k 10 120 python3 tools/repeat_variant.py syn_small "-b 20 -t 1 -y 2" 10 > gpurun_out/r4h/swar16.txt 2>&1
echo "cur swar16 rc=$? $(tail -1 gpurun_out/r4h/swar16.txt)"
