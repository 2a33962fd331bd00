# round 5: the LDS-poison golden group timed out in r5at (first test on the box):
# time the child directly with the default library, the poison build, and poison
# builds with mbcnt (pmb) and with the 24-bit hash (phash) on top
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5au
mkdir -p $O /tmp/r5au_data
cd $R
for v in default poison pmb phash; do
  LIB=$R/ghostm_amd/lib/libghostm_hip_$v.so; [ $v = default ] && LIB=$R/ghostm_amd/lib/libghostm_hip.so
  s=$(date +%s.%N)
  GHOSTM_LIB_PATH=$LIB GHOSTM_LDS_POISON_PATTERN=0xA5A5A5A5 timeout -k 10 240 python3 tests/lds_poison_child.py golden /tmp/r5au_data > $O/$v.out 2> $O/$v.err
  rc=$?
  e=$(date +%s.%N)
  echo "$v rc=$rc $(python3 -c "print(round($e-$s,1))") s $(tail -c 300 $O/$v.out)"
  [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && { echo "stop after $v"; exit 1; }
done
echo done
