# round 6 zj: where a fresh `ghostm aln` process spends its start: cfg3 data,
# three cold runs each with the HIP runtime's default code-object loading and
# with HIP_ENABLE_DEFERRED_LOADING=0/1, GHOSTM_TRACE timelines (the device
# binding mark is the runtime start)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6zj
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u bench.py --preset cfg3 --steps 2 --warmup 1 --no-cpu --no-e2e --workdir /tmp/r6zj_cfg3 > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
D=/tmp/r6zj_cfg3
for v in def 0 1; do
  for i in 1 2 3; do
    if [ $v = def ]; then unset HIP_ENABLE_DEFERRED_LOADING; else export HIP_ENABLE_DEFERRED_LOADING=$v; fi
    s=$(date +%s.%N)
    GHOSTM_TRACE=1 timeout -k 10 120 ghostm_amd/bin/ghostm aln -i $D/q/q -d $D/db/db -o /tmp/r6zj_out -D 0 > $O/trace_${v}_$i.log 2>&1 || { echo "aln $v failed"; tail -5 $O/trace_${v}_$i.log; exit 1; }
    e=$(date +%s.%N)
    echo "deferred=$v run $i: $(python3 -c "print(round(($e-$s)*1e3,1))") ms; $(grep -m1 ' bound ' $O/trace_${v}_$i.log | awk '{print "bound at", $2, "ms"}'); $(grep -m1 ' run_end ' $O/trace_${v}_$i.log | awk '{print "run_end at", $2, "ms"}')"
  done
done
unset HIP_ENABLE_DEFERRED_LOADING
echo done
