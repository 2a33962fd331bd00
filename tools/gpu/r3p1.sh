# K2 (unit-pair) stall breakdown: LDS wait and issue counters, one cfg4 step
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3p1
mkdir -p $O /tmp/ghostm_ab_data
cd /tmp
B="$R/bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --workdir /tmp/ghostm_ab_data"
timeout -k 10 300 python3 $B > $O/data.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d $O/p1 -o run -- python3 $B > $O/p1.log 2>&1
echo "p1 rc=$?"
