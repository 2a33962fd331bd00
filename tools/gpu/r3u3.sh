# PMC of the unit K2 kernel vs the 16-bit-row kernel (issue and LDS counters)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3u3
mkdir -p $O /tmp/ghostm_ab_data
cd /tmp
B="$R/bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --workdir /tmp/ghostm_ab_data"
for v in unit swar16; do
  GHOSTM_K2=$v timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE \
    --output-format csv -d $O/sq_$v -o run -- python3 $B > $O/sq_$v.log 2>&1 || exit $?
  GHOSTM_K2=$v timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE \
    --output-format csv -d $O/lds_$v -o run -- python3 $B > $O/lds_$v.log 2>&1 || exit $?
done
ls -R $O | head -30
