# round 4: VALU issue by waves per SIMD: v_fma_f32 / v_fmac_f32_e32 /
# v_pk_maximum3_f16 / v_add_u32 / v_pk_mad_u16 / v_max_u32 at 1, 2, 4, 8 waves per SIMD,
# 16 independent chains per wave; wall-time rates, then the same binary under one PMC pass
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4d
timeout -k 10 120 tools/microbench/valu_waves > gpurun_out/r4d/valu_waves.txt 2>&1 || exit $?
cat gpurun_out/r4d/valu_waves.txt
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES \
  --output-format csv -d $R/gpurun_out/r4d/pmc -o run -- $R/tools/microbench/valu_waves > $R/gpurun_out/r4d/pmc.log 2>&1 || exit $?
python3 $R/tools/valu_pmc_summary.py $R/gpurun_out/r4d/pmc valu_waves | tee $R/gpurun_out/r4d/valu_waves_pmc.txt
