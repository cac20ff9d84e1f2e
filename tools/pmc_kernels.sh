# PMC counters of the per-kernel microbenchmark, one rocprofv3 run per counter group
# (counter runs use --kernel-trace only; no sys/runtime traces).  Groups via $PMC_GROUPS
# (';'-separated) or the defaults below.
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
GROUPS_DEFAULT="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS;SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT;TA_TA_BUSY_sum TD_TD_BUSY_sum SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
IFS=';' read -ra GS <<< "${PMC_GROUPS:-$GROUPS_DEFAULT}"
i=0
for G in "${GS[@]}"; do
  i=$((i+1))
  PYTHONPATH=$R timeout -k 10 240 rocprofv3 --kernel-trace --pmc $G -d $R/gpurun_out/pmc/g$i -o run --output-format csv -- python $R/tools/kernel_bench.py --iters 3 > $R/gpurun_out/pmc_g$i.log 2>&1 || echo "group $i failed: $G" >> $R/gpurun_out/pmc_fail.log
done
