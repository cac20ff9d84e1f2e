# PMC counters, one rocprofv3 run per counter group (--kernel-trace only: never with
# sys/runtime traces; each group within the per-block slot limits):
#   bash tools/gpu_pmc.sh [kernel_bench|transmux]   groups via $PMC_GROUPS (';'-separated),
#   batch size via $PMC_SEGS (distinct segments; > 85 x 3 MB
#   spills the 256 MB Infinity Cache, so FETCH_SIZE counts HBM reads), extra transmux_bench
#   arguments via $PMC_ARGS (e.g. --verify: the fused-CRC decrypt too), output dir via $PMC_OUT
#   -> gpurun_out/$PMC_OUT/g<i>/ and pmc_g<i>.log
set -eo pipefail
R=$GRAFT_REPO_ROOT
WHAT=${1:-kernel_bench}
if [ "$WHAT" = transmux ]; then PROG="$R/tools/transmux_bench.py --segs ${PMC_SEGS:-64} --pool ${PMC_SEGS:-64} --iters 3 ${PMC_ARGS:-}"; else PROG="$R/tools/kernel_bench.py --iters 3"; fi
cd /tmp && export TMPDIR=/tmp
GROUPS_DEFAULT="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS;SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT;FETCH_SIZE;WRITE_SIZE"
IFS=';' read -ra GS <<< "${PMC_GROUPS:-$GROUPS_DEFAULT}"
i=0
mkdir -p $R/gpurun_out/${PMC_OUT:-pmc}
for G in "${GS[@]}"; do
  i=$((i+1))
  PYTHONPATH=$R timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $G -d $R/gpurun_out/${PMC_OUT:-pmc}/g$i -o run --output-format csv -- python3 $PROG > $R/gpurun_out/${PMC_OUT:-pmc}/pmc_g$i.log 2>&1
done
