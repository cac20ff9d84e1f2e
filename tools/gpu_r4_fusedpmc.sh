# The two-level fused CRC on one MI355X: GPU tests of the CRC kernels, transmux batch timing
# (plain / fused verify / separate CRC kernel), then PMC groups on the same batch: effective
# clock (GRBM_GUI_ACTIVE per ns), VALU / MFMA / LDS instruction counts per kernel.
#   bash tools/gpu_r4_fusedpmc.sh   -> gpurun_out/r4_fused2/*
set -eo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${FUSED_OUT:-r4_fused2}
cd $R
export PYTHONPATH=$R
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_transmux.py -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 300 python tools/transmux_bench.py --segs 256 --iters 10 --verify > $O/bench.log 2>&1
timeout -k 10 300 python tools/transmux_bench.py --segs 256 --pool 256 --iters 10 --verify > $O/bench_pool256.log 2>&1
PMC_OUT=${FUSED_OUT:-r4_fused2}/pmc PMC_SEGS=256 PMC_ARGS=--verify \
  PMC_GROUPS="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS;SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU;SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT" \
  bash $R/tools/gpu_pmc.sh transmux
cat $O/bench*.log | grep '^{'
