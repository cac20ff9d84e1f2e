# Round-2 profile set: GPU tests, kernel stats of one bench round (rocprofv3 --kernel-trace
# --stats), PMC counter groups (one rocprofv3 run each, kernel trace only), and a headline
# bench run under --kernel-trace --memory-copy-trace --stats.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=$R/gpurun_out/r2prof
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python tools/kernel_bench.py > $O/kernel_bench.json 2> $O/kernel_bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kstats -o run --output-format csv -- python $R/tools/kernel_bench.py > $O/kstats.log 2>&1
i=0
for G in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT" "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TA_TA_BUSY_sum TD_TD_BUSY_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $G -d $O/pmc/g$i -o run --output-format csv -- python $R/tools/kernel_bench.py --iters 3 > $O/pmc_g$i.log 2>&1
done
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/bench -o run --output-format csv -- python $R/bench.py --steps 20 --warmup 5 --verbose > $O/bench.log 2>&1
