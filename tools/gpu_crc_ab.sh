# CRC residue kernels A/B on one box: GPU tests, then rocprofv3 kernel stats of the kernel
# bench with the line-coalesced kernel (default) and the register kernel (HLSP2P_CRC_KERNEL=regs).
set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/crcab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/crcab/gpu_tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
for v in line regs; do
  HLSP2P_CRC_KERNEL=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/crcab/$v -o run --output-format csv -- python $R/tools/kernel_bench.py > $R/gpurun_out/crcab/$v.log 2>&1
done
