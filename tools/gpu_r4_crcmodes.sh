# Kernel forms of the CRC fused into the AES-CBC decrypt (aes_cbc.hip kCrc), timed on one
# 256-segment transmux batch, plus a kernel trace of the fused batch (fold kernel time).
#   bash tools/gpu_r4_crcmodes.sh   -> gpurun_out/r4_crcmodes/*
set -eo pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_crcmodes
export PYTHONPATH=$R
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -m gpu -k "fused or crc" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 300 python tools/transmux_bench.py --segs 256 --iters 10 --verify > $O/modes.log 2>&1
timeout -k 10 300 python tools/transmux_bench.py --segs 256 --pool 256 --iters 10 --verify > $O/modes_pool256.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/transmux_bench.py --segs 256 --iters 5 --verify > $O/prof.log 2>&1
cat $O/modes*.log | grep '^{'
