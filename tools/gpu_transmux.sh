# Isolated transmux batch (256 x 3 MB AES-128 segments): decrypt + four-kernel demux timing,
# then a kernel trace of the same.   bash tools/gpu_transmux.sh   -> gpurun_out/transmux/*
set -eo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/transmux
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_transmux.py -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
PYTHONPATH=$R timeout -k 10 300 python tools/transmux_bench.py --segs 256 --iters 10 > $O/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace -d $O/db -o run -- python3 $R/tools/transmux_bench.py --segs 256 --iters 5 > $O/prof.log 2>&1
python3 $R/tools/rocpd_kernels.py $(ls $O/db/*.db | head -1) > $O/kernels.txt
grep '^{' $O/bench.log
