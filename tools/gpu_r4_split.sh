# Split transmux batches (decrypt on the current stream with CUs left free, demux + fused-verify
# fold on a second stream): reserve sweep on 128 / 256-segment batches, GPU tests of the
# transmux paths, and a kernel trace of the split sequence.   bash tools/gpu_r4_split.sh
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${SPLIT_OUT:-r4_split}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_transmux.py tests/test_kernels_gpu.py tests/test_fleet.py -x -v -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 300 python tools/transmux_bench.py --segs 128 --pool 64 --iters 20 --split 0,32,48,64,80,96 > $O/split128.log 2>&1
timeout -k 10 300 python tools/transmux_bench.py --segs 256 --pool 256 --iters 10 --verify --split 0,48,64,80 > $O/split256.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/prof -o run -- python3 $R/tools/transmux_bench.py --segs 128 --pool 64 --iters 6 --split 64 > $R/$O/prof.log 2>&1
grep -h '^{' $R/$O/split*.log
