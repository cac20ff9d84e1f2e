# one-pass demux (split default): correctness vs oracle / four-pass / fused, then timings + kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3h
timeout -k 10 300 python -u -m pytest tests/test_transmux_fused.py tests/test_transmux.py tests/test_kernels_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $R/gpurun_out/r3h/tests.log 2>&1 &&
PYTHONPATH=$R timeout -k 10 300 python tools/transmux_bench.py --segs 256 --iters 10 > $R/gpurun_out/r3h/tb256.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r3h/prof -o run -- python3 $R/tools/transmux_bench.py --segs 256 --iters 5 > $R/gpurun_out/r3h/prof.log 2>&1
