# fused transmux: correctness after the per-class ES offsets, then isolated timing decomposition
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3e
timeout -k 10 300 python -u -m pytest tests/test_transmux_fused.py tests/test_transmux.py tests/test_kernels_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $R/gpurun_out/r3e/tests.log 2>&1 &&
PYTHONPATH=$R timeout -k 10 300 python tools/transmux_bench.py --segs 256 --iters 10 > $R/gpurun_out/r3e/tb256.log 2>&1 &&
PYTHONPATH=$R timeout -k 10 300 python tools/transmux_bench.py --segs 64 --iters 20 > $R/gpurun_out/r3e/tb64.log 2>&1
