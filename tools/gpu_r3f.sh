# warp-specialised fused transmux: correctness, then isolated timing decomposition + role timers
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3f
timeout -k 10 240 python -u -m pytest tests/test_transmux_fused.py -x -v -m gpu --timeout 60 --timeout-method thread -p no:cacheprovider > $R/gpurun_out/r3f/tests.log 2>&1 &&
PYTHONPATH=$R timeout -k 10 300 python tools/transmux_bench.py --segs 256 --iters 10 --prof > $R/gpurun_out/r3f/tb256.log 2>&1 &&
PYTHONPATH=$R timeout -k 10 300 python tools/transmux_bench.py --segs 256 --iters 10 --prof --flags 1 > $R/gpurun_out/r3f/tb256_noprio.log 2>&1
