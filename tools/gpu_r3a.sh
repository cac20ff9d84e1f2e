# Round-3 first check: GPU tests, headline bench, HBM-origin probe (the N=8 per-GPU bound)
set -o pipefail
mkdir -p gpurun_out/r3a
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3a/gpu_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3a/bench.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --ingest hbm --verbose > gpurun_out/r3a/hbm.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --config hostcost --verbose > gpurun_out/r3a/hostcost.log 2>&1
