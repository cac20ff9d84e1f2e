set -o pipefail
mkdir -p gpurun_out/r2a
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a/pytest.log 2>&1 &&
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --verbose > gpurun_out/r2a/bench.log 2>&1 &&
timeout -k 10 120 python bench.py --config hostcost --steps 40 --warmup 10 --verbose > gpurun_out/r2a/hostcost.log 2>&1 &&
HLSP2P_PROFILE=gpurun_out/r2a/prof timeout -k 10 180 python bench.py --config hostcost --steps 40 --warmup 10 > gpurun_out/r2a/hostcost_prof.log 2>&1
