# One iteration on the MI355X: GPU tests, per-kernel microbenchmark + rocprofv3 kernel
# stats, and the 1080p / host-ceiling benches.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/kern gpurun_out/host
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/kern/tests.log 2>&1
PYTHONPATH=$R timeout -k 10 120 python tools/kernel_bench.py > gpurun_out/kern/bench.json 2> gpurun_out/kern/bench.err
timeout -k 10 300 python bench.py --steps 30 --warmup 6 --verbose > gpurun_out/host/bench_1080p.log 2>&1
timeout -k 10 300 python bench.py --config hostcost --steps 30 --warmup 6 --verbose > gpurun_out/host/bench_hostcost.log 2>&1
cd /tmp && export TMPDIR=/tmp
PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kern/prof -o run --output-format csv -- python $R/tools/kernel_bench.py > $R/gpurun_out/kern/prof.log 2>&1
