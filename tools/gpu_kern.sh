# Kernel iteration loop on one MI355X: GPU kernel tests, the per-kernel microbenchmark
# (HIP-event timings + host-oracle checks) and its rocprofv3 kernel stats.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/kern
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/kern/tests.log 2>&1
PYTHONPATH=$R timeout -k 10 120 python tools/kernel_bench.py > gpurun_out/kern/bench.json 2> gpurun_out/kern/bench.err
cd /tmp && export TMPDIR=/tmp
PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kern/prof -o run --output-format csv -- python $R/tools/kernel_bench.py > $R/gpurun_out/kern/prof.log 2>&1
