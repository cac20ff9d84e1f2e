# rocprofv3 kernel stats of the per-kernel microbenchmark (tools/kernel_bench.py)
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kprof -o run --output-format csv -- python $R/tools/kernel_bench.py > $R/gpurun_out/kprof.log 2>&1
