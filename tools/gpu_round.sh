set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 6 --verbose > gpurun_out/bench_pipe.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 6 --verbose --sync-steps --players 0 > gpurun_out/bench_sync.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/prof2 -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 4 > $R/gpurun_out/prof2.log 2>&1
