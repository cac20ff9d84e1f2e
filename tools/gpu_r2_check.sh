# Round-2 re-entry check: GPU tests, 1-GPU headline bench, host-cost probe, kernel stats.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --verbose > $O/bench_1080p.log 2>&1
timeout -k 10 300 python bench.py --config hostcost --verbose > $O/bench_hostcost.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/$O/prof -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 3 > $R/$O/prof.log 2>&1
