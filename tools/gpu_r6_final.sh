#!/bin/bash
# Round-end validation on one MI355X: the GPU test suite (audit on), smoke(), the headline
# bench at its defaults, and a rocprofv3 kernel summary of a short headline run.
set -e
mkdir -p gpurun_out/r6_final
export PYTHONPATH=.
timeout -k 10 900 python -u -m pytest -x -v --timeout 450 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r6_final/gpu_tests.log 2>&1
tail -3 gpurun_out/r6_final/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/r6_final/smoke.log 2>&1
tail -1 gpurun_out/r6_final/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r6_final/head.json 2> gpurun_out/r6_final/head.err
grep '^{' gpurun_out/r6_final/head.json | cut -c1-400
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_final/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
  > gpurun_out/r6_final/prof_bench.log 2>&1
echo profiled
