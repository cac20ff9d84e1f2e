#!/bin/bash
# rocprofv3 kernel summary of the N=8 single-GPU projection (RCCL plane): RCCL's kernels beside
# the transmux kernels.
set -e
mkdir -p gpurun_out/r6_project_prof
export PYTHONPATH=.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_project_prof/prof -o run -- python3 tools/project_swarm.py --peers 8 --steps 30 --warmup 10 \
  > gpurun_out/r6_project_prof/prof.log 2>&1
grep '^{' gpurun_out/r6_project_prof/prof.log | cut -c1-300 || true
echo profiled
