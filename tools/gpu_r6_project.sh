#!/bin/bash
# One rank of an N-rank swarm on one MI355X (tools/project_swarm.py), N = 2, 4, 8, plus N=1 bench.
set -e
mkdir -p gpurun_out/r6_project
export PYTHONPATH=.
timeout -k 10 240 python -u tools/project_swarm.py --peers 8 --steps 10 --warmup 5 \
  > gpurun_out/r6_project/smoke8.json 2> gpurun_out/r6_project/smoke8.err
cat gpurun_out/r6_project/smoke8.json | cut -c1-600
timeout -k 10 240 python -u bench.py --steps 60 --warmup 20 > gpurun_out/r6_project/n1_bench.json 2> gpurun_out/r6_project/n1_bench.err
cut -c1-300 gpurun_out/r6_project/n1_bench.json
for n in 2 4 8; do
  timeout -k 10 300 python -u tools/project_swarm.py --peers $n --steps 60 --warmup 20 --verbose \
    > gpurun_out/r6_project/n$n.json 2> gpurun_out/r6_project/n$n.err
  cut -c1-700 gpurun_out/r6_project/n$n.json
done
