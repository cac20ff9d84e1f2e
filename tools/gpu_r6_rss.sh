#!/bin/bash
# Resident host memory of the projection's rank by stage (RCCL init, first exchanges, ...).
set -e
mkdir -p gpurun_out/r6_mem
export PYTHONPATH=.
for plane in rccl; do
  timeout -k 10 300 python -u tools/project_swarm.py --peers 8 --plane $plane --steps 200 --warmup 20 > gpurun_out/r6_mem/rss_$plane.json 2> gpurun_out/r6_mem/rss_$plane.err
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['host_memory_MiB'], d['rss_MiB_by_stage'])" gpurun_out/r6_mem/rss_$plane.json $plane
done
