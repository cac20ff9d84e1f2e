#!/bin/bash
# The N=8 projection at 64 / 96 / 128 fragments in flight per player (host cost per step amortized).
set -e
mkdir -p gpurun_out/r6_inflight
export PYTHONPATH=.
for k in 64 128 96; do
  timeout -k 10 300 python -u tools/project_swarm.py --peers 8 --steps 60 --warmup 20 --inflight $k --verbose \
    > gpurun_out/r6_inflight/n8_k$k.json 2> gpurun_out/r6_inflight/n8_k$k.err
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['bench_record']; p=r['per_rank'][0]; print(sys.argv[2], d['measured_ms_per_step'], d['measured_per_rank_value'], r['offload_ratio'], r['errors'], round(p['cdn_GBps'],1), round(p['wait_device_us'],1))" gpurun_out/r6_inflight/n8_k$k.json k$k
done
timeout -k 10 300 python -u tools/project_swarm.py --peers 4 --steps 40 --warmup 10 --inflight 128 \
  > gpurun_out/r6_inflight/n4_k128.json 2> gpurun_out/r6_inflight/n4_k128.err
python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['bench_record']; print('n4 k128', d['measured_ms_per_step'], d['measured_per_rank_value'], r['offload_ratio'], r['errors'])" gpurun_out/r6_inflight/n4_k128.json
