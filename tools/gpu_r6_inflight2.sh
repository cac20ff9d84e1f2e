#!/bin/bash
# Interleaved A/B of the N=8 projection at 64 and 96 fragments in flight per player.
set -e
mkdir -p gpurun_out/r6_inflight
export PYTHONPATH=.
for rep in 1 2; do for k in 64 96; do
  timeout -k 10 300 python -u tools/project_swarm.py --peers 8 --steps 60 --warmup 20 --inflight $k \
    > gpurun_out/r6_inflight/ab_n8_k${k}_$rep.json 2> gpurun_out/r6_inflight/ab_n8_k${k}_$rep.err
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['bench_record']; p=r['per_rank'][0]; print(sys.argv[2], d['measured_ms_per_step'], d['measured_per_rank_value'], r['offload_ratio'], r['errors'], round(p['cdn_GBps'],1), round(p['wait_device_us'],1))" gpurun_out/r6_inflight/ab_n8_k${k}_$rep.json k$k.$rep
done; done
