#!/bin/bash
# Host peak memory (VmHWM) of the rank against the step count: N=1 bench and the N=8 projection
# (copy and RCCL planes) -- is the projection soak's 8.4 GiB a leak, and whose?
set -e
mkdir -p gpurun_out/r6_mem
export PYTHONPATH=.
hwm() { grep -o "hbm peak [0-9.]* GiB host peak [0-9.]* GiB" "$1" | head -1; }
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 20 --inflight 96 --verbose > gpurun_out/r6_mem/n1_2000.json 2> gpurun_out/r6_mem/n1_2000.err
echo "n1 k96 2000: $(hwm gpurun_out/r6_mem/n1_2000.err)"
for s in 500 2000; do
  timeout -k 10 300 python -u tools/project_swarm.py --peers 8 --plane copy --steps $s --warmup 20 --verbose > gpurun_out/r6_mem/copy_$s.json 2> gpurun_out/r6_mem/copy_$s.err
  echo "n8 copy $s: $(hwm gpurun_out/r6_mem/copy_$s.err)"
done
timeout -k 10 300 python -u tools/project_swarm.py --peers 8 --plane rccl --steps 500 --warmup 20 --verbose > gpurun_out/r6_mem/rccl_500.json 2> gpurun_out/r6_mem/rccl_500.err
echo "n8 rccl 500: $(hwm gpurun_out/r6_mem/rccl_500.err)"
timeout -k 10 300 python -u tools/project_swarm.py --peers 8 --config abr5 --churn 2 --steps 60 --warmup 10 > gpurun_out/r6_mem/abr5_churn8.json 2> gpurun_out/r6_mem/abr5_churn8.err
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['bench_record']; p=r['per_rank'][0]; print('abr5 churn', d['measured_ms_per_step'], d['measured_per_rank_value'], r['offload_ratio'], r['errors'], p['crc_failures'], round(p['cdn_GBps'],1))" gpurun_out/r6_mem/abr5_churn8.json
