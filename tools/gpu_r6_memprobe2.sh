#!/bin/bash
# Where the RCCL plane's host resident memory is (RssAnon / RssShmem), and the ABR + churn
# projection at N=8.
set -e
mkdir -p gpurun_out/r6_mem
export PYTHONPATH=.
for plane in copy rccl; do
  timeout -k 10 300 python -u tools/project_swarm.py --peers 8 --plane $plane --steps 300 --warmup 20 > gpurun_out/r6_mem/st_$plane.json 2> gpurun_out/r6_mem/st_$plane.err
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['measured_per_rank_value'], d['host_memory_MiB'])" gpurun_out/r6_mem/st_$plane.json $plane
done
timeout -k 10 300 python -u tools/project_swarm.py --peers 8 --config abr5 --churn 2 --steps 60 --warmup 10 > gpurun_out/r6_mem/abr5_churn8.json 2> gpurun_out/r6_mem/abr5_churn8.err
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['bench_record']; p=r['per_rank'][0]; print('abr5 churn', d['measured_ms_per_step'], d['measured_per_rank_value'], r['offload_ratio'], r['errors'], p['crc_failures'], round(p['cdn_GBps'],1))" gpurun_out/r6_mem/abr5_churn8.json
