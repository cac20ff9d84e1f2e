#!/bin/bash
# The N=8 single-GPU projection (RCCL self-exchange receives) on the other BASELINE configs.
set -e
mkdir -p gpurun_out/r6_project_cfg
export PYTHONPATH=.
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u tools/project_swarm.py --peers 8 "$@" > gpurun_out/r6_project_cfg/$name.json 2> gpurun_out/r6_project_cfg/$name.err
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['bench_record']; p=r['per_rank'][0]; print(sys.argv[2], d['measured_ms_per_step'], d['measured_per_rank_value'], r['offload_ratio'], r['errors'], p['crc_failures'], round(p['cdn_GBps'],1), r['config'].get('model','')[:60])" gpurun_out/r6_project_cfg/$name.json $name
}
run abr5 --config abr5 --steps 40 --warmup 10
run 4k25m --config 4k25m --steps 30 --warmup 10 --cache-gb 24
run live --config 1080p6m-live --steps 200 --warmup 40
run hostcost --config hostcost --steps 60 --warmup 20
run dvr --steps 60 --warmup 20
