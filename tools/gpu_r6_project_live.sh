#!/bin/bash
# The N=8 projection on the live config and the DVR headline shape after the seeder rotation.
set -e
mkdir -p gpurun_out/r6_project_cfg
export PYTHONPATH=.
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u tools/project_swarm.py --peers 8 "$@" > gpurun_out/r6_project_cfg/$name.json 2> gpurun_out/r6_project_cfg/$name.err
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['bench_record']; p=r['per_rank'][0]; print(sys.argv[2], d['measured_ms_per_step'], d['measured_per_rank_value'], r['offload_ratio'], r['errors'], p['crc_failures'], round(p['cdn_GBps'],2), d['received_rows'])" gpurun_out/r6_project_cfg/$name.json $name
}
run live_rot --config 1080p6m-live --steps 200 --warmup 40
run dvr_rot --steps 60 --warmup 20
