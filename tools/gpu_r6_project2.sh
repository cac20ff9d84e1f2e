#!/bin/bash
# The single-GPU projection with RCCL moving the received bytes (one-rank self-exchange):
# N=8 at the bench defaults, the D2D-copy plane for comparison, the CU-reserve calibration
# on the N=8 shape, and N=2 / N=4.
set -e
mkdir -p gpurun_out/r6_project2
export PYTHONPATH=.
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u tools/project_swarm.py "$@" --verbose > gpurun_out/r6_project2/$name.json 2> gpurun_out/r6_project2/$name.err
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['bench_record']; p=r['per_rank'][0]; print(sys.argv[2], d['plane'], d['rccl_spans'], d['measured_ms_per_step'], d['measured_per_rank_value'], r['offload_ratio'], r['errors'], p['crc_failures'], round(p['cdn_GBps'],1), p['cu_reserve'], r.get('calibration'))" gpurun_out/r6_project2/$name.json $name
}
run n8_rccl --peers 8 --steps 60 --warmup 20
run n8_copy --peers 8 --steps 60 --warmup 20 --plane copy
run n8_rccl_calib --peers 8 --steps 60 --warmup 20 --cu-calibrate force
run n4_rccl --peers 4 --steps 40 --warmup 10
run n2_rccl --peers 2 --steps 40 --warmup 10
