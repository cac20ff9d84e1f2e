#!/bin/bash
# The N=8 projection over 2,000 steps (stability), and a rocprofv3 kernel summary of a short
# N=8 projection (RCCL's kernels beside the transmux).
set -e
mkdir -p gpurun_out/r6_project_soak
export PYTHONPATH=.
timeout -k 10 600 python -u tools/project_swarm.py --peers 8 --steps 2000 --warmup 50 --verbose \
  > gpurun_out/r6_project_soak/soak8.json 2> gpurun_out/r6_project_soak/soak8.err
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['bench_record']; p=r['per_rank'][0]; print('soak', d['measured_ms_per_step'], d['measured_per_rank_value'], r['offload_ratio'], r['errors'], p['crc_failures'], round(p['cdn_GBps'],1))" gpurun_out/r6_project_soak/soak8.json
grep "tenth\|hbm peak" gpurun_out/r6_project_soak/soak8.err | cut -c1-300
timeout -k 10 300 python -u tools/project_swarm.py --peers 8 --config abr5 --churn 2 --steps 60 --warmup 10 \
  > gpurun_out/r6_project_soak/abr5_churn8.json 2> gpurun_out/r6_project_soak/abr5_churn8.err
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['bench_record']; p=r['per_rank'][0]; print('abr5 churn', d['measured_ms_per_step'], d['measured_per_rank_value'], r['offload_ratio'], r['errors'], p['crc_failures'], round(p['cdn_GBps'],1))" gpurun_out/r6_project_soak/abr5_churn8.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_project_soak/prof -o run -- python3 tools/project_swarm.py --peers 8 --steps 30 --warmup 10 \
  > gpurun_out/r6_project_soak/prof.log 2>&1
echo profiled
