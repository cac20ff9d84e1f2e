#!/bin/bash
# Round 6: the rank's host cost per step with peers (N=2 over the native RCCL plane, socket
# rehearsal on one GPU) against N=1, both with the HBM-resident origin (no PCIe bound), fleet
# players, --verbose phase timers.  profiles/r6_hostcost.
set -o pipefail
out=gpurun_out/r6_hostcost
mkdir -p $out
timeout -k 10 300 python -u bench.py --ingest hbm --steps 60 --warmup 5 --verbose > $out/n1_hbm.json 2> $out/n1_hbm.err || exit $?
HLSP2P_RCCL_REHEARSAL=socket timeout -k 10 500 python -u bench.py --gpus 2 --ingest hbm --steps 40 --warmup 5 \
    --verbose --cu-calibrate off > $out/n2_socket_hbm.json 2> $out/n2_socket_hbm.err || exit $?
