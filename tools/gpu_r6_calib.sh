#!/bin/bash
# Round 6: the CU-reserve calibration on the native RCCL plane (socket rehearsal, 2 ranks on
# the one GPU, fleet players) and the same candidates on the one-rank self-exchange rehearsal
# of an N=8 round beside the transmux (tools/overlap_n8.py).  profiles/r6_calib.
set -o pipefail
out=gpurun_out/r6_calib
mkdir -p $out
export HLSP2P_RCCL_LOG_DIR=$PWD/$out/rccl_logs
HLSP2P_RCCL_REHEARSAL=socket timeout -k 10 500 python -u bench.py --gpus 2 --steps 20 --warmup 3 --cache-gb 4 \
    --ingest hbm > $out/rehearsal_n2_fleet.json 2> $out/rehearsal_n2_fleet.err || exit $?
HLSP2P_RCCL_REHEARSAL=socket timeout -k 10 400 python -u bench.py --gpus 2 --steps 20 --warmup 3 --cache-gb 2 \
    --inflight 16 --players 0 --ingest hbm > $out/rehearsal_n2_inproc.json 2> $out/rehearsal_n2_inproc.err || exit $?
PYTHONPATH=. timeout -k 10 300 python -u tools/overlap_n8.py --options r0,r32,r64,r96 --only-steady --steady 10 \
    --iters 3 --repeat 2 > $out/overlap_world1.txt 2> $out/overlap_world1.err || exit $?
