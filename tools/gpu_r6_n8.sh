#!/bin/bash
# Round 6: the driver's N=8 command shape (bench.py --gpus 8, self-launched, default fleet
# config) on the one-GPU box over the native RCCL plane's socket transport: the record's wire
# (NET/Socket on every pair, parsed from RCCL's log), the calibration before warmup, the
# per-rank rows.  profiles/r6_n8.
set -o pipefail
out=gpurun_out/r6_n8
mkdir -p $out
export HLSP2P_RCCL_LOG_DIR=$PWD/$out/rccl_logs
HLSP2P_RCCL_REHEARSAL=socket timeout -k 10 900 python -u bench.py --gpus 8 --steps 20 --warmup 5 --cache-gb 4 \
    > $out/n8.json 2> $out/n8.err || exit $?
