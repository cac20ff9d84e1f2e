# Stress cases of the native RCCL plane with ranks sharing ONE MI355X (socket transport
# rehearsal): the driver's default N=8 shape, tight arenas (backpressure), churn, the
# in-process player, the ABR ladder and the live channel.  Each case runs under its own
# time limit; the first case that fails in any way ends the script.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R HLSP2P_RCCL_REHEARSAL=socket GPU_MAX_HW_QUEUES=1
O=gpurun_out/${STRESS_OUT:-r5_rccl_stress}
mkdir -p $O
timeout -k 10 400 python -u bench.py --gpus 8 > $O/n8_default.log 2>&1
timeout -k 10 400 python -u bench.py --gpus 8 --steps 40 --warmup 3 --cache-gb 2 > $O/n8_tight.log 2>&1
timeout -k 10 400 python -u bench.py --gpus 8 --steps 30 --warmup 3 --cache-gb 4 --churn 2 > $O/n8_churn.log 2>&1
timeout -k 10 300 python -u bench.py --gpus 4 --players 0 --steps 60 --warmup 3 --cache-gb 4 --corrupt-recv 3 > $O/n4_inproc.log 2>&1
timeout -k 10 400 python -u bench.py --gpus 4 --config abr5 --steps 40 --warmup 3 --cache-gb 4 --churn 2 > $O/n4_abr_churn.log 2>&1
timeout -k 10 400 python -u bench.py --gpus 4 --config 1080p6m-live --steps 30 --warmup 3 --cache-gb 4 > $O/n4_live.log 2>&1
grep -h '^{' $O/*.log | cut -c1-200
