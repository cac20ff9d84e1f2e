# Second batch of native-RCCL-plane stress cases (ranks sharing ONE MI355X over the socket
# transport): 4K segments at N=4 with the default arena, the ABR ladder at N=8, the
# in-process player at N=8 with corruption, and a 300-step N=2 run.  The first failure ends it.
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R HLSP2P_RCCL_REHEARSAL=socket GPU_MAX_HW_QUEUES=1
O=gpurun_out/r5_rccl_stress2
mkdir -p $O
timeout -k 10 400 python -u bench.py --gpus 4 --config 4k25m --steps 20 --warmup 3 > $O/n4_4k.log 2>&1
timeout -k 10 400 python -u bench.py --gpus 8 --config abr5 --steps 30 --warmup 3 --cache-gb 4 > $O/n8_abr.log 2>&1
timeout -k 10 400 python -u bench.py --gpus 8 --players 0 --steps 60 --warmup 3 --cache-gb 4 --corrupt-recv 3 > $O/n8_inproc.log 2>&1
timeout -k 10 500 python -u bench.py --gpus 2 --steps 300 --warmup 5 > $O/n2_300.log 2>&1
grep -h '^{' $O/*.log | cut -c1-200
