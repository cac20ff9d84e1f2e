# GPU tests, smoke, the N=1 headline, then the driver's N=8 command and a tight-arena N=8 run
# on the native RCCL plane (socket-transport rehearsal: ranks share the one MI355X).
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${VAL_OUT:-r5_final}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py --verbose > $O/headline.log 2>&1
HLSP2P_RCCL_REHEARSAL=socket GPU_MAX_HW_QUEUES=1 timeout -k 10 400 python -u bench.py --gpus 8 > $O/n8_default.log 2>&1
HLSP2P_RCCL_REHEARSAL=socket GPU_MAX_HW_QUEUES=1 timeout -k 10 400 python -u bench.py --gpus 8 --steps 40 --warmup 3 --cache-gb 2 --corrupt-recv 3 > $O/n8_tight.log 2>&1
tail -1 $O/gpu_tests.log
grep -h '^{' $O/headline.log $O/n8_default.log $O/n8_tight.log | cut -c1-180
