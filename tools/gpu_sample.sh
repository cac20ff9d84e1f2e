# Statistical host profile of the GPU bench path (pure-Python mode) + the compiled-mode
# phase timers, on the same box.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/sample
mkdir -p $O
SAMPLE_TOP=400 HLSJS_P2P_PURE=1 timeout -k 10 300 python tools/sample_prof.py --config ${CONFIG:-hostcost} --steps 1500 --warmup 10 --verbose > $O/pure.out 2> $O/pure.txt
timeout -k 10 300 python bench.py --config ${CONFIG:-hostcost} --steps 100 --warmup 10 --verbose > $O/compiled.out 2> $O/compiled.txt
