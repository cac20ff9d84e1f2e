# hipGraph question: host cost per launch, eager vs graph replay (tools/graph_probe.py), and
# the kernel / copy timeline of the host-bound config (launches per step, device idle time).
set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/graph
mkdir -p $O
timeout -k 10 180 python tools/graph_probe.py > $O/graph_probe.json 2> $O/graph_probe.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/$O/prof -o run --output-format csv -- python $R/bench.py --config hostcost --steps 20 --warmup 4 > $R/$O/prof.log 2>&1
