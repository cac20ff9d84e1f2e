# Does batch k's demux overlap batch k+1's decrypt when consecutive transmux batches alternate
# over two streams and the decrypt grid leaves CUs free?   bash tools/gpu_r4_overlap.sh
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4_overlap
mkdir -p $O
timeout -k 10 300 python tools/transmux_bench.py --segs 128 --pool 64 --iters 20 --overlap 1:0,2:0,2:32,2:64,2:96,1:64 > $O/overlap.log 2>&1
timeout -k 10 300 python tools/transmux_bench.py --segs 128 --pool 64 --iters 20 --overlap 1:0,2:0,2:32,2:64,2:96,1:64 > $O/overlap2.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/prof -o run -- python3 $R/tools/transmux_bench.py --segs 128 --pool 64 --iters 6 --overlap 2:64 > $R/$O/prof.log 2>&1
grep -h '^{' $R/$O/overlap*.log
