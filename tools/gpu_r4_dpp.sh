# Wave scans and sums of the demux kernels on DPP (row_shr / row_bcast) instead of ds_bpermute
# shuffles: GPU tests of the demux paths, the isolated batch twice, and a kernel trace.
#   bash tools/gpu_r4_dpp.sh -> gpurun_out/r4_dpp/*
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${DPP_OUT:-r4_dpp}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_transmux.py tests/test_kernels_gpu.py tests/test_torch_ops.py tests/test_fleet.py -x -v -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python tools/transmux_bench.py --segs 256 --pool 256 --iters 10 --verify > $O/tm_$i.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/prof -o run -- python3 $R/tools/transmux_bench.py --segs 256 --pool 256 --iters 5 --verify > $R/$O/prof.log 2>&1
grep -H '^{' $R/$O/tm_*.log | cut -c1-330
tail -1 $R/$O/tests.log
