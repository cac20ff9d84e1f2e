# The fused verify's fold and combine as one kernel per segment (crc32_fold_combine_kernel):
# GPU tests, then the isolated batch three times.  (The A/B against the two-kernel form used a
# temporary knob, since removed with that form: profiles/r4_dpp/NOTES.md.)
#   bash tools/gpu_r4_foldcombine.sh -> gpurun_out/r4_foldcombine/*
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4_foldcombine
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_transmux.py tests/test_kernels_gpu.py tests/test_torch_ops.py tests/test_fleet.py -x -v -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_multirank_gpu.py -x -v -m gpu -k corrupted --timeout 300 --timeout-method thread -p no:cacheprovider > $O/multirank.log 2>&1
for i in 1 2 3; do
  timeout -k 10 200 python tools/transmux_bench.py --segs 256 --pool 256 --iters 10 --verify > $O/fc1_$i.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/prof -o run -- python3 $R/tools/transmux_bench.py --segs 256 --pool 256 --iters 5 --verify > $R/$O/prof.log 2>&1
cd $R
grep -h -o '"fused_us_per_seg": [0-9.]*' $O/fc1_*.log | tr '\n' ' '; echo " <- fold+combine"
tail -1 $O/tests.log; tail -1 $O/multirank.log
