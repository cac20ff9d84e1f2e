# AES-CBC decrypt with buffer-resource loads/stores over each segment (out-of-range blocks read
# as 0 and their stores drop: no per-block predicates or zero fills) and the replicated InvSbox
# final round: GPU tests, the isolated batch twice, a kernel trace:
#   bash tools/gpu_r4_aesbuf.sh -> gpurun_out/r4_aesbuf_final/*
# (the interleaved A/B against the global-load form: profiles/r4_aesbuf/NOTES.md)
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4_aesbuf_final
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python tools/transmux_bench.py --segs 256 --pool 256 --iters 10 --verify > $O/tm_$i.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/prof -o run -- python3 $R/tools/transmux_bench.py --segs 256 --pool 256 --iters 5 --verify > $R/$O/prof.log 2>&1
grep -H '^{' $R/$O/tm_*.log | cut -c1-330
