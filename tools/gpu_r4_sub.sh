# Transmux batch split into back-to-back sub-batches so a sub-batch's plaintext is still in the
# 256 MiB Infinity Cache when the gather reads it:  bash tools/gpu_r4_sub.sh -> gpurun_out/r4_sub/*
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${SUB_OUT:-r4_sub}
mkdir -p $O
for i in 1 2; do
  for s in 0 128 64 32 16; do
    timeout -k 10 200 python tools/transmux_bench.py --segs 256 --pool 256 --iters 10 --verify --sub $s > $O/sub${s}_$i.log 2>&1
  done
done
cd /tmp && export TMPDIR=/tmp
for s in 0 32; do
  PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$s -o run -- python3 $R/tools/transmux_bench.py --segs 256 --pool 256 --iters 5 --verify --sub $s > $R/$O/prof_$s.log 2>&1
done
grep -H '^{' $R/$O/sub*.log | cut -c1-330
