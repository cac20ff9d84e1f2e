# Kernel traces of the N=8 overlap rehearsal (tools/overlap_n8.py), CU reserve 8 vs 64:
# how much RCCL kernel time runs beside a resident decrypt grid (tools/overlap_trace.py).
set -eo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_trace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for opt in base r64; do
  PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace -d $O/$opt -o run -- python3 $R/tools/overlap_n8.py --iters 1 --steady 10 --options $opt > $O/$opt.log 2>&1
  python3 $R/tools/overlap_trace.py $(ls $O/$opt/*.db | head -1) > $O/$opt.json
  python3 $R/tools/rocpd_kernels.py $(ls $O/$opt/*.db | head -1) > $O/${opt}_kernels.txt
  cat $O/$opt.json
done
