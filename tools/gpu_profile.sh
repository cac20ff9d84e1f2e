# Kernel-level profile of a bench run (rocprofv3 --kernel-trace; no PMC here — see
# gpu_pmc.sh): bash tools/gpu_profile.sh NAME [bench.py args ...]
#   -> gpurun_out/profile/NAME/ (rocpd database) and NAME/kernels.txt (tools/rocpd_kernels.py)
set -eo pipefail
R=$GRAFT_REPO_ROOT
NAME=${1:?name}
shift
O=$R/gpurun_out/profile/$NAME
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PYTHONPATH=$R timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $O/db -o run -- python3 $R/bench.py --steps 20 --warmup 5 "$@" > $O/bench.log 2>&1
python3 $R/tools/rocpd_kernels.py $(ls $O/db/*.db | head -1) > $O/kernels.txt
head -25 $O/kernels.txt
