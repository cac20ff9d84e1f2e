# Same-box A/B of an environment switch on the headline bench (interleaved runs):
#   bash tools/gpu_ab_env.sh VAR VALUE_A VALUE_B [bench args...]
set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
VAR=$1; A=$2; B=$3; shift 3
mkdir -p gpurun_out/abenv
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abenv/gpu_tests.log 2>&1
for i in 1 2 3; do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 200 python bench.py --verbose "$@" > gpurun_out/abenv/${VAR}_${v}_$i.log 2>&1
  done
done
