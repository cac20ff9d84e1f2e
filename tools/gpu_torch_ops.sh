# torch.ops.hlsp2p dispatcher registration on the MI355X: the kernel suite through the dispatcher.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tops
timeout -k 10 300 python -u -m pytest tests/test_torch_ops.py tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/tops/test.log 2>&1
