# Packet-header records from the decrypt for the demux scan (aes_cbc.hip AesHdr): GPU tests
# of the transmux paths, then the isolated batch with records off / on, kernel traces of both.
#   bash tools/gpu_r4_hdr.sh  -> gpurun_out/r4_hdr/*
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${HDR_OUT:-r4_hdr}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_transmux.py tests/test_kernels_gpu.py tests/test_torch_ops.py tests/test_fleet.py -x -v -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
for i in 1 2; do
  HLSP2P_HDR_RECORDS=0 timeout -k 10 300 python tools/transmux_bench.py --segs 256 --pool 256 --iters 10 --verify > $O/off_$i.log 2>&1
  HLSP2P_HDR_RECORDS=1 timeout -k 10 300 python tools/transmux_bench.py --segs 256 --pool 256 --iters 10 --verify > $O/on_$i.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
HLSP2P_HDR_RECORDS=0 PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/prof_off -o run -- python3 $R/tools/transmux_bench.py --segs 256 --pool 256 --iters 5 --verify > $R/$O/prof_off.log 2>&1
HLSP2P_HDR_RECORDS=1 PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/prof_on -o run -- python3 $R/tools/transmux_bench.py --segs 256 --pool 256 --iters 5 --verify > $R/$O/prof_on.log 2>&1
grep -H '^{' $R/$O/off_*.log $R/$O/on_*.log | cut -c1-330
