# CRC matrix-core variants (fp4 f8f6f4 vs i8) on one bench round: correctness tests, then
# interleaved kernel_bench runs and a rocprofv3 kernel-stats pass of each.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/crcv
mkdir -p $O
for v in fp4 i8; do
  HLSP2P_CRC_MFMA=$v timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_crc_algebra.py -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1
done
for i in 1 2; do
  for v in fp4 i8; do
    HLSP2P_CRC_MFMA=$v timeout -k 10 120 python tools/kernel_bench.py > $O/kb_${v}_$i.json 2> $O/kb_${v}_$i.err
  done
done
cd /tmp && export TMPDIR=/tmp
for v in fp4 i8; do
  HLSP2P_CRC_MFMA=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$v -o run --output-format csv -- python $R/tools/kernel_bench.py > $R/$O/prof_$v.log 2>&1
done
