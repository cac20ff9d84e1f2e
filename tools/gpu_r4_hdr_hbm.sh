# HBM-origin probe (device-bound) with the decrypt's packet-header records off / on, interleaved.
set -eo pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r4_hdr_hbm
mkdir -p $O
for i in 1 2; do
  HLSP2P_HDR_RECORDS=0 timeout -k 10 300 python bench.py --ingest hbm --steps 100 --warmup 6 > $O/off_$i.log 2>&1
  HLSP2P_HDR_RECORDS=1 timeout -k 10 300 python bench.py --ingest hbm --steps 100 --warmup 6 > $O/on_$i.log 2>&1
done
grep -H '^{' $O/*.log | cut -c1-200
