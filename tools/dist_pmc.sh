#!/bin/bash
set -eo pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp RGBD_SERIAL=1
for v in build build_c1 build_c2 build_c3; do
  RGBD_HIP_LIB=$R/rgbd-slam_amd/$v/librgbd_hip.so timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU -d $R/gpurun_out/dpmc/$v -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 2 --no-cpu-baseline --flag-chain-steps 0 > $R/gpurun_out/dpmc/$v.log 2>&1
  python3 $R/tools/pmc_summary.py $R/gpurun_out/dpmc/$v | grep -E "kernel|k_distribute"
done
