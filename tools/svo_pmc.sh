#!/bin/bash
# PMC passes over tools/svo_prof.py (run on the GPU box)
set -eo pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/svo_pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/tools/svo_prof.py > $OUT/trace.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/sq -o run --output-format csv -- python3 $R/tools/svo_prof.py > $OUT/sq.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS -d $OUT/lds -o run --output-format csv -- python3 $R/tools/svo_prof.py > $OUT/lds.log 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $R/tools/svo_prof.py > $OUT/fetch.log 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $R/tools/svo_prof.py > $OUT/write.log 2>&1
echo done
