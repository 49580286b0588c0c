#!/bin/bash
# rocprofv3 passes over a short bench run (run on the GPU box through gpurun):
#   kernel trace + stats, then separate PMC passes (counters are never combined with other traces).
# usage: [SERIAL=1] tools/profile.sh <tag> [bench args...]
#   SERIAL=1 runs the library single-stream (RGBD_SERIAL=1: kernels never overlap), so the device-wide
#   TCC / SQ counters of a dispatch belong to that kernel alone (the attributable pass set).
set -eo pipefail
TAG=${1:-prof}; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
if [ "${SERIAL:-0}" != "0" ]; then export RGBD_SERIAL=1; fi
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --flag-chain-steps 0 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/bench_trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/pmc_sq" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/pmc_sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS -d "$OUT/pmc_lds" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/pmc_lds.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/pmc_write.log" 2>&1
echo "profile done: $OUT"
