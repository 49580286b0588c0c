#!/bin/bash
# Two serial PMC passes (SQ issue / wait counters; LDS) over a short bench run: per-kernel counters that
# belong to that kernel alone (RGBD_SERIAL=1).  usage: tools/pmc_quick.sh <tag> [bench args...]
set -eo pipefail
TAG=${1:-pmcq}; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export RGBD_SERIAL=1
ARGS="--steps 2 --warmup 2 --no-cpu-baseline --flag-chain-steps 0 --flag-chain-one-steps 0 --lowtex-steps 0 $*"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS -d "$OUT/pmc_sq" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/pmc_sq.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_MISC -d "$OUT/pmc_x" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/pmc_x.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$OUT/pmc_sq" "$OUT/pmc_x" --json "$OUT/pmc.json" > "$OUT/pmc.txt"
find "$OUT" -name "*_counter_collection.csv" -size +1M -delete   # keep the copy-back under 64 MiB
echo "pmc done: $OUT"
