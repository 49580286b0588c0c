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
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --flag-chain-steps 0 --flag-chain-one-steps 0 --lowtex-steps 0 $*"
timeout -k 10 170 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/bench_trace.log" 2>&1 && echo "pass $(basename "$OUT")/bench_trace ok"
timeout -k 10 170 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/pmc_sq" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/pmc_sq.log" 2>&1 && echo "pass $(basename "$OUT")/pmc_sq ok"
timeout -k 10 170 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS -d "$OUT/pmc_lds" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/pmc_lds.log" 2>&1 && echo "pass $(basename "$OUT")/pmc_lds ok"
timeout -k 10 170 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE -d "$OUT/pmc_valu" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/pmc_valu.log" 2>&1 && echo "pass $(basename "$OUT")/pmc_valu ok"
timeout -k 10 170 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/pmc_fetch.log" 2>&1 && echo "pass $(basename "$OUT")/pmc_fetch ok"
timeout -k 10 170 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/pmc_write.log" 2>&1 && echo "pass $(basename "$OUT")/pmc_write ok"
python3 "$R/tools/pmc_summary.py" "$OUT/pmc_sq" "$OUT/pmc_lds" "$OUT/pmc_valu" "$OUT/pmc_fetch" "$OUT/pmc_write" --json "$OUT/pmc_summary.json" > "$OUT/pmc_summary.txt" 2>&1 || true
cp "$OUT/trace/run_kernel_stats.csv" "$OUT/kernel_stats.csv" 2>/dev/null || true
# the raw per-dispatch CSVs stay on the box (gpurun copies back at most 64 MiB); the summaries above are kept
rm -f "$OUT"/pmc_*/run_counter_collection.csv "$OUT/trace/run_kernel_trace.csv"
echo "profile done: $OUT"
