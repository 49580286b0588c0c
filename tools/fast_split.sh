#!/bin/bash
# VALU / SALU of k_fast's blur blocks against its FAST segments: the profiling build (make prof) with
# RGBD_PROF_FAST_SPLIT=1 dispatches them as two k_fast launches (blur-only grid first); one serial PMC pass,
# summarised per (kernel, grid size).  usage: tools/fast_split.sh <tag>
set -eo pipefail
TAG=${1:-fast_split}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export RGBD_SERIAL=1 RGBD_PROF_FAST_SPLIT=1 RGBD_HIP_LIB=$R/rgbd-slam_amd/build_prof/librgbd_hip.so
ARGS="--steps 2 --warmup 2 --no-cpu-baseline --flag-chain-steps 0 --flag-chain-one-steps 0 --se3-chain-one-steps 0 --cfg3-chain-steps 0"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS -d "$OUT/pmc" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/pmc.log" 2>&1
python3 "$R/tools/pmc_summary.py" --by-grid "$OUT/pmc" > "$OUT/split.txt"
grep -E "kernel|k_fast" "$OUT/split.txt"
find "$OUT" -name "*_counter_collection.csv" -size +1M -delete
