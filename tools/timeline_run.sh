#!/bin/bash
# Kernel timeline of a short default bench (through gpurun): tools/timeline_run.sh <tag> [steps to print] [bench args]
# Writes gpurun_out/<tag>/timeline.txt (tools/timeline.py) and drops the raw trace.
set -o pipefail
TAG=${1:-tl}; NS=${2:-6}; shift 2 || shift $#
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 12 --warmup 3 --no-cpu-baseline --flag-chain-steps 0 --flag-chain-one-steps 0 --se3-chain-one-steps 0 "$@" > "$O/bench.log" 2>&1 || exit 1
python3 "$R/tools/timeline.py" "$O/trace/run_kernel_trace.csv" --steps "$NS" --out "$O/timeline.txt" > /dev/null
rm -f "$O/trace/run_kernel_trace.csv"
tail -1 "$O/bench.log" | cut -c1-200
