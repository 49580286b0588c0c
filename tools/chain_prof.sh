#!/bin/bash
# Kernel trace of the reference-semantics outlier-flag chain (flag_chain_one: ONE unbroken chain over the
# batch) through gpurun, reduced to a per-round breakdown (tools/chain_trace.py).
# usage: tools/chain_prof.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-chain}; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --flag-chain-steps 0 --flag-chain-one-steps 1 --se3-chain-one-steps 0 "$@" > "$O/bench.log" 2>&1 || { echo "chain trace failed"; tail -20 "$O/bench.log"; exit 1; }
python3 "$R/tools/chain_trace.py" "$O/trace/run_kernel_trace.csv" --out "$O/chain.txt"
cp "$O/trace/run_kernel_stats.csv" "$O/kernel_stats.csv" 2>/dev/null || true
rm -f "$O/trace/run_kernel_trace.csv"
grep '^{' "$O/bench.log" | tail -1 > "$O/bench.json"
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('flag_chain_one', d.get('flag_chain_one'), 'se3_chain_one', d.get('se3_chain_one'))" "$O/bench.json"
