#!/bin/bash
# BASELINE.json configs 2-5 on one GPU (the driver runs the multi-GPU scaling): one bench per config,
# each under its own time limit; JSON lines into gpurun_out/<tag>/.  usage: tools/configs.sh <tag>
set -eo pipefail
TAG=${1:-cfg}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
run() { local name=$1; shift; timeout -k 10 400 python3 -u "$R/bench.py" "$@" > "$O/$name.log" 2>&1; tail -1 "$O/$name.log" > "$O/$name.json"; echo "$name done"; }
run cfg2 --steps 20 --warmup 3
run cfg3 --solver se3 --preset fr2 --nfeatures 2000 --no-cpu-baseline --steps 20 --warmup 3
run cfg4 --mode sequences --preset icl --no-cpu-baseline --flag-chain-steps 0
run cfg5 --preset corbs --posegraph --no-cpu-baseline --flag-chain-steps 0
run svo --extractor svo --no-cpu-baseline --flag-chain-steps 0
