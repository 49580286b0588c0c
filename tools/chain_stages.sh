#!/bin/bash
# Per-stage breakdown of the flag chain's pair (profiling build: k_pnp_chain's stage clocks, hyp_eval's EPnP
# stage cycles) from one flag_chain_one step.  usage: tools/chain_stages.sh <tag>
set -o pipefail
TAG=${1:-chain_stages}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
RGBD_HIP_LIB=$R/rgbd-slam_amd/${PROF_BUILD:-build_prof}/librgbd_hip.so timeout -k 10 200 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --flag-chain-steps 0 --flag-chain-one-steps 1 --se3-chain-one-steps 0 --cfg3-chain-steps 0 > "$O/prof.log" 2> "$O/prof.err" || { echo "prof run failed"; tail -5 "$O/prof.err"; exit 1; }
grep "chain_prof\|pnp_prof" "$O/prof.err" | tail -4 | tee "$O/stages.txt"
