#!/bin/bash
# Per-stage breakdown of the se3 chain's kernels (profiling build: k_lane_match's and the RansacSE3
# hypothesis blocks' stage clocks) from one se3_chain_one step.  usage: tools/se3_stages.sh <tag>
set -o pipefail
TAG=${1:-se3_stages}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
RGBD_HIP_LIB=$R/rgbd-slam_amd/${PROF_BUILD:-build_prof}/librgbd_hip.so timeout -k 10 200 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --flag-chain-steps 0 --flag-chain-one-steps 0 --cfg3-chain-steps 0 --se3-chain-one-steps 1 > "$O/prof.log" 2> "$O/prof.err" || { echo "prof run failed"; tail -5 "$O/prof.err"; exit 1; }
grep "lane_prof\|hyp_prof\|lm_prof\|sort_prof\|replay_prof\|svd_prof\|sort_seg\|wp_prof" "$O/prof.err" | tail -14 | tee "$O/stages.txt"
