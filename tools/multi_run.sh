#!/bin/bash
# One GPU call, several evidence steps (through gpurun), stopping at the first failure:
#   tools/chain_ab.sh <tag>  (the -m gpu suite, flag-chain trace, stage profile, default bench)
#   tools/timeline_run.sh <tag>/tl  (kernel timeline of the default bench's steady state)
#   SERIAL=1 tools/profile.sh <tag>/prof  (kernel trace + the serial PMC passes)
#   ab:<build dir>  (tools/ab_lib.sh: the variant build's extraction tests, then bench A/B x3)
#   tlv:<build dir>  (the timeline with the variant build)
# usage: tools/multi_run.sh <tag> [chain|timeline|profile|ab:<dir>|tlv:<dir> ...]   (default: the first three)
set -o pipefail
TAG=${1:-multi}; shift || true
STEPS=${*:-chain timeline profile}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out/$TAG"
for s in $STEPS; do
  case $s in
    chain) bash "$R/tools/chain_ab.sh" "$TAG" || exit 1 ;;
    timeline) bash "$R/tools/timeline_run.sh" "$TAG/tl" 6 || { echo "timeline failed"; exit 1; }
              head -60 "$R/gpurun_out/$TAG/tl/timeline.txt" ;;
    ab:*) V=${s#ab:}; bash "$R/tools/ab_lib.sh" "$V" 3 || { echo "ab $V failed"; exit 1; } ;;
    tlv:*) V=${s#tlv:}; RGBD_HIP_LIB=$R/rgbd-slam_amd/$V/librgbd_hip.so bash "$R/tools/timeline_run.sh" "$TAG/tl_$V" 6 || { echo "timeline $V failed"; exit 1; }
           grep -A3 "^step" "$R/gpurun_out/$TAG/tl_$V/timeline.txt" | head -12; grep "knn2m\|queue" "$R/gpurun_out/$TAG/tl_$V/timeline.txt" | head -12 ;;
    profile) SERIAL=1 timeout -k 10 900 bash "$R/tools/profile.sh" "$TAG/prof" || { echo "profile failed"; exit 1; }
             cat "$R/gpurun_out/$TAG/prof/pmc_summary.txt" | head -40 ;;
  esac
done
echo "multi_run done"
