#!/bin/bash
# Quadtree stage profile (profiling build, serial): [dist_prof] lines of frame 0 levels 0-3 per env shape.
# usage: tools/dist_prof.sh <tag> "<ENV=V ...>"...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
i=0
for e in "$@"; do
  i=$((i+1))
  env $e RGBD_HIP_LIB=$R/rgbd-slam_amd/build_prof/librgbd_hip.so timeout -k 10 200 python3 -u tools/orb_prof.py 1024 > "$O/prof_$i.log" 2>&1 || { echo "prof $e failed"; tail -5 "$O/prof_$i.log"; exit 1; }
  echo "== $e"; grep "dist_prof\|desc_prof" "$O/prof_$i.log" | tail -5
done
