#!/bin/bash
# Bench each in-tree library variant (RGBD_HIP_LIB) once: tools/sweep.sh <tag> <variant dirs...> [-- bench args]
# (run on the GPU box through gpurun; one bench process at a time, each under its own time limit)
set -o pipefail
TAG=$1; shift
V=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done; [ "$1" == "--" ] && shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out/$TAG"
for v in "${V[@]}"; do
  lib="$R/rgbd-slam_amd/$v/librgbd_hip.so"
  RGBD_HIP_LIB=$lib timeout -k 10 240 python3 -u "$R/bench.py" --no-cpu-baseline --flag-chain-steps 0 "$@" > "$R/gpurun_out/$TAG/$v.log" 2>&1 || { echo "variant $v failed rc=$?"; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['value'],d['ms_per_step_median'],{k:v[0] for k,v in d['kernels_ms_warmup'].items() if v[0]>0.3})" "$R/gpurun_out/$TAG/$v.log" "$v"
done
