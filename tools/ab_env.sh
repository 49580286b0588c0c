#!/bin/bash
# A/B of one environment knob on the default bench: tools/ab_env.sh <tag> <VAR> <v1> <v2> [rounds] [-- bench args]
# (run on the GPU box through gpurun; one bench process at a time, each under its own time limit)
set -o pipefail
TAG=$1; VAR=$2; A=$3; B=$4; N=${5:-2}; shift 5 || shift $#
[ "$1" == "--" ] && shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out/$TAG"
for i in $(seq 1 $N); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 240 python3 -u "$R/bench.py" --no-cpu-baseline --flag-chain-steps 0 --flag-chain-one-steps 0 "$@" > "$R/gpurun_out/$TAG/$VAR-$v-$i.log" 2>&1 || { echo "$VAR=$v failed rc=$?"; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['value'],d['ms_per_step_median'],{k:v[0] for k,v in d['kernels_ms_warmup'].items() if v[0]>0.2})" "$R/gpurun_out/$TAG/$VAR-$v-$i.log" "$VAR=$v"
  done
done
