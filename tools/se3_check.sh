#!/bin/bash
# GPU check of the tracking chains (through gpurun): the given GPU tests, then bench runs whose se3_chain_one /
# se3_chain_one_cfg3 legs time the single RansacSE3 chains.  usage: tools/se3_check.sh <tag> [runs]
set -o pipefail
TAG=${1:-se3}
RUNS=${2:-2}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python3 -u -m pytest $TESTS -m gpu -x -v --timeout 400 --timeout-method thread > "$O/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$O/tests.log"; exit 1; }
  echo "tests: $(tail -1 "$O/tests.log")"
fi
# LIBS: in-tree builds to time (dir names under rgbd-slam_amd/, e.g. "build build_c1"); runs alternate between them
for i in $(seq 1 $RUNS); do
  for lib in ${LIBS:-build}; do
    RGBD_HIP_LIB=$R/rgbd-slam_amd/$lib/librgbd_hip.so timeout -k 10 240 python3 -u bench.py --no-cpu-baseline --steps 5 --warmup 2 --flag-chain-steps 0 ${BENCH_ARGS} > "$O/bench_${lib}_$i.log" 2>&1 || { echo "bench failed ($lib)"; tail -20 "$O/bench_${lib}_$i.log"; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith('{')][-1]); g=lambda k: (d.get(k) or {}).get('value'); u=lambda k: (d.get(k) or {}).get('us_per_pair'); print(sys.argv[2], 'bench', d['value'], d['ms_per_step'], 'flag_one', g('flag_chain_one'), 'se3_one', g('se3_chain_one'), u('se3_chain_one'), 'cfg3', g('se3_chain_one_cfg3'), u('se3_chain_one_cfg3'), 'lowtex', g('lowtex'), (d.get('lowtex') or {}).get('k_fast_ms'))" "$O/bench_${lib}_$i.log" "$lib"
  done
done
