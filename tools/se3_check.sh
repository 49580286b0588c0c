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
for i in $(seq 1 $RUNS); do
  timeout -k 10 240 python3 -u bench.py --no-cpu-baseline --steps 5 --warmup 2 --flag-chain-steps 0 ${BENCH_ARGS} > "$O/bench$i.log" 2>&1 || { echo "bench failed"; tail -20 "$O/bench$i.log"; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith('{')][-1]); g=lambda k: (d.get(k) or {}).get('value'); print('bench', d['value'], d['ms_per_step'], 'flag_one', g('flag_chain_one'), 'se3_one', g('se3_chain_one'), (d.get('se3_chain_one') or {}).get('us_per_pair'), 'cfg3', g('se3_chain_one_cfg3'))" "$O/bench$i.log"
done
