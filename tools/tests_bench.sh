#!/bin/bash
# GPU tests + smoke + the default bench (through gpurun).  usage: tools/tests_bench.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-tb}; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 200 --timeout-method thread > "$O/gputest.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$O/gputest.log"; exit 1; }
echo "tests: $(tail -1 "$O/gputest.log")"
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$O/smoke.log"; exit 1; }
echo "smoke ok: $(tail -1 "$O/smoke.log")"
timeout -k 10 400 python3 -u bench.py "$@" > "$O/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" > "$O/bench.json"
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['ms_per_step'], d['ms_per_step_median'], 'flag1', (d.get('flag_chain_one') or {}).get('value'), 'se3one', (d.get('se3_chain_one') or {}).get('value'), {k: v[0] for k, v in d['kernels_ms_warmup'].items()})" "$O/bench.json"
