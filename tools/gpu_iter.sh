#!/bin/bash
# One GPU iteration (through gpurun): the full -m gpu suite, the default bench, then two serial PMC
# passes (tools/pmc_quick.sh).  usage: tools/gpu_iter.sh <tag> [bench args...]
set -eo pipefail
TAG=${1:-iter}; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/gputest.log" 2>&1
echo "tests: $(tail -1 "$O/gputest.log")"
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline "$@" > "$O/bench.log" 2>&1
tail -1 "$O/bench.log" > "$O/bench.json"
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['ms_per_step'], d['ms_per_step_median'], {k: v[0] for k, v in d['kernels_ms_warmup'].items()})" "$O/bench.json"
"$R/tools/pmc_quick.sh" "$TAG/pmc" "$@"
cat "$O/pmc/pmc.txt"
