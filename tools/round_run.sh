#!/bin/bash
# Round-end evidence on one GPU (through gpurun): the -m gpu suite, the default bench as the driver runs it,
# the smoke entry point, then the serial rocprofv3 passes (tools/profile.sh).  usage: tools/round_run.sh <tag>
set -o pipefail
TAG=${1:-round}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$O/gputest.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$O/gputest.log"; exit 1; }
echo "tests: $(tail -1 "$O/gputest.log")"
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$O/smoke.log"; exit 1; }
echo "smoke ok"
timeout -k 10 400 python3 -u bench.py > "$O/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" > "$O/bench.json"
echo "bench: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['ms_per_step_median'])" "$O/bench.json")"
SERIAL=1 timeout -k 10 900 bash "$R/tools/profile.sh" "$TAG/prof" || { echo "profile failed"; exit 1; }
echo done
