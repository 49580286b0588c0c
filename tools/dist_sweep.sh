#!/bin/bash
# Environment-shape sweep (through gpurun): the extraction GPU tests under each shape, then the default bench
# per shape, twice.  Each shape is a space-separated "VAR=V ..." string ("-" for none).
# usage: tools/dist_sweep.sh <tag> <shape>...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
i=0
for sh in "$@"; do
  i=$((i+1)); e=${sh/#-/}
  env $e timeout -k 10 300 python3 -u -m pytest tests/test_gpu_extract.py tests/test_gpu_bench_shape.py -x -q --timeout 120 --timeout-method thread > "$O/tests_$i.log" 2>&1 || { echo "tests [$sh] failed"; tail -30 "$O/tests_$i.log"; exit 1; }
  echo "tests [$sh]: $(tail -1 "$O/tests_$i.log")"
done
for rep in 1 2; do
  i=0
  for sh in "$@"; do
    i=$((i+1)); e=${sh/#-/}
    env $e timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --flag-chain-steps 0 --flag-chain-one-steps 0 > "$O/bench_${i}_$rep.log" 2>&1 || { echo "bench [$sh] failed"; tail -20 "$O/bench_${i}_$rep.log"; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['value'],d['ms_per_step_median'],{k:v[0] for k,v in d['kernels_ms_warmup'].items() if v[0]>0.1})" "$O/bench_${i}_$rep.log" "[$sh]"
  done
done
