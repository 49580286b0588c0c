#!/bin/bash
# Quick GPU check (through gpurun): the extraction GPU tests, two default bench runs without the CPU and chain
# legs, then serial WRITE_SIZE / FETCH_SIZE passes (per-kernel HBM bytes).  usage: tools/quick_check.sh <tag>
set -o pipefail
TAG=${1:-quick}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 -u -m pytest ${TESTS:-tests/test_gpu_extract.py} -m gpu -x -q --timeout 150 --timeout-method thread > "$O/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$O/tests.log"; exit 1; }
echo "tests: $(tail -1 "$O/tests.log")"
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --cfg3-chain-steps 0 --flag-chain-steps 0 --se3-chain-one-steps 0 ${BENCH_ARGS:---flag-chain-one-steps 0} > "$O/bench$i.log" 2>&1 || { echo "bench failed"; tail -20 "$O/bench$i.log"; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith('{')][-1]); k=d['kernels_ms_warmup']; print('bench', d['value'], d['ms_per_step'], (d.get('flag_chain_one') or {}).get('value'), {n: v[0] for n, v in k.items()})" "$O/bench$i.log"
done
if [ -n "$PMC" ]; then
  cd /tmp && export TMPDIR=/tmp
  for c in WRITE_SIZE FETCH_SIZE; do
    RGBD_SERIAL=1 timeout -k 10 170 rocprofv3 --pmc $c -d "$O/pmc_$c" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 2 --no-cpu-baseline --cfg3-chain-steps 0 --flag-chain-steps 0 --flag-chain-one-steps 0 --se3-chain-one-steps 0 > "$O/pmc_$c.log" 2>&1 || { echo "pmc $c failed"; exit 1; }
    echo "pmc $c done"
  done
  python3 "$R/tools/pmc_summary.py" "$O/pmc_WRITE_SIZE" "$O/pmc_FETCH_SIZE" --json "$O/pmc.json" > "$O/pmc.txt" 2>&1 || true
  rm -f "$O"/pmc_*/run_counter_collection.csv
  grep -E "k_distribute|k_fast|k_describe|k_pyramid" "$O/pmc.txt" | head -8
fi
