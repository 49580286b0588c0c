#!/bin/bash
set -o pipefail
O=gpurun_out/${TAG}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_extract.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for i in 1 2 3; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --cfg3-chain-steps 0 --flag-chain-steps 0 --se3-chain-one-steps 0 --flag-chain-one-steps 0 > $O/bench$i.log 2>&1 || { echo "bench failed"; tail -20 $O/bench$i.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith('{')][-1]); k=d['kernels_ms_warmup']; print('bench', d['value'], d['ms_per_step'], k['k_distribute'][0], k['k_describe'][0])" $O/bench$i.log
done
