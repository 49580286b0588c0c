#!/bin/bash
set -o pipefail
O=gpurun_out/r05_ctx; mkdir -p $O
for rep in 1 2; do
for L in 1 2 3; do
  timeout -k 10 200 python3 -u bench.py --lanes $L --no-cpu-baseline --flag-chain-steps 0 --flag-chain-one-steps 0 --se3-chain-one-steps 0 --cfg3-chain-steps 0 > $O/b_${L}_$rep.log 2>&1 || { echo "bench L=$L failed"; tail -5 $O/b_${L}_$rep.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith('{')][-1]); print('L', sys.argv[2], d['value'], d['ms_per_step'], d['ms_per_step_median'])" $O/b_${L}_$rep.log $L
done
done
