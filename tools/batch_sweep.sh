#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
for b in 1024 1536 2048 3072; do
  timeout -k 10 240 python3 -u $R/bench.py --no-cpu-baseline --flag-chain-steps 0 --steps 60 --batch $b > $R/gpurun_out/bs_$b.log 2>&1 || { echo "batch $b failed"; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['value'],d['ms_per_step'])" $R/gpurun_out/bs_$b.log $b
done
