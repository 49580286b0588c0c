#!/bin/bash
# A/B of another in-tree build of the library against build/ (through gpurun): the extraction GPU tests on
# the variant, then the default bench alternately on both.  usage: [BASE=<base build>] [TESTS=<files>] tools/ab_lib.sh <variant build dir> [reps]
set -eo pipefail
V=$1; N=${2:-2}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/ab_$(basename "$V")
BL=$R/rgbd-slam_amd/${BASE:-build}/librgbd_hip.so
mkdir -p "$O"
cd "$R"
RGBD_HIP_LIB=$R/rgbd-slam_amd/$V/librgbd_hip.so timeout -k 10 300 python3 -u -m pytest ${TESTS:-tests/test_gpu_extract.py tests/test_gpu_bench_shape.py} -x -q --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1
echo "variant tests: $(tail -1 "$O/tests.log")"
for i in $(seq 1 "$N"); do
  RGBD_HIP_LIB=$BL timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --flag-chain-steps 0 --flag-chain-one-steps 0 --se3-chain-one-steps 0 --cfg3-chain-steps 0 > "$O/base$i.log" 2>&1
  RGBD_HIP_LIB=$R/rgbd-slam_amd/$V/librgbd_hip.so timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --flag-chain-steps 0 --flag-chain-one-steps 0 --se3-chain-one-steps 0 --cfg3-chain-steps 0 > "$O/var$i.log" 2>&1
done
for f in "$O"/base*.log "$O"/var*.log; do
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith('{')][-1]); k=d['kernels_ms_warmup']; print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], {n: k[n][0] for n in ('k_fast','k_distribute','k_describe','k_pyramid') if n in k})" "$f"
done
