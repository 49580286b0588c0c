#!/bin/bash
# A/B through gpurun: GPU extraction tests on the default build, a kernel-trace run of each library, then
# tools/se3_check.sh's alternating bench runs.  usage: LIBS="build build_x" tools/ab_run.sh <tag> [runs]
set -o pipefail
TAG=${1:-ab}; RUNS=${2:-2}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${TAG}p; mkdir -p "$O"
cd "$R"
timeout -k 10 400 python3 -u -m pytest ${TESTS:-tests/test_gpu_extract.py tests/test_gpu_lowtex.py tests/test_gpu_config5.py} -m gpu -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
cd /tmp && export TMPDIR=/tmp
for lib in ${LIBS:-build}; do
  RGBD_HIP_LIB=$R/rgbd-slam_amd/$lib/librgbd_hip.so timeout -k 10 170 rocprofv3 --kernel-trace --stats -d "$O/$lib" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --flag-chain-steps 0 --flag-chain-one-steps 0 --lowtex-steps 0 > "$O/$lib.log" 2>&1 || exit 1
  rm -f "$O/$lib/run_kernel_trace.csv"
done
cd "$R" && LIBS="${LIBS:-build}" bash tools/se3_check.sh "$TAG" "$RUNS"
