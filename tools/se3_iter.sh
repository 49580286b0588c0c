#!/bin/bash
# One GPU iteration of the device-resident RansacSE3 chain (through gpurun): its parity tests, the config-3
# bench with chain statistics, and a kernel trace of the same bench.  usage: tools/se3_iter.sh <tag> [bench args]
set -o pipefail
TAG=${1:-se3}; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_track.py tests/test_gpu_lanes.py tests/test_gpu_gicp.py \
    tests/test_gpu_ransac.py tests/test_gpu_cpp_dropin.py -q --timeout 250 --timeout-method thread > "$O/gputest.log" 2>&1
echo "tests: $(tail -1 "$O/gputest.log")"
ARGS="--solver se3 --preset fr2 --nfeatures 2000 --steps 3 --warmup 1 --no-cpu-baseline $*"
timeout -k 10 300 python3 -u bench.py $ARGS > "$O/bench_se3.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$O/trace.log" 2>&1
rm -f "$O/trace/run_kernel_trace.csv"
echo done
