#!/bin/bash
# GPU parity of experiment builds: the given tests against each library of VARIANTS (dirs under rgbd-slam_amd/),
# selected with RGBD_HIP_LIB; stops at the first failure.  usage: VARIANTS="build_x build_y" tools/variant_tests.sh <tag> <tests...>
set -o pipefail
TAG=${1:-variants}; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for v in $VARIANTS; do
  RGBD_HIP_LIB=$R/rgbd-slam_amd/$v/librgbd_hip.so timeout -k 10 ${TEST_TIMEOUT:-300} python3 -u -m pytest "$@" -m gpu -x -q --timeout 200 --timeout-method thread > "$O/tests_$v.log" 2>&1 || { echo "tests failed ($v)"; tail -30 "$O/tests_$v.log"; exit 1; }
  echo "$v: $(tail -1 "$O/tests_$v.log")"
done
