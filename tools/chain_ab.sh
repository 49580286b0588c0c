#!/bin/bash
# Flag-chain A/B through gpurun: the -m gpu suite, the flag_chain_one kernel trace of an older in-tree build
# (build_old/, when present) and of the current build, the profiling build's per-stage breakdown of the
# chain kernel, then the default bench.  usage: tools/chain_ab.sh <tag>
set -o pipefail
TAG=${1:-chain_ab}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$O/gputest.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$O/gputest.log"; exit 1; }
echo "tests: $(tail -1 "$O/gputest.log")"
if [ -f "$R/rgbd-slam_amd/build_old/librgbd_hip.so" ]; then
  RGBD_HIP_LIB=$R/rgbd-slam_amd/build_old/librgbd_hip.so bash "$R/tools/chain_prof.sh" "$TAG/old" || exit 1
  cat "$O/old/chain.txt"
fi
bash "$R/tools/chain_prof.sh" "$TAG/new" || exit 1
python3 "$R/tools/kstats.py" "$O/new/kernel_stats.csv" | grep -i "chain\|gather\|knn" || true
cd "$R"
RGBD_HIP_LIB=$R/rgbd-slam_amd/build_prof/librgbd_hip.so timeout -k 10 200 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --flag-chain-steps 0 --flag-chain-one-steps 1 > "$O/prof.log" 2> "$O/prof.err" || { echo "prof run failed"; tail -5 "$O/prof.err"; exit 1; }
grep "chain_prof\|pnp_prof\|ref_prof" "$O/prof.err" | tail -6
grep "fast_prof\|desc_prof" "$O/prof.err" | tail -2
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > "$O/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$O/bench.log"; exit 1; }
grep '^{' "$O/bench.log" | tail -1 > "$O/bench.json"
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['ms_per_step'], d['ms_per_step_median'], 'flag_chain', d['flag_chain']['value'], 'one', d['flag_chain_one']['value'], 'se3_one', (d.get('se3_chain_one') or {}).get('value'))" "$O/bench.json"
