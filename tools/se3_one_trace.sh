#!/bin/bash
# Kernel trace of the se3_chain_one leg alone (the tracker's RansacSE3 -> second reference -> GICP chain over
# the batch, one lane): per-kernel mean duration and the mean gap before each kernel (dispatch latency of a
# serially dependent launch sequence).  usage: tools/se3_one_trace.sh <tag> [bench args]
set -o pipefail
TAG=${1:-se3_one}; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --flag-chain-steps 0 --flag-chain-one-steps 0 --cfg3-chain-steps 0 --se3-chain-one-steps 1 "$@" > "$O/bench.log" 2>&1 || { echo "trace failed"; tail -5 "$O/bench.log"; exit 1; }
python3 - "$O/trace/run_kernel_trace.csv" > "$O/se3_one.txt" <<'PY'
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
lane = {"k_lane_match", "k_ransac_hyp_lanes", "k_lane_replay", "k_knn2m"}
# the last contiguous run of lane-chain kernels (the timed se3_chain_one call)
seq, cur = [], []
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("rgbd::", "").replace("void ", "")
    if n in lane: cur.append((n, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    elif n.startswith("k_gicp") or n.startswith("__amd"):
        continue
    else:
        if len(cur) > len(seq): seq = cur
        cur = []
if len(cur) > len(seq): seq = cur
dur, gap, cnt = collections.defaultdict(float), collections.defaultdict(float), collections.Counter()
ph = {"k_ransac_hyp_lanes": 0, "k_lane_replay": 0}
for i, (n, s, e) in enumerate(seq):
    if n == "k_lane_match": ph = {"k_ransac_hyp_lanes": 0, "k_lane_replay": 0}
    if n in ph:   # the round's phase 0, 1, 2 (launch order inside the round)
        k = n + "[%d]" % ph[n]; ph[n] += 1
    else:
        k = n
    dur[k] += e - s; cnt[k] += 1
    if i: gap[k] += s - seq[i - 1][2]
span = (seq[-1][2] - seq[0][1]) / 1e3 if seq else 0
print("lane-chain dispatches %d over %.1f us" % (len(seq), span))
for n in sorted(cnt): print("%-20s n %6d  mean dur %7.2f us  mean gap before %6.2f us" % (n, cnt[n], dur[n] / cnt[n] / 1e3, gap[n] / cnt[n] / 1e3))
PY
cat "$O/se3_one.txt"
grep '^{' "$O/bench.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('se3_chain_one', (d.get('se3_chain_one') or {}).get('value'))"
rm -f "$O/trace/run_kernel_trace.csv"
