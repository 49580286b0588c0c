"""Per-round breakdown of the outlier-flag chain from a rocprofv3 kernel trace (run_kernel_trace.csv).

A round of the per-round flag chain (round 3's pnp_host.cpp flag_rounds: one launch sequence per pair) is a
k_match_gather dispatch followed by the PnP kernels (and copies) up to the next k_pnp_flags.  For every
kernel of a round: its duration and the gap since the previous kernel of the round ended (launch latency +
host work in between); medians over the rounds.  With the fused chain (k_pnp_chain, round 4) there are no
rounds: the kernel's duration per pair is the number, and the profiling build's [chain_prof] line splits it.

    python tools/chain_trace.py <run_kernel_trace.csv> [--skip 8] [--out chain.txt]
"""
import argparse
import csv
import re
import statistics as stt


def short(name):
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=8, help="rounds skipped at the start (warm-up)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    pnp = {"k_match_gather", "k_pnp_sample", "k_pnp_hyp", "k_pnp_replay", "k_pnp_refine", "k_pnp_flags"}
    rounds, cur = [], None
    for r in rows:
        if r[2] == "k_match_gather":
            cur = [r]
        elif cur is not None:
            if r[2] in pnp or "copy" in r[2].lower() or "fill" in r[2].lower():
                cur.append(r)
                if r[2] == "k_pnp_flags":
                    rounds.append(cur)
                    cur = None
            else:
                cur = None   # another kernel inside: not a flag round
    # a round's length runs to the next round's gather when the two are consecutive
    starts = [rd[0][0] for rd in rounds]
    rounds = rounds[a.skip:]
    lines = [f"{len(rounds)} rounds (after skipping {a.skip})"]
    if not rounds:
        print(lines[0])
        return
    per = {}
    order = []
    total = []
    starts = starts[a.skip:]
    for j, rd in enumerate(rounds):
        if j + 1 < len(rounds) and starts[j + 1] - rd[-1][1] < 200000:   # consecutive (< 200 us apart)
            total.append((starts[j + 1] - rd[0][0]) / 1e3)
        else:
            total.append((rd[-1][1] - rd[0][0]) / 1e3)
        prev_end = None
        seen = {}
        for s, e, n in rd:
            k = n if n not in seen else f"{n}#{seen[n] + 1}"
            seen[n] = seen.get(n, 0) + 1
            if k not in order:
                order.append(k)
            gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
            per.setdefault(k, []).append(((e - s) / 1e3, gap))
            prev_end = e
    lines.append(f"round (gather start to next gather start): median {stt.median(total):.1f} us, "
                 f"mean {stt.mean(total):.1f} us")
    lines.append(f"{'kernel':22s} {'rounds':>6s} {'dur med':>9s} {'dur mean':>9s} {'gap med':>9s} {'gap mean':>9s}")
    sdur = sgap = 0.0
    for k in order:
        v = per[k]
        d = [x[0] for x in v]
        g = [x[1] for x in v]
        sdur += stt.mean(d) * len(v) / len(rounds)
        sgap += stt.mean(g) * len(v) / len(rounds)
        lines.append(f"{k:22s} {len(v):6d} {stt.median(d):9.1f} {stt.mean(d):9.1f} {stt.median(g):9.1f} {stt.mean(g):9.1f}")
    lines.append(f"per round: kernels {sdur:.1f} us, gaps inside the round {sgap:.1f} us, "
                 f"rest (after the round's last kernel) {stt.mean(total) - sdur - sgap:.1f} us")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
