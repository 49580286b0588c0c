"""Per-step kernel timeline from a rocprofv3 kernel trace (run_kernel_trace.csv).

Takes the k_pyramid dispatches as step boundaries and prints, for a few steps in the middle of the run,
every kernel that ran inside [pyramid_k start, pyramid_{k+1} start): start / end relative to the step start,
duration, and its queue, plus each step's busy union per queue and the gaps on the launch chain.

    python tools/timeline.py <run_kernel_trace.csv> [--steps 3] [--out timeline.txt]
"""
import argparse
import csv
import re


def short(name):
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), q))
    rows.sort()
    pyr = [r for r in rows if r[2] == "k_pyramid"]
    lines = []
    if len(pyr) < 3:
        lines.append(f"only {len(pyr)} k_pyramid dispatches")
    else:
        mid = len(pyr) // 2
        ks = range(max(0, mid - a.steps // 2), min(len(pyr) - 1, mid - a.steps // 2 + a.steps))
        for k in ks:
            t0, t1 = pyr[k][0], pyr[k + 1][0]
            lines.append(f"step {k}: {(t1 - t0) / 1e3:.1f} us (pyramid start to next pyramid start)")
            busy = {}
            for s, e, n, q in rows:
                if e <= t0 or s >= t1:
                    continue
                lines.append(f"  {n:18s} q{q:>3s} {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:9.1f}")
                busy.setdefault(q, []).append((max(s, t0), min(e, t1)))
            for q, iv in sorted(busy.items()):
                iv.sort()
                tot, cs, ce = 0, None, None
                for s, e in iv:
                    if cs is None or s > ce:
                        if cs is not None:
                            tot += ce - cs
                        cs, ce = s, e
                    else:
                        ce = max(ce, e)
                tot += ce - cs
                lines.append(f"  queue {q}: busy {tot / 1e3:.1f} us of {(t1 - t0) / 1e3:.1f}")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
