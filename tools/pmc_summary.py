"""Summarise rocprofv3 counter CSVs per kernel (mean per dispatch): python tools/pmc_summary.py <dir>..."""
import csv
import sys
from collections import defaultdict


def load(path):
    acc = defaultdict(lambda: defaultdict(list))
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"].split("(")[0].replace("rgbd::", "")
        acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


def main():
    args = sys.argv[1:]
    out_json = None
    if "--json" in args:
        i = args.index("--json")
        out_json = args[i + 1]
        args = args[:i] + args[i + 2:]
    tot = defaultdict(dict)
    for d in args:
        for k, cs in load(d + "/run_counter_collection.csv").items():
            for c, v in cs.items():
                tot[k][c] = sum(v) / len(v)
    if out_json:
        import json
        json.dump({k: v for k, v in tot.items() if not k.startswith("__amd")}, open(out_json, "w"), indent=1,
                  sort_keys=True)
    cols = sorted({c for v in tot.values() for c in v})
    print("kernel".ljust(16) + "".join(c[-14:].rjust(15) for c in cols))
    for k in sorted(tot):
        if k.startswith("__amd"):
            continue
        print(k[:16].ljust(16) + "".join(("%.4g" % tot[k].get(c, float("nan"))).rjust(15) for c in cols))


if __name__ == "__main__":
    main()
