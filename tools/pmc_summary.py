"""Summarise rocprofv3 counter CSVs per kernel (mean per dispatch): python tools/pmc_summary.py <dir>..."""
import csv
import sys
from collections import defaultdict


BY_GRID = False   # --by-grid: key dispatches by kernel name @ grid size (e.g. k_fast's split launches)


def load(path):
    acc = defaultdict(lambda: defaultdict(list))
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"].split("(")[0].replace("rgbd::", "")
        if BY_GRID:
            name += "@" + row["Grid_Size"]
        acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
        if row["Counter_Name"] == "SQ_WAVES":   # dispatch duration (ns) under the counter pass, once per dispatch
            acc[name]["dur_ns"].append(float(row["End_Timestamp"]) - float(row["Start_Timestamp"]))
    return acc


def main():
    global BY_GRID
    args = sys.argv[1:]
    if "--by-grid" in args:
        BY_GRID = True
        args.remove("--by-grid")
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
    w = 28 if BY_GRID else 16
    print("kernel".ljust(w) + "".join(c[-14:].rjust(15) for c in cols))
    for k in sorted(tot):
        if k.startswith("__amd"):
            continue
        print(k[:w].ljust(w) + "".join(("%.4g" % tot[k].get(c, float("nan"))).rjust(15) for c in cols))


if __name__ == "__main__":
    main()
