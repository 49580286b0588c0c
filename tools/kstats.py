"""Print a rocprofv3 run_kernel_stats.csv compactly: python tools/kstats.py <csv> [steps]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 0
for r in rows:
    tot = float(r["TotalDurationNs"]) / 1e6
    print(r["Name"].split("(")[0].replace("rgbd::", "")[:26].ljust(27), r["Calls"].rjust(6), ("%.2f ms" % tot).rjust(11),
          ("%.1f us" % (float(r["AverageNs"]) / 1e3)).rjust(11), ("min %.1f max %.1f" % (float(r["MinNs"]) / 1e3,
                                                                               float(r["MaxNs"]) / 1e3)).rjust(22),
          ("%.2f ms/step" % (tot / steps)) if steps else "")
