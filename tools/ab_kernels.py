"""Per-kernel average durations of tools/ab_run.sh's kernel-trace runs (gpurun_out/<tag>p/<lib>/run_kernel_stats.csv).
usage: python tools/ab_kernels.py gpurun_out/<tag>p [name substrings...]"""
import csv
import glob
import os
import sys


def main(d, keys):
    for f in sorted(glob.glob(os.path.join(d, "*", "run_kernel_stats.csv"))):
        lib = os.path.basename(os.path.dirname(f))
        for x in csv.DictReader(open(f)):
            n = x["Name"].split("(")[0].replace("rgbd::", "")
            if not keys or any(k in n for k in keys):
                print("%-12s %-34s calls %5s avg %9.1f us" % (lib, n, x["Calls"], float(x["AverageNs"]) / 1e3))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:] or ["pyr", "k_fast", "describe"])
