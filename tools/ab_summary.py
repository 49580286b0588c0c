"""One line per bench run of a tools/se3_check.sh A/B directory (gpurun_out/<tag>/bench_<lib>_<run>.log):
headline, flag_chain_one, se3_chain_one, the config-3 chain and the lowtex leg.
usage: python tools/ab_summary.py gpurun_out/<tag> > profiles/.../<tag>.txt"""
import glob
import json
import os
import re
import sys


def main(d):
    runs = []
    for f in glob.glob(os.path.join(d, "bench_*.log")):
        m = re.match(r"^bench_(.*)_(\d+)\.log$", os.path.basename(f))
        if not m:
            continue
        lines = [l for l in open(f).read().splitlines() if l.startswith("{")]
        if not lines:
            continue
        runs.append((int(m.group(2)), os.path.getmtime(f), m.group(1), json.loads(lines[-1])))
    for run, _, lib, j in sorted(runs):
        def g(k, f="value"):
            return (j.get(k) or {}).get(f)
        print("%-12s run %d: headline %.0f frames/s %s ms | flag_chain_one %s | se3_chain_one %s (%s us/pair) | "
              "cfg3 %s (%s us/pair) | lowtex %s (k_fast %s ms)"
              % (lib, run, j["value"], j["ms_per_step"], g("flag_chain_one"), g("se3_chain_one"),
                 g("se3_chain_one", "us_per_pair"), g("se3_chain_one_cfg3"), g("se3_chain_one_cfg3", "us_per_pair"),
                 g("lowtex"), g("lowtex", "k_fast_ms")))


if __name__ == "__main__":
    main(sys.argv[1])
