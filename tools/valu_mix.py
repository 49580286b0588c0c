"""Static VALU instruction mix of the gfx950 kernels, priced at the measured issue costs.

Disassembles the device code objects of rgbd-slam_amd/build/*.o (llvm-objdump), counts every VALU
mnemonic per kernel, and prices each at its measured cost in cycles per wave64 instruction per SIMD
(profiles/r02_ubench/valu_rate.txt, tools/ubench/valu_rate.hip: 8 independent chains per wave, every
SIMD loaded).  Mnemonics the microbenchmark did not cover take the cost of their encoding class, which
is what the table shows: VOP1/VOP2/VOPC (e32, DPP, SDWA) ~2.3 cycles, VOP3 forms (e64 and the 3-operand
ops), packed, dot and 16-bit 3-input ~4.3 / 8.3 cycles, 64-bit integer / f64 ~8.6 (half rate assumed).

The weighted mean is written to profiles/valu_mix.json; bench.py multiplies SQ_INSTS_VALU by it to price
roofline.valu.frac_priced (the static mix stands in for the dynamic one: the hot loops are unrolled, so
the text is dominated by the loop bodies).  Also prints the k_fast row-body breakdown by phase.

    python tools/valu_mix.py [--kernels k_fast k_pyramid ...]
"""
import argparse
import glob
import json
import os
import re
import subprocess
import tempfile
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def rate_table(path):
    t = {}
    for line in open(path):
        m = re.match(r"(v_\w+)\s+[\d.]+ ms\s+([\d.]+) cyc", line)
        if m:
            t[m.group(1)] = float(m.group(2))
    return t


def base_name(mn):
    return re.sub(r"_(e32|e64|sdwa|dpp)$", "", mn)


def cost(mn, table):
    b = base_name(mn)
    if b in table:
        # a VOP2 op in its VOP3 (e64) encoding is a VOP3 form (measured ~4.3)
        if mn.endswith("_e64") and table[b] < 3.0:
            return 4.3
        return table[b]
    if re.search(r"_(f64|u64|i64|b64)$", b) or "_u64_" in b or "_i64_" in b or b.startswith("v_lshl_add_u64"):
        return 8.6
    if b.startswith("v_pk_") or b.startswith("v_dot") or "3_" in b or b.endswith("3"):
        return 4.3
    if mn.endswith("_e64") or b.startswith(("v_mad", "v_mbcnt", "v_bcnt", "v_bfe", "v_perm", "v_align", "v_lshl_or",
                                            "v_add3", "v_or3", "v_and_or", "v_lshl_add", "v_add_lshl", "v_med3",
                                            "v_min3", "v_max3", "v_sad", "v_cvt_pk", "v_mul_hi", "v_mul_lo")):
        return 4.3
    return 2.3


def disassemble(objs):
    """kernel name -> list of mnemonics (VALU only)."""
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for o in objs:
            dst = os.path.join(td, os.path.basename(o))
            subprocess.run(["cp", o, dst], check=True)
            subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", dst], check=True, capture_output=True, cwd=td)
            for co in glob.glob(dst + ".*gfx950*"):
                dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True,
                                     capture_output=True, text=True).stdout
                cur = None
                for line in dis.splitlines():
                    m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
                    if m:
                        dm = re.search(r"(k_\w+?)E", m.group(1))
                        cur = dm.group(1) if dm else m.group(1)
                        out.setdefault(cur, [])
                        continue
                    m = re.match(r"^\s+(v_\w+)", line)
                    if m and cur and not m.group(1).startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
                        out[cur].append(m.group(1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", nargs="*", default=None)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "valu_mix.json"))
    args = ap.parse_args()
    table = rate_table(os.path.join(ROOT, "profiles", "r02_ubench", "valu_rate.txt"))
    objs = sorted(glob.glob(os.path.join(ROOT, "rgbd-slam_amd", "build", "*.hip.o")))
    kern = disassemble(objs)
    res = {}
    for k, mns in sorted(kern.items()):
        if not k.startswith("k_") or (args.kernels and k not in args.kernels) or not mns:
            continue
        c = Counter(mns)
        tot = sum(c.values())
        cyc = sum(n * cost(mn, table) for mn, n in c.items())
        cls = Counter()
        for mn, n in c.items():
            cls["%.1f" % cost(mn, table)] += n
        res[k] = {"static_valu": tot, "cycles_per_inst": round(cyc / tot, 3),
                  "by_cost_class": dict(sorted(cls.items())),
                  "top": [[mn, n] for mn, n in c.most_common(12)]}
        print(f"{k:20s} {tot:6d} VALU  {cyc / tot:5.2f} cyc/inst  classes {dict(sorted(cls.items()))}")
    json.dump(res, open(args.out, "w"), indent=1)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
