"""Per-kernel-name PMC totals of a ``rocprofv3 --pmc ... --output-format csv`` run (any program):
mean kernel time, MFMA busy fraction, LDS bank-conflict ratio, wait fractions, L2 hit rate —
whichever of the counters the run collected.

    python tools/pmc_kernels.py DIR/PREFIX [--skip 2]
"""
import argparse
import collections
import csv
import re

CLK, SIMDS = 2.4e9, 256 * 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix")
    ap.add_argument("--skip", type=int, default=2, help="first dispatches of each kernel to drop (warm-up)")
    a = ap.parse_args()
    disp = {}
    with open(a.prefix + "_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            d = int(r["Dispatch_Id"])
            e = disp.setdefault(d, {"name": re.sub(r"\(.*$", "", r["Kernel_Name"]).replace("void ", ""),
                                    "t": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), "c": {}})
            e["c"][r["Counter_Name"]] = e["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    seen = collections.Counter()
    agg = collections.OrderedDict()
    for d in sorted(disp):
        e = disp[d]
        seen[e["name"]] += 1
        if seen[e["name"]] <= a.skip:
            continue
        s = agg.setdefault(e["name"], collections.Counter())
        s["n"] += 1
        s["t"] += e["t"]
        for k, v in e["c"].items():
            s[k] += v
    for name, s in agg.items():
        t = s["t"] / 1e9
        out = [f"{name[:70]:70s} n={s['n']:3d} {s['t'] / s['n'] / 1e3:8.1f} us"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in s:
            out.append(f"mfma {s['SQ_VALU_MFMA_BUSY_CYCLES'] / (t * CLK * SIMDS):.3f}")
        if s.get("SQ_LDS_IDX_ACTIVE"):
            out.append(f"ldsconf {s['SQ_LDS_BANK_CONFLICT'] / s['SQ_LDS_IDX_ACTIVE']:.3f}")
        if s.get("SQ_WAVE_CYCLES"):
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_LDS", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VMEM",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC"):
                if k in s:
                    out.append(f"{k[3:].lower()} {s[k] / s['SQ_WAVE_CYCLES']:.3f}")
        if s.get("TCC_HIT_sum") or s.get("TCC_MISS_sum"):
            h, m = s["TCC_HIT_sum"], s["TCC_MISS_sum"]
            out.append(f"L2hit {h / max(h + m, 1):.3f} ({(h + m) / s['n'] * 128 / 1e6:.0f} MB/dispatch @128B)")
        if "TCC_EA0_RDREQ_sum" in s:
            out.append(f"ea_rd {s['TCC_EA0_RDREQ_sum'] / s['n']:.3g}")
        print(" | ".join(out))


if __name__ == "__main__":
    main()
