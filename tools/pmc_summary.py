"""Per-kernel PMC summary of one or more ``rocprofv3 --pmc ... --output-format csv`` passes.

usage: python tools/pmc_summary.py DIR/PREFIX [DIR/PREFIX2 ...] --steps 3 [--marker input_stage] [--md out.md]

Counters expected (over all passes): SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_WAIT_ANY.  Only the last
``--steps`` training steps of each pass are used (a step starts at the ``--marker`` kernel), so
autotuning and warm-up are excluded; the passes' selected dispatch sequences must match kernel for
kernel (same program, same tune cache) and are merged by position.  Collect at most 4 SQ counters
per pass and no tracing domain beside --pmc: a round-3 pass of all 8 SQ counters together with
--kernel-trace segfaulted inside rocprofv3 at the first dispatch (tools/pmc_session.sh).

Derived (per kernel class, summed over its dispatches):
  MFMA util   = SQ_VALU_MFMA_BUSY_CYCLES / (kernel time x 2.4 GHz x 1024 SIMDs)
  LDS confl.  = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE   (extra cycles per LDS-array cycle)
  wait frac.  = SQ_WAIT_ANY / SQ_WAVE_CYCLES,  LDS-issue stall = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES
Kernel times come from the PMC run (serialised dispatches), so they are upper bounds.
"""
import argparse
import collections
import csv
import re

CLK = 2.4e9
SIMDS = 256 * 4


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*\)$", "", name)
    return name.replace("idc::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix", nargs="+")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--marker", default="input_stage")
    ap.add_argument("--md", default=None)
    ap.add_argument("--bytes", action="store_true",
                    help="traffic table from FETCH_SIZE / WRITE_SIZE passes (KB per dispatch)")
    a = ap.parse_args()
    merged = None
    for prefix in a.prefix:
        disp = {}
        order = []
        with open(prefix + "_counter_collection.csv") as f:
            for r in csv.DictReader(f):
                d = int(r["Dispatch_Id"])
                if d not in disp:
                    disp[d] = {"name": r["Kernel_Name"], "t": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])}
                    order.append(d)
                disp[d][r["Counter_Name"]] = disp[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        order.sort()
        marks = [d for d in order if a.marker in disp[d]["name"]]
        first = marks[-a.steps]
        sel = [disp[d] for d in order if d >= first]
        if merged is None:
            merged = sel
            continue
        if [e["name"] for e in sel] != [e["name"] for e in merged]:
            raise SystemExit(f"{prefix}: dispatch sequence differs from the first pass")
        for e0, e in zip(merged, sel):
            e0["t"] = min(e0["t"], e["t"])
            for k, v in e.items():
                if k not in ("name", "t"):
                    e0[k] = v
    sel = merged
    agg = collections.OrderedDict()
    for e in sel:
        k = short(e["name"])
        s = agg.setdefault(k, collections.Counter())
        s["n"] += 1
        for key, v in e.items():
            if key != "name":
                s[key] += v
    if a.bytes:
        return bytes_table(agg, a)
    rows = []
    tot_t = sum(s["t"] for s in agg.values())
    tot_mfma = sum(s["SQ_VALU_MFMA_BUSY_CYCLES"] for s in agg.values())
    for k, s in agg.items():
        t = s["t"] * 1e-9
        util = s["SQ_VALU_MFMA_BUSY_CYCLES"] / (t * CLK * SIMDS) if t else 0.0
        lds = s["SQ_LDS_BANK_CONFLICT"] / s["SQ_LDS_IDX_ACTIVE"] if s["SQ_LDS_IDX_ACTIVE"] else 0.0
        wait = s["SQ_WAIT_ANY"] / s["SQ_WAVE_CYCLES"] if s["SQ_WAVE_CYCLES"] else 0.0
        ldsw = s["SQ_WAIT_INST_LDS"] / s["SQ_WAVE_CYCLES"] if s["SQ_WAVE_CYCLES"] else 0.0
        rows.append((s["t"], k, s["n"] / a.steps, s["t"] / 1e3 / a.steps, util, lds, wait, ldsw))
    for key in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_LDS_IDX_ACTIVE", "SQ_WAVE_CYCLES"):
        if not any(s[key] for s in agg.values()):
            print(f"warning: no {key} in any pass")
    rows.sort(reverse=True)
    lines = [f"# PMC summary per kernel ({a.steps} steps, rocprofv3 --pmc, serialised dispatches)", "",
             f"- kernel time per step under PMC: {tot_t / 1e6 / a.steps:.3f} ms",
             f"- whole-step MFMA utilisation: {tot_mfma / (tot_t * 1e-9 * CLK * SIMDS):.1%}", "",
             "| kernel | calls/step | us/step | MFMA util | LDS bank-conflict cycles / LDS cycles | wave wait frac | LDS issue stall |",
             "|---|---:|---:|---:|---:|---:|---:|"]
    for _, k, n, us, util, lds, wait, ldsw in rows[:40]:
        lines.append(f"| `{k}` | {n:.0f} | {us:.1f} | {util:.1%} | {lds:.3f} | {wait:.2f} | {ldsw:.3f} |")
    out = "\n".join(lines) + "\n"
    print(out)
    if a.md:
        with open(a.md, "w") as f:
            f.write(out)


def bytes_table(agg, a):
    """Per kernel class: MB read / written per step (FETCH_SIZE / WRITE_SIZE are in KB) and the
    implied HBM-side bandwidth over the serialised kernel time."""
    rows = []
    tot_t = sum(s["t"] for s in agg.values())
    tot_r = sum(s["FETCH_SIZE"] for s in agg.values()) / 1e3 / a.steps
    tot_w = sum(s["WRITE_SIZE"] for s in agg.values()) / 1e3 / a.steps
    for k, s in agg.items():
        us = s["t"] / 1e3 / a.steps
        rd, wr = s["FETCH_SIZE"] / 1e3 / a.steps, s["WRITE_SIZE"] / 1e3 / a.steps
        bw = (rd + wr) / 1e3 / (us * 1e-6) if us else 0.0  # GB/s
        rows.append((s["t"], k, s["n"] / a.steps, us, rd, wr, bw))
    rows.sort(reverse=True)
    lines = [f"# PMC traffic per kernel ({a.steps} steps, rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, "
             "serialised dispatches)", "",
             f"- kernel time per step under PMC: {tot_t / 1e6 / a.steps:.3f} ms",
             f"- read {tot_r:.1f} MB + written {tot_w:.1f} MB per step", "",
             "| kernel | calls/step | us/step | MB read/step | MB written/step | GB/s |",
             "|---|---:|---:|---:|---:|---:|"]
    for _, k, n, us, rd, wr, bw in rows[:40]:
        lines.append(f"| `{k}` | {n:.0f} | {us:.1f} | {rd:.1f} | {wr:.1f} | {bw:.0f} |")
    out = "\n".join(lines) + "\n"
    print(out)
    if a.md:
        with open(a.md, "w") as f:
            f.write(out)


if __name__ == "__main__":
    main()
