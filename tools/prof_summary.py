"""Summarise a rocprofv3 ``--kernel-trace`` database (rocpd SQLite) per training step.

usage: python tools/prof_summary.py gpurun_out/prof/dn_results.db --steps 10 [--marker input_stage]
       [--md profiles/densenet121_bs256_kernels.md]

Only dispatches from the last ``--steps`` steps are counted (a step starts at the ``--marker``
kernel, the first kernel of every fused step), so plan-time autotuning and warm-up are excluded.
"""
import argparse
import collections
import re
import sqlite3


def short(name: str) -> str:
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*\)$", "", name)
    return name.replace("idc::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--marker", default="input_stage")
    ap.add_argument("--md", default=None)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    try:  # full 3-D launch geometry (grid sizes are in work-items)
        rows = [(n, s, e, (gx // max(wx, 1)) * (gy // max(wy, 1)) * (gz // max(wz, 1)), 1, vg, ag, lds)
                for n, s, e, gx, gy, gz, wx, wy, wz, vg, ag, lds in c.execute(
                    "select name, start, end, grid_x, grid_y, grid_z, workgroup_x, workgroup_y, workgroup_z, "
                    "vgpr_count, accum_vgpr_count, lds_size from kernels order by start")]
    except sqlite3.OperationalError:  # older schema: x only
        rows = list(c.execute("select name, start, end, grid_x, workgroup_x, vgpr_count, accum_vgpr_count, "
                              "lds_size from kernels order by start"))
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    if len(marks) < a.steps:
        raise SystemExit(f"only {len(marks)} '{a.marker}' dispatches found")
    lo = marks[-a.steps]
    sel = rows[lo:]
    t0, t1 = sel[0][1], max(r[2] for r in sel)
    agg = collections.OrderedDict()
    busy = 0
    for name, s, e, gx, wx, vg, ag, lds in sel:
        k = short(name)
        d = agg.setdefault(k, [0, 0.0, gx // max(wx, 1), vg, ag, lds])
        d[0] += 1
        d[1] += (e - s)
        busy += (e - s)
    wall_ms = (t1 - t0) / 1e6 / a.steps
    busy_ms = busy / 1e6 / a.steps
    lines = [f"# Kernel time per step ({a.steps} steps, rocprofv3 --kernel-trace)", "",
             f"- wall per step (first to last dispatch): **{wall_ms:.3f} ms**",
             f"- summed kernel time per step: **{busy_ms:.3f} ms** ({100 * busy_ms / wall_ms:.1f}% of wall)",
             f"- dispatches per step: {len(sel) / a.steps:.0f}", "",
             "| kernel | calls/step | us/step | % | avg us | grid WGs | vgpr/agpr | LDS B |",
             "|---|---:|---:|---:|---:|---:|---:|---:|"]
    for k, (n, t, wg, vg, ag, lds) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        us = t / 1e3 / a.steps
        lines.append(f"| `{k}` | {n / a.steps:.0f} | {us:.1f} | {100 * t / busy:.1f} | {t / 1e3 / n:.2f} | "
                     f"{wg} | {vg}/{ag} | {lds} |")
    out = "\n".join(lines) + "\n"
    print(out)
    if a.md:
        with open(a.md, "w") as f:
            f.write(out)


if __name__ == "__main__":
    main()
