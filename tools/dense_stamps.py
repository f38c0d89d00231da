"""Per-phase timing of the persistent dense-stage launches (csrc/kernels/dense_stage.hip forward,
dense_stage_bwd.hip backward) from the kernels' own s_memrealtime stamps (IDC_DS_STAMPS=1: 8
stamps per work item, 100 MHz clock; persist.h NSTAMP).

    python tools/dense_stamps.py [--model densenet121] [--batch 256] [--steps 5] [--md out.md]

Forward stamp points:
  A (1x1):  0 ticket | 1 older slices ready (B_{l-2}) | 2 older-channel partial sums done |
            3 newest slice ready (B_{l-1}) | 4 newest operands staged + MFMA | 5 tile in LDS |
            6 stores + statistics issued | 7 published
  B (3x3):  0 ticket | 1 weights issued | 2 t ready (A_l) | 3 operands staged | 4 MFMA done |
            5 stores issued | 6 statistics issued | 7 published
Backward (dense_stage_bwd.hip): 0 ticket | 1 dependencies ready | 2 operands staged | 3 before publish.

For every phase it reports (us): the chain step (this phase's last publish - the previous phase's),
the hand-off (first tile's dependency cleared - previous phase's last publish), and the median of
every stamp-to-stamp interval over the phase's tiles.
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NSTAMP = 8


def _phase_rows(a, spans, ready_idx, end_idx):
    """spans: [(name, lo, hi)] ticket ranges in queue order."""
    import numpy as np
    rows = []
    prev_end = 0.0
    for name, lo, hi in spans:
        blk = a[lo:hi]
        kind = name.rstrip("0123456789")
        ri, ei = ready_idx.get(kind, 1), end_idx.get(kind, NSTAMP - 1)
        end = float(np.nanmax(blk[:, ei]))
        iv = []
        for k in range(1, ei + 1):
            d = blk[:, k] - blk[:, k - 1]  # NaN where a stamp point is not reached by this phase kind
            iv.append(float(np.nanmedian(d)) if np.isfinite(d).any() else float("nan"))
        rows.append({"phase": name, "end": end, "step": end - prev_end,
                     "handoff": float(np.nanmin(blk[:, ri])) - prev_end, "iv": iv})
        prev_end = end
    return rows


def _table(rows, title):
    import statistics as stt
    out = [title, ""]
    kinds = sorted({r["phase"].rstrip("0123456789") for r in rows})
    for k in kinds:
        rr = [r for r in rows if r["phase"].rstrip("0123456789") == k][1:] or \
             [r for r in rows if r["phase"].rstrip("0123456789") == k]
        n = len(rr[0]["iv"])
        def mean_iv(i):
            v = [r["iv"][i] for r in rr if r["iv"][i] == r["iv"][i]]
            return f"{stt.mean(v):.2f}" if v else "-"
        ivs = " / ".join(mean_iv(i) for i in range(n))
        out.append(f"- {k}: {len(rr)} phases, mean step {stt.mean(r['step'] for r in rr):.2f} us, hand-off "
                   f"{stt.mean(r['handoff'] for r in rr):.2f}, median stamp intervals {ivs}")
    out += ["", "| phase | end | step | handoff | stamp intervals (median over tiles) |", "|---|---:|---:|---:|---|"]
    for r in rows:
        out.append(f"| {r['phase']} | {r['end']:.1f} | {r['step']:.2f} | {r['handoff']:.2f} | "
                   + " ".join(f"{v:.2f}" if v == v else "-" for v in r["iv"]) + " |")
    out.append("")
    return out


def analyse_fwd(st, nlayers: int, M: int, ksplit: int = 1):
    import numpy as np
    nmt = (M + 31) // 32
    nA, nB = 2 * nmt * max(1, ksplit), nmt  # split K: helpers (no stamps past 2) + finalizers
    per = nA + nB
    a = st.reshape(nlayers * per, NSTAMP).astype(np.float64)
    a[a == 0] = np.nan  # stamp points a tile never reaches stay 0
    a = (a - np.nanmin(a[:, 0])) * 0.01  # 10 ns ticks -> us
    spans = []
    lookahead = os.environ.get("IDC_DS_LOOKAHEAD", "1") != "0" and nlayers > 1 and 256 >= 2 * nmt + 16
    if not lookahead:
        for l in range(nlayers):
            spans.append((f"A{l}", l * per, l * per + nA))
            spans.append((f"B{l}", l * per + nA, (l + 1) * per))
    else:  # dense_stage.hip lookahead order [A0][A1 B0][A2 B1]...[B_{L-1}]
        spans.append(("A0", 0, nA))
        for j in range(1, nlayers):
            b0 = nA + (j - 1) * per
            spans.append((f"A{j}", b0, b0 + nA))
            spans.append((f"B{j - 1}", b0 + nA, b0 + per))
        spans.append((f"B{nlayers - 1}", nA + (nlayers - 1) * per, nlayers * per))
    return _phase_rows(a, spans, {"A": 3, "B": 2}, {"A": 7, "B": 7})


def analyse_rows(st, nlayers: int, G: int, M: int):
    """Row-resident launch (dense_rows.hip): per layer, the median over workgroups of each
    interval [start, BN1 table, act1 staged, 1x1 done, barrier 1 passed, act2 staged, 3x3 done,
    barrier 2 passed] and the layer's span (first start to the next layer's last start)."""
    import numpy as np
    a = st.reshape(nlayers, G, NSTAMP).astype(np.float64)
    a[a == 0] = np.nan
    a = (a - np.nanmin(a[:, :, 0])) * 0.01
    names = ["bn1tab", "act1", "1x1", "bar1", "act2", "3x3", "bar2"]
    out = [f"## row-resident launch: {nlayers} layers, M = {M} rows, {G} workgroups, span "
           f"{np.nanmax(a[-1]) :.1f} us", "",
           "| layer | start | " + " | ".join(names) + " | next start |", "|---|---:|" + "---:|" * (len(names) + 1)]
    for l in range(nlayers):
        iv = [np.nanmedian(a[l, :, k + 1] - a[l, :, k]) for k in range(len(names))]
        nxt = np.nanmax(a[l + 1, :, 0]) if l + 1 < nlayers else np.nanmax(a[l])
        out.append(f"| {l} | {np.nanmin(a[l, :, 0]):.1f} | " + " | ".join(f"{v:.2f}" for v in iv) + f" | {nxt:.1f} |")
    out.append("")
    return out


def analyse_rows_bwd(st, nlayers: int, G: int, M: int):
    """Row-resident backward (dense_rows_bwd.hip), layers in processing order (L-1 .. 0): median
    over workgroups of [dy staged, 3x3 dgrad + bn2 sums, barrier A, dT, 1x1 dgrad + bn1 sums,
    barrier B, pending-affine update]."""
    import numpy as np
    a = st.reshape(nlayers, G, NSTAMP).astype(np.float64)
    a[a == 0] = np.nan
    a = (a - np.nanmin(a[:, :, 0])) * 0.01
    names = ["dy", "3x3", "barA", "dT", "1x1", "barB", "aff"]
    out = [f"## row-resident backward: {nlayers} layers, M = {M} rows, {G} workgroups, span "
           f"{np.nanmax(a) - np.nanmin(a):.1f} us", "",
           "| layer | start | " + " | ".join(names) + " |", "|---|---:|" + "---:|" * len(names)]
    for l in range(nlayers - 1, -1, -1):
        iv = [np.nanmedian(a[l, :, k + 1] - a[l, :, k]) for k in range(len(names))]
        out.append(f"| {l} | {np.nanmin(a[l, :, 0]):.1f} | " + " | ".join(f"{v:.2f}" for v in iv) + " |")
    out.append("")
    return out


def analyse_bwd(st, phases):
    import numpy as np
    n = phases[-1][0] + phases[-1][3]
    a = st.reshape(-1, NSTAMP)[:n].astype(np.float64)
    a[a == 0] = np.nan
    a = (a - np.nanmin(a[:, 0])) * 0.01
    names = {1: "P", 2: "QN", 3: "G", 4: "GIN", 5: "FIN1", 6: "FIN2"}
    spans = [(f"{names[k]}{l}", f, f + t) for f, k, l, t in phases]
    return _phase_rows(a, spans, {k: 1 for k in names.values()}, {k: 3 for k in names.values()})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="densenet121")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--md", default=None)
    args = ap.parse_args()
    os.environ["IDC_DS_STAMPS"] = "1"
    import torch

    from idc_models_amd.engine import Model, RMSprop
    from idc_models_amd.models import build_model

    dev = torch.device("cuda", 0)
    net = build_model(args.model, num_outputs=1, seed=1234)
    m = Model(net, device=dev)
    m.compile(RMSprop(1e-4), "binary_crossentropy", [], backend="fused")
    H, W, C = net.input_shape
    x = torch.randint(0, 256, (args.batch, H, W, C), dtype=torch.uint8, device=dev)
    y = torch.randint(0, 2, (args.batch,), device=dev)
    for _ in range(args.steps):
        m.impl.train_step(x, y)
    torch.cuda.synchronize()
    p = m.impl._prog(args.batch, True, torch.uint8)
    out = []
    for si, (stamps, nl, M, ks, G) in enumerate(getattr(p.b, "dense_stamps", [])):
        if G:
            out += analyse_rows(stamps.cpu().numpy(), nl, G, M)
            continue
        rows = analyse_fwd(stamps.cpu().numpy(), nl, M, ks)
        out += _table(rows, f"## forward launch {si}: {nl} layers, M = {M} rows, K split {ks}, span {rows[-1]['end']:.1f} us "
                            f"(err counter {int(p.b.dense_err[0])})")
    for si, rec in enumerate(getattr(p.b, "dense_bwd_stamps", [])):
        if rec[1] is None:  # row-resident backward: (stamps, None, M, workgroups, layers)
            out += analyse_rows_bwd(rec[0].cpu().numpy(), rec[4], rec[3], rec[2])
            continue
        stamps, phases, M = rec
        rows = analyse_bwd(stamps.cpu().numpy(), phases)
        out += _table(rows, f"## backward launch {si}: M = {M} rows, span {max(r['end'] for r in rows):.1f} us")
    text = "\n".join(out)
    print(text)
    if args.md:
        with open(args.md, "w") as f:
            f.write(f"# Dense-stage phase timing ({args.model}, batch {args.batch}, in-kernel s_memrealtime stamps, "
                    f"last of {args.steps} steps)\n\n" + text + "\n")


if __name__ == "__main__":
    main()
