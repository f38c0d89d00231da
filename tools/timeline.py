"""Critical-path view of one training step from a rocprofv3 rocpd database.

    python tools/timeline.py gpurun_out/prof/<tag>_results.db [--marker input_stage] [--top 15]

Splits the step into forward / backward / optimizer on the main queue (the queue that runs the
input-staging kernel), reports busy time and inter-kernel gaps per phase, the side-lane (weight
gradient) queue's busy time, and the top kernels per phase by time.
"""
import argparse
import collections
import re
import sqlite3


def short(n: str) -> str:
    return re.sub(r"\(.*\)$", "", n.replace("void ", "").replace("idc::", ""))[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="input_stage")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--gaps", type=int, default=0, help="list the N largest backward main-lane gaps "
                    "with the kernels around them and what the side lane ran meanwhile")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end, queue_id from kernels order by start"))
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    if len(marks) < 3:
        raise SystemExit("need >= 3 steps")
    # the step with the median wall time among the complete steps after warm-up (one step can
    # carry a host hiccup, e.g. a Python GC pause before its optimizer launch)
    cand = list(range(max(1, len(marks) - 8), len(marks) - 1))
    walls = sorted((rows[marks[j + 1]][1] - rows[marks[j]][1], j) for j in cand)
    j = walls[len(walls) // 2][1]
    lo, hi = marks[j], marks[j + 1]
    step = rows[lo:hi]
    q0 = step[0][3]
    main_q = [r for r in step if r[3] == q0]
    side_q = [r for r in step if r[3] != q0]
    wall = (rows[hi][1] - step[0][1]) / 1e3
    names = [short(r[0]) for r in main_q]
    hf = max(i for i, n in enumerate(names) if n.startswith("head_fwd"))
    opt = [i for i, n in enumerate(names) if n.startswith(("rmsprop", "cast_weights"))]
    op0 = min(opt) if opt else len(main_q)
    phases = {"forward": main_q[:hf + 1], "backward": main_q[hf + 1:op0], "optimizer": main_q[op0:]}
    print(f"step wall {wall:.1f} us, {len(step)} kernels ({len(main_q)} main, {len(side_q)} side)")
    for name, rs in phases.items():
        if not rs:
            continue
        busy = sum(r[2] - r[1] for r in rs) / 1e3
        span = (rs[-1][2] - rs[0][1]) / 1e3
        print(f"  {name:9s} span {span:8.1f} us  busy {busy:8.1f}  gaps {span - busy:7.1f}  kernels {len(rs)}")
    if side_q:
        busy = sum(r[2] - r[1] for r in side_q) / 1e3
        print(f"  side lane busy {busy:8.1f} us over {(side_q[-1][2] - side_q[0][1]) / 1e3:.1f} us")
    if a.gaps:
        bw = phases["backward"]
        gl = sorted(((bw[i + 1][1] - bw[i][2]) / 1e3, i) for i in range(len(bw) - 1))[::-1][:a.gaps]
        print(f"-- largest backward gaps (of {len(bw) - 1})")
        for g, i in gl:
            t0, t1 = bw[i][2], bw[i + 1][1]
            side = [short(r[0]) for r in side_q if r[1] < t1 and r[2] > t0]
            print(f"   {g:7.2f} us after {short(bw[i][0])[:44]} -> {short(bw[i + 1][0])[:44]}"
                  f"  side: {', '.join(side)[:90] or '-'}")
    for name, rs in list(phases.items()) + [("side", side_q)]:
        agg, cnt = collections.Counter(), collections.Counter()
        for r in rs:
            k = short(r[0])
            agg[k] += (r[2] - r[1]) / 1e3
            cnt[k] += 1
        print(f"-- {name}")
        for k, v in agg.most_common(a.top):
            print(f"   {v:8.1f} us {cnt[k]:4d}x {v / cnt[k]:6.2f}  {k}")


if __name__ == "__main__":
    main()
