"""How much of a run's GPU time has kernels from several queues in flight at once.

    python tools/queue_overlap.py gpurun_out/prof/<tag>_results.db [--last-frac 0.5]

Reads the rocprofv3 ``--kernel-trace`` database, keeps the last ``--last-frac`` of the trace
(skips plan-time autotuning and warm-up), and reports the wall span, the time with at least one
kernel running, the time with kernels from >= 2 queues running together, and per-queue totals.
Used for the concurrent federated clients (fed/fedavg.py ``concurrent_clients``).
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last-frac", type=float, default=0.5)
    a = ap.parse_args()
    rows = list(sqlite3.connect(a.db).execute("select start, end, queue_id from kernels order by start"))
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    cut = t1 - (t1 - t0) * a.last_frac
    rows = [r for r in rows if r[0] >= cut]
    ev = []
    per_q = collections.Counter()
    for s, e, q in rows:
        ev.append((s, 1, q))
        ev.append((e, -1, q))
        per_q[q] += e - s
    ev.sort()
    active = collections.Counter()
    busy = multi = 0
    prev = ev[0][0]
    for t, d, q in ev:
        n_q = sum(1 for v in active.values() if v > 0)
        if n_q >= 1:
            busy += t - prev
        if n_q >= 2:
            multi += t - prev
        active[q] += d
        prev = t
    span = ev[-1][0] - ev[0][0]
    print(f"span {span / 1e6:.1f} ms, {len(rows)} kernels on {len(per_q)} queues")
    print(f"  any kernel running {busy / 1e6:.1f} ms ({100 * busy / span:.1f}%)")
    print(f"  >= 2 queues running {multi / 1e6:.1f} ms ({100 * multi / span:.1f}%)")
    for q, v in per_q.most_common():
        print(f"  queue {q}: {v / 1e6:.1f} ms kernel time")


if __name__ == "__main__":
    main()
