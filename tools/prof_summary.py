#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace run (rocpd SQLite .db or the CSV
kernel_trace file): per-kernel stats (calls, total/avg/min/max ms, share) and
the kernel timeline of one collect() step (the `--step`-th launch of the
--marker kernel up to the next one, or bursts split at --gap ms of idle device).  Used to produce the profiles/*.txt summaries."""
import argparse
import csv
import sqlite3
import statistics
import sys


def load(path):
    rows = []
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, s, e, sid, q, gx in c.execute("select name,start,end,stream_id,queue_id,grid_x from kernels"):
            rows.append((name, int(s), int(e), sid, q, gx))
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             r.get("Stream_Id", ""), r.get("Queue_Id", ""), int(r.get("Grid_Size_X", r.get("Grid_Size", 0)))))
    rows.sort(key=lambda r: r[1])
    return rows


def short(n):
    return n.split("(")[0].replace("void ", "").replace("fsdkr::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=2)
    ap.add_argument("--gap", type=float, default=0.0, help="split steps at device idle gaps of this many ms")
    ap.add_argument("--marker", default="ped_hash", help="kernel launched once per step")
    a = ap.parse_args()
    rows = load(a.trace)
    by = {}
    for r in rows:
        by.setdefault(short(r[0]), []).append((r[2] - r[1]) / 1e6)
    tot = sum(sum(v) for v in by.values())
    print(f"{'kernel':44s} {'calls':>6s} {'total_ms':>10s} {'avg_ms':>9s} {'min_ms':>9s} {'max_ms':>9s} {'pct':>6s}")
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:44s} {len(v):6d} {sum(v):10.3f} {statistics.mean(v):9.3f} {min(v):9.3f} {max(v):9.3f} "
              f"{100 * sum(v) / tot:6.2f}")
    if a.gap:
        # steps = bursts of kernels separated by >= gap ms of device idle time
        idx, end = [], None
        for i, r in enumerate(rows):
            if "copyBuffer" in r[0]:
                continue
            if end is None or r[1] - end > a.gap * 1e6:
                idx.append(i)
            end = r[2] if end is None else max(end, r[2])
    else:
        idx = [i for i, r in enumerate(rows) if a.marker in r[0]]
    step = a.step if a.step >= 0 else len(idx) + a.step
    if 0 <= step < len(idx):
        i0 = idx[step]
        i1 = idx[step + 1] if step + 1 < len(idx) else len(rows)
        t0 = rows[i0][1]
        print(f"\ntimeline of collect step {a.step} (ms from the step's first kernel; stream/queue ids from the trace)")
        for r in rows[i0:i1]:
            if "copyBuffer" in r[0]:
                continue
            print(f"  {short(r[0]):40s} stream={r[3]!s:3s} queue={r[4]!s:3s} grid={r[5]:8d} "
                  f"start={(r[1] - t0) / 1e6:8.2f} end={(r[2] - t0) / 1e6:8.2f} dur={(r[2] - r[1]) / 1e6:8.2f}")
        last = max(r[2] for r in rows[i0:i1] if "copyBuffer" not in r[0])
        print(f"  step span (first kernel start -> last kernel end): {(last - t0) / 1e6:.2f} ms")


if __name__ == "__main__":
    sys.exit(main())
