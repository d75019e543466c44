#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 SQLite (rocpd) database, optionally restricted to the last
``--window-ms`` of GPU time (the steady-state timed iterations of a benchmark).

    python tools/rocpd_summary.py gpurun_out/prof/run_results.db --window-ms 93 --per 10
"""
from __future__ import annotations

import argparse
import sqlite3
import sys


def last_gap_start(db, gap_ms: float) -> int:
    """Start time of the first dispatch after the LAST idle gap longer than ``gap_ms`` (a benchmark
    sleeps before its steady-state loop, so everything after the gap is steady state)."""
    rows = db.execute("select start, end from kernels order by start").fetchall()
    cut, prev_end = rows[0][0], None
    for st, en in rows:
        if prev_end is not None and st - prev_end > gap_ms * 1e6:
            cut = st
        prev_end = en if prev_end is None else max(prev_end, en)
    return cut


def summarize(db_path: str, window_ms: float = 0.0, per: int = 1, top: int = 30,
              after_gap_ms: float = 0.0) -> str:
    db = sqlite3.connect(db_path)
    emax = db.execute("select max(end) from kernels").fetchone()[0]
    where = f"where start > {emax - window_ms * 1e6}" if window_ms > 0 else ""
    if after_gap_ms > 0:
        where = f"where start >= {last_gap_start(db, after_gap_ms)}"
    tot_ns, count, span = db.execute(
        f"select sum(end-start), count(*), max(end)-min(start) from kernels {where}").fetchone()
    rows = db.execute(
        f"select name, count(*), sum(end-start), avg(end-start) from kernels {where} "
        f"group by name order by 3 desc limit {top}").fetchall()
    out = [f"# {db_path}: {count} dispatches, busy {tot_ns / 1e6:.3f} ms over {span / 1e6:.3f} ms"
           + (f" (last {window_ms} ms)" if window_ms else "")
           + (f"; per-iteration columns divide by {per}" if per > 1 else ""),
           f"{'ms/iter':>9} {'share':>6} {'calls/iter':>10} {'avg_us':>8}  kernel"]
    for name, n, s, a in rows:
        out.append(f"{s / 1e6 / per:9.3f} {100 * s / tot_ns:5.1f}% {n / per:10.1f} {a / 1e3:8.1f}  "
                   f"{name[:120]}")
    return "\n".join(out)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("db")
    ap.add_argument("--window-ms", type=float, default=0.0)
    ap.add_argument("--per", type=int, default=1, help="iterations inside the window")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--after-gap-ms", type=float, default=0.0,
                    help="only dispatches after the last idle gap longer than this (steady state)")
    a = ap.parse_args(argv)
    print(summarize(a.db, a.window_ms, a.per, a.top, a.after_gap_ms))
    return 0


if __name__ == "__main__":
    sys.exit(main())
