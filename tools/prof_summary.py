"""Summarise rocprofv3 SQLite outputs (kernel trace + PMC passes) of tools/profile.sh into text/CSV.

usage: python tools/prof_summary.py <profile dir> [kernel substring]
"""
from __future__ import annotations

import sqlite3
import sys
from pathlib import Path


def rows(db: Path, sql: str):
    c = sqlite3.connect(str(db))
    try:
        return c.execute(sql).fetchall()
    finally:
        c.close()


def main():
    d = Path(sys.argv[1])
    ksub = sys.argv[2] if len(sys.argv) > 2 else ""
    out = []
    kt = d / "kt" / "run_results.db"
    if kt.exists():
        out.append("# kernel trace (rocprofv3 --kernel-trace --stats): name, calls, total_us, avg_us, pct (rocprofv3 stats table: microseconds)")
        for name, calls, tot, avg, pct in rows(kt, "select name,total_calls,total_duration,average,percentage "
                                                    "from top_kernels order by total_duration desc"):
            out.append(f"{name[:140]!s},{calls},{tot:.0f},{avg:.0f},{pct:.2f}")
        info = rows(kt, "select name,vgpr_count,accum_vgpr_count,sgpr_count,scratch_size,grid_x,workgroup_x "
                        "from kernels group by name")
        out.append("# resources: name, vgpr, agpr, sgpr, scratch, grid, wg")
        for r in info:
            if ksub in r[0]:
                out.append(",".join(str(x) for x in (r[0][:100],) + r[1:]))
        # per-dispatch durations of the kernel, in launch order: the bench's warm-up launches come
        # first, so the mean of the last `--steps` dispatches is the figure comparable with its
        # HIP-event kernel_ms
        cols = [c[1] for c in rows(kt, "pragma table_info(kernels)")]
        if ksub and "start" in cols and "end" in cols:
            ds = [(e - s) * 1e-3 for nm, s, e in rows(kt, "select name, start, end from kernels order by start")
                  if ksub in nm]
            if ds:
                out.append("# dispatches of the kernel (us, launch order): " + " ".join(f"{x:.1f}" for x in ds))
                tail = ds[-5:]
                out.append(f"# mean of the last {len(tail)} dispatches (us): {sum(tail) / len(tail):.1f}")
        elif ksub:
            out.append("# kernels table columns: " + " ".join(cols))
    for p in ("sq", "fetch", "write"):
        db = d / p / "run_results.db"
        if not db.exists():
            continue
        out.append(f"# PMC pass {p}: kernel, counter, mean value per dispatch, dispatches")
        for name, cn, val, cnt in rows(db, "select k.name, e.counter_name, avg(e.v), count(*) from "
                                           "(select dispatch_id, counter_name, sum(counter_value) v from pmc_events "
                                           "group by dispatch_id, counter_name) e join kernels k on "
                                           "k.dispatch_id = e.dispatch_id group by k.name, e.counter_name"):
            if ksub in name:
                out.append(f"{name[:100]},{cn},{val:.6g},{cnt}")
    print("\n".join(out))


if __name__ == "__main__":
    main()
