"""Summarise a rocprofv3 kernel-trace database (rocpd sqlite) into a stats table."""
import json
import sqlite3
import sys


def summarise(db_path):
    c = sqlite3.connect(db_path)
    rows = c.execute("select name, count(*), avg(end-start), min(end-start), max(end-start), "
                     "sum(end-start), max(lds_size), max(vgpr_count), max(grid_x), max(grid_y), "
                     "max(grid_z) from kernels group by name order by sum(end-start) desc").fetchall()
    total = sum(r[5] for r in rows) or 1
    out = []
    for r in rows:
        out.append({"kernel": r[0], "calls": r[1], "avg_us": r[2] / 1e3, "min_us": r[3] / 1e3,
                    "max_us": r[4] / 1e3, "total_us": r[5] / 1e3, "pct": 100.0 * r[5] / total,
                    "lds": r[6], "vgpr": r[7], "grid": [r[8], r[9], r[10]]})
    return out


if __name__ == "__main__":
    res = summarise(sys.argv[1])
    print(f"{'calls':>5} {'avg_us':>9} {'min_us':>9} {'max_us':>9} {'total_us':>10} {'pct':>6}  kernel")
    for r in res:
        print(f"{r['calls']:5d} {r['avg_us']:9.2f} {r['min_us']:9.2f} {r['max_us']:9.2f} "
              f"{r['total_us']:10.1f} {r['pct']:6.1f}  {r['kernel'][:110]}")
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(res, f, indent=1)
