"""Per-kernel time summary of a rocprofv3 rocpd database (the default output of
rocprofv3 --kernel-trace on ROCm 7.2): name, calls, total / mean / min / max us,
share of the kernel time.  Usage: python tools/rocpd_summary.py <db> [--csv out.csv]"""
import argparse
import glob
import sqlite3


def summary(db: str):
    con = sqlite3.connect(db)
    tabs = [r[0] for r in con.execute("select name from sqlite_master where type='table'")]
    kd = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    ks = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    cols = [r[1] for r in con.execute(f"pragma table_info({ks})")]
    name_col = "kernel_name" if "kernel_name" in cols else ("display_name" if "display_name" in cols else "name")
    rows = con.execute(f"select s.{name_col}, d.end - d.start from {kd} d join {ks} s on d.kernel_id = s.id").fetchall()
    agg = {}
    for name, dt in rows:
        a = agg.setdefault(name, [])
        a.append(dt / 1000.0)
    total = sum(sum(v) for v in agg.values()) or 1.0
    out = []
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        out.append((name, len(v), sum(v), sum(v) / len(v), min(v), max(v), 100.0 * sum(v) / total))
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--csv")
    p.add_argument("--top", type=int, default=25)
    a = p.parse_args()
    dbs = glob.glob(a.db) if "*" in a.db else [a.db]
    rows = summary(dbs[0])
    lines = ['"Name","Calls","TotalUs","MeanUs","MinUs","MaxUs","Percentage"']
    for r in rows:
        lines.append('"%s",%d,%.1f,%.2f,%.2f,%.2f,%.2f' % r)
    if a.csv:
        open(a.csv, "w").write("\n".join(lines) + "\n")
    for r in rows[: a.top]:
        print("%-100s %5d %10.1f %9.2f %6.2f%%" % (r[0][:100], r[1], r[2], r[3], r[6]))


if __name__ == "__main__":
    main()
