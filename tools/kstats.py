"""Per-kernel duration summary of a rocprofv3 run (rocpd SQLite output or --stats CSV)."""
import csv
import sqlite3
import sys


def from_db(path):
    db = sqlite3.connect(path)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else cols[0])
    rows = db.execute(f"select {name}, count(*), avg(end-start), min(end-start), max(end-start) "
                      f"from kernels group by {name} order by sum(end-start) desc").fetchall()
    return rows


def from_csv(path):
    return [(r["Name"], int(r["Calls"]), float(r["AverageNs"]), float(r["MinNs"]), float(r["MaxNs"]))
            for r in csv.DictReader(open(path))]


def main():
    path = sys.argv[1]
    rows = from_db(path) if path.endswith(".db") else from_csv(path)
    print(f"{'kernel':60s} {'calls':>6s} {'avg_us':>10s} {'min_us':>10s} {'max_us':>10s}")
    for n, c, a, lo, hi in rows:
        print(f"{str(n)[:60]:60s} {c:6d} {a / 1e3:10.2f} {lo / 1e3:10.2f} {hi / 1e3:10.2f}")


if __name__ == "__main__":
    main()
