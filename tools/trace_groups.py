"""Per-call spans of a rocprofv3 kernel trace (--kernel-trace csv): kernels whose names contain
one of the given substrings are grouped into calls (a new call starts after a gap of more than
--gap us), and each call's span and per-kernel [start, end] offsets are printed.
    python tools/trace_groups.py <kernel_trace.csv> <substring>[,<substring>...] [--gap US] [--show N]"""
import csv
import sys


def main():
    path, subs = sys.argv[1], sys.argv[2].split(",")
    gap = float(sys.argv[sys.argv.index("--gap") + 1]) if "--gap" in sys.argv else 20.0
    show = int(sys.argv[sys.argv.index("--show") + 1]) if "--show" in sys.argv else 2
    rows = [r for r in csv.DictReader(open(path)) if any(s in r["Kernel_Name"] for s in subs)]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    calls, cur, end = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if cur and s - end > gap * 1e3:
            calls.append(cur)
            cur = []
        cur.append((s, e, r))
        end = e if end is None or not cur[:-1] else max(end, e)
    if cur:
        calls.append(cur)
    spans = sorted((max(e for _, e, _ in c) - c[0][0]) / 1e3 for c in calls)
    print(f"{len(calls)} calls, span median {spans[len(spans) // 2]:.1f} us, min {spans[0]:.1f} us")
    for c in calls[-show:]:
        t0 = c[0][0]
        for s, e, r in c:
            print(f"  {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q{r['Queue_Id']} {r['Kernel_Name'][:80]}")
        print()


if __name__ == "__main__":
    main()
