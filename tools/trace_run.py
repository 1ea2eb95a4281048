"""One run of a repeated launch sequence from a rocprofv3 kernel trace: the kernels between the
last two launches of MARKER (a substring of its name), start offset, duration and queue.
    python tools/trace_run.py kernel_trace.csv MARKER"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if sys.argv[2] in r["Kernel_Name"]]
s, e = idx[-2], idx[-1]
run = [r for r in rows[s + 1:e + 1] if "copyBuffer" not in r["Kernel_Name"]]
t0 = int(run[0]["Start_Timestamp"])
for r in run:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(st - t0) / 1000:8.1f} {(en - st) / 1000:7.1f} q{r['Queue_Id']} {r['Kernel_Name'][:80]}")
