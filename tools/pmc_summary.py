"""Summarise rocprofv3 --pmc CSVs: per kernel, counters averaged per dispatch."""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "fec::" not in name:
            continue
        name = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("fec::", "")
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(name, r["Counter_Name"])].add(r["Dispatch_Id"])
for name, cs in agg.items():
    print(name)
    for c, v in sorted(cs.items()):
        nd = len(disp[(name, c)])
        print(f"   {c:24s} {v / nd:14.5g}")
