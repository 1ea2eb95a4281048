"""Summarise rocprofv3 --pmc CSVs: per kernel, counters averaged per dispatch.

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE counts half the bytes of wide (16 B per
lane) coalesced streaming reads (/opt/skills/guides/MI355X_MICROARCH.md, HBM section), so the HBM
read bytes are FETCH_SIZE x 1024 x 2; WRITE_SIZE x 1024 is exact for 16-byte stores.  Both the raw
and the corrected figures are printed, with the corrected total per dispatch."""
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
    per = {}
    for c, v in sorted(cs.items()):
        nd = len(disp[(name, c)])
        per[c] = v / nd
        print(f"   {c:24s} {v / nd:14.5g}")
    if "FETCH_SIZE" in per:
        rd = per["FETCH_SIZE"] * 1024 * 2
        print(f"   {'HBM read bytes':24s} {rd:14.5g}   (FETCH_SIZE x 1024 x 2, the gfx950 correction)")
        if "WRITE_SIZE" in per:
            wr = per["WRITE_SIZE"] * 1024
            print(f"   {'HBM write bytes':24s} {wr:14.5g}   (WRITE_SIZE x 1024)")
            print(f"   {'HBM traffic bytes':24s} {rd + wr:14.5g}")
