"""Per-kernel average duration from a rocprofv3 --kernel-trace --stats summary (kernel_stats.csv),
as a JSON that bench.py attaches to its roofline when the kernel sources match (SHA-256 of csrc/,
like the PMC traffic figure):
  python tools/kernel_time.py OUT.json RUN_TAG path/to/*_kernel_stats.csv"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import kernel_sources_digest  # noqa: E402

out, tag, path = sys.argv[1], sys.argv[2], sys.argv[3]
digest = kernel_sources_digest()
res = {}
for r in csv.DictReader(open(path)):
    name = r["Name"]
    if "fec::" not in name:
        continue
    name = name.split("(")[0].replace("void ", "").replace("fec::", "")
    res[name] = {"avg_ns": float(r["AverageNs"]), "calls": int(r["Calls"]), "min_ns": float(r["MinNs"]),
                 "max_ns": float(r["MaxNs"]), "run": tag, "stats_csv": os.path.basename(path),
                 "sources_sha256": digest}
json.dump(res, open(out, "w"), indent=1, sort_keys=True)
print(json.dumps(res, indent=1))
