"""HBM traffic per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/pmc_traffic.sh).

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch.  Per MI355X_MICROARCH.md (HBM / rocprofv3): on
gfx950 FETCH_SIZE counts half the bytes of a wide coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16-byte streaming stores.  Writes {kernel: {...}} as JSON.
A directory's workload is its name without trailing digits (step1, step2 -> step): a kernel that
runs in several workloads (the encoder in the headline step and in the relay chain, at 1 M and
360 k packets) is averaged over the first workload's passes only, so a per-launch figure never
mixes launch sizes.

  python tools/pmc_traffic.py OUT.json RUN_TAG pmc_dir [pmc_dir ...]
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import kernel_sources_digest  # noqa: E402

out, tag, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
digest = kernel_sources_digest()
vals = collections.defaultdict(lambda: collections.defaultdict(list))
owner = {}  # kernel -> the workload its figures come from
for d in dirs:
    workload = os.path.basename(os.path.normpath(d)).rstrip("0123456789")
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"]
            if "fec::" not in name:
                continue
            name = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("fec::", "")
            if owner.setdefault(name, workload) != workload:
                continue
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
for name, cs in vals.items():
    if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
        continue
    fetch = 2.0 * 1024 * sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
    write = 1024 * sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
    res[name] = {"fetch_bytes": round(fetch), "write_bytes": round(write),
                 "traffic_bytes": round(fetch + write), "run": tag, "workload": owner[name],
                 "sources_sha256": digest,
                 "note": "FETCH_SIZE x2 (gfx950 correction), WRITE_SIZE as read; per launch"}
json.dump(res, open(out, "w"), indent=1, sort_keys=True)
print(json.dumps(res, indent=1))
