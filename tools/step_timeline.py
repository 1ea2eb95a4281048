"""Per-step timeline of the bench step from a rocprofv3 --kernel-trace CSV (kernel_trace.csv):
for every encoder launch, the kernels up to the next one with their start / end relative to the
encoder's start (median over the steps), so the gaps between the step's kernels show.
  python tools/step_timeline.py path/to/*_kernel_trace.csv [--last 200]"""
import argparse
import csv
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--last", type=int, default=200, help="steps at the end of the trace to use")
args = ap.parse_args()

rows = []
for r in csv.DictReader(open(args.trace)):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fec::", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
rows.sort()
steps = []
cur = None
for s, e, name in rows:
    if name.startswith("fec_encode"):
        cur = [(s, e, name)]
        steps.append(cur)
    elif cur is not None:
        cur.append((s, e, name))
import collections
common = collections.Counter(len(st) for st in steps if len(st) > 1).most_common(1)[0][0]
steps = [st for st in steps[:-1] if len(st) == common][-args.last:]
if not steps:
    raise SystemExit("no complete steps")
print(f"{len(steps)} steps, {len(steps[0])} kernels each")
period = statistics.median(steps[i + 1][0][0] - steps[i][0][0] for i in range(len(steps) - 1))
print(f"step period (encoder start to encoder start): {period / 1e3:.1f} us")
for j, (_, _, name) in enumerate(steps[0]):
    st = statistics.median(x[j][0] - x[0][0] for x in steps)
    en = statistics.median(x[j][1] - x[0][0] for x in steps)
    print(f"  {name[:48]:48s} start {st / 1e3:8.1f}  end {en / 1e3:8.1f}  dur {(en - st) / 1e3:7.1f} us")
