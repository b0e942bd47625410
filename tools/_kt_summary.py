"""Compact per-kernel-name summary of a rocprofv3 csv dir (kernel trace or counter
collection): name -> calls, mean ms (trace) or mean counter values (pmc)."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
for path in glob.glob(root + "/**/*kernel_trace.csv", recursive=True):
    agg = defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"][:90]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        if sum(v) > 1.0:
            print(f"TRACE {len(v):4d} {sum(v) / len(v):8.3f} ms  {k}")
for path in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
    agg = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in agg.items():
        vals = {c: sum(v) / len(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        if any(x > 1e5 for x in vals.values()):
            print(f"PMC {n:4d} " + " ".join(f"{c}={x:.6g}" for c, x in vals.items()) + f"  {k}")
# KT_SERIES=<substring>: the last 24 durations of every kernel whose name holds it
import os  # noqa: E402
pat = os.environ.get("KT_SERIES")
if pat:
    for path in glob.glob(root + "/**/*kernel_trace.csv", recursive=True):
        rows = [r for r in csv.DictReader(open(path)) if pat in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        for r in rows[-24:]:
            print(f"SERIES {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6:8.3f} ms  "
                  f"{r['Kernel_Name'][:100]}")
