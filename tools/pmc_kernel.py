#!/usr/bin/env python3
"""Mean per-dispatch PMC counter values of kernels matching a name, from the
counter_collection CSVs under a rocprofv3 output directory.  Development tool.

usage: tools/pmc_kernel.py <dir> <kernel-substring>..."""
import collections
import csv
import glob
import os
import sys

root, pats = sys.argv[1], sys.argv[2:]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            name = r.get("Kernel_Name", "")
            for p in pats:
                if p in name:
                    vals[p][r["Counter_Name"]].append(float(r["Counter_Value"]))
for p in pats:
    print(f"== {p}")
    for c, v in sorted(vals[p].items()):
        print(f"  {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
