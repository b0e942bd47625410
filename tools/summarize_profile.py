#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (gpurun_out/prof_<tag>/) into profiles/.

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats, as
produced) and profiles/<tag>_summary.{json,md}: per hot-path kernel the average
duration and the per-dispatch PMC counters, plus the HBM traffic estimate
corrected as MI355X_MICROARCH.md §HBM prescribes (FETCH_SIZE and WRITE_SIZE
are KB; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming
reads, so the read side is also given x2; WRITE_SIZE is exact for 16-B stores).
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import re
import shutil
import sys

HOT = ("bwd_tile_kernel", "tile_combine_kernel", "bwd_bin_sum_kernel", "fwd_panel_kernel", "carry_fixup_kernel", "carry_fixup_owner_kernel", "bwd_panel_kernel",
       "bwd_segsum_kernel", "bwd_local_kernel", "fwd_warp4_kernel", "bwd_warp4_kernel",
       "fwd_rel4_panel_kernel", "bwd_local_rel8_kernel", "grad_interleave_kernel",
       "cbsr_bank_order_kernel", "rows_sum_kernel", "bwd_multi_stage_kernel",
       "fwd_rel8_gather_kernel", "bwd_rel8_gather_stage_kernel", "cbsr_colmask_kernel")


def kname(full: str) -> str:
    """Kernel base name from a truncated (-T) or full rocprofv3 name."""
    s = full.replace("(anonymous namespace)::", "")
    if s.startswith("void "):
        s = s[5:]
    return re.split(r"[<(]", s)[0].split("::")[-1].strip()


def main(tag: str, root: str = ".", workload: str | None = None):
    src = os.path.join(root, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(root, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))[0]
    shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    kern = {}
    for r in csv.DictReader(open(stats)):
        name = kname(r["Name"])
        if any(name.endswith(h) for h in HOT):
            kern[name] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                          "min_ms": float(r["MinNs"]) / 1e6, "max_ms": float(r["MaxNs"]) / 1e6}
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(src, "pmc_*", "*counter_collection.csv")):
        per_dispatch = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per_dispatch[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = kname(r["Kernel_Name"])
        for (d, c), v in per_dispatch.items():
            n = names[d]
            if any(n.endswith(h) for h in HOT):
                pmc[n][c].append(v)
    out = {"tag": tag, "kernels": {}}
    for n in sorted(set(kern) | set(pmc)):
        row = dict(kern.get(n, {}))
        for c, vals in pmc.get(n, {}).items():
            row[c] = sum(vals) / len(vals)
        if "FETCH_SIZE" in row:
            row["hbm_read_bytes_raw"] = row["FETCH_SIZE"] * 1024
            row["hbm_read_bytes_x2"] = row["FETCH_SIZE"] * 2048
        if "WRITE_SIZE" in row:
            row["hbm_write_bytes"] = row["WRITE_SIZE"] * 1024
        if "TCC_HIT_sum" in row and "TCC_MISS_sum" in row:
            t = row["TCC_HIT_sum"] + row["TCC_MISS_sum"]
            row["l2_hit_rate"] = row["TCC_HIT_sum"] / t if t else None
        out["kernels"][n] = row
    json.dump(out, open(os.path.join(dst, f"{tag}_summary.json"), "w"), indent=1)
    if workload:  # per-launch HBM traffic of each kernel, read by bench.py
        idx_path = os.path.join(dst, "pmc_traffic.json")
        idx = json.load(open(idx_path)) if os.path.exists(idx_path) else {}
        k = out["kernels"]

        per_launch = {n: r["hbm_read_bytes_x2"] + r["hbm_write_bytes"] for n, r in k.items()
                      if "hbm_read_bytes_x2" in r and "hbm_write_bytes" in r}
        # bench.py composes a call's traffic from these (launches per call known there);
        # the entry is keyed to the kernel sources it measured (bench.py refuses a
        # profile whose key differs from the tree's), so it must be summarised from
        # the same tree that ran the profile
        sys.path.insert(0, os.path.abspath(root))
        from bench import kernel_source_sha
        issue = {}
        for n, r in k.items():
            c = {x: r[x] for x in ("avg_ms", "GRBM_GUI_ACTIVE", "SQ_INSTS_SALU", "SQ_INSTS_VALU",
                                   "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_LDS_IDX_ACTIVE",
                                   "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY",
                                   "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES") if x in r}
            if "GRBM_GUI_ACTIVE" in c and len(c) > 2:
                issue[n] = c
        idx[workload] = {"profile": tag, "source_sha": kernel_source_sha(os.path.abspath(root)),
                         "kernels": per_launch, "issue": issue}
        json.dump(idx, open(idx_path, "w"), indent=1)
    with open(os.path.join(dst, f"{tag}_summary.md"), "w") as fh:
        fh.write(f"# rocprofv3 summary `{tag}`\n\nSource: `tools/profile.sh {tag}` "
                 "(kernel trace + stats pass, then one PMC group per pass).\n\n")
        fh.write("| kernel | calls | avg ms | HBM read (x2 corr.) GB | HBM write GB | L2 hit |\n")
        fh.write("|---|---|---|---|---|---|\n")
        for n, r in out["kernels"].items():
            rd = r.get("hbm_read_bytes_x2")
            wr = r.get("hbm_write_bytes")
            hit = r.get("l2_hit_rate")
            fh.write(f"| {n} | {r.get('calls', '')} | {r.get('avg_ms', float('nan')):.3f} | "
                     f"{'' if rd is None else f'{rd / 1e9:.2f}'} | "
                     f"{'' if wr is None else f'{wr / 1e9:.2f}'} | "
                     f"{'' if hit is None else f'{hit:.2f}'} |\n")
    print(json.dumps(out, indent=1)[:3000])


if __name__ == "__main__":
    main(sys.argv[1], ".", sys.argv[2] if len(sys.argv) > 2 else None)
