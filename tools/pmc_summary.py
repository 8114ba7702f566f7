"""Summarise rocprofv3 --pmc CSV output: mean counter value per dispatch of the
kernels whose name contains a substring (experiment tool).

    python tools/pmc_summary.py gpurun_out/pmc [kernel_substring] [--skip N]

Reads every *counter_collection.csv below the directory (one per PMC pass).
`--skip N` drops the first N matching dispatches of each pass (activation
pre-roll rounds of tools/perf_round.py run before the timed rounds).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarise(root, sub="", skip=0, last=None):
    out = {}
    for path in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        per_disp = defaultdict(dict)
        with open(path) as f:
            for row in csv.DictReader(f):
                if sub not in row["Kernel_Name"]:
                    continue
                per_disp[int(row["Dispatch_Id"])][row["Counter_Name"]] = (
                    per_disp[int(row["Dispatch_Id"])].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"]))
        ids = sorted(per_disp)[skip:]
        if last:
            ids = ids[-last:]
        sums = defaultdict(float)
        for d in ids:
            for k, v in per_disp[d].items():
                sums[k] += v
        for k, v in sums.items():
            out[k] = v / max(1, len(ids))
        out.setdefault("_dispatches", 0)
        out["_dispatches"] = max(out["_dispatches"], len(ids))
    return out


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    skip = 0
    last = None
    for a in sys.argv[1:]:
        if a.startswith("--skip="):
            skip = int(a.split("=")[1])
        if a.startswith("--last="):
            last = int(a.split("=")[1])
    res = summarise(args[0], args[1] if len(args) > 1 else "", skip, last)
    print(json.dumps(res, indent=1, sort_keys=True))
