"""Per-kernel mean of every PMC counter collected by tools/pmc_passes.sh (rocprofv3 csv output).
Usage: python tools/pmc_summary.py <dir> [--json out.json]"""
import collections
import csv
import glob
import json
import os
import sys


def main(d, out_json=None, quiet=False):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            per_dispatch = collections.defaultdict(float)
            names = {}
            for r in csv.DictReader(f):
                key = (r["Dispatch_Id"], r["Counter_Name"])
                per_dispatch[key] += float(r["Counter_Value"])      # summed over XCD/SE instances
                names[r["Dispatch_Id"]] = r["Kernel_Name"]
            for (disp, ctr), v in per_dispatch.items():
                acc[names[disp]][ctr].append(v)
    res = {}
    for k, ctrs in sorted(acc.items()):
        short = k.split("(")[0]
        res[short] = {c: sum(v) / len(v) for c, v in sorted(ctrs.items())}
        res[short]["dispatches"] = max(len(v) for v in ctrs.values())
        if quiet:
            continue
        print(short)
        for c, v in sorted(res[short].items()):
            print(f"   {c:28s} {v:18.1f}")
    if out_json:
        with open(out_json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[3] if len(sys.argv) > 3 and sys.argv[2] == "--json" else None)
