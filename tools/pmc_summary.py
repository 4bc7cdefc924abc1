#!/usr/bin/env python3
"""Summarise rocprofv3 PMC csv files: per-kernel average counter value per dispatch."""
import collections, csv, glob, os, sys
root = sys.argv[1]
for d in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
    agg = collections.defaultdict(float); cnt = collections.Counter()
    for r in csv.DictReader(open(d)):
        k = r["Kernel_Name"].split("(")[0]
        if "rocclr" in k:
            continue
        agg[(k, r["Counter_Name"])] += float(r["Counter_Value"]); cnt[(k, r["Counter_Name"])] += 1
    for (k, c), v in sorted(agg.items()):
        print("%-28s %-24s %.6g" % (k, c, v / cnt[(k, c)]))
