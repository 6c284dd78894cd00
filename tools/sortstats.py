"""Sums the rocPRIM sort kernels (and the rowgrad helpers) of rocprofv3 --stats CSVs: one line per file."""
import csv
import sys

for path in sys.argv[1:]:
    tot, calls = {}, {}
    with open(path) as f:
        for r in csv.DictReader(f):
            n = r["Name"]
            k = ("merge_sort" if "merge_sort" in n else "onesweep" if "onesweep" in n else
                 "histogram" if "histogram" in n else "rocprim_other" if "rocprim" in n else None)
            if k:
                tot[k] = tot.get(k, 0) + int(r["TotalDurationNs"])
                calls[k] = calls.get(k, 0) + int(r["Calls"])
    print(path, {k: (calls[k], round(tot[k] / 1e3, 1)) for k in tot})
