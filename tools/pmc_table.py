"""Per-kernel table of tools/pmc_kbench.sh passes (mean per dispatch; SQ_*_CYCLES / WAIT / ACTIVE in
quad-cycles per MI355X_MICROARCH.md).   python tools/pmc_table.py <outdir>"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
data = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
    per = defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(f)):
        k = int(r["Dispatch_Id"])
        names[k] = r["Kernel_Name"]
        per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for k, cs in per.items():
        for c, v in cs.items():
            data[names[k][:60]][c].append(v)
for kname, cs in data.items():
    print(kname)
    for c in sorted(cs):
        v = cs[c]
        print(f"   {c:28s} {sum(v) / len(v):16.1f}")
