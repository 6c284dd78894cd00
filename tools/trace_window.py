"""Prints the kernels around each occurrence of a name in a rocprofv3 kernel trace (start offset, duration,
stream, gap to the previous dispatch end on any stream), for the first --n occurrences after --skip.

    python tools/trace_window.py trace_kernel_trace.csv clip_finalize --before 6 --after 4
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("name")
ap.add_argument("--before", type=int, default=6)
ap.add_argument("--after", type=int, default=4)
ap.add_argument("--skip", type=int, default=12)
ap.add_argument("--n", type=int, default=2)
args = ap.parse_args()
rows = []
with open(args.trace) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:70],
                     r.get("Stream_Id") or r.get("Queue_Id") or "?"))
rows.sort()
hits = [i for i, r in enumerate(rows) if args.name in r[2]][args.skip:args.skip + args.n]
for i in hits:
    lo, hi = max(0, i - args.before), min(len(rows), i + args.after + 1)
    t0 = rows[lo][0]
    end = rows[lo][1]
    print(f"--- occurrence at row {i}")
    for s, e, n, sid in rows[lo:hi]:
        print(f"{(s - t0) / 1e3:9.2f} us  dur {(e - s) / 1e3:8.2f}  gap {(s - end) / 1e3:7.2f}  stream {sid:>3}  {n}")
        end = max(end, e)
