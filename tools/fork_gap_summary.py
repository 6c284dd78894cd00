"""Summarises tools/fork_gap_probe.py's kernel trace: for each big fill (A) the gap to the next main-stream
kernel, grouped by the pattern order (plain, fork, fork0; 20 each after 9 warm-up patterns)."""
import csv
import statistics
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", "")))
rows.sort()
main_sid = rows[0][3]
mains = [r for r in rows if r[3] == main_sid]
# A and B alternate on the main stream: pairs (A, B)
pairs = [(mains[i], mains[i + 1]) for i in range(0, len(mains) - 1, 2)]
pairs = pairs[9:]
for n, k in enumerate(("plain", "fork", "fork0")):
    g = [(b[0] - a[1]) / 1e3 for a, b in pairs[20 * n:20 * n + 20]]
    print(f"{k:6s} gap A->B us: median {statistics.median(g):.2f}  min {min(g):.2f}  max {max(g):.2f}")
