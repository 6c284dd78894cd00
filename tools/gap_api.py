"""Host HIP API calls issued while the device sits in its largest idle gaps of the timed steps (bench.py
--markers under rocprofv3 --kernel-trace --hip-runtime-trace): which call the device is waiting on.

    python tools/gap_api.py <trace_kernel_trace.csv> <trace_hip_api_trace.csv> [--gaps 3]
"""
import argparse
import csv
from collections import Counter

from prof_summary import load, timed_window


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("ktrace")
    ap.add_argument("api")
    ap.add_argument("--gaps", type=int, default=3)
    args = ap.parse_args()
    rows = load(args.ktrace)
    a, b = timed_window(rows)
    inner = rows[a + 1:b]
    gaps = []
    last_end, last_name = rows[a][1], "marker"
    for s, e, n in inner:
        if s > last_end:
            gaps.append((s - last_end, last_end, s, last_name, n))
        if e > last_end:
            last_end, last_name = e, n
    api = []
    with open(args.api) as fh:
        for r in csv.DictReader(fh):
            api.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]))
    api.sort()
    t0, t1 = rows[a][1], rows[b][0]
    win = [x for x in api if t0 <= x[0] <= t1]
    tot = Counter()
    for s, e, f in win:
        tot[f] += e - s
    print("host API time in the timed window (us, top 15):")
    for f, t in tot.most_common(15):
        print(f"  {t / 1e3:10.1f}  {f}")
    for g, gs, ge, pn, nn in sorted(gaps, reverse=True)[:args.gaps]:
        print(f"\ngap {g / 1e3:.1f} us after {pn.split('(')[0][:50]} before {nn.split('(')[0][:50]}")
        for s, e, f in api:
            if e >= gs - 20000 and s <= ge:
                print(f"  {(s - gs) / 1e3:9.1f} .. {(e - gs) / 1e3:9.1f}  {f}")


if __name__ == "__main__":
    main()
