"""rocprofv3 kernel trace -> per-stream summary of the TIMED steps (markdown): which kernels each HIP stream runs,
per step, and how much of each stream's time overlaps the other's.  The main stream (the one holding the most
kernel time) is the step's critical path; the side stream's kernels only cost what they do not overlap.

    python tools/stream_summary.py gpurun_out/prof/.../trace_kernel_trace.csv --steps 20 [--top 40]
"""
import argparse
import csv
from collections import defaultdict

MARKER = "step_marker_kernel"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    rows = []
    with open(args.trace) as fh:
        for r in csv.DictReader(fh):
            sid = r.get("Stream_Id") or r.get("Queue_Id") or "0"
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], sid))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if MARKER in r[2]]
    if len(marks) < 2:
        raise SystemExit("expected two step markers (bench.py --markers)")
    rows = rows[marks[0] + 1:marks[1]]
    n = args.steps
    by_stream = defaultdict(list)
    for r in rows:
        by_stream[r[3]].append(r)
    tot = {s: sum(e - b for b, e, _, _ in v) for s, v in by_stream.items()}
    order = sorted(tot, key=tot.get, reverse=True)
    span = (rows[-1][1] - rows[0][0]) if rows else 0
    print("# Per-stream kernel time, timed steps\n")
    print(f"{len(rows)} dispatches; span {span / 1e3 / n:.1f} us/step.\n")
    # busy intervals per stream and their overlap with the main stream
    def busy(v):
        iv = sorted((b, e) for b, e, _, _ in v)
        out = []
        for b, e in iv:
            if out and b <= out[-1][1]:
                out[-1][1] = max(out[-1][1], e)
            else:
                out.append([b, e])
        return out
    main = busy(by_stream[order[0]])
    for s in order:
        v = by_stream[s]
        bs = busy(v)
        ov = 0
        j = 0
        for b, e in bs:
            while j < len(main) and main[j][1] <= b:
                j += 1
            k = j
            while k < len(main) and main[k][0] < e:
                ov += max(0, min(e, main[k][1]) - max(b, main[k][0]))
                k += 1
        busy_t = sum(e - b for b, e in bs)
        print(f"## stream {s}: {len(v) / n:.1f} dispatches/step, kernels {tot[s] / 1e3 / n:.1f} us/step, busy "
              f"{busy_t / 1e3 / n:.1f} us/step" + ("" if s == order[0] else
                                                      f", of which overlapping stream {order[0]} {ov / 1e3 / n:.1f}"))
        print()
        agg = defaultdict(lambda: [0, 0])
        for b, e, k, _ in v:
            agg[k][0] += 1
            agg[k][1] += e - b
        print("| us/step | calls/step | avg us | kernel |\n|---:|---:|---:|---|")
        for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:args.top]:
            print(f"| {t / 1e3 / n:.1f} | {c / n:.2f} | {t / 1e3 / c:.1f} | `{k[:110]}` |")
        print()


if __name__ == "__main__":
    main()
