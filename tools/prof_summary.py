"""rocprofv3 kernel trace -> per-step kernel summary of the TIMED steps only (markdown).

bench.py --markers launches an empty ``step_marker_kernel`` right before the first timed step and
right after the timed region's final flush; only the dispatches between those two markers are
summarised, so setup kernels (weight init, synthetic data, warm-up) stay out of the per-step figures.
Reported beside the per-kernel table: the span between the markers (device wall time of the timed
region), the summed kernel time, and the difference = inter-kernel idle per step.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof -o trace -- \
        python bench.py --steps 20 --warmup 10 --no-cpu-baseline --markers
    python tools/prof_summary.py gpurun_out/prof/.../trace_kernel_trace.csv --steps 20 > profiles/r02/x.md
"""
import argparse
import csv
from collections import defaultdict

MARKER = "step_marker_kernel"


def load(path):
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def timed_window(rows):
    marks = [i for i, r in enumerate(rows) if MARKER in r[2]]
    if len(marks) < 2:
        raise SystemExit(f"expected two {MARKER} dispatches (bench.py --markers), found {len(marks)}")
    return marks[0], marks[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace", help="rocprofv3 *_kernel_trace.csv")
    ap.add_argument("--steps", type=int, required=True, help="timed steps between the markers")
    ap.add_argument("--top", type=int, default=50)
    ap.add_argument("--title", default="rocprofv3 kernel trace, timed steps only")
    args = ap.parse_args()
    rows = load(args.trace)
    a, b = timed_window(rows)
    inner = rows[a + 1:b]
    span = rows[b][0] - rows[a][1]
    agg = defaultdict(lambda: [0, 0])
    busy = 0
    last_end = rows[a][1]
    for s, e, n in inner:
        agg[n][0] += e - s
        agg[n][1] += 1
        # device-busy time: union of the dispatch intervals (a single stream: they do not overlap)
        busy += max(0, e - max(s, last_end))
        last_end = max(last_end, e)
    tot = sum(v[0] for v in agg.values())
    st = args.steps
    print(f"# {args.title}\n")
    print(f"{len(inner)} dispatches in the timed region ({len(inner) / st:.1f} per step).  Marker-to-marker span "
          f"{span / 1e6:.3f} ms = {span / 1e3 / st:.1f} us/step; kernels {tot / 1e3 / st:.1f} us/step; device busy "
          f"{busy / 1e3 / st:.1f} us/step; idle between dispatches {(span - busy) / 1e3 / st:.1f} us/step.\n")
    print("| us/step | share | calls/step | avg us | kernel |\n|---:|---:|---:|---:|---|")
    for n, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:args.top]:
        print(f"| {t / 1e3 / st:.1f} | {t / tot:.3f} | {c / st:.2f} | {t / c / 1e3:.1f} | `{n[:110]}` |")


if __name__ == "__main__":
    main()
