"""rocprofv3 kernel trace -> where the device sits idle between dispatches in the TIMED steps (bench.py
--markers): every idle interval of the dispatch-interval union is charged to the (kernel that ended last,
kernel that starts next) pair; pairs ranked by idle microseconds per step.

    python tools/gap_summary.py gpurun_out/prof/.../trace_kernel_trace.csv --steps 20
"""
import argparse
from collections import defaultdict

from prof_summary import load, timed_window


def short(n):
    n = n.split("(")[0]
    return n.replace("void ", "").replace("ctr::", "")[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    rows = load(args.trace)
    a, b = timed_window(rows)
    inner = rows[a + 1:b]
    gaps = defaultdict(lambda: [0, 0])
    last_end, last_name = rows[a][1], "marker"
    for s, e, n in inner:
        if s > last_end:
            g = gaps[(short(last_name), short(n))]
            g[0] += s - last_end
            g[1] += 1
        if e > last_end:
            last_end, last_name = e, n
    tot = sum(v[0] for v in gaps.values())
    print(f"idle {tot / 1e3 / args.steps:.1f} us/step over {sum(v[1] for v in gaps.values()) / args.steps:.1f} gaps/step\n")
    print("| us/step | gaps/step | avg us | after | before |\n|---:|---:|---:|---|---|")
    for (p, n), (t, c) in sorted(gaps.items(), key=lambda kv: -kv[1][0])[:args.top]:
        print(f"| {t / 1e3 / args.steps:.1f} | {c / args.steps:.2f} | {t / c / 1e3:.2f} | `{p}` | `{n}` |")


if __name__ == "__main__":
    main()
