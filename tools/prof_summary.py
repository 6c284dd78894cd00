"""rocprofv3 --stats kernel summary (run_kernel_stats.csv) -> markdown table, per-step figures.

    python tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv --steps 13 [--top 45] > profiles/r01/x.md
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, required=True, help="steps the profiled command ran (warm-up + timed)")
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--title", default="rocprofv3 kernel summary")
    args = ap.parse_args()
    rows = []
    with open(args.csv) as fh:
        for r in csv.DictReader(fh):
            rows.append((float(r["TotalDurationNs"]), int(r["Calls"]), float(r["AverageNs"]), r["Name"]))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    print(f"# {args.title}\n")
    print(f"Total device time {tot / 1e6:.2f} ms over {args.steps} steps (incl. setup-only kernels) = "
          f"{tot / 1e3 / args.steps:.1f} us/step.\n")
    print("| us/step | calls/step | avg us | kernel |\n|---:|---:|---:|---|")
    for t, c, avg, name in rows[:args.top]:
        print(f"| {t / 1e3 / args.steps:.1f} | {c / args.steps:.1f} | {avg / 1e3:.1f} | `{name[:110]}` |")


if __name__ == "__main__":
    main()
