"""rocprofv3 --pmc passes (tools/pmc_r02.sh) -> one per-kernel table of the TIMED steps (markdown).

Every pass ran ``bench.py --markers``; only dispatches between the two ``step_marker_kernel``s count.
Per kernel: the average counter value per dispatch, joined over the passes by kernel name, plus the
non-PMC kernel duration from a kernel-trace summary (PMC runs serialise dispatches, so their own
timestamps are not used).  Derived columns:
  * HBM bytes  = 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024; gfx950 FETCH_SIZE counts half of wide
    streaming reads, MI355X_MICROARCH.md "HBM")
  * MFMA TF/s  = (SQ_INSTS_VALU_MFMA_MOPS_F32 + _BF16, each when collected -- the f32 one comes from the "mops" pass
    of tools/profile.sh; without it f32-MFMA kernels read 0) x 512 FLOP / duration; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES /
    (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
  * VALU issue = SQ_INSTS_VALU x 2 cycles (a wave64 VALU instruction on a 32-wide SIMD) / (duration x
    2.4 GHz x 1024 SIMDs): the fraction of the chip's VALU issue slots the kernel's vector instructions fill
  * LDS conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles per LDS-array cycle)
  * wave-time split = SQ_WAIT_ANY, SQ_WAIT_INST_ANY (of which SQ_WAIT_INST_LDS) over SQ_WAVE_CYCLES

    python tools/pmc_summary.py gpurun_out/pmc --passes fetch write mfma lds --trace-md profiles/r02/x.md
"""
import argparse
import csv
import os
import re
from collections import defaultdict

MARKER = "step_marker_kernel"


def load_pass(path):
    """{kernel: {counter: mean value per dispatch}} over the dispatches between the markers."""
    by_disp = defaultdict(dict)
    names = {}
    with open(path) as fh:
        for r in csv.DictReader(fh):
            d = int(r["Dispatch_Id"])
            names[d] = r["Kernel_Name"]
            by_disp[d][r["Counter_Name"]] = by_disp[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    order = sorted(names)
    marks = [d for d in order if MARKER in names[d]]
    if len(marks) < 2:
        raise SystemExit(f"{path}: no step markers")
    agg = defaultdict(lambda: defaultdict(list))
    for d in order:
        if marks[0] < d < marks[1]:
            for c, v in by_disp[d].items():
                agg[names[d]][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}


def trace_durations(md):
    """avg us per launch by kernel name from a tools/prof_summary.py table."""
    out = {}
    if md and os.path.exists(md):
        for line in open(md):
            m = re.match(r"\| ([\d.]+) \| [\d.]+ \| ([\d.]+) \| ([\d.]+) \| `(.*)` \|", line)
            if m:
                out[m.group(4)] = float(m.group(3))
    return out


def short(n, width=70):
    n = n.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n).replace("ctr::", "").replace("void ", "")
    return n[:width]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--passes", nargs="+", required=True)
    ap.add_argument("--trace-md", default=None, help="tools/prof_summary.py output of the same config")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--title", default="PMC counters per kernel, timed steps")
    args = ap.parse_args()
    data = defaultdict(dict)
    for p in args.passes:
        f = os.path.join(args.dir, p, f"{p}_counter_collection.csv")
        for k, cs in load_pass(f).items():
            data[k].update(cs)
    dur = trace_durations(args.trace_md)
    keys = [k for k in data if k[:110] in dur] or list(data)
    keys.sort(key=lambda k: -dur.get(k[:110], 0.0))
    print(f"# {args.title}\n")
    print("Counters: averages per dispatch over the timed steps of each pass (tools/pmc_summary.py).  "
          "Duration: the non-PMC kernel trace.\n")
    print("| kernel | avg us | HBM MB (2F+W) | write MB | MFMA TF/s | MFMA busy | LDS confl | VALU insts/wave | "
          "VALU issue | wait-mem | wait-issue (LDS) |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k in keys[:args.top]:
        c = data[k]
        us = dur.get(k[:110])
        hb = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024 / 1e6 if "FETCH_SIZE" in c and "WRITE_SIZE" in c else None
        wr = c["WRITE_SIZE"] * 1024 / 1e6 if "WRITE_SIZE" in c else None
        mops = [c[n] for n in ("SQ_INSTS_VALU_MFMA_MOPS_F32", "SQ_INSTS_VALU_MFMA_MOPS_BF16") if n in c]
        tf = sum(mops) * 512 / (us * 1e-6) / 1e12 if us and mops else None
        busy = (c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)
                if c.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in c else None)
        lds = (c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"] if c.get("SQ_LDS_IDX_ACTIVE") else None)
        valu = c["SQ_INSTS_VALU"] / c["SQ_WAVES"] if c.get("SQ_WAVES") and "SQ_INSTS_VALU" in c else None
        # VALU issue fraction: wave64 VALU instructions x 2 cycles over (duration x 2.4 GHz x 1024 SIMDs)
        vis = c["SQ_INSTS_VALU"] * 2 / (us * 1e-6 * 2.4e9 * 1024) if us and "SQ_INSTS_VALU" in c else None
        wc = c.get("SQ_WAVE_CYCLES")
        wmem = c["SQ_WAIT_ANY"] / wc if wc and "SQ_WAIT_ANY" in c else None
        wiss = (f"{c['SQ_WAIT_INST_ANY'] / wc:.2f} ({c['SQ_WAIT_INST_LDS'] / wc:.2f})"
                if wc and "SQ_WAIT_INST_ANY" in c and "SQ_WAIT_INST_LDS" in c else "")
        f = lambda v, fmt: "" if v is None else format(v, fmt)     # noqa: E731
        print(f"| `{short(k)}` | {f(us, '.1f')} | {f(hb, '.1f')} | {f(wr, '.1f')} | {f(tf, '.1f')} | {f(busy, '.2f')} | "
              f"{f(lds, '.3f')} | {f(valu, '.0f')} | {f(vis, '.2f')} | {f(wmem, '.2f')} | {wiss} |")


if __name__ == "__main__":
    main()
