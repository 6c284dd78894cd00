"""Isolated lazy-table flush (ctr_lazy_flush_pair / ctr_lazy_flush) on a synthetic lazy state at the cfg2
shape, for A/B timing of flush variants (CTR_LIB_PATH).  Not part of the product.

Pair tables: 2 x R rows of width W (att | rep); row states: a fraction --nz of the rows stepped at a tick
U[1, T-1] (moments non-zero), --cur current (tick T), the rest never touched (tick 0, zero moments).
Cat tables: 35 tables of 1e6 rows, widths from the cfg2 arch, the same state mix.

    python tools/flushbench.py [--T 25] [--nz 0.45] [--which pair,cat] [--iters 3]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "toss-next-ctr-prediction_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from tossctr import _lib  # noqa: E402
from tossctr._lib import call  # noqa: E402

NZ = -2 ** 31


def ptr(t, e=0):
    return t.data_ptr() + e * t.element_size()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=25)
    ap.add_argument("--nz", type=float, default=0.45)
    ap.add_argument("--cur", type=float, default=0.02)
    ap.add_argument("--R", type=int, default=10_000_000)
    ap.add_argument("--W", type=int, default=32)
    ap.add_argument("--which", default="pair,cat")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--no-ema", action="store_true")
    ap.add_argument("--round4", action="store_true", help="cat widths rounded up to a multiple of 4 (probe)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device=dev).manual_seed(0)
    T = args.T
    hist = torch.zeros((T + 2) * _lib.query("ctr_opt_hist_entry_bytes"), dtype=torch.uint8, device=dev)
    for t in range(1, T + 1):
        call("ctr_opt_hist_record", ptr(hist), t, 3e-4 * min(1.0, t / 10), 1e-4, 0.9, 0.999, 1e-8, t, 0.999, 1, 1, st)

    def state(rows):
        u = torch.rand(rows, generator=g, device=dev)
        s = torch.zeros(rows, dtype=torch.int32, device=dev)
        nzm = u < args.nz
        s[nzm] = torch.randint(1, T, (int(nzm.sum()),), generator=g, device=dev, dtype=torch.int32) | NZ
        s[(u >= args.nz) & (u < args.nz + args.cur)] = T
        return s

    def arrays(n, rows_nz):
        P = torch.randn(n, generator=g, device=dev)
        E = P.clone()
        M = torch.randn(n, generator=g, device=dev) * 1e-3 * rows_nz
        V = torch.rand(n, generator=g, device=dev) * 1e-6 * rows_nz
        return P, M, V, (None if args.no_ema else E)

    def run(name, fn, last, last0, nbytes):
        ts = []
        for _ in range(args.iters):
            last.copy_(last0)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        t = sorted(ts)[len(ts) // 2]
        print(f"{name}: {t:.3f} ms  ({nbytes / t / 1e6:.0f} GB/s of p/e/m/v state bytes)")

    if "pair" in args.which:
        R, W = args.R, args.W
        s0 = state(R)
        last = torch.empty(2 * R, dtype=torch.int32, device=dev)
        last0 = torch.cat([s0, s0])
        rows_nz = ((s0 < 0).float()).repeat_interleave(W).repeat(2)
        P, M, V, E = arrays(2 * R * W, rows_nz)
        del rows_nz
        arr = (_lib.LazyTab * 2)()
        for i in range(2):
            arr[i].p_off, arr[i].rows, arr[i].width, arr[i].key_base, arr[i].last = i * R * W, R, W, 0, ptr(last, i * R)
        tabs = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).to(dev)
        nb = 2 * R * W * 4 * (2 if E is not None else 1) * 2 * (1 + args.nz)
        run("pair flush", lambda: call("ctr_lazy_flush_pair", ptr(tabs), W, R, ptr(P), ptr(M), ptr(V),
                                       ptr(E) if E is not None else None, ptr(hist), T, st), last, last0, nb)
        del P, M, V, E
    if "cat" in args.which:
        from tossctr.configs import BENCH_CONFIGS, N_NUM_NEXT, cat_cardinals
        from tossctr.arch import Arch
        cfg = BENCH_CONFIGS["cfg2"](batch_size=4096)
        cards = cat_cardinals(cfg)
        a = Arch.from_cfg(cfg, 10_000_000, N_NUM_NEXT, N_NUM_NEXT, cards, list(cfg["data"]["cat_cols"]))
        rows = list(a.cat_cards)
        widths = list(a.cat_dims)
        if args.round4:
            widths = [(w + 3) // 4 * 4 for w in widths]
        tot_rows = sum(rows)
        s0 = state(tot_rows)
        last = torch.empty(tot_rows, dtype=torch.int32, device=dev)
        nz_el = torch.cat([(s0[o:o + r] < 0).float().repeat_interleave(w)
                           for o, r, w in zip(np.cumsum([0] + rows[:-1]), rows, widths)])
        n = int(nz_el.numel())
        P, M, V, E = arrays(n, nz_el)
        del nz_el
        arr = (_lib.LazyTab * len(rows))()
        po, ro = 0, 0
        for i, (r, w) in enumerate(zip(rows, widths)):
            arr[i].p_off, arr[i].rows, arr[i].width, arr[i].key_base, arr[i].last = po, r, w, ro, ptr(last, ro)
            po += r * w
            ro += r
        tabs = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).to(dev)
        nb = n * 4 * (2 if E is not None else 1) * 2 * (1 + args.nz)
        run(f"cat flush ({len(rows)} tables, {tot_rows / 1e6:.1f} M rows, {n / 1e6:.0f} M elements)",
            lambda: call("ctr_lazy_flush", ptr(tabs), len(rows), max(rows), ptr(P), ptr(M), ptr(V),
                         ptr(E) if E is not None else None, ptr(hist), T, st), last, s0, nb)


if __name__ == "__main__":
    main()
