"""Isolated launches of the encoder-layer kernels at the cfg2 shape (M = 4096 x 60 rows, D = 32,
FF = 384, H = 8) for rocprofv3 PMC passes and quick A/B timing.  Not part of the product.

    python tools/kbench.py [--which ffn,attn] [--iters 10] [--D 32] [--K 60]
"""
import argparse
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "toss-next-ctr-prediction_amd"))

import torch  # noqa: E402

from tossctr import _lib  # noqa: E402
from tossctr._lib import call  # noqa: E402


def ptr(t):
    return t.data_ptr() if t is not None else None


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="ffn,attn")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--K", type=int, default=60)
    ap.add_argument("--D", type=int, default=32)
    ap.add_argument("--FF", type=int, default=384)
    ap.add_argument("--H", type=int, default=8)
    ap.add_argument("--p", type=float, default=0.1, help="dropout probability (0: no dropout)")
    args = ap.parse_args()
    torch.manual_seed(0)
    st = torch.cuda.current_stream().cuda_stream
    B, K, D, FF, H = args.B, args.K, args.D, args.FF, args.H
    M = B * K
    which = args.which.split(",")
    if "ffn" in which:
        x = torch.randn(M, D, device="cuda")
        W1 = torch.randn(FF, D, device="cuda") / math.sqrt(D)
        b1 = torch.randn(FF, device="cuda") * 0.1
        W2 = torch.randn(D, FF, device="cuda") / math.sqrt(FF)
        b2 = torch.randn(D, device="cuda") * 0.1
        nw = torch.ones(D, device="cuda")
        thr = int(round(args.p * (1 << 24)))
        mask = torch.zeros(_lib.query("ctr_ffn_mask_words", M, FF), dtype=torch.int32, device="cuda")
        y, h, r = torch.empty(M, D, device="cuda"), torch.empty(M, D, device="cuda"), torch.empty(M, device="cuda")
        dh, dx = torch.randn(M, D, device="cuda"), torch.empty(M, D, device="cuda")
        o_b1, o_w2 = FF * D, FF * D + FF
        ld = (o_w2 + D * FF + 3) // 4 * 4
        nb = _lib.query("ctr_ffn_slab_rows", M, D)
        slab = torch.zeros(nb, ld, device="cuda")
        fwd = lambda: call("ctr_ffn_fwd", ptr(x), M, D, FF, ptr(W1), ptr(b1), ptr(W2), ptr(b2), ptr(nw), 1e-6, 12345,
                           thr, 1.0 / 0.9, ptr(mask), ptr(y), ptr(h), ptr(r), st)
        bwd = lambda: call("ctr_ffn_bwd", ptr(x), ptr(dh), M, D, FF, ptr(W1), ptr(b1), ptr(W2), 12345, thr, 1.0 / 0.9,
                           ptr(mask), ptr(dx), ptr(slab), ld, o_b1, o_w2, st)
        tf = timeit(fwd, args.iters)
        tb = timeit(bwd, args.iters)
        print(f"ffn_fwd M={M} D={D} FF={FF}: {tf * 1e3:.1f} us  {4.0 * M * FF * D / tf / 1e9:.1f} TF/s")
        print(f"ffn_bwd M={M} D={D} FF={FF}: {tb * 1e3:.1f} us  {8.0 * M * FF * D / tb / 1e9:.1f} TF/s")
    if "attn" in which:
        qkv = torch.randn(M, 3 * D, device="cuda")
        rel = torch.randn(2 * K + 1, device="cuda") * 0.1
        thr = int(round(args.p * (1 << 24)))
        scale = 1.0 / math.sqrt(D // H)
        amask = torch.zeros(_lib.query("ctr_attn_mask_words", B, K, H), dtype=torch.int32, device="cuda")
        o = torch.empty(M, D, device="cuda")
        mrow, lrow = torch.empty(B * H * K, device="cuda"), torch.empty(B * H * K, device="cuda")
        do = torch.randn(M, D, device="cuda")
        dqkv = torch.empty(M, 3 * D, device="cuda")
        nparts = _lib.query("ctr_attn_bwd_nparts", H, K, D) * B
        drp = torch.empty(nparts, 2 * K + 1, device="cuda")
        fwd = lambda: call("ctr_attn_fwd", ptr(qkv), B, K, H, D, ptr(rel), K, scale, 777, thr, 1.0 / 0.9, ptr(amask),
                           ptr(o), ptr(mrow), ptr(lrow), st)
        bwd = lambda: call("ctr_attn_bwd", ptr(qkv), ptr(o), ptr(do), B, K, H, D, ptr(rel), K, scale, 777, thr,
                           1.0 / 0.9, ptr(amask), ptr(mrow), ptr(lrow), ptr(dqkv), ptr(drp), st)
        tf = timeit(fwd, args.iters)
        tb = timeit(bwd, args.iters)
        print(f"attn_fwd B={B} K={K} H={H} D={D}: {tf * 1e3:.1f} us")
        print(f"attn_bwd B={B} K={K} H={H} D={D}: {tb * 1e3:.1f} us")


if __name__ == "__main__":
    main()
