"""Isolated launches of the cfg2 encoder-layer attention kernels (amp bf16, attn_mf.hip): the fused layer
forward (ctr_attn_layer_fwd_bf) and the attention backward with the out-projection's input grad inside
(ctr_attn_bwd_bf_oproj), B = 4096, K = 60, H = 8, D = 32, dropout 0.1, positional bias -- for A/B timing of
kernel variants (CTR_LIB_PATH) and rocprofv3 passes.  Not part of the product.

    python tools/attnbench.py [--iters 20] [--B 4096] [--K 60]
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
from tossctr.rng import drop_args  # noqa: E402


def ptr(t):
    return t.data_ptr() if t is not None else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--K", type=int, default=60)
    args = ap.parse_args()
    B, K, H, D = args.B, args.K, 8, 32
    M = B * K
    g = torch.Generator(device="cuda").manual_seed(0)
    st = torch.cuda.current_stream().cuda_stream
    x = torch.randn(M, D, device="cuda", generator=g)
    w_in = torch.randn(3 * D, D, device="cuda", generator=g) / math.sqrt(D)
    b_in = torch.randn(3 * D, device="cuda", generator=g) * 0.1
    w_out = torch.randn(D, D, device="cuda", generator=g) / math.sqrt(D)
    b_out = torch.randn(D, device="cuda", generator=g) * 0.1
    nw1 = 1 + 0.1 * torch.randn(D, device="cuda", generator=g)
    rel = torch.randn(2 * K + 1, H, device="cuda", generator=g)
    relmean = torch.empty(2 * K + 1, device="cuda")
    key, thr, sc = drop_args((3 << 32) | 1, 1, 0.1, True)
    mask = torch.zeros(_lib.query("ctr_attn_mask_words", B, K, H), dtype=torch.int32, device="cuda")
    qkv, o = torch.empty(M, 3 * D, device="cuda"), torch.empty(M, D, device="cuda")
    mrow, lrow = torch.empty(B * H * K, device="cuda"), torch.empty(B * H * K, device="cuda")
    h1, r1, x1 = torch.empty(M, D, device="cuda"), torch.empty(M, device="cuda"), torch.empty(M, D, device="cuda")
    scale = float(torch.tensor(math.sqrt(1.0 / (D // H)), dtype=torch.float32))
    fwd = lambda: call("ctr_attn_layer_fwd_bf", ptr(x), B, K, H, D, ptr(w_in), ptr(b_in), ptr(rel), ptr(relmean),  # noqa: E731
                       K, scale, key, thr, sc, ptr(mask), ptr(w_out), ptr(b_out), ptr(nw1), 1e-6, ptr(qkv), ptr(o),
                       ptr(mrow), ptr(lrow), ptr(h1), ptr(r1), ptr(x1), st)
    dh1 = torch.randn(M, D, device="cuda", generator=g)
    dqkv = torch.empty(M, 3 * D, device="cuda")
    nparts = _lib.query("ctr_attn_bwd_bf_nparts", H) * B
    drel = torch.empty(nparts * (2 * K + 1), device="cuda")
    bwd = lambda: call("ctr_attn_bwd_bf_oproj", ptr(qkv), ptr(o), ptr(dh1), ptr(w_out), B, K, H, D, ptr(relmean), K,  # noqa: E731
                       scale, key, thr, sc, ptr(mask), ptr(mrow), ptr(lrow), ptr(dqkv), ptr(drel), st)
    for name, fn in (("layer_fwd", fwd), ("attn_bwd_oproj", bwd)):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        print(f"{name} B={B} K={K}: {a.elapsed_time(b) / args.iters * 1e3:.1f} us", flush=True)
    print("checksum", float(dqkv.double().abs().sum()), float(x1.double().abs().sum()))


if __name__ == "__main__":
    main()
