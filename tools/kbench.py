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
    ap.add_argument("--nobias", action="store_true", help="attn: no positional bias")
    ap.add_argument("--bf16", action="store_true", help="ffn: the amp bf16 kernels (CTR_FFN_BF16); rowgemm: rowgemm_bf")
    ap.add_argument("--norms", action="store_true", help="ffn: the norm-fused backward (ctr_ffn_bwd_norms, as the step)")
    ap.add_argument("--shapes", default="", help="gemm: comma-separated indices of the shape list")
    ap.add_argument("--variant", type=int, default=0, help="gemmig: ctr_gemm_bf16_set_variant")
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
        thr = int(round(args.p * (1 << 16)))
        mask = torch.zeros(_lib.query("ctr_ffn_mask_words", M, FF), dtype=torch.int32, device="cuda")
        y, h, r = torch.empty(M, D, device="cuda"), torch.empty(M, D, device="cuda"), torch.empty(M, device="cuda")
        dh, dx = torch.randn(M, D, device="cuda"), torch.empty(M, D, device="cuda")
        o_b1, o_w2 = FF * D, FF * D + FF
        ld = (o_w2 + D * FF + 3) // 4 * 4
        fl = 1 if args.bf16 else 0
        wbf = torch.empty(3 * FF * D, dtype=torch.bfloat16, device="cuda") if fl else None
        nb = _lib.query("ctr_ffn_slab_rows", M, D, FF, fl)
        slab = torch.zeros(nb, ld, device="cuda")
        fwd = lambda: call("ctr_ffn_fwd", ptr(x), M, D, FF, ptr(W1), ptr(b1), ptr(W2), ptr(b2), ptr(nw), 1e-6, 12345,
                           thr, 1.0 / 0.9, ptr(mask), ptr(y), ptr(h), ptr(r), ptr(wbf), fl, st)
        bwd = lambda: call("ctr_ffn_bwd", ptr(x), ptr(dh), M, D, FF, ptr(W1), ptr(b1), ptr(W2), 12345, thr, 1.0 / 0.9,
                           ptr(mask), ptr(dx), ptr(slab), ld, o_b1, o_w2, ptr(wbf), fl, st)
        if args.norms:
            h1, r1 = torch.randn(M, D, device="cuda"), torch.rand(M, device="cuda") + 0.5
            h2, r2 = torch.randn(M, D, device="cuda"), torch.rand(M, device="cuda") + 0.5
            o = [0, D, D + FF * D, D + FF * D + FF, D + 2 * FF * D + FF, 2 * D + 2 * FF * D + FF]
            ldn = (o[-1] + D + 3) // 4 * 4
            slab = torch.zeros(nb, ldn, device="cuda")
            bwd = lambda: call("ctr_ffn_bwd_norms", ptr(x), ptr(dh), ptr(h2), ptr(r2), ptr(nw), ptr(h1), ptr(r1), ptr(nw),
                               M, D, FF, ptr(W1), ptr(b1), ptr(W2), 12345, thr, 1.0 / 0.9, ptr(mask), ptr(dx), ptr(slab),
                               ldn, *o, ptr(wbf), fl, st)
        tf = timeit(fwd, args.iters)
        tb = timeit(bwd, args.iters)
        print(f"ffn_fwd M={M} D={D} FF={FF}: {tf * 1e3:.1f} us  {4.0 * M * FF * D / tf / 1e9:.1f} TF/s")
        print(f"ffn_bwd M={M} D={D} FF={FF}: {tb * 1e3:.1f} us  {8.0 * M * FF * D / tb / 1e9:.1f} TF/s")
    if "rowgemm" in which:
        rg = "ctr_rowgemm_bf" if args.bf16 else "ctr_rowgemm"     # --bf16: the amp D = 64 row kernels
        x = torch.randn(M, D, device="cuda")
        Win, bin_ = torch.randn(3 * D, D, device="cuda"), torch.randn(3 * D, device="cuda")
        Wout, bout = torch.randn(D, D, device="cuda"), torch.randn(D, device="cuda")
        qkv, o, x1 = torch.empty(M, 3 * D, device="cuda"), torch.randn(M, D, device="cuda"), torch.empty(M, D, device="cuda")
        h1, r1, nw = torch.empty(M, D, device="cuda"), torch.empty(M, device="cuda"), torch.ones(D, device="cuda")
        dh1, do, dq, dx = (torch.randn(M, D, device="cuda"), torch.empty(M, D, device="cuda"),
                           torch.randn(M, 3 * D, device="cuda"), torch.empty(M, D, device="cuda"))
        cases = {
            "qkv": lambda: call(rg, M, D, 3 * D, ptr(x), D, ptr(Win), 1, ptr(qkv), 3 * D, ptr(bin_), None, 0,
                                None, 0, None, None, None, 0.0, st),
            "out+norm": lambda: call(rg, M, D, D, ptr(o), D, ptr(Wout), 1, ptr(x1), D, ptr(bout), None, 0,
                                     ptr(x), D, ptr(nw), ptr(h1), ptr(r1), 1e-6, st),
            "do": lambda: call(rg, M, D, D, ptr(dh1), D, ptr(Wout), 0, ptr(do), D, None, None, 0, None, 0,
                               None, None, None, 0.0, st),
            "dx": lambda: call(rg, M, 3 * D, D, ptr(dq), 3 * D, ptr(Win), 0, ptr(dx), D, None, ptr(dh1), D,
                               None, 0, None, None, None, 0.0, st),
        }
        mb = {"qkv": 4 * M * 4 * D, "out+norm": 4 * M * (5 * D + 1), "do": 8 * M * D, "dx": 4 * M * 5 * D}
        for n, fn in cases.items():
            t = timeit(fn, args.iters)
            print(f"{rg} {n} M={M} D={D}: {t * 1e3:.1f} us  {mb[n] / t / 1e6:.0f} GB/s")
        for no, ni, dy, xx in ((3 * D, D, dq, x), (D, D, dh1, o)):
            rows = _lib.query(rg + "_wgrad_rows", M)
            ld = (no * ni + 64 + no + 3) // 4 * 4
            slab = torch.zeros(rows, ld, device="cuda")
            fn = lambda: call(rg + "_wgrad", ptr(dy), no, ptr(xx), ni, M, no, ni, ptr(slab), ld, no * ni + 64, st)
            t = timeit(fn, args.iters)
            print(f"{rg}_wgrad {no}x{ni} M={M}: {t * 1e3:.1f} us  {4 * M * (no + ni) / t / 1e6:.0f} GB/s")
    if "gemm" in which:        # the QNN MLP's big GEMMs at each split-K factor
        shapes = [(4096, 512, 6400, 0, 1), (4096, 512, 7552, 0, 1), (512, 7552, 4096, 1, 0), (4096, 7552, 512, 0, 0), (512, 6400, 4096, 1, 0), (4096, 6400, 512, 0, 0),
                  (4096, 1152, 512, 0, 0), (4096, 512, 1152, 0, 1), (512, 1152, 4096, 1, 0),
                  (32, 96, 4096, 1, 0), (1, 256, 4096, 1, 0), (1, 32, 4096, 1, 0), (96, 1152, 4096, 1, 0),
                  (256, 512, 4096, 1, 0), (1024, 96, 4096, 1, 0), (32, 96, 245760, 1, 0)]
        if args.shapes:
            shapes = [shapes[int(i)] for i in args.shapes.split(",")]
        for (Mg, Ng, Kg, ta, tb) in shapes:
            Ag = torch.randn((Kg, Mg) if ta else (Mg, Kg), device="cuda")
            Bg = torch.randn((Ng, Kg) if tb else (Kg, Ng), device="cuda")
            Cg = torch.empty(Mg, Ng, device="cuda")
            res = []
            for fl in ((1, 3) if args.bf16 else (0,)):
                for sp in (1, 2, 3, 4, 5, 6, 8, 12):
                    if sp > max(1, Kg // 64):
                        continue
                    ws = torch.empty(sp * Mg * Ng + 16, device="cuda")
                    fn = lambda: call("ctr_gemm_ex", Mg, Ng, Kg, ptr(Ag), Ag.shape[1], ta, ptr(Bg), Bg.shape[1], tb,
                                      ptr(Cg), Ng, None, sp, ptr(ws), None, fl, st)
                    t = timeit(fn, args.iters)
                    res.append(f"f{fl}s{sp}:{2.0 * Mg * Ng * Kg / t / 1e9:.0f}")
            torch.backends.cuda.matmul.allow_tf32 = False      # the library's fp32 path, for reference
            a_op, b_op = (Ag.t() if ta else Ag), (Bg.t() if tb else Bg)
            if args.bf16:
                a_op, b_op = a_op.bfloat16(), b_op.bfloat16()
                Cb = torch.empty(Mg, Ng, device="cuda", dtype=torch.bfloat16)
                t = timeit(lambda: torch.matmul(a_op, b_op, out=Cb), args.iters)
            else:
                t = timeit(lambda: torch.matmul(a_op, b_op, out=Cg), args.iters)
            res.append(f"torch:{2.0 * Mg * Ng * Kg / t / 1e9:.0f}")
            print(f"gemm M={Mg} N={Ng} K={Kg} ta={ta} tb={tb} TF/s: " + " ".join(res))
    if "gemmbf" in which:      # ctr_gemm_bf16 (bf16 operands in HBM) on the QNN MLP's three big products, per kernel form
        for var in (1, 2, 3):      # ctr_gemm_bf16_set_variant: two-stage 128 x 128, ring 256 x 128, ring 128 x 128
            _lib.query("ctr_gemm_bf16_set_variant", var)
            for (Mg, Ng, Kg, ta, tb) in [(4096, 512, 7552, 0, 1), (512, 7552, 4096, 1, 0), (4096, 7552, 512, 0, 0)]:
                Ag = torch.randn((Kg, Mg) if ta else (Mg, Kg), device="cuda").bfloat16()
                Bg = torch.randn((Ng, Kg) if tb else (Kg, Ng), device="cuda").bfloat16()
                Cg = torch.empty(Mg, Ng, device="cuda")
                res = []
                for sp in (1, 2, 4, 8):
                    ws = torch.empty(sp * Mg * Ng + 16, device="cuda")
                    fn = lambda: call("ctr_gemm_bf16", Mg, Ng, Kg, ptr(Ag), Ag.shape[1], ta, ptr(Bg), Bg.shape[1], tb,
                                      ptr(Cg), Ng, None, sp, ptr(ws), None, st)
                    t = timeit(fn, args.iters)
                    res.append(f"s{sp}:{2.0 * Mg * Ng * Kg / t / 1e9:.0f}({t * 1e3:.0f}us)")
                print(f"v{var} gemm_bf16 M={Mg} N={Ng} K={Kg} ta={ta} tb={tb} TF/s: " + " ".join(res))
            # the input grad as the step runs it: bf16 [dz | dinter] output split at column 6400
            Mg, Ng, Kg, nc = 4096, 7552, 512, 6400
            Ag = torch.randn(Mg, Kg, device="cuda").bfloat16()
            Bg = torch.randn(Kg, Ng, device="cuda").bfloat16()
            C1 = torch.empty(Mg, nc, device="cuda", dtype=torch.bfloat16)
            C2 = torch.empty(Mg, Ng - nc, device="cuda", dtype=torch.bfloat16)
            seg = _lib.GemmSeg(C2=ptr(C2), ldc2=Ng - nc, nc=nc)
            fn = lambda: call("ctr_gemm_bf16_ex", Mg, Ng, Kg, ptr(Ag), Kg, 0, ptr(Bg), Ng, 0, ptr(C1), nc, None, 1, None,
                              seg, 1, st)
            t = timeit(fn, args.iters)
            print(f"v{var} gemm_bf16 out bf16 + C2 M={Mg} N={Ng} K={Kg}: {2.0 * Mg * Ng * Kg / t / 1e9:.0f} TF/s "
                  f"({t * 1e3:.0f}us)")
        _lib.query("ctr_gemm_bf16_set_variant", 0)
    if "gemmig" in which:      # the QNN MLP's input grad alone (bf16 [dz | dinter] out), one kernel form: PMC passes
        _lib.query("ctr_gemm_bf16_set_variant", args.variant)
        Mg, Ng, Kg, nc = 4096, 7552, 512, 6400
        Ag = torch.randn(Mg, Kg, device="cuda").bfloat16()
        Bg = torch.randn(Kg, Ng, device="cuda").bfloat16()
        C1 = torch.empty(Mg, nc, device="cuda", dtype=torch.bfloat16)
        C2 = torch.empty(Mg, Ng - nc, device="cuda", dtype=torch.bfloat16)
        seg = _lib.GemmSeg(C2=ptr(C2), ldc2=Ng - nc, nc=nc)
        fn = lambda: call("ctr_gemm_bf16_ex", Mg, Ng, Kg, ptr(Ag), Kg, 0, ptr(Bg), Ng, 0, ptr(C1), nc, None, 1, None,
                          seg, 1, st)
        t = timeit(fn, args.iters)
        print(f"v{args.variant} input grad: {2.0 * Mg * Ng * Kg / t / 1e9:.0f} TF/s ({t * 1e3:.0f}us)")
        _lib.query("ctr_gemm_bf16_set_variant", 0)
    if "attn" in which or "attnbf" in which:
        qkv = torch.randn(M, 3 * D, device="cuda")
        rel = torch.randn(2 * K + 1, device="cuda") * 0.1
        thr = int(round(args.p * (1 << 16)))
        scale = 1.0 / math.sqrt(D // H)
        amask = torch.zeros(_lib.query("ctr_attn_mask_words", B, K, H), dtype=torch.int32, device="cuda")
        o = torch.empty(M, D, device="cuda")
        mrow, lrow = torch.empty(B * H * K, device="cuda"), torch.empty(B * H * K, device="cuda")
        do = torch.randn(M, D, device="cuda")
        dqkv = torch.empty(M, 3 * D, device="cuda")
        nparts = _lib.query("ctr_attn_bwd_nparts", H, K, D) * B
        drp = torch.empty(nparts, 2 * K + 1, device="cuda")
        rel = None if args.nobias else rel
        fwd = lambda: call("ctr_attn_fwd", ptr(qkv), B, K, H, D, ptr(rel), K, scale, 777, thr, 1.0 / 0.9, ptr(amask),
                           ptr(o), ptr(mrow), ptr(lrow), st)
        bwd = lambda: call("ctr_attn_bwd", ptr(qkv), ptr(o), ptr(do), B, K, H, D, ptr(rel), K, scale, 777, thr,
                           1.0 / 0.9, ptr(amask), ptr(mrow), ptr(lrow), ptr(dqkv), ptr(drp), st)
        for generic in ((0, 1) if "attn" in which else ()):   # packed (where it applies), then generic
            _lib.query("ctr_attn_set_generic", generic)
            tf = timeit(fwd, args.iters)
            tb = timeit(bwd, args.iters)
            print(f"attn_fwd{' generic' if generic else ''} B={B} K={K} H={H} D={D}: {tf * 1e3:.1f} us")
            print(f"attn_bwd{' generic' if generic else ''} B={B} K={K} H={H} D={D}: {tb * 1e3:.1f} us")
        _lib.query("ctr_attn_set_generic", 0)
    if "attnbf" in which and _lib.query("ctr_attn_bf_ok", K, H, D):
        # the amp bf16-MFMA attention (attn_mf.hip)
        nparts = _lib.query("ctr_attn_bwd_bf_nparts", H) * B
        drp = torch.empty(nparts, 2 * K + 1, device="cuda")
        fwd = lambda: call("ctr_attn_fwd_bf", ptr(qkv), B, K, H, D, ptr(rel), K, scale, 777, thr, 1.0 / 0.9,
                           ptr(amask), ptr(o), ptr(mrow), ptr(lrow), st)
        bwd = lambda: call("ctr_attn_bwd_bf", ptr(qkv), ptr(o), ptr(do), B, K, H, D, ptr(rel), K, scale, 777, thr,
                           1.0 / 0.9, ptr(amask), ptr(mrow), ptr(lrow), ptr(dqkv), ptr(drp), st)
        tf = timeit(fwd, args.iters)
        tb = timeit(bwd, args.iters)
        print(f"attn_fwd_bf B={B} K={K} H={H} D={D}: {tf * 1e3:.1f} us")
        print(f"attn_bwd_bf B={B} K={K} H={H} D={D}: {tb * 1e3:.1f} us")


if __name__ == "__main__":
    main()
