"""Per-kernel microbenchmarks on the GPU box: the step's GEMM shapes (TFLOP/s, GB/s) and HBM copy
calibration.  Not part of the product; used to decide what to tune next."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "toss-next-ctr-prediction_amd"))

import torch  # noqa: E402

from tossctr import _lib  # noqa: E402
from tossctr._lib import GemmEpi  # noqa: E402


def ptr(t, e=0):
    return t.data_ptr() + e * t.element_size() if t is not None else None


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def gemm_case(name, M, N, K, ta, tb, epi=None, splits=1):
    A = torch.randn((K, M) if ta else (M, K), device="cuda")
    B = torch.randn((N, K) if tb else (K, N), device="cuda")
    C = torch.empty(M, N, device="cuda")
    ws = torch.empty(max(1, splits * M * N), device="cuda")
    aux = torch.randn(M, N, device="cuda")
    e = None
    if epi == "gelu":
        bias = torch.randn(N, device="cuda")
        pre = torch.empty(M, N, device="cuda")
        e = GemmEpi(bias=ptr(bias), act=2, pre=ptr(pre), drop_key=123, drop_thresh=1677722, drop_scale=1.1111)
    elif epi == "dgelu":
        e = GemmEpi(dact=2, aux=ptr(aux), drop_key=123, drop_thresh=1677722, drop_scale=1.1111)
    st = torch.cuda.current_stream().cuda_stream
    ms = timeit(lambda: _lib.call("ctr_gemm", M, N, K, ptr(A), A.shape[1], ta, ptr(B), B.shape[1], tb, ptr(C), N, e,
                                  splits, ptr(ws), st))
    flops = 2.0 * M * N * K
    byts = 4.0 * (M * K + K * N + M * N * (3 if epi else 1))
    print(f"{name:34s} M={M:7d} N={N:5d} K={K:7d} s={splits:3d}: {ms*1e3:8.1f} us  "
          f"{flops/ms/1e9:7.1f} TF/s  {byts/ms/1e6:7.1f} GB/s", flush=True)


def main():
    n = 1 << 28
    x = torch.empty(n, device="cuda")
    y = torch.empty(n, device="cuda")
    ms = timeit(lambda: y.copy_(x))
    print(f"torch copy 1 GiB: {ms*1e3:.1f} us = {2*4*n/ms/1e6:.1f} GB/s", flush=True)
    B, K_, D, FF = 4096, 60, 32, 384
    M = B * K_
    gemm_case("qkv fwd", M, 96, 32, 0, 1)
    gemm_case("ffn1 fwd (gelu+drop epi)", M, FF, D, 0, 1, "gelu")
    gemm_case("ffn2 fwd", M, D, FF, 0, 1)
    gemm_case("ffn dact bwd (dgelu epi)", M, FF, D, 0, 0, "dgelu")
    gemm_case("ffn1 dX bwd", M, D, FF, 0, 0)
    gemm_case("ffn2 dW (split)", D, FF, M, 1, 0, None, 128)
    gemm_case("ffn1 dW (split)", FF, D, M, 1, 0, None, 128)
    gemm_case("mlp0a fwd z@W0a^T", B, 512, 6400, 0, 1)
    gemm_case("mlp0a dX", B, 6400, 512, 0, 0)
    gemm_case("mlp0a dW (split)", 512, 6400, B, 1, 0, None, 8)
    gemm_case("qnn A = z@Ucat", B * 200, 96, 32, 0, 0)
    gemm_case("square 4096", 4096, 4096, 4096, 0, 0)


if __name__ == "__main__":
    main()
