"""fp32 vs bf16-operand GEMM (ctr_gemm_ex) on the QNN MLP shapes of the cfg2 step (B = 4096, MLP input
7552 = 6400 + 1152, hidden 512 / 256): forward, dX and dW products, with the engine's split-K choice.
Not part of the product.   python tools/gemm_bench.py [--iters 20]"""
import argparse
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "toss-next-ctr-prediction_amd"))

import torch  # noqa: E402

from tossctr import _lib  # noqa: E402
from tossctr.engine import Engine  # noqa: E402


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
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    st = torch.cuda.current_stream().cuda_stream
    shapes = [("fwd  z@W0^T", 4096, 512, 7552, 0, 1), ("dW0 = dh^T [z|i]", 512, 7552, 4096, 1, 0),
              ("dX = dh W0", 4096, 7552, 512, 0, 0), ("fwd h0@W1^T", 4096, 256, 512, 0, 1),
              ("inter = quad Vfull", 4096, 1152, 96, 0, 0)]
    for name, M, N, K, ta, tb in shapes:
        A = torch.randn((K, M) if ta else (M, K), device="cuda")
        B = torch.randn((N, K) if tb else (K, N), device="cuda")
        C = torch.empty(M, N, device="cuda")
        tiles = Engine._tiles(M, N)
        sp = Engine._split_factor(M, N, K, 256 if not ta else 64) if K >= 512 and tiles < 256 else 1
        ws = torch.empty(max(1, sp * M * N), device="cuda")
        for flags in (0, 1):
            f = lambda: _lib.call("ctr_gemm_ex", M, N, K, A.data_ptr(), A.shape[1], ta, B.data_ptr(), B.shape[1], tb,  # noqa: E731
                                  C.data_ptr(), N, None, sp, ws.data_ptr(), None, flags, st)
            ms = timeit(f, args.iters)
            print(f"{name:20s} M={M:5d} N={N:5d} K={K:5d} splits={sp:2d} {'bf16' if flags else 'fp32'}: "
                  f"{ms * 1e3:8.1f} us  {2.0 * M * N * K / ms / 1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
