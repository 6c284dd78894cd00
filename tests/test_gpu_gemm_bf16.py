"""GPU parity of the bf16-operand GEMM (ctr_gemm_bf16: glds-staged LDS tiles, swizzled k-contiguous and
transposed-read k-major layouts) against a torch fp64 product of the same bf16-rounded operands.  The
kernel's only freedom is the fp32 accumulation order, so the bound is fp32 rounding (rel 1e-5)."""
import pytest
import torch

from test_gpu_kernels import _lib, ptr, rel, stream

pytestmark = pytest.mark.gpu


def bf16_image(L, x):
    """ctr_to_bf16 of a fp32 matrix (the product path's converter), checked against torch's RNE cast."""
    out = torch.empty(x.shape, dtype=torch.bfloat16, device="cuda")
    L.call("ctr_to_bf16", ptr(x), x.shape[1], x.shape[0], x.shape[1], ptr(out), x.shape[1], stream())
    assert torch.equal(out, x.bfloat16())
    return out


@pytest.mark.parametrize("M,N,K,ta,tb", [(4096, 512, 7552, 0, 1), (512, 7552, 4096, 1, 0), (4096, 7552, 512, 0, 0),
                                         (300, 136, 192, 0, 1), (136, 264, 128, 1, 0), (72, 200, 64, 1, 1),
                                         (257, 88, 320, 0, 0),
                                         # the ring kernel (M >= 256): every operand layout, one or two k-steps per
                                         # tile (epilogue stores inside the counted-wait window), row / column tails
                                         (520, 264, 192, 1, 1), (1024, 1000, 64, 0, 1), (600, 520, 128, 0, 0),
                                         (384, 2048, 64, 1, 0), (2000, 7552, 512, 0, 0)])
@pytest.mark.parametrize("splits", [1, 3])
@pytest.mark.parametrize("variant", [0, 1, 2, 3])     # automatic, two-stage, ring 256 x 128, ring 128 x 128
def test_gemm_bf16_vs_torch(M, N, K, ta, tb, splits, variant):
    L = _lib()
    L.query("ctr_gemm_bf16_set_variant", variant)
    assert L.query("ctr_gemm_bf16_ok", M, N, K, M if ta else K, ta, K if tb else N, tb, splits)
    g = torch.Generator(device="cuda").manual_seed(M * 13 + N + K)
    A = torch.randn((K, M) if ta else (M, K), device="cuda", generator=g)
    B = torch.randn((N, K) if tb else (K, N), device="cuda", generator=g)
    Ab, Bb = bf16_image(L, A), bf16_image(L, B)
    C = torch.full((M, N), float("nan"), device="cuda")
    ws = torch.empty(splits * M * N + 16, device="cuda")
    L.call("ctr_gemm_bf16", M, N, K, ptr(Ab), Ab.shape[1], ta, ptr(Bb), Bb.shape[1], tb, ptr(C), N, None, splits,
           ptr(ws), None, stream())
    a64 = (Ab.t() if ta else Ab).double()
    b64 = (Bb.t() if tb else Bb).double()
    ref = a64 @ b64
    assert torch.isfinite(C).all()
    assert rel(C.double(), ref) < 1e-5
    # deterministic: a second call writes the same bits (a staged tile read before its DMA landed would not)
    C2 = torch.full_like(C, float("nan"))
    L.call("ctr_gemm_bf16", M, N, K, ptr(Ab), Ab.shape[1], ta, ptr(Bb), Bb.shape[1], tb, ptr(C2), N, None, splits,
           ptr(ws), None, stream())
    L.query("ctr_gemm_bf16_set_variant", 0)
    assert torch.equal(C, C2)


def test_gemm_bf16_epilogue_and_c2():
    """bias + ReLU + pre-activation store (the MLP forward's epilogue) and the C2 result segment
    ([dz | dinter] = dcur W0, split at column nc)."""
    L = _lib()
    M, N, K = 520, 384, 256
    g = torch.Generator(device="cuda").manual_seed(5)
    A = torch.randn(M, K, device="cuda", generator=g)
    W = torch.randn(N, K, device="cuda", generator=g)
    bias = torch.randn(N, device="cuda", generator=g)
    Ab, Wb = bf16_image(L, A), bf16_image(L, W)
    C, pre = torch.empty(M, N, device="cuda"), torch.empty(M, N, device="cuda")
    epi = L.GemmEpi(bias=ptr(bias), act=1, pre=ptr(pre))
    L.call("ctr_gemm_bf16", M, N, K, ptr(Ab), K, 0, ptr(Wb), K, 1, ptr(C), N, epi, 1, None, None, stream())
    z = Ab.double() @ Wb.double().t() + bias.double()
    assert rel(pre.double(), z) < 1e-5
    assert rel(C.double(), z.clamp_min(0)) < 1e-5
    nc = 256
    C1 = torch.empty(M, nc, device="cuda")
    C2 = torch.empty(M, N - nc, device="cuda")
    seg = L.GemmSeg(C2=ptr(C2), ldc2=N - nc, nc=nc)
    Wk = bf16_image(L, W.t().contiguous())      # B stored (K, N): the dA product's W0 layout
    L.call("ctr_gemm_bf16", M, N, K, ptr(Ab), K, 0, ptr(Wk), N, 0, ptr(C1), nc, None, 1, None, seg, stream())
    full = Ab.double() @ Wk.double()
    assert rel(C1.double(), full[:, :nc]) < 1e-5
    assert rel(C2.double(), full[:, nc:]) < 1e-5


@pytest.mark.parametrize("M,N,K,nc", [(4096, 7552, 512, 6400), (520, 384, 256, 256), (257, 88, 128, 0)])
def test_gemm_bf16_out_bf16_is_rounded_fp32(M, N, K, nc):
    """CTR_GEMM_OUT_BF16 (the QNN MLP's input grad [dz | dinter] under amp): every element is the RNE bf16 of
    the fp32 result the same call writes without the flag -- same accumulation, only the store differs --
    including the C2 segment and a row tail (M % 128 != 0)."""
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = torch.randn(M, K, device="cuda", generator=g)
    Wk = torch.randn(K, N, device="cuda", generator=g)
    Ab, Wb = bf16_image(L, A), bf16_image(L, Wk)
    n2 = N - nc
    seg = L.GemmSeg(C2=None, ldc2=0, nc=N)
    C32 = torch.empty(M, N, device="cuda")
    L.call("ctr_gemm_bf16_ex", M, N, K, ptr(Ab), K, 0, ptr(Wb), N, 0, ptr(C32), N, None, 1, None, None, 0, stream())
    C1 = torch.empty(M, nc if nc else N, dtype=torch.bfloat16, device="cuda")
    C2 = torch.empty(M, max(n2, 1), dtype=torch.bfloat16, device="cuda")
    if nc:
        seg = L.GemmSeg(C2=ptr(C2), ldc2=n2, nc=nc)
    L.call("ctr_gemm_bf16_ex", M, N, K, ptr(Ab), K, 0, ptr(Wb), N, 0, ptr(C1), C1.shape[1], None, 1, None,
           seg if nc else None, 1, stream())
    ref = C32.bfloat16()
    if nc:
        assert torch.equal(C1, ref[:, :nc]) and torch.equal(C2, ref[:, nc:])
    else:
        assert torch.equal(C1, ref)
    assert rel(C32.double(), Ab.double() @ Wb.double()) < 1e-5


def test_gemm_bf16_epilogue_stays_inside_n():
    """N far below the 128-column tile (the tiny configs' MLP: N = 32 / 40): the epilogue's pre-activation
    stores and aux / add reads stop at column N -- a guard region past the last row stays untouched."""
    L = _lib()
    M, N, K = 300, 40, 128
    g = torch.Generator(device="cuda").manual_seed(7)
    A = torch.randn(M, K, device="cuda", generator=g)
    W = torch.randn(N, K, device="cuda", generator=g)
    bias = torch.randn(N, device="cuda", generator=g)
    Ab, Wb = bf16_image(L, A), bf16_image(L, W)
    C = torch.full((M + 8, N), 7.0, device="cuda")
    pre = torch.full((M + 8, N), 7.0, device="cuda")
    epi = L.GemmEpi(bias=ptr(bias), act=1, pre=ptr(pre))
    L.call("ctr_gemm_bf16", M, N, K, ptr(Ab), K, 0, ptr(Wb), K, 1, ptr(C), N, epi, 1, None, None, stream())
    z = Ab.double() @ Wb.double().t() + bias.double()
    assert rel(pre[:M].double(), z) < 1e-5
    assert rel(C[:M].double(), z.clamp_min(0)) < 1e-5
    assert (pre[M:] == 7.0).all() and (C[M:] == 7.0).all()
