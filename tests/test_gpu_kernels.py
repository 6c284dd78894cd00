"""GPU unit parity of the HIP kernels (called through the C-ABI) against plain torch fp32 references."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _lib():
    from tossctr import _lib
    return _lib


def ptr(t, e=0):
    return t.data_ptr() + e * t.element_size() if t is not None else None


def stream():
    return torch.cuda.current_stream().cuda_stream


def rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("M,N,K,ta,tb", [(300, 96, 32, 0, 1), (257, 384, 32, 0, 1), (130, 32, 384, 0, 1),
                                         (64, 512, 7552, 0, 1), (384, 32, 5000, 1, 0), (33, 70, 19, 1, 1),
                                         (1, 32, 4096, 1, 0), (4096, 1, 256, 0, 1), (200, 130, 64, 0, 0)])
@pytest.mark.parametrize("splits", [1, 7])
def test_gemm_vs_torch(M, N, K, ta, tb, splits):
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N)
    A = torch.randn((K, M) if ta else (M, K), device="cuda", generator=g)
    B = torch.randn((N, K) if tb else (K, N), device="cuda", generator=g)
    C = torch.empty(M, N, device="cuda")
    ws = torch.empty(splits * M * N + 16, device="cuda")
    L.call("ctr_gemm", M, N, K, ptr(A), A.shape[1], ta, ptr(B), B.shape[1], tb, ptr(C), N, None, splits, ptr(ws),
           stream())
    ref = (A.t() if ta else A).double() @ (B.t() if tb else B).double()
    assert rel(C.double(), ref) < 1e-5


@pytest.mark.parametrize("M,N,K,ta,tb", [(300, 96, 32, 0, 1), (257, 384, 45, 0, 1), (130, 32, 384, 0, 1),
                                         (64, 512, 7552, 0, 1), (384, 32, 5000, 1, 0), (33, 70, 19, 1, 1),
                                         (1, 32, 4096, 1, 0), (4096, 1, 256, 0, 1), (200, 130, 64, 0, 0),
                                         (4096, 512, 7552, 0, 1), (512, 7552, 4096, 1, 0), (4096, 7552, 512, 0, 0)])
@pytest.mark.parametrize("splits", [1, 7])
def test_gemm_bf16_vs_torch(M, N, K, ta, tb, splits):
    """ctr_gemm_ex(CTR_GEMM_BF16) -- amp: bf16 -- against the fp64 product of the bf16-ROUNDED operands
    (torch's round-to-nearest-even .bfloat16()): bf16 x bf16 products are exact in fp32, so only the fp32
    accumulation order separates them (1e-5).  Shapes include the QNN MLP's forward / dW / dX."""
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + 1)
    A = torch.randn((K, M) if ta else (M, K), device="cuda", generator=g)
    B = torch.randn((N, K) if tb else (K, N), device="cuda", generator=g)
    C = torch.empty(M, N, device="cuda")
    ws = torch.empty(splits * M * N + 16, device="cuda")
    L.call("ctr_gemm_ex", M, N, K, ptr(A), A.shape[1], ta, ptr(B), B.shape[1], tb, ptr(C), N, None, splits, ptr(ws),
           None, 1, stream())
    Ab, Bb = A.bfloat16().double(), B.bfloat16().double()
    ref = (Ab.t() if ta else Ab) @ (Bb.t() if tb else Bb)
    assert rel(C.double(), ref) < 1e-5


def test_gemm_bf16_epilogues_and_segments():
    """bf16 operands under the fused epilogues the model uses (bias + ReLU + dropout with the pre-activation
    stored; residual + RMSNorm) and the [z | inter] operand / result segments of the QNN MLP."""
    L = _lib()
    from tossctr.rng import drop_args
    M, N, K, kc = 700, 384, 200, 128
    g = torch.Generator(device="cuda").manual_seed(5)
    A1 = torch.randn(M, kc, device="cuda", generator=g)
    A2 = torch.randn(M, K - kc, device="cuda", generator=g)
    W = torch.randn(N, K, device="cuda", generator=g) * 0.1
    b = torch.randn(N, device="cuda", generator=g)
    out, pre = torch.empty(M, N, device="cuda"), torch.empty(M, N, device="cuda")
    dk = drop_args(77, 3, 0.2, True)
    epi = L.GemmEpi(bias=ptr(b), act=1, pre=ptr(pre), drop_key=dk[0], drop_thresh=dk[1], drop_scale=dk[2])
    L.call("ctr_gemm_ex", M, N, K, ptr(A1), kc, 0, ptr(W), K, 1, ptr(out), N, epi, 1, None,
           L.GemmSeg(A2=ptr(A2), lda2=K - kc, ka=kc), 1, stream())
    Ab = torch.cat([A1, A2], 1).bfloat16().double()
    pre_ref = Ab @ W.bfloat16().double().t() + b.double()
    assert rel(pre.double(), pre_ref) < 1e-5
    ref_relu = torch.relu(pre_ref)
    kept = out != 0
    assert rel(out.double()[kept], (ref_relu * dk[2])[kept]) < 1e-5
    D = 32
    W2 = torch.randn(D, N, device="cuda", generator=g) * 0.05
    resid = torch.randn(M, D, device="cuda", generator=g)
    nw = torch.rand(D, device="cuda", generator=g) + 0.5
    y, h, r = torch.empty(M, D, device="cuda"), torch.empty(M, D, device="cuda"), torch.empty(M, device="cuda")
    epi2 = L.GemmEpi(resid=ptr(resid), ld_resid=D, norm_w=ptr(nw), norm_h=ptr(h), norm_r=ptr(r), norm_eps=1e-6)
    L.call("ctr_gemm_ex", M, D, N, ptr(out), N, 0, ptr(W2), N, 1, ptr(y), D, epi2, 1, None, None, 1, stream())
    h_ref = resid.double() + out.bfloat16().double() @ W2.bfloat16().double().t()
    y_ref = nw.double() * h_ref * torch.rsqrt(h_ref.pow(2).mean(-1, keepdim=True) + 1e-6)
    assert rel(h.double(), h_ref) < 1e-5 and rel(y.double(), y_ref) < 1e-5


def test_gemm_epilogues():
    L = _lib()
    M, N, K = 517, 384, 32
    x = torch.randn(M, K, device="cuda")
    W = torch.randn(N, K, device="cuda") * 0.2
    b = torch.randn(N, device="cuda")
    out = torch.empty(M, N, device="cuda")
    pre = torch.empty(M, N, device="cuda")
    epi = L.GemmEpi(bias=ptr(b), act=2, pre=ptr(pre))
    L.call("ctr_gemm", M, N, K, ptr(x), K, 0, ptr(W), K, 1, ptr(out), N, epi, 1, None, stream())
    a_ref = x @ W.t() + b
    assert rel(pre, a_ref) < 1e-5
    assert rel(out, torch.nn.functional.gelu(a_ref)) < 1e-5
    # fused residual + RMSNorm, N = D = 32
    D = 32
    W2 = torch.randn(D, N, device="cuda") * 0.05
    b2 = torch.randn(D, device="cuda")
    res = torch.randn(M, D, device="cuda")
    w = torch.rand(D, device="cuda") + 0.5
    y, h, r = (torch.empty(M, D, device="cuda"), torch.empty(M, D, device="cuda"), torch.empty(M, device="cuda"))
    epi = L.GemmEpi(bias=ptr(b2), resid=ptr(res), ld_resid=D, norm_w=ptr(w), norm_h=ptr(h), norm_r=ptr(r),
                    norm_eps=1e-6)
    L.call("ctr_gemm", M, D, N, ptr(out), N, 0, ptr(W2), N, 1, ptr(y), D, epi, 1, None, stream())
    h_ref = res + (out @ W2.t() + b2)
    y_ref = w * h_ref * torch.rsqrt(h_ref.pow(2).mean(-1, keepdim=True) + 1e-6)
    assert rel(h, h_ref) < 1e-5 and rel(y, y_ref) < 1e-5
    # backward epilogue: relu' x dropout mask
    aux = torch.randn(M, N, device="cuda")
    dy = torch.randn(M, D, device="cuda")
    dgrad = torch.empty(M, N, device="cuda")
    from tossctr.rng import drop_args
    key, th, sc = drop_args(99, 5, 0.2, True)
    epi = L.GemmEpi(dact=1, aux=ptr(aux), drop_key=key, drop_thresh=th, drop_scale=sc)
    L.call("ctr_gemm", M, N, D, ptr(dy), D, 0, ptr(W2), N, 0, ptr(dgrad), N, epi, 1, None, stream())
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import rng as orng
    keep = torch.from_numpy(orng.keep_mask(99, 5, 0.2, (M, N))).cuda()
    ref = (dy @ W2) * keep.float() * sc * (aux > 0).float()
    assert rel(dgrad, ref) < 1e-5


@pytest.mark.parametrize("n,width,kmax,kbits", [(5000, 24, 700, 10),
                                                 # > 2M keys: the run-length block counts scanned once first (scan.h)
                                                 (3_000_017, 4, 1_500_000, 21)])
def test_rowgrad_dedup_matches_numpy(n, width, kmax, kbits):
    L = _lib()
    rng = np.random.default_rng(n)
    keys = rng.integers(0, kmax, n).astype(np.uint32)
    keys[rng.random(n) < 0.05] = 0xFFFFFFFF
    vals = rng.standard_normal((n, width)).astype(np.float32)
    kt = torch.from_numpy(keys.view(np.int32)).cuda()
    vt = torch.from_numpy(vals).cuda()
    uk = torch.empty(n, dtype=torch.int32, device="cuda")
    ug = torch.empty(n, width, device="cuda")
    nu = torch.zeros(1, dtype=torch.int32, device="cuda")
    wsz = L.query("ctr_rowgrad_ws_size", n)
    ws = torch.empty(wsz, dtype=torch.uint8, device="cuda")
    L.call("ctr_rowgrad", ptr(kt), ptr(vt), n, width, width, kbits, ptr(uk), ptr(ug), ptr(nu), ptr(ws), wsz, stream())
    torch.cuda.synchronize()
    u = int(nu.item())
    got_k = uk[:u].cpu().numpy().view(np.uint32)
    ref_k = np.unique(keys)
    assert np.array_equal(got_k, ref_k)
    ref = np.zeros((len(ref_k), width))
    pos = np.searchsorted(ref_k, keys)
    np.add.at(ref, pos, vals.astype(np.float64))
    ref[ref_k == 0xFFFFFFFF] = 0.0          # the dropped (pad) group is not summed
    assert np.abs(ug[:u].cpu().numpy() - ref).max() < 1e-4
    # bitwise reproducible
    ug2 = torch.empty_like(ug)
    L.call("ctr_rowgrad", ptr(kt), ptr(vt), n, width, width, kbits, ptr(uk), ptr(ug2), ptr(nu), ptr(ws), wsz, stream())
    assert torch.equal(ug[:u], ug2[:u])


@pytest.mark.parametrize("cap", [1000, 3_000_000])
def test_shard_offsets_scan(cap):
    """ctr_shard_offsets: the exclusive scan of the keys' table widths (scan.h), in one pass for <= 2M words and
    with the block sums scanned once first beyond."""
    L = _lib()
    rng = np.random.default_rng(cap)
    lbase = np.array([0, 1000, 5000, 9000], np.uint32)
    dims = np.array([3, 17, 64, 1], np.int32)
    keys = rng.integers(0, 10000, cap).astype(np.uint32)
    width = dims[np.searchsorted(lbase, keys, side="right") - 1].astype(np.int64)
    ref = np.concatenate([[0], np.cumsum(width)]).astype(np.uint32)
    kt = torch.from_numpy(keys.view(np.int32)).cuda()
    lb = torch.from_numpy(lbase.view(np.int32)).cuda()
    dm = torch.from_numpy(dims).cuda()
    off = torch.full((cap + 1,), -1, dtype=torch.int32, device="cuda")
    wsz = L.query("ctr_shard_offsets_ws_size", cap)
    ws = torch.empty(wsz, dtype=torch.uint8, device="cuda")
    L.call("ctr_shard_offsets", ptr(kt), None, cap, cap, 0xFFFFFFFF, ptr(lb), ptr(dm), 4, ptr(off), 1, 0, None, ptr(ws),
           wsz, stream())
    assert np.array_equal(off.cpu().numpy().view(np.uint32), ref)


@pytest.mark.parametrize("K,H,D,p", [(60, 8, 32, 0.1), (16, 4, 16, 0.0), (148, 8, 64, 0.1), (37, 2, 16, 0.3),
                                     (64, 4, 16, 0.2), (61, 8, 32, 0.1), (50, 8, 16, 0.1), (64, 8, 64, 0.1),
                                     (40, 6, 24, 0.1), (1, 8, 32, 0.1),
                                     # K > 64: the multi-wave recompute backward (dh <= 8; partial last
                                     # waves, exactly full waves, the K = 100 / 120 configs), dh = 16 tile
                                     (100, 8, 32, 0.1), (120, 8, 64, 0.15), (65, 2, 16, 0.0), (128, 16, 32, 0.2),
                                     (200, 4, 8, 0.1), (256, 8, 64, 0.1), (100, 4, 64, 0.1)])
@pytest.mark.parametrize("generic", [0, 1])      # 0: the packed forward where it applies (K <= 64 even, dh 4/8)
def test_attention_fwd_bwd_vs_torch(K, H, D, p, generic):
    L = _lib()
    L.query("ctr_attn_set_generic", generic)
    from tossctr.rng import drop_args
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import rng as orng
    B, dh = 5, D // H
    tk = K + 3
    qkv = torch.randn(B * K, 3 * D, device="cuda", requires_grad=True)
    rel_w = torch.randn(2 * tk + 1, H, device="cuda", requires_grad=True)
    dk = drop_args(1234, 7, p, True)
    relmean = torch.empty(2 * tk + 1, device="cuda")
    L.call("ctr_pos_bias_mean", ptr(rel_w), H, 2 * tk + 1, ptr(relmean), stream())
    o = torch.empty(B * K, D, device="cuda")
    mrow = torch.empty(B * H * K, device="cuda")
    lrow = torch.empty(B * H * K, device="cuda")
    scale = float(np.float32(math.sqrt(1.0 / dh)))
    mask = torch.zeros(L.query("ctr_attn_mask_words", B, K, H), dtype=torch.int32, device="cuda")
    L.call("ctr_attn_fwd", ptr(qkv), B, K, H, D, ptr(relmean), tk, scale, *dk, ptr(mask), ptr(o), ptr(mrow),
           ptr(lrow), stream())
    L.query("ctr_attn_set_generic", 0)
    # torch reference (MHA explicit path semantics)
    q, k, v = qkv.view(B, K, 3 * D).split(D, -1)
    q = q.reshape(B, K, H, dh).transpose(1, 2)
    k = k.reshape(B, K, H, dh).transpose(1, 2)
    v = v.reshape(B, K, H, dh).transpose(1, 2)
    i = torch.arange(K, device="cuda")[:, None]
    j = torch.arange(K, device="cuda")[None, :]
    bias = rel_w[(j - i).clamp(-tk, tk) + tk].permute(2, 0, 1).mean(0)
    s = bias + (q * scale) @ k.transpose(-1, -2)
    a = torch.softmax(s, -1)
    if p > 0:
        keep = torch.from_numpy(orng.keep_mask(1234, 7, p, (B * H, K, K))).cuda().view(B, H, K, K)
        a = a * keep.float() / (1 - p)
    o_ref = (a @ v).transpose(1, 2).reshape(B * K, D)
    assert rel(o, o_ref.detach()) < 5e-6
    if p > 0:   # the stored keep bits are exactly the oracle's mask
        km = keep.view(B * H * K, K).cpu().numpy()
        words = mask[:B * H * K * ((K + 31) // 32)].view(B * H * K, -1).cpu().numpy().view(np.uint32)
        bits = (words[:, np.arange(K) // 32] >> (np.arange(K) % 32).astype(np.uint32)) & 1
        assert np.array_equal(bits.astype(bool), km)
    do = torch.randn(B * K, D, device="cuda")
    o_ref.backward(do)
    dqkv = torch.empty(B * K, 3 * D, device="cuda")
    nparts = L.query("ctr_attn_bwd_nparts", H, K, D) * B
    drp = torch.empty(nparts, 2 * tk + 1, device="cuda")
    L.call("ctr_attn_bwd", ptr(qkv), ptr(o), ptr(do), B, K, H, D, ptr(relmean), tk, scale, *dk, ptr(mask), ptr(mrow),
           ptr(lrow), ptr(dqkv), ptr(drp), stream())
    drel = torch.empty(2 * tk + 1, H, device="cuda")
    L.call("ctr_pos_bias_grad", ptr(drp), nparts, H, 2 * tk + 1, ptr(drel), stream())
    assert rel(dqkv, qkv.grad) < 1e-5
    if K == 1:      # softmax over one key: the exact grad is 0, ours is the rounding residue of dp - do.o
        assert drel.abs().max() < 1e-6 and rel_w.grad.abs().max() == 0
    else:
        assert rel(drel, rel_w.grad) < 1e-5


def attn_bf_keep_bits(mask, B, H, K):
    """(B*H, K, K) keep bits from ctr_attn_fwd_bf's lane-layout mask (attn_mf.hip): per head NW x 64 words;
    element (i = 16 ti + c, j = 16 tj + 4 g + r) is bit pos % 32 of word pos // 32 of lane 16 g + c, with
    pos = 16 ti + 4 tj + r for nt = ceil(K / 16) <= 4 (NW 2), pos = 4 nt tj + 4 ti + r beyond (NW ceil(4 nt^2 / 32))."""
    nt = (K + 15) // 16
    nw = 2 if nt <= 4 else (4 * nt * nt + 31) // 32
    words = mask.cpu().numpy().view(np.uint32)[:B * H * 64 * nw].reshape(B * H, nw, 64)
    i = np.arange(K)[:, None]
    j = np.arange(K)[None, :]
    ti, c, tj, g, r = i // 16, i % 16, j // 16, (j % 16) // 4, j % 4
    pos = (16 * ti + 4 * tj + r) if nt <= 4 else (4 * nt * tj + 4 * ti + r)
    w = words[:, pos >> 5, 16 * g + c]
    return ((w >> (pos & 31).astype(np.uint32)[None]) & 1).astype(bool)


def _bfr32(t):
    """RNE bf16 of an fp32 tensor, as fp64."""
    return t.float().to(torch.bfloat16).double()


def attn_bf_emulate(qkv, B, K, H, D, scale, rel, keep, dscale, do=None, do_stat=None, o_kernel=None):
    """fp64 emulation of the amp bf16 attention (attn_mf.hip): every MFMA operand rounded to bf16 exactly where the
    kernels round it -- q * scale (the fp32 product), k, v, dO, the masked unnormalised p (exp(s - max), before the
    1 / l and dropout scales; for K > 64 as the two-term split hi + lo) in the forward, dS and p~ = p keep / (1 - p)
    in the backward -- everything else in fp64: s = q k^T + rel (natural units; the kernels' log2 units are a change
    of base), softmax statistics, dS = p (dp~ - D_i) with D_i = bf16(dO_i) . o_i.  ``rel``: (K, K) bias or None; ``keep``: (B, H, K, K) bool or None; ``do_stat``: the dO
    whose fp32 values form D_i = dO_i . o_i (the kernels take the fp32 dO and the forward's fp32 o,
    ``o_kernel``).  Returns o, and with ``do``: dq, dk, dv and the per-offset dS sums (2K - 1,) over samples and
    heads (offset j - i + K - 1)."""
    dh = D // H
    q, k, v = qkv.float().view(B, K, 3 * D).split(D, -1)
    sh = lambda t: t.reshape(B, K, H, dh).transpose(1, 2)          # noqa: E731
    qb, kb, vb = sh(_bfr32(q * scale)), sh(_bfr32(k)), sh(_bfr32(v))
    s = qb @ kb.transpose(-1, -2)
    if rel is not None:
        s = s + rel.double()
    mx = s.amax(-1, keepdim=True)
    pe = torch.exp(s - mx)
    lsum = pe.sum(-1, keepdim=True)
    kf = keep.double() * dscale if keep is not None else None
    pm = pe * (keep.double() if keep is not None else 1.0)
    pmb = _bfr32(pm)
    if K > 64:      # the two-term split of p (attn_mf.hip lo_bf4): hi = bf16(p), lo = bf16(p - hi)
        pmb = pmb + _bfr32(pm - pmb)
    o = (pmb @ vb) * ((dscale if keep is not None else 1.0) / lsum)
    o = o.transpose(1, 2).reshape(B * K, D)
    if do is None:
        return o
    dob = sh(_bfr32(do))
    ok = sh(o_kernel.double() if o_kernel is not None else o)
    dst = sh(_bfr32(do_stat) if do_stat is not None else _bfr32(do))      # D_i from bf16(dO), as the kernels
    Di = (dst * ok).sum(-1, keepdim=True)
    p_ = pe / lsum
    dp = dob @ vb.transpose(-1, -2)
    dpk = dp * kf if kf is not None else dp
    pt = p_ * kf if kf is not None else p_
    ds = p_ * (dpk - Di)
    dsb = _bfr32(ds)
    dq = (dsb @ kb) * scale
    dk = dsb.transpose(-1, -2) @ qb
    dv = _bfr32(pt).transpose(-1, -2) @ dob
    un = lambda t: t.transpose(1, 2).reshape(B * K, D)             # noqa: E731
    tot = ds.sum((0, 1))                                            # (K, K): [i][j]
    i = torch.arange(K, device=qkv.device)[:, None]
    j = torch.arange(K, device=qkv.device)[None, :]
    diag = torch.zeros(2 * K - 1, dtype=torch.float64, device=qkv.device).index_add_(
        0, (j - i + K - 1).reshape(-1), tot.reshape(-1))
    return o, un(dq), un(dk), un(dv), diag


def rel_table(relmean, K, tk):
    """(K, K) bias rel[j - i + tk] of a (2 tk + 1,) head-mean table."""
    i = torch.arange(K, device=relmean.device)[:, None]
    j = torch.arange(K, device=relmean.device)[None, :]
    return relmean[(j - i).clamp(-tk, tk) + tk]


def drel_from_diag(diag, K, tk, H):
    """The positional-bias grad (2 tk + 1, H) of the per-offset dS sums: rel_w[e, h] enters through the head mean."""
    out = torch.zeros(2 * tk + 1, dtype=torch.float64, device=diag.device)
    d = torch.arange(-(K - 1), K, device=diag.device)
    out.index_add_(0, d.clamp(-tk, tk) + tk, diag)
    return (out / H)[:, None].expand(2 * tk + 1, H)


ATT_BF_TOL = 2e-4    # bf16 emulation: only rare rounding-boundary flips of an operand element differ


@pytest.mark.parametrize("K,H,D,p", [(60, 8, 32, 0.1), (16, 4, 16, 0.0), (37, 2, 8, 0.3), (64, 4, 16, 0.2),
                                     (61, 8, 32, 0.1), (50, 8, 64, 0.1), (64, 8, 64, 0.1), (40, 6, 24, 0.1),
                                     (1, 8, 32, 0.1), (60, 8, 64, 0.0), (33, 3, 24, 0.1),
                                     # K > 64 (attn_bwd_mfl_kernel, compact staging): cfg3 (K 100, dh 4), cfg4
                                     # (K 148, dh 8), v3_k120, odd K, one key past a tile, the 160 maximum
                                     (100, 8, 32, 0.1), (148, 8, 64, 0.1), (120, 8, 64, 0.15), (97, 4, 16, 0.2),
                                     (65, 2, 16, 0.0), (160, 8, 64, 0.1), (129, 3, 24, 0.1)])
@pytest.mark.parametrize("bias", [True, False])
def test_attention_bf16_vs_emulation(K, H, D, p, bias):
    """amp: the bf16-MFMA attention (ctr_attn_fwd_bf / ctr_attn_bwd_bf) against an fp64 emulation with the
    kernels' bf16-rounded operands (attn_bf_emulate) at ATT_BF_TOL; keep bits exactly the oracle's; a second
    backward bitwise equal."""
    L = _lib()
    assert L.query("ctr_attn_bf_ok", K, H, D) == 1
    from tossctr.rng import drop_args
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import rng as orng
    B, dh = 7, D // H
    tk = K + 3
    g = torch.Generator(device="cuda").manual_seed(K * 131 + H)
    qkv = torch.randn(B * K, 3 * D, device="cuda", generator=g)
    rel_w = torch.randn(2 * tk + 1, H, device="cuda", generator=g)
    dk = drop_args(4321, 9, p, True)
    relmean = torch.empty(2 * tk + 1, device="cuda")
    L.call("ctr_pos_bias_mean", ptr(rel_w), H, 2 * tk + 1, ptr(relmean), stream())
    o = torch.empty(B * K, D, device="cuda")
    mrow = torch.empty(B * H * K, device="cuda")
    lrow = torch.empty(B * H * K, device="cuda")
    scale = float(np.float32(math.sqrt(1.0 / dh)))
    mask = torch.zeros(L.query("ctr_attn_mask_words", B, K, H), dtype=torch.int32, device="cuda")
    rm = ptr(relmean) if bias else None
    L.call("ctr_attn_fwd_bf", ptr(qkv), B, K, H, D, rm, tk, scale, *dk, ptr(mask), ptr(o), ptr(mrow), ptr(lrow),
           stream())
    keep = None
    if p > 0:
        km = orng.keep_mask(4321, 9, p, (B * H, K, K))
        assert np.array_equal(attn_bf_keep_bits(mask, B, H, K), km)
        keep = torch.from_numpy(km).cuda().view(B, H, K, K)
    do = torch.randn(B * K, D, device="cuda", generator=g)
    rt = rel_table(relmean, K, tk) if bias else None
    o_ref, dq_r, dk_r, dv_r, diag = attn_bf_emulate(qkv, B, K, H, D, scale, rt, keep, dk[2], do, o_kernel=o)
    assert rel(o.double(), o_ref) < ATT_BF_TOL, rel(o.double(), o_ref)
    dqkv = torch.full((B * K, 3 * D), float("nan"), device="cuda")
    nparts = L.query("ctr_attn_bwd_bf_nparts", H) * B
    drp = torch.full((nparts, 2 * tk + 1), float("nan"), device="cuda")
    L.call("ctr_attn_bwd_bf", ptr(qkv), ptr(o), ptr(do), B, K, H, D, rm, tk, scale, *dk, ptr(mask), ptr(mrow),
           ptr(lrow), ptr(dqkv), ptr(drp), stream())
    torch.cuda.synchronize()
    assert torch.isfinite(dqkv).all()
    dq, dkk, dv = (t.double() for t in dqkv.split(D, -1))
    if K == 1:      # softmax over one key: exact dq = dk = 0; ours (and the emulation's) the bf16 residue dO_b - dO
        assert dq.abs().max() < 0.05 and dkk.abs().max() < 0.05 and rel(dv, dv_r) < ATT_BF_TOL
    else:
        errs = (rel(dq, dq_r), rel(dkk, dk_r), rel(dv, dv_r))
        assert max(errs) < ATT_BF_TOL, errs
    drp_first = drp.clone()           # ctr_pos_bias_grad reduces the partials in place
    if bias:
        assert torch.isfinite(drp).all()
        drel = torch.empty(2 * tk + 1, H, device="cuda")
        L.call("ctr_pos_bias_grad", ptr(drp), nparts, H, 2 * tk + 1, ptr(drel), stream())
        if K == 1:      # exact grad 0; ours the bf16 residue of dp - do.o
            assert drel.abs().max() < 0.1
        else:
            assert rel(drel.double(), drel_from_diag(diag, K, tk, H)) < ATT_BF_TOL
    # deterministic: a second backward is bitwise identical
    dqkv2 = torch.empty_like(dqkv)
    drp2 = torch.empty_like(drp)
    L.call("ctr_attn_bwd_bf", ptr(qkv), ptr(o), ptr(do), B, K, H, D, rm, tk, scale, *dk, ptr(mask), ptr(mrow),
           ptr(lrow), ptr(dqkv2), ptr(drp2), stream())
    torch.cuda.synchronize()
    assert torch.equal(dqkv, dqkv2) and (not bias or torch.equal(drp_first, drp2))


@pytest.mark.parametrize("p", [0.1, 0.0])
def test_attn_layer_bf16_full_batch_vs_emulation(p):
    """The two attention entry points the bench times, at its shape (cfg2: B = 4096, K = 60, H = 8, D = 32 -- the
    XCD-aware 1-D grid of attn_mf.hip over 4096 samples x 2 head groups): ctr_attn_layer_fwd_bf against fp64 --
    in_proj (fp32 MFMA: 1e-6), the attention against attn_bf_emulate on the kernel's own qkv (ATT_BF_TOL), out_proj +
    residual + RMSNorm on the kernel's own o (1e-6), the keep bits exactly the oracle's -- and ctr_attn_bwd_bf_oproj
    (dO = dh1 W_out formed inside) against the emulation at ATT_BF_TOL (dq, dk, dv, the positional-bias grad)."""
    L = _lib()
    B, K, H, D = 4096, 60, 8, 32
    assert L.query("ctr_attn_layer_fwd_ok", K, H, D) == 1 and L.query("ctr_attn_bwd_bf_oproj_ok", K, H, D) == 1
    from tossctr.rng import drop_args
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import rng as orng
    dh, tk, M = D // H, K, B * K
    g = torch.Generator(device="cuda").manual_seed(4096 + int(p * 10))
    x = torch.randn(M, D, device="cuda", generator=g)
    w_in = torch.randn(3 * D, D, device="cuda", generator=g) * D ** -0.5
    b_in = torch.randn(3 * D, device="cuda", generator=g) * 0.1
    w_out = torch.randn(D, D, device="cuda", generator=g) * D ** -0.5
    b_out = torch.randn(D, device="cuda", generator=g) * 0.1
    nw = 1 + 0.1 * torch.randn(D, device="cuda", generator=g)
    rel_w = torch.randn(2 * tk + 1, H, device="cuda", generator=g)
    relmean = torch.full((2 * tk + 1,), float("nan"), device="cuda")
    dk = drop_args(2024, 5, p, True)
    scale = float(np.float32(math.sqrt(1.0 / dh)))
    st = stream()
    qkv = torch.full((M, 3 * D), float("nan"), device="cuda")
    o = torch.full((M, D), float("nan"), device="cuda")
    mrow = torch.full((B * H * K,), float("nan"), device="cuda")
    lrow = torch.full((B * H * K,), float("nan"), device="cuda")
    mask = torch.zeros(L.query("ctr_attn_mask_words", B, K, H), dtype=torch.int32, device="cuda")
    h1 = torch.full((M, D), float("nan"), device="cuda")
    r1 = torch.full((M,), float("nan"), device="cuda")
    x1 = torch.full((M, D), float("nan"), device="cuda")
    L.call("ctr_attn_layer_fwd_bf", ptr(x), B, K, H, D, ptr(w_in), ptr(b_in), ptr(rel_w), ptr(relmean), tk, scale,
           *dk, ptr(mask), ptr(w_out), ptr(b_out), ptr(nw), 1e-6, ptr(qkv), ptr(o), ptr(mrow), ptr(lrow), ptr(h1),
           ptr(r1), ptr(x1), st)
    torch.cuda.synchronize()
    assert rel(relmean.double(), rel_w.double().mean(1)) < 1e-6
    assert rel(qkv.double(), x.double() @ w_in.double().t() + b_in.double()) < 1e-6
    keep = None
    if p > 0:
        km = orng.keep_mask(2024, 5, p, (B * H, K, K))
        assert np.array_equal(attn_bf_keep_bits(mask, B, H, K), km)
        keep = torch.from_numpy(km).cuda().view(B, H, K, K)
        del km
    rt = rel_table(relmean, K, tk)
    o_ref = attn_bf_emulate(qkv, B, K, H, D, scale, rt, keep, dk[2])
    assert rel(o.double(), o_ref) < ATT_BF_TOL, rel(o.double(), o_ref)
    del o_ref
    h1r = x.double() + o.double() @ w_out.double().t() + b_out.double()
    r1r = 1.0 / torch.sqrt((h1r * h1r).mean(1) + 1e-6)
    assert rel(h1.double(), h1r) < 1e-6 and rel(r1.double(), r1r) < 1e-6
    assert rel(x1.double(), nw.double() * h1r * r1r[:, None]) < 1e-6
    del h1r
    dh1 = torch.randn(M, D, device="cuda", generator=g)
    nparts = L.query("ctr_attn_bwd_bf_nparts", H) * B
    dqkv = torch.full((M, 3 * D), float("nan"), device="cuda")
    drp = torch.full((nparts, 2 * tk + 1), float("nan"), device="cuda")
    L.call("ctr_attn_bwd_bf_oproj", ptr(qkv), ptr(o), ptr(dh1), ptr(w_out), B, K, H, D, ptr(relmean), tk, scale, *dk,
           ptr(mask), ptr(mrow), ptr(lrow), ptr(dqkv), ptr(drp), st)
    drel = torch.empty(2 * tk + 1, H, device="cuda")
    L.call("ctr_pos_bias_grad", ptr(drp), nparts, H, 2 * tk + 1, ptr(drel), st)
    torch.cuda.synchronize()
    do64 = dh1.double() @ w_out.double()
    _, dq_r, dk_r, dv_r, diag = attn_bf_emulate(qkv, B, K, H, D, scale, rt, keep, dk[2], do64, o_kernel=o)
    dq, dkk, dv = (t.double() for t in dqkv.split(D, -1))
    errs = (rel(dq, dq_r), rel(dkk, dk_r), rel(dv, dv_r), rel(drel.double(), drel_from_diag(diag, K, tk, H)))
    assert max(errs) < ATT_BF_TOL, errs


@pytest.mark.parametrize("K,H,D,p", [(100, 8, 32, 0.1), (148, 8, 64, 0.1)])
def test_attention_bf16_full_batch_k_gt_64(K, H, D, p):
    """The K > 64 bf16 attention (ctr_attn_fwd_bf / ctr_attn_bwd_bf: attn_bwd_mfl_kernel's compact staging) at the
    production batch of BASELINE cfg3 (K = 100, D = 32, dh 4) and cfg4 (K = 148, D = 64, dh 8): B = 4096 samples over
    the full grid, against the fp64 emulation (attn_bf_emulate) at ATT_BF_TOL, evaluated in sample chunks (norms
    accumulated over the whole batch); the keep bits exactly the oracle's in every chunk."""
    L = _lib()
    assert L.query("ctr_attn_bf_ok", K, H, D) == 1
    from tossctr.rng import drop_args
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import rng as orng
    B, dh, tk = 4096, D // H, K
    g = torch.Generator(device="cuda").manual_seed(K * 4099 + D)
    qkv = torch.randn(B * K, 3 * D, device="cuda", generator=g)
    rel_w = torch.randn(2 * tk + 1, H, device="cuda", generator=g)
    dk = drop_args(9876, 11, p, True)
    relmean = torch.empty(2 * tk + 1, device="cuda")
    st = stream()
    L.call("ctr_pos_bias_mean", ptr(rel_w), H, 2 * tk + 1, ptr(relmean), st)
    o = torch.full((B * K, D), float("nan"), device="cuda")
    mrow = torch.empty(B * H * K, device="cuda")
    lrow = torch.empty(B * H * K, device="cuda")
    scale = float(np.float32(math.sqrt(1.0 / dh)))
    nmask = L.query("ctr_attn_mask_words", B, K, H)
    mask = torch.zeros(nmask, dtype=torch.int32, device="cuda")
    L.call("ctr_attn_fwd_bf", ptr(qkv), B, K, H, D, ptr(relmean), tk, scale, *dk, ptr(mask), ptr(o), ptr(mrow),
           ptr(lrow), st)
    do = torch.randn(B * K, D, device="cuda", generator=g)
    dqkv = torch.full((B * K, 3 * D), float("nan"), device="cuda")
    nparts = L.query("ctr_attn_bwd_bf_nparts", H) * B
    drp = torch.full((nparts, 2 * tk + 1), float("nan"), device="cuda")
    L.call("ctr_attn_bwd_bf", ptr(qkv), ptr(o), ptr(do), B, K, H, D, ptr(relmean), tk, scale, *dk, ptr(mask),
           ptr(mrow), ptr(lrow), ptr(dqkv), ptr(drp), st)
    drel = torch.empty(2 * tk + 1, H, device="cuda")
    L.call("ctr_pos_bias_grad", ptr(drp), nparts, H, 2 * tk + 1, ptr(drel), st)
    torch.cuda.synchronize()
    assert torch.isfinite(o).all() and torch.isfinite(dqkv).all()
    km = orng.keep_mask(9876, 11, p, (B * H, K, K))
    nt = (K + 15) // 16
    wps = H * 64 * (2 if nt <= 4 else (4 * nt * nt + 31) // 32)      # mask words per sample
    assert nmask >= B * wps
    rt = rel_table(relmean, K, tk)
    err = np.zeros(4)
    nrm = np.zeros(4)
    diag = torch.zeros(2 * K - 1, dtype=torch.float64, device="cuda")
    CH = 256
    for c0 in range(0, B, CH):
        c1 = min(B, c0 + CH)
        n = c1 - c0
        kc = km[c0 * H:c1 * H]
        assert np.array_equal(attn_bf_keep_bits(mask[c0 * wps:c1 * wps], n, H, K), kc), c0
        keep = torch.from_numpy(kc).cuda().view(n, H, K, K)
        r0, r1 = c0 * K, c1 * K
        o_r, dq_r, dk_r, dv_r, dg = attn_bf_emulate(qkv[r0:r1], n, K, H, D, scale, rt, keep, dk[2], do[r0:r1],
                                                    o_kernel=o[r0:r1])
        diag += dg
        dq, dkk, dv = (t.double() for t in dqkv[r0:r1].split(D, -1))
        for i, (x, y) in enumerate(((o[r0:r1].double(), o_r), (dq, dq_r), (dkk, dk_r), (dv, dv_r))):
            err[i] += float(((x - y) ** 2).sum())
            nrm[i] += float((y ** 2).sum())
        del keep, o_r, dq_r, dk_r, dv_r
    errs = list(np.sqrt(err / nrm)) + [rel(drel.double(), drel_from_diag(diag, K, tk, H))]
    assert max(errs) < ATT_BF_TOL, errs


@pytest.mark.parametrize("K,H,p", [(60, 8, 0.1), (64, 8, 0.1), (61, 8, 0.1), (48, 4, 0.2), (33, 8, 0.0),
                                   (17, 4, 0.1), (1, 8, 0.1), (50, 4, 0.0)])
@pytest.mark.parametrize("bias", [True, False])
def test_attn_layer_fwd_equals_three_launches(K, H, p, bias):
    """amp: ctr_attn_layer_fwd_bf (in_proj -> attention -> out_proj + residual + RMSNorm in one launch) writes
    bit for bit what ctr_rowgemm + ctr_attn_fwd_bf + ctr_rowgemm write: qkv, o, mrow, lrow, the keep bits, h1, r1,
    x1 (the same summation orders; the three-launch path is covered against torch above)."""
    L = _lib()
    D = 32
    assert L.query("ctr_attn_layer_fwd_ok", K, H, D) == 1
    from tossctr.rng import drop_args
    B, dh, tk = 37, D // H, K
    g = torch.Generator(device="cuda").manual_seed(K * 17 + H)
    x = torch.randn(B * K, D, device="cuda", generator=g)
    w_in = torch.randn(3 * D, D, device="cuda", generator=g) * D ** -0.5
    b_in = torch.randn(3 * D, device="cuda", generator=g) * 0.1
    w_out = torch.randn(D, D, device="cuda", generator=g) * D ** -0.5
    b_out = torch.randn(D, device="cuda", generator=g) * 0.1
    nw = 1 + 0.1 * torch.randn(D, device="cuda", generator=g)
    rel_w = torch.randn(2 * tk + 1, H, device="cuda", generator=g)
    relmean = torch.empty(2 * tk + 1, device="cuda")
    L.call("ctr_pos_bias_mean", ptr(rel_w), H, 2 * tk + 1, ptr(relmean), stream())
    rm = ptr(relmean) if bias else None
    f_relmean = torch.full_like(relmean, float("nan"))
    dk = drop_args(777, 3, p, True)
    scale = float(np.float32(math.sqrt(1.0 / dh)))
    st = stream()

    def bufs():
        return dict(qkv=torch.full((B * K, 3 * D), float("nan"), device="cuda"),
                    o=torch.full((B * K, D), float("nan"), device="cuda"),
                    mrow=torch.full((B * H * K,), float("nan"), device="cuda"),
                    lrow=torch.full((B * H * K,), float("nan"), device="cuda"),
                    mask=torch.zeros(L.query("ctr_attn_mask_words", B, K, H), dtype=torch.int32, device="cuda"),
                    h1=torch.full((B * K, D), float("nan"), device="cuda"),
                    r1=torch.full((B * K,), float("nan"), device="cuda"),
                    x1=torch.full((B * K, D), float("nan"), device="cuda"))
    r, f = bufs(), bufs()
    M = B * K
    L.call("ctr_rowgemm", M, D, 3 * D, ptr(x), D, ptr(w_in), 1, ptr(r["qkv"]), 3 * D, ptr(b_in), None, 0, None, 0,
           None, None, None, 1e-6, st)
    L.call("ctr_attn_fwd_bf", ptr(r["qkv"]), B, K, H, D, rm, tk, scale, *dk, ptr(r["mask"]), ptr(r["o"]),
           ptr(r["mrow"]), ptr(r["lrow"]), st)
    L.call("ctr_rowgemm", M, D, D, ptr(r["o"]), D, ptr(w_out), 1, ptr(r["x1"]), D, ptr(b_out), None, 0, ptr(x), D,
           ptr(nw), ptr(r["h1"]), ptr(r["r1"]), 1e-6, st)
    L.call("ctr_attn_layer_fwd_bf", ptr(x), B, K, H, D, ptr(w_in), ptr(b_in), ptr(rel_w) if bias else None,
           ptr(f_relmean) if bias else None, tk, scale, *dk, ptr(f["mask"]),
           ptr(w_out), ptr(b_out), ptr(nw), 1e-6, ptr(f["qkv"]), ptr(f["o"]), ptr(f["mrow"]), ptr(f["lrow"]),
           ptr(f["h1"]), ptr(f["r1"]), ptr(f["x1"]), st)
    # the bf16-qkv form: every other output the same bits, qkv16 = bf16(q * scale) | bf16(k) | bf16(v) (RNE)
    h = bufs()
    qkv16 = torch.full((B * K, 3 * D), float("nan"), device="cuda", dtype=torch.bfloat16)
    L.call("ctr_attn_layer_fwd_bf16", ptr(x), B, K, H, D, ptr(w_in), ptr(b_in), ptr(rel_w) if bias else None,
           ptr(f_relmean) if bias else None, tk, scale, *dk, ptr(h["mask"]),
           ptr(w_out), ptr(b_out), ptr(nw), 1e-6, ptr(qkv16), ptr(h["o"]), ptr(h["mrow"]), ptr(h["lrow"]),
           ptr(h["h1"]), ptr(h["r1"]), ptr(h["x1"]), st)
    torch.cuda.synchronize()
    for name in r:
        a, b = r[name], f[name]
        assert torch.equal(a.view(torch.int32), b.view(torch.int32)), \
            (name, int((a.view(torch.int32) != b.view(torch.int32)).sum()), a.numel())
        if name != "qkv":
            assert torch.equal(a.view(torch.int32), h[name].view(torch.int32)), name
    if bias:     # the head-mean table the kernel formed and wrote for the backward
        assert torch.equal(relmean.view(torch.int32), f_relmean.view(torch.int32))
    want = torch.cat([r["qkv"][:, :D] * scale, r["qkv"][:, D:]], 1).bfloat16()
    assert torch.equal(qkv16.view(torch.int16), want.view(torch.int16)), int((qkv16 != want).sum())


@pytest.mark.parametrize("K,H,p", [(60, 8, 0.1), (64, 8, 0.1), (61, 8, 0.1), (48, 4, 0.2), (33, 8, 0.0),
                                   (17, 4, 0.1), (1, 8, 0.1), (50, 4, 0.0)])
@pytest.mark.parametrize("bias", [True, False])
def test_attn_bwd_oproj_equals_two_launches(K, H, p, bias):
    """amp: ctr_attn_bwd_bf_oproj (dO = dh1 W_out formed inside the attention backward) writes bit for bit what
    ctr_rowgemm(dh1, W_out) + ctr_attn_bwd_bf write: dqkv and the positional-bias partials."""
    L = _lib()
    D = 32
    assert L.query("ctr_attn_bwd_bf_oproj_ok", K, H, D) == 1
    from tossctr.rng import drop_args
    B, dh, tk = 37, D // H, K
    g = torch.Generator(device="cuda").manual_seed(K * 29 + H)
    qkv = torch.randn(B * K, 3 * D, device="cuda", generator=g)
    dh1 = torch.randn(B * K, D, device="cuda", generator=g)
    w_out = torch.randn(D, D, device="cuda", generator=g) * D ** -0.5
    relmean = torch.randn(2 * tk + 1, device="cuda", generator=g)
    rm = ptr(relmean) if bias else None
    dk = drop_args(555, 5, p, True)
    scale = float(np.float32(math.sqrt(1.0 / dh)))
    st = stream()
    o = torch.empty(B * K, D, device="cuda")
    mrow = torch.empty(B * H * K, device="cuda")
    lrow = torch.empty(B * H * K, device="cuda")
    mask = torch.zeros(L.query("ctr_attn_mask_words", B, K, H), dtype=torch.int32, device="cuda")
    L.call("ctr_attn_fwd_bf", ptr(qkv), B, K, H, D, rm, tk, scale, *dk, ptr(mask), ptr(o), ptr(mrow), ptr(lrow), st)
    nparts = L.query("ctr_attn_bwd_bf_nparts", H) * B
    do = torch.empty(B * K, D, device="cuda")
    L.call("ctr_rowgemm", B * K, D, D, ptr(dh1), D, ptr(w_out), 0, ptr(do), D, None, None, 0, None, 0, None, None, None,
           1e-6, st)
    r_dqkv = torch.full((B * K, 3 * D), float("nan"), device="cuda")
    r_drp = torch.full((nparts, 2 * tk + 1), float("nan"), device="cuda")
    L.call("ctr_attn_bwd_bf", ptr(qkv), ptr(o), ptr(do), B, K, H, D, rm, tk, scale, *dk, ptr(mask), ptr(mrow),
           ptr(lrow), ptr(r_dqkv), ptr(r_drp), st)
    f_dqkv = torch.full_like(r_dqkv, float("nan"))
    f_drp = torch.full_like(r_drp, float("nan"))
    L.call("ctr_attn_bwd_bf_oproj", ptr(qkv), ptr(o), ptr(dh1), ptr(w_out), B, K, H, D, rm, tk, scale, *dk, ptr(mask),
           ptr(mrow), ptr(lrow), ptr(f_dqkv), ptr(f_drp), st)
    # the bf16 form: qkv16 as the layer forward stores it, dqkv16 = the RNE bf16 of the same dq / dk / dv
    qkv16 = torch.cat([qkv[:, :D] * scale, qkv[:, D:]], 1).bfloat16()
    h_dqkv = torch.full((B * K, 3 * D), float("nan"), device="cuda", dtype=torch.bfloat16)
    h_drp = torch.full_like(r_drp, float("nan"))
    L.call("ctr_attn_bwd_bf_oproj16", ptr(qkv16), ptr(o), ptr(dh1), ptr(w_out), B, K, H, D, rm, tk, scale, *dk,
           ptr(mask), ptr(mrow), ptr(lrow), ptr(h_dqkv), ptr(h_drp), st)
    torch.cuda.synchronize()
    assert torch.equal(r_dqkv.view(torch.int32), f_dqkv.view(torch.int32)), int((r_dqkv != f_dqkv).sum())
    assert torch.equal(h_dqkv.view(torch.int16), r_dqkv.bfloat16().view(torch.int16)), \
        int((h_dqkv != r_dqkv.bfloat16()).sum())
    if bias:
        assert torch.equal(r_drp.view(torch.int32), f_drp.view(torch.int32))
        assert torch.equal(r_drp.view(torch.int32), h_drp.view(torch.int32))


@pytest.mark.parametrize("K,H,p", [(60, 8, 0.1), (64, 8, 0.1), (61, 8, 0.1), (48, 4, 0.2), (33, 8, 0.0),
                                   (17, 4, 0.1), (1, 8, 0.1), (50, 4, 0.0)])
@pytest.mark.parametrize("bias", [True, False])
def test_attn_bwd_layer_equals_two_launches(K, H, p, bias):
    """amp: ctr_attn_bwd_bf_layer16 (one workgroup per sample: dO = dh1 W_out, the attention backward, then
    dx = dqkv16 W_in + dh1 from the workgroup's own rows) writes bit for bit what ctr_attn_bwd_bf_oproj16 +
    ctr_rowgemm_a16(add = dh1) write: dqkv16 and dx; its one positional-bias row per sample is the sum of the H / 4
    head-group rows (the same bits at H = 4, one group)."""
    L = _lib()
    D = 32
    assert L.query("ctr_attn_bwd_bf_layer_ok", K, H, D) == 1
    from tossctr.rng import drop_args
    B, dh, tk = 37, D // H, K
    g = torch.Generator(device="cuda").manual_seed(K * 31 + H)
    qkv = torch.randn(B * K, 3 * D, device="cuda", generator=g)
    dh1 = torch.randn(B * K, D, device="cuda", generator=g)
    w_out = torch.randn(D, D, device="cuda", generator=g) * D ** -0.5
    w_in = torch.randn(3 * D, D, device="cuda", generator=g) * D ** -0.5
    relmean = torch.randn(2 * tk + 1, device="cuda", generator=g)
    rm = ptr(relmean) if bias else None
    dk = drop_args(556, 5, p, True)
    scale = float(np.float32(math.sqrt(1.0 / dh)))
    st = stream()
    o = torch.empty(B * K, D, device="cuda")
    mrow = torch.empty(B * H * K, device="cuda")
    lrow = torch.empty(B * H * K, device="cuda")
    mask = torch.zeros(L.query("ctr_attn_mask_words", B, K, H), dtype=torch.int32, device="cuda")
    L.call("ctr_attn_fwd_bf", ptr(qkv), B, K, H, D, rm, tk, scale, *dk, ptr(mask), ptr(o), ptr(mrow), ptr(lrow), st)
    qkv16 = torch.cat([qkv[:, :D] * scale, qkv[:, D:]], 1).bfloat16()
    ng = L.query("ctr_attn_bwd_bf_nparts", H)
    r_dqkv = torch.full((B * K, 3 * D), float("nan"), device="cuda", dtype=torch.bfloat16)
    r_drp = torch.full((ng * B, 2 * tk + 1), float("nan"), device="cuda")
    L.call("ctr_attn_bwd_bf_oproj16", ptr(qkv16), ptr(o), ptr(dh1), ptr(w_out), B, K, H, D, rm, tk, scale, *dk,
           ptr(mask), ptr(mrow), ptr(lrow), ptr(r_dqkv), ptr(r_drp), st)
    r_dx = torch.full((B * K, D), float("nan"), device="cuda")
    L.call("ctr_rowgemm_a16", B * K, 3 * D, D, ptr(r_dqkv), 3 * D, ptr(w_in), 0, ptr(r_dx), D, None, ptr(dh1), D, st)
    f_dqkv = torch.full_like(r_dqkv, float("nan"))
    f_drp = torch.full((B, 2 * tk + 1), float("nan"), device="cuda")
    f_dx = torch.full_like(r_dx, float("nan"))
    L.call("ctr_attn_bwd_bf_layer16", ptr(qkv16), ptr(o), ptr(dh1), ptr(w_out), ptr(w_in), B, K, H, D, rm, tk, scale,
           *dk, ptr(mask), ptr(mrow), ptr(lrow), ptr(f_dqkv), ptr(f_drp), ptr(f_dx), st)
    torch.cuda.synchronize()
    assert torch.equal(f_dqkv.view(torch.int16), r_dqkv.view(torch.int16)), int((f_dqkv != r_dqkv).sum())
    assert torch.equal(f_dx.view(torch.int32), r_dx.view(torch.int32)), int((f_dx != r_dx).sum())
    if bias:
        want = r_drp.view(B, ng, -1).sum(1)
        if ng == 1:
            assert torch.equal(f_drp.view(torch.int32), want.view(torch.int32))
        else:
            torch.testing.assert_close(f_drp, want, rtol=1e-5, atol=1e-5 * float(want.abs().max()))


@pytest.mark.parametrize("M", [245760, 1000, 33, 1])
@pytest.mark.parametrize("add", [True, False])
def test_rowgemm_bf16_operand_forms_equal_fp32_forms(M, add):
    """amp: the in-projection backward on the bf16 dqkv -- ctr_rowgemm_a16 and ctr_rowgemm_wgrad_y16 -- give the bits
    of ctr_rowgemm / ctr_rowgemm_wgrad on the same values widened to fp32 (M = 245,760 is cfg2's B*K)."""
    L = _lib()
    D = 32
    g = torch.Generator(device="cuda").manual_seed(M + add)
    dq16 = torch.randn(M, 3 * D, device="cuda", generator=g).bfloat16()
    dq32 = dq16.float()
    W = torch.randn(3 * D, D, device="cuda", generator=g) * D ** -0.5
    dh1 = torch.randn(M, D, device="cuda", generator=g)
    x = torch.randn(M, D, device="cuda", generator=g)
    st = stream()
    ref = torch.full((M, D), float("nan"), device="cuda")
    got = torch.full_like(ref, float("nan"))
    L.call("ctr_rowgemm", M, 3 * D, D, ptr(dq32), 3 * D, ptr(W), 0, ptr(ref), D, None, ptr(dh1) if add else None,
           D if add else 0, None, 0, None, None, None, 1e-6, st)
    L.call("ctr_rowgemm_a16", M, 3 * D, D, ptr(dq16), 3 * D, ptr(W), 0, ptr(got), D, None, ptr(dh1) if add else None,
           D if add else 0, st)
    rows = L.query("ctr_rowgemm_wgrad_rows", M)
    o_db = 3 * D * D
    ld = (o_db + 3 * D + 3) // 4 * 4
    s_ref = torch.zeros(rows, ld, device="cuda")
    s_got = torch.zeros(rows, ld, device="cuda")
    L.call("ctr_rowgemm_wgrad", ptr(dq32), 3 * D, ptr(x), D, M, 3 * D, D, ptr(s_ref), ld, o_db, st)
    L.call("ctr_rowgemm_wgrad_y16", ptr(dq16), 3 * D, ptr(x), D, M, 3 * D, D, ptr(s_got), ld, o_db, st)
    torch.cuda.synchronize()
    assert torch.equal(ref.view(torch.int32), got.view(torch.int32)), int((ref != got).sum())
    assert torch.equal(s_ref.view(torch.int32), s_got.view(torch.int32)), int((s_ref != s_got).sum())
    want = dq32.double() @ W.double() + (dh1.double() if add else 0.0)
    assert float((ref.double() - want).norm() / want.norm()) < 1e-6
    dw = s_ref.double().sum(0)
    assert float((dw[:o_db].view(3 * D, D) - dq32.double().t() @ x.double()).norm() /
                 (dq32.double().t() @ x.double()).norm()) < 1e-6


@pytest.mark.parametrize("B,F0,F1,D,fe", [(4096, 82, 82, 32, 16), (1000, 35, 7, 64, 8), (37, 5, 3, 16, 4)])
def test_feat_embed_two_groups_equal_two_calls(B, F0, F1, D, fe):
    """ctr_feat_embed_fwd2 / _bwd2 (numeric + binary group in one launch per kernel) write the bits of two
    single-group calls: the outputs, dW, dbias (group 0 only, as the binary embedding has none) and dP."""
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(B + F0 + F1)
    xs = [torch.randn(B, F, device="cuda", generator=g) for F in (F0, F1)]
    Ws = [torch.randn(F, fe, device="cuda", generator=g) for F in (F0, F1)]
    bias = torch.randn(F0, fe, device="cuda", generator=g)
    Ps = [torch.randn(D, fe, device="cuda", generator=g) / fe ** 0.5 for _ in range(2)]
    ld = (F0 + F1) * D + 8
    st = stream()
    outs = [torch.full((B, ld), float("nan"), device="cuda") for _ in range(2)]
    offs = (0, F0 * D)
    L.call("ctr_feat_embed_fwd", ptr(xs[0]), B, F0, ptr(Ws[0]), ptr(bias), ptr(Ps[0]), fe, D, ptr(outs[0], offs[0]), ld, st)
    L.call("ctr_feat_embed_fwd", ptr(xs[1]), B, F1, ptr(Ws[1]), None, ptr(Ps[1]), fe, D, ptr(outs[0], offs[1]), ld, st)
    L.call("ctr_feat_embed_fwd2", ptr(xs[0]), F0, ptr(Ws[0]), ptr(bias), ptr(Ps[0]), ptr(outs[1], offs[0]),
           ptr(xs[1]), F1, ptr(Ws[1]), None, ptr(Ps[1]), ptr(outs[1], offs[1]), B, fe, D, ld, st)
    torch.cuda.synchronize()
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))
    dout = torch.randn(B, ld, device="cuda", generator=g)
    ws = [torch.empty(L.query("ctr_feat_embed_bwd_ws", B, F, D) // 4 + 1, device="cuda") for F in (F0, F1, F0, F1)]

    def grads():
        return ([torch.full((F, fe), float("nan"), device="cuda") for F in (F0, F1)],
                torch.full((F0, fe), float("nan"), device="cuda"),
                [torch.full((D, fe), float("nan"), device="cuda") for _ in range(2)])
    (dWa, dba, dPa), (dWb, dbb, dPb) = grads(), grads()
    L.call("ctr_feat_embed_bwd", ptr(xs[0]), B, F0, ptr(Ws[0]), ptr(bias), ptr(Ps[0]), fe, D, ptr(dout, offs[0]), ld,
           ptr(dWa[0]), ptr(dba), ptr(dPa[0]), ptr(ws[0]), st)
    L.call("ctr_feat_embed_bwd", ptr(xs[1]), B, F1, ptr(Ws[1]), None, ptr(Ps[1]), fe, D, ptr(dout, offs[1]), ld,
           ptr(dWa[1]), None, ptr(dPa[1]), ptr(ws[1]), st)
    L.call("ctr_feat_embed_bwd2", ptr(xs[0]), F0, ptr(Ws[0]), ptr(bias), ptr(Ps[0]), ptr(dout, offs[0]), ptr(dWb[0]),
           ptr(dbb), ptr(dPb[0]), ptr(ws[2]), ptr(xs[1]), F1, ptr(Ws[1]), None, ptr(Ps[1]), ptr(dout, offs[1]),
           ptr(dWb[1]), None, ptr(dPb[1]), ptr(ws[3]), B, fe, D, ld, st)
    torch.cuda.synchronize()
    for a_, b_ in zip(dWa + [dba] + dPa, dWb + [dbb] + dPb):
        assert torch.equal(a_.view(torch.int32), b_.view(torch.int32))


@pytest.mark.parametrize("B,F,D,fe,bias", [(4096, 82, 32, 16, True), (4096, 82, 32, 16, False), (1000, 35, 64, 8, True),
                                           (37, 5, 16, 4, True), (300, 3, 256, 16, True), (257, 7, 48, 24, False)])
def test_feat_embed_vs_fp64(B, F, D, fe, bias):
    """NumericFeatureEmbedding / BinaryFeatureEmbedding (src/models/feature_embed.py:19-27, 42-48): out = (x W + b) P^T
    and its backward (dW, dbias, dP) against an fp64 torch reference; B = 4096 / F = 82 / D = 32 is the bench's."""
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(B + F + D)
    x = torch.randn(B, F, device="cuda", generator=g)
    W = torch.randn(F, fe, device="cuda", generator=g)
    bv = torch.randn(F, fe, device="cuda", generator=g) if bias else None
    P = torch.randn(D, fe, device="cuda", generator=g) / fe ** 0.5
    out_ld = F * D + 5                        # a row stride wider than the block, as in the stacked token matrix
    out = torch.full((B, out_ld), float("nan"), device="cuda")
    st = stream()
    L.call("ctr_feat_embed_fwd", ptr(x), B, F, ptr(W), ptr(bv) if bias else None, ptr(P), fe, D, ptr(out), out_ld, st)
    xd, Wd, Pd = x.double(), W.double(), P.double()
    h = xd[:, :, None] * Wd[None] + (bv.double()[None] if bias else 0.0)
    ref = torch.einsum("bfk,dk->bfd", h, Pd).reshape(B, F * D)
    torch.cuda.synchronize()
    got = out[:, :F * D].double()
    assert torch.isnan(out[:, F * D:]).all(), "wrote past the block"
    assert float((got - ref).norm() / ref.norm()) < 1e-6
    dout_t = torch.randn(B, out_ld, device="cuda", generator=g)
    ws = torch.empty(L.query("ctr_feat_embed_bwd_ws", B, F, D) // 4 + 1, device="cuda")
    dW = torch.full_like(W, float("nan"))
    db = torch.full_like(W, float("nan"))
    dP = torch.full_like(P, float("nan"))
    L.call("ctr_feat_embed_bwd", ptr(x), B, F, ptr(W), ptr(bv) if bias else None, ptr(P), fe, D, ptr(dout_t), out_ld,
           ptr(dW), ptr(db) if bias else None, ptr(dP), ptr(ws), st)
    go = dout_t[:, :F * D].double().reshape(B, F, D)
    gh = torch.einsum("bfd,dk->bfk", go, Pd)                       # dL/dh
    r_dW = (gh * xd[:, :, None]).sum(0)
    r_db = gh.sum(0)
    r_dP = torch.einsum("bfd,bfk->dk", go, h)
    torch.cuda.synchronize()
    for name, a, r in (("dW", dW, r_dW), ("dP", dP, r_dP)) + ((("dbias", db, r_db),) if bias else ()):
        assert float((a.double() - r).norm() / r.norm()) < 1e-5, name


@pytest.mark.parametrize("L_,K,D", [(100, 60, 32), (40, 40, 16), (400, 148, 64), (7, 3, 8)])
def test_topk_select_vs_torch(L_, K, D):
    L = _lib()
    B, vocab = 33, 500
    g = torch.Generator().manual_seed(L_)
    E_att = torch.randn(vocab, D, generator=g)
    E_rep = torch.randn(vocab, D, generator=g)
    E_att[0] = 0
    E_rep[0] = 0
    seq = torch.randint(1, vocab, (B, L_), generator=g)
    lens = torch.randint(0, L_ + 1, (B,), generator=g)
    for b in range(B):
        seq[b, : L_ - int(lens[b])] = 0
    q = torch.randn(B, D, generator=g)
    pos = torch.arange(L_)
    dlog = torch.log(torch.exp(-(L_ - 1 - pos).float() / 64.0) + 1e-8)
    sc = (E_att[seq] * q[:, None]).sum(-1) + dlog
    sc = sc.masked_fill(seq == 0, -1e9)
    vals_ref, idx_ref = sc.topk(K, 1)
    cu = lambda t: t.cuda().contiguous()
    seq_d, q_d, Ea, Er, dl = cu(seq.int()), cu(q), cu(E_att), cu(E_rep), cu(dlog)
    idx = torch.empty(B, K, dtype=torch.int32, device="cuda")
    tok = torch.empty(B, K, dtype=torch.int32, device="cuda")
    vals = torch.empty(B, K, device="cuda")
    sel = torch.empty(B, K, D, device="cuda")
    L.call("ctr_dare_topk_fwd", ptr(seq_d), B, L_, ptr(q_d), ptr(Ea), ptr(Er), D, ptr(dl), K, 0, ptr(idx), ptr(tok),
           ptr(vals), ptr(sel), stream())
    torch.cuda.synchronize()
    assert torch.allclose(vals.cpu(), vals_ref, rtol=1e-5, atol=1e-5)
    # index sets agree on the real (non-pad) selections
    for b in range(B):
        real = vals_ref[b] > -1e8
        assert set(idx.cpu()[b][real].tolist()) == set(idx_ref[b][real].tolist())
    sel_ref = torch.gather(E_rep[seq], 1, idx.cpu().long()[..., None].expand(-1, -1, D))
    assert torch.equal(sel.cpu(), sel_ref)


def test_fused_adamw_matches_torch():
    """ctr_adamw_ema on a dense segment == torch.optim.AdamW + clip + EMA arithmetic."""
    L = _lib()
    n = 10_240
    p0 = torch.randn(n)
    g = torch.randn(n)
    p_t = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([p_t], lr=3e-3, weight_decay=1e-2)
    shadow_ref = p0.clone()
    P = p0.cuda().clone()
    Mm, V, E = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda"), p0.cuda().clone()
    G = g.cuda()
    segs = (L.OptSeg * 1)()
    segs[0].p_off, segs[0].n, segs[0].width, segs[0].kind, segs[0].g_off = 0, n, 1, 0, 0
    CH = L.query("ctr_opt_chunk_elems")
    chunks = [(0, e, min(n, e + CH)) for e in range(0, n, CH)]
    carr = (L.OptChunk * len(chunks))()
    for i, (s_, a_, b_) in enumerate(chunks):
        carr[i].seg, carr[i].e0, carr[i].e1 = s_, a_, b_
    to_dev = lambda arr: torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).cuda()
    sd, cd = to_dev(segs), to_dev(carr)
    coef = torch.tensor([0.0, 0.5], device="cuda")
    for step in range(1, 4):
        p_t.grad = g.clone() * 0.5
        opt.step()
        with torch.no_grad():
            shadow_ref.mul_(0.9).add_(p_t.detach(), alpha=0.1)
        kr = torch.zeros(2 * len(chunks), dtype=torch.int32, device="cuda")
        L.call("ctr_adamw_ema", ptr(cd), len(chunks), ptr(sd), ptr(kr), ptr(P), ptr(Mm), ptr(V), ptr(E), ptr(G),
               ptr(coef, 1),
               3e-3, 1e-2, 0.9, 0.999, 1e-8, step, 0.9, 1, 1, stream())
    torch.cuda.synchronize()
    # a few ulp: the kernel's fused multiply-adds vs torch's separately rounded CPU ops
    assert torch.allclose(P.cpu(), p_t.detach(), rtol=1e-6, atol=1e-6)
    assert torch.allclose(E.cpu(), shadow_ref, rtol=1e-6, atol=1e-6)


def ffn_keep_bits(fmask, M, FF, D):
    """(M, FF) keep bits from ctr_ffn_fwd's mask buffer (ffn.hip FfnTile::LW): D <= 32 lane words
    ((chunk, 128-row tile, g, c) dwords, bit 4i + rr of row 128t + 16i + 4g + rr), else chunk-major
    (FF/16, M) uint16 row words."""
    rows, cols = np.arange(M), np.arange(FF)
    if D <= 32:
        T = (M + 127) // 128
        words = fmask.cpu().numpy().view(np.uint32)[:FF // 16 * T * 64].reshape(FF // 16, T, 4, 16)
        w = words[(cols // 16)[None, :], (rows // 128)[:, None], ((rows % 16) // 4)[:, None], (cols % 16)[None, :]]
        return ((w >> (4 * ((rows % 128) // 16) + rows % 4).astype(np.uint32)[:, None]) & 1).astype(bool)
    words = fmask.cpu().numpy().view(np.uint16)[:M * (FF // 16)].reshape(FF // 16, M).T
    return ((words[:, cols // 16] >> (cols % 16).astype(np.uint16)) & 1).astype(bool)


@pytest.mark.parametrize("M,D,FF,p", [(300, 32, 384, 0.1), (1000, 16, 48, 0.1), (130, 64, 384, 0.15),
                                      (4097, 32, 384, 0.0), (64, 32, 16, 0.5), (517, 32, 64, 0.2)])
def test_fused_ffn_vs_torch(M, D, FF, p):
    """ffn.hip: Linear -> GELU -> Dropout -> Linear -> +x -> RMSNorm forward, and its backward
    (dx incl. the residual, per-workgroup [dW1 | db1 | dW2] slabs reduced by ctr_colsum) vs autograd."""
    from oracle.rng import keep_mask
    from tossctr.rng import drop_args
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(M + D + FF)
    x = torch.randn(M, D, device="cuda", generator=g)
    W1 = torch.randn(FF, D, device="cuda", generator=g) / math.sqrt(D)
    b1 = torch.randn(FF, device="cuda", generator=g) * 0.1
    W2 = torch.randn(D, FF, device="cuda", generator=g) / math.sqrt(FF)
    b2 = torch.randn(D, device="cuda", generator=g) * 0.1
    nw = 1 + 0.1 * torch.randn(D, device="cuda", generator=g)
    seed, site = (5 << 32) | 9, 4
    key, thresh, scale = drop_args(seed, site, p, True)
    y, h, r = (torch.empty(M, D, device="cuda"), torch.empty(M, D, device="cuda"), torch.empty(M, device="cuda"))
    fmask = torch.zeros(L.query("ctr_ffn_mask_words", M, FF), dtype=torch.int32, device="cuda")
    L.call("ctr_ffn_fwd", ptr(x), M, D, FF, ptr(W1), ptr(b1), ptr(W2), ptr(b2), ptr(nw), 1e-6, key, thresh, scale,
           ptr(fmask), ptr(y), ptr(h), ptr(r), None, 0, stream())
    mask = torch.from_numpy(keep_mask(seed, site, p, (M, FF)).astype(np.float32)).cuda() if p > 0 else \
        torch.ones(M, FF, device="cuda")
    xr, W1r, b1r, W2r = (t.detach().double().requires_grad_() for t in (x, W1, b1, W2))
    pre = xr @ W1r.t() + b1r
    fo = torch.nn.functional.gelu(pre) * mask.double() * float(np.float32(scale if p > 0 else 1.0))
    hr = xr + (fo @ W2r.t() + b2.double())
    rr = 1.0 / torch.sqrt((hr * hr).mean(1) + 1e-6)
    assert rel(h.double(), hr) < 1e-5
    assert rel(r.double(), rr) < 1e-5
    assert rel(y.double(), nw.double() * hr * rr[:, None]) < 1e-5
    if p > 0:   # stored keep bits == the oracle mask
        assert np.array_equal(ffn_keep_bits(fmask, M, FF, D), mask.cpu().numpy().astype(bool))
    # backward from a random grad wrt h
    dh = torch.randn(M, D, device="cuda", generator=g)
    hr.backward(dh.double())
    dx = torch.empty(M, D, device="cuda")
    nb = L.query("ctr_ffn_slab_rows", M, D, FF, 0)
    o_b1 = FF * D
    o_w2 = o_b1 + (FF + 63) // 64 * 64
    ld = o_w2 + D * FF
    slab = torch.zeros(nb, ld, device="cuda")
    L.call("ctr_ffn_bwd", ptr(x), ptr(dh), M, D, FF, ptr(W1), ptr(b1), ptr(W2), key, thresh, scale, ptr(fmask),
           ptr(dx), ptr(slab), ld, o_b1, o_w2, None, 0, stream())
    red = slab.double().sum(0)
    assert rel(dx.double(), xr.grad) < 1e-5
    assert rel(red[:FF * D].view(FF, D), W1r.grad) < 1e-5
    assert rel(red[o_b1:o_b1 + FF], b1r.grad) < 1e-5
    assert rel(red[o_w2:o_w2 + D * FF].view(D, FF), W2r.grad) < 1e-5
    assert float(red[o_b1 + FF:o_w2].abs().max()) == 0.0 if o_w2 > o_b1 + FF else True


@pytest.mark.parametrize("M,D,FF,p", [(300, 32, 384, 0.1), (1000, 16, 48, 0.1), (130, 64, 384, 0.15),
                                      (4097, 32, 384, 0.0), (64, 32, 16, 0.5)])
def test_ffn_bwd_norms_vs_torch(M, D, FF, p):
    """ctr_ffn_bwd_norms: the encoder layer's norm2 backward -> FFN backward (+ residual) -> norm1
    backward in one kernel (dare.py:53-70, norm_first=False) vs autograd through
    h1 -> x1 = RMSNorm(h1; n1) -> h2 = x1 + FFN(x1) -> x2 = RMSNorm(h2; n2): dh1 and the six parameter
    grads from the per-workgroup slab (arena order, padding gaps stay zero)."""
    from oracle.rng import keep_mask
    from tossctr.rng import drop_args
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(7 * M + D + FF)
    h1 = torch.randn(M, D, device="cuda", generator=g) * 1.5
    W1 = torch.randn(FF, D, device="cuda", generator=g) / math.sqrt(D)
    b1 = torch.randn(FF, device="cuda", generator=g) * 0.1
    W2 = torch.randn(D, FF, device="cuda", generator=g) / math.sqrt(FF)
    b2 = torch.randn(D, device="cuda", generator=g) * 0.1
    n1 = 1 + 0.1 * torch.randn(D, device="cuda", generator=g)
    n2 = 1 + 0.1 * torch.randn(D, device="cuda", generator=g)
    seed, site = (3 << 32) | 11, 6
    key, thresh, scale = drop_args(seed, site, p, True)
    r1 = 1.0 / torch.sqrt((h1 * h1).mean(1) + 1e-6)
    x1 = (n1 * h1 * r1[:, None]).contiguous()
    x2, h2, r2 = (torch.empty(M, D, device="cuda"), torch.empty(M, D, device="cuda"), torch.empty(M, device="cuda"))
    fmask = torch.zeros(L.query("ctr_ffn_mask_words", M, FF), dtype=torch.int32, device="cuda")
    L.call("ctr_ffn_fwd", ptr(x1), M, D, FF, ptr(W1), ptr(b1), ptr(W2), ptr(b2), ptr(n2), 1e-6, key, thresh, scale,
           ptr(fmask), ptr(x2), ptr(h2), ptr(r2), None, 0, stream())
    mask = torch.from_numpy(keep_mask(seed, site, p, (M, FF)).astype(np.float32)).cuda() if p > 0 else \
        torch.ones(M, FF, device="cuda")
    h1r, W1r, b1r, W2r, b2r, n1r, n2r = (t.detach().double().requires_grad_() for t in (h1, W1, b1, W2, b2, n1, n2))
    x1r = n1r * h1r / torch.sqrt((h1r * h1r).mean(1, keepdim=True) + 1e-6)
    fo = torch.nn.functional.gelu(x1r @ W1r.t() + b1r) * mask.double() * float(np.float32(scale if p > 0 else 1.0))
    h2r = x1r + (fo @ W2r.t() + b2r)
    x2r = n2r * h2r / torch.sqrt((h2r * h2r).mean(1, keepdim=True) + 1e-6)
    dy = torch.randn(M, D, device="cuda", generator=g)
    x2r.backward(dy.double())
    # slab in an arena-like layout with 64-float alignment gaps
    al = lambda v: (v + 63) // 64 * 64
    o_n1 = 0
    o_w1 = al(o_n1 + D)
    o_b1 = al(o_w1 + FF * D)
    o_w2 = al(o_b1 + FF)
    o_b2 = al(o_w2 + D * FF)
    o_n2 = al(o_b2 + D)
    ld = o_n2 + D
    nb = L.query("ctr_ffn_slab_rows", M, D, FF, 0)
    slab = torch.zeros(nb, ld, device="cuda")
    dh1 = torch.empty(M, D, device="cuda")
    L.call("ctr_ffn_bwd_norms", ptr(x1), ptr(dy), ptr(h2), ptr(r2), ptr(n2), ptr(h1), ptr(r1), ptr(n1), M, D, FF,
           ptr(W1), ptr(b1), ptr(W2), key, thresh, scale, ptr(fmask), ptr(dh1), ptr(slab), ld,
           o_n1, o_w1, o_b1, o_w2, o_b2, o_n2, None, 0, stream())
    red = slab.double().sum(0)
    assert rel(dh1.double(), h1r.grad) < 1e-5
    assert rel(red[o_n1:o_n1 + D], n1r.grad) < 1e-5
    assert rel(red[o_w1:o_w1 + FF * D].view(FF, D), W1r.grad) < 1e-5
    assert rel(red[o_b1:o_b1 + FF], b1r.grad) < 1e-5
    assert rel(red[o_w2:o_w2 + D * FF].view(D, FF), W2r.grad) < 1e-5
    assert rel(red[o_b2:o_b2 + D], b2r.grad) < 1e-5
    assert rel(red[o_n2:o_n2 + D], n2r.grad) < 1e-5
    used = torch.zeros(ld, dtype=torch.bool)
    for o, n in ((o_n1, D), (o_w1, FF * D), (o_b1, FF), (o_w2, D * FF), (o_b2, D), (o_n2, D)):
        used[o:o + n] = True
    gaps = slab[:, ~used.cuda()]
    assert gaps.numel() == 0 or float(gaps.abs().max()) == 0.0


def ffn_keep_bits_bf(fmask, M, FF):
    """(M, FF) keep bits of the amp bf16 FFN kernels (ffn.hip "row words"): word
    (chunk * nb16 + row // 16) * 16 + row % 16 holds bit f for column 32 chunk + f."""
    nb16 = (M + 15) // 16
    words = fmask.cpu().numpy().view(np.uint32)[:FF // 32 * nb16 * 16].reshape(FF // 32, nb16 * 16)
    rows, cols = np.arange(M), np.arange(FF)
    w = words[(cols // 32)[None, :], rows[:, None]]
    return ((w >> (cols % 32).astype(np.uint32)[None, :]) & 1).astype(bool)


def _bfr(t):
    return t.to(torch.bfloat16).double()


def ffn_ref_bf16(x, W1, b1, W2, b2, keep, dh):
    """fp64 reference of the amp bf16 FFN: every product's operands rounded to bf16 (RNE), exact GELU,
    fp32-kept residual; returns h and, for the grad dh wrt h, (dx, dW1, db1, dW2)."""
    pre = _bfr(x) @ _bfr(W1).t() + b1.double()
    cdf = 0.5 * (1 + torch.special.erf(pre / math.sqrt(2.0)))
    fo = pre * cdf * keep
    h = x.double() + (_bfr(fo) @ _bfr(W2).t() + b2.double())
    dfo = _bfr(dh) @ _bfr(W2)
    gg = cdf + pre * torch.exp(-0.5 * pre * pre) / math.sqrt(2 * math.pi)
    da = dfo * keep * gg
    # db1: the reference's bias grad sums its bf16 grad_output (the bf16-rounded dact); the column-owner
    # backward sums the fp32 dact -- both forms are returned, a kernel must match one (rel_db1)
    return h, (_bfr(da) @ _bfr(W1) + dh.double(), _bfr(da).t() @ _bfr(x), (_bfr(da).sum(0), da.sum(0)),
               _bfr(dh).t() @ _bfr(fo))


def rel_db1(got, refs):
    return min(rel(got, r) for r in refs)


BF_TOL = 2e-4     # bf16 emulation: only rare rounding-boundary flips of an operand element differ


@pytest.mark.parametrize("M,D,FF,p", [(300, 32, 384, 0.1), (130, 64, 384, 0.15), (4097, 32, 384, 0.0),
                                      (517, 32, 64, 0.2), (64, 32, 32, 0.5), (70001, 32, 384, 0.1),
                                      (140003, 64, 96, 0.1), (70001, 64, 384, 0.1), (4097, 64, 128, 0.15),
                                      (9001, 64, 256, 0.0), (606208, 64, 384, 0.15)])
def test_fused_ffn_bf16_vs_emulation(M, D, FF, p):
    """amp bf16 FFN kernels (CTR_FFN_BF16) vs an fp64 emulation with bf16-rounded product operands; the
    persistent backward (M > 512 tiles: several tiles per workgroup, slab rows accumulated) included."""
    from oracle.rng import keep_mask
    from tossctr.rng import drop_args
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(M + D + FF + 1)
    x = torch.randn(M, D, device="cuda", generator=g)
    W1 = torch.randn(FF, D, device="cuda", generator=g) / math.sqrt(D)
    b1 = torch.randn(FF, device="cuda", generator=g) * 0.1
    W2 = torch.randn(D, FF, device="cuda", generator=g) / math.sqrt(FF)
    b2 = torch.randn(D, device="cuda", generator=g) * 0.1
    nw = 1 + 0.1 * torch.randn(D, device="cuda", generator=g)
    seed, site = (5 << 32) | 9, 4
    key, thresh, scale = drop_args(seed, site, p, True)
    y, h, r = (torch.empty(M, D, device="cuda"), torch.empty(M, D, device="cuda"), torch.empty(M, device="cuda"))
    fmask = torch.zeros(L.query("ctr_ffn_mask_words", M, FF), dtype=torch.int32, device="cuda")
    wbf = torch.empty(3 * FF * D, dtype=torch.bfloat16, device="cuda")
    L.call("ctr_ffn_fwd", ptr(x), M, D, FF, ptr(W1), ptr(b1), ptr(W2), ptr(b2), ptr(nw), 1e-6, key, thresh, scale,
           ptr(fmask), ptr(y), ptr(h), ptr(r), ptr(wbf), 1, stream())
    # the weight images the backward reads
    assert torch.equal(wbf[:FF * D].view(FF, D), W1.to(torch.bfloat16))
    assert torch.equal(wbf[FF * D:2 * FF * D].view(FF, D), W2.t().to(torch.bfloat16))
    assert torch.equal(wbf[2 * FF * D:].view(D, FF), W1.t().to(torch.bfloat16))
    km = keep_mask(seed, site, p, (M, FF)) if p > 0 else np.ones((M, FF), bool)
    keep = torch.from_numpy(km.astype(np.float64)).cuda() * float(np.float32(scale if p > 0 else 1.0))
    dh = torch.randn(M, D, device="cuda", generator=g)
    hr, (dxr, dW1r, db1r, dW2r) = ffn_ref_bf16(x, W1, b1, W2, b2, keep, dh)
    rr = 1.0 / torch.sqrt((hr * hr).mean(1) + 1e-6)
    assert rel(h.double(), hr) < BF_TOL
    assert rel(r.double(), rr) < BF_TOL
    assert rel(y.double(), nw.double() * hr * rr[:, None]) < BF_TOL
    if p > 0:
        assert np.array_equal(ffn_keep_bits_bf(fmask, M, FF), km)
    dx = torch.empty(M, D, device="cuda")
    nb = L.query("ctr_ffn_slab_rows", M, D, FF, 1)
    assert nb <= 512
    o_b1 = FF * D
    o_w2 = o_b1 + (FF + 63) // 64 * 64
    ld = o_w2 + D * FF
    slab = torch.full((nb, ld), float("nan"), device="cuda")       # every used entry must be written
    slab[:, o_b1 + FF:o_w2] = 0
    L.call("ctr_ffn_bwd", ptr(x), ptr(dh), M, D, FF, ptr(W1), ptr(b1), ptr(W2), key, thresh, scale, ptr(fmask),
           ptr(dx), ptr(slab), ld, o_b1, o_w2, ptr(wbf), 1, stream())
    red = slab.double().sum(0)
    assert rel(dx.double(), dxr) < BF_TOL
    assert rel(red[:FF * D].view(FF, D), dW1r) < BF_TOL
    assert rel_db1(red[o_b1:o_b1 + FF], db1r) < BF_TOL
    assert rel(red[o_w2:o_w2 + D * FF].view(D, FF), dW2r) < BF_TOL
    # deterministic: a second run is bitwise identical
    slab2 = torch.empty_like(slab)
    slab2[:, o_b1 + FF:o_w2] = 0
    dx2 = torch.empty_like(dx)
    L.call("ctr_ffn_bwd", ptr(x), ptr(dh), M, D, FF, ptr(W1), ptr(b1), ptr(W2), key, thresh, scale, ptr(fmask),
           ptr(dx2), ptr(slab2), ld, o_b1, o_w2, ptr(wbf), 1, stream())
    assert torch.equal(dx, dx2) and torch.equal(slab, slab2)


@pytest.mark.parametrize("M,D,FF,p", [(300, 32, 384, 0.1), (130, 64, 384, 0.15), (70001, 32, 384, 0.1),
                                      (70001, 64, 64, 0.0), (70001, 64, 384, 0.15), (33, 64, 128, 0.1),
                                      (20000, 64, 256, 0.0)])
def test_ffn_bwd_norms_bf16_vs_emulation(M, D, FF, p):
    """ctr_ffn_bwd_norms with CTR_FFN_BF16: norm2 backward -> bf16 FFN backward -> norm1 backward, the six
    parameter grads accumulated over each persistent workgroup's tiles."""
    from oracle.rng import keep_mask
    from tossctr.rng import drop_args
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(7 * M + D + FF + 1)
    h1 = torch.randn(M, D, device="cuda", generator=g) * 1.5
    W1 = torch.randn(FF, D, device="cuda", generator=g) / math.sqrt(D)
    b1 = torch.randn(FF, device="cuda", generator=g) * 0.1
    W2 = torch.randn(D, FF, device="cuda", generator=g) / math.sqrt(FF)
    b2 = torch.randn(D, device="cuda", generator=g) * 0.1
    n1 = 1 + 0.1 * torch.randn(D, device="cuda", generator=g)
    n2 = 1 + 0.1 * torch.randn(D, device="cuda", generator=g)
    seed, site = (3 << 32) | 11, 6
    key, thresh, scale = drop_args(seed, site, p, True)
    r1 = 1.0 / torch.sqrt((h1 * h1).mean(1) + 1e-6)
    x1 = (n1 * h1 * r1[:, None]).contiguous()
    x2, h2, r2 = (torch.empty(M, D, device="cuda"), torch.empty(M, D, device="cuda"), torch.empty(M, device="cuda"))
    fmask = torch.zeros(L.query("ctr_ffn_mask_words", M, FF), dtype=torch.int32, device="cuda")
    wbf = torch.empty(3 * FF * D, dtype=torch.bfloat16, device="cuda")
    L.call("ctr_ffn_fwd", ptr(x1), M, D, FF, ptr(W1), ptr(b1), ptr(W2), ptr(b2), ptr(n2), 1e-6, key, thresh, scale,
           ptr(fmask), ptr(x2), ptr(h2), ptr(r2), ptr(wbf), 1, stream())
    km = keep_mask(seed, site, p, (M, FF)) if p > 0 else np.ones((M, FF), bool)
    keep = torch.from_numpy(km.astype(np.float64)).cuda() * float(np.float32(scale if p > 0 else 1.0))
    dy = torch.randn(M, D, device="cuda", generator=g)
    # norm2 backward in fp64 on the kernel's own h2 (its forward is checked above)
    h2v, n2r = h2.double().requires_grad_(), n2.double().requires_grad_()
    (n2r * h2v / torch.sqrt((h2v * h2v).mean(1, keepdim=True) + 1e-6)).backward(dy.double())
    dh2 = h2v.grad
    _, (dx1, dW1r, db1r, dW2r) = ffn_ref_bf16(x1, W1, b1, W2, b2, keep, dh2)
    h1r, n1r = h1.double().requires_grad_(), n1.double().requires_grad_()
    (n1r * h1r / torch.sqrt((h1r * h1r).mean(1, keepdim=True) + 1e-6)).backward(dx1)
    al = lambda v: (v + 63) // 64 * 64
    o_n1 = 0
    o_w1 = al(o_n1 + D)
    o_b1 = al(o_w1 + FF * D)
    o_w2 = al(o_b1 + FF)
    o_b2 = al(o_w2 + D * FF)
    o_n2 = al(o_b2 + D)
    ld = o_n2 + D
    nb = L.query("ctr_ffn_slab_rows", M, D, FF, 1)
    slab = torch.zeros(nb, ld, device="cuda")
    dh1 = torch.empty(M, D, device="cuda")
    L.call("ctr_ffn_bwd_norms", ptr(x1), ptr(dy), ptr(h2), ptr(r2), ptr(n2), ptr(h1), ptr(r1), ptr(n1), M, D, FF,
           ptr(W1), ptr(b1), ptr(W2), key, thresh, scale, ptr(fmask), ptr(dh1), ptr(slab), ld,
           o_n1, o_w1, o_b1, o_w2, o_b2, o_n2, ptr(wbf), 1, stream())
    red = slab.double().sum(0)
    assert rel(dh1.double(), h1r.grad) < BF_TOL
    assert rel(red[o_n1:o_n1 + D], n1r.grad) < BF_TOL
    assert rel(red[o_w1:o_w1 + FF * D].view(FF, D), dW1r) < BF_TOL
    assert rel_db1(red[o_b1:o_b1 + FF], db1r) < BF_TOL
    assert rel(red[o_w2:o_w2 + D * FF].view(D, FF), dW2r) < BF_TOL
    assert rel(red[o_b2:o_b2 + D], dh2.sum(0)) < BF_TOL
    assert rel(red[o_n2:o_n2 + D], n2r.grad) < BF_TOL


@pytest.mark.parametrize("B,F,D,QR", [(37, 23, 16, 8), (64, 200, 32, 96), (9, 27, 64, 96), (5, 3, 32, 20)])
def test_qnn_gram_vs_torch(B, F, D, QR):
    """qnn.hip Gram form of _pair_interaction_all (src/models/qnn_alpha.py:86-97) vs the A = z @ U
    formulation with autograd: S, quad, dz (incl. the added residual grad) and dUcat."""
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(B * F + D)
    z = torch.randn(B, F, D, device="cuda", generator=g)
    U = torch.randn(D, QR, device="cuda", generator=g) * 0.1
    zsum, G = torch.empty(B, D, device="cuda"), torch.empty(B, D * D, device="cuda")
    S, quad = torch.empty(B, QR, device="cuda"), torch.empty(B, QR, device="cuda")
    L.call("ctr_qnn_gram_fwd", ptr(z), B, F, D, ptr(U), QR, ptr(zsum), ptr(G), ptr(S), ptr(quad), stream())
    zr, Ur = z.double().requires_grad_(), U.double().requires_grad_()
    A = zr @ Ur
    s_ref = A.sum(1)
    q_ref = s_ref * s_ref - (A * A).sum(1)
    assert rel(S.double(), s_ref.detach()) < 1e-5
    assert rel(quad.double(), q_ref.detach()) < 1e-5
    assert rel(G.double().view(B, D, D), (zr.transpose(1, 2) @ zr).detach()) < 1e-5
    dquad = torch.randn(B, QR, device="cuda", generator=g)
    dz_add = torch.randn(B, F, D, device="cuda", generator=g)
    q_ref.backward(dquad.double())
    dz, DS = torch.empty(B, F, D, device="cuda"), torch.empty(B, QR, device="cuda")
    L.call("ctr_qnn_gram_bwd", ptr(z), B, F, D, ptr(U), QR, ptr(S), ptr(dquad), ptr(dz_add), 0, ptr(dz), ptr(DS),
           stream())
    assert rel(dz.double(), zr.grad + dz_add.double()) < 1e-5
    # amp: the addend (the QNN MLP's input grad) arrives as bf16; the same sums with its values widened
    dz_add_bf = dz_add.bfloat16()
    dz2 = torch.empty_like(dz)
    L.call("ctr_qnn_gram_bwd", ptr(z), B, F, D, ptr(U), QR, ptr(S), ptr(dquad), ptr(dz_add_bf), 1, ptr(dz2), ptr(DS),
           stream())
    assert rel(dz2.double(), zr.grad + dz_add_bf.double()) < 1e-5
    T1 = (zsum.t() @ DS).contiguous()
    T = (G.t() @ dquad).contiguous()
    du = torch.empty(D, QR, device="cuda")
    L.call("ctr_qnn_du_combine", ptr(T1), ptr(T), ptr(U), D, QR, ptr(du), stream())
    assert rel(du.double(), Ur.grad) < 1e-5


@pytest.mark.parametrize("B,F,D,QR", [(64, 200, 32, 96), (4096, 200, 32, 96), (9, 27, 64, 96), (5, 3, 32, 20),
                                      (37, 33, 32, 8), (16, 40, 64, 40)])
def test_qnn_gram_zbf_vs_fp64(B, F, D, QR):
    """amp: the pair interaction on bf16(z) read from the [z | inter] bf16 image (ctr_qnn_gram_fwd_zbf / _bwd_zbf):
    forward S, quad, G, zsum = the exact function of bf16(z) (fp64 reference of the same bf16 values, 1e-5); backward
    dz against an fp64 emulation with M = U diag(dquad) U^T rounded to bf16 as the kernel's product takes it (1e-4)
    and against the exact gradient of the bf16-z function (bf16-level, 1e-2); B = 4096 / F = 200 / QR = 96 is cfg2's."""
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(B * F + D + 7)
    ldz = F * D + 24                                   # the image's row: z, then the interaction columns
    img = torch.randn(B, ldz, device="cuda", generator=g).bfloat16()
    zb = img[:, :F * D].reshape(B, F, D)
    U = torch.randn(D, QR, device="cuda", generator=g) * 0.1
    zsum, G = torch.empty(B, D, device="cuda"), torch.empty(B, D * D, device="cuda")
    S, quad = torch.empty(B, QR, device="cuda"), torch.empty(B, QR, device="cuda")
    L.call("ctr_qnn_gram_fwd_zbf", ptr(img), ldz, B, F, D, ptr(U), QR, ptr(zsum), ptr(G), ptr(S), ptr(quad), 0,
           stream())
    zr, Ur = zb.double().requires_grad_(), U.double()
    A = zr @ Ur
    s_ref = A.sum(1)
    q_ref = s_ref * s_ref - (A * A).sum(1)
    assert rel(zsum.double(), zr.detach().sum(1)) < 1e-6
    assert rel(G.double().view(B, D, D), (zr.transpose(1, 2) @ zr).detach()) < 1e-6
    assert rel(S.double(), s_ref.detach()) < 1e-5
    assert rel(quad.double(), q_ref.detach()) < 1e-5
    dquad = torch.randn(B, QR, device="cuda", generator=g)
    dz_add = torch.randn(B, F, D, device="cuda", generator=g).bfloat16()
    q_ref.backward(dquad.double())
    dz, DS = torch.full((B, F, D), float("nan"), device="cuda"), torch.empty(B, QR, device="cuda")
    L.call("ctr_qnn_gram_bwd_zbf", ptr(img), ldz, F * D, B, F, D, ptr(U), QR, ptr(S), ptr(dquad), ptr(dz_add), 1,
           ptr(dz), ptr(DS), stream())
    torch.cuda.synchronize()
    dqd = dquad.double()
    M = torch.einsum("dk,bk,ek->bde", Ur, dqd, Ur)
    Mb = M.float().bfloat16().double()            # the kernel forms M in fp32, then rounds it to bf16
    w = 2.0 * torch.einsum("dk,bk->bd", Ur, dqd * S.double())
    emu = w[:, None, :] - 2.0 * torch.einsum("bfd,bde->bfe", zr.detach(), Mb) + dz_add.double()
    # (an fp32 M within ~1e-7 of a bf16 rounding midpoint may round the other way than the fp64-then-fp32 emulation's)
    assert rel(dz.double(), emu) < 1e-4
    assert rel(dz.double(), zr.grad + dz_add.double()) < 1e-2
    assert rel(DS.double(), dqd * S.double()) < 1e-6


def test_qnn_vfull_roundtrip():
    L = _lib()
    H, R, P = 3, 4, 5
    V = torch.randn(H, R, P, device="cuda")
    vf = torch.full((H * R, H * P), 7.0, device="cuda")
    L.call("ctr_qnn_vfull", ptr(V), H, R, P, ptr(vf), 0, stream())
    ref = torch.block_diag(*[V[h] for h in range(H)])
    assert torch.equal(vf, ref)
    back = torch.empty_like(V)
    L.call("ctr_qnn_vfull", ptr(vf), H, R, P, ptr(back), 1, stream())
    assert torch.equal(back, V)


@pytest.mark.parametrize("K,N", [(32, 96), (32, 32), (96, 32), (16, 48), (48, 16), (16, 16)])
@pytest.mark.parametrize("M", [1000, 77])
def test_rowgemm_vs_torch(K, N, M):
    """rowgemm.hip: C = A W^T (+bias) / A W (+add) / fused residual + RMSNorm, vs torch fp64."""
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(K * 1000 + N + M)
    A = torch.randn(M, K, device="cuda", generator=g)
    Wt = torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)      # nn.Linear layout (tb = 1)
    Wn = torch.randn(K, N, device="cuda", generator=g) / math.sqrt(K)      # (K, N) layout (tb = 0)
    b = torch.randn(N, device="cuda", generator=g)
    add = torch.randn(M, N, device="cuda", generator=g)
    C = torch.full((M, N), float("nan"), device="cuda")
    st = stream()
    L.call("ctr_rowgemm", M, K, N, ptr(A), K, ptr(Wt), 1, ptr(C), N, ptr(b), None, 0, None, 0, None, None, None, 0.0, st)
    assert rel(C.double(), A.double() @ Wt.double().t() + b.double()) < 1e-6
    L.call("ctr_rowgemm", M, K, N, ptr(A), K, ptr(Wn), 0, ptr(C), N, None, ptr(add), N, None, 0, None, None, None, 0.0,
           st)
    assert rel(C.double(), A.double() @ Wn.double() + add.double()) < 1e-6
    if K == N:      # out_proj: residual + RMSNorm epilogue
        res = torch.randn(M, N, device="cuda", generator=g)
        w = torch.rand(N, device="cuda", generator=g) + 0.5
        h, r = torch.empty(M, N, device="cuda"), torch.empty(M, device="cuda")
        L.call("ctr_rowgemm", M, K, N, ptr(A), K, ptr(Wt), 1, ptr(C), N, ptr(b), None, 0, ptr(res), N, ptr(w), ptr(h),
               ptr(r), 1e-6, st)
        h_ref = res.double() + (A.double() @ Wt.double().t() + b.double())
        r_ref = torch.rsqrt(h_ref.pow(2).mean(-1) + 1e-6)
        assert rel(h.double(), h_ref) < 1e-6 and rel(r.double(), r_ref) < 1e-6
        assert rel(C.double(), w.double() * h_ref * r_ref[:, None]) < 1e-6


@pytest.mark.parametrize("NO,NIN", [(96, 32), (32, 32), (48, 16), (16, 16)])
@pytest.mark.parametrize("M", [245760, 1001, 5])
def test_rowgemm_wgrad_vs_torch(NO, NIN, M):
    """dW = dY^T X and db = colsum(dY) in one pass, slab rows reduced by ctr_colsum, vs torch fp64."""
    L = _lib()
    if M == 245760 and NO != 96:
        pytest.skip("full size checked once")
    g = torch.Generator(device="cuda").manual_seed(NO + NIN + M)
    dY = torch.randn(M, NO, device="cuda", generator=g)
    X = torch.randn(M, NIN, device="cuda", generator=g)
    o_db = NO * NIN + 8                     # a padding gap before the bias, as in the grad arena
    n_sl = o_db + NO
    ld = (n_sl + 3) // 4 * 4
    rows = L.query("ctr_rowgemm_wgrad_rows", M)
    slab = torch.zeros(rows, ld, device="cuda")
    L.call("ctr_rowgemm_wgrad", ptr(dY), NO, ptr(X), NIN, M, NO, NIN, ptr(slab), ld, o_db, stream())
    out = torch.full((n_sl,), float("nan"), device="cuda")
    ws = torch.empty(L.query("ctr_colsum_ws_size", rows, n_sl) // 4 + 1, device="cuda")
    L.call("ctr_colsum", ptr(slab), ld, rows, n_sl, 1.0, ptr(out), ptr(ws), stream())
    assert rel(out[:NO * NIN].double().view(NO, NIN), dY.double().t() @ X.double()) < 1e-6
    assert rel(out[o_db:].double(), dY.double().sum(0)) < 1e-6
    assert float(out[NO * NIN:o_db].abs().max()) == 0.0


@pytest.mark.parametrize("M,N", [(1000, 16), (77, 32), (300, 64), (50, 100), (40, 300), (33, 2000), (64, 6400),
                                  (9, 12800), (5000, 64)])
def test_layernorm_vs_torch(M, N):
    """layernorm.hip (norm != "rms": nn.LayerNorm, eps 1e-5): y, the saved mean / rstd, y's bf16 image, and the
    backward's dx (+ add) and dw / db partial rows against torch fp64, for every row-width form."""
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(M * 13 + N)
    x = torch.randn(M, N, device="cuda", generator=g) * 2 + 0.5
    w = 1 + 0.2 * torch.randn(N, device="cuda", generator=g)
    b = 0.1 * torch.randn(N, device="cuda", generator=g)
    y = torch.full((M, N), float("nan"), device="cuda")
    mu, rs = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
    ybf = torch.empty(M, N + 8, device="cuda", dtype=torch.bfloat16)
    L.call("ctr_layernorm_fwd", ptr(x), N, M, N, ptr(w), ptr(b), 1e-5, ptr(y), N, ptr(mu), ptr(rs), ptr(ybf), N + 8,
           stream())
    xd = x.double().requires_grad_(True)
    wd, bd = w.double().requires_grad_(True), b.double().requires_grad_(True)
    ref = torch.nn.functional.layer_norm(xd, (N,), wd, bd, 1e-5)
    assert rel(y.double(), ref.detach()) < 1e-6
    assert rel(mu.double(), x.double().mean(-1)) < 1e-6
    assert rel(rs.double(), torch.rsqrt(x.double().var(-1, unbiased=False) + 1e-5)) < 1e-6
    assert torch.equal(ybf[:, :N], y.to(torch.bfloat16))
    dy = torch.randn(M, N, device="cuda", generator=g)
    add = torch.randn(M, N, device="cuda", generator=g)
    ref.backward(dy.double())
    nparts = L.query("ctr_layernorm_bwd_nparts", M, N)
    dwp = torch.full((nparts, N), float("nan"), device="cuda")
    dbp = torch.full((nparts, N), float("nan"), device="cuda")
    dx = torch.full((M, N), float("nan"), device="cuda")
    L.call("ctr_layernorm_bwd", ptr(dy), N, ptr(x), N, ptr(mu), ptr(rs), ptr(w), M, N, ptr(dx), N, ptr(add), N,
           ptr(dwp), ptr(dbp), stream())
    assert rel(dx.double(), xd.grad + add.double()) < 1e-5
    assert rel(dwp.double().sum(0), wd.grad) < 1e-5
    assert rel(dbp.double().sum(0), bd.grad) < 1e-5


@pytest.mark.parametrize("nparts,n,H", [(8192, 297, 8), (4096, 201, 4), (13, 65, 2), (1, 3, 4), (0, 9, 4)])
def test_pos_bias_grad_vs_torch(nparts, n, H):
    """ctr_pos_bias_grad: drel[d, h] = sum_p part[p, d] / H for every head (the head-mean bias's grad), the
    partials reduced in place in chunks; (8192, 297): cfg4's B x head groups and 2 top_k + 1."""
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(nparts + n)
    part = torch.randn(max(nparts, 1), n, device="cuda", generator=g)
    ref = part[:nparts].double().sum(0) / H
    drel = torch.full((n, H), float("nan"), device="cuda")
    L.call("ctr_pos_bias_grad", ptr(part), nparts, H, n, ptr(drel), stream())
    assert rel(drel.double(), ref[:, None].expand(n, H)) < 1e-6 if nparts else float(drel.abs().max()) == 0.0


@pytest.mark.parametrize("M,N", [(300, 20), (300, 64), (77, 1000), (64, 5000), (4096, 9024), (33, 16384),
                                  (17, 20000)])
def test_rmsnorm_bwd_vs_torch(M, N):
    """ctr_rmsnorm_bwd (dh and the per-block dw partials) vs torch fp64 for every row-width form: small rows,
    256-thread rows, the 16-byte forms up to 8192 and (1024 threads) 16384 wide, the two-pass fallback beyond.
    (4096, 9024): a QNN input norm width of the cfg4 shape class."""
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N)
    dy = torch.randn(M, N, device="cuda", generator=g)
    h = torch.randn(M, N, device="cuda", generator=g)
    w = torch.rand(N, device="cuda", generator=g) + 0.5
    r = torch.rsqrt(h.double().pow(2).mean(-1) + 1e-6).float()
    nparts = L.query("ctr_rmsnorm_bwd_nparts", M, N)
    dwp = torch.full((nparts, N), float("nan"), device="cuda")
    dh = torch.full((M, N), float("nan"), device="cuda")
    L.call("ctr_rmsnorm_bwd", ptr(dy), N, ptr(h), N, ptr(r), ptr(w), M, N, ptr(dh), N, None, 0, ptr(dwp), stream())
    gd, hd, rd, wd = dy.double(), h.double(), r.double()[:, None], w.double()
    dot = (wd * gd * hd).sum(-1, keepdim=True)
    ref = wd * gd * rd - hd * rd.pow(3) / N * dot
    assert rel(dh.double(), ref) < 1e-5
    assert rel(dwp.double().sum(0), (gd * hd * rd).sum(0)) < 1e-5


@pytest.mark.parametrize("K,N", [(64, 192), (64, 64), (192, 64)])
@pytest.mark.parametrize("M", [606208, 1000, 77, 5])
def test_rowgemm_bf_vs_emulation(K, N, M):
    """rowgemm_bf.hip (amp, D = 64): C = A W^T (+bias) / A W (+add) / fused residual + RMSNorm on bf16-rounded
    operands, vs an fp64 emulation with the same rounded operands (only the fp32 summation order differs).
    M = 606,208 is cfg4's B*K (4096 x 148): the persistent walk over every row block."""
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(K * 1000 + N + M)
    A = torch.randn(M, K, device="cuda", generator=g)
    Wt = torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)      # nn.Linear layout (tb = 1)
    Wn = torch.randn(K, N, device="cuda", generator=g) / math.sqrt(K)      # (K, N) layout (tb = 0)
    b = torch.randn(N, device="cuda", generator=g)
    add = torch.randn(M, N, device="cuda", generator=g)
    C = torch.full((M, N), float("nan"), device="cuda")
    st = stream()
    Ab = _bfr(A)
    L.call("ctr_rowgemm_bf", M, K, N, ptr(A), K, ptr(Wt), 1, ptr(C), N, ptr(b), None, 0, None, 0, None, None, None,
           0.0, st)
    assert rel(C.double(), Ab @ _bfr(Wt).t() + b.double()) < 1e-6
    L.call("ctr_rowgemm_bf", M, K, N, ptr(A), K, ptr(Wn), 0, ptr(C), N, None, ptr(add), N, None, 0, None, None, None,
           0.0, st)
    assert rel(C.double(), Ab @ _bfr(Wn) + add.double()) < 1e-6
    # an fp32 product would differ from the bf16 one by ~2^-9 relative: the emulation pins the operand rounding
    assert rel(C.double(), A.double() @ Wn.double() + add.double()) > 1e-4
    # tb = 1 with bias AND add: the LayerNorm encoder's out_proj + residual h = x + o W^T + b (engine.py, amp D = 64)
    L.call("ctr_rowgemm_bf", M, K, N, ptr(A), K, ptr(Wt), 1, ptr(C), N, ptr(b), ptr(add), N, None, 0, None, None, None,
           0.0, st)
    assert rel(C.double(), Ab @ _bfr(Wt).t() + b.double() + add.double()) < 1e-6
    if K == N:      # out_proj: residual + RMSNorm epilogue
        res = torch.randn(M, N, device="cuda", generator=g)
        w = torch.rand(N, device="cuda", generator=g) + 0.5
        h, r = torch.empty(M, N, device="cuda"), torch.empty(M, device="cuda")
        L.call("ctr_rowgemm_bf", M, K, N, ptr(A), K, ptr(Wt), 1, ptr(C), N, ptr(b), None, 0, ptr(res), N, ptr(w),
               ptr(h), ptr(r), 1e-6, st)
        h_ref = res.double() + (Ab @ _bfr(Wt).t() + b.double())
        r_ref = torch.rsqrt(h_ref.pow(2).mean(-1) + 1e-6)
        assert rel(h.double(), h_ref) < 1e-6 and rel(r.double(), r_ref) < 1e-6
        assert rel(C.double(), w.double() * h_ref * r_ref[:, None]) < 1e-6


@pytest.mark.parametrize("NO,NIN", [(192, 64), (64, 64)])
@pytest.mark.parametrize("M", [606208, 1001, 5])
def test_rowgemm_bf_wgrad_vs_emulation(NO, NIN, M):
    """amp, D = 64: dW = dY^T X on bf16-rounded operands (fp64 emulation) and db = colsum of the fp32 dY, slab
    rows reduced by ctr_colsum."""
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(NO + NIN + M)
    dY = torch.randn(M, NO, device="cuda", generator=g)
    X = torch.randn(M, NIN, device="cuda", generator=g)
    o_db = NO * NIN + 8                     # a padding gap before the bias, as in the grad arena
    n_sl = o_db + NO
    ld = (n_sl + 3) // 4 * 4
    rows = L.query("ctr_rowgemm_bf_wgrad_rows", M)
    slab = torch.zeros(rows, ld, device="cuda")
    L.call("ctr_rowgemm_bf_wgrad", ptr(dY), NO, ptr(X), NIN, M, NO, NIN, ptr(slab), ld, o_db, stream())
    out = torch.full((n_sl,), float("nan"), device="cuda")
    ws = torch.empty(L.query("ctr_colsum_ws_size", rows, n_sl) // 4 + 1, device="cuda")
    L.call("ctr_colsum", ptr(slab), ld, rows, n_sl, 1.0, ptr(out), ptr(ws), stream())
    assert rel(out[:NO * NIN].double().view(NO, NIN), _bfr(dY).t() @ _bfr(X)) < 1e-6
    assert rel(out[o_db:].double(), dY.double().sum(0)) < 1e-6
    assert float(out[NO * NIN:o_db].abs().max()) == 0.0


@pytest.mark.parametrize("M,N,ld", [(1, 4, 4), (7, 3, 3), (4096, 512, 512), (4096, 513, 516), (1023, 8432, 8432),
                                    (5000, 257, 260), (64, 1, 1), (129, 260, 264), (0, 8, 8)])
def test_colsum_vs_torch(M, N, ld):
    """ctr_colsum (out = column sums / div) vs torch fp64: the float4 form (N, ld multiples of 4) and the
    scalar form, ragged row chunks, few and many partials."""
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N)
    X = torch.randn(max(M, 1), ld, device="cuda", generator=g)
    out = torch.full((N,), float("nan"), device="cuda")
    ws = torch.empty(L.query("ctr_colsum_ws_size", M, N) // 4 + 1, device="cuda")
    L.call("ctr_colsum", ptr(X), ld, M, N, 3.0, ptr(out), ptr(ws), stream())
    torch.cuda.synchronize()
    ref = X[:M, :N].double().sum(0) / 3.0
    assert rel(out.double(), ref) < 1e-6


@pytest.mark.parametrize("M,N,K,cut,splits", [(4096, 512, 7552, 6400, 8), (300, 200, 130, 70, 1),
                                              (257, 130, 99, 33, 3), (64, 7552, 512, 6400, 1)])
def test_gemm_segments_vs_torch(M, N, K, cut, splits):
    """ctr_gemm_seg: A = [A1 | A2] split at column `cut` (the QNN MLP input [z | inter]), B = [B1 | B2]
    split at column `cut`, C written as [C1 | C2] -- each against torch on the concatenated operands."""
    from tossctr._lib import GemmEpi, GemmSeg
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(M + N + K + cut)
    ws = torch.empty(splits * M * max(N, K) + 16, device="cuda")
    # A segments (ta = 0), B as a (N, K) weight (tb = 1), bias + ReLU epilogue
    kc = min(cut, K)
    A1, A2 = torch.randn(M, kc, device="cuda", generator=g), torch.randn(M, K - kc, device="cuda", generator=g)
    W = torch.randn(N, K, device="cuda", generator=g)
    bias = torch.randn(N, device="cuda", generator=g)
    C = torch.empty(M, N, device="cuda")
    L.call("ctr_gemm_seg", M, N, K, ptr(A1), kc, 0, ptr(W), K, 1, ptr(C), N, GemmEpi(bias=ptr(bias), act=1), splits,
           ptr(ws), GemmSeg(A2=ptr(A2), lda2=K - kc, ka=kc), stream())
    ref = torch.relu(torch.cat([A1, A2], 1).double() @ W.double().t() + bias.double())
    assert rel(C.double(), ref) < 1e-5
    # B segments (tb = 0): C = X^T [B1 | B2]
    nc = min(cut, N)
    X = torch.randn(K, M, device="cuda", generator=g)
    B1, B2 = torch.randn(K, nc, device="cuda", generator=g), torch.randn(K, N - nc, device="cuda", generator=g)
    C = torch.empty(M, N, device="cuda")
    L.call("ctr_gemm_seg", M, N, K, ptr(X), M, 1, ptr(B1), nc, 0, ptr(C), N, None, splits, ptr(ws),
           GemmSeg(B2=ptr(B2), ldb2=N - nc, nb=nc), stream())
    assert rel(C.double(), X.double().t() @ torch.cat([B1, B2], 1).double()) < 1e-5
    # C segments: [C1 | C2] = A W
    if N > 96:
        A = torch.randn(M, K, device="cuda", generator=g)
        Wt = torch.randn(K, N, device="cuda", generator=g)
        C1 = torch.full((M, nc), float("nan"), device="cuda")
        C2 = torch.full((M, N - nc), float("nan"), device="cuda")
        L.call("ctr_gemm_seg", M, N, K, ptr(A), K, 0, ptr(Wt), N, 0, ptr(C1), nc, None, splits, ptr(ws),
               GemmSeg(C2=ptr(C2), ldc2=N - nc, nc=nc), stream())
        ref = A.double() @ Wt.double()
        assert rel(torch.cat([C1, C2], 1).double(), ref) < 1e-5


def test_colsum_multi_matches_sums_and_is_deterministic():
    """ctr_colsum_multi (the backward's deferred slab sums): several segments of different shapes and strides in
    one launch pair == each segment's fp64 column sum (/ div), bitwise equal on a second run."""
    import ctypes
    from tossctr._lib import ColsumSeg
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(17)
    shapes = [(256, 25088, 25088, 1.0), (1920, 3168, 3172, 1.0), (7, 4, 8, 2.0), (513, 1056, 1056, 4096.0),
              (64, 260, 264, 1.0)]
    Xs, outs, segs = [], [], []
    for M, N, ld, div in shapes:
        X = torch.randn(M, ld, device="cuda", generator=g)
        out = torch.full((N + 1,), float("nan"), device="cuda")
        Xs.append(X)
        outs.append(out)
        segs.append(ColsumSeg(ptr(X), ld, M, N, ptr(out), div, 0))
    arr = (ColsumSeg * len(segs))(*segs)
    assert all(L.query("ctr_colsum_multi_ok", ctypes.byref(s_)) for s_ in segs)
    nb = L.query("ctr_colsum_multi_ws_size", arr, len(segs))
    ws = torch.empty(nb // 4 + 1, device="cuda")
    L.call("ctr_colsum_multi", arr, len(segs), ptr(ws), nb, stream())
    first = [o.clone() for o in outs]
    for (M, N, ld, div), X, o in zip(shapes, Xs, outs):
        ref = X[:, :N].double().sum(0) / div
        assert rel(o[:N].double(), ref) < 1e-6
        assert torch.isnan(o[N])                      # nothing past N is written
    L.call("ctr_colsum_multi", arr, len(segs), ptr(ws), nb, stream())
    for a, b in zip(first, outs):
        assert torch.equal(a[:-1], b[:-1])


@pytest.mark.parametrize("n", [1, 3, 4, 1027, 4_482_602])
def test_zero_f32(n):
    """ctr_zero_f32 (the grad arena's clear before each backward): every element of [0, n) zero, nothing past it
    touched (tails of 1-3 elements after the 16-byte stores)."""
    L = _lib()
    buf = torch.full((n + 8,), 7.0, device="cuda")
    L.call("ctr_zero_f32", ptr(buf), n, stream())
    torch.cuda.synchronize()
    assert (buf[:n] == 0).all() and (buf[n:] == 7.0).all()


@pytest.mark.parametrize("case", ["cfg2", "ragged", "empty"])
def test_sqnorm_all_equals_separate_calls(case):
    """ctr_sqnorm_all (dense + three compact row-grad tables in one launch) writes bit for bit the partials of
    ctr_sqnorm_dense + ctr_sqnorm_rows x 3, so ctr_clip_finalize gives the same norm: trailing INVALID key group,
    a row stride that is not a multiple of 4 (strided path), an empty table."""
    import ctypes as C
    from tossctr import _lib as TL
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(len(case))
    inv = 0xFFFFFFFF
    n_dense = {"cfg2": 1_234_567, "ragged": 1001, "empty": 0}[case]
    dense = torch.randn(n_dense + 1, device="cuda", generator=g)[1:] if case == "ragged" else \
        torch.randn(max(n_dense, 1), device="cuda", generator=g)[:n_dense]
    tabs = []
    for j, (rows, width, ld, n_valid, with_inv) in enumerate({
            "cfg2": [(300_000, 32, 32, 250_000, True), (300_000, 32, 32, 250_000, True), (80_000, 33, 36, 70_000, False)],
            "ragged": [(1000, 33, 33, 999, True), (17, 8, 8, 3, False), (5, 64, 64, 4, True)],
            "empty": [(16, 32, 32, 0, False), (16, 32, 32, 0, False), (16, 33, 36, 0, False)]}[case]):
        G = torch.randn(rows, ld, device="cuda", generator=g)
        G[:, width:] = 0.0
        nu = n_valid + (1 if with_inv else 0)
        keys = torch.arange(rows, device="cuda", dtype=torch.int32)
        if with_inv:
            keys[nu - 1] = -1                   # 0xFFFFFFFF as uint32
        tabs.append((keys, G, torch.tensor([nu], device="cuda", dtype=torch.int32), width, ld))
    P = L.query("ctr_norm_nparts_per_call")
    st = stream()
    ref = torch.full((4 * P,), float("nan"), device="cuda")
    L.call("ctr_sqnorm_dense", ptr(dense), n_dense, ptr(ref), st)
    for j, (keys, G, nu, width, ld) in enumerate(tabs):
        L.call("ctr_sqnorm_rows", ptr(keys), ptr(G), ptr(nu), width, ld, inv, ptr(ref, (j + 1) * P), st)
    arr = (TL.SqnormRows * 3)()
    for o, (keys, G, nu, width, ld) in zip(arr, tabs):
        o.keys, o.G, o.n_uniq, o.width, o.ld = ptr(keys), ptr(G), ptr(nu), width, ld
    got = torch.full_like(ref, float("nan"))
    L.call("ctr_sqnorm_all", ptr(dense), n_dense, arr, 3, inv, ptr(got), st)
    out_r = torch.zeros(2, device="cuda")
    out_g = torch.zeros(2, device="cuda")
    L.call("ctr_clip_finalize", ptr(ref), 4 * P, 1.0, 1.0, ptr(out_r), st)
    L.call("ctr_clip_finalize", ptr(got), 4 * P, 1.0, 1.0, ptr(out_g), st)
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int32), ref.view(torch.int32)), int((got != ref).sum())
    assert torch.equal(out_g.view(torch.int32), out_r.view(torch.int32))
    want = float(dense.double().pow(2).sum()) + sum(float(G[:int(nu.item()) - (1 if int(nu.item()) and int(k[int(nu.item()) - 1].item()) == -1 else 0)].double().pow(2).sum()) for k, G, nu, _, _ in tabs)
    assert abs(float(out_g[0]) - math.sqrt(want)) <= 1e-5 * math.sqrt(want) + 1e-30
