"""Deterministic synthetic params / batches / fingerprints for parity fixtures.

TEST INFRASTRUCTURE (see oracle/__init__.py).  The same functions run in the
golden generator (which feeds them to the reference) and in the tests on the
GPU box (which feed them to the HIP path), so large fixtures only need to store
seeds + fingerprints, not weights.
"""
from __future__ import annotations

import zlib

import numpy as np


def _key_seed(seed: int, key: str) -> int:
    return (seed * 1_000_003 + zlib.crc32(key.encode())) & 0xFFFFFFFF


def make_params(shapes, seed: int, pad_id: int = 0):
    """Reference-like init (nn.Embedding N(0,1), nn.Linear U(+-1/sqrt(fan_in))), perturbed so
    norms/biases are non-trivial.  ``shapes``: list of (state_dict key, shape)."""
    out = {}
    for k, shp in shapes:
        r = np.random.default_rng(_key_seed(seed, k))
        if "cat_embs" in k or "emb_att" in k or "emb_rep" in k or "pbias.rel" in k:
            a = r.standard_normal(shp)
            if ("emb_att" in k or "emb_rep" in k):
                a[pad_id] = 0.0
        elif k.endswith(("norm1.w", "norm2.w", "pre_norm.w", "norm1.weight", "norm2.weight", "pre_norm.weight")):
            a = 1.0 + 0.1 * r.standard_normal(shp)
        elif k.endswith(("norm1.bias", "norm2.bias", "pre_norm.bias")):       # LayerNorm bias
            a = 0.1 * r.standard_normal(shp)
        elif k in ("qnn.U", "qnn.V"):
            a = 0.2 * r.standard_normal(shp)
        elif k in ("num_embed.weight", "mask_embed.weight"):
            a = 0.3 * r.standard_normal(shp)
        elif k == "num_embed.bias":
            a = 0.1 * r.standard_normal(shp)
        else:
            fan_in = shp[-1] if len(shp) > 1 else max(1, shp[0])
            bound = 1.0 / np.sqrt(fan_in)
            a = r.uniform(-bound, bound, shp)
        out[k] = a.astype(np.float32)
    return out


def reference_init(A, seed: int):
    """The reference's own initial parameters: ``torch.manual_seed(seed); CTRModel(...)``, restated as the
    torch.nn default initialisers the reference's constructors run, drawn from torch's CPU generator in the
    reference's construction order (src/models/wrapper.py:24-100; feature_embed.py:15-17,38-40; dare.py:43-51,
    89-90,106-114; qnn_alpha.py:64-84).  ``A``: oracle.model.Arch.  Returns {state_dict key: float32 ndarray}.
    Pinned bitwise against the reference's model by tests/golden/gen_golden.py (``init: reference`` cases)."""
    import math

    import torch
    from torch.nn import init

    out = {}
    torch.manual_seed(seed)

    def linear(key, n_out, n_in, bias=True):      # nn.Linear.reset_parameters
        w = torch.empty(n_out, n_in)
        init.kaiming_uniform_(w, a=math.sqrt(5))
        out[key + ".weight"] = w
        if bias:
            b = torch.empty(n_out)
            bound = 1 / math.sqrt(n_in) if n_in > 0 else 0
            init.uniform_(b, -bound, bound)
            out[key + ".bias"] = b

    def embedding(key, rows, width, pad=None):    # nn.Embedding.reset_parameters
        w = torch.empty(rows, width)
        init.normal_(w)
        if pad is not None:
            w[pad].zero_()
        out[key] = w

    D, fe = A.D, A.f_embed
    if A.Fn > 0:
        out["num_embed.weight"] = torch.randn(A.Fn, fe) * 0.02
        out["num_embed.bias"] = torch.zeros(A.Fn, fe)
        linear("num_embed.out_proj", D, fe, bias=False)
    if A.Fm > 0:
        out["mask_embed.weight"] = torch.randn(A.Fm, fe) * 0.02
        linear("mask_embed.out_proj", D, fe, bias=False)
    for c, card, d in zip(A.cat_names, A.cat_cards, A.cat_dims):
        embedding(f"cat_embs.{c}.weight", card, d)
        linear(f"cat_proj.{c}", D, d, bias=False)
    linear("ctx_mlp.0", D, D * ((A.Fn > 0) + (A.Fm > 0) + 1))
    embedding("dare.emb_att.weight", A.seq_vocab, D, A.pad_id)
    embedding("dare.emb_rep.weight", A.seq_vocab, D, A.pad_id)
    for i in range(A.n_layers):
        p = f"dare.layers.{i}."
        # nn.MultiheadAttention: out_proj (an nn.Linear) is built first, then _reset_parameters draws
        # xavier_uniform_ for in_proj_weight and zeroes both biases
        linear(p + "mha.out_proj", D, D)
        w = torch.empty(3 * D, D)
        init.xavier_uniform_(w)
        out[p + "mha.in_proj_weight"] = w
        out[p + "mha.in_proj_bias"] = torch.zeros(3 * D)
        out[p + "mha.out_proj.bias"].zero_()
        if A.layer_norm:
            out[p + "norm1.weight"], out[p + "norm1.bias"] = torch.ones(D), torch.zeros(D)
        else:
            out[p + "norm1.w"] = torch.ones(D)
        linear(p + "ffn.0", A.ffn_hidden, D)
        linear(p + "ffn.3", D, A.ffn_hidden)
        if A.layer_norm:
            out[p + "norm2.weight"], out[p + "norm2.bias"] = torch.ones(D), torch.zeros(D)
        else:
            out[p + "norm2.w"] = torch.ones(D)
        if A.add_pos:
            embedding(p + "pbias.rel.weight", 2 * A.top_k + 1, A.H)
    linear("dare.aux_head", 1, D)
    if A.use_qnn:
        FD, C = A.F * D, A.qh * A.qP
        if A.qnn_layer_norm:
            out["qnn.pre_norm.weight"], out["qnn.pre_norm.bias"] = torch.ones(FD), torch.zeros(FD)
        else:
            out["qnn.pre_norm.w"] = torch.ones(FD)
        out["qnn.U"] = torch.randn(A.qh, D, A.qr) * 0.02
        out["qnn.V"] = torch.randn(A.qh, A.qr, A.qP) * 0.02
        if A.use_se:
            linear("qnn.se.fc.0", C // A.se_r, C)
            linear("qnn.se.fc.2", C, C // A.se_r)
        din = C + FD
        for j, h in enumerate(A.mlp_hidden):
            linear(f"qnn.mlp.{3 * j}", h, din)
            din = h
        linear(f"qnn.mlp.{3 * len(A.mlp_hidden)}", 1, din)
    else:
        linear("fc.0", 512, D * (1 + (A.Fn > 0) + (A.Fm > 0) + A.Fc))
        linear("fc.3", 1, 512)
    return {k: out[k].numpy() for k, _ in A.param_shapes()}


def make_batch(B, Fn, Fm, cards, L, vocab, seed, pad_id=0, edge_rows=True, lognormal=False, pos_rate=0.3):
    r = np.random.default_rng(seed)
    X_num = r.standard_normal((B, Fn)).astype(np.float32)
    if lognormal and Fn > 0:
        sel = r.random((B, Fn)) < 0.3
        X_num[sel] = np.minimum(r.lognormal(0.0, 2.0, sel.sum()), 1e6).astype(np.float32)
    X_mask = (r.random((B, Fm)) < 0.1).astype(np.uint8)
    if Fn == Fm and Fn > 0:
        X_num[X_mask.astype(bool)] = 0.0
    X_cat = np.stack([r.integers(0, c, B) for c in cards], axis=1).astype(np.int32) if cards else \
        np.zeros((B, 0), np.int32)
    seq = np.full((B, L), pad_id, dtype=np.int32)
    lens = r.integers(0, L + 1, B)
    for b in range(B):
        n = int(lens[b])
        if n:
            seq[b, L - n:] = r.integers(1, vocab, n)        # right-aligned, left-padded
    if edge_rows and B >= 4:
        seq[0] = pad_id                                     # empty history
        seq[1] = pad_id
        seq[1, L - 3:] = r.integers(1, vocab, 3)            # fewer than K real tokens
        seq[2, L // 2:] = r.integers(1, vocab)              # one token repeated
        seq[3] = r.integers(1, vocab, L)                    # full row
    y = (r.random(B) < pos_rate).astype(np.int8)
    if B >= 2:
        y[0], y[1] = 1, 0
    groups = r.integers(0, 2**31 - 1, B).astype(np.int64)
    return dict(X_num=X_num, X_mask=X_mask, X_cat=X_cat, seq=seq, y=y, groups=groups)


NPROJ = 8      # Gaussian projections per fingerprint: a statistical estimate of ||got - ref||


def fingerprint(a: np.ndarray, seed: int = 7, n: int = 2048):
    """Size-independent summary: sampled elements + float64 sum / sumsq / random projection, plus
    NPROJ Gaussian projections ``projs``: for d = got - ref, (R got - projs)_i ~ N(0, ||d||^2), so
    the projections estimate the norm of the difference without storing ref."""
    a = np.asarray(a, dtype=np.float32).ravel()
    r = np.random.default_rng(seed + a.size)
    idx = np.sort(r.choice(a.size, size=min(n, a.size), replace=False)).astype(np.int64)
    proj = r.standard_normal(a.size).astype(np.float32)
    a64 = a.astype(np.float64)
    return dict(idx=idx, vals=a[idx], sum=a64.sum(), sumsq=(a64 * a64).sum(),
                proj=float(a64 @ proj.astype(np.float64)), projs=project(a64))


def fingerprint_proj_vec(size: int, seed: int = 7):
    r = np.random.default_rng(seed + size)
    r.choice(size, size=min(2048, size), replace=False)
    return r.standard_normal(size).astype(np.float32)


def project(a: np.ndarray, seed: int = 11, chunk: int = 1 << 20) -> np.ndarray:
    """R @ a (float64) for the (NPROJ, a.size) standard-normal matrix R of ``seed`` and a.size,
    generated in column chunks so large tensors never materialise R."""
    a = np.asarray(a, dtype=np.float64).ravel()
    r = np.random.default_rng(seed * 7919 + a.size)
    out = np.zeros(NPROJ, np.float64)
    for c0 in range(0, a.size, chunk):
        c1 = min(a.size, c0 + chunk)
        R = r.standard_normal((NPROJ, c1 - c0), dtype=np.float32)
        out += R.astype(np.float64) @ a[c0:c1]
    return out
