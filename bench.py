"""Training-throughput benchmark: BASELINE.json metric "training samples/sec at bs=4096 seq_len=100,
1/2/4/8 MI355X vs CPU ref" on config 2 (cfgs/dare_qnn_next.yaml + hash_buckets=1e6, emb_dim=32,
seq_len=100, bs=4096, bf16 -- amp: bf16 as BASELINE.json quotes it; --amp none for the fp32 path).

A step = one full reference training step (src/train.py:152-199): forward -> bce_wll_style + 0.1*aux
-> backward -> clip_grad_norm_(0.5) -> AdamW -> EMA(0.999), over the full model (1.24 B params incl.
the 10M x 32 DARE tables and 35 x 1e6-row hashed tables).  Inputs are synthetic (SURVEY §8(d)
distributions) and already resident in HBM.  Multi-GPU: one process per GPU (torchrun), data-parallel
(per-GPU batch 4096, weak scaling): dense grads all-reduced over RCCL; embedding tables row-sharded
over the ranks (rows fetched from / grads routed to their owners with RCCL all-to-alls; --tables
replicated all-gathers row grads instead).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
"""
import argparse
import gc
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(REPO, "toss-next-ctr-prediction_amd")
for _p in (REPO, PKG_DIR):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def synth_batches(nb, B, L, Fn, Fm, cards, vocab, device, seed):
    """SURVEY §8(d) synthetic rows: X_num N(0,1) (0 where masked), X_mask Bern(0.1), X_cat U[0,hb),
    seq right-aligned lengths U{0..L} tokens U[1,vocab), y Bern(0.019)."""
    g = torch.Generator(device=device).manual_seed(seed)
    out = []
    cards_t = torch.tensor(cards, device=device, dtype=torch.float64)
    for _ in range(nb):
        X_mask = (torch.rand(B, Fm, device=device, generator=g) < 0.1).float()
        X_num = torch.randn(B, Fn, device=device, generator=g)
        if Fn == Fm:
            X_num = X_num * (1 - X_mask)
        X_cat = (torch.rand(B, len(cards), device=device, generator=g, dtype=torch.float64) * cards_t).floor()
        X_cat = X_cat.clamp_max(cards_t - 1).to(torch.int32)
        lens = torch.randint(0, L + 1, (B, 1), device=device, generator=g)
        toks = torch.randint(1, vocab, (B, L), device=device, generator=g, dtype=torch.int32)
        pos = torch.arange(L, device=device)[None, :]
        seq = torch.where(pos >= L - lens, toks, torch.zeros_like(toks)).contiguous()
        y = (torch.rand(B, device=device, generator=g) < 0.019).float()
        y[0] = 1.0
        out.append(((X_num.contiguous(), X_mask.contiguous(), X_cat.contiguous(), seq), y))
    return out


WORKLOADS = {
    "cfg2": "cfgs/dare_qnn_next.yaml + hash_buckets=1e6, emb_dim=32, seq_len={L}, bs={B} per GPU, full train step "
            "incl. clip+AdamW+EMA over {P:.2f}B params",
    "cfg3": "cfgs/dare_qnn_next_k100_s1.yaml (K=100, S1) + hash_buckets=1e6, emb_dim=32, seq_len={L}, bs={B} per GPU, "
            "full train step incl. clip+AdamW+EMA over {P:.2f}B params",
    "cfg4": "cfgs/v3_k148_s1.yaml (D=64, K=148, 4 layers, EMA off), seq_len={L}, bs={B} per GPU, full train step "
            "incl. clip+AdamW over {P:.2f}B params",
    "cfg5": "k100_s1 shape + hash_buckets=1e8, emb_dim=64 (row-sharded tables), seq_len={L}, bs={B} per GPU, "
            "full train step incl. clip+AdamW+EMA over {P:.2f}B params",
}
MFMA_F32_PEAK_TFS = 157.3   # MI355X dense fp32 MFMA (v_mfma_f32_16x16x4_f32), MI355X_MICROARCH.md
MFMA_BF16_PEAK_TFS = 16 * MFMA_F32_PEAK_TFS   # dense bf16 MFMA = 16x the fp32 rate (~2.5 PF), same guide


PROFILE_STEPS = 5       # untimed steps after the timed region that fill the per-kernel table


def kernel_work(name, a, B, ffn_M, amp="bf16", ffn_flags=0):
    """Algorithmic work of one launch of a timed entry point: {"flops": [(flop, peak dtype)], "bytes": HBM bytes,
    "flop_note": ...} or None -- SURVEY §8(d)'s per-unit figures x the units one launch processes (DESIGN.md §5,
    "Roofline accounting").  Every kernel is then priced on its BINDING roof (price()): its floor time is
    max(sum flop / peak of its dtype, bytes / 8 TB/s).

    FFN (src/models/dare.py:45-48,66-69): the four products, 8 FF D flop per row backward, 4 forward (the backward's
    pre-activation recompute not counted); bytes per row: forward reads x (4 D) and writes the output and the
    pre-norm sum (8 D), the norm's rsqrt (4) and the dropout keep bits (FF / 8); the norm-fused backward reads x1,
    dy, h2, h1 (16 D) and r1, r2 (8), the keep bits, and writes dh1 (4 D) -- the weight-grad outputs are a few
    hundred KB.  Attention core (dare.py:53-62, MHA over K candidates): QK^T and PV = 4 K^2 D flop per sample forward,
    dP, dS K, dK, dV = 8 K^2 D backward; bytes per (sample, candidate) row: qkv (12 D), o (4 D), row max / sum
    (8 H) forward, + dO, and dqkv written (32 D) backward, plus the keep bits per (sample, head) in the kernels' lane
    layout.  The fused layer forward adds in_proj and out_proj (8 D^2 flop per row on fp32 MFMA) and reads x (4 D),
    writes h1, x1 (8 D) and r1 (4); ``_oproj`` forms dO = dh1 W_out inside (2 D^2 flop per row, fp32 MFMA), the layer
    backward (``_layer16``) also dx = dqkv W_in + dh1 (6 D^2 flop, dx written: 4 D).
    QNN pair interaction (src/models/qnn_alpha.py:86-97): the reference's A = z U projection, 2 F D QR flop per
    sample (the north star's "feature_embed_dim x proj_dim projection"), forward; its backward recomputes A and forms
    dz = dA U^T, 4 F D QR (the Gram form executes fewer flops -- priced at the reference's); bytes: z (4 F D) read,
    and the per-sample outputs.  QNN MLP first layer (qnn_alpha.py:123-129) on bf16 operands: 2 M N K flop; bytes:
    both bf16 operands once and the output (fp32, or bf16 for the input grad)."""
    D, FF = a.D, a.ffn_hidden
    kb = (FF // 8) if a.ffn_p > 0 else 0
    fdt = "bf16" if (amp == "bf16" and ffn_flags) else "f32"
    if name in ("ctr_ffn_bwd", "ctr_ffn_bwd_norms"):
        per_row = (20 * D + 8 + kb) if name == "ctr_ffn_bwd_norms" else (12 * D + kb)
        return {"flops": [(8.0 * ffn_M * FF * D, fdt)], "bytes": float(ffn_M * per_row)}
    if name == "ctr_ffn_fwd":
        return {"flops": [(4.0 * ffn_M * FF * D, fdt)], "bytes": float(ffn_M * (12 * D + 4 + kb))}
    K = ffn_M // max(1, B)
    H = a.H
    nt = (K + 15) // 16
    mask_bf = B * H * 64 * 4 * (2 if nt <= 4 else (4 * nt * nt + 31) // 32) if a.mha_p > 0 else 0
    mask_f32 = B * H * K * ((K + 31) // 32) * 4 if a.mha_p > 0 else 0
    fwd_b, bwd_b = B * K * (16 * D + 8 * H), B * K * (32 * D + 8 * H)
    if name == "ctr_attn_fwd":
        return {"flops": [(4.0 * B * K * K * D, "f32")], "bytes": float(fwd_b + mask_f32)}
    if name == "ctr_attn_bwd":
        return {"flops": [(8.0 * B * K * K * D, "f32")], "bytes": float(bwd_b + mask_f32)}
    if name == "ctr_attn_fwd_bf":
        return {"flops": [(4.0 * B * K * K * D, "bf16")], "bytes": float(fwd_b + mask_bf)}
    if name == "ctr_attn_bwd_bf":
        return {"flops": [(8.0 * B * K * K * D, "bf16")], "bytes": float(bwd_b + mask_bf)}
    if name in ("ctr_attn_bwd_bf_oproj", "ctr_attn_bwd_bf_oproj16"):   # reads dh1 rows in place of dO (same bytes)
        q16 = 12 * D * B * K if name.endswith("16") else 0                # qkv read, dqkv written in bf16
        return {"flops": [(8.0 * B * K * K * D, "bf16"), (2.0 * B * K * D * D, "f32")],
                "bytes": float(bwd_b - q16 + mask_bf)}
    if name == "ctr_attn_bwd_bf_layer16":     # + dx = dqkv W_in + dh1 (6 D^2 flop per row, fp32 MFMA; dx written)
        return {"flops": [(8.0 * B * K * K * D, "bf16"), (8.0 * B * K * D * D, "f32")],
                "bytes": float(bwd_b - 12 * D * B * K + 4 * D * B * K + mask_bf)}
    if name in ("ctr_attn_layer_fwd_bf", "ctr_attn_layer_fwd_bf16"):
        qkv_b = 6 * D if name.endswith("16") else 12 * D
        return {"flops": [(4.0 * B * K * K * D, "bf16"), (8.0 * B * K * D * D, "f32")],
                "bytes": float(B * K * (16 * D + qkv_b + 4 + 8 * H) + mask_bf)}
    if name in ("ctr_qnn_gram_fwd", "ctr_qnn_gram_bwd", "ctr_qnn_gram_fwd_zbf", "ctr_qnn_gram_bwd_zbf") and a.use_qnn:
        F, QR = a.F, a.qh * a.qr
        zb, dt = (2, "bf16") if name.endswith("_zbf") else (4, "f32")    # the bf16-z forms read z's bf16 image
        if name.startswith("ctr_qnn_gram_fwd"):     # z read; zsum, G (D x D), S, quad written
            return {"flops": [(2.0 * B * F * D * QR, dt)],
                    "bytes": float(B * (zb * F * D + 4 * D + 4 * D * D + 8 * QR)),
                    "flop_note": "reference A = z U (2 F D QR per sample); the Gram form executes 2 F D^2 + 2 D^2 QR"}
        add = 2 if amp == "bf16" else 4    # the MLP's input grad, bf16 under amp
        return {"flops": [(4.0 * B * F * D * QR, dt)],
                "bytes": float(B * ((zb + 4 + add) * F * D + 12 * QR)),
                "flop_note": "reference A recompute + dz = dA U^T (4 F D QR per sample); the Gram form executes less"}
    if name.startswith("ctr_gemm_bf16_ex@"):
        shp = name.split("@")[1]
        bf_out = shp.endswith("b")
        M, N, Kk = (int(x) for x in shp.rstrip("b").split("x"))
        return {"flops": [(2.0 * M * N * Kk, "bf16")], "bytes": float(2 * (M * Kk + Kk * N) + (2 if bf_out else 4) * M * N)}
    return None


PEAK_TFS = {"f32": MFMA_F32_PEAK_TFS, "bf16": MFMA_BF16_PEAK_TFS}   # dense MFMA (f32 = the f32 vector rate too)


def price(name, a, B, ffn_M, amp, ffn_flags, launch_ms):
    """The roofline of one timed entry point, or None: its binding roof is the larger of the compute floor
    (sum over its products of flop / dense peak of their dtype) and the HBM floor (algorithmic bytes / 8 TB/s);
    frac = that floor / the measured launch time.  ``achieved`` / ``peak`` are in the binding roof's units
    (GB/s against 8 TB/s, or TFLOP/s against the products' combined peak)."""
    w = kernel_work(name, a, B, ffn_M, amp, ffn_flags)
    if w is None:
        return None
    t = launch_ms * 1e-3
    flops = sum(f for f, _ in w["flops"])
    t_f = sum(f / (PEAK_TFS[d] * 1e12) for f, d in w["flops"])
    t_b = w["bytes"] / (HBM_PEAK_GBS * 1e9)
    dts = sorted({d for _, d in w["flops"]})
    out = {"bound": "hbm" if t_b >= t_f else "mfma", "flops": flops, "bytes": w["bytes"],
           "floor_us": round(max(t_f, t_b) * 1e6, 2), "compute_floor_us": round(t_f * 1e6, 2),
           "hbm_floor_us": round(t_b * 1e6, 2), "frac": max(t_f, t_b) / t, "mfma_dtype": "+".join(dts),
           "hbm_frac": t_b / t, "mfma_frac": t_f / t}
    if "flop_note" in w:
        out["flop_note"] = w["flop_note"]
    if out["bound"] == "hbm":
        out.update(achieved=w["bytes"] / t / 1e9, peak=HBM_PEAK_GBS, unit="GB/s")
    else:
        out.update(achieved=flops / t / 1e12, peak=flops / t_f / 1e12, unit="TFLOP/s")
    return out


def step_bytes_dense_equiv(a, B, L, with_ema):
    """SURVEY §8(d) algorithmic bytes of one reference-semantics step (dense AdamW/EMA over every
    parameter + the per-sample gather/row-grad traffic):
        Bopt * (P_emb + P_dense) + B * [inp + 12 * (L*D + K*D + sum d_c)].
    What a dense implementation must move; NOT this build's roofline (the exact-lazy tables move far
    less, step_bytes_lazy)."""
    shapes = a.param_shapes()
    p_all = sum(int(np.prod(s)) for _, s, _ in shapes)
    bopt = 56 if with_ema else 44
    return bopt * p_all + B * per_sample_bytes(a, L)


def per_sample_bytes(a, L):
    """SURVEY §8(d) per-sample term: on-disk inputs + fp32 row gather (4 B) and row-grad read-modify-write
    (8 B) of the L att rows, K rep rows and sum d_c categorical floats."""
    inp = 4 * a.Fn + a.Fm + 4 * a.Fc + 4 * L + 1
    return inp + 12 * (L * a.D + a.K_eff(L) * a.D + sum(a.cat_dims))


def lazy_row_classes(opt):
    """Per table (key, rows, width, rows that have taken a gradient tick): bit 31 of a row's lazy state word
    (csrc/lazy.hip LAST_NZ) -- such a row's replay moves p, m, v (, e); a row without it has zero moments and
    moves p (, e) only.  Read after the run's flush (the flush leaves the bit alone)."""
    ar = opt.arena
    keys = ["dare.emb_att.weight", "dare.emb_rep.weight"] + [f"cat_embs.{c}.weight" for c in opt.engine.a.cat_names]
    out, r0 = [], 0
    for k in keys:
        rows, width = ar.shapes[k]
        nz = int((opt.last[r0:r0 + rows] < 0).sum().item())
        out.append((k, rows, width, nz))
        r0 += rows
    return out


def step_bytes_lazy(a, B, L, opt, U, timed_steps, with_ema, classes):
    """Algorithmic HBM bytes of one step of THIS build (exact-lazy tables, SURVEY §8(d) row-lazy form,
    with U measured in the run), at what each kind of row must move (fp32; with EMA):
      * stepped rows (a gradient tick taken: non-zero moments) read + write p, m, v, e = 32 B per element;
      * zero-moment rows (never stepped) read + write p and e only = 16 B (idle ticks keep m, v at +0);
    B x per-sample term; the dense-parameter stream (read p, m, v, (e), grad, write p, m, v, (e)); the forward's
    touch of the rows the batch reads (each brought current once); the real tick on the rows that get a gradient
    (read the row's class, write p, m, v, e, read the compact grad row); and the run's final flush of every
    table row by its class (``classes``, lazy_row_classes) plus its state word (read + write), spread over the
    timed steps.  The touch / update rows are split by the fraction of stepped rows of their table group.
    U = {"seq_fwd": unique tokens read, "seq_bwd": unique top-K tokens (both DARE tables),
    "cat_fwd"/"cat_bwd": unique (table, row) floats} -- rows, or floats for cat (sum of d_c)."""
    ar = opt.arena
    full = 32 if with_ema else 24        # p, m, v (, e) read + written, fp32
    zero = 16 if with_ema else 8         # p (, e) read + written
    lo, hi = ar.nograd_range
    dense = ar.n_dense_grad * (full + 4) + ((hi - lo) * 12 if with_ema else 0)
    D = a.D
    seq = [c for c in classes if ".emb_" in c[0]]
    cat = [c for c in classes if c[0].startswith("cat_embs.")]
    f_seq = sum(c[3] for c in seq) / max(1, sum(c[1] for c in seq))
    f_cat = sum(c[3] * c[2] for c in cat) / max(1, sum(c[1] * c[2] for c in cat))
    mix = lambda f: f * full + (1 - f) * zero                                                 # noqa: E731
    touch = 2 * U["seq_fwd"] * D * mix(f_seq) + U["cat_fwd"] * mix(f_cat)
    update = (2 * U["seq_bwd"] * D * (mix(f_seq) / 2 + full / 2 + 4) + U["cat_bwd"] * (mix(f_cat) / 2 + full / 2 + 4))
    flush = sum(nz * w * full + (rows - nz) * w * zero + 8 * rows for _, rows, w, nz in classes) / max(1, timed_steps)
    return {"per_sample": B * per_sample_bytes(a, L), "dense_opt": dense, "touch": touch, "update": update,
            "flush": flush}


def fwd_flops_per_sample(a, L):
    """Multiply-add = 2 FLOPs of the matrix products of one sample's forward (SURVEY §8(a) FLOP census:
    21.5 MF at cfg2); the backward does twice that (input and weight gradients)."""
    D, K = a.D, a.K_eff(L)
    f = 2 * a.Fn * a.f_embed * D + 2 * a.Fm * a.f_embed * D + 2 * sum(a.cat_dims) * D
    if a.query_mode != "S1":
        f += 2 * a.nctx * D * D
    f += 2 * L * D                                    # top-K scores
    for _ in range(a.n_layers):
        f += 2 * K * D * 3 * D + 2 * K * D * D        # in / out projections
        f += 2 * 2 * K * K * D                        # scores + PV over all heads
        f += 2 * 2 * K * D * a.ffn_hidden             # FFN
    f += 2 * K * D + 2 * D                            # pool + aux head
    if a.use_qnn:
        FD, C = a.F * D, a.C
        f += a.qh * (2 * a.F * D * a.qr + 2 * a.qr * a.qP)
        dims = [FD + C] + list(a.mlp_hidden) + [1]
        f += sum(2 * x * y for x, y in zip(dims[:-1], dims[1:]))
    else:
        nin = D * (1 + (a.Fn > 0) + (a.Fm > 0) + a.Fc)
        f += 2 * nin * 512 + 2 * 512
    return f


def measure_unique(model, batch, tg):
    """U of one step (step_bytes_lazy): unique tokens / categorical rows of the batch, and the unique
    keys of its compact table gradients."""
    a = model.arch
    X_cat, seq = batch[2], batch[3]
    seq_fwd = int(torch.unique(seq[seq != a.pad_id]).numel())
    dims = torch.tensor(a.cat_dims, device=X_cat.device, dtype=torch.int64)
    base = torch.tensor(np.cumsum([0] + a.cat_cards[:-1]), device=X_cat.device, dtype=torch.int64)
    keys = torch.unique(X_cat.long() + base[None, :])
    col = torch.searchsorted(base, keys, right=True) - 1
    cat_fwd = int(dims[col].sum())
    seq_bwd = int(tg["att"]["n_uniq"].item())
    n_cat = int(tg["cat"]["n_uniq"].item())
    ck = tg["cat"]["keys"][:n_cat].long()
    col_b = torch.searchsorted(base, ck, right=True) - 1
    cat_bwd = int(dims[col_b.clamp(0, len(a.cat_dims) - 1)].sum())
    return {"seq_fwd": seq_fwd, "seq_bwd": seq_bwd, "cat_fwd": cat_fwd, "cat_bwd": cat_bwd}


def opt_algorithmic_bytes(opt, with_ema):
    """HBM bytes one fused clip/AdamW/EMA launch must move (per element: read+write p, m, v (+ema) = 24
    (+8) B; dense grads read 4 B; no-grad params EMA-only: read p, e, write e = 12 B; plus the touched
    table rows' compact grads)."""
    ar = opt.arena
    per = 32 if with_ema else 24
    b = ar.n_dense_grad * (per + 4)
    lo, hi = ar.nograd_range
    if with_ema:
        b += (hi - lo) * 12
    lo, hi = ar.table_range
    b += (hi - lo) * per
    tg = opt.engine.tg
    for name in ("att", "rep", "cat"):
        t = tg[name]
        b += int(t["n_uniq"].item()) * t["width"] * 4
    return b


PMC_ROUNDS = ("r06", "r05", "r04", "r03", "r02", "r01")      # newest committed PMC summaries first


def pmc_traffic(name):
    """HBM bytes per launch of the entry point's kernel from the committed rocprofv3 PMC summaries
    (profiles/r0N/pmc_{fetch,write}.csv, newest round: separate --pmc FETCH_SIZE / WRITE_SIZE passes of this bench),
    corrected as MI355X_MICROARCH.md prescribes (gfx950 FETCH_SIZE counts half of wide streaming reads:
    x2).  None when the summaries are absent."""
    import csv
    bwd = ("ffn_bwd_own_kernel", "ffn_bwd_bf_kernel", "ffn_bwd_cols_kernel", "ffn_bwd_kernel")   # preferred first
    kerns = {"ctr_ffn_bwd": bwd, "ctr_ffn_bwd_norms": bwd, "ctr_ffn_fwd": ("ffn_fwd_bfw_kernel", "ffn_fwd_bf_kernel", "ffn_fwd_kernel"),
             "ctr_attn_bwd": ("attn_bwd_wave_kernel", "attn_bwd_kernel"),
             "ctr_attn_fwd": ("attn_fwd_pk_kernel", "attn_fwd_kernel"),
             "ctr_attn_bwd_bf": ("attn_bwd_mf_kernel",), "ctr_attn_fwd_bf": ("attn_fwd_mf_kernel",),
             "ctr_attn_layer_fwd_bf": ("attn_layer_fwd_kernel",), "ctr_attn_bwd_bf_oproj": ("attn_bwd_mf_kernel",),
             "ctr_attn_layer_fwd_bf16": ("attn_layer_fwd_kernel",),
             "ctr_attn_bwd_bf_oproj16": ("attn_bwd_mf_kernel",), "ctr_attn_bwd_bf_layer16": ("attn_bwd_mf_kernel",)}.get(name)
    if kerns is None:
        return None
    base = next((os.path.join(REPO, "profiles", r) for r in PMC_ROUNDS
                 if os.path.exists(os.path.join(REPO, "profiles", r, "pmc_fetch.csv"))), None)
    if base is None:
        return None
    vals = {}
    for ctr, fn in (("FETCH_SIZE", "pmc_fetch.csv"), ("WRITE_SIZE", "pmc_write.csv")):
        path = os.path.join(base, fn)
        if not os.path.exists(path):
            return None
        xs = {k: [] for k in kerns}
        with open(path) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") != ctr:
                    continue
                for k in kerns:
                    if k + "<" in r.get("Kernel_Name", ""):
                        xs[k].append(float(r["Counter_Value"]))
                        break
        hit = next((xs[k] for k in kerns if xs[k]), None)
        if not hit:
            return None
        vals[ctr] = sum(hit) / len(hit) * 1024.0    # rocprofv3 reports KB
    return round(2.0 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"])


def cpu_model():
    """The host CPU's model name (/proc/cpuinfo), as SURVEY §8(d) asks the baseline to state it."""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cfg, B, L, seed=0, timed=3):
    """The CPU oracle (oracle/model.py: torch fp32 restatement of the reference step, pinned against the
    reference by tests/golden) timed on this host (SURVEY §8(d) protocol): 1 warm-up + ``timed`` steps
    at the benchmark shape, the median step reported."""
    from oracle.model import TrainState, make_arch
    from tossctr.configs import N_NUM_NEXT, cat_cardinals
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 8)))
    cards = cat_cardinals(cfg)
    cols = list(cfg["data"]["cat_cols"])
    A = make_arch(cfg, 10_000_000, N_NUM_NEXT, N_NUM_NEXT, cards, cols)
    gen = torch.Generator().manual_seed(seed)
    P = {}
    for k, shp in A.param_shapes():
        t = torch.empty(shp)
        if "emb" in k or "pbias" in k:
            t.normal_(0, 1, generator=gen)
        elif k.endswith(".w"):
            t.fill_(1.0)
        else:
            t.uniform_(-0.05, 0.05, generator=gen)
        P[k] = t
    st = TrainState(P, A, 3e-4, 1e-4, 0.5, ema_cfg=cfg["ema"])
    st.native_dropout = True     # torch's bernoulli dropout, as the reference draws it (the cost, not the masks)
    del P
    batches = synth_batches(1 + timed, B, L, N_NUM_NEXT, N_NUM_NEXT, list(cards.values()), 10_000_000, "cpu",
                            seed + 1)
    times = []
    for (inp, y) in batches:
        X_num, X_mask, X_cat, seq = inp
        b = {"X_num": X_num, "X_mask": X_mask, "X_cat": X_cat.long(), "seq": seq.long()}
        t0 = time.perf_counter()
        st.step(b, y, 3e-4, seed)
        times.append(time.perf_counter() - t0)
    t = float(np.median(times[1:]))
    return {"value": round(B / t, 2), "unit": "samples/s", "cores": torch.get_num_threads(), "kind": "port",
            "cpu": cpu_model(),
            "sample": f"oracle fp32 train step (fwd+bwd+clip+AdamW+EMA, 1.24B params; torch bernoulli dropout "
                      f"as the reference; tools/cpu_calibrate.py) at bs={B}, L={L}: "
                      f"1 warm-up + {timed} timed steps, median {t:.1f} s "
                      f"({', '.join(f'{x:.1f}' for x in times[1:])} s)"}


def launch_ranks(n):
    """``bench.py --gpus N`` without a launcher: start the N ranks (one process per GPU) as children under
    torch.distributed.run on 127.0.0.1, with this process's own arguments, and return their exit status (non-zero when
    any rank fails).  Rank 0 prints the JSON line to the stdout this process shares with it.  Nothing here touches
    the GPU: the children initialise it, each on its own card (LOCAL_RANK)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")    # dmabuf IPC: what RCCL needs on this host driver
    return subprocess.run(cmd, env=env).returncode


def build_run(args, amp, dev, pg, rank, shard):
    """The benchmarked training setup: the config's model (random init of the reference's architecture), EMA, the
    fused AdamW (exact-lazy tables unless --dense-opt), min(steps + warmup, 256) distinct synthetic batches resident
    in HBM, and ``run(i, gstep)`` = one training step on batch i at global step gstep (lr from the reference's
    cosine-warmup schedule)."""
    from tossctr import CTRModel, FusedAdamW, build_ema
    from tossctr.configs import BENCH_CONFIGS, N_NUM_NEXT, cat_cardinals
    from tossctr.train import cosine_warmup_lr
    cfg = BENCH_CONFIGS[args.config](batch_size=args.batch)
    if args.seq_len is None:
        args.seq_len = int(cfg["sequence"]["max_len"])
    cfg["sequence"]["max_len"] = args.seq_len
    cfg["amp"] = amp
    cards = cat_cardinals(cfg)
    cols = list(cfg["data"]["cat_cols"])
    vocab = 10_000_000                                   # src/train.py:116
    torch.manual_seed(cfg["seed"])
    model = CTRModel(cfg, vocab, N_NUM_NEXT, N_NUM_NEXT, cards, cols, device=dev, process_group=pg,
                     shard_tables=shard)
    model.reset_parameters(torch.Generator(device=dev).manual_seed(cfg["seed"]))
    ema = build_ema(model, cfg)
    tr = cfg["train"]
    opt = FusedAdamW(model, lr=tr["lr"], weight_decay=tr["weight_decay"], max_grad_norm=tr["grad_clip_norm"],
                     ema=ema, process_group=pg, lazy=not args.dense_opt)
    nb = min(args.steps + args.warmup, 256)     # distinct batches: lazy rows see realistic skip gaps
    data = synth_batches(nb, args.batch, args.seq_len, N_NUM_NEXT, N_NUM_NEXT, list(cards.values()), vocab, dev,
                         seed=1000 + rank)
    steps_per_epoch = 1000

    def run(i, gstep):
        inp, y = data[i % nb]
        opt.param_groups[0]["lr"] = cosine_warmup_lr(0, gstep, steps_per_epoch, tr["lr"], tr["warmup_epochs"],
                                                     tr["epochs"])
        # row-sharded tables: the next batch's exchange is planned beside this step (tossctr/shard.py)
        nxt = data[(i + 1) % nb][0] if shard else None
        return model.train_step(inp, y, opt, global_step=gstep + 1, next_inputs=nxt)
    return cfg, model, ema, opt, data, run


def fp32_secondary(args, dev):
    """``secondary.fp32``: the same protocol (args.warmup untimed + args.steps timed steps, the exact-lazy flush of
    the timed ticks inside the timed region) on a FRESH model at ``amp: none`` -- the precision every reference yaml
    trains at (cfgs/dare_qnn_next.yaml:5 ``amp: none``) -- beside the bf16 headline BASELINE.json quotes cfg2 at."""
    cfg, model, ema, opt, data, run = build_run(args, "none", dev, None, 0, False)
    g = 0
    for _ in range(args.warmup):
        run(g, g)
        g += 1
    model.sync()
    torch.cuda.synchronize()
    gc.collect()
    gc.disable()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = run(g, g)
        g += 1
    model.sync()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    gc.enable()
    if not math.isfinite(float(loss.item())):
        raise RuntimeError("non-finite loss (fp32 secondary)")
    ms = elapsed / args.steps * 1e3
    out = {"value": round(args.batch * args.steps / elapsed, 1), "unit": "samples/s", "ms_per_step": round(ms, 3),
           "steps": args.steps, "warmup": args.warmup, "dtype": "fp32",
           "precision": "fp32 everywhere (amp: none, the reference yamls' setting): fp32 VALU attention, fp32 FFN and "
                        "GEMM kernels (fp32 MFMA where they use it)",
           "protocol": "fresh model, same warm-up / timed steps / timed flush as the headline"}
    del model, opt, ema, data
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)    # 20 warm-up, >= 100 timed steps
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--seq-len", type=int, default=None, help="default: the config's (100; cfg4 400)")
    ap.add_argument("--config", choices=("cfg2", "cfg3", "cfg4", "cfg5"), default="cfg2",
                    help="BASELINE.json config (the metric is quoted on cfg2; cfg5 needs 8 GPUs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fp32-secondary", action="store_true",
                    help="skip secondary.fp32 (the same protocol at amp: none, on a fresh model; N = 1 only)")
    ap.add_argument("--kernel-events", choices=("all", "none"), default="all",
                    help="HIP events around the big kernels' calls in the timed steps (none: no roofline)")
    ap.add_argument("--gc-in-steps", action="store_true",
                    help="leave Python's cyclic garbage collector running in the timed steps (A/B of its host stalls)")
    ap.add_argument("--markers", action="store_true",
                    help="launch an empty step_marker_kernel around the timed region (tools/prof_summary.py)")
    ap.add_argument("--dense-opt", action="store_true",
                    help="step the tables in the dense AdamW/EMA stream instead of the exact lazy path")
    ap.add_argument("--amp", choices=("none", "bf16"), default="bf16",
                    help="cfg['amp'] (src/train.py:133-139): bf16 (BASELINE.json config 2 is quoted at bf16) = bf16 "
                         "MFMA operands, fp32 accumulation, fp32 master weights / optimizer state / tables; none = fp32")
    ap.add_argument("--tables", choices=("sharded", "replicated"), default="sharded",
                    help="N > 1: row-shard the embedding tables over the ranks (all-to-all row fetch / grad "
                         "routing) or replicate them (all-gather of row grads)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU "
                         f"(bench.py --gpus N starts them itself when WORLD_SIZE is unset)")
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())   # ranks > cards: rehearsal
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = None
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("CTR_DIST_BACKEND", "nccl")    # gloo: functional rehearsal on one card
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)
        pg = dist.group.WORLD

    shard = pg is not None and args.tables == "sharded"
    cfg, model, ema, opt, data, run = build_run(args, args.amp, dev, pg, rank, shard)
    nb = len(data)

    g = 0
    for _ in range(args.warmup):
        run(g, g)
        g += 1
    model.sync()
    torch.cuda.synchronize()
    if pg is not None:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    from tossctr import _lib
    # HIP events cost host time per bracketed call (~0.1 ms per step for the whole list below when the step is
    # host-issue sensitive), so the timed steps bracket only the roofline candidates (the kernels with an
    # algorithmic work count, kernel_work); the per-kernel table comes from extra steps after the timed region
    roof_timed = ("ctr_ffn_bwd", "ctr_ffn_bwd_norms", "ctr_ffn_fwd", "ctr_attn_bwd", "ctr_attn_fwd",
                  "ctr_attn_bwd_bf", "ctr_attn_fwd_bf", "ctr_attn_layer_fwd_bf", "ctr_attn_bwd_bf_oproj",
                  "ctr_attn_layer_fwd_bf16", "ctr_attn_bwd_bf_oproj16", "ctr_attn_bwd_bf_layer16",
                  "ctr_qnn_gram_fwd", "ctr_qnn_gram_bwd", "ctr_qnn_gram_fwd_zbf", "ctr_qnn_gram_bwd_zbf",
                  "ctr_gemm_bf16_ex")
    timed = roof_timed + ("ctr_lazy_flush", "ctr_lazy_flush_pair",
                          "ctr_lazy_touch", "ctr_lazy_touch_pair", "ctr_lazy_touch_pair_hot", "ctr_lazy_update", "ctr_lazy_update_pair",
                          "ctr_adamw_ema", "ctr_adamw_ema_hist")
    # a HIP event recorded between two kernels costs a boundary of its own (≈ 5 µs each on MI355X: 10–12 µs gaps around
    # every bracketed launch), so the candidates are ranked on a few untimed probe steps first and the timed steps
    # bracket only the dominant one -- the roofline kernel, still timed live in the timed region
    probe, roof_kernel, roof_every = {}, None, 1
    if args.kernel_events == "all":
        a_ = model.arch
        _lib.time_calls(roof_timed)
        for _ in range(PROFILE_STEPS):
            run(g, g)
            g += 1
        torch.cuda.synchronize()
        probe = _lib.timed_ms()
        _lib.time_calls(())
        fm_ = args.batch * a_.K_eff(args.seq_len)
        ranked = sorted(probe, key=lambda n: probe[n][0] * probe[n][1], reverse=True)
        roof_kernel = next((n for n in ranked if price(n, a_, args.batch, fm_, args.amp, model.engine.ffn_flags,
                                                       probe[n][1]) is not None), None)     # may carry a shape key
        if roof_kernel is not None:
            # one launch of the dominant kernel per step is bracketed, the layers' launches of it (the same shape) in
            # turn: each bracketed launch costs the step two event boundaries (≈ 13 µs idle after it in the trace)
            roof_every = max(1, round(probe[roof_kernel][0] / PROFILE_STEPS))
            _lib.time_calls((roof_kernel,), every=roof_every)
        torch.cuda.synchronize()
    # the host issues the step a few hundred dispatches ahead of the device at most (the HIP queue depth): a cyclic
    # garbage collection of the interpreter's heap mid-step (≈ 2 ms, once in ~20 steps in the kernel trace) leaves the
    # GPU idle that long (level at 20 + 5 steps after the collect below: 3.549 vs 3.554 ms, tools/_ab_gc.sh).
    gc.collect()
    if not args.gc_in_steps:
        gc.disable()
    if args.markers:
        _lib.call("ctr_step_marker", 1, torch.cuda.current_stream(dev).cuda_stream)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = run(g, g)
        g += 1
    # lazy tables: the ticks rows skipped are owed work -- pay all of it inside the timed region
    fl = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    fl[0].record()
    model.sync()
    fl[1].record()
    if args.markers:
        _lib.call("ctr_step_marker", 2, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    if pg is not None:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    gc.enable()
    flush_ms = fl[0].elapsed_time(fl[1])
    kstats_timed = _lib.timed_ms()
    _lib.time_calls(())
    opt_ms, kstats = None, {}
    if args.kernel_events == "all":      # per-kernel table: a few more steps, every listed call bracketed
        opt.time_kernels(True)
        _lib.time_calls(timed)
        for _ in range(PROFILE_STEPS):
            run(g, g)
            g += 1
        model.sync()
        opt_ms = opt.kernel_ms()
        opt.time_kernels(False)
        kstats = _lib.timed_ms()
        _lib.time_calls(())
    # U of the exact-lazy byte count: the unique rows of the last timed step's batch and gradients; the tables'
    # row classes (stepped / zero-moment) for the flush bytes
    U = measure_unique(model, data[(g - 1) % nb][0], model.engine.tg) if world == 1 else None
    classes = lazy_row_classes(opt) if world == 1 and not args.dense_opt else None
    if pg is not None:
        t = torch.tensor([elapsed], device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    if not math.isfinite(float(loss.item())):
        raise RuntimeError("non-finite loss")
    if rank == 0:
        ms = elapsed / args.steps * 1e3
        samples = args.batch * world * args.steps / elapsed
        # dominant timed kernel (by device time per step) and its roofline
        a = model.arch
        ffn_M = args.batch * a.K_eff(args.seq_len)
        per_step = {n: c * ms / PROFILE_STEPS for n, (c, ms) in kstats.items()}
        kernels = {n: {"calls_per_step": round(kstats[n][0] / PROFILE_STEPS, 2), "avg_launch_ms": round(kstats[n][1], 4),
                       "ms_per_step": round(per_step[n], 4)} for n in kstats}
        per_step_t = {n: c * roof_every * ms / args.steps for n, (c, ms) in kstats_timed.items()}
        roof = None
        for n in sorted(per_step_t, key=per_step_t.get, reverse=True):
            pr = price(n, a, args.batch, ffn_M, args.amp, model.engine.ffn_flags, kstats_timed[n][1])
            if pr is None:
                continue
            roof = {"bound": pr["bound"], "kernel": n, "achieved": round(pr["achieved"], 2), "peak": round(pr["peak"], 1),
                    "unit": pr["unit"], "frac": round(pr["frac"], 4), "mfma_dtype": pr["mfma_dtype"],
                    "traffic": pmc_traffic(n) if args.config == "cfg2" else None,
                    "algorithmic_bytes": pr["bytes"], "algorithmic_flops": pr["flops"],
                    "floor_us": pr["floor_us"], "hbm_floor_us": pr["hbm_floor_us"],
                    "compute_floor_us": pr["compute_floor_us"],
                    "avg_launch_ms": round(kstats_timed[n][1], 4), "ms_per_step": round(per_step_t[n], 4),
                    "share_of_step": round(per_step_t[n] / ms, 4),
                    "timing": f"HIP events in the timed steps (1 of every {roof_every} launches, "
                              f"{kstats_timed[n][0]} bracketed)",
                    "pricing": "binding roof: frac = max(sum flop / dense MFMA peak of the dtype, algorithmic bytes / "
                               "8 TB/s) / measured launch time (kernel_work)"}
            # every priced candidate, dominant first: the roofline kernel from the timed steps, the others from the
            # probe steps before them (ranked there; only the dominant one is bracketed in the timed region)
            roof["priced"] = {}
            per_step_p = {m_: c * t_ / PROFILE_STEPS for m_, (c, t_) in probe.items()}
            src = [(n, kstats_timed[n], per_step_t[n], "timed")] + [
                (m_, probe[m_], per_step_p[m_], "probe") for m_ in sorted(per_step_p, key=per_step_p.get, reverse=True)
                if m_ != n]
            for m_, (c_, t_), ps_, how in src:
                pr_ = price(m_, a, args.batch, ffn_M, args.amp, model.engine.ffn_flags, t_)
                if pr_ is None:
                    continue
                ent = {"bound": pr_["bound"], "ms_per_step": round(ps_, 4), "avg_launch_ms": round(t_, 4),
                       "achieved": round(pr_["achieved"], 2), "peak": round(pr_["peak"], 1), "unit": pr_["unit"],
                       "frac": round(pr_["frac"], 4), "hbm_frac": round(pr_["hbm_frac"], 4),
                       "mfma_frac": round(pr_["mfma_frac"], 4), "mfma_dtype": pr_["mfma_dtype"],
                       "bytes": pr_["bytes"], "flops": pr_["flops"], "steps": how}
                if "flop_note" in pr_:
                    ent["flop_note"] = pr_["flop_note"]
                roof["priced"][m_] = ent
            break
        rec = {
            "metric": "training samples/sec at bs=4096 seq_len=100, 1/2/4/8 MI355X vs CPU ref"
                      + ("" if args.config == "cfg2" else f" [{args.config}: not the headline config]"),
            "value": round(samples, 1), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32" if args.amp == "none" else "bf16",
            "precision": ("fp32 everywhere" if args.amp == "none" else
                          "amp bf16: bf16 MFMA operands with fp32 accumulation in the FFN, the QNN/head GEMMs and "
                          "the attention products" + ("" if model.engine.attn_bf else " (this shape: fp32 attention)")
                          + "; softmax, projections, norms, embeddings, optimizer state and master weights fp32"),
            "data": "synthetic (SURVEY 8(d) distributions), HBM-resident",
            "config": {"workload": WORKLOADS[args.config].format(B=args.batch, L=args.seq_len,
                                                                 P=sum(int(np.prod(sh)) for _, sh, _ in
                                                                       a.param_shapes()) / 1e9),
                       "global_batch": args.batch * world, "seq_len": args.seq_len,
                       "parallelism": f"dp{world}" + ("" if world == 1 else
                                                     f", tables {'row-sharded' if shard else 'replicated'}")},
            "roofline": roof,
            "kernels": kernels,
            "kernels_note": f"HIP events on {PROFILE_STEPS} extra steps after the timed region (the flush: once, over those "
                            f"{PROFILE_STEPS} ticks; the timed region's flush is flush_ms); the roofline candidates ranked "
                            f"on {PROFILE_STEPS} untimed probe steps before it, only the dominant one bracketed while timed",
            "opt_ms_per_step": round(opt_ms, 3) if opt_ms is not None else None,
            "table_update": "dense stream" if args.dense_opt else "exact lazy (replay on read/grad; final flush timed)",
            "flush_ms": round(flush_ms, 3),
        }
        # whole-step figures: FLOPs of the matrix products against the MFMA peak of the run's dtype (bf16 under
        # amp: bf16; the fp32 figure beside it); HBM bytes of this build's exact-lazy step (U measured above)
        # against 8 TB/s; the dense-equivalent bytes of the reference semantics only for comparison with a dense
        # implementation's ceiling
        flops = 3.0 * fwd_flops_per_sample(a, args.seq_len) * args.batch
        fpeak = MFMA_BF16_PEAK_TFS if args.amp == "bf16" else MFMA_F32_PEAK_TFS
        rec["step_flops"] = {"flop_per_step": flops, "achieved": round(flops / (ms * 1e-3) / 1e12, 2),
                             "peak": fpeak, "unit": "TFLOP/s", "peak_dtype": "bf16" if args.amp == "bf16" else "f32",
                             "frac": round(flops / (ms * 1e-3) / 1e12 / fpeak, 4),
                             "frac_of_fp32_peak": round(flops / (ms * 1e-3) / 1e12 / MFMA_F32_PEAK_TFS, 4)}
        if U is not None and not args.dense_opt:
            parts = step_bytes_lazy(a, args.batch, args.seq_len, opt, U, args.steps, ema is not None, classes)
            tb = sum(parts.values())
            rec["step_hbm"] = {"mode": "exact-lazy row bytes (SURVEY 8(d) row-lazy form, U measured)",
                               "unique": U, "bytes": {k: int(v) for k, v in parts.items()},
                               "bytes_per_step": int(tb), "achieved": round(tb / (ms * 1e-3) / 1e9, 1),
                               "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": round(tb / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        rec["dense_equivalent_bytes"] = step_bytes_dense_equiv(a, args.batch, args.seq_len, ema is not None)
        if world == 1 and not args.no_fp32_secondary:
            del data, model, opt, ema, run
            gc.collect()
            torch.cuda.empty_cache()
            rec["secondary"] = {"fp32": fp32_secondary(args, dev)}
        if world == 1 and not args.no_cpu_baseline and args.config == "cfg2":
            rec["cpu_baseline"] = cpu_baseline(cfg, args.batch, args.seq_len)
        else:
            rec["cpu_baseline"] = None
        print(json.dumps(rec), flush=True)
    if pg is not None:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
