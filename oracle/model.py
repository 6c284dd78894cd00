"""Functional torch-CPU restatement of the reference CTRModel forward + train step.

TEST INFRASTRUCTURE (see oracle/__init__.py).  Written from scratch against the
reference semantics; every block cites the reference line it restates.  Params
are a flat ``{state_dict_key: tensor}`` dict with the reference's key names, so
fixtures, the HIP model and this oracle exchange weights by name.

Dropout masks come from ``oracle.rng`` (the build's counter-based RNG) instead
of torch's bernoulli stream; see oracle/rng.py.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn.functional as F

from . import rng

# dropout site ids -- shared spec with tossctr/rng.py and the kernels
SITE_EMB = 0
SITE_ATTN0 = 1      # + 2*layer
SITE_FFN0 = 2       # + 2*layer
SITE_DARE = 100
SITE_QNN = 101
SITE_MLP0 = 102     # + hidden layer index
SITE_FC = 110


def site_attn(i):
    return SITE_ATTN0 + 2 * i


def site_ffn(i):
    return SITE_FFN0 + 2 * i


@dataclass
class Dropper:
    """Applies reference-style dropout ``x * (mask / (1-p))`` with hash masks.  ``native``: torch's own
    ``F.dropout`` (bernoulli_ masks, the reference's exact op) -- for TIMING the CPU baseline only, where
    the masks' values do not matter but their cost does (tools/cpu_calibrate.py)."""
    seed: int
    training: bool = True
    double: bool = False
    record: dict = field(default_factory=dict)
    native: bool = False

    def __call__(self, site: int, x: torch.Tensor, p: float) -> torch.Tensor:
        if not self.training or p <= 0.0:
            return x
        if self.native:
            return F.dropout(x, p, training=True)
        keep = torch.from_numpy(rng.keep_mask(self.seed, site, p, tuple(x.shape)))
        self.record[site] = keep
        noise = keep.to(x.dtype) / (1.0 - p)            # _dropout_impl: bernoulli_(1-p).div_(1-p)
        return x * noise


def rmsnorm(x, w, eps=1e-6):
    # src/models/dare.py:12-13, src/models/qnn_alpha.py:11-12
    return w * x * torch.rsqrt(x.pow(2).mean(dim=-1, keepdim=True) + eps)


def norm(x, P, name, layer):
    # src/models/dare.py:15-18 make_norm: "rms" -> RMSNorm (weight `w`), any other name -> nn.LayerNorm(d) (weight,
    # bias, eps 1e-5)
    if layer:
        return F.layer_norm(x, (x.shape[-1],), P[name + ".weight"], P[name + ".bias"], 1e-5)
    return rmsnorm(x, P[name + ".w"])


def norm_params(name, d, layer):
    return [(name + ".weight", (d,)), (name + ".bias", (d,))] if layer else [(name + ".w", (d,))]


def decay_log_table(L: int, tau: float, dtype=torch.float32) -> torch.Tensor:
    # src/models/dare.py:126-130
    pos = torch.arange(L)
    decay = torch.exp(-(L - 1 - pos).to(dtype) / max(1.0, float(tau)))
    return torch.log(decay + 1e-8)


def pos_bias_mask(rel: torch.Tensor, K: int, max_len: int) -> torch.Tensor:
    # src/models/dare.py:29-37 and :56-60 (mean over heads of the relative bias)
    i = torch.arange(K).unsqueeze(1)
    j = torch.arange(K).unsqueeze(0)
    d = (j - i).clamp(-max_len, max_len) + max_len
    return rel[d].permute(2, 0, 1).mean(0)


def topk_select(P, seq, q, K, tau, pad_id, dtype):
    # src/models/dare.py:116-138
    # nn.Embedding(..., padding_idx=pad_id): the pad row receives no gradient (src/models/dare.py:89-90)
    att = F.embedding(seq, P["dare.emb_att.weight"], padding_idx=pad_id)
    rep = F.embedding(seq, P["dare.emb_rep.weight"], padding_idx=pad_id)
    B, L, D = att.shape
    scores = (att * q.unsqueeze(1)).sum(-1) + decay_log_table(L, tau, dtype)
    scores = scores.masked_fill(seq == pad_id, -1e9)
    k = min(K, L)
    vals, idx = scores.topk(k=k, dim=1)
    sel = torch.gather(rep, 1, idx.unsqueeze(-1).expand(-1, -1, D))
    return sel, vals, idx


def encoder_layer(P, pre, x, H, mha_p, ffn_p, add_pos, top_k, drop, li, layer_norm=False):
    # src/models/dare.py:53-70; MHA explicit (need_weights=True) path of
    # torch.nn.functional.multi_head_attention_forward (batch_first)
    B, K, D = x.shape
    dh = D // H
    W = P[pre + "mha.in_proj_weight"]
    bqkv = P[pre + "mha.in_proj_bias"]
    qkv = x @ W.t() + bqkv
    q, k, v = qkv.split(D, dim=-1)
    q = q.reshape(B, K, H, dh).transpose(1, 2)
    k = k.reshape(B, K, H, dh).transpose(1, 2)
    v = v.reshape(B, K, H, dh).transpose(1, 2)
    s = (q * math.sqrt(1.0 / float(dh))) @ k.transpose(-2, -1)
    if add_pos:
        s = pos_bias_mask(P[pre + "pbias.rel.weight"], K, top_k) + s
    a = torch.softmax(s, dim=-1)
    a = drop(site_attn(li), a, mha_p)
    o = (a @ v).transpose(1, 2).reshape(B, K, D)
    h = o @ P[pre + "mha.out_proj.weight"].t() + P[pre + "mha.out_proj.bias"]
    x = norm(x + h, P, pre + "norm1", layer_norm)
    f = F.gelu(x @ P[pre + "ffn.0.weight"].t() + P[pre + "ffn.0.bias"])
    f = drop(site_ffn(li), f, ffn_p)
    f = f @ P[pre + "ffn.3.weight"].t() + P[pre + "ffn.3.bias"]
    return norm(x + f, P, pre + "norm2", layer_norm)


class Arch:
    """Static shape/config facts derived from a reference-style cfg dict (src/models/wrapper.py:11-104)."""

    def __init__(self, cfg, seq_vocab, num_dim, mask_dim, cat_cardinals, cat_cols):
        m, s = cfg["model"], cfg["sequence"]
        qa = m["qnn_alpha"]
        self.D = m["emb_dim"]
        self.f_embed = int(qa.get("feature_embed_dim", max(8, self.D // 4)))
        self.p_emb = float(m.get("embedding_dropout", 0.0))
        self.cat_cols = list(cat_cols)
        dims = m.get("cat_embedding_dims", {})
        self.cat_dims = [int(dims.get(c, self.D)) for c in cat_cardinals]
        self.cat_cards = [int(cat_cardinals[c]) for c in cat_cardinals]
        self.cat_names = list(cat_cardinals)
        self.Fn, self.Fm, self.Fc = num_dim, mask_dim, len(cat_cardinals)
        self.seq_vocab = seq_vocab
        self.query_mode = s["query_mode"]
        self.query_key = s["query_key"]
        self.top_k = s["top_k"]
        self.tau = s["recency_tau"]
        self.pad_id = s["pad_id"]
        self.p_dare = float(m["dare_dropout"])
        t = s.get("tfm", {}) or {}
        self.tb = bool(s["transformer_block"])
        self.n_layers = t.get("n_layers", 2) if self.tb else 0
        self.H = t.get("n_heads", 4)
        self.mha_p = t.get("mha_dropout", 0.1)
        self.ffn_hidden = t.get("ffn_hidden", 256)
        self.ffn_p = t.get("ffn_dropout", 0.1)
        self.add_pos = t.get("add_positional_bias", True)
        self.gating = t.get("gating", "softmax") if t else "softmax"
        self.layer_norm = self.tb and str(t.get("norm", "rms")).lower() != "rms"
        self.qnn_layer_norm = bool(qa["enabled"]) and str(qa.get("norm", "rms")).lower() != "rms"
        self.use_qnn = bool(qa["enabled"])
        if self.use_qnn:
            self.qh, self.qr, self.qP = qa["heads"], qa["rank"], qa["proj_dim"]
            self.mlp_hidden = list(qa["mlp_hidden"])
            self.qnn_p = float(qa["dropout"])
            self.use_se = bool(qa["use_se"])
            self.se_r = int(qa.get("se_reduction", 8))
            self.use_residual = bool(qa["use_residual"])
            self.pair_grouping = qa["pair_grouping"]
            self.F = 1 + self.Fn + self.Fm + self.Fc
        self.aux_w = float(qa.get("aux_head_weight", 0.0))

    def qnn_blocks(self):
        """src/models/wrapper.py:66-75: the feature blocks of the QNN input [u | num | mask | cat], in that order
        (a block only when its features are present)."""
        sizes = [1] + [n for n in (self.Fn, self.Fm) if n > 0] + [self.Fc]     # seq, num?, mask?, cat
        out, o = [], 0
        for n in sizes:
            out.append((o, o + n))
            o += n
        return out

    def param_shapes(self):
        """state_dict keys/shapes in reference registration order (src/models/wrapper.py:24-100)."""
        D, fe = self.D, self.f_embed
        out = []
        if self.Fn > 0:
            out += [("num_embed.weight", (self.Fn, fe)), ("num_embed.bias", (self.Fn, fe)),
                    ("num_embed.out_proj.weight", (D, fe))]
        if self.Fm > 0:
            out += [("mask_embed.weight", (self.Fm, fe)), ("mask_embed.out_proj.weight", (D, fe))]
        for c, card, d in zip(self.cat_names, self.cat_cards, self.cat_dims):
            out.append((f"cat_embs.{c}.weight", (card, d)))
        for c, d in zip(self.cat_names, self.cat_dims):
            out.append((f"cat_proj.{c}.weight", (D, d)))
        ctx_in = D * ((self.Fn > 0) + (self.Fm > 0) + 1)
        out += [("ctx_mlp.0.weight", (D, ctx_in)), ("ctx_mlp.0.bias", (D,))]
        out += [("dare.emb_att.weight", (self.seq_vocab, D)), ("dare.emb_rep.weight", (self.seq_vocab, D))]
        for i in range(self.n_layers):
            p = f"dare.layers.{i}."
            out += [(p + "mha.in_proj_weight", (3 * D, D)), (p + "mha.in_proj_bias", (3 * D,)),
                    (p + "mha.out_proj.weight", (D, D)), (p + "mha.out_proj.bias", (D,)),
                    *norm_params(p + "norm1", D, self.layer_norm),
                    (p + "ffn.0.weight", (self.ffn_hidden, D)), (p + "ffn.0.bias", (self.ffn_hidden,)),
                    (p + "ffn.3.weight", (D, self.ffn_hidden)), (p + "ffn.3.bias", (D,)),
                    *norm_params(p + "norm2", D, self.layer_norm)]
            if self.add_pos:
                out.append((p + "pbias.rel.weight", (2 * self.top_k + 1, self.H)))
        out += [("dare.aux_head.weight", (1, D)), ("dare.aux_head.bias", (1,))]
        if self.use_qnn:
            FD = self.F * D
            C = self.qh * self.qP
            out += [("qnn.U", (self.qh, D, self.qr)), ("qnn.V", (self.qh, self.qr, self.qP)),
                    *norm_params("qnn.pre_norm", FD, self.qnn_layer_norm)]
            if self.use_se:
                Cr = C // self.se_r
                out += [("qnn.se.fc.0.weight", (Cr, C)), ("qnn.se.fc.0.bias", (Cr,)),
                        ("qnn.se.fc.2.weight", (C, Cr)), ("qnn.se.fc.2.bias", (C,))]
            din = C + FD
            for j, h in enumerate(self.mlp_hidden):
                out += [(f"qnn.mlp.{3 * j}.weight", (h, din)), (f"qnn.mlp.{3 * j}.bias", (h,))]
                din = h
            j = len(self.mlp_hidden)
            out += [(f"qnn.mlp.{3 * j}.weight", (1, din)), (f"qnn.mlp.{3 * j}.bias", (1,))]
        else:
            nin = D * (1 + (self.Fn > 0) + (self.Fm > 0) + self.Fc)
            out += [("fc.0.weight", (512, nin)), ("fc.0.bias", (512,)), ("fc.3.weight", (1, 512)),
                    ("fc.3.bias", (1,))]
        return out

    def grad_params(self):
        """Keys that receive a gradient (torch leaves the others' .grad None; AdamW skips them)."""
        keys = [k for k, _ in self.param_shapes()]
        skip = set()
        if self.query_mode == "S1":                 # src/models/wrapper.py:129-131: ctx_mlp unused
            skip |= {"ctx_mlp.0.weight", "ctx_mlp.0.bias"}
        if self.aux_w <= 0:                         # src/train.py:165-168: aux logit not in the loss
            skip |= {"dare.aux_head.weight", "dare.aux_head.bias"}
        return [k for k in keys if k not in skip]


def make_arch(cfg, seq_vocab, num_dim, mask_dim, cat_cardinals, cat_cols):
    return Arch(cfg, seq_vocab, num_dim, mask_dim, cat_cardinals, cat_cols)


def forward(P, batch, A: Arch, drop: Dropper, dtype=torch.float32, record=None):
    """CTRModel.forward (src/models/wrapper.py:138-176). Returns (logits, prob, aux)."""
    X_num = batch["X_num"].to(dtype)
    X_mask = batch["X_mask"].to(dtype)
    X_cat = batch["X_cat"].long()
    seq = batch["seq"].long()
    D = A.D
    num_e = mask_e = None
    if A.Fn > 0:   # src/models/feature_embed.py:19-27
        e = X_num.unsqueeze(-1) * P["num_embed.weight"] + P["num_embed.bias"]
        num_e = e @ P["num_embed.out_proj.weight"].t()
    if A.Fm > 0:   # src/models/feature_embed.py:42-48
        e = X_mask.unsqueeze(-1) * P["mask_embed.weight"]
        mask_e = e @ P["mask_embed.out_proj.weight"].t()
    cat_embs = []  # src/models/wrapper.py:106-112 (iterates cat_cols_order, X_cat column i)
    for i, c in enumerate(A.cat_cols):
        cat_embs.append(P[f"cat_embs.{c}.weight"][X_cat[:, i]] @ P[f"cat_proj.{c}.weight"].t())
    cat_stack = torch.stack(cat_embs, dim=1)
    cat_stack = drop(SITE_EMB, cat_stack, A.p_emb)            # src/models/wrapper.py:149-150
    parts = []                                                # src/models/wrapper.py:114-126
    if num_e is not None:
        parts.append(num_e.mean(dim=1))
    if mask_e is not None:
        parts.append(mask_e.mean(dim=1))
    parts.append(torch.stack(cat_embs, dim=1).mean(dim=1))
    ctx = torch.cat(parts, dim=1)
    qi = A.cat_cols.index(A.query_key) if A.query_mode != "S2" else None
    if A.query_mode == "S1":                                  # src/models/wrapper.py:128-136
        query = cat_embs[qi]
    elif A.query_mode == "S2":
        query = torch.relu(ctx @ P["ctx_mlp.0.weight"].t() + P["ctx_mlp.0.bias"])
    else:
        query = 0.5 * (cat_embs[qi] + torch.relu(ctx @ P["ctx_mlp.0.weight"].t() + P["ctx_mlp.0.bias"]))
    x, vals, idx = topk_select(P, seq, query, A.top_k, A.tau, A.pad_id, dtype)
    if record is not None:
        record["topk_idx"], record["topk_vals"], record["query"] = idx, vals, query
    for li in range(A.n_layers):                              # src/models/dare.py:142-146
        x = encoder_layer(P, f"dare.layers.{li}.", x, A.H, A.mha_p, A.ffn_p, A.add_pos, A.top_k, drop, li,
                          A.layer_norm)
    if A.gating == "relu":                                    # src/models/dare.py:150-155
        w = torch.relu(vals)
        w = w / (w.sum(dim=1, keepdim=True) + 1e-12)
    else:
        w = torch.softmax(vals, dim=1)
    u = (x * w.unsqueeze(-1)).sum(dim=1)
    u = drop(SITE_DARE, u, A.p_dare)
    aux = (u @ P["dare.aux_head.weight"].t() + P["dare.aux_head.bias"]).squeeze(1)
    if A.use_qnn:                                             # src/models/wrapper.py:160-166
        feats = [u.unsqueeze(1)]
        if num_e is not None:
            feats.append(num_e)
        if mask_e is not None:
            feats.append(mask_e)
        feats.append(cat_stack)
        xF = torch.cat(feats, dim=1)
        logits = qnn_forward(P, xF, A, drop)
    else:                                                     # src/models/wrapper.py:167-173
        feats = [u]
        if num_e is not None:
            feats.append(num_e.mean(dim=1))
        if mask_e is not None:
            feats.append(mask_e.mean(dim=1))
        feats += cat_embs
        h = torch.relu(torch.cat(feats, dim=1) @ P["fc.0.weight"].t() + P["fc.0.bias"])
        h = drop(SITE_FC, h, 0.1)
        logits = (h @ P["fc.3.weight"].t() + P["fc.3.bias"]).squeeze(1)
    return logits, torch.sigmoid(logits), aux


def _pair_all(P, z, A: Arch):
    # src/models/qnn_alpha.py:86-97
    outs = []
    for h in range(A.qh):
        Ah = z @ P["qnn.U"][h]
        s = Ah.sum(dim=1)
        quad = s * s - (Ah * Ah).sum(dim=1)
        outs.append(quad @ P["qnn.V"][h])
    return torch.cat(outs, dim=1)


def qnn_forward(P, feats, A: Arch, drop):
    # src/models/qnn_alpha.py:109-130
    B, Fq, D = feats.shape
    z = norm(feats.reshape(B, Fq * D), P, "qnn.pre_norm", A.qnn_layer_norm).reshape(B, Fq, D)
    blocks = [(s, e) for s, e in A.qnn_blocks() if e - s > 1] if A.pair_grouping == "block" else []
    if blocks:   # :99-108: the interaction within each block of more than one feature, summed over the blocks
        inter = torch.stack([_pair_all(P, z[:, s:e, :], A) for s, e in blocks], dim=0).sum(dim=0)
    else:
        inter = _pair_all(P, z, A)
    if A.use_se:   # src/models/qnn_alpha.py:17-26
        m = inter.mean(dim=0, keepdim=True)
        g = torch.relu(m @ P["qnn.se.fc.0.weight"].t() + P["qnn.se.fc.0.bias"])
        g = torch.sigmoid(g @ P["qnn.se.fc.2.weight"].t() + P["qnn.se.fc.2.bias"])
        inter = inter * g
    inter = drop(SITE_QNN, inter, A.qnn_p)
    base = z.reshape(B, Fq * D)
    out = torch.cat([base if A.use_residual else base.detach(), inter], dim=1)
    for j, _ in enumerate(A.mlp_hidden):
        out = torch.relu(out @ P[f"qnn.mlp.{3 * j}.weight"].t() + P[f"qnn.mlp.{3 * j}.bias"])
        out = drop(SITE_MLP0 + j, out, A.qnn_p)
    j = len(A.mlp_hidden)
    return (out @ P[f"qnn.mlp.{3 * j}.weight"].t() + P[f"qnn.mlp.{3 * j}.bias"]).squeeze(1)


def bce_wll_style(logits, labels):
    """src/train.py:71-90 restated: 0.5*mean_pos softplus(-z) + 0.5*mean_neg softplus(z)."""
    y = labels.to(dtype=logits.dtype)
    pos = y > 0.5
    neg = ~pos
    pl = F.softplus(-logits[pos]).mean() if pos.any() else torch.zeros((), dtype=logits.dtype)
    nl = F.softplus(logits[neg]).mean() if neg.any() else torch.zeros((), dtype=logits.dtype)
    return 0.5 * (pl + nl)


def cosine_warmup_lr(epoch, step, steps_per_epoch, base_lr, warmup_epochs=1, total_epochs=10):
    """src/utils/sched.py:3-11 restated."""
    g = epoch * steps_per_epoch + step
    w = warmup_epochs * steps_per_epoch
    tot = total_epochs * steps_per_epoch
    if g < w:
        return base_lr * (g + 1) / max(1, w)
    prog = (g - w) / max(1, tot - w)
    return 0.5 * base_lr * (1.0 + math.cos(math.pi * prog))


def ema_decay(base, warmup_steps, warmup_type, n_updates):
    """src/utils/ema.py:72-88 restated."""
    if warmup_steps <= 0 or warmup_type == "none":
        return base
    t = min(1.0, (n_updates + 1) / warmup_steps)
    if warmup_type == "linear":
        d = 1.0 - (1.0 - base) * t
    elif warmup_type == "cosine":
        d = 1.0 - (1.0 - base) * 0.5 * (1 + math.cos(math.pi * (1 - t)))
    else:
        d = base
    return float(max(0.0, min(1.0, d)))


class TrainState:
    """Optimizer + EMA state of the restated step loop (src/train.py:152-203)."""

    def __init__(self, P, A: Arch, lr, wd, clip, ema_cfg=None, betas=(0.9, 0.999), eps=1e-8):
        self.P = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}
        self.A, self.lr, self.wd, self.clip = A, lr, wd, clip
        self.b1, self.b2, self.eps = betas[0], betas[1], eps
        self.grad_keys = A.grad_params()
        self.m = {k: torch.zeros_like(self.P[k]) for k in self.grad_keys}
        self.v = {k: torch.zeros_like(self.P[k]) for k in self.grad_keys}
        self.step_n = 0
        self.ema_cfg = ema_cfg
        self.ema_n = 0
        self.shadow = {k: v.detach().clone() for k, v in self.P.items()} if ema_cfg else None

    native_dropout = False      # cpu baseline timing: torch's bernoulli dropout (Dropper.native)

    def grads(self, batch, y, seed, record=None):
        """forward -> loss (+aux) -> backward on one batch (src/train.py:158-192): (loss, outputs, grads)."""
        drop = Dropper(seed, training=True, native=self.native_dropout)
        for p in self.P.values():
            p.grad = None
        logits, prob, aux = forward(self.P, batch, self.A, drop, record=record)
        loss = bce_wll_style(logits, y)
        if self.A.aux_w > 0:
            loss = loss + self.A.aux_w * bce_wll_style(aux, y)
        loss.backward()
        grads = {k: self.P[k].grad.detach().clone() for k in self.grad_keys}
        return loss.detach(), (logits.detach(), prob.detach(), aux.detach()), grads

    @torch.no_grad()
    def apply(self, grads, lr):
        """clip_grad_norm_ -> AdamW -> EMA with the given grads (src/train.py:185-199).  Returns the norm."""
        gnorm = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g) for g in grads.values()]))
        coef = torch.clamp(self.clip / (gnorm + 1e-6), max=1.0) if self.clip > 0 else None
        self.step_n += 1
        bc1 = 1 - self.b1 ** self.step_n
        bc2 = 1 - self.b2 ** self.step_n
        for k in self.grad_keys:   # torch/optim/adam.py _single_tensor_adam (decoupled wd)
            p, g, m, v = self.P[k], grads[k], self.m[k], self.v[k]
            if coef is not None:
                g.mul_(coef)
            p.mul_(1 - lr * self.wd)
            m.lerp_(g, 1 - self.b1)
            v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            denom = (v.sqrt() / (bc2 ** 0.5)).add_(self.eps)
            p.addcdiv_(m, denom, value=-(lr / bc1))
        if self.shadow is not None:   # src/utils/ema.py:92-131
            e = self.ema_cfg
            d = ema_decay(float(e.get("decay", 0.999)), int(e.get("warmup_steps", 0)),
                          str(e.get("warmup_type", "linear")), self.ema_n)
            for k, p in self.P.items():
                self.shadow[k].mul_(d).add_(p.detach(), alpha=1.0 - d)
            self.ema_n += 1
        return gnorm

    def step(self, batch, y, lr, seed, record=None):
        """One step: forward -> loss -> backward -> clip -> AdamW -> EMA. Returns (loss, outputs, grads, gnorm)."""
        loss, outs, grads = self.grads(batch, y, seed, record=record)
        gnorm = self.apply({k: g.clone() for k, g in grads.items()}, lr)
        return loss, outs, grads, gnorm

    def step_data_parallel(self, batches, ys, lr, seeds):
        """One data-parallel step of the reference applied per replica: every replica's
        grads on its own batch (its own SE batch mean and loss class counts), averaged as DDP does, then
        one clip -> AdamW -> EMA.  Returns (losses, averaged grads before the clip, gnorm)."""
        losses, acc = [], None
        for b, y, sd in zip(batches, ys, seeds):
            loss, _, g = self.grads(b, y, sd)
            losses.append(loss)
            acc = g if acc is None else {k: acc[k] + g[k] for k in acc}
        avg = {k: v / len(batches) for k, v in acc.items()}
        mean_grads = {k: v.clone() for k, v in avg.items()}
        gnorm = self.apply(avg, lr)
        return losses, mean_grads, gnorm
