"""Static model shape derived from a reference-style cfg dict.

Mirrors the constructor logic of the reference ``CTRModel`` (src/models/wrapper.py:8-104),
``DARE`` (src/models/dare.py:78-110), ``DAREEncoderLayer`` (src/models/dare.py:39-51) and
``QNNAlphaDetailed`` (src/models/qnn_alpha.py:39-84): which parameters exist, their shapes and
their state_dict key order.
"""
from __future__ import annotations

from dataclasses import dataclass, field

QUERY_MODES = {"S1": 0, "S2": 1, "concat": 2}


@dataclass
class Arch:
    D: int
    f_embed: int
    p_emb: float
    cat_cols: list
    cat_names: list
    cat_cards: list
    cat_dims: list
    Fn: int
    Fm: int
    seq_vocab: int
    query_mode: str
    query_key: str
    top_k: int
    tau: float
    pad_id: int
    p_dare: float
    tb: bool
    n_layers: int
    H: int
    mha_p: float
    ffn_hidden: int
    ffn_p: float
    add_pos: bool
    gating: str
    norm: str
    use_qnn: bool
    aux_w: float
    qh: int = 0
    qr: int = 0
    qP: int = 0
    mlp_hidden: list = field(default_factory=list)
    qnn_p: float = 0.0
    use_se: bool = True
    se_r: int = 8
    use_residual: bool = True
    pair_grouping: str = "all"
    qnn_norm: str = "rms"
    amp: str = "none"          # cfg["amp"] (src/train.py:133-139): "none" (fp32) or "bf16"

    @property
    def Fc(self):
        return len(self.cat_names)

    @property
    def F(self):
        return 1 + self.Fn + self.Fm + self.Fc

    @property
    def C(self):
        return self.qh * self.qP

    def qnn_blocks(self):
        """The QNN's interaction blocks (pair_grouping 'block', src/models/qnn_alpha.py:99-108): the slices of the
        input [u | num | mask | cat] (src/models/wrapper.py:66-75) holding more than one feature, in that order;
        empty for 'all' (or when no block has two features: the reference then falls back to all pairs)."""
        if self.pair_grouping != "block":
            return []
        sizes = [1] + [n for n in (self.Fn, self.Fm) if n > 0] + [self.Fc]
        out, o = [], 0
        for n in sizes:
            if n > 1:
                out.append((o, o + n))
            o += n
        return out

    @property
    def nctx(self):
        return (self.Fn > 0) + (self.Fm > 0) + 1

    def K_eff(self, L):
        return min(self.top_k, L)

    @staticmethod
    def from_cfg(cfg, seq_vocab, num_feat_dim, mask_feat_dim, cat_cardinals, cat_cols_order):
        m, s = cfg["model"], cfg["sequence"]
        qa = m["qnn_alpha"]
        D = int(m["emb_dim"])
        dims_map = m.get("cat_embedding_dims", {}) or {}
        t = s.get("tfm", {}) or {}
        tb = bool(s["transformer_block"])
        a = Arch(
            D=D, f_embed=int(qa.get("feature_embed_dim", max(8, D // 4))),
            p_emb=float(m.get("embedding_dropout", 0.0)),
            cat_cols=list(cat_cols_order), cat_names=list(cat_cardinals),
            cat_cards=[int(cat_cardinals[c]) for c in cat_cardinals],
            cat_dims=[int(dims_map.get(c, D)) for c in cat_cardinals],
            Fn=int(num_feat_dim), Fm=int(mask_feat_dim), seq_vocab=int(seq_vocab),
            query_mode=s["query_mode"], query_key=s["query_key"], top_k=int(s["top_k"]),
            tau=float(s["recency_tau"]), pad_id=int(s["pad_id"]), p_dare=float(m["dare_dropout"]),
            tb=tb, n_layers=int(t.get("n_layers", 2)) if tb else 0, H=int(t.get("n_heads", 4)),
            mha_p=float(t.get("mha_dropout", 0.1)), ffn_hidden=int(t.get("ffn_hidden", 256)),
            ffn_p=float(t.get("ffn_dropout", 0.1)), add_pos=bool(t.get("add_positional_bias", True)),
            gating=t.get("gating", "softmax") if t else "softmax", norm=str(t.get("norm", "rms")),
            use_qnn=bool(qa["enabled"]), aux_w=float(qa.get("aux_head_weight", 0.0)),
            amp=str(cfg.get("amp", "none") or "none").lower(),
        )
        if a.use_qnn:
            a.qh, a.qr, a.qP = int(qa["heads"]), int(qa["rank"]), int(qa["proj_dim"])
            a.mlp_hidden = [int(h) for h in qa["mlp_hidden"]]
            a.qnn_p = float(qa["dropout"])
            a.use_se = bool(qa["use_se"])
            a.se_r = int(qa.get("se_reduction", 8))
            a.use_residual = bool(qa["use_residual"])
            a.pair_grouping = qa["pair_grouping"]
            a.qnn_norm = str(qa.get("norm", "rms"))
        a.validate()
        return a

    def validate(self):
        if self.query_mode not in QUERY_MODES:
            raise ValueError(f"unknown query_mode {self.query_mode}")
        if self.query_mode != "S2" and self.query_key not in self.cat_cols:
            raise ValueError(f"query_key {self.query_key} not in cat columns")
        if self.use_qnn and self.pair_grouping not in ("all", "block"):
            raise ValueError(f"unknown pair_grouping {self.pair_grouping!r}")
        if self.amp not in ("none", "bf16"):
            raise NotImplementedError(f"amp: {self.amp!r} -- the MI355X path runs fp32 or bf16 (amp: bf16)")
        if self.gating not in ("softmax", "relu"):
            raise ValueError(f"unknown gating {self.gating}")
        if self.D % 4 or self.D > 64:
            raise NotImplementedError("emb_dim must be a multiple of 4 and <= 64")
        if self.tb and (self.D % self.H or self.D // self.H > 16):
            raise NotImplementedError("n_heads must divide emb_dim with head dim <= 16")
        for d in self.cat_dims:
            if d < 4 or d > 64:
                raise NotImplementedError("cat_embedding_dims must be in [4, 64]")

    @property
    def layer_norm(self):
        """src/models/dare.py:15-18 make_norm: any norm name but "rms" is nn.LayerNorm (weight + bias, eps 1e-5)."""
        return bool(self.tb) and self.norm.lower() != "rms"

    @property
    def qnn_layer_norm(self):
        return bool(self.use_qnn) and self.qnn_norm.lower() != "rms"

    def param_shapes(self):
        """(state_dict key, shape, kind) in reference order; kind: 'dense' or 'table'."""
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
        out += [("ctx_mlp.0.weight", (D, self.nctx * D)), ("ctx_mlp.0.bias", (D,))]
        out += [("dare.emb_att.weight", (self.seq_vocab, D)), ("dare.emb_rep.weight", (self.seq_vocab, D))]
        for i in range(self.n_layers):
            p = f"dare.layers.{i}."
            out += [(p + "mha.in_proj_weight", (3 * D, D)), (p + "mha.in_proj_bias", (3 * D,)),
                    (p + "mha.out_proj.weight", (D, D)), (p + "mha.out_proj.bias", (D,)),
                    *self._norm_params(p + "norm1", D, self.layer_norm),
                    (p + "ffn.0.weight", (self.ffn_hidden, D)), (p + "ffn.0.bias", (self.ffn_hidden,)),
                    (p + "ffn.3.weight", (D, self.ffn_hidden)), (p + "ffn.3.bias", (D,)),
                    *self._norm_params(p + "norm2", D, self.layer_norm)]
            if self.add_pos:
                out.append((p + "pbias.rel.weight", (2 * self.top_k + 1, self.H)))
        out += [("dare.aux_head.weight", (1, D)), ("dare.aux_head.bias", (1,))]
        if self.use_qnn:
            FD, C = self.F * D, self.C
            out += [("qnn.U", (self.qh, D, self.qr)), ("qnn.V", (self.qh, self.qr, self.qP)),
                    *self._norm_params("qnn.pre_norm", FD, self.qnn_layer_norm)]
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
        return [(k, s, "table" if k.startswith("cat_embs.") or ".emb_" in k else "dense") for k, s in out]

    @staticmethod
    def _norm_params(name, d, layer):
        """RMSNorm: `w` (src/models/dare.py:10); nn.LayerNorm: `weight`, `bias`."""
        return [(name + ".weight", (d,)), (name + ".bias", (d,))] if layer else [(name + ".w", (d,))]

    def no_grad_keys(self):
        """Params whose .grad stays None in the reference step (AdamW skips them; EMA still tracks them)."""
        skip = set()
        if self.query_mode == "S1":     # src/models/wrapper.py:129-131: ctx_mlp never used
            skip |= {"ctx_mlp.0.weight", "ctx_mlp.0.bias"}
        if self.aux_w <= 0:             # src/train.py:165-168: aux logit not in the loss
            skip |= {"dare.aux_head.weight", "dare.aux_head.bias"}
        return skip
