"""Generate the golden parity fixtures by running the REFERENCE on CPU.

Runs only in the build container (``/root/reference`` is absent on the GPU box);
the outputs ``tests/golden/*.npz`` are committed data: inputs, seeds and the
reference's outputs / grads / post-step params (full, or fingerprints for large
tensors -- see oracle/synth.py).

What is executed from the reference (never copied into the repo):
  * ``src.models.wrapper.CTRModel`` (src/models/wrapper.py) -- forward/backward
  * ``src.utils.ema.build_ema`` / ``ModelEMA.update`` (src/utils/ema.py:92-131, 200-216)
  * ``src.utils.sched.cosine_warmup_lr`` (src/utils/sched.py:3-11)
  * ``bce_wll_style`` (src/train.py:71-90): ``src.train`` itself is not importable
    here (tensorboard missing via src/utils/log.py:3), so the function's own
    source is located by ``ast`` in src/train.py and executed.
  * ``torch.optim.AdamW`` + ``nn.utils.clip_grad_norm_`` exactly as
    src/train.py:133-139,185-195 drive them.
Dropout: ``torch.nn.functional.dropout`` is patched to apply the build's
counter-based masks (oracle/rng.py) in the reference's call order.

Usage:  python tests/golden/gen_golden.py            (writes tests/golden/*.npz)
"""
from __future__ import annotations

import ast
import copy
import json
import os
import sys

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, REF)

from oracle import rng, synth                      # noqa: E402
from oracle.model import (SITE_DARE, SITE_EMB, SITE_FC, SITE_MLP0, SITE_QNN,  # noqa: E402
                          make_arch, site_attn, site_ffn)

FULL_LIMIT = 40_000     # tensors up to this many elements are stored in full


def load_ref():
    from src.models.wrapper import CTRModel
    from src.models import dare as ref_dare
    from src.utils.ema import build_ema
    from src.utils.sched import cosine_warmup_lr
    src = open(os.path.join(REF, "src/train.py")).read()
    tree = ast.parse(src)
    fn = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "bce_wll_style"][0]
    ns = {"torch": torch, "F": F}
    exec(compile(ast.Module(body=[fn], type_ignores=[]), "src/train.py", "exec"), ns)
    return CTRModel, ref_dare, build_ema, cosine_warmup_lr, ns["bce_wll_style"]


def dropout_sites(A):
    """Reference F.dropout call order for one training forward (src/models/wrapper.py:150,
    src/models/dare.py:43-46,158, src/models/qnn_alpha.py:81,121)."""
    sites = [(SITE_EMB, A.p_emb)]
    for i in range(A.n_layers):
        if A.mha_p > 0:
            sites.append((site_attn(i), A.mha_p))
        sites.append((site_ffn(i), A.ffn_p))
    sites.append((SITE_DARE, A.p_dare))
    if A.use_qnn:
        sites.append((SITE_QNN, A.qnn_p))
        sites += [(SITE_MLP0 + j, A.qnn_p) for j in range(len(A.mlp_hidden))]
    else:
        sites.append((SITE_FC, 0.1))
    return sites


class DropPatch:
    def __init__(self, A):
        self.sites = dropout_sites(A)
        self.orig = F.dropout
        self.seed = None
        self.calls = 0

    def __call__(self, x, p=0.5, training=True, inplace=False):
        site, p_expect = self.sites[self.calls]
        self.calls += 1
        assert abs(p - p_expect) < 1e-12, (site, p, p_expect)
        if not training or p == 0.0:
            return x
        keep = torch.from_numpy(rng.keep_mask(self.seed, site, p, tuple(x.shape)))
        return x * keep.to(x.dtype).div_(1 - p)

    def __enter__(self):
        F.dropout = self
        return self

    def __exit__(self, *a):
        F.dropout = self.orig


def put(store, name, a, full=None):
    a = np.asarray(a)
    if full is None:
        full = a.size <= FULL_LIMIT
    if full or a.dtype.kind != "f":
        store[name] = a
    else:
        for k, v in synth.fingerprint(a).items():
            store[f"{name}@{k}"] = np.asarray(v)


def run_case(name, cfg, B, L, vocab, Fn, Fm, cat_cards, steps, pseed, bseed, store_params, train_cfg,
             y_override=None, lognormal=False):
    CTRModel, ref_dare, build_ema, cosine_warmup_lr, bce_wll_style = load_ref()
    cat_cols = list(cat_cards)
    A = make_arch(cfg, vocab, Fn, Fm, cat_cards, cat_cols)
    torch.manual_seed(0)
    model = CTRModel(cfg, vocab, Fn, Fm, dict(cat_cards), cat_cols)
    P0 = synth.make_params(A.param_shapes(), pseed, pad_id=A.pad_id)
    sd = model.state_dict()
    assert list(sd.keys()) == [k for k, _ in A.param_shapes()], "state_dict order/keys mismatch"
    model.load_state_dict({k: torch.from_numpy(v) for k, v in P0.items()}, strict=True)
    ema = build_ema(model, cfg)
    opt = torch.optim.AdamW(model.parameters(), lr=train_cfg["lr"], weight_decay=train_cfg["wd"])
    aux_w = float(cfg["model"]["qnn_alpha"].get("aux_head_weight", 0.0))
    store = {}
    meta = dict(name=name, cfg=cfg, B=B, L=L, vocab=vocab, Fn=Fn, Fm=Fm, cat_cards=cat_cards,
                steps=steps, pseed=pseed, bseed=bseed, store_params=store_params, train=train_cfg,
                lrs=[], seeds=[])
    if store_params:
        for k, v in P0.items():
            store[f"p0/{k}"] = v
    topk_rec = {}
    orig_topk = ref_dare.DARE.topk_select

    def topk_rec_wrap(self, seq_ids, query_vec):
        orig_gather = torch.gather

        def g(inp, dim, index, **kw):
            topk_rec["idx"] = index[:, :, 0].clone()
            return orig_gather(inp, dim, index, **kw)
        torch.gather = g
        try:
            sel, vals = orig_topk(self, seq_ids, query_vec)
        finally:
            torch.gather = orig_gather
        topk_rec["vals"] = vals.detach().clone()
        topk_rec["query"] = query_vec.detach().clone()
        return sel, vals

    ref_dare.DARE.topk_select = topk_rec_wrap
    patch = DropPatch(A)
    spe = train_cfg["steps_per_epoch"]
    try:
        for t in range(steps):
            bt = synth.make_batch(B, Fn, Fm, list(cat_cards.values()), L, vocab, bseed + t,
                                  pad_id=A.pad_id, lognormal=lognormal)
            if y_override is not None and y_override.get(t) is not None:
                bt["y"] = np.full(B, y_override[t], np.int8)
            for k, v in bt.items():
                store[f"in{t}/{k}"] = v
            batch = {"X_num": torch.from_numpy(bt["X_num"]).float(),
                     "X_mask": torch.from_numpy(bt["X_mask"]).float(),
                     "X_cat": torch.from_numpy(bt["X_cat"]).long(),
                     "seq": torch.from_numpy(bt["seq"]).long()}
            y = torch.from_numpy(bt["y"]).float()
            lr = cosine_warmup_lr(0, t, spe, train_cfg["lr"], train_cfg["warmup_epochs"], train_cfg["epochs"])
            seed = (pseed << 32) | (t + 1)
            meta["lrs"].append(lr)
            meta["seeds"].append(seed)
            model.train()
            opt.param_groups[0]["lr"] = lr
            opt.zero_grad(set_to_none=True)
            patch.seed, patch.calls = seed, 0
            with patch:
                logits, prob, aux = model(batch)
            assert patch.calls == len(patch.sites), (patch.calls, patch.sites)
            loss = bce_wll_style(logits, y)
            if aux_w > 0:
                loss = loss + aux_w * bce_wll_style(aux, y)
            loss.backward()
            if t == 0:   # raw (pre-clip) grads of the first step
                names = []
                for k, p in model.named_parameters():
                    if p.grad is None:
                        continue
                    names.append(k)
                    put(store, f"grad0/{k}", p.grad.numpy().copy())
                meta["grad_keys"] = names
            gn = nn.utils.clip_grad_norm_(model.parameters(), train_cfg["clip"]) if train_cfg["clip"] > 0 else None
            store[f"out{t}/logits"] = logits.detach().numpy()
            store[f"out{t}/prob"] = prob.detach().numpy()
            store[f"out{t}/aux"] = aux.detach().numpy()
            store[f"out{t}/loss"] = np.float64(loss.item())
            store[f"out{t}/gnorm"] = np.float64(float(gn) if gn is not None else -1.0)
            store[f"out{t}/topk_idx"] = topk_rec["idx"].numpy().astype(np.int32)
            store[f"out{t}/topk_vals"] = topk_rec["vals"].numpy()
            store[f"out{t}/query"] = topk_rec["query"].numpy()
            opt.step()
            if ema is not None:
                ema.update(model, t + 1)
        for k, p in model.named_parameters():
            put(store, f"pT/{k}", p.detach().numpy())
            if p in opt.state and len(opt.state[p]):
                put(store, f"mT/{k}", opt.state[p]["exp_avg"].numpy())
                put(store, f"vT/{k}", opt.state[p]["exp_avg_sq"].numpy())
        if ema is not None:
            for k, v in ema.shadow_params.items():
                put(store, f"emaT/{k}", v.numpy())
        # eval forward with the final params on the last batch
        model.eval()
        patch.calls = 0
        with torch.no_grad():
            z, p_, a_ = model(batch)
        store["eval/logits"], store["eval/prob"], store["eval/aux"] = z.numpy(), p_.numpy(), a_.numpy()
    finally:
        ref_dare.DARE.topk_select = orig_topk
    store["meta"] = np.array(json.dumps(meta))
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **store)
    print(f"wrote {path}: {os.path.getsize(path) / 1e6:.2f} MB, {len(store)} arrays")


def tiny_cfg(query_mode="concat", gating="softmax", emb_drop=0.0, aux_w=0.1, qnn=True, tb=True,
             D=16, K=16, H=4, layers=2, ema=True):
    dims = {"c0": 8, "c1": 12, "c2": 16, "c3": 4, "c4": 20}
    cfg = {
        "model": {"emb_dim": D, "embedding_dropout": emb_drop, "cat_embedding_dims": dims, "dare_dropout": 0.2,
                  "qnn_alpha": {"enabled": qnn, "feature_embed_dim": 8, "heads": 2, "rank": 4, "proj_dim": 16,
                                "mlp_hidden": [32, 16], "dropout": 0.2, "use_se": True, "se_reduction": 4,
                                "use_residual": True, "norm": "rms", "pair_grouping": "all",
                                "aux_head_weight": aux_w}},
        "sequence": {"tfm": {"n_layers": layers, "n_heads": H, "mha_dropout": 0.1, "ffn_hidden": 48,
                             "ffn_dropout": 0.1, "norm": "rms", "gating": gating, "add_positional_bias": True},
                     "query_mode": query_mode, "transformer_block": tb, "top_k": K, "recency_tau": 16,
                     "pad_id": 0, "query_key": "c1"},
    }
    if ema:
        cfg["ema"] = {"enabled": True, "decay": 0.99, "warmup_steps": 5, "warmup_type": "linear"}
    return cfg


def cfg2_cfg():
    """cfgs/dare_qnn_next.yaml model/sequence blocks with the BASELINE cfg2 overrides (D=32)."""
    import yaml
    c = yaml.safe_load(open(os.path.join(REF, "cfgs/dare_qnn_next.yaml")))
    cfg = {"model": copy.deepcopy(c["model"]), "sequence": copy.deepcopy(c["sequence"]),
           "ema": copy.deepcopy(c["ema"])}
    cfg["model"]["emb_dim"] = 32
    cfg["sequence"]["max_len"] = 100
    return cfg, list(c["data"]["cat_cols"])


def k148_cfg():
    import yaml
    c = yaml.safe_load(open(os.path.join(REF, "cfgs/v3_k148_s1.yaml")))
    cfg = {"model": copy.deepcopy(c["model"]), "sequence": copy.deepcopy(c["sequence"])}
    cfg["sequence"]["tfm"]["n_layers"] = 1
    cfg["model"]["qnn_alpha"]["mlp_hidden"] = [64, 32]
    return cfg, list(c["data"]["cat_cols"])


def main():
    torch.set_num_threads(8)
    tr = dict(lr=3e-3, wd=1e-4, clip=0.5, steps_per_epoch=4, warmup_epochs=1, epochs=3)
    cards = {"c0": 300, "c1": 500, "c2": 1000, "c3": 200, "c4": 700}
    run_case("tiny_concat", tiny_cfg(), B=64, L=32, vocab=5000, Fn=6, Fm=6, cat_cards=cards, steps=3,
             pseed=11, bseed=100, store_params=True, train_cfg=tr)
    run_case("tiny_s1_relu", tiny_cfg(query_mode="S1", gating="relu", emb_drop=0.1, aux_w=0.0, ema=False),
             B=48, L=24, vocab=3000, Fn=5, Fm=4, cat_cards=cards, steps=2, pseed=12, bseed=200,
             store_params=True, train_cfg=dict(tr, clip=0.0), y_override={1: 0}, lognormal=True)
    run_case("tiny_s2", tiny_cfg(query_mode="S2", layers=1, K=8, H=2), B=32, L=12, vocab=2000, Fn=3, Fm=3,
             cat_cards=cards, steps=2, pseed=13, bseed=300, store_params=True, train_cfg=tr)
    run_case("base_fc", tiny_cfg(query_mode="S1", qnn=False, tb=False, K=20, ema=False), B=40, L=40,
             vocab=4000, Fn=4, Fm=4, cat_cards=cards, steps=2, pseed=14, bseed=400, store_params=True,
             train_cfg=dict(tr, clip=1.0))
    cfg2, cols = cfg2_cfg()
    run_case("cfg2_dims", cfg2, B=8, L=100, vocab=3000, Fn=82, Fm=82, cat_cards={c: 200 for c in cols},
             steps=1, pseed=21, bseed=500, store_params=False,
             train_cfg=dict(lr=3e-4, wd=1e-4, clip=0.5, steps_per_epoch=10, warmup_epochs=2, epochs=8))
    cfg4, cols4 = k148_cfg()
    run_case("k148", cfg4, B=4, L=160, vocab=2000, Fn=10, Fm=10, cat_cards={c: 100 for c in cols4[:6]},
             steps=1, pseed=31, bseed=600, store_params=False,
             train_cfg=dict(lr=3e-4, wd=1e-4, clip=0.5, steps_per_epoch=10, warmup_epochs=2, epochs=8))


if __name__ == "__main__":
    main()
