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
import contextlib
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
ALLOW_EPS = 1e-4        # gradient perturbation of the update-sensitivity replays (update_allowance): the
                        # north star's 1e-4 rtol on gradients, as a norm-wise relative error
ALLOW_REPLAYS = 2


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


def put(store, name, a, full=None, rows=None):
    """Store ``a`` in full when small, else its fingerprint (oracle/synth.py); for an embedding table
    also the rows the fixture's batches touch (``rows``), in full: ``name@rows`` / ``name@rowvals``."""
    a = np.asarray(a)
    if full is None:
        full = a.size <= FULL_LIMIT
    if full or a.dtype.kind != "f":
        store[name] = a
    else:
        for k, v in synth.fingerprint(a).items():
            store[f"{name}@{k}"] = np.asarray(v)
        if rows is not None:
            store[f"{name}@rows"] = np.asarray(rows, np.int64)
            store[f"{name}@rowvals"] = a.reshape(a.shape[0], -1)[rows]


def adamw_replay(P0, gsteps, lrs, wd, ema_cfg, eps_rel, seed):
    """torch.optim.AdamW's single-tensor step (decoupled wd; torch/optim/adam.py) + ModelEMA.update
    (src/utils/ema.py:92-131) replayed from P0 over recorded clipped gradients, each nonzero gradient
    element perturbed by N(0, (eps_rel * rms(g))^2) -- a stand-in for another implementation whose
    gradients differ from the reference's by reduction-order rounding of relative size eps_rel."""
    from oracle.model import ema_decay
    gen = torch.Generator().manual_seed(seed)
    P = {k: torch.from_numpy(v.copy()) for k, v in P0.items()}
    m, v = {}, {}
    sh = {k: t.clone() for k, t in P.items()} if ema_cfg else None
    for t, (gs, lr) in enumerate(zip(gsteps, lrs)):
        bc1, bc2 = 1 - 0.9 ** (t + 1), 1 - 0.999 ** (t + 1)
        for k, g in gs.items():
            if eps_rel > 0:
                nz = g != 0
                rms = float(g[nz].pow(2).mean().sqrt()) if bool(nz.any()) else 0.0
                g = g + torch.randn(g.shape, generator=gen) * (eps_rel * rms) * nz
            p = P[k]
            mk, vk = m.setdefault(k, torch.zeros_like(p)), v.setdefault(k, torch.zeros_like(p))
            p.mul_(1 - lr * wd)
            mk.lerp_(g, 1 - 0.9)
            vk.mul_(0.999).addcmul_(g, g, value=1 - 0.999)
            p.addcdiv_(mk, (vk.sqrt() / bc2 ** 0.5).add_(1e-8), value=-(lr / bc1))
        if sh is not None:
            d = ema_decay(float(ema_cfg.get("decay", 0.999)), int(ema_cfg.get("warmup_steps", 0)),
                          str(ema_cfg.get("warmup_type", "linear")), t)
            for k in sh:
                sh[k].mul_(d).add_(P[k], alpha=1.0 - d)
    return P, sh, m, v


def update_allowance(P0, gsteps, lrs, wd, ema_cfg, pT, shT, mT, vT, replays=ALLOW_REPLAYS):
    """Per-element allowances for comparing the update pT - p0, the EMA shadow's, and both Adam moments:
    3x the largest deviation over ALLOW_REPLAYS replays whose gradients are perturbed by a norm-wise
    relative ALLOW_EPS -- what gradients within the north star's tolerance can do to the state after the
    fixture's steps.  AdamW's m_hat / (sqrt(v_hat) + eps) is ill-conditioned where the (clipped) gradient
    is within a few eps of 0 or a cancellation residue far below its tensor's scale, and the first
    moment cancels where consecutive gradients oppose; the replays measure that element by element
    instead of guessing it.  The unperturbed replay must reproduce the reference bitwise."""
    P, sh, m0, v0 = adamw_replay(P0, gsteps, lrs, wd, ema_cfg, 0.0, 0)
    for k in P:
        assert np.array_equal(P[k].numpy(), pT[k]), f"AdamW replay differs from the reference on {k}"
    for k in mT:
        assert np.array_equal(m0[k].numpy(), mT[k]) and np.array_equal(v0[k].numpy(), vT[k]), k
    z = {k: np.zeros(v.size) for k, v in P0.items()}
    al = {"dT": dict(z), "demaT": dict(z) if sh is not None else {}, "mT": {k: z[k] for k in mT},
          "vT": {k: z[k] for k in mT}}
    refs = {"dT": pT, "demaT": shT, "mT": mT, "vT": vT}
    for r in range(replays):
        got = dict(zip(("dT", "demaT", "mT", "vT"), adamw_replay(P0, gsteps, lrs, wd, ema_cfg, ALLOW_EPS, 1000 + r)))
        for kind, d in al.items():
            for k in d:
                dev = np.abs(got[kind][k].numpy().astype(np.float64) - refs[kind][k].astype(np.float64)).ravel()
                d[k] = np.maximum(d[k], 3 * dev)
    return al


def put_allow(store, name, allow, rows, shape):
    """An allowance vector in full (small tensors) or where the checks read it: at the fingerprint's
    sampled elements (``@idx``), at the touched rows (``@rows``), and its L2 norm (``@norm``)."""
    allow = np.asarray(allow, np.float64).ravel()
    if allow.size <= FULL_LIMIT:
        store[name] = allow.astype(np.float32)
        return
    idx = synth.fingerprint(np.zeros(allow.size, np.float32))["idx"]
    store[f"{name}@idx"] = allow[idx].astype(np.float32)
    if rows is not None:
        store[f"{name}@rows"] = allow.reshape(shape[0], -1)[rows].astype(np.float32)
    store[f"{name}@norm"] = np.float64(np.linalg.norm(allow))


def run_case(name, cfg, B, L, vocab, Fn, Fm, cat_cards, steps, pseed, bseed, store_params, train_cfg,
             y_override=None, lognormal=False, amp_twin=None, allow_replays=ALLOW_REPLAYS, init="synthetic"):
    """One fixture.  ``amp_twin``: the name of the fp32 fixture this case repeats (same inputs, seeds and
    parameters) under ``amp: bf16`` -- the forward and the loss run inside
    ``torch.autocast("cpu", dtype=torch.bfloat16)`` as src/train.py:158-164 wraps them in
    ``torch.cuda.amp.autocast(dtype=bfloat16)`` (CPU autocast here: no GPU in the generating container);
    backward, clip, AdamW and EMA outside it, on the fp32 master parameters.

    ``init="reference"``: the parameters are the reference's OWN initialisation (``torch.manual_seed(pseed)``
    before ``CTRModel(...)``), which ``oracle.synth.reference_init`` restates -- asserted bitwise here, so the
    GPU box (no reference there) rebuilds P0 from the seed; ``"synthetic"``: ``oracle.synth.make_params``."""
    CTRModel, ref_dare, build_ema, cosine_warmup_lr, bce_wll_style = load_ref()
    if amp_twin is not None:
        cfg = dict(cfg, amp="bf16")
    amp_ctx = (lambda: torch.autocast("cpu", dtype=torch.bfloat16)) if amp_twin else contextlib.nullcontext
    cat_cols = list(cat_cards)
    A = make_arch(cfg, vocab, Fn, Fm, cat_cards, cat_cols)
    torch.manual_seed(pseed if init == "reference" else 0)
    model = CTRModel(cfg, vocab, Fn, Fm, dict(cat_cards), cat_cols)
    sd = model.state_dict()
    assert list(sd.keys()) == [k for k, _ in A.param_shapes()], "state_dict order/keys mismatch"
    if init == "reference":
        P0 = synth.reference_init(A, pseed)
        for k, v in sd.items():
            assert np.array_equal(v.numpy(), P0[k]), f"reference_init differs from the reference's init on {k}"
    else:
        P0 = synth.make_params(A.param_shapes(), pseed, pad_id=A.pad_id)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in P0.items()}, strict=True)
    ema = build_ema(model, cfg)
    opt = torch.optim.AdamW(model.parameters(), lr=train_cfg["lr"], weight_decay=train_cfg["wd"])
    aux_w = float(cfg["model"]["qnn_alpha"].get("aux_head_weight", 0.0))
    store = {}
    meta = dict(name=name, cfg=cfg, B=B, L=L, vocab=vocab, Fn=Fn, Fm=Fm, cat_cards=cat_cards,
                steps=steps, pseed=pseed, bseed=bseed, store_params=store_params, train=train_cfg,
                lrs=[], seeds=[], amp="bf16" if amp_twin else "none", twin=amp_twin, init=init)
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
    touched = {}     # table key -> rows any batch of the fixture reads
    gsteps = []      # the clipped gradients AdamW consumed at each step

    def touch(key, ids):
        touched[key] = np.union1d(touched.get(key, np.zeros(0, np.int64)), np.asarray(ids, np.int64).ravel())
    try:
        for t in range(steps):
            bt = synth.make_batch(B, Fn, Fm, list(cat_cards.values()), L, vocab, bseed + t,
                                  pad_id=A.pad_id, lognormal=lognormal)
            if y_override is not None and y_override.get(t) is not None:
                bt["y"] = np.full(B, y_override[t], np.int8)
            touch("dare.emb_att.weight", bt["seq"])
            touch("dare.emb_rep.weight", bt["seq"])
            for i, c in enumerate(cat_cols):
                touch(f"cat_embs.{c}.weight", bt["X_cat"][:, i])
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
            with patch, amp_ctx():
                logits, prob, aux = model(batch)
                loss = bce_wll_style(logits, y)
                if aux_w > 0:
                    loss = loss + aux_w * bce_wll_style(aux, y)
            assert patch.calls == len(patch.sites), (patch.calls, patch.sites)
            loss.backward()
            if t == 0:   # raw (pre-clip) grads of the first step
                names = []
                for k, p in model.named_parameters():
                    if p.grad is None:
                        continue
                    names.append(k)
                    put(store, f"grad0/{k}", p.grad.numpy().copy(), rows=touched.get(k))
                meta["grad_keys"] = names
            gn = nn.utils.clip_grad_norm_(model.parameters(), train_cfg["clip"]) if train_cfg["clip"] > 0 else None
            store[f"out{t}/logits"] = logits.detach().float().numpy()
            store[f"out{t}/prob"] = prob.detach().float().numpy()
            store[f"out{t}/aux"] = aux.detach().float().numpy()
            store[f"out{t}/loss"] = np.float64(loss.item())
            store[f"out{t}/gnorm"] = np.float64(float(gn) if gn is not None else -1.0)
            store[f"out{t}/topk_idx"] = topk_rec["idx"].numpy().astype(np.int32)
            store[f"out{t}/topk_vals"] = topk_rec["vals"].float().numpy()
            store[f"out{t}/query"] = topk_rec["query"].float().numpy()
            gsteps.append({k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None})
            opt.step()
            if ema is not None:
                ema.update(model, t + 1)
        shadow = dict(ema.shadow_params) if ema is not None else {}
        # per-element allowances for the update comparisons (see update_allowance)
        pT = {k: p.detach().numpy() for k, p in model.named_parameters()}
        mT = {k: opt.state[p]["exp_avg"].numpy() for k, p in model.named_parameters() if p in opt.state and opt.state[p]}
        vT = {k: opt.state[p]["exp_avg_sq"].numpy() for k, p in model.named_parameters()
              if p in opt.state and opt.state[p]}
        # bf16 twins are compared through their bf16-vs-fp32 noise band, not the replay allowances
        allow = {} if amp_twin else update_allowance(P0, gsteps, meta["lrs"], train_cfg["wd"],
                                                     cfg.get("ema") if ema else None, pT,
                                                     {k: v.numpy() for k, v in shadow.items()}, mT, vT,
                                                     replays=allow_replays)
        for kind, d in allow.items():
            if kind not in ("dT", "demaT"):     # moments are compared without an allowance
                continue
            for k, a in d.items():
                put_allow(store, f"{kind}allow/{k}", a, touched.get(k), P0[k].shape)
        for k, p in model.named_parameters():
            rows = touched.get(k)
            put(store, f"pT/{k}", p.detach().numpy())
            # the update itself, dT = pT - p0: what the parity tests compare norm-wise
            put(store, f"dT/{k}", p.detach().numpy().astype(np.float64) - P0[k].astype(np.float64), rows=rows)
            if p in opt.state and len(opt.state[p]):
                put(store, f"mT/{k}", opt.state[p]["exp_avg"].numpy(), rows=rows)
                put(store, f"vT/{k}", opt.state[p]["exp_avg_sq"].numpy(), rows=rows)
        if ema is not None:
            for k, v in ema.shadow_params.items():
                put(store, f"emaT/{k}", v.numpy())
                put(store, f"demaT/{k}", v.numpy().astype(np.float64) - P0[k].astype(np.float64),
                    rows=touched.get(k))
        # eval forward with the final params on the last batch
        model.eval()
        patch.calls = 0
        with torch.no_grad(), amp_ctx():
            z, p_, a_ = model(batch)
        store["eval/logits"], store["eval/prob"], store["eval/aux"] = (z.float().numpy(), p_.float().numpy(),
                                                                        a_.float().numpy())
    finally:
        ref_dare.DARE.topk_select = orig_topk
    store["meta"] = np.array(json.dumps(meta))
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **store)
    print(f"wrote {path}: {os.path.getsize(path) / 1e6:.2f} MB, {len(store)} arrays")


def tiny_cfg(query_mode="concat", gating="softmax", emb_drop=0.0, aux_w=0.1, qnn=True, tb=True,
             D=16, K=16, H=4, layers=2, ema=True, ffn_hidden=48, pair_grouping="all", norm="rms", qnn_norm="rms"):
    dims = {"c0": 8, "c1": 12, "c2": 16, "c3": 4, "c4": 20}
    cfg = {
        "model": {"emb_dim": D, "embedding_dropout": emb_drop, "cat_embedding_dims": dims, "dare_dropout": 0.2,
                  "qnn_alpha": {"enabled": qnn, "feature_embed_dim": 8, "heads": 2, "rank": 4, "proj_dim": 16,
                                "mlp_hidden": [32, 16], "dropout": 0.2, "use_se": True, "se_reduction": 4,
                                "use_residual": True, "norm": qnn_norm, "pair_grouping": pair_grouping,
                                "aux_head_weight": aux_w}},
        "sequence": {"tfm": {"n_layers": layers, "n_heads": H, "mha_dropout": 0.1, "ffn_hidden": ffn_hidden,
                             "ffn_dropout": 0.1, "norm": norm, "gating": gating, "add_positional_bias": True},
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


def cfg4_full_cfg():
    """cfgs/v3_k148_s1.yaml as-is (BASELINE config 4): D = 64, L = 400, K = 148, 4 encoder layers, S1, the
    full QNN head (MLP 13952 -> 512 -> 256 -> 1), EMA off."""
    import yaml
    c = yaml.safe_load(open(os.path.join(REF, "cfgs/v3_k148_s1.yaml")))
    cfg = {"model": copy.deepcopy(c["model"]), "sequence": copy.deepcopy(c["sequence"])}
    return cfg, list(c["data"]["cat_cols"]), len(c["data"]["num_cols_explicit"])


def cfg3_cfg():
    """cfgs/dare_qnn_next_k100_s1.yaml (BASELINE config 3: K=100, query S1, EMA on) with the cfg2
    overrides D=32, L=100."""
    import yaml
    c = yaml.safe_load(open(os.path.join(REF, "cfgs/dare_qnn_next_k100_s1.yaml")))
    cfg = {"model": copy.deepcopy(c["model"]), "sequence": copy.deepcopy(c["sequence"]),
           "ema": copy.deepcopy(c["ema"])}
    cfg["model"]["emb_dim"] = 32
    cfg["sequence"]["max_len"] = 100
    return cfg, list(c["data"]["cat_cols"])


def k120_cfg():
    """cfgs/v3_k120_s1.yaml as-is (D=64, K=120, S1) with 2 of its 4 encoder layers and a narrower MLP."""
    import yaml
    c = yaml.safe_load(open(os.path.join(REF, "cfgs/v3_k120_s1.yaml")))
    cfg = {"model": copy.deepcopy(c["model"]), "sequence": copy.deepcopy(c["sequence"])}
    cfg["sequence"]["tfm"]["n_layers"] = 2
    cfg["model"]["qnn_alpha"]["mlp_hidden"] = [64, 32]
    return cfg, list(c["data"]["cat_cols"])


def gen_infer():
    """Fold-ensemble + calibration fixtures: the reference's own
    ``src.utils.metrics.ensemble_probs`` (src/utils/metrics.py:48-86) and ``src.utils.calibration.Calibrator``
    (src/utils/calibration.py:54-110) run on fixed inputs; writes tests/golden/infer_ref.npz."""
    from src.utils.calibration import Calibrator
    from src.utils.metrics import ensemble_probs
    r = np.random.default_rng(4242)
    store = {}
    B = 257
    methods = ["mean", "geom_mean", "logit_mean", "median", "trim_mean", "weighted", "val_weighted", "rank_avg"]
    meta = {"B": B, "Ms": [2, 3, 4, 5], "methods": methods, "trim_ratio": 0.34, "val_weight_temperature": 5.0}
    for M in meta["Ms"]:
        z = (2.0 * r.standard_normal((M, B))).astype(np.float32)
        z[:, 5] = 30.0                      # saturated: every model clips to 1 - 1e-7
        z[:, 6] = -30.0
        z[1:, 7] = z[0, 7]                  # equal across models (median / trim ties)
        # the reference's inference loop clamps each model's probabilities (src/infer.py:122);
        # no exact ties inside one model, so rank_avg's argsort order is unambiguous
        p = torch.clamp(torch.sigmoid(torch.from_numpy(z)), 1e-7, 1.0 - 1e-7)
        assert all(torch.unique(p[i]).numel() == B for i in range(M))
        p_list = [p[i].clone() for i in range(M)]
        scores = r.uniform(0.30, 0.36, M).astype(np.float32)
        weights = r.uniform(0.1, 1.0, M).astype(np.float32)
        store[f"ens{M}/p"] = p.numpy()
        store[f"ens{M}/scores"] = scores
        store[f"ens{M}/weights"] = weights
        for method in methods:
            w, use = None, method
            if method == "val_weighted":     # src/infer.py:135-149
                w = torch.softmax(torch.from_numpy(scores) / max(1e-6, meta["val_weight_temperature"]), dim=0)
                use = "weighted"
            elif method == "weighted":       # src/infer.py:150-154
                w = torch.from_numpy(weights)
            try:
                out = ensemble_probs(use, p_list, weights=w, trim_ratio=meta["trim_ratio"])
            except RuntimeError as e:
                # rank_avg: _rank_avg_stack scatters an int64 arange into a float tensor
                # (src/utils/metrics.py:43), which torch rejects -- the reference cannot run it
                meta.setdefault("raises", {})[method] = str(e).splitlines()[0]
                continue
            store[f"ens{M}/{method}"] = out.numpy()
    # calibration: logits from a miscalibrated model, labels drawn from a sharper one
    n = 6000
    z = (1.5 * r.standard_normal(n) - 1.0).astype(np.float32)
    y = (r.random(n) < 1.0 / (1.0 + np.exp(-(0.6 * z - 1.5)))).astype(np.int64)
    zq = np.concatenate([np.linspace(-60, 60, 241), z[:500]]).astype(np.float32)
    store["cal/z"], store["cal/y"], store["cal/zq"] = z, y, zq
    zf = np.round(z).clip(-2, 2).astype(np.float32)        # 5 distinct values: isotonic falls back
    store["cal/z_few"] = zf
    cases = [("temperature", z), ("isotonic", z), ("temperature+isotonic", z), ("isotonic", zf),
             ("temperature+isotonic", zf)]
    meta["cal_cases"] = []
    for i, (method, zz) in enumerate(cases):
        cal = Calibrator(method=method, lr=0.05, iters=200)
        cal.fit(zz, y)
        tag = f"cal{i}"
        meta["cal_cases"].append({"tag": tag, "method": method, "few": zz is zf})
        if cal.temp_scaler is not None:
            T = torch.clamp(torch.exp(cal.temp_scaler.log_temp.detach()), cal.clamp_T[0], cal.clamp_T[1])
            store[f"{tag}/T"] = np.float64(float(T))
        if cal.iso is not None:
            store[f"{tag}/iso_x"] = np.asarray(cal.iso.X_thresholds_, np.float64)
            store[f"{tag}/iso_y"] = np.asarray(cal.iso.y_thresholds_, np.float64)
        store[f"{tag}/pq"] = cal.predict_proba(zq)
    store["meta"] = np.array(json.dumps(meta))
    path = os.path.join(HERE, "infer_ref.npz")
    np.savez_compressed(path, **store)
    print(f"wrote {path}: {os.path.getsize(path) / 1e6:.2f} MB, {len(store)} arrays")


def main():
    torch.set_num_threads(8)
    if "--infer-only" in sys.argv:
        gen_infer()
        return
    if "--bf16-only" in sys.argv:
        gen_bf16()
        return
    if "--r3" in sys.argv:
        gen_r3()
        return
    if "--cfg4" in sys.argv:
        gen_r3(only_cfg4=True)
        return
    if "--r4" in sys.argv:
        gen_r4()
        return
    if "--r5" in sys.argv:
        gen_r5()
        return
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
    # lr 3e-3 without warmup: the update (~3e-3 per step) spans ~1e4 fp32 ulps of the |p| ~ 1 table
    # entries it moves, so pT - p0 can be compared at 1e-4 (at warmup lrs ~1e-5 it would be ~100 ulps)
    big_tr = dict(lr=3e-3, wd=1e-4, clip=0.5, steps_per_epoch=10, warmup_epochs=0, epochs=8)
    cfg2, cols = cfg2_cfg()
    run_case("cfg2_dims", cfg2, B=8, L=100, vocab=3000, Fn=82, Fm=82, cat_cards={c: 200 for c in cols},
             steps=2, pseed=21, bseed=500, store_params=False, train_cfg=big_tr)
    cfg3, cols3 = cfg3_cfg()
    run_case("cfg3_dims", cfg3, B=8, L=100, vocab=3000, Fn=82, Fm=82, cat_cards={c: 200 for c in cols3},
             steps=2, pseed=41, bseed=700, store_params=False, train_cfg=big_tr)
    cfg4, cols4 = k148_cfg()
    run_case("k148", cfg4, B=4, L=160, vocab=2000, Fn=10, Fm=10, cat_cards={c: 100 for c in cols4[:6]},
             steps=2, pseed=31, bseed=600, store_params=False, train_cfg=big_tr)
    cfg5, cols5 = k120_cfg()
    run_case("k120", cfg5, B=6, L=150, vocab=2000, Fn=10, Fm=10, cat_cards={c: 100 for c in cols5[:6]},
             steps=2, pseed=51, bseed=800, store_params=False, train_cfg=big_tr)
    gen_infer()
    gen_bf16()
    gen_r3()
    gen_r4()


def gen_r5():
    """Round 5: QNN pair_grouping 'block' (src/models/qnn_alpha.py:99-108, block slices src/models/wrapper.py:66-75):
    [u | 6 numeric | 1 mask | 5 categorical] features -- u and the single mask feature fall in one-feature blocks,
    which the block form leaves out of every interaction; and LayerNorm norms (tiny_ln)."""
    tr = dict(lr=3e-3, wd=1e-4, clip=0.5, steps_per_epoch=4, warmup_epochs=1, epochs=3)
    cards = {"c0": 300, "c1": 500, "c2": 1000, "c3": 200, "c4": 700}
    run_case("tiny_block", tiny_cfg(pair_grouping="block"), B=48, L=24, vocab=4000, Fn=6, Fm=1, cat_cards=cards,
             steps=3, pseed=15, bseed=500, store_params=True, train_cfg=tr)
    # LayerNorm (src/models/dare.py:15-18: any norm name but "rms" is nn.LayerNorm) in the encoder layers and the
    # QNN pre-norm
    run_case("tiny_ln", tiny_cfg(norm="layer", qnn_norm="layer"), B=40, L=24, vocab=4000, Fn=6, Fm=3,
             cat_cards=cards, steps=3, pseed=16, bseed=520, store_params=True, train_cfg=tr)


def gen_r3(only_cfg4=False):
    """Round-3 cases: BASELINE config 4 at its true lengths (L = 400, K = 148, D = 64, 4 layers, every
    categorical and numeric column of the yaml) in fp32 and amp bf16; config 3 (K = 100, S1) in amp bf16;
    and a two-layer encoder whose FFN width (40) is not a multiple of 16, so the FFN runs as separate
    GEMMs + RMSNorm backwards instead of the fused kernel."""
    big_tr = dict(lr=3e-3, wd=1e-4, clip=0.5, steps_per_epoch=10, warmup_epochs=0, epochs=8)
    cfg4, cols4, nnum = cfg4_full_cfg()
    # the yaml's own lr (3e-4): at 3e-3 the first update moves this deep (4-layer, D = 64) model so far that the
    # second step's gradients carry the first step's ill-conditioned AdamW elements (see golden_util.
    # Fixture.ill_conditioned) into every moment
    tr4 = dict(big_tr, lr=3e-4)
    kw4 = dict(B=3, L=400, vocab=2000, Fn=nnum, Fm=nnum, cat_cards={c: 100 for c in cols4}, steps=2, pseed=61,
               bseed=900, store_params=False, train_cfg=tr4)
    # B = 3 single-sample categorical rows: many table-grad elements sit near AdamW's eps after the clip,
    # where the update is ill-conditioned -- more replays for a representative allowance
    run_case("cfg4_full", cfg4, **kw4, allow_replays=8)
    run_case("cfg4_full_bf16", cfg4, **kw4, amp_twin="cfg4_full")
    if only_cfg4:
        return
    cfg3, cols3 = cfg3_cfg()
    run_case("cfg3_dims_bf16", cfg3, B=8, L=100, vocab=3000, Fn=82, Fm=82, cat_cards={c: 200 for c in cols3},
             steps=2, pseed=41, bseed=700, store_params=False, train_cfg=big_tr, amp_twin="cfg3_dims")
    tr = dict(lr=3e-3, wd=1e-4, clip=0.5, steps_per_epoch=4, warmup_epochs=1, epochs=3)
    cards = {"c0": 300, "c1": 500, "c2": 1000, "c3": 200, "c4": 700}
    run_case("tiny_ffn40", tiny_cfg(D=32, H=4, ffn_hidden=40), B=40, L=28, vocab=3000, Fn=5, Fm=5,
             cat_cards=cards, steps=2, pseed=15, bseed=1000, store_params=True, train_cfg=tr)


def gen_r4():
    """Round-4 case: BASELINE config 2's widths in the regime the reference trains in -- its OWN
    initialisation (oracle.synth.reference_init, checked bitwise in run_case) and the yaml's lr 3e-4
    (cfgs/dare_qnn_next.yaml:254), no warm-up -- so the logits stay near 0 (loss ~0.7) and the clip at 0.5
    is mild, unlike cfg2_dims (synthetic init, lr 3e-3: saturated logits, every step clipped ~1000x).
    fp32 and its amp bf16 twin, three steps."""
    tr = dict(lr=3e-4, wd=1e-4, clip=0.5, steps_per_epoch=10, warmup_epochs=0, epochs=8)
    cfg2, cols = cfg2_cfg()
    kw = dict(B=16, L=100, vocab=3000, Fn=82, Fm=82, cat_cards={c: 200 for c in cols}, steps=3, pseed=71,
              bseed=1100, store_params=False, train_cfg=tr, init="reference")
    run_case("cfg2_ref", cfg2, **kw)
    run_case("cfg2_ref_bf16", cfg2, **kw, amp_twin="cfg2_ref")


def gen_bf16():
    """amp: bf16 twins of three fp32 fixtures (same inputs, seeds, parameters): the noise band the
    parity tests compare the bf16 build against is the reference's own bf16-vs-fp32 deviation."""
    tr = dict(lr=3e-3, wd=1e-4, clip=0.5, steps_per_epoch=4, warmup_epochs=1, epochs=3)
    cards = {"c0": 300, "c1": 500, "c2": 1000, "c3": 200, "c4": 700}
    run_case("tiny_concat_bf16", tiny_cfg(), B=64, L=32, vocab=5000, Fn=6, Fm=6, cat_cards=cards, steps=3,
             pseed=11, bseed=100, store_params=True, train_cfg=tr, amp_twin="tiny_concat")
    big_tr = dict(lr=3e-3, wd=1e-4, clip=0.5, steps_per_epoch=10, warmup_epochs=0, epochs=8)
    cfg2, cols = cfg2_cfg()
    run_case("cfg2_dims_bf16", cfg2, B=8, L=100, vocab=3000, Fn=82, Fm=82, cat_cards={c: 200 for c in cols},
             steps=2, pseed=21, bseed=500, store_params=False, train_cfg=big_tr, amp_twin="cfg2_dims")
    cfg4, cols4 = k148_cfg()
    run_case("k148_bf16", cfg4, B=4, L=160, vocab=2000, Fn=10, Fm=10, cat_cards={c: 100 for c in cols4[:6]},
             steps=2, pseed=31, bseed=600, store_params=False, train_cfg=big_tr, amp_twin="k148")


if __name__ == "__main__":
    main()
