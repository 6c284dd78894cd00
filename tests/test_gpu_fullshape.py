"""Training steps at the bench's FULL shape against the CPU oracle.

BASELINE config 2 exactly as bench.py runs it (tossctr.configs.dare_qnn_next: D = 32, L = 100, K = 60, 3
encoder layers, 82 + 82 + 35 features, MLP 7552-512-256; B = 4096; DARE tables 10,000,000 x 32, hashed tables
1,000,000 x d_c) from the reference's own initialisation (oracle.synth.reference_init, pinned bitwise against
the reference by tests/golden/gen_golden.py), the yaml's lr 3e-4, clip 0.5, EMA 0.999.  Batch-size- and
grid-size-dependent code runs at its production size: the persistent FFN row walk over 245,760 rows, the rocPRIM
sorts of 409,600 top-K keys and 143,360 categorical keys, the lazy touch / update class lists.  The fp32 oracle
(oracle.model.TrainState, ~30 s and ~35 GB of host memory on the GPU box's 16 threads) runs ONCE per module on the
shared batch; both tests compare with it.

test_cfg2_full_shape_step_matches_oracle -- the HIP step in fp32 (amp none: the fp32 VALU attention kernels of
attn.hip, the fp32 FFN kernels; north star: 1e-4 rtol on fp32 logits / grads):
  * loss (1e-5 relative), logits (norm-wise 1e-4), the clip's global grad norm (1e-4 relative);
  * top-K: the token in every slot exactly, the position wherever the score is not tied;
  * both Adam moments after the step -- m = 0.1 * clip_coef * g and v = 0.001 * (clip_coef * g)^2 pin the
    gradient of every dense parameter and of every touched table row (norm-wise 2e-4 / 4e-4, the moment
    tolerances of golden_util.Fixture.check_moment);
  * the parameter update p1 - p0 and the EMA shadow's on the dense parameters and the touched rows (norm-wise
    1e-4 + 2 fp32 ulps on the well-conditioned elements; elementwise: one lr for any element (a noise-level
    gradient may step either way) and 1e-2 of lr + 2 ulps where the gradient is well above its noise);
  * untouched table rows (a sample of 4096 per table): the decay-only step p0 (1 - lr wd) and its EMA,
    within 1 fp32 ulp.

test_cfg2_full_shape_bf16_step -- the step the bench times (amp bf16: the fused layer forward
ctr_attn_layer_fwd_bf with the XCD-aware bf16-MFMA attention grid over 4096 samples, ctr_attn_bwd_bf_oproj, the
persistent bf16 FFN kernels, the bf16-operand QNN MLP GEMMs -- asserted to be the entry points that ran) against
the same fp32 oracle, within AMP_BAND_K (1) x the REFERENCE's own bf16-vs-fp32 deviation of each quantity
(tests/golden/amp_band_cfg2.json, written by tests/golden/gen_amp_band.py from the reference-run cfg2_ref /
cfg2_ref_bf16 fixtures: src/train.py:158-168 under autocast vs fp32).  The build keeps more in fp32 than autocast
(master weights, softmax, norms, every element-wise op), so its deviation from fp32 should not exceed the
reference's own: loss, grad norm, logits, and both Adam moments of every parameter (m pins the clipped gradient of the
dense parameters and of every touched table row); the AdamW step and the EMA against the build's own moments; the
untouched rows' decay-only step as in the fp32 test."""
import json
import os
import zlib

import numpy as np
import pytest
import torch

from golden_util import close_enough, key_bias_mask, to_torch_batch

pytestmark = pytest.mark.gpu

LR, WD, CLIP = 3e-4, 1e-4, 0.5
HERE = os.path.dirname(os.path.abspath(__file__))
# bf16 tolerance: the build's deviation from the fp32 oracle within this many times the reference's own bf16-vs-
# fp32 deviation of the same quantity -- 1: no further from fp32 than the reference's own autocast run is (measured
# at the end of round 5: at most 0.56 of it on every quantity, profiles/r05/gputest_fullshape_bf16.log; the small-
# shape bf16 fixture checks use golden_util.BF16_BAND = 3 against both reference runs)
AMP_BAND_K = 1.0


def _touched(b, cols):
    out = {"dare.emb_att.weight": np.unique(b["seq"]), "dare.emb_rep.weight": np.unique(b["seq"])}
    for i, c in enumerate(cols):
        out[f"cat_embs.{c}.weight"] = np.unique(b["X_cat"][:, i])
    return out


@pytest.fixture(scope="module")
def shape():
    from oracle.model import make_arch
    from oracle.synth import make_batch, reference_init
    from tossctr.configs import N_NUM_NEXT, cat_cardinals, dare_qnn_next
    cfg = dare_qnn_next()
    cards = cat_cardinals(cfg)
    cols = list(cards)
    vocab, B, L, Fn = 10_000_000, 4096, 100, N_NUM_NEXT
    A = make_arch(cfg, vocab, Fn, Fn, cards, cols)
    P0 = {k: torch.from_numpy(v) for k, v in reference_init(A, 2024).items()}
    b = make_batch(B, Fn, Fn, list(cards.values()), L, vocab, seed=31337, pos_rate=0.019)
    touched = _touched(b, cols)
    free = {}
    for k, shp in A.param_shapes():
        if k in touched:
            r = np.random.default_rng(zlib.crc32(k.encode()))
            free[k] = np.setdiff1d(r.choice(shp[0], 4096, replace=False), touched[k])
    return dict(cfg=cfg, cards=cards, cols=cols, vocab=vocab, B=B, Fn=Fn, A=A, P0=P0, b=b, touched=touched, free=free,
                seed=(777 << 32) | 1)


@pytest.fixture(scope="module")
def oracle_step(shape):
    """The reference semantics (fp32 CPU oracle) on the shared batch: loss, logits, gnorm, top-K, and per parameter
    p / m / v / EMA after the step (touched rows + the sampled untouched rows of every table, dense in full)."""
    from oracle.model import TrainState
    torch.set_num_threads(16)
    A, P0, b, cfg = shape["A"], shape["P0"], shape["b"], shape["cfg"]
    st = TrainState(P0, A, LR, WD, CLIP, ema_cfg=cfg["ema"])
    rec = {}
    loss, (logits, _, _), grads = st.grads(to_torch_batch(b), torch.from_numpy(b["y"]).float(), shape["seed"],
                                           record=rec)
    for p in st.P.values():      # host memory: the dense table grads exist once (TrainState.step clones them)
        p.grad = None
    gnorm = st.apply(grads, LR)
    del grads
    out = {"loss": float(loss), "logits": logits.detach().double().numpy(), "gnorm": float(gnorm),
           "idx": rec["topk_idx"].numpy().astype(np.int64), "vals": rec["topk_vals"].detach().double().numpy(),
           "params": {}}
    for k, _ in A.param_shapes():
        ent = {}
        if k in shape["touched"]:
            rows = torch.from_numpy(shape["touched"][k])
            fr = torch.from_numpy(shape["free"][k])
            sel = lambda t: t[rows].double().clone()                                           # noqa: E731
            ent["p_free"] = st.P[k].detach()[fr].clone()
            ent["e_free"] = st.shadow[k][fr].clone()
        else:
            sel = lambda t: t.double().clone()                                                 # noqa: E731
        ent["p"] = sel(st.P[k].detach())
        ent["e"] = sel(st.shadow[k])
        ent["m"] = sel(st.m[k]) if k in st.m else None
        ent["v"] = sel(st.v[k]) if k in st.v else None
        out["params"][k] = ent
    del st
    return out


def _hip_step(shape, amp, record=()):
    """One fused HIP training step (compact table grads, exact lazy AdamW / EMA) on the shared batch; the
    entry points named in ``record`` are counted (tossctr._lib.time_calls)."""
    from tossctr import CTRModel, FusedAdamW, _lib, build_ema
    cfg = dict(shape["cfg"], amp=amp)
    model = CTRModel(cfg, shape["vocab"], shape["Fn"], shape["Fn"], shape["cards"], shape["cols"], device="cuda:0")
    model.load_state_dict(shape["P0"])
    ema = build_ema(model, cfg)
    opt = FusedAdamW(model, lr=LR, weight_decay=WD, max_grad_norm=CLIP, ema=ema, lazy=True)
    model.train()
    b = shape["b"]
    _lib.time_calls(record)
    loss = float(model.train_step(model.stage(to_torch_batch(b)), torch.from_numpy(b["y"]).float().cuda(), opt,
                                  global_step=1, seed=shape["seed"]).item())
    calls = {n: c for n, (c, _) in _lib.timed_ms().items()}
    _lib.time_calls(())
    eng = model.engine
    flags = {"attn_bf": eng.attn_bf, "attn_layer": eng.attn_layer, "attn_oproj": eng.attn_oproj,
             "ffn_flags": eng.ffn_flags, "bf16": eng.bf16}
    sv = eng.last
    res = {"loss": loss, "logits": sv["logits"].double().cpu().numpy(), "idx": sv["idx"].cpu().numpy().astype(np.int64),
           "gnorm": float(opt.norm_out[0].item()), "calls": calls, "flags": flags, "params": {}}
    model.sync()
    ar = model.arena
    for k in ar.order:
        views = {n: ar._view(buf, k) for n, buf in (("p", ar.buf), ("m", opt.m), ("v", opt.v), ("e", ema.shadow))}
        if ar.kind[k] == "table":
            rows = torch.from_numpy(shape["touched"][k]).cuda()
            ent = {n: v[rows].double().cpu() for n, v in views.items()}
            fr = torch.from_numpy(shape["free"][k]).cuda()
            ent["p_free"] = views["p"][fr].cpu()
            ent["e_free"] = views["e"][fr].cpu()
        else:
            ent = {n: v.double().cpu() for n, v in views.items()}
        res["params"][k] = ent
    del model, opt, ema
    torch.cuda.empty_cache()
    return res


def _tied(vals):
    tied = np.zeros(vals.shape, bool)
    for i in range(vals.shape[0]):
        _, inv, cnt = np.unique(vals[i], return_inverse=True, return_counts=True)
        tied[i] = cnt[inv] > 1
    return tied


def _check_untouched(shape, k, g, r):
    """Untouched rows take the decay-only step (a zero gradient) and the EMA of it."""
    assert torch.allclose(g["p_free"], r["p_free"], rtol=1.2e-7, atol=0), k
    assert torch.allclose(g["e_free"], r["e_free"], rtol=2.4e-7, atol=0), k


@pytest.mark.timeout(900)
def test_cfg2_full_shape_step_matches_oracle(shape, oracle_step):
    got = _hip_step(shape, "none")
    ref, A, b = oracle_step, shape["A"], shape["b"]
    assert not got["flags"]["bf16"]
    assert abs(got["loss"] - ref["loss"]) <= 1e-5 * max(1.0, abs(ref["loss"])), (got["loss"], ref["loss"])
    close_enough(got["logits"], ref["logits"], 1e-4, 1e-5, "logits")
    assert abs(got["gnorm"] - ref["gnorm"]) <= 1e-4 * ref["gnorm"], (got["gnorm"], ref["gnorm"])

    seq = b["seq"].astype(np.int64)
    tok_g, tok_r = np.take_along_axis(seq, got["idx"], 1), np.take_along_axis(seq, ref["idx"], 1)
    assert np.array_equal(tok_g, tok_r), np.argwhere(tok_g != tok_r)[:5]
    sel = (tok_r != A.pad_id) & ~_tied(ref["vals"])
    assert np.array_equal(got["idx"][sel], ref["idx"][sel])

    for k, _ in A.param_shapes():
        g, r = got["params"][k], ref["params"][k]
        p0 = shape["P0"][k]
        if k in shape["touched"]:
            p0 = p0[torch.from_numpy(shape["touched"][k])]
            _check_untouched(shape, k, g, r)
        if r["m"] is not None:
            close_enough(g["m"].numpy().ravel(), r["m"].numpy().ravel(), 2e-4, 0.0, f"m:{k}")
            close_enough(g["v"].numpy().ravel(), r["v"].numpy().ravel(), 4e-4, 0.0, f"v:{k}")
        base = p0.double().numpy().ravel()
        dg = g["p"].numpy().ravel() - base
        dr = r["p"].numpy().ravel() - base
        ulp = 2.0 * np.spacing(np.abs(base + dr).astype(np.float32)).astype(np.float64)
        assert np.abs(dg - dr).max(initial=0) <= LR, k
        if r["v"] is not None:
            # well above the gradient's noise: an AdamW step from zero moments is lr * g / (|g| + eps') there, the
            # same to ~1e-2 of lr whatever the gradient's rounding -- a sign flip or a halved step fails
            # (the MHA key bias's exact gradient is 0: noise, golden_util.key_bias_mask)
            m = np.abs(r["m"].numpy().ravel())
            strong = m >= 1e-3 * np.sqrt(np.mean(m * m) + 1e-300)
            kb = key_bias_mask(A, k)
            if kb is not None:
                strong &= ~kb
            assert (np.abs(dg - dr)[strong] <= 1e-2 * LR + ulp[strong]).all(), k
            good = np.sqrt(r["v"].numpy().ravel() / (1 - 0.999)) >= 100 * 1e-8
            close_enough(dg[good], dr[good], 1e-4, 0.0, f"dp:{k}", ulp[good], elem_rtol=1e-2)
        eg = g["e"].numpy().ravel() - base
        er = r["e"].numpy().ravel() - base
        assert np.abs(eg - er).max(initial=0) <= 0.01 * LR + 1e-6, k


# the entry points of the step bench.py times under amp: bf16 (tossctr/engine.py), one or more calls each
BF16_ENTRY_POINTS = ("ctr_attn_layer_fwd_bf", "ctr_attn_bwd_bf_oproj", "ctr_ffn_fwd", "ctr_ffn_bwd_norms",
                     "ctr_gemm_bf16_ex")


@pytest.mark.timeout(900)
def test_cfg2_full_shape_bf16_step(shape, oracle_step):
    with open(os.path.join(HERE, "golden", "amp_band_cfg2.json")) as fh:
        band = json.load(fh)
    got = _hip_step(shape, "bf16", record=BF16_ENTRY_POINTS)
    ref, A, b = oracle_step, shape["A"], shape["b"]
    nl = A.n_layers
    fl = got["flags"]
    assert fl["bf16"] and fl["attn_bf"] and fl["attn_layer"] and fl["attn_oproj"] and fl["ffn_flags"] == 1, fl
    c = got["calls"]
    assert c.get("ctr_attn_layer_fwd_bf") == nl and c.get("ctr_attn_bwd_bf_oproj") == nl, c
    gemm_bf = sum(v for n, v in c.items() if n.startswith("ctr_gemm_bf16_ex"))     # keyed per shape (_lib)
    assert c.get("ctr_ffn_fwd") == nl and c.get("ctr_ffn_bwd_norms") == nl and gemm_bf >= 3, c
    K = AMP_BAND_K
    report, fails = [], []

    def within(label, err, nrm, delta, floor=0.0):
        tol = K * delta * nrm + floor
        report.append((label, err / max(nrm, 1e-300), delta, err / max(delta * nrm, 1e-300)))
        if err > tol:
            fails.append(f"{label}: |got - fp32| / |fp32| = {err / max(nrm, 1e-300):.3e} > {K} x reference bf16 "
                         f"deviation {delta:.3e}")

    within("loss", abs(got["loss"] - ref["loss"]), abs(ref["loss"]), band["scalars"]["loss"])
    within("gnorm", abs(got["gnorm"] - ref["gnorm"]), ref["gnorm"], band["scalars"]["gnorm"])
    within("logits", float(np.linalg.norm(got["logits"] - ref["logits"])), float(np.linalg.norm(ref["logits"])),
           band["outputs"]["logits"])
    # top-K: the scores come from the query path (its GEMMs on bf16 operands), so a slot may differ where two
    # candidates' scores are within bf16 rounding of each other; every other slot selects the same token
    seq = b["seq"].astype(np.int64)
    tok_g, tok_r = np.take_along_axis(seq, got["idx"], 1), np.take_along_axis(seq, ref["idx"], 1)
    same = float(np.mean(np.sort(tok_g, 1) == np.sort(tok_r, 1)))
    if same < 0.999:
        fails.append(f"top-K tokens agree on {same:.5f} of the slots")
    nflip = nstrong = 0
    for k, _ in A.param_shapes():
        g, r = got["params"][k], ref["params"][k]
        p0 = shape["P0"][k]
        if k in shape["touched"]:
            p0 = p0[torch.from_numpy(shape["touched"][k])]
            _check_untouched(shape, k, g, r)
        if r["m"] is None:
            continue
        # m = 0.1 coef g: the gradient's deviation plus the clip coefficient's (the gnorm's)
        dk = band["grads"][k] + band["scalars"]["gnorm"]
        mr, vr = r["m"].numpy().ravel(), r["v"].numpy().ravel()
        within(f"m:{k}", float(np.linalg.norm(g["m"].numpy().ravel() - mr)), float(np.linalg.norm(mr)), dk,
               1e-4 * float(np.linalg.norm(mr)))
        within(f"v:{k}", float(np.linalg.norm(g["v"].numpy().ravel() - vr)), float(np.linalg.norm(vr)), 2 * dk,
               1e-4 * float(np.linalg.norm(vr)))
        # the update and the EMA: the first AdamW step is a function of the step's own moments, p1 = p0 (1 - lr wd)
        # - lr (m / bc1) / (sqrt(v / bc2) + eps), so it is checked against the build's own m, v (the moments carry
        # the gradient, checked against the band above): 1e-5 of lr (the kernel's hardware sqrt / reciprocal) + 2
        # fp32 ulps.  Where the bf16 gradient of an element crosses 0 (a sum over 4096 samples with cancellation)
        # the step flips sign, as the reference's own bf16 steps do: against the oracle every element is within
        # 2 lr, and the flipped fraction of the well-conditioned (sqrt(v_hat) >= 100 eps) elements is reported
        base = p0.double().numpy().ravel()
        mg, vg = g["m"].numpy().ravel(), g["v"].numpy().ravel()
        pg, pr_ = g["p"].numpy().ravel(), r["p"].numpy().ravel()
        p1 = base * (1 - LR * WD) - LR * (mg / 0.1) / (np.sqrt(vg / 1e-3) + 1e-8)
        ulp = 2.0 * np.spacing(np.abs(p1).astype(np.float32)).astype(np.float64)
        if not (np.abs(pg - p1) <= 1e-5 * LR + ulp).all():
            fails.append(f"AdamW step of the build's own moments: {k} (max {np.abs(pg - p1).max() / LR:.2e} lr)")
        if not (np.abs(pg - pr_) <= 2 * LR + ulp).all():
            fails.append(f"update beyond 2 lr of the oracle's: {k}")
        good = np.sqrt(vr / 1e-3) >= 100 * 1e-8
        kb = key_bias_mask(A, k)
        if kb is not None:
            good &= ~kb
        nflip += int((np.sign(mg[good]) != np.sign(mr[good])).sum())
        nstrong += int(good.sum())
        # e1 = fma(e0, d, fl(omd p1)) in fp32 (csrc/adam.h ema_elem), d = fp32(0.999), omd = fp32(1 - d), e0 = p0
        d32 = np.float32(0.999)
        omd = np.float64(np.float32(1.0 - np.float64(d32)))
        x = (omd * pg).astype(np.float32).astype(np.float64)
        e1 = (base * np.float64(d32) + x).astype(np.float32).astype(np.float64)
        if not (np.abs(g["e"].numpy().ravel() - e1) <= np.spacing(np.abs(e1).astype(np.float32))).all():
            fails.append(f"EMA of the build's own step: {k}")
    worst = sorted(report[3:], key=lambda x: -x[3])[:10]
    print(f"\nbf16 full-shape step vs fp32 oracle (rel. deviation, reference band, ratio); top-K slots equal {same:.5f}; "
          f"AdamW steps of well-conditioned elements whose sign differs from the oracle's: {nflip} of {nstrong}:")
    for row in report[:3] + worst:
        print(f"  {row[0]:45s} {row[1]:.3e}  {row[2]:.3e}  {row[3]:.2f}")
    assert not fails, fails
