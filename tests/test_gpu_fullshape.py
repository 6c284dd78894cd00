"""Training steps at the BASELINE configs' FULL shape against the CPU oracle.

The configs exactly as bench.py runs them (tossctr.configs.BENCH_CONFIGS; golden_util.FULL_SHAPE), at the production
batch, from the reference's own initialisation (oracle.synth.reference_init, pinned bitwise against the reference by
tests/golden/gen_golden.py), the yaml's lr 3e-4, clip 0.5 and EMA:
  * cfg2 -- dare_qnn_next + hash_buckets 1e6, D = 32, L = 100, K = 60, 3 layers, concat query, EMA 0.999; B = 4096;
  * cfg3 -- dare_qnn_next_k100_s1 (K = 100 >= L: every real token selected, S1 query; the K > 64 attention kernels of
    attn_mf.hip / attn.hip); B = 4096;
  * cfg4 -- v3_k148_s1 as-is (D = 64, L = 400, K = 148, 4 layers, hashed tables of 1-6k rows, EMA off; the D = 64 bf16
    row kernels of rowgemm_bf.hip); B = 1024 (the reference's CPU step at 4096 does not fit 62 GB).
DARE tables 10,000,000 x D, 82 + 82 + 35 features, the QNN head.  Batch-size- and grid-size-dependent code runs at its
production size: the persistent FFN row walk, the rocPRIM sorts of the top-K and categorical keys, the lazy touch /
update class lists.  The fp32 oracle (oracle.model.TrainState, ~30 s and ~35 GB of host memory on the GPU box's 16
threads) runs ONCE per config on the shared batch; both tests of the config compare with it.

test_full_shape_step_matches_oracle -- the HIP step in fp32 (amp none: the fp32 attention kernels of attn.hip, the
fp32 FFN kernels; north star: 1e-4 rtol on fp32 logits / grads):
  * loss (1e-5 relative), logits (norm-wise 1e-4), the clip's global grad norm (1e-4 relative);
  * top-K: the token in every slot exactly, the position wherever the score is not tied;
  * both Adam moments after the step -- m = 0.1 * clip_coef * g and v = 0.001 * (clip_coef * g)^2 pin the
    gradient of every dense parameter and of every touched table row (norm-wise 2e-4 / 4e-4, the moment
    tolerances of golden_util.Fixture.check_moment).  Where the fp32 step and the fp32 oracle differ by more, the
    gradient is ill-conditioned in fp32 itself (sums over 4096 x K rows with cancellation: at cfg3 the numeric
    embeddings, every categorical table, several encoder weights, ~2-7e-4 from the truth in BOTH implementations): an
    fp64 oracle (oracle64) then arbitrates, _arbitrated_checks;
  * the parameter update p1 - p0 and the EMA shadow's on the dense parameters and the touched rows (norm-wise
    1e-4 + 2 fp32 ulps on the well-conditioned elements; elementwise: one lr for any element (a noise-level
    gradient may step either way) and 1e-2 of lr + 2 ulps where the gradient is well above its noise);
  * untouched table rows (a sample of up to 4096 per table): the decay-only step p0 (1 - lr wd) and its EMA,
    within 1 fp32 ulp.

test_full_shape_bf16_step -- the step the bench times (amp bf16; the entry points of that config's bf16 path --
asserted to be the ones that ran) against the same fp32 oracle, within AMP_BAND_K (1) x the REFERENCE's own
bf16-vs-fp32 deviation of each quantity AT THIS SAME STEP: tests/golden/amp_band_full_<cfg>.json, written by
tests/golden/gen_amp_band_full.py running the reference on this batch, init and dropout masks in fp32 and under
autocast(bfloat16) (src/train.py:158-168).  The build keeps more in fp32 than autocast (master weights, softmax, norms,
every element-wise op), so its deviation from fp32 should not exceed the reference's own: loss, grad norm, logits, and
both Adam moments of every parameter (m pins the clipped gradient of the dense parameters and of every touched table
row); the AdamW step and the EMA against the build's own moments; the untouched rows' decay-only step as in the fp32
test."""
import json
import os
import zlib

import numpy as np
import pytest
import torch

from golden_util import (FULL_SHAPE, FULL_SHAPE_DSEED, FULL_SHAPE_PSEED, close_enough, full_shape_case,
                         full_shape_touched, key_bias_mask, to_torch_batch)

pytestmark = pytest.mark.gpu

LR, WD, CLIP = 3e-4, 1e-4, 0.5
HERE = os.path.dirname(os.path.abspath(__file__))
# bf16 tolerance: the build's deviation from the fp32 oracle within this many times the reference's own bf16-vs-
# fp32 deviation of the same quantity at the same step -- 1: no further from fp32 than the reference's own autocast
# run is (the small-shape bf16 fixture checks use golden_util.BF16_BAND = 3 against both reference runs)
AMP_BAND_K = 1.0
N_FREE = 4096      # untouched rows sampled per table
SCALAR_FLOOR = 2.0 ** -9


@pytest.fixture(scope="module", params=list(FULL_SHAPE))
def shape(request):
    from oracle.synth import reference_init
    name = request.param
    cfg, cards, cols, A, B, L, vocab, Fn, b = full_shape_case(name)
    P0 = {k: torch.from_numpy(v) for k, v in reference_init(A, FULL_SHAPE_PSEED).items()}
    touched = full_shape_touched(b, cols)
    free = {}
    for k, shp in A.param_shapes():
        if k in touched:
            r = np.random.default_rng(zlib.crc32(k.encode()))
            free[k] = np.setdiff1d(r.choice(shp[0], min(N_FREE, shp[0]), replace=False), touched[k])
    ema_on = bool(cfg.get("ema", {}).get("enabled", False))
    yield dict(name=name, cfg=cfg, cards=cards, cols=cols, vocab=vocab, B=B, L=L, Fn=Fn, A=A, P0=P0, b=b,
               touched=touched, free=free, seed=FULL_SHAPE_DSEED, ema=ema_on)


@pytest.fixture(scope="module")
def oracle_step(shape):
    """The reference semantics (fp32 CPU oracle) on the shared batch: loss, logits, gnorm, top-K, and per parameter
    p / m / v / EMA after the step (touched rows + the sampled untouched rows of every table, dense in full)."""
    from oracle.model import TrainState
    torch.set_num_threads(16)
    A, P0, b, cfg = shape["A"], shape["P0"], shape["b"], shape["cfg"]
    st = TrainState(P0, A, LR, WD, CLIP, ema_cfg=cfg["ema"] if shape["ema"] else None)
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
            if st.shadow is not None:
                ent["e_free"] = st.shadow[k][fr].clone()
        else:
            sel = lambda t: t.double().clone()                                                 # noqa: E731
        ent["p"] = sel(st.P[k].detach())
        ent["e"] = sel(st.shadow[k]) if st.shadow is not None else None
        ent["m"] = sel(st.m[k]) if k in st.m else None
        ent["v"] = sel(st.v[k]) if k in st.v else None
        out["params"][k] = ent
    del st
    yield out


@pytest.fixture(scope="module")
def oracle64(shape):
    """On first use: the oracle's step-0 gradients in fp64 (oracle.model.forward at float64, the same batch, init
    and dropout masks) for every parameter (tables at the touched rows), as the moments they give: m64 = 0.1 c g, v64 = 0.001 (c g)^2 with
    the fp64 clip coefficient c.  The arbiter where the fp32 HIP step and the fp32 oracle differ by more than the
    moment tolerance: a gradient that is a sum over 4096 x K rows with heavy cancellation is no better than a few
    1e-4 in fp32, in either implementation (~20 GB of host memory, ~1 min)."""
    cache = {}

    def get():
        if not cache:
            from oracle.model import Dropper, bce_wll_style, forward
            A, b = shape["A"], shape["b"]
            P = {k: v.double().requires_grad_(True) for k, v in shape["P0"].items()}
            drop = Dropper(shape["seed"], training=True)
            logits, _, aux = forward(P, to_torch_batch(b), A, drop, dtype=torch.float64)
            y = torch.from_numpy(b["y"]).double()
            loss = bce_wll_style(logits, y)
            if A.aux_w > 0:
                loss = loss + A.aux_w * bce_wll_style(aux, y)
            loss.backward()
            keys = A.grad_params()
            sq = sum(float(P[k].grad.pow(2).sum()) for k in keys)
            coef = min(1.0, CLIP / (sq ** 0.5 + 1e-6))
            for k in keys:
                g = P[k].grad.detach()
                if k in shape["touched"]:         # tables: the rows the batch reads (every other row's grad is 0)
                    g = g[torch.from_numpy(shape["touched"][k])]
                g = g * coef
                cache[k] = (0.1 * g, 0.001 * g * g)
            del P, logits, aux, loss
        return cache

    yield get
    cache.clear()


def _direct_checks(A, k, g, r, dg, dr, ulp):
    """The HIP step against the fp32 oracle: both Adam moments (norm-wise 2e-4 / 4e-4, golden_util's moment
    tolerances), the update within one lr anywhere, within 1e-2 lr (+ 2 ulps) where the gradient is well above its
    noise, and norm-wise 1e-4 on the well-conditioned elements."""
    close_enough(g["m"].numpy().ravel(), r["m"].numpy().ravel(), 2e-4, 0.0, f"m:{k}")
    close_enough(g["v"].numpy().ravel(), r["v"].numpy().ravel(), 4e-4, 0.0, f"v:{k}")
    assert np.abs(dg - dr).max(initial=0) <= LR, f"update beyond one lr: {k}"
    # well above the gradient's noise: an AdamW step from zero moments is lr * g / (|g| + eps') there, the same to
    # ~1e-2 of lr whatever the gradient's rounding -- a sign flip or a halved step fails (the MHA key bias's exact
    # gradient is 0: noise, golden_util.key_bias_mask)
    m = np.abs(r["m"].numpy().ravel())
    strong = m >= 1e-3 * np.sqrt(np.mean(m * m) + 1e-300)
    kb = key_bias_mask(A, k)
    if kb is not None:
        strong &= ~kb
    assert (np.abs(dg - dr)[strong] <= 1e-2 * LR + ulp[strong]).all(), f"update of strong elements: {k}"
    good = np.sqrt(r["v"].numpy().ravel() / (1 - 0.999)) >= 100 * 1e-8
    close_enough(dg[good], dr[good], 1e-4, 0.0, f"dp:{k}", ulp[good], elem_rtol=1e-2)


_ARB = []       # (tensor, HIP error, fp32 oracle error) vs fp64 of every arbitrated moment, for the aggregate check


def _arbitrated_checks(k, g, r, dg, dr, ulp, base, oracle64):
    """A tensor whose gradient is ill-conditioned in fp32 itself (both fp32 results a few 1e-4 from the truth, in
    different directions): the fp64 oracle's moments m64, v64 and its first AdamW step d64 decide.
      * moments: within 1.5x the fp32 oracle's distance from fp64 over every arbitrated tensor together (the test's
        aggregate check), and per tensor within max(1e-3, 4x the oracle's) -- two error norms of one draw each differ
        by up to ~3x (measured at cfg3: the positional-bias grad, a diagonal sum of dS whose rows sum to 0 exactly,
        HIP 5.0e-4 / oracle 1.5e-4; the numeric embeddings HIP 3.8e-4 / oracle 4.1e-4);
      * the update within two lr anywhere (a noise-level gradient's step may take either sign in either);
      * on the elements fp32 resolves (|m64| >= 10x the oracle's rms error on the tensor) and that are well above
        eps, norm-wise no further from the fp64 step d64 than max(1e-4, 3x the oracle); the count of steps off d64
        by over 1e-2 lr (+ the step's sensitivity to that noise where |g| is near eps, d/dg lr g / (|g| + eps) =
        lr eps / (|g| + eps)^2) is reported for both -- per element the fp32 noise is heavy-tailed (a row whose few
        samples cancel).
    Returns a note for the report."""
    m64, v64 = (t.numpy().ravel() for t in oracle64()[k])
    notes = []
    for name, gm, rm, t, rtol in (("m", g["m"], r["m"], m64, 2e-4), ("v", g["v"], r["v"], v64, 4e-4)):
        n64 = np.linalg.norm(t)
        e_hip = np.linalg.norm(gm.numpy().ravel() - t) / n64
        e_or = np.linalg.norm(rm.numpy().ravel() - t) / n64
        assert e_hip <= max(1e-3, 4.0 * e_or), (f"{name}:{k}", e_hip, e_or)
        _ARB.append((f"{name}:{k}", e_hip, e_or))
        notes.append(f"{name} HIP {e_hip:.2e} / oracle {e_or:.2e}")
    assert np.abs(dg - dr).max(initial=0) <= 2 * LR, k
    d64 = base * (1 - LR * WD) - LR * (m64 / 0.1) / (np.sqrt(v64 / 1e-3) + 1e-8) - base
    noise = np.sqrt(np.mean((r["m"].numpy().ravel() - m64) ** 2))
    res = np.abs(m64) >= 10.0 * noise
    sens = LR * 1e-8 / (np.abs(m64) / 0.1 + 1e-8) ** 2 * (3.0 * noise / 0.1)
    tol = 1e-2 * LR + sens + ulp
    n_hip = int((res & (np.abs(dg - d64) > tol)).sum())
    n_or = int((res & (np.abs(dr - d64) > tol)).sum())
    good = (np.sqrt(v64 / (1 - 0.999)) >= 100 * 1e-8) & res
    e_hip = np.linalg.norm(dg[good] - d64[good])
    e_or = np.linalg.norm(dr[good] - d64[good])
    assert e_hip <= max(1e-4 * np.linalg.norm(d64[good]), 3.0 * e_or), (k, e_hip, e_or)
    notes.append(f"steps off fp64 by > 1e-2 lr: HIP {n_hip}, oracle {n_or} of {int(res.sum())}")
    return "; ".join(notes)


def _hip_step(shape, amp, record=()):
    """One fused HIP training step (compact table grads, exact lazy AdamW / EMA) on the shared batch; the
    entry points named in ``record`` are counted (tossctr._lib.time_calls)."""
    from tossctr import CTRModel, FusedAdamW, _lib, build_ema
    cfg = dict(shape["cfg"], amp=amp)
    model = CTRModel(cfg, shape["vocab"], shape["Fn"], shape["Fn"], shape["cards"], shape["cols"], device="cuda:0")
    model.load_state_dict(shape["P0"])
    ema = build_ema(model, cfg)
    assert (ema is not None) == shape["ema"]
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
             "ffn_flags": eng.ffn_flags, "bf16": eng.bf16, "rowgemm_bf": eng.rowgemm_bf, "qkv16": eng.qkv16,
             "attn_layer_bwd": eng.attn_layer_bwd}
    sv = eng.last
    res = {"loss": loss, "logits": sv["logits"].double().cpu().numpy(), "idx": sv["idx"].cpu().numpy().astype(np.int64),
           "gnorm": float(opt.norm_out[0].item()), "calls": calls, "flags": flags, "params": {}}
    model.sync()
    ar = model.arena
    bufs = [("p", ar.buf), ("m", opt.m), ("v", opt.v)] + ([("e", ema.shadow)] if ema is not None else [])
    for k in ar.order:
        views = {n: ar._view(buf, k) for n, buf in bufs}
        if ar.kind[k] == "table":
            rows = torch.from_numpy(shape["touched"][k]).cuda()
            ent = {n: v[rows].double().cpu() for n, v in views.items()}
            fr = torch.from_numpy(shape["free"][k]).cuda()
            ent["p_free"] = views["p"][fr].cpu()
            if ema is not None:
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


def _near_tied(vals, rtol=2e-6):
    """Slots whose (descending) oracle score is within rtol of a neighbour's: an fp32 dot product summed in another
    order may swap the two (SURVEY §7 hard part 2)."""
    v = np.asarray(vals, np.float64)
    gap = np.abs(np.diff(v, axis=1)) <= rtol * np.maximum(1.0, np.abs(v[:, 1:]))
    out = np.zeros(v.shape, bool)
    out[:, 1:] |= gap
    out[:, :-1] |= gap
    return out


def _check_untouched(shape, k, g, r):
    """Untouched rows take the decay-only step (a zero gradient) and the EMA of it."""
    assert torch.allclose(g["p_free"], r["p_free"], rtol=1.2e-7, atol=0), k
    if "e_free" in r:
        assert torch.allclose(g["e_free"], r["e_free"], rtol=2.4e-7, atol=0), k


def _check_topk_fp32(got, ref, A, b):
    """The token in every slot exactly, except where the oracle's score is near-tied with a neighbour's (then the pair
    may swap: the multiset of the row's tokens must still agree); the position wherever the score is not tied."""
    seq = b["seq"].astype(np.int64)
    tok_g, tok_r = np.take_along_axis(seq, got["idx"], 1), np.take_along_axis(seq, ref["idx"], 1)
    near = _near_tied(ref["vals"])
    bad = (tok_g != tok_r) & ~near
    assert not bad.any(), np.argwhere(bad)[:5]
    rows = np.flatnonzero(((tok_g != tok_r) & near).any(1))
    for i in rows:
        assert np.array_equal(np.sort(tok_g[i]), np.sort(tok_r[i])), i
    sel = (tok_r != A.pad_id) & ~_tied(ref["vals"]) & ~near
    assert np.array_equal(got["idx"][sel], ref["idx"][sel])
    return int(((tok_g != tok_r) & near).sum())


@pytest.mark.timeout(900)
def test_full_shape_step_matches_oracle(shape, oracle_step, oracle64):
    ref, A, b = oracle_step, shape["A"], shape["b"]
    # the oracle itself at this shape: the reference's own fp32 step on the same batch, init and masks
    # (tests/golden/gen_amp_band_full.py records its loss and grad norm)
    with open(os.path.join(HERE, "golden", f"amp_band_full_{shape['name']}.json")) as fh:
        r32 = json.load(fh)["fp32"]
    assert abs(ref["loss"] - r32["loss"]) <= 1e-6 * abs(r32["loss"]), (ref["loss"], r32["loss"])
    assert abs(ref["gnorm"] - r32["gnorm"]) <= 1e-6 * r32["gnorm"], (ref["gnorm"], r32["gnorm"])
    got = _hip_step(shape, "none")
    assert not got["flags"]["bf16"]
    assert abs(got["loss"] - ref["loss"]) <= 1e-5 * max(1.0, abs(ref["loss"])), (got["loss"], ref["loss"])
    close_enough(got["logits"], ref["logits"], 1e-4, 1e-5, "logits")
    assert abs(got["gnorm"] - ref["gnorm"]) <= 1e-4 * ref["gnorm"], (got["gnorm"], ref["gnorm"])
    _ARB.clear()
    swaps = _check_topk_fp32(got, ref, A, b)
    print(f"\n{shape['name']} B = {shape['B']}: loss {got['loss']:.7f} (oracle {ref['loss']:.7f}), gnorm {got['gnorm']:.6f} "
          f"(oracle {ref['gnorm']:.6f}), near-tie top-K swaps {swaps}")

    for k, _ in A.param_shapes():
        g, r = got["params"][k], ref["params"][k]
        p0 = shape["P0"][k]
        if k in shape["touched"]:
            p0 = p0[torch.from_numpy(shape["touched"][k])]
            _check_untouched(shape, k, g, r)
        base = p0.double().numpy().ravel()
        dg = g["p"].numpy().ravel() - base
        dr = r["p"].numpy().ravel() - base
        ulp = 2.0 * np.spacing(np.abs(base + dr).astype(np.float32)).astype(np.float64)
        if r["m"] is not None:
            try:
                _direct_checks(A, k, g, r, dg, dr, ulp)
            except AssertionError as e:
                # the two fp32 results differ beyond the tolerances: the fp64 oracle arbitrates
                note = _arbitrated_checks(k, g, r, dg, dr, ulp, base, oracle64)
                print(f"  {k}: {str(e).splitlines()[0][:90]} -> fp64: {note}")
        else:
            assert np.abs(dg - dr).max(initial=0) <= LR, k
        if r["e"] is not None:
            eg = g["e"].numpy().ravel() - base
            er = r["e"].numpy().ravel() - base
            assert np.abs(eg - er).max(initial=0) <= 0.01 * LR + 1e-6, k
    if _ARB:
        eh = np.sqrt(np.mean([x[1] ** 2 for x in _ARB]))
        eo = np.sqrt(np.mean([x[2] ** 2 for x in _ARB]))
        print(f"  {len(_ARB)} moments arbitrated by fp64: rms error HIP {eh:.2e}, fp32 oracle {eo:.2e}")
        assert eh <= 1.5 * eo, (eh, eo)


# the entry points of the step bench.py times under amp: bf16 (tossctr/engine.py), per config: the fused layer
# forward / oproj-folded attention backward at K <= 64, D = 32 (cfg2); the separate bf16 attention kernels at K > 64
# (cfg3, cfg4: attn_bwd_mfl_kernel) and the D = 64 bf16 row kernels (cfg4)
# (cfg2 with the bf16 qkv / dqkv: the *16 forms and the in-projection backward on the bf16 grad)
BF16_ENTRY_POINTS = ("ctr_attn_layer_fwd_bf", "ctr_attn_bwd_bf_oproj", "ctr_attn_fwd_bf", "ctr_attn_bwd_bf",
                     "ctr_attn_layer_fwd_bf16", "ctr_attn_bwd_bf_oproj16", "ctr_rowgemm_a16", "ctr_rowgemm_wgrad_y16",
                     "ctr_ffn_fwd", "ctr_ffn_bwd_norms", "ctr_gemm_bf16_ex", "ctr_rowgemm_bf", "ctr_rowgemm",
                     "ctr_qnn_gram_fwd_zbf", "ctr_qnn_gram_bwd_zbf", "ctr_attn_bwd_bf_layer16")


@pytest.mark.timeout(900)
def test_full_shape_bf16_step(shape, oracle_step):
    with open(os.path.join(HERE, "golden", f"amp_band_full_{shape['name']}.json")) as fh:
        band = json.load(fh)
    assert band["B"] == shape["B"] and band["L"] == shape["L"]
    got = _hip_step(shape, "bf16", record=BF16_ENTRY_POINTS)
    ref, A, b = oracle_step, shape["A"], shape["b"]
    nl = A.n_layers
    fl = got["flags"]
    c = got["calls"]
    assert fl["bf16"] and fl["attn_bf"] and fl["ffn_flags"] == 1, fl
    if A.top_k <= 64:
        assert fl["attn_layer"] and fl["attn_oproj"], fl
        assert c.get("ctr_attn_layer_fwd_bf16") == nl and c.get("ctr_attn_bwd_bf_oproj16") == nl, c
        assert fl["qkv16"] and c.get("ctr_rowgemm_a16") == nl and c.get("ctr_rowgemm_wgrad_y16") == nl, (fl, c)
        # the one-launch attention half of the layer backward is opt-in (CTR_ATTN_LAYER_BWD=1: slower, engine.py)
        assert not fl["attn_layer_bwd"] and not c.get("ctr_attn_bwd_bf_layer16"), (fl, c)
    else:
        assert not fl["attn_layer"] and not fl["attn_oproj"], fl
        assert c.get("ctr_attn_fwd_bf") == nl and c.get("ctr_attn_bwd_bf") == nl, c
    if A.D == 64:
        assert fl["rowgemm_bf"] and c.get("ctr_rowgemm_bf", 0) >= 2 * nl and not c.get("ctr_rowgemm"), (fl, c)
    # the pair interaction on bf16(z), read from the MLP's [z | inter] image at D = 32 (cfg2, cfg3); D = 64 (cfg4)
    # keeps the fp32-z Gram products (with bf16 z its step measured 1.15 x the reference's own band on the last MLP
    # layer's grad, profiles/r06/gputest_gram_zbf.log)
    want = 1 if A.D == 32 else 0
    assert c.get("ctr_qnn_gram_fwd_zbf", 0) == want and c.get("ctr_qnn_gram_bwd_zbf", 0) == want, c
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

    # scalars: ONE draw of the reference's bf16 rounding (cfg4's grad norm moved 2.4e-4 in it, cfg2's 1.8e-2) says
    # little about the spread, so they also pass within one bf16 unit roundoff (2^-9) of the value
    within("loss", abs(got["loss"] - ref["loss"]), abs(ref["loss"]), band["scalars"]["loss"],
           SCALAR_FLOOR * abs(ref["loss"]))
    # the grad norm cannot move by more than the whole gradient does (|‖g + e‖ - ‖g‖| <= ‖e‖): besides its own band it
    # is allowed the reference's per-tensor gradient bands aggregated over the step, sqrt(sum_k (band_k ‖m_k‖)^2) /
    # ‖m‖ (m = 0.1 c g: the oracle's clipped gradient, tables at the touched rows -- zero elsewhere)
    num = den = 0.0
    for k, _ in A.param_shapes():
        mk = ref["params"][k]["m"]
        if mk is not None and k in band["grads"]:
            n2 = float((mk.double() ** 2).sum())
            num += (band["grads"][k] ** 2) * n2
            den += n2
    agg = (num / den) ** 0.5 if den > 0 else 0.0
    within("gnorm", abs(got["gnorm"] - ref["gnorm"]), ref["gnorm"], max(band["scalars"]["gnorm"], agg),
           SCALAR_FLOOR * ref["gnorm"])
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
        if "e" not in g:
            continue
        # e1 = fma(e0, d, fl(omd p1)) in fp32 (csrc/adam.h ema_elem), d = fp32(0.999), omd = fp32(1 - d), e0 = p0
        d32 = np.float32(0.999)
        omd = np.float64(np.float32(1.0 - np.float64(d32)))
        x = (omd * pg).astype(np.float32).astype(np.float64)
        e1 = (base * np.float64(d32) + x).astype(np.float32).astype(np.float64)
        if not (np.abs(g["e"].numpy().ravel() - e1) <= np.spacing(np.abs(e1).astype(np.float32))).all():
            fails.append(f"EMA of the build's own step: {k}")
    worst = sorted(report[3:], key=lambda x: -x[3])[:10]
    print(f"\n{shape['name']} B = {shape['B']}: bf16 full-shape step vs fp32 oracle (rel. deviation, reference band, ratio); top-K slots equal {same:.5f}; "
          f"AdamW steps of well-conditioned elements whose sign differs from the oracle's: {nflip} of {nstrong}:")
    for row in report[:3] + worst:
        print(f"  {row[0]:45s} {row[1]:.3e}  {row[2]:.3e}  {row[3]:.2f}")
    assert not fails, fails
