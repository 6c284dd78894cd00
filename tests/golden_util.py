"""Fixture loading / comparison helpers shared by the CPU and GPU parity tests."""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from oracle import synth
from oracle.model import make_arch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["tiny_concat", "tiny_s1_relu", "tiny_s2", "base_fc", "cfg2_dims", "cfg3_dims", "k148", "k120", "cfg4_full",
         "tiny_ffn40", "cfg2_ref", "tiny_block", "tiny_ln"]
# amp: bf16 twins (gen_golden.gen_bf16): the reference under torch.autocast(bfloat16) on the inputs,
# seeds and parameters of the fp32 fixture named in meta["twin"]
BF16_CASES = ["tiny_concat_bf16", "cfg2_dims_bf16", "cfg3_dims_bf16", "k148_bf16", "cfg4_full_bf16", "cfg2_ref_bf16"]
# AdamW updates elementwise (Fixture.check_update): |d| <= 2 ulp + the replayed-conditioning allowance +
# ELEM_RTOL_UPDATE (10 |ref| + max |ref|); ill-conditioned elements (sqrt(v_hat) < 100 eps) only norm-wise
ELEM_RTOL_UPDATE = 1e-3
BF16_BAND = 3.0      # bf16 tolerance: within 3x the reference's own bf16-vs-fp32 deviation ...
BF16_FLOOR = 1e-4    # ... or 1e-4 of the tensor's norm, whichever is larger
# scalars (loss, grad norm): one draw of the bf16 rounding says little about its spread, so the floor is
# 4 bf16 unit roundoffs (4 x 2^-9) of the value
BF16_SCALAR_FLOOR = 4 * 2.0 ** -9
# tensors of fewer than BF16_FEW elements (the output layers' biases, ...): their gradients are batch sums
# of per-sample terms of both signs (sum of dlogits over 8 samples), where bf16 rounding of the terms is
# amplified by the cancellation -- measured: 4.8% between the bf16 build and the reference's bf16 run on
# the final bias's Adam moment, 3.9% against its fp32 run; the floor there is 10% of the value
BF16_FEW = 64
BF16_FEW_FLOOR = 0.1


def key_bias_mask(arch, key):
    """Elements whose exact gradient is identically zero, so the reference's value is rounding noise:
    the key slice [D, 2D) of every MHA ``in_proj_bias`` (adding a constant to a query's keys shifts all
    its scores equally; softmax is shift-invariant).  AdamW turns that noise into +-lr steps of
    arbitrary sign, so update / moment comparisons leave these elements out (and a separate check
    bounds the gradient itself).  None for every other key."""
    if not key.endswith("mha.in_proj_bias"):
        return None
    m = np.zeros(3 * arch.D, bool)
    m[arch.D:2 * arch.D] = True
    return m


class Fixture:
    def __init__(self, name):
        self.name = name
        self.z = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
        self.meta = json.loads(str(self.z["meta"]))
        m = self.meta
        self.cat_cards = {k: int(v) for k, v in m["cat_cards"].items()}
        self.cat_cols = list(self.cat_cards)
        self.arch = make_arch(m["cfg"], m["vocab"], m["Fn"], m["Fm"], self.cat_cards, self.cat_cols)

    def params0(self):
        if self.meta.get("init") == "reference":     # the reference's own init, restated (gen_golden.run_case)
            return synth.reference_init(self.arch, self.meta["pseed"])
        if self.meta["store_params"]:
            return {k: self.z[f"p0/{k}"] for k, _ in self.arch.param_shapes()}
        return synth.make_params(self.arch.param_shapes(), self.meta["pseed"], pad_id=self.arch.pad_id)

    def batch(self, t):
        return {k: self.z[f"in{t}/{k}"] for k in ("X_num", "X_mask", "X_cat", "seq", "y", "groups")}

    def has(self, name):
        return name in self.z.files or f"{name}@idx" in self.z.files

    def check(self, name, got, rtol=1e-4, atol=1e-6, what=None, exclude=None, base=None, elem_rtol=None, allow=None,
              ulps=2.0,
              skip=None):
        """Compare ``got`` with the stored full tensor or its fingerprint.

        Full tensors: norm-wise relative error <= rtol and elementwise (close_enough).  Fingerprinted
        (large) tensors: the sampled elements as above; the rows the fixture's batches touch (embedding
        tables) in full as above; the squared norm within 2 rtol; and the norm of the difference
        estimated from NPROJ Gaussian projections (oracle/synth.py: each projected difference is
        N(0, ||got - ref||^2)) <= 3 rtol ||ref|| -- a flat 3x margin on a chi-square(8) estimate, false
        alarm ~1e-9 at an error of exactly rtol.  ``exclude``: boolean mask (flat) of elements left out
        (full tensors only).

        ``base`` (flat, like got): for an update d = pT - p0 pass p0.  The reference's pT is an fp32
        number, so its own rounding puts an uncertainty of half an ulp of |pT| on d -- at |p| ~ 1 and
        lr = 3e-4 that is 2e-4 of |d|, above any rtol one could ask of d itself; every comparison of such
        a difference therefore allows 2 ulp(|p0 + ref|) per element on top of the rtol terms (and their
        L2 norm in the norm-wise test).  ``elem_rtol``: the elementwise factor when it differs from rtol
        (AdamW updates: an element whose gradient nearly cancels between steps has an ill-conditioned
        m/sqrt(v); two CPU implementations of the reference differ by up to 1e-3 of such an element)."""
        if isinstance(got, torch.Tensor):
            got = got.detach().cpu().numpy()
        got = np.asarray(got, dtype=np.float64).ravel()
        if base is not None:
            base = np.asarray(base.detach().cpu().numpy() if isinstance(base, torch.Tensor) else base,
                              np.float64).ravel()
        label = what or f"{self.name}:{name}"

        def ulp(ref, b, extra=None):
            u = None if b is None else ulps * np.spacing(np.abs(b + ref).astype(np.float32)).astype(np.float64)
            if extra is not None:
                u = extra.astype(np.float64) if u is None else u + extra
            return u

        al = self.allowance(allow) if allow else None
        sk = skip(self) if skip else None      # {"full" | "idx", "rows"}: elements left out of the elementwise test

        if name in self.z.files:
            ref = np.asarray(self.z[name], dtype=np.float64).ravel()
            assert got.shape == ref.shape, (label, got.shape, ref.shape)
            b = base
            a = None if al is None else al["full"]
            if exclude is not None:
                got, ref = got[~exclude], ref[~exclude]
                b = None if b is None else b[~exclude]
                a = None if a is None else a[~exclude]
            close_enough(got, ref, rtol, atol, label, ulp(ref, b, a), elem_rtol,
                         None if sk is None or exclude is not None else sk["full"])
            return
        assert exclude is None, label
        fp = {k: self.z[f"{name}@{k}"] for k in ("idx", "vals", "sumsq", "projs")}
        vals = fp["vals"].astype(np.float64)
        close_enough(got[fp["idx"]], vals, rtol, atol, label + "[sampled]",
                     ulp(vals, None if base is None else base[fp["idx"]], None if al is None else al["idx"]),
                     elem_rtol, None if sk is None else sk["idx"])
        if f"{name}@rows" in self.z.files:
            rows = self.z[f"{name}@rows"]
            ref_rows = self.z[f"{name}@rowvals"].astype(np.float64)
            w = ref_rows.shape[1]
            br = None if base is None else base.reshape(-1, w)[rows].ravel()
            close_enough(got.reshape(-1, w)[rows].ravel(), ref_rows.ravel(), rtol, atol, label + "[touched rows]",
                         ulp(ref_rows.ravel(), br, None if al is None else al["rows"].ravel()), elem_rtol,
                         None if sk is None or sk["rows"] is None else sk["rows"].ravel())
        sumsq = float(fp["sumsq"])
        slack = (0.0 if base is None else float(np.linalg.norm(ulp(0.0 * base, base)))) + \
            (0.0 if al is None else float(al["norm"]))
        assert abs((got * got).sum() - sumsq) <= 2 * rtol * sumsq + atol * atol * got.size + \
            2 * slack * np.sqrt(sumsq) + slack * slack, (label, "sumsq")
        e = synth.project(got) - fp["projs"].astype(np.float64)
        est = float(np.sqrt(np.mean(e * e)))
        assert est <= 3 * (rtol * np.sqrt(sumsq) + slack) + atol * np.sqrt(got.size), (
            f"{label}: projected difference norm {est:.3e} vs ||ref|| {np.sqrt(sumsq):.3e} (rtol {rtol})")


    def allowance(self, name):
        """The generator's per-element allowance ``name`` (gen_golden.update_allowance): {"full"} for a
        small tensor, else {"idx", "rows", "norm"}."""
        if name in self.z.files:
            a = self.z[name].astype(np.float64)
            return {"full": a, "norm": float(np.linalg.norm(a))}
        return {"idx": self.z[f"{name}@idx"].astype(np.float64),
                "rows": self.z[f"{name}@rows"].astype(np.float64) if f"{name}@rows" in self.z.files else None,
                "norm": float(self.z[f"{name}@norm"])}

    def check_update(self, kind, key, got_delta, p0, rtol=1e-4, exclude=None):
        """An AdamW update (kind "dT": pT - p0) or the EMA shadow's (kind "demaT") against the reference's:
        norm-wise rtol plus, per element, 2 ulp of the fp32 result (4 for the EMA shadow: each step's
        d e + (1 - d) p rounds once more and carries the parameter's rounding) and the replayed conditioning
        allowance (gen_golden.update_allowance); elementwise at ELEM_RTOL_UPDATE (1 % of the element plus 0.1 %
        of the tensor's largest update)."""
        return self.check(f"{kind}/{key}", got_delta, rtol, 1e-12, exclude=exclude, base=p0, elem_rtol=ELEM_RTOL_UPDATE,
                          ulps=4.0 if kind == "demaT" else 2.0,
                          allow=f"{kind}allow/{key}", skip=lambda fx: fx.ill_conditioned(key))

    def ill_conditioned(self, key, factor=100.0):
        """Elements whose final AdamW denominator sqrt(v_T / bc2) + eps is dominated by eps: sqrt(v_T / bc2) <
        factor * eps (the criterion of tests/test_gpu_shard.py's data-parallel check).  There m / denom is
        a cancellation residue of near-zero gradients -- two fp32 implementations with different summation
        orders step such an element by different fractions of lr (cfg4_full: a DARE att row whose gradient is
        a softmax-cancellation residue of ~1e-9, GPU 4x smaller than the reference, update 1/3 of the
        reference's).  They stay in the norm-wise test; the elementwise test leaves them out.  None when the
        fixture holds no v_T for ``key`` (no gradient)."""
        name = f"vT/{key}"
        if not self.has(name):
            return None
        bc2 = 1.0 - 0.999 ** int(self.meta["steps"])
        lim = (factor * 1e-8) ** 2 * bc2
        if name in self.z.files:
            return {"full": np.asarray(self.z[name], np.float64).ravel() < lim}
        out = {"idx": self.z[f"{name}@vals"].astype(np.float64) < lim, "rows": None}
        if f"{name}@rowvals" in self.z.files:
            out["rows"] = self.z[f"{name}@rowvals"].astype(np.float64) < lim
        return out


    def check_moment(self, kind, key, got, rtol=None):
        """An Adam moment after the fixture's steps (kind "mT" / "vT"), norm-wise and elementwise at 2e-4
        for m and 4e-4 for v (quadratic in the gradient: twice its relative error):
        the gradient of step t > 0 is taken at parameters that already carry the earlier steps' (1e-5 ..
        1e-4) deviations, and m sums the steps' gradients with cancellation where they oppose -- measured
        GPU vs reference after two steps: up to 1.5e-4 (a one-element bias), 1.3e-4 (sampled v of the SE
        fc.2 weight)."""
        if rtol is None:
            rtol = 2e-4 if kind == "mT" else 4e-4
        return self.check(f"{kind}/{key}", got, rtol, 0.0)


def _exact_subset(fx, name):
    """(index array or None = all, exact reference values there) of a stored tensor: the whole tensor
    when stored in full, else the fingerprint's sampled elements plus the touched rows' elements."""
    if name in fx.z.files:
        return None, np.asarray(fx.z[name], np.float64).ravel()
    idx = fx.z[f"{name}@idx"].astype(np.int64)
    vals = fx.z[f"{name}@vals"].astype(np.float64)
    if f"{name}@rows" in fx.z.files:
        rows = fx.z[f"{name}@rows"].astype(np.int64)
        rv = fx.z[f"{name}@rowvals"].astype(np.float64)
        w = rv.shape[1]
        ridx = (rows[:, None] * w + np.arange(w)[None, :]).ravel()
        keep = ~np.isin(idx, ridx)
        idx = np.concatenate([idx[keep], ridx])
        vals = np.concatenate([vals[keep], rv.ravel()])
    return idx, vals


def check_bf16_band(fx16, fx32, name, got, label=None, update=False, p0=None, flips=0):
    """amp: bf16 parity.  ``got`` (the build under amp: bf16) is compared with the reference run under
    autocast(bfloat16) (``fx16``) and in fp32 (``fx32``, the twin fixture): the norm of the difference
    to EACH must stay within BF16_BAND x the reference's own bf16-vs-fp32 deviation, or BF16_FLOOR of
    the tensor's norm.  Norms over the whole tensor when it is stored in full, else over the exact
    sampled elements + touched rows (the same subset for all three), and the projected whole-tensor
    estimate within twice that bound.

    ``flips`` (multi-step runs only: moments and updates after >= 2 AdamW steps): up to that many LONE
    outlier elements -- one element carrying more than half of the squared deviation -- are left out of
    all three norms.  AdamW's first step moves every element by ~lr sign(g): an element whose step-0
    gradient is within bf16 rounding of 0 steps either way, which changes its (and its neighbours') later
    gradients by far more than rounding.  Measured (tools/amp_band_report.py, profiles/r03/amp_band_*.log):
    cfg4_full_bf16's vT/qnn.mlp.0.weight is 3.5x its band with ONE of its 2048 sampled elements carrying
    94 % of the squared deviation (the reference's own bf16-vs-fp32 band: one element 48 %, ten 97 %);
    every other tensor of the five cases is within 1.5x.  Tensors under BF16_FEW elements never drop one."""
    label = label or f"{fx16.name}:{name}"
    if isinstance(got, torch.Tensor):
        got = got.detach().cpu().double().numpy()
    got = np.asarray(got, np.float64).ravel()
    idx, r16 = _exact_subset(fx16, name)
    idx32, r32 = _exact_subset(fx32, name)
    if idx is not None:
        assert idx32 is not None, label
        pos = {int(i): j for j, i in enumerate(idx32)}
        sel = np.array([pos.get(int(i), -1) for i in idx])
        have = sel >= 0
        idx, r16, r32 = idx[have], r16[have], r32[sel[have]]
    g = got if idx is None else got[idx]
    assert g.shape == r16.shape == r32.shape, (label, g.shape, r16.shape, r32.shape)
    p0s = None
    if update and p0 is not None:
        p0 = np.asarray(p0.detach().cpu().double().numpy() if isinstance(p0, torch.Tensor) else p0, np.float64).ravel()
        p0s = p0 if idx is None else p0[idx]
    if flips and g.size >= BF16_FEW:
        keep = np.ones(g.size, bool)
        for _ in range(flips):
            d = np.maximum((g - r16) ** 2, (g - r32) ** 2) * keep
            j = int(np.argmax(d))
            if d[j] <= 0.5 * d.sum():
                break
            keep[j] = False
        if not keep.all():
            g, r16, r32 = g[keep], r16[keep], r32[keep]
            p0s = None if p0s is None else p0s[keep]
    band = float(np.linalg.norm(r32 - r16))
    nrm = max(float(np.linalg.norm(r16)), float(np.linalg.norm(r32)))
    floor = (BF16_FLOOR if got.size >= BF16_FEW else BF16_FEW_FLOOR) * nrm
    if update and got.size < BF16_FEW:
        # an AdamW step takes ~lr * sign(g) where the gradient is tiny: an element whose gradient is within
        # bf16 noise of 0 steps either way, and one such flip moves a small tensor's update (or its EMA
        # shadow's) by up to twice its largest element
        floor = max(floor, 2.0 * max(float(np.abs(r16).max(initial=0)), float(np.abs(r32).max(initial=0))))
    if p0s is not None:
        # an update pT - p0 (or the EMA shadow's) carries the fp32 rounding of the result itself: 2 ulps per
        # element, as the fp32 checks allow (Fixture.check_update).  Where the reference's bf16 and fp32 runs
        # round alike (band 0: a parameter without gradient, whose EMA shadow d s + (1 - d) p drifts by
        # rounding alone) this is the whole tolerance
        floor += float(np.linalg.norm(2.0 * np.spacing(np.abs(p0s + r32).astype(np.float32)).astype(np.float64)))
    tol = BF16_BAND * band + floor + 1e-30
    e16, e32 = float(np.linalg.norm(g - r16)), float(np.linalg.norm(g - r32))
    assert e16 <= tol and e32 <= tol, (
        f"{label}: |got - ref_bf16| {e16:.3e}, |got - ref_fp32| {e32:.3e} vs band |ref_fp32 - ref_bf16| "
        f"{band:.3e} (tol {tol:.3e}, |ref| {nrm:.3e})")
    if idx is not None:          # whole tensor through the projections (chi-square estimates: 2x slack)
        p16 = fx16.z[f"{name}@projs"].astype(np.float64)
        p32 = fx32.z[f"{name}@projs"].astype(np.float64)
        pg = synth.project(got)
        est = lambda d: float(np.sqrt(np.mean(d * d)))    # noqa: E731
        nb = np.sqrt(max(float(fx16.z[f"{name}@sumsq"]), float(fx32.z[f"{name}@sumsq"])))
        ptol = 2 * (BF16_BAND * est(p32 - p16) + BF16_FLOOR * nb) + 1e-30
        assert est(pg - p16) <= ptol and est(pg - p32) <= ptol, (
            f"{label}: projected |got - ref_bf16| {est(pg - p16):.3e}, |got - ref_fp32| {est(pg - p32):.3e} vs "
            f"band {est(p32 - p16):.3e} (tol {ptol:.3e})")
    return e16, e32, band


def close_enough(got, ref, rtol, atol, label, ulp=None, elem_rtol=None, skip=None):
    """Norm-wise ||got - ref|| <= rtol ||ref|| (+ ||ulp||) AND elementwise
    |d| <= atol (+ ulp) + e*(10|ref| + max|ref|) with e = elem_rtol (default rtol); ``skip`` (boolean, like
    ref): elements left out of the elementwise test only."""
    d = np.abs(got - ref)
    nrm = np.linalg.norm(ref)
    u = 0.0 if ulp is None else ulp
    un = 0.0 if ulp is None else float(np.linalg.norm(ulp))
    err = np.linalg.norm(got - ref)
    rel = err / (nrm + 1e-30)
    e = rtol if elem_rtol is None else elem_rtol
    bad = d > atol + u + 10 * e * np.abs(ref) + e * np.abs(ref).max(initial=0)
    if skip is not None:
        bad &= ~np.asarray(skip, bool)
    ok_norm = err <= rtol * nrm + un or (nrm == 0 and d.max(initial=0) <= atol)
    assert ok_norm and not bad.any(), (
        f"{label}: normwise rel err {rel:.3e} (rtol {rtol}{'' if ulp is None else f', +ulp {un / (nrm + 1e-30):.1e}'}), "
        f"{bad.sum()} elems beyond elementwise tol; max abs diff {d.max(initial=0):.3e}")


def check_topk(fx, t, idx_got, vals_got, label=""):
    """DARE top-K indices (src/models/dare.py:131-137) against the reference's (``out{t}/topk_idx``).

    Exact, slot by slot, wherever the reference's choice is determined by the scores:
      * every slot selects the same TOKEN (so the gathered rep rows are identical);
      * every real-token slot selects the same POSITION, unless its score is bitwise tied with another
        selected slot (then only the token must agree: a tie between distinct positions of one token --
        the same embedding row -- is harmless, and a tie between distinct tokens has not occurred);
      * pad slots (score exactly -1e9) are the last ones, each a distinct pad position.  Which of the
        tied pad positions torch.topk returns, and in what order, is libstdc++'s nth_element/sort
        detail; every pad row is the zero padding_idx row with the same score, so the model's outputs
        and gradients do not depend on it.  The HIP kernel takes pads in ascending position.
    Scores within 1e-5 (relative, or absolute near 0)."""
    ref = fx.z[f"out{t}/topk_idx"].astype(np.int64)
    rv = fx.z[f"out{t}/topk_vals"].astype(np.float64)
    seq = fx.z[f"in{t}/seq"].astype(np.int64)
    got = np.asarray(idx_got, np.int64)
    assert got.shape == ref.shape, (label, got.shape, ref.shape)
    pad = fx.arch.pad_id
    tok_ref = np.take_along_axis(seq, ref, 1)
    tok_got = np.take_along_axis(seq, got, 1)
    assert np.array_equal(tok_got, tok_ref), (label, "token per slot", np.argwhere(tok_got != tok_ref)[:5])
    real = tok_ref != pad
    dup = np.zeros_like(real)
    for b in range(rv.shape[0]):
        _, inv, cnt = np.unique(rv[b], return_inverse=True, return_counts=True)
        dup[b] = cnt[inv] > 1
    sel = real & ~dup
    assert np.array_equal(got[sel], ref[sel]), (label, "positions", np.argwhere((got != ref) & sel)[:5])
    for b in range(got.shape[0]):
        p = got[b, ~real[b]]
        assert np.all(seq[b, p] == pad) and len(np.unique(p)) == p.size, (label, "pad slots", b)
        if real[b].any() and (~real[b]).any():
            assert real[b].argmin() == real[b].sum(), (label, "pads must follow the real tokens", b)
    gv = np.asarray(vals_got, np.float64)
    assert np.all(np.abs(gv - rv) <= 1e-5 * np.maximum(1.0, np.abs(rv))), (label, "scores")


def to_torch_batch(b):
    return {"X_num": torch.from_numpy(b["X_num"]).float(), "X_mask": torch.from_numpy(b["X_mask"]).float(),
            "X_cat": torch.from_numpy(b["X_cat"]).long(), "seq": torch.from_numpy(b["seq"]).long()}


# The full-shape step cases (tests/test_gpu_fullshape.py; their reference bf16 bands: tests/golden/gen_amp_band_full.py):
# the BASELINE configs as bench.py runs them, at the production batch (cfg4 at 1024, the size SURVEY §6 ran the
# reference at on CPU -- 4096 does not fit a 62 GB host there), from the reference's own initialisation
FULL_SHAPE = {"cfg2": dict(B=4096), "cfg3": dict(B=4096), "cfg4": dict(B=1024)}
FULL_SHAPE_PSEED = 2024            # torch.manual_seed before CTRModel(...): oracle.synth.reference_init
FULL_SHAPE_BSEED = 31337
FULL_SHAPE_DSEED = (777 << 32) | 1  # dropout seed of the step (the cfg seed 777, step 1)


def full_shape_case(name):
    """(cfg, cards, cols, arch, B, L, vocab, Fn, batch) of a FULL_SHAPE case: tossctr.configs.BENCH_CONFIGS[name] (the
    reference yaml restated with BASELINE.json's overrides), vocab 10M (src/train.py:116), the yaml's max_len, the
    SURVEY §8(d) batch distributions (oracle.synth.make_batch, positive rate 0.019)."""
    from tossctr.configs import BENCH_CONFIGS, N_NUM_NEXT, cat_cardinals
    B = FULL_SHAPE[name]["B"]
    cfg = BENCH_CONFIGS[name](batch_size=B)
    cards = cat_cardinals(cfg)
    cols = list(cards)
    vocab, L, Fn = 10_000_000, int(cfg["sequence"]["max_len"]), N_NUM_NEXT
    A = make_arch(cfg, vocab, Fn, Fn, cards, cols)
    b = synth.make_batch(B, Fn, Fn, list(cards.values()), L, vocab, seed=FULL_SHAPE_BSEED, pos_rate=0.019)
    return cfg, cards, cols, A, B, L, vocab, Fn, b


def full_shape_touched(b, cols):
    """Table key -> the rows the batch reads (unique token ids for both DARE tables, per column for the cats)."""
    out = {"dare.emb_att.weight": np.unique(b["seq"]), "dare.emb_rep.weight": np.unique(b["seq"])}
    for i, c in enumerate(cols):
        out[f"cat_embs.{c}.weight"] = np.unique(b["X_cat"][:, i])
    return out
