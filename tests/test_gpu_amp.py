"""amp: bf16 on the GPU (src/train.py:133-139,158-164).

The build under ``amp: bf16`` runs every product on the GEMM kernel with bf16-rounded operands on bf16
MFMA, fp32 accumulation; parameters, optimizer state, tables and the element-wise math stay fp32.  The
reference under autocast rounds more (every autocast op's output too), so the two cannot agree to fp32
precision.  Tolerance (golden_util.check_bf16_band): the norm of the difference to the reference's bf16
run AND to its fp32 run within 3x the reference's own bf16-vs-fp32 deviation, or 1e-4 of the tensor's
norm -- outputs, every step-0 gradient, the updates, both moments and the EMA shadow.  Scalars (loss,
grad norm): 3x band or 4 bf16 unit roundoffs (4 x 2^-9) of the value; tensors under 64 elements
(output-layer biases: cancelling batch sums) 3x band or 10% of their norm (golden_util.BF16_FEW_FLOOR);
their updates also one sign flip (twice the largest element: an AdamW step is ~lr sign(g))."""
import numpy as np
import pytest
import torch

from golden_util import BF16_BAND, BF16_CASES, BF16_SCALAR_FLOOR, Fixture, check_bf16_band, to_torch_batch

pytestmark = pytest.mark.gpu


def build(fx):
    from tossctr import CTRModel
    m = fx.meta
    model = CTRModel(m["cfg"], m["vocab"], m["Fn"], m["Fm"], fx.cat_cards, fx.cat_cols, device="cuda:0")
    model.load_state_dict({k: torch.from_numpy(v) for k, v in fx.params0().items()})
    assert model.engine.bf16, "cfg amp: bf16 must select the bf16 GEMM path"
    return model


def bce(z, y):
    pos = y > 0.5
    pl = torch.nn.functional.softplus(-z[pos]).mean() if pos.any() else z.sum() * 0
    nl = torch.nn.functional.softplus(z[~pos]).mean() if (~pos).any() else z.sum() * 0
    return 0.5 * (pl + nl)


def scalar_band(got, r16, r32, label):
    band = abs(r32 - r16)
    tol = BF16_BAND * band + BF16_SCALAR_FLOOR * max(abs(r16), abs(r32))
    assert abs(got - r16) <= tol and abs(got - r32) <= tol, (label, got, r16, r32)


@pytest.mark.parametrize("case", BF16_CASES)
def test_bf16_autograd_step0_within_band(case):
    f16 = Fixture(case)
    f32 = Fixture(f16.meta["twin"])
    m = f16.meta
    model = build(f16)
    model.train()
    b = f16.batch(0)
    z, p, a = model(to_torch_batch(b), seed=m["seeds"][0])
    check_bf16_band(f16, f32, "out0/logits", z)
    check_bf16_band(f16, f32, "out0/aux", a)
    y = torch.from_numpy(b["y"]).float().cuda()
    loss = bce(z, y)
    if model.aux_weight > 0:
        loss = loss + model.aux_weight * bce(a, y)
    scalar_band(loss.item(), float(f16.z["out0/loss"]), float(f32.z["out0/loss"]), f"{case} loss")
    loss.backward()
    got = {k: prm.grad for k, prm in model.named_parameters() if prm.grad is not None}
    assert sorted(got) == sorted(m["grad_keys"])
    for k, g in got.items():
        check_bf16_band(f16, f32, f"grad0/{k}", g)


@pytest.mark.parametrize("case", BF16_CASES)
def test_bf16_fused_steps_within_band(case):
    from tossctr import FusedAdamW, build_ema
    f16 = Fixture(case)
    f32 = Fixture(f16.meta["twin"])
    m, tr = f16.meta, f16.meta["train"]
    model = build(f16)
    ema = build_ema(model, m["cfg"])
    opt = FusedAdamW(model, lr=tr["lr"], weight_decay=tr["wd"], max_grad_norm=tr["clip"], ema=ema, lazy=True)
    p0 = {k: torch.from_numpy(v).double() for k, v in f16.params0().items()}
    for t in range(m["steps"]):
        b = f16.batch(t)
        opt.param_groups[0]["lr"] = m["lrs"][t]
        loss = model.train_step(model.stage(to_torch_batch(b)), torch.from_numpy(b["y"]).float().cuda(), opt,
                                global_step=t + 1, seed=m["seeds"][t])
        scalar_band(loss.item(), float(f16.z[f"out{t}/loss"]), float(f32.z[f"out{t}/loss"]), f"{case} loss {t}")
        if tr["clip"] > 0:
            scalar_band(float(opt.norm_out[0].item()), float(f16.z[f"out{t}/gnorm"]), float(f32.z[f"out{t}/gnorm"]),
                        f"{case} gnorm {t}")
    # after the first AdamW step a lone element may take the other sign step (golden_util.check_bf16_band):
    # measured only on cfg4_full_bf16 (vT/qnn.mlp.0.weight, profiles/r03/amp_band_start.log), so only that
    # case may leave one such element out; every other case is held to the full band
    fl = 1 if case == "cfg4_full_bf16" and m["steps"] > 1 else 0
    sd = model.state_dict()
    for k, v in sd.items():
        check_bf16_band(f16, f32, f"dT/{k}", v.double().cpu() - p0[k], update=True, p0=p0[k], flips=fl)
    ar = model.arena
    for k in m["grad_keys"]:
        check_bf16_band(f16, f32, f"mT/{k}", ar._view(opt.m, k), flips=fl)
        check_bf16_band(f16, f32, f"vT/{k}", ar._view(opt.v, k), flips=fl)
    if ema is not None:
        for k, v in ema.shadow_params().items():
            check_bf16_band(f16, f32, f"demaT/{k}", v.double().cpu() - p0[k], update=True, p0=p0[k], flips=fl)


def test_bf16_differs_from_fp32_build():
    """amp: bf16 really changes the arithmetic (not a silent fp32 run), and amp: none is untouched."""
    from tossctr import CTRModel
    f16 = Fixture("cfg2_dims_bf16")
    m = f16.meta
    outs = {}
    for amp in ("none", "bf16"):
        model = CTRModel(dict(m["cfg"], amp=amp), m["vocab"], m["Fn"], m["Fm"], f16.cat_cards, f16.cat_cols,
                         device="cuda:0")
        model.load_state_dict({k: torch.from_numpy(v) for k, v in f16.params0().items()})
        model.eval()
        with torch.no_grad():
            outs[amp] = model(to_torch_batch(f16.batch(0)))[0].double().cpu()
    assert outs["none"].shape == (m["B"],)
    rel = float((outs["bf16"] - outs["none"]).norm() / outs["none"].norm())
    assert 1e-6 < rel < 5e-2, rel
    assert np.isfinite(outs["bf16"].numpy()).all()
