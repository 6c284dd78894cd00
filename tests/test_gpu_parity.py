"""Model-level parity on the GPU: the HIP path (through libctrhip.so) vs the reference's golden
fixtures (tests/golden, produced by running the reference) and vs the CPU oracle.

Tolerances (north_star: fp32 logits/grads within 1e-4 rtol): norm-wise relative error <= 1e-4 with an
elementwise slack of 1e-3*|ref| + 1e-4*max|ref| (summation order differs from torch's MKL/SLEEF CPU
kernels; large tensors through their fingerprints, golden_util.Fixture.check).  After the optimizer
steps: both Adam moments norm-wise at 1e-4; the update pT - p0 and the EMA shadow's norm-wise at 1e-4
on top of 2 fp32 ulps of the result and the generator's replayed AdamW conditioning allowance
(Fixture.check_update).  Top-K indices exactly (golden_util.check_topk)."""
import numpy as np
import pytest
import torch

from golden_util import CASES, Fixture, check_topk, to_torch_batch
from oracle.model import Dropper, forward as oracle_forward

pytestmark = pytest.mark.gpu
RTOL = 1e-4


def build(fx):
    from tossctr import CTRModel
    m = fx.meta
    model = CTRModel(m["cfg"], m["vocab"], m["Fn"], m["Fm"], fx.cat_cards, fx.cat_cols, device="cuda:0")
    model.load_state_dict({k: torch.from_numpy(v) for k, v in fx.params0().items()})
    return model


def bce(z, y):
    pos = y > 0.5
    pl = torch.nn.functional.softplus(-z[pos]).mean() if pos.any() else z.sum() * 0
    nl = torch.nn.functional.softplus(z[~pos]).mean() if (~pos).any() else z.sum() * 0
    return 0.5 * (pl + nl)


@pytest.mark.parametrize("case", CASES)
def test_autograd_path_step0_matches_reference(case):
    """model(batch) -> loss.backward() (the reference's own loop shape) at step 0: outputs + every grad."""
    fx = Fixture(case)
    m = fx.meta
    model = build(fx)
    model.train()
    b = fx.batch(0)
    z, p, a = model(to_torch_batch(b), seed=m["seeds"][0])
    fx.check("out0/logits", z, RTOL, 1e-5)
    fx.check("out0/prob", p, RTOL, 1e-6)
    fx.check("out0/aux", a, RTOL, 1e-5)
    y = torch.from_numpy(b["y"]).float().cuda()
    loss = bce(z, y)
    if model.aux_weight > 0:
        loss = loss + model.aux_weight * bce(a, y)
    assert abs(loss.item() - float(fx.z["out0/loss"])) < RTOL * max(1.0, abs(loss.item()))
    sv = model.engine.last
    check_topk(fx, 0, sv["idx"].cpu().numpy(), sv["vals"].cpu().numpy(), fx.name)
    loss.backward()
    got_keys = [k for k, prm in model.named_parameters() if prm.grad is not None]
    assert sorted(got_keys) == sorted(m["grad_keys"])
    for k, prm in model.named_parameters():
        if prm.grad is not None:
            fx.check(f"grad0/{k}", prm.grad, RTOL, 1e-7)


@pytest.mark.parametrize("lazy", [True, False], ids=["lazy", "dense"])
@pytest.mark.parametrize("case", CASES)
def test_fused_train_steps_match_reference(case, lazy):
    """The fused path (compact table grads + clip/AdamW/EMA; tables lazy or in the dense stream) over
    all fixture steps."""
    from tossctr import FusedAdamW, build_ema
    fx = Fixture(case)
    m, tr = fx.meta, fx.meta["train"]
    model = build(fx)
    ema = build_ema(model, m["cfg"])
    opt = FusedAdamW(model, lr=tr["lr"], weight_decay=tr["wd"], max_grad_norm=tr["clip"], ema=ema, lazy=lazy)
    p0 = {k: torch.from_numpy(v).double() for k, v in fx.params0().items()}
    for t in range(m["steps"]):
        b = fx.batch(t)
        opt.param_groups[0]["lr"] = m["lrs"][t]
        inputs = model.stage(to_torch_batch(b))
        y = torch.from_numpy(b["y"]).float().cuda()
        loss = model.train_step(inputs, y, opt, global_step=t + 1, seed=m["seeds"][t])
        assert abs(loss.item() - float(fx.z[f"out{t}/loss"])) < RTOL * max(1.0, abs(loss.item())), t
        if tr["clip"] > 0:
            gn = float(opt.norm_out[0].item())
            assert abs(gn - float(fx.z[f"out{t}/gnorm"])) < RTOL * gn, (gn, float(fx.z[f"out{t}/gnorm"]))
        sv = model.engine.last
        check_topk(fx, t, sv["idx"].cpu().numpy(), sv["vals"].cpu().numpy(), f"{fx.name} step {t}")
    sd = model.state_dict()
    for k, v in sd.items():
        fx.check_update("dT", k, v.double().cpu() - p0[k], p0[k])
    ar = model.arena
    for k in m["grad_keys"]:
        fx.check_moment("mT", k, ar._view(opt.m, k))
        fx.check_moment("vT", k, ar._view(opt.v, k))
    if ema is not None:
        for k, v in ema.shadow_params().items():
            fx.check_update("demaT", k, v.double().cpu() - p0[k], p0[k])


@pytest.mark.parametrize("case", CASES)
def test_eval_forward_matches_oracle(case):
    fx = Fixture(case)
    model = build(fx)
    model.eval()
    b = fx.batch(0)
    with torch.no_grad():
        z, p, a = model(to_torch_batch(b))
    P = {k: torch.from_numpy(v) for k, v in fx.params0().items()}
    zr, pr, ar = oracle_forward(P, to_torch_batch(b), fx.arch, Dropper(0, training=False))
    for got, ref, name in ((z, zr, "logits"), (a, ar, "aux")):
        got, ref = got.cpu().double(), ref.double()
        assert float((got - ref).norm() / (ref.norm() + 1e-30)) < RTOL, name


def test_fused_step_is_deterministic():
    from tossctr import FusedAdamW
    fx = Fixture("tiny_concat")
    m, tr = fx.meta, fx.meta["train"]
    outs = []
    for _ in range(2):
        model = build(fx)
        opt = FusedAdamW(model, lr=tr["lr"], weight_decay=tr["wd"], max_grad_norm=tr["clip"])
        b = fx.batch(0)
        model.train_step(model.stage(to_torch_batch(b)), torch.from_numpy(b["y"]).float().cuda(), opt, 1,
                         seed=m["seeds"][0])
        model.sync()
        outs.append(model.arena.buf.clone())
    assert torch.equal(outs[0], outs[1])


def test_no_cpu_fallback_library_loaded():
    import tossctr._lib as L
    lib = L.load()
    assert lib._name.endswith("libctrhip.so")
    assert L.query("ctr_abi_version") == 1


def test_non_contributing_step_is_a_zero_gradient_step():
    """train_step(contribute=False) -- a data-parallel rank without rows on an epoch's last step
    (tossctr.train.rank_slice) -- adds nothing: from fresh moments AdamW with a zero gradient only
    decays, p <- p (1 - lr wd) (torch/optim/adam.py), for every element."""
    from tossctr import FusedAdamW
    fx = Fixture("tiny_concat")
    m, tr = fx.meta, fx.meta["train"]
    model = build(fx)
    p0 = {k: v.detach().clone() for k, v in model.state_dict().items()}
    lr, wd = 0.25, 0.125          # exact in fp32: 1 - lr wd = 0.96875 whatever precision forms it
    opt = FusedAdamW(model, lr=lr, weight_decay=wd, max_grad_norm=tr["clip"])
    b = fx.batch(0)
    loss = model.train_step(model.stage(to_torch_batch(b)), torch.from_numpy(b["y"]).float().cuda(), opt, 1,
                            seed=m["seeds"][0], contribute=False)
    assert float(loss.item()) == 0.0
    assert float(opt.norm_out[0].item()) == 0.0
    skip = set(model.no_grad)
    for k, v in model.state_dict().items():
        want = p0[k] if k in skip else p0[k] * np.float32(1.0 - lr * wd)
        assert torch.equal(v, want), k
