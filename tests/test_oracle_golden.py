"""Pin the CPU oracle (oracle/model.py) against the reference's own outputs (tests/golden/*.npz)."""
import numpy as np
import pytest
import torch

from golden_util import CASES, Fixture, to_torch_batch
from oracle import rng
from oracle.model import Dropper, TrainState, forward


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference(case):
    fx = Fixture(case)
    m, A = fx.meta, fx.arch
    tr = m["train"]
    P = {k: torch.from_numpy(v) for k, v in fx.params0().items()}
    st = TrainState(P, A, tr["lr"], tr["wd"], tr["clip"], ema_cfg=m["cfg"].get("ema") if
                    m["cfg"].get("ema", {}).get("enabled") else None)
    assert sorted(A.grad_params()) == sorted(m["grad_keys"])
    for t in range(m["steps"]):
        b = fx.batch(t)
        rec = {}
        loss, (z, p, a), grads, gn = st.step(to_torch_batch(b), torch.from_numpy(b["y"]).float(),
                                             m["lrs"][t], m["seeds"][t], record=rec)
        fx.check(f"out{t}/logits", z, 1e-5, 1e-6)
        fx.check(f"out{t}/prob", p, 1e-5, 1e-7)
        fx.check(f"out{t}/aux", a, 1e-5, 1e-6)
        assert abs(float(loss) - float(fx.z[f"out{t}/loss"])) < 1e-5 * max(1, abs(float(loss)))
        if tr["clip"] > 0:
            assert abs(float(gn) - float(fx.z[f"out{t}/gnorm"])) < 1e-5 * float(gn)
        assert np.array_equal(rec["topk_idx"].numpy(), fx.z[f"out{t}/topk_idx"])
        fx.check(f"out{t}/topk_vals", rec["topk_vals"], 1e-6, 1e-5)
        if t == 0:
            # north-star tolerance (1e-4 rtol): the fixtures come from one host's CPU kernels, and the
            # reduction order of torch's CPU GEMMs differs between CPU models (1.4e-5 seen on the
            # cfg2-width DARE rep-table grad on a host other than the one that wrote the fixtures)
            for k, g in grads.items():
                fx.check(f"grad0/{k}", g, 1e-4, 1e-8)
    # the update pT - p0 and the EMA shadow's, norm-wise at 1e-4 (+ fp32 ulps and the replayed AdamW
    # conditioning allowance, tests/golden_util.Fixture.check_update); both moments norm-wise at 1e-4
    for k, v in st.P.items():
        fx.check_update("dT", k, v.detach().double() - P[k].double(), P[k])
    for k in st.grad_keys:
        fx.check_moment("mT", k, st.m[k])
        fx.check_moment("vT", k, st.v[k])
    if st.shadow is not None:
        for k, v in st.shadow.items():
            fx.check_update("demaT", k, v.double() - P[k].double(), P[k])
    with torch.no_grad():
        z, p, a = forward(st.P, to_torch_batch(fx.batch(m["steps"] - 1)), A, Dropper(0, training=False))
    # after the optimizer steps the parameters themselves agree only within the update allowances above;
    # cfg4_full (4 layers at D = 64) carries that to 1.4e-5 on its eval logits, so it alone is held to the
    # north star's 1e-4 and every other case to 1e-5
    ev = 1e-4 if case == "cfg4_full" else 1e-5
    fx.check("eval/logits", z, ev, 1e-6)
    fx.check("eval/aux", a, ev, 1e-6)


def test_rng_mask_rate_and_determinism():
    k1 = rng.keep_mask(12345, 3, 0.1, (1000, 100))
    k2 = rng.keep_mask(12345, 3, 0.1, (1000, 100))
    assert np.array_equal(k1, k2)
    assert abs(k1.mean() - 0.9) < 0.005
    k3 = rng.keep_mask(12345, 4, 0.1, (1000, 100))
    assert (k1 != k3).mean() > 0.1
    assert rng.keep_mask(1, 1, 0.0, (10,)).all()
