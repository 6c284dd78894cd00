"""amp: bf16 host logic and fixtures (no GPU).

The bf16 fixtures (tests/golden/*_bf16.npz, gen_golden.gen_bf16) are the reference run under
``torch.autocast(bfloat16)`` on the inputs, seeds and parameters of an fp32 fixture (its "twin").  The
GPU test (tests/test_gpu_amp.py) holds the bf16 build within BF16_BAND x the reference's own
bf16-vs-fp32 deviation of both; here: the twins really share their inputs, the band is bf16-sized, the
fp32 oracle lies inside it (so the band check can pass at all), and the configuration plumbing."""
import numpy as np
import pytest
import torch

from golden_util import BF16_CASES, Fixture, check_bf16_band, to_torch_batch
from oracle.model import TrainState


@pytest.mark.parametrize("case", BF16_CASES)
def test_bf16_twin_shares_inputs_and_seeds(case):
    f16 = Fixture(case)
    f32 = Fixture(f16.meta["twin"])
    assert f16.meta["amp"] == "bf16" and f16.meta["cfg"]["amp"] == "bf16"
    assert f16.meta["seeds"] == f32.meta["seeds"] and f16.meta["lrs"] == f32.meta["lrs"]
    for t in range(f16.meta["steps"]):
        for k, v in f16.batch(t).items():
            assert np.array_equal(v, f32.batch(t)[k]), (case, t, k)
    p16, p32 = f16.params0(), f32.params0()
    assert all(np.array_equal(p16[k], p32[k]) for k in p32)


@pytest.mark.parametrize("case", BF16_CASES)
def test_bf16_band_is_bf16_sized(case):
    """The reference's bf16 logits deviate from its fp32 ones by bf16 rounding (2^-8 relative per
    rounded operand), neither bitwise equal nor beyond a few percent."""
    f16 = Fixture(case)
    f32 = Fixture(f16.meta["twin"])
    z16, z32 = f16.z["out0/logits"].astype(np.float64), f32.z["out0/logits"].astype(np.float64)
    rel = np.linalg.norm(z16 - z32) / np.linalg.norm(z32)
    assert 1e-5 < rel < 5e-2, rel


@pytest.mark.parametrize("case", BF16_CASES)
def test_fp32_oracle_is_inside_the_bf16_band(case):
    """The check the GPU bf16 test applies, run on the fp32 oracle: outputs and step-0 grads."""
    f16 = Fixture(case)
    f32 = Fixture(f16.meta["twin"])
    m, A = f32.meta, f32.arch
    tr = m["train"]
    P = {k: torch.from_numpy(v) for k, v in f32.params0().items()}
    st = TrainState(P, A, tr["lr"], tr["wd"], tr["clip"],
                    ema_cfg=m["cfg"].get("ema") if m["cfg"].get("ema", {}).get("enabled") else None)
    b = f32.batch(0)
    _, (z, p, a), grads, _ = st.step(to_torch_batch(b), torch.from_numpy(b["y"]).float(), m["lrs"][0],
                                     m["seeds"][0])
    check_bf16_band(f16, f32, "out0/logits", z)
    check_bf16_band(f16, f32, "out0/aux", a)
    for k, g in grads.items():
        check_bf16_band(f16, f32, f"grad0/{k}", g)


def test_arch_reads_amp():
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "toss-next-ctr-prediction_amd"))
    from tossctr.arch import Arch
    f16 = Fixture("tiny_concat_bf16")
    m = f16.meta
    args = (m["vocab"], m["Fn"], m["Fm"], f16.cat_cards, f16.cat_cols)
    assert Arch.from_cfg(m["cfg"], *args).amp == "bf16"
    assert Arch.from_cfg(dict(m["cfg"], amp="none"), *args).amp == "none"
    assert Arch.from_cfg({k: v for k, v in m["cfg"].items() if k != "amp"}, *args).amp == "none"
    with pytest.raises(NotImplementedError):
        Arch.from_cfg(dict(m["cfg"], amp="fp16"), *args).validate()
