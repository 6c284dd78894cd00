"""CPU-only checks: the C-ABI library loads and exports every symbol include/ctr_hip.h declares, the
ctypes signature table covers the header, and the host logic (arch / state_dict layout / dropout keys /
optimizer layout) agrees with the oracle and the reference fixtures.  No kernel is launched."""
import ctypes
import os
import re

import numpy as np
import pytest

from golden_util import CASES, Fixture

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "ctr_hip.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ctr_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from tossctr import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libctrhip.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_ctypes_table_matches_header():
    from tossctr import _lib
    assert sorted(_lib.SIGS) == header_functions()


@pytest.mark.parametrize("case", CASES)
def test_arch_layout_matches_reference_state_dict(case):
    from tossctr.arch import Arch
    fx = Fixture(case)
    m = fx.meta
    a = Arch.from_cfg(m["cfg"], m["vocab"], m["Fn"], m["Fm"], fx.cat_cards, fx.cat_cols)
    mine = [(k, tuple(s)) for k, s, _ in a.param_shapes()]
    ref = [(k, tuple(s)) for k, s in fx.arch.param_shapes()]
    assert mine == ref
    # params that get no grad in the reference step (fixture grad keys are the reference's own)
    assert sorted(k for k, _ in mine if k not in a.no_grad_keys()) == sorted(m["grad_keys"])


def test_dropout_keys_match_oracle_spec():
    from oracle import rng as orng
    from tossctr import rng
    for seed in (0, 1, (11 << 32) | 3, 2**63 - 1):
        for site in (0, 1, 2, 100, 101, 102, 110):
            assert rng.site_key(seed, site) == orng.site_key(seed, site)
    key, th, sc = rng.drop_args(5, 3, 0.1, True)
    assert th == orng.thresh16(0.1) and np.float32(sc) == orng.dropout_scale(0.1)
    assert rng.drop_args(5, 3, 0.1, False) == (0, 0, 1.0)


def test_lr_schedule_matches_oracle():
    from oracle.model import cosine_warmup_lr as ref
    from tossctr.train import cosine_warmup_lr
    for ep in range(4):
        for st in range(0, 50, 7):
            assert cosine_warmup_lr(ep, st, 50, 3e-4, 2, 8) == ref(ep, st, 50, 3e-4, 2, 8)


def test_ema_decay_schedule_matches_oracle():
    from oracle.model import ema_decay
    from tossctr.optim import ema_decay_at
    for wt in ("linear", "cosine", "none"):
        for n in (0, 1, 10, 3000, 5000):
            assert ema_decay_at(0.999, 3000, wt, n) == ema_decay(0.999, 3000, wt, n)
