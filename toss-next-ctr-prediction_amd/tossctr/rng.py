"""Host side of the counter-based dropout RNG (device side: csrc/common.h).

Per training step a 64-bit seed; per dropout site a 32-bit key derived from (seed, site).  The
kernels hash (key, element index) -- so masks are recomputed in the backward pass instead of stored.
"""
from __future__ import annotations

M32 = 0xFFFFFFFF

SITE_EMB = 0          # emb_dropout on the stacked cat embeddings  (src/models/wrapper.py:150)
SITE_ATTN0 = 1        # + 2*layer: MHA attention-probability dropout (src/models/dare.py:43)
SITE_FFN0 = 2         # + 2*layer: FFN dropout                     (src/models/dare.py:46)
SITE_DARE = 100       # u_seq dropout                              (src/models/dare.py:158)
SITE_QNN = 101        # interaction dropout                        (src/models/qnn_alpha.py:121)
SITE_MLP0 = 102       # + j: MLP hidden dropout                    (src/models/qnn_alpha.py:81)
SITE_FC = 110         # fc head dropout (QNN disabled)             (src/models/wrapper.py:98)


def _mix32(x):
    x &= M32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & M32
    x ^= x >> 16
    return x


def site_key(seed: int, site: int) -> int:
    lo, hi = seed & M32, (seed >> 32) & M32
    return _mix32(lo ^ _mix32((hi + site * 0x9E3779B9) & M32))


def drop_args(seed: int, site: int, p: float, training: bool):
    """(key, thresh16, scale) for the kernels (csrc/common.h); thresh 0 disables dropout (eval or p == 0),
    so any p > 0 gets at least 1."""
    import numpy as np
    if not training or p <= 0.0:
        return (0, 0, 1.0)
    thresh = min(1 << 16, max(1, int(round(float(p) * (1 << 16)))))
    scale = float(np.float32(1.0) / np.float32(1.0 - p))
    return (site_key(seed, site), thresh, scale)


def step_seed(base_seed: int, step: int) -> int:
    return ((base_seed & M32) << 32) | (step & M32)
