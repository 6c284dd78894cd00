"""numpy restatement of the counter-based dropout RNG the HIP kernels use.

TEST INFRASTRUCTURE (see oracle/__init__.py).

The reference draws dropout masks with ``torch.bernoulli_`` (CPU generator,
``torch.nn.functional.dropout`` -> ``at::native::_dropout_impl``); that stream
cannot be reproduced on the GPU.  The build therefore defines its own
counter-based mask (spec below, kernel side in ``csrc/common.h``) and the
parity fixtures inject exactly these masks into the reference through a
patched ``F.dropout`` (tests/golden/gen_golden.py).  Dropout application itself
follows the reference: ``y = x * (mask / (1 - p))`` (``_dropout_impl``).

Spec (all u32 arithmetic, wrapping):
    mix32(x)      = lowbias32 finaliser
    site_key      = mix32(lo(seed) ^ mix32(hi(seed) + site * 0x9E3779B9))
    bits(key, i)  = mix32((i >> 1) ^ key)           # one hash per element pair (2k, 2k+1)
    u(i)          = i odd ? bits >> 16 : bits & 0xFFFF
    keep(i)       = u(i) >= thresh16(p),  thresh16 = max(1, round(p * 2^16)) for p > 0
"""
from __future__ import annotations

import numpy as np

M32 = 0xFFFFFFFF


def mix32_np(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint32, copy=True)
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def mix32_int(x: int) -> int:
    x &= M32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & M32
    x ^= x >> 16
    return x


def site_key(seed: int, site: int) -> int:
    lo, hi = seed & M32, (seed >> 32) & M32
    return mix32_int(lo ^ mix32_int((hi + site * 0x9E3779B9) & M32))


def thresh16(p: float) -> int:
    if p <= 0.0:
        return 0
    return min(1 << 16, max(1, int(round(float(p) * (1 << 16)))))


_POOL = None


def _pool():
    global _POOL
    if _POOL is None:
        import concurrent.futures
        import os
        _POOL = concurrent.futures.ThreadPoolExecutor(max_workers=os.cpu_count() or 1)
    return _POOL


def keep_mask(seed: int, site: int, p: float, shape) -> np.ndarray:
    """Boolean keep-mask over a tensor of ``shape`` indexed by its C-order linear index: one hash per
    element pair (2k, 2k+1), the low half for the even element and the high half for the odd one.  Large
    masks are hashed in chunks on a thread pool (numpy's ufunc loops release the GIL), so the CPU baseline
    that times the oracle's train step is not bound by a single-threaded mask generator."""
    n = int(np.prod(shape))
    key = np.uint32(site_key(seed, site))
    thr = np.uint32(thresh16(p))
    npair = (n + 1) // 2
    out = np.empty(2 * npair, dtype=bool)

    def work(lo, hi):
        b = mix32_np(np.arange(lo, hi, dtype=np.uint32) ^ key)
        out[2 * lo:2 * hi:2] = (b & np.uint32(0xFFFF)) >= thr
        out[2 * lo + 1:2 * hi:2] = (b >> np.uint32(16)) >= thr

    CH = 1 << 20
    if npair <= CH:
        work(0, npair)
    else:
        list(_pool().map(lambda lo: work(lo, min(npair, lo + CH)), range(0, npair, CH)))
    return out[:n].reshape(shape)


def dropout_scale(p: float) -> np.float32:
    return np.float32(1.0) / np.float32(1.0 - p)
