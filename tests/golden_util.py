"""Fixture loading / comparison helpers shared by the CPU and GPU parity tests."""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from oracle import synth
from oracle.model import make_arch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["tiny_concat", "tiny_s1_relu", "tiny_s2", "base_fc", "cfg2_dims", "k148"]


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
        if self.meta["store_params"]:
            return {k: self.z[f"p0/{k}"] for k, _ in self.arch.param_shapes()}
        return synth.make_params(self.arch.param_shapes(), self.meta["pseed"], pad_id=self.arch.pad_id)

    def batch(self, t):
        return {k: self.z[f"in{t}/{k}"] for k in ("X_num", "X_mask", "X_cat", "seq", "y", "groups")}

    def has(self, name):
        return name in self.z.files or f"{name}@idx" in self.z.files

    def check(self, name, got, rtol=1e-4, atol=1e-6, what=None):
        """Compare ``got`` with the stored full tensor or its fingerprint (norm-wise + elementwise)."""
        if isinstance(got, torch.Tensor):
            got = got.detach().cpu().numpy()
        got = np.asarray(got, dtype=np.float64).ravel()
        label = what or f"{self.name}:{name}"
        if name in self.z.files:
            ref = np.asarray(self.z[name], dtype=np.float64).ravel()
            assert got.shape == ref.shape, (label, got.shape, ref.shape)
            close_enough(got, ref, rtol, atol, label)
            return
        fp = {k: self.z[f"{name}@{k}"] for k in ("idx", "vals", "sum", "sumsq", "proj")}
        close_enough(got[fp["idx"]], fp["vals"].astype(np.float64), rtol, atol, label + "[sampled]")
        scale = np.sqrt(float(fp["sumsq"])) * np.sqrt(got.size) + 1e-30
        assert abs(got.sum() - float(fp["sum"])) <= rtol * scale + atol * got.size, (label, "sum")
        assert abs((got * got).sum() - float(fp["sumsq"])) <= 2 * rtol * float(fp["sumsq"]) + atol, (label, "sumsq")
        proj = synth.fingerprint_proj_vec(got.size).astype(np.float64)
        assert abs(got @ proj - float(fp["proj"])) <= rtol * scale + atol * got.size, (label, "proj")


def close_enough(got, ref, rtol, atol, label):
    """Norm-wise relative error <= rtol AND elementwise |d| <= atol + rtol*(10|ref| + max|ref|)."""
    d = np.abs(got - ref)
    nrm = np.linalg.norm(ref)
    rel = np.linalg.norm(got - ref) / (nrm + 1e-30)
    bad = d > atol + 10 * rtol * np.abs(ref) + rtol * np.abs(ref).max(initial=0)
    assert (rel <= rtol or nrm == 0 and d.max(initial=0) <= atol) and not bad.any(), (
        f"{label}: normwise rel err {rel:.3e} (rtol {rtol}), {bad.sum()} elems beyond elementwise tol; "
        f"max abs diff {d.max(initial=0):.3e}")


def to_torch_batch(b):
    return {"X_num": torch.from_numpy(b["X_num"]).float(), "X_mask": torch.from_numpy(b["X_mask"]).float(),
            "X_cat": torch.from_numpy(b["X_cat"]).long(), "seq": torch.from_numpy(b["seq"]).long()}
