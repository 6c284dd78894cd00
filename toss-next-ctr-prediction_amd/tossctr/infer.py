"""Fold-ensemble inference -- drop-in for src/infer.py (``main(cfg_path)``) on MI355X.

Same inputs and output as the reference (src/infer.py:10-173): the test manifest
``data.manifest_test``, every ``ckpt_folds_*.pt`` under ``logging.log_dir/exp_name`` in any of the
three checkpoint formats the reference accepts (src/infer.py:31-67), EMA weights copied over the
model when the checkpoint carries them (:88-93), per-model calibration when ``calibration.enabled``
(:109-116), ``ensemble.method`` over the models (:125-158, src/utils/metrics.py:48-86), and
``submission.csv`` with header ``ID,clicked`` (:164-173).

MI355X mechanics: the test shards are staged into HBM once (data.DeviceShards) and each batch is the
reference's (consecutive ``train.batch_size`` rows -- the SE gate depends on batch composition);
every fold model runs the HIP forward (engine.forward); calibration and the ensemble run on device
(csrc/infer.hip) instead of the reference's per-batch CPU round trip of the logits.
"""
from __future__ import annotations

import argparse
import glob
import json
import os

import numpy as np
import torch

from . import _lib
from ._lib import call
from .engine import ptr

ENSEMBLE_METHODS = {"mean": 0, "geom_mean": 1, "logit_mean": 2, "median": 3, "trim_mean": 4, "weighted": 5}


def _load(path):
    """torch.load with the safe (weights-only) unpickler: this package's checkpoints hold tensors, dicts,
    lists and floats only.  A checkpoint written by the reference's own trainer pickles its sklearn
    calibrator object, which only the full unpickler reads -- that executes code from the file, so it is
    opt-in (CTR_TRUST_CHECKPOINTS=1) for files the user produced themselves."""
    try:
        return torch.load(path, map_location="cpu", weights_only=True)
    except Exception as e:
        if os.environ.get("CTR_TRUST_CHECKPOINTS") != "1":
            raise RuntimeError(f"{path}: not loadable with weights_only=True ({e}); set CTR_TRUST_CHECKPOINTS=1 "
                               "to unpickle a checkpoint you wrote yourself") from e
        return torch.load(path, map_location="cpu", weights_only=False)


def load_checkpoints(paths):
    """[(state, score)] from checkpoint files in the reference's three formats (src/infer.py:31-67):
    a (state, score) tuple, a dict ({"state", "score"} or the state itself), or {"folds": [...]}."""
    entries = []
    for path in paths:
        obj = _load(path)
        if isinstance(obj, tuple) and len(obj) == 2:
            state, score = obj
            entries.append((state, float(score) if score is not None else -1.0))
            continue
        if isinstance(obj, dict) and "folds" not in obj:
            state = obj.get("state", obj)
            score = obj.get("best_score", obj.get("score", -1.0))
            if "model" not in state:
                raise KeyError(f"Checkpoint {path} has no 'model' key in state")
            entries.append((state, float(score)))
            continue
        if isinstance(obj, dict) and "folds" in obj:
            for item in obj["folds"]:
                if isinstance(item, tuple) and len(item) == 2:
                    s, sc = item
                    entries.append((s, float(sc) if sc is not None else -1.0))
                elif isinstance(item, dict):
                    s = item.get("state", item)
                    sc = item.get("best_score", item.get("score", -1.0))
                    if "model" not in s:
                        raise KeyError("Combined checkpoint entry has no 'model' key")
                    entries.append((s, float(sc)))
                else:
                    raise TypeError(f"Unknown entry type inside 'folds' for {path}: {type(item)}")
            continue
        raise TypeError(f"Unknown checkpoint format for {path}: {type(obj)}")
    return entries


def calibrator_params(cal):
    """(T or None, iso_x or None, iso_y or None) of a checkpoint's calibrator: this package's dict form
    ({"method", "temperature", "iso_x", "iso_y"}) or the reference's Calibrator object
    (src/utils/calibration.py:54-110: temp_scaler.log_temp with clamp_T, iso.X_thresholds_/y_thresholds_)."""
    if cal is None:
        return None, None, None
    if isinstance(cal, dict):
        T = cal.get("temperature")
        ix, iy = cal.get("iso_x"), cal.get("iso_y")
        return (None if T is None else float(T), None if ix is None else np.asarray(ix, np.float32),
                None if iy is None else np.asarray(iy, np.float32))
    T = None
    ts = getattr(cal, "temp_scaler", None)
    if ts is not None:
        t = torch.exp(ts.log_temp.detach().float())
        clamp_T = getattr(cal, "clamp_T", (0.2, 5.0))
        if clamp_T is not None:
            t = torch.clamp(t, clamp_T[0], clamp_T[1])
        T = float(t)
    elif getattr(cal, "log_temp", None) is not None:      # this package's Calibrator object
        T = float(cal.temperature)
    iso = getattr(cal, "iso", None)
    if iso is not None:
        return T, np.asarray(iso.X_thresholds_, np.float32), np.asarray(iso.y_thresholds_, np.float32)
    return T, None, None


class _Calib:
    def __init__(self, cal, device):
        T, ix, iy = calibrator_params(cal)
        self.T = T
        self.ix = torch.from_numpy(ix).to(device) if ix is not None else None
        self.iy = torch.from_numpy(iy).to(device) if iy is not None else None

    def __call__(self, z, out, st, enabled):
        use = enabled and (self.T is not None or self.ix is not None)
        call("ctr_calibrate", ptr(z), z.numel(), float(self.T or 1.0), int(use and self.T is not None),
             ptr(self.ix) if use else None, ptr(self.iy) if use else None,
             int(self.ix.numel()) if (use and self.ix is not None) else 0, ptr(out), st)


def ensemble(method, P, weights=None, trim_ratio=0.0):
    """ensemble_probs (src/utils/metrics.py:48-86) over P (M, B) device probabilities."""
    M, B = P.shape
    if M == 1:
        return P[0].clone()
    if method == "rank_avg":        # per-model ranks (argsort) -- torch's sort on the device
        ranks = []
        for p in P:
            order = torch.argsort(p)
            r = torch.zeros_like(p).scatter_(0, order, torch.arange(B, device=p.device, dtype=p.dtype))
            ranks.append((r + 1).float() / (B + 1.0))
        return torch.stack(ranks, 0).mean(0)
    if method not in ENSEMBLE_METHODS:
        raise ValueError(f"Unknown ensemble method: {method}")
    k = 0
    if method == "trim_mean":
        k = int(max(0, min(M // 2, round(M * trim_ratio))))
        if k == 0 or 2 * k >= M:
            method, k = "mean", 0
    if method == "weighted" and weights is None:
        raise AssertionError("weights required for method='weighted'")
    out = torch.empty(B, dtype=torch.float32, device=P.device)
    w = weights.float().contiguous() if weights is not None else None
    call("ctr_ensemble", ptr(P), M, B, ENSEMBLE_METHODS[method], ptr(w), k, ptr(out),
         torch.cuda.current_stream(P.device).cuda_stream)
    return out


def resolve_weights(method, scores, ens_cfg, n_models, device):
    """(method used, weights) as src/infer.py:130-156 resolves them: ``val_weighted`` -> softmax of the
    fold scores / val_weight_temperature with method "weighted"; ``weighted`` -> the configured weights
    (one per model); anything else unweighted.  A single model ignores the ensemble settings."""
    if n_models <= 1:
        return method, None
    if method == "val_weighted":
        temp = float(ens_cfg.get("val_weight_temperature", 10.0))
        s = torch.tensor(scores, dtype=torch.float32, device=device)
        return "weighted", torch.softmax(s / max(1e-6, temp), dim=0)
    if method == "weighted":
        w_cfg = ens_cfg.get("weights", [])
        assert len(w_cfg) == n_models, "weights length must match #folds/models"
        return "weighted", torch.tensor(w_cfg, dtype=torch.float32, device=device)
    return method, None


def _read_ids(manifest):
    ids = []
    for m in manifest["shards"]:
        p = m.get("ids", {}).get("path")
        ids.append(np.load(p, allow_pickle=False) if p and os.path.exists(p) else
                   np.arange(m["start"], m["end"]).astype(str))
    return np.concatenate(ids) if ids else np.zeros(0, dtype=str)


@torch.no_grad()
def main(cfg_path_or_dict, device=None):
    """src/infer.py:10-173.  Returns the submission path."""
    from .data import DeviceShards
    from .optim import ArenaEMA
    from .wrapper import CTRModel
    if isinstance(cfg_path_or_dict, dict):
        cfg = cfg_path_or_dict
    else:
        import yaml
        with open(cfg_path_or_dict) as f:
            cfg = yaml.safe_load(f)
    _lib.load()
    device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    man_path = cfg["data"]["manifest_test"]
    with open(man_path) as f:
        man = json.load(f)
    out_dir = os.path.join(cfg["logging"]["log_dir"], cfg["exp_name"])
    paths = sorted(glob.glob(os.path.join(out_dir, "ckpt_folds_*.pt")))
    assert paths, "No checkpoints found"
    entries = load_checkpoints(paths)
    first = man["shards"][0]
    x_num_dim = int(np.load(first["X_num"]["path"], mmap_mode="r").shape[1])
    x_mask_dim = int(np.load(first["X_mask"]["path"], mmap_mode="r").shape[1])
    seq_vocab = int(cfg.get("seq_vocab", 10_000_000))                         # src/infer.py:77
    cat_cols = cfg["data"]["cat_cols"]
    cards = {c: int(cfg["data"]["hash_buckets"].get(c, 1000003)) + int(cfg["data"].get("hash_buckets_margin", 0))
             for c in cat_cols}
    models, calibs = [], []
    for state, _ in entries:
        m = CTRModel(cfg, seq_vocab, x_num_dim, x_mask_dim, cards, cat_cols, device=device)
        m.load_state_dict(state["model"], strict=True)
        m.eval()
        ema_state = state.get("ema")
        if ema_state is not None:                                               # src/infer.py:88-93
            ema = ArenaEMA(m, base_decay=ema_state.get("base_decay", 0.999))
            ema.load_state_dict(ema_state)
            ema.copy_to(m)
            del ema
        models.append(m)
        calibs.append(_Calib(state.get("calibrator"), device))
    ens = cfg.get("ensemble", {}) or {}
    method, trim = ens.get("method", "logit_mean"), float(ens.get("trim_ratio", 0.0))
    method, weights = resolve_weights(method, [sc for _, sc in entries], ens, len(models), device)
    cal_on = bool(cfg.get("calibration", {}).get("enabled", False))
    store = DeviceShards(man_path, device)
    n, bs = store.rows, int(cfg["train"]["batch_size"])
    ids = _read_ids(man)
    st = torch.cuda.current_stream(device).cuda_stream
    preds = torch.empty(n, dtype=torch.float32, device=device)
    all_idx = torch.arange(n, dtype=torch.int64, device=device)
    P = torch.empty(len(models), bs, dtype=torch.float32, device=device)
    for s0 in range(0, n, bs):
        idx = all_idx[s0:s0 + bs]
        b = idx.numel()
        inputs, _ = store.batch(idx, slot=1)
        for mi, m in enumerate(models):
            z, _, _, _ = m.engine.forward(*inputs, training=False, seed=0, save=False)
            calibs[mi](z, P[mi, :b], st, cal_on)
        preds[s0:s0 + b] = ensemble(method, P[:, :b].contiguous(), weights, trim)
    p = preds.cpu().numpy()
    os.makedirs(out_dir, exist_ok=True)
    rows = np.empty((n, 2), dtype=object)
    rows[:, 0] = ids.astype(str)
    rows[:, 1] = p.astype(np.float64)
    path = os.path.join(out_dir, "submission.csv")
    np.savetxt(path, rows, delimiter=",", header="ID,clicked", comments="", fmt=["%s", "%.8f"])
    return path


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", required=True)
    main(ap.parse_args().cfg)
