"""Fold-ensemble inference (tossctr/infer.py, drop-in for src/infer.py) end to end on a tiny test
cache: three fold checkpoints in the reference's three formats (one with EMA weights, calibrators:
temperature, temperature + isotonic, none), every ensemble method, against the CPU oracle forward
(oracle/model.py, pinned to the reference) + a numpy/torch restatement of the reference's calibration
(src/utils/calibration.py:102-110) and ensemble_probs (src/utils/metrics.py:48-86)."""
import os

import numpy as np
import pytest
import torch

from golden_util import close_enough

pytestmark = pytest.mark.gpu

COLS = ["c0", "c1", "c2", "c3"]


def _cfg(tmp, man, method):
    from test_gpu_train import tiny_run_cfg
    cfg = tiny_run_cfg(tmp, None)
    cfg["data"]["manifest_test"] = man
    cfg["train"]["batch_size"] = 96          # 250 rows -> two full batches and a ragged one
    cfg["ensemble"] = {"method": method, "trim_ratio": 0.34, "weights": [0.2, 0.3, 0.5],
                       "val_weight_temperature": 5.0}
    return cfg


def _ref_calibrate(z, cal):
    """src/utils/calibration.py:102-110 in fp32 (temperature) + np.interp (isotonic, clip)."""
    if cal is None:
        return None
    zt = z.astype(np.float32)
    if cal.get("temperature") is not None:
        zt = (zt / np.float32(cal["temperature"])).astype(np.float32)
    p = 1.0 / (1.0 + np.exp(-np.clip(zt, -50.0, 50.0)))
    if cal.get("iso_x") is not None:
        p = np.interp(np.clip(p, 1e-7, 1 - 1e-7), cal["iso_x"], cal["iso_y"])
    return np.clip(p, 1e-7, 1 - 1e-7)


def _ref_ensemble(method, ps, scores, ens):
    P = torch.tensor(np.stack(ps), dtype=torch.float64)
    M = P.shape[0]
    w = None
    if method == "val_weighted":
        w = torch.softmax(torch.tensor(scores, dtype=torch.float64) / ens["val_weight_temperature"], 0)
        method = "weighted"
    elif method == "weighted":
        w = torch.tensor(ens["weights"], dtype=torch.float64)
    if w is not None:
        w = w / w.sum()
    if method in ("mean", "weighted"):
        return (P.mean(0) if w is None else (P * w.view(-1, 1)).sum(0)).numpy()
    if method == "geom_mean":
        return torch.exp(torch.log(P.clamp(1e-7, 1 - 1e-7)).mean(0)).numpy()
    if method == "logit_mean":
        Pc = P.clamp(1e-7, 1 - 1e-7)
        return torch.sigmoid((torch.log(Pc) - torch.log1p(-Pc)).mean(0)).numpy()
    if method == "median":
        return torch.median(P, 0).values.numpy()
    if method == "trim_mean":
        k = int(max(0, min(M // 2, round(M * ens["trim_ratio"]))))
        return P.mean(0).numpy() if k == 0 else torch.sort(P, 0)[0][k:M - k].mean(0).numpy()
    if method == "rank_avg":
        r = [(torch.argsort(torch.argsort(p)).double() + 1) / (p.numel() + 1.0) for p in P]
        return torch.stack(r).mean(0).numpy()
    raise ValueError(method)


@pytest.mark.parametrize("method", ["logit_mean", "mean", "geom_mean", "median", "trim_mean", "weighted",
                                    "val_weighted", "rank_avg"])
def test_fold_ensemble_inference_matches_oracle(tmp_path, method):
    from oracle.model import Dropper, forward, make_arch
    from oracle.synth import make_params
    from tossctr.data import synth_rows, write_shard_cache
    from tossctr.infer import main
    arr = synth_rows(250, 6, 6, [203] * 4, 24, 3000, seed=11, pos_rate=0.2)
    man = write_shard_cache(str(tmp_path / "test"), arr, shard_rows=100, num_cols=[f"n{i}" for i in range(6)],
                            cat_cols=COLS, group_key="c0", is_train=False)
    cfg = _cfg(str(tmp_path), man, method)
    cards = {c: 203 for c in COLS}
    A = make_arch(cfg, 3000, 6, 6, cards, COLS)
    shapes = A.param_shapes()
    out_dir = os.path.join(cfg["logging"]["log_dir"], cfg["exp_name"])
    os.makedirs(out_dir)
    P = [make_params(shapes, s, A.pad_id) for s in (21, 22, 23)]
    shadow = make_params(shapes, 99, A.pad_id)
    t = lambda d: {k: torch.from_numpy(v) for k, v in d.items()}
    cals = [{"method": "temperature", "temperature": 1.6},
            {"method": "temperature+isotonic", "temperature": 0.8,
             "iso_x": [0.05, 0.3, 0.5, 0.7, 0.95], "iso_y": [0.01, 0.2, 0.25, 0.6, 0.99]},
            None]
    ema = {"base_decay": 0.999, "warmup_steps": 0, "warmup_type": "linear", "update_after_step": 0,
           "update_interval": 1, "ema_on_buffers": "copy", "offload_to_cpu": False, "pin_memory": False,
           "param_filter": [], "num_updates": 5, "shadow_params": t(shadow), "shadow_buffers": {}}
    states = [{"model": t(P[0]), "calibrator": cals[0]},
              {"model": t(P[1]), "calibrator": cals[1], "ema": ema},
              {"model": t(P[2]), "calibrator": cals[2]}]
    scores = [0.31, 0.35, 0.33]
    torch.save({"state": states[0], "score": scores[0]}, os.path.join(out_dir, "ckpt_folds_0.pt"))
    torch.save((states[1], scores[1]), os.path.join(out_dir, "ckpt_folds_1.pt"))
    torch.save({"folds": [{"state": states[2], "best_score": scores[2]}]}, os.path.join(out_dir, "ckpt_folds_2.pt"))
    path = main(cfg)
    got = np.loadtxt(path, delimiter=",", skiprows=1, dtype=str)
    assert list(got[:, 0]) == [f"ID_{i:08d}" for i in range(250)]
    got_p = got[:, 1].astype(np.float64)
    # oracle: eval forward per reference batch with the weights each checkpoint resolves to
    eff = [P[0], shadow, P[2]]        # model 1 runs on its EMA shadow (src/infer.py:88-93)
    bs = cfg["train"]["batch_size"]
    ref = []
    for s0 in range(0, 250, bs):
        b = {k: torch.from_numpy(np.asarray(arr[k][s0:s0 + bs])) for k in ("X_num", "X_mask", "X_cat", "seq")}
        b["X_mask"] = b["X_mask"].float()
        ps = []
        for mi in range(3):
            z, prob, _ = forward(t(eff[mi]), b, A, Dropper(0, training=False))
            p = _ref_calibrate(z.numpy(), cals[mi])
            ps.append(np.clip(prob.numpy(), 1e-7, 1 - 1e-7) if p is None else p)
        ref.append(_ref_ensemble(method, ps, scores, cfg["ensemble"]))
    ref = np.concatenate(ref)
    close_enough(got_p, ref, 1e-5, 2e-7, f"ensemble {method}")


def _infer_fixture():
    import json
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "infer_ref.npz"))
    return z, json.loads(str(z["meta"]))


@pytest.mark.parametrize("M", [2, 3, 4, 5])
@pytest.mark.parametrize("method", ["mean", "geom_mean", "logit_mean", "median", "trim_mean", "weighted",
                                    "val_weighted"])
def test_ensemble_matches_reference_fixture(M, method):
    """tossctr.infer.ensemble (csrc/infer.hip) + resolve_weights vs the reference's own ensemble_probs run
    on the same per-model probabilities (tests/golden/infer_ref.npz; src/utils/metrics.py:48-86,
    src/infer.py:130-158).  rank_avg is absent: the reference's _rank_avg_stack raises for float inputs
    (src/utils/metrics.py:43 scatters an int64 arange into a float tensor), see DESIGN.md §8."""
    from tossctr.infer import ensemble, resolve_weights
    z, meta = _infer_fixture()
    ens = {"trim_ratio": meta["trim_ratio"], "val_weight_temperature": meta["val_weight_temperature"],
           "weights": [float(w) for w in z[f"ens{M}/weights"]]}
    P = torch.from_numpy(z[f"ens{M}/p"]).cuda()
    use, w = resolve_weights(method, [float(s) for s in z[f"ens{M}/scores"]], ens, M, P.device)
    got = ensemble(use, P.contiguous(), w, meta["trim_ratio"]).cpu().numpy().astype(np.float64)
    ref = z[f"ens{M}/{method}"].astype(np.float64)
    if np.isnan(ref).all():
        # trim_mean with 2k == M: the reference averages an empty slice (NaN); this build keeps the mean
        assert method == "trim_mean" and 2 * int(round(M * meta["trim_ratio"])) >= M
        ref = z[f"ens{M}/mean"].astype(np.float64)
    close_enough(got, ref, 1e-6, 1e-9, f"ensemble {method} M={M}")


@pytest.mark.parametrize("i", range(5))
def test_device_calibration_matches_reference_fixture(i):
    """The K-fold loop's calibration on device vs the reference's Calibrator on the same logits
    (tests/golden/infer_ref.npz; src/utils/calibration.py:54-110): the LBFGS temperature fit whose
    closure runs in csrc/metrics.hip (its float64 reductions follow other LBFGS iterates than torch's
    float32 CPU ones: converged T within 2e-4), and the device calibration map (ctr_calibrate, fed the
    reference's own T / isotonic thresholds) on logits spanning the clip range."""
    from tossctr.infer import _Calib
    from tossctr.metrics import Calibrator, DeviceMetrics
    z, meta = _infer_fixture()
    case = meta["cal_cases"][i]
    tag = case["tag"]
    logits = z["cal/z_few"] if case["few"] else z["cal/z"]
    dev = torch.device("cuda", 0)
    cal = Calibrator(method=case["method"], lr=0.05, iters=200).fit(
        logits, z["cal/y"], device_metrics=DeviceMetrics(dev), z_dev=torch.from_numpy(logits).float().to(dev),
        y_dev=torch.from_numpy(z["cal/y"].astype(np.float32)).to(dev))
    if f"{tag}/T" in z.files:
        assert abs(cal.temperature - float(z[f"{tag}/T"])) <= 2e-4 * float(z[f"{tag}/T"])
    else:
        assert cal.temperature is None
    assert (cal.iso is None) == (f"{tag}/iso_x" not in z.files)
    ref_state = {"temperature": float(z[f"{tag}/T"]) if f"{tag}/T" in z.files else None}
    if f"{tag}/iso_x" in z.files:
        ref_state.update(iso_x=z[f"{tag}/iso_x"].tolist(), iso_y=z[f"{tag}/iso_y"].tolist())
    zq = torch.from_numpy(z["cal/zq"]).to(dev)
    out = torch.empty_like(zq)
    _Calib(ref_state, dev)(zq, out, torch.cuda.current_stream(dev).cuda_stream, True)
    close_enough(out.cpu().numpy().astype(np.float64), z[f"{tag}/pq"].astype(np.float64), 1e-6, 1e-9,
                 f"calibration {case['method']}")
