"""Host logic of the fold-ensemble inference (tossctr/infer.py, drop-in for src/infer.py): the three
checkpoint formats the reference accepts (src/infer.py:31-67) and calibrator parameter extraction."""
import numpy as np
import pytest
import torch


def test_checkpoint_formats(tmp_path):
    from tossctr.infer import load_checkpoints
    st = {"model": {"w": torch.ones(2)}, "calibrator": None}
    torch.save({"state": st, "score": 0.25}, tmp_path / "ckpt_folds_0.pt")            # this package / src/train.py
    torch.save((st, 0.5), tmp_path / "ckpt_folds_1.pt")                                 # (state, score) tuple
    torch.save({"folds": [(st, 0.1), {"state": st, "best_score": 0.2}, {"model": st["model"]}]},
               tmp_path / "ckpt_folds_2.pt")                                            # combined
    torch.save({"model": st["model"], "best_score": 0.7}, tmp_path / "ckpt_folds_3.pt")  # bare state dict
    ents = load_checkpoints(sorted(str(p) for p in tmp_path.glob("ckpt_folds_*.pt")))
    assert [s for _, s in ents] == [0.25, 0.5, 0.1, 0.2, -1.0, 0.7]
    assert all("model" in e[0] for e in ents)
    torch.save({"state": {"nomodel": 1}}, tmp_path / "bad.pt")
    with pytest.raises(KeyError):
        load_checkpoints([str(tmp_path / "bad.pt")])


def test_calibrator_params():
    from tossctr.infer import calibrator_params
    assert calibrator_params(None) == (None, None, None)
    T, ix, iy = calibrator_params({"method": "temperature", "temperature": 1.7})
    assert T == 1.7 and ix is None and iy is None
    T, ix, iy = calibrator_params({"temperature": None, "iso_x": [0.1, 0.5], "iso_y": [0.0, 1.0]})
    assert T is None and np.array_equal(ix, np.float32([0.1, 0.5])) and iy.dtype == np.float32

    class Scaler:      # shape of src/utils/calibration.py:12-20 TemperatureScaler
        log_temp = torch.nn.Parameter(torch.tensor(np.log(9.0), dtype=torch.float32))

    class Iso:
        X_thresholds_ = np.array([0.2, 0.4, 0.9])
        y_thresholds_ = np.array([0.0, 0.5, 1.0])

    class RefCal:      # shape of src/utils/calibration.py:54-66 Calibrator
        temp_scaler, iso, clamp_T = Scaler(), Iso(), (0.2, 5.0)

    T, ix, iy = calibrator_params(RefCal())
    assert T == pytest.approx(5.0) and list(ix) == pytest.approx([0.2, 0.4, 0.9]) and len(iy) == 3


def _infer_fixture():
    import json
    import os
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "infer_ref.npz"))
    return z, json.loads(str(z["meta"]))


@pytest.mark.parametrize("i", range(5))
def test_host_calibrator_matches_reference(i):
    """tossctr.metrics.Calibrator (host path) vs the reference's own Calibrator run on the same logits
    (tests/golden/infer_ref.npz, gen_golden.gen_infer; src/utils/calibration.py:54-110): fitted
    temperature, isotonic thresholds (incl. the min_iso_nodes fallback) and predict_proba."""
    from tossctr.metrics import Calibrator
    z, meta = _infer_fixture()
    case = meta["cal_cases"][i]
    tag = case["tag"]
    logits = z["cal/z_few"] if case["few"] else z["cal/z"]
    cal = Calibrator(method=case["method"], lr=0.05, iters=200).fit(logits, z["cal/y"])
    if f"{tag}/T" in z.files:
        assert cal.temperature == pytest.approx(float(z[f"{tag}/T"]), rel=1e-6)
    else:
        assert cal.temperature is None
    if f"{tag}/iso_x" in z.files:
        np.testing.assert_allclose(cal.iso.X_thresholds_, z[f"{tag}/iso_x"], rtol=1e-7)
        np.testing.assert_allclose(cal.iso.y_thresholds_, z[f"{tag}/iso_y"], rtol=1e-7)
    else:
        assert cal.iso is None
    np.testing.assert_allclose(cal.predict_proba(z["cal/zq"]), z[f"{tag}/pq"], rtol=1e-6, atol=1e-9)
