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
