"""Device validation metrics (csrc/metrics.hip via tossctr.metrics.DeviceMetrics) against the reference's
host definitions (src/utils/metrics.py:5-29 with sklearn's average_precision_score, restated in
tossctr.metrics.final_score) and the temperature fit (src/utils/calibration.py:23-52, torch LBFGS on CPU,
restated in tossctr.metrics.Calibrator)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _case(n, pos_rate, seed, ties=False, extreme=False):
    rng = np.random.default_rng(seed)
    y = (rng.random(n) < pos_rate).astype(np.int64)
    z = (rng.standard_normal(n) * 1.7 + 1.2 * y - 3.0).astype(np.float32)
    if ties:                           # many equal scores: sklearn groups them into one threshold
        z = np.round(z * 4) / 4
    if extreme:                        # sigmoid saturates / the 1 - 1e-12 clip merges these
        z[:n // 20] = rng.uniform(28, 60, n // 20).astype(np.float32)
        z[n // 20:n // 10] = rng.uniform(-60, -30, n // 10 - n // 20).astype(np.float32)
    return z, y


@pytest.mark.parametrize("n,pos_rate,ties,extreme", [(50000, 0.02, False, False), (20011, 0.3, True, False),
                                                     (7777, 0.1, False, True), (1000, 0.5, True, True),
                                                     (513, 0.0, False, False), (300, 1.0, False, False)])
def test_device_ap_wll_matches_sklearn(n, pos_rate, ties, extreme):
    from tossctr.metrics import DeviceMetrics, final_score
    z, y = _case(n, pos_rate, seed=n, ties=ties, extreme=extreme)
    dm = DeviceMetrics("cuda")
    got = dm.final_score(torch.from_numpy(z).cuda(), torch.from_numpy(y.astype(np.float32)).cuda())
    ref = final_score(y, 1.0 / (1.0 + np.exp(-z.astype(np.float64))))
    for g, r in zip(got, ref):
        if np.isnan(r):
            assert np.isnan(g)
        else:
            assert abs(g - r) <= 1e-12 * max(1.0, abs(r)), (got, ref)


def test_device_temperature_fit_matches_host_lbfgs():
    from tossctr.metrics import Calibrator, DeviceMetrics, final_score
    z, y = _case(40000, 0.05, seed=3)
    z = z * 1.8                                       # over-confident logits: T well above 1
    host = Calibrator("temperature").fit(z, y)
    dm = DeviceMetrics("cuda")
    zd, yd = torch.from_numpy(z).cuda(), torch.from_numpy(y.astype(np.float32)).cuda()
    dev = Calibrator("temperature").fit(z, y, device_metrics=dm, z_dev=zd, y_dev=yd)
    assert abs(dev.temperature - host.temperature) <= 1e-4 * host.temperature, (dev.temperature, host.temperature)
    # calibrated score on device == host predict_proba + final_score: both form float32 probabilities
    # (the reference's datapath); the device expf and numpy's float32 exp may differ by an ulp
    got = dm.final_score(zd, yd, T=host.temperature)
    ref = final_score(y, host.predict_proba(z))
    for g, r in zip(got, ref):
        assert abs(g - r) <= 1e-6 * max(1.0, abs(r)), (got, ref)
