"""Validation metrics, calibration and logging for the K-fold loop (host reference versions + DeviceMetrics).

Restates src/utils/metrics.py:5-29 (AP, 50:50 weighted logloss, Score), src/utils/calibration.py
(temperature scaling by LBFGS on the 50:50 WLL, optional isotonic) and src/utils/log.py (console + CSV;
TensorBoard is optional and skipped when the package is absent).
"""
from __future__ import annotations

import csv
import os
import time

import numpy as np


def weighted_logloss_50_50(y_true, y_prob, eps=1e-12):
    """src/utils/metrics.py:5-16."""
    y_true = y_true.astype(np.float64, copy=False)
    y_prob = np.nan_to_num(y_prob, nan=0.5, posinf=1.0, neginf=0.0)
    y_prob = np.clip(y_prob.astype(np.float64, copy=False), eps, 1 - eps)
    pos = y_true == 1
    neg = ~pos
    if pos.sum() == 0 or neg.sum() == 0:
        return float("nan")
    return 0.5 * (-np.log(y_prob[pos]).mean() + -np.log(1.0 - y_prob[neg]).mean())


def ap_score(y_true, y_prob):
    """src/utils/metrics.py:18-24."""
    from sklearn.metrics import average_precision_score
    if y_true.mean() in [0.0, 1.0] or len(np.unique(y_true)) < 2:
        return 0.0
    y_prob = np.clip(np.nan_to_num(y_prob, nan=0.5, posinf=1.0, neginf=0.0), 1e-12, 1 - 1e-12)
    return float(average_precision_score(y_true, y_prob))


def final_score(y_true, y_prob):
    """src/utils/metrics.py:26-29: (AP, WLL, 0.5*AP + 0.5*WLL)."""
    ap = ap_score(y_true, y_prob)
    wll = weighted_logloss_50_50(y_true, y_prob)
    return ap, wll, 0.5 * ap + 0.5 * wll


def _sigmoid_np(z):
    z = np.clip(z, -50.0, 50.0)
    return 1.0 / (1.0 + np.exp(-z))


class DeviceMetrics:
    """The same metrics and the temperature fit on device (csrc/metrics.hip) for logits / labels that are
    already in HBM: AP + 50:50 WLL + Score of sigmoid(z) (or of the temperature-calibrated probabilities)
    and fit_temperature's LBFGS (torch.optim.LBFGS on the scalar log-temperature, as the reference runs it)
    whose closure evaluates the loss and its gradient over all rows in one kernel."""

    def __init__(self, device):
        import torch
        self.device = torch.device(device)
        self._ws = None
        self._out = torch.empty(8, dtype=torch.float64, device=self.device)

    def _stream(self):
        import torch
        return torch.cuda.current_stream(self.device).cuda_stream

    def _workspace(self, n):
        import torch
        from . import _lib
        need = int(_lib.query("ctr_metrics_ws_size", n))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self._ws

    def final_score(self, z, y, T=None):
        """(AP, WLL, Score) of sigmoid(z) (f64, as the loop's p_raw) or, with T, of the calibrator's
        clip(sigmoid(z/T)) -- src/utils/metrics.py:26-29 on device.  z, y: float32 device tensors."""
        import torch
        from ._lib import call
        n = z.numel()
        p = torch.empty(max(n, 1), dtype=torch.float64, device=self.device)
        st = self._stream()
        call("ctr_val_prob", z.data_ptr(), n, float(T or 1.0), int(T is not None), p.data_ptr(), st)
        ws = self._workspace(n)
        call("ctr_ap_wll", p.data_ptr(), y.data_ptr(), n, self._out.data_ptr(), ws.data_ptr(), ws.numel(), st)
        ap, wll = (float(v) for v in self._out[:2].cpu())
        return ap, wll, 0.5 * ap + 0.5 * wll

    def fit_temperature(self, z, y, lr=0.05, iters=200, clamp_T=(0.2, 5.0), l2_reg=1e-3):
        """src/utils/calibration.py:23-52: LBFGS(strong_wolfe) on log T of the 50:50 WLL + l2 (T - 1)^2.
        Returns the fitted log-temperature (CPU scalar tensor)."""
        import torch
        from ._lib import call
        n = z.numel()
        w_pos = max(float((y == 1).float().mean()), 1e-6)
        w_neg = 1.0 - w_pos
        ws = self._workspace(n)
        st = self._stream()
        log_temp = torch.nn.Parameter(torch.tensor(np.log(1.0), dtype=torch.float32))
        opt = torch.optim.LBFGS([log_temp], lr=lr, max_iter=iters, line_search_fn="strong_wolfe")

        def closure():
            opt.zero_grad()
            t_raw = float(torch.exp(log_temp.detach()))
            clamped = clamp_T is not None and not (clamp_T[0] <= t_raw <= clamp_T[1])
            T = float(np.float32(min(max(t_raw, clamp_T[0]), clamp_T[1]) if clamp_T is not None else t_raw))
            call("ctr_temp_nll", z.data_ptr(), y.data_ptr(), n, T, self._out.data_ptr(), ws.data_ptr(), ws.numel(), st)
            s_pos, s_neg, g_pos, g_neg = (float(v) for v in self._out[:4].cpu())
            loss = 0.5 * (-(s_pos / n) / w_pos - (s_neg / n) / w_neg) + l2_reg * (T - 1.0) ** 2
            dT = 0.5 * (-(g_pos / n) / w_pos - (g_neg / n) / w_neg) + 2.0 * l2_reg * (T - 1.0)
            log_temp.grad = torch.tensor(0.0 if clamped else dT * T, dtype=torch.float32)
            return torch.tensor(loss, dtype=torch.float32)

        opt.step(closure)
        return log_temp.detach()


class Calibrator:
    """src/utils/calibration.py:54-110: 'temperature' | 'isotonic' | 'temperature+isotonic'."""

    def __init__(self, method="temperature", lr=0.05, iters=200, clamp_T=(0.2, 5.0), l2_reg=1e-3, min_iso_nodes=8):
        self.method, self.lr, self.iters = method, lr, iters
        self.clamp_T, self.l2_reg, self.min_iso_nodes = clamp_T, l2_reg, min_iso_nodes
        self.log_temp = None
        self.iso = None

    def _T(self, log_temp):
        import torch
        T = torch.exp(log_temp)
        return torch.clamp(T, self.clamp_T[0], self.clamp_T[1]) if self.clamp_T is not None else T

    def _fit_temperature(self, z, y):
        import torch
        z = torch.tensor(z, dtype=torch.float32)
        t = torch.tensor(y.astype(np.float32))
        log_temp = torch.nn.Parameter(torch.tensor(np.log(1.0), dtype=torch.float32))
        opt = torch.optim.LBFGS([log_temp], lr=self.lr, max_iter=self.iters, line_search_fn="strong_wolfe")
        with torch.no_grad():
            w_pos = (t == 1).float().mean().clamp(min=1e-6)
            w_neg = 1.0 - w_pos

        def closure():
            # the reference's autograd graph exactly (src/utils/calibration.py:36-49): T is formed twice,
            # once for the scaled logits and once for the regulariser, so the two gradient paths through
            # exp(log_temp) are summed in the same order and LBFGS follows the same iterates bitwise
            opt.zero_grad()
            p = torch.sigmoid(z / self._T(log_temp)).clamp(1e-7, 1 - 1e-7)
            loss_pos = -(t * torch.log(p)).mean() / w_pos
            loss_neg = -((1 - t) * torch.log(1 - p)).mean() / w_neg
            T = self._T(log_temp)
            loss = 0.5 * (loss_pos + loss_neg) + self.l2_reg * (T - 1.0) ** 2
            loss.backward()
            return loss
        opt.step(closure)
        self.log_temp = log_temp.detach()

    @property
    def temperature(self):
        return None if self.log_temp is None else float(self._T(self.log_temp))

    def fit(self, logits, y, device_metrics=None, z_dev=None, y_dev=None):
        """``device_metrics`` (+ the same logits / labels as float32 device tensors): the temperature's
        LBFGS closure runs on device (DeviceMetrics.fit_temperature); isotonic stays on the host."""
        z = np.asarray(logits, dtype=np.float64)
        y = np.asarray(y, dtype=np.int32)
        if self.method in ("temperature", "temperature+isotonic"):
            if device_metrics is not None:
                self.log_temp = device_metrics.fit_temperature(z_dev, y_dev, lr=self.lr, iters=self.iters,
                                                               clamp_T=self.clamp_T, l2_reg=self.l2_reg)
            else:
                self._fit_temperature(z, y)
        if self.method in ("isotonic", "temperature+isotonic"):
            from sklearn.isotonic import IsotonicRegression
            p = _sigmoid_np(self._scaled(z))
            n_pos, n_neg = max(1, int(y.sum())), max(1, int((y == 0).sum()))
            sw = np.where(y == 1, 0.5 / n_pos, 0.5 / n_neg)
            if np.unique(p).size < self.min_iso_nodes:
                self.iso = None
            else:
                self.iso = IsotonicRegression(y_min=0.0, y_max=1.0, out_of_bounds="clip")
                self.iso.fit(p, y, sample_weight=sw)
        return self

    def _scaled(self, z):
        """The temperature-scaled logits as the reference forms them: TemperatureScaler on a float32
        tensor (src/utils/calibration.py:81-83,104-106), so the sigmoid after it runs in float32; the raw
        float64 logits when no temperature was fitted."""
        if self.log_temp is None:
            return z
        return z.astype(np.float32) / np.float32(self.temperature)

    def predict_proba(self, logits):
        z = np.asarray(logits, dtype=np.float64)
        p = _sigmoid_np(self._scaled(z))
        if self.iso is not None:
            p = self.iso.predict(np.clip(p, 1e-7, 1 - 1e-7))
        return np.clip(p, 1e-7, 1 - 1e-7)


class Logger:
    """src/utils/log.py: console rows + train_log.csv (+ TensorBoard scalars when available)."""

    COLS = ["fold", "epoch", "split", "loss", "AP", "WLL", "Score", "lr", "bs", "K", "tau"]

    def __init__(self, log_dir, tb=True, csv_log=True, quiet=False, csv_name="train_log.csv"):
        self.tb = None
        if tb:
            try:
                from torch.utils.tensorboard import SummaryWriter
                self.tb = SummaryWriter(log_dir)
            except Exception:
                self.tb = None
        self.quiet = quiet
        self.csv_path = os.path.join(log_dir, csv_name) if csv_log else None
        if self.csv_path:
            os.makedirs(log_dir, exist_ok=True)
            if not os.path.exists(self.csv_path):
                with open(self.csv_path, "w", newline="") as f:
                    csv.writer(f).writerow(["time"] + self.COLS)

    def scalars(self, tag, step, **kw):
        if self.tb:
            for k, v in kw.items():
                self.tb.add_scalar(f"{tag}/{k}", v, step)

    def row(self, **kw):
        if not self.quiet:
            print("  ".join(f"{k}={v}" for k, v in kw.items()), flush=True)

    def csv(self, **kw):
        if self.csv_path:
            with open(self.csv_path, "a", newline="") as f:
                csv.writer(f).writerow([time.strftime("%Y-%m-%d %H:%M:%S")] + [kw.get(k, "") for k in self.COLS])
