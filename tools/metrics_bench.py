"""Per-epoch validation cost: device metrics + temperature fit (csrc/metrics.hip) vs the reference's host
path (sklearn AP + numpy WLL + torch-CPU LBFGS) on one fold's validation rows (N/5 of the 10.7 M-row
training set by default).  Not part of the product.

    python tools/metrics_bench.py [--n 2140000]
"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "toss-next-ctr-prediction_amd"))

import torch  # noqa: E402

from tossctr.metrics import Calibrator, DeviceMetrics, final_score  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2_140_000)
    args = ap.parse_args()
    rng = np.random.default_rng(0)
    true = rng.standard_normal(args.n) * 1.5 - 4.5                 # calibrated logits, ~2 % positives
    y = (rng.random(args.n) < 1.0 / (1.0 + np.exp(-true))).astype(np.int64)
    z = (true * 1.6).astype(np.float32)                                # over-confident model: T ~ 1.6
    zd, yd = torch.from_numpy(z).cuda(), torch.from_numpy(y.astype(np.float32)).cuda()
    dm = DeviceMetrics("cuda")
    dm.final_score(zd, yd)                                 # warm-up: first launches load the kernels
    Calibrator("temperature", iters=2).fit(z, y, device_metrics=dm, z_dev=zd, y_dev=yd)
    dm.final_score(zd, yd, T=1.5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s_dev = dm.final_score(zd, yd)
    t1 = time.perf_counter()
    cal = Calibrator("temperature").fit(z, y, device_metrics=dm, z_dev=zd, y_dev=yd)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    s_cal = dm.final_score(zd, yd, T=cal.temperature)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    s_host = final_score(y, 1.0 / (1.0 + np.exp(-z.astype(np.float64))))
    t4 = time.perf_counter()
    hcal = Calibrator("temperature").fit(z, y)
    t5 = time.perf_counter()
    s_hcal = final_score(y, hcal.predict_proba(z))
    t6 = time.perf_counter()
    print(f"n={args.n}")
    print(f"  device: Score {(t1 - t0) * 1e3:.1f} ms, temperature fit {(t2 - t1) * 1e3:.1f} ms, calibrated Score "
          f"{(t3 - t2) * 1e3:.1f} ms -> Score {s_dev[2]:.9f}, T {cal.temperature:.6f}, cal Score {s_cal[2]:.9f}")
    print(f"  host ({torch.get_num_threads()} threads): Score {(t4 - t3) * 1e3:.1f} ms, temperature fit "
          f"{(t5 - t4) * 1e3:.1f} ms, calibrated Score {(t6 - t5) * 1e3:.1f} ms -> Score {s_host[2]:.9f}, "
          f"T {hcal.temperature:.6f}, cal Score {s_hcal[2]:.9f}")


if __name__ == "__main__":
    main()
