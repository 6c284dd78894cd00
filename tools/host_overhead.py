"""Host-side cost of the training step (GPU box): how long the Python launch loop takes vs the device.

    python tools/host_overhead.py [--steps 50]

Prints per-step wall time with a sync at the end (device-bound figure) and the time the host needs to
issue the step's launches (measured before the final sync), plus a cProfile of the host side."""
import argparse
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "toss-next-ctr-prediction_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    from tossctr import CTRModel, FusedAdamW, build_ema
    from tossctr.configs import BENCH_CONFIGS, N_NUM_NEXT, cat_cardinals
    dev = torch.device("cuda", 0)
    cfg = BENCH_CONFIGS["cfg2"](batch_size=4096)
    L = int(cfg["sequence"]["max_len"])
    cards = cat_cardinals(cfg)
    model = CTRModel(cfg, 10_000_000, N_NUM_NEXT, N_NUM_NEXT, cards, list(cfg["data"]["cat_cols"]), device=dev)
    model.reset_parameters(torch.Generator(device=dev).manual_seed(cfg["seed"]))
    ema = build_ema(model, cfg)
    tr = cfg["train"]
    opt = FusedAdamW(model, lr=tr["lr"], weight_decay=tr["weight_decay"], max_grad_norm=tr["grad_clip_norm"], ema=ema)
    data = bench.synth_batches(16, 4096, L, N_NUM_NEXT, N_NUM_NEXT, list(cards.values()), 10_000_000, dev, seed=1)
    g = [0]

    def run():
        inp, y = data[g[0] % 16]
        g[0] += 1
        return model.train_step(inp, y, opt, global_step=g[0])

    for _ in range(10):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(f"per step: wall {t_all / args.steps * 1e3:.3f} ms, host issue {t_issue / args.steps * 1e3:.3f} ms")
    prof = cProfile.Profile()
    torch.cuda.synchronize()
    prof.enable()
    for _ in range(10):
        run()
    prof.disable()
    torch.cuda.synchronize()
    pstats.Stats(prof).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
