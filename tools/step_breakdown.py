"""Per-call device-time breakdown of one cfg2 training step (B=4096, L=100): every C-ABI entry point
and every GEMM shape, timed with HIP events on the engine's stream.  Diagnostic tool (GPU box):

    python tools/step_breakdown.py [--steps 3]
"""
import argparse
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "toss-next-ctr-prediction_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    import bench
    from tossctr import CTRModel, FusedAdamW, build_ema, _lib
    from tossctr.configs import N_NUM_NEXT, cat_cardinals, dare_qnn_next
    from tossctr.engine import Engine

    dev = torch.device("cuda", 0)
    cfg = dare_qnn_next()
    cards = cat_cardinals(cfg)
    model = CTRModel(cfg, 10_000_000, N_NUM_NEXT, N_NUM_NEXT, cards, list(cfg["data"]["cat_cols"]), device=dev)
    model.reset_parameters(torch.Generator(device=dev).manual_seed(1))
    ema = build_ema(model, cfg)
    tr = cfg["train"]
    opt = FusedAdamW(model, lr=tr["lr"], weight_decay=tr["weight_decay"], max_grad_norm=tr["grad_clip_norm"], ema=ema)
    data = bench.synth_batches(args.steps + 2, 4096, 100, N_NUM_NEXT, N_NUM_NEXT, list(cards.values()), 10_000_000,
                               dev, seed=5)
    for i in range(2):
        model.train_step(*data[i], opt, global_step=i + 1)
    torch.cuda.synchronize()

    rec = []
    orig_call = _lib.call

    def timed_call(name, *a):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = orig_call(name, *a)
        e1.record()
        tag = name
        if name == "ctr_gemm":
            M, N, K, _, _, ta, _, _, tb = a[:9]
            tag = f"ctr_gemm M={M} N={N} K={K} ta={ta} tb={tb} splits={a[12]}"
        rec.append((tag, e0, e1))
        return rc

    import tossctr.engine as E
    import tossctr.optim as O
    _lib.call = timed_call
    E.call = timed_call
    O.call = timed_call
    for i in range(args.steps):
        model.train_step(*data[2 + i], opt, global_step=3 + i)
    torch.cuda.synchronize()
    agg = collections.defaultdict(lambda: [0, 0.0])
    for tag, e0, e1 in rec:
        agg[tag][0] += 1
        agg[tag][1] += e0.elapsed_time(e1)
    tot = sum(v[1] for v in agg.values()) / args.steps
    print(f"total device time of timed calls per step: {tot:.3f} ms")
    for tag, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{ms / args.steps * 1e3:9.1f} us/step  {n / args.steps:5.1f} calls  {tag}")


if __name__ == "__main__":
    main()
