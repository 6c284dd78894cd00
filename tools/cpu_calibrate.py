"""CPU-baseline calibration: the oracle (oracle/model.py, the CPU baseline bench.py times on
the GPU box as ``cpu_baseline``) timed beside the REFERENCE itself on identical cfg2-shape batches, same
cores, same protocol (1 warm-up + 3 timed steps, median).  Runs only in the build container: it imports the
reference from /root/reference (never shipped); the log goes to profiles/.

The reference step is src/train.py:152-199 with ``amp: none`` (CUDA autocast is a no-op on CPU):
zero_grad -> CTRModel.forward -> bce_wll_style(+0.1 aux) -> backward -> clip_grad_norm_(0.5) -> AdamW ->
ModelEMA.update; the oracle's TrainState.step is the same step, timed -- like bench.py's cpu_baseline -- with
torch's own F.dropout (bernoulli_ masks, the reference's op; ``TrainState.native_dropout``) instead of the
counter-hash masks its parity mode injects: the baseline measures the reference's cost, not the masks.

    python tools/cpu_calibrate.py [--batch 4096] [--threads N] [--timed 3]
"""
import argparse
import gc
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "toss-next-ctr-prediction_amd"), os.path.join(REPO, "tests", "golden")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def batches(cfg, B, L, n, seed):
    from bench import synth_batches
    from tossctr.configs import N_NUM_NEXT, cat_cardinals
    cards = cat_cardinals(cfg)
    out = []
    for inp, y in synth_batches(n, B, L, N_NUM_NEXT, N_NUM_NEXT, list(cards.values()), 10_000_000, "cpu", seed):
        X_num, X_mask, X_cat, seq = inp
        out.append(({"X_num": X_num, "X_mask": X_mask, "X_cat": X_cat.long(), "seq": seq.long()}, y))
    return out


def init_params(shapes, seed):
    """bench.cpu_baseline's initialisation (the values do not change the step's cost)."""
    gen = torch.Generator().manual_seed(seed)
    P = {}
    for k, shp in shapes:
        t = torch.empty(shp)
        if "emb" in k or "pbias" in k:
            t.normal_(0, 1, generator=gen)
        elif k.endswith(".w"):
            t.fill_(1.0)
        else:
            t.uniform_(-0.05, 0.05, generator=gen)
        P[k] = t
    return P


def time_reference(cfg, data, lr):
    from gen_golden import load_ref
    from tossctr.configs import N_NUM_NEXT, cat_cardinals
    CTRModel, _, build_ema, _, bce_wll_style = load_ref()
    cards = cat_cardinals(cfg)
    cols = list(cfg["data"]["cat_cols"])
    torch.manual_seed(0)
    model = CTRModel(cfg, 10_000_000, N_NUM_NEXT, N_NUM_NEXT, dict(cards), cols)
    with torch.no_grad():
        for k, v in init_params([(k, tuple(p.shape)) for k, p in model.state_dict().items()], 0).items():
            model.state_dict()[k].copy_(v)
    ema = build_ema(model, cfg)
    opt = torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=cfg["train"]["weight_decay"])
    aux_w = float(cfg["model"]["qnn_alpha"].get("aux_head_weight", 0.0))
    times = []
    for t, (b, y) in enumerate(data):
        t0 = time.perf_counter()
        model.train()
        opt.zero_grad(set_to_none=True)
        logits, prob, aux = model(b)
        loss = bce_wll_style(logits, y)
        if aux_w > 0:
            loss = loss + aux_w * bce_wll_style(aux, y)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), cfg["train"]["grad_clip_norm"])
        opt.step()
        if ema is not None:
            ema.update(model, t + 1)
        float(loss.detach().cpu())                      # src/train.py:202
        times.append(time.perf_counter() - t0)
    del model, opt, ema
    gc.collect()
    return times


def time_oracle(cfg, data, lr):
    from oracle.model import TrainState, make_arch
    from tossctr.configs import N_NUM_NEXT, cat_cardinals
    cards = cat_cardinals(cfg)
    cols = list(cfg["data"]["cat_cols"])
    A = make_arch(cfg, 10_000_000, N_NUM_NEXT, N_NUM_NEXT, cards, cols)
    st = TrainState(init_params(A.param_shapes(), 0), A, lr, cfg["train"]["weight_decay"],
                    cfg["train"]["grad_clip_norm"], ema_cfg=cfg["ema"])
    st.native_dropout = True     # as bench.py's cpu_baseline: torch's bernoulli dropout, the reference's op
    times = []
    for t, (b, y) in enumerate(data):
        t0 = time.perf_counter()
        st.step(b, y, lr, t + 1)
        times.append(time.perf_counter() - t0)
    del st
    gc.collect()
    return times


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--timed", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=2,
                    help="reference / oracle phases alternate this many times (host-load drift cancels)")
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    from bench import cpu_model
    from tossctr.configs import BENCH_CONFIGS
    cfg = BENCH_CONFIGS["cfg2"](batch_size=args.batch)
    cfg["amp"] = "none"
    L = int(cfg["sequence"]["max_len"])
    data = batches(cfg, args.batch, L, 1 + args.timed, 1)
    lr = 3e-4
    res = {"reference": [], "oracle": []}
    for rd in range(args.rounds):
        for name, fn in (("reference", time_reference), ("oracle", time_oracle)):
            ts = fn(cfg, data, lr)
            res[name] += ts[1:]
            print(f"round {rd} {name}: steps {', '.join(f'{x:.2f}' for x in ts)} s (first = warm-up)", flush=True)
    for name in res:
        med = float(np.median(res[name]))
        print(f"{name}: median of {len(res[name])} timed steps {med:.2f} s = {args.batch / med:.1f} samples/s",
              flush=True)
        res[name] = med
    ratio = res["oracle"] / res["reference"]
    print(f"cfg2 shape (bs={args.batch}, L={L}, fp32), {torch.get_num_threads()} threads on {cpu_model()}: "
          f"oracle / reference step time = {ratio:.3f} ({'within' if abs(ratio - 1) <= 0.10 else 'OUTSIDE'} 10 %)",
          flush=True)


if __name__ == "__main__":
    main()
