"""Debug aid: run a golden case's fused steps on the GPU and dump params / Adam moments of chosen keys
after every step (gpurun_out/parity_dump_<case>.npz), for comparison with the oracle on the host.
usage: python tools/parity_dump.py CASE KEY [KEY ...] [--dense]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "toss-next-ctr-prediction_amd")]

from golden_util import Fixture, to_torch_batch  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    case, keys = args[0], args[1:]
    from tossctr import CTRModel, FusedAdamW, build_ema
    fx = Fixture(case)
    m, tr = fx.meta, fx.meta["train"]
    model = CTRModel(m["cfg"], m["vocab"], m["Fn"], m["Fm"], fx.cat_cards, fx.cat_cols, device="cuda:0")
    model.load_state_dict({k: torch.from_numpy(v) for k, v in fx.params0().items()})
    ema = build_ema(model, m["cfg"])
    opt = FusedAdamW(model, lr=tr["lr"], weight_decay=tr["wd"], max_grad_norm=tr["clip"], ema=ema,
                     lazy="--dense" not in sys.argv)
    out = {}
    for t in range(m["steps"]):
        b = fx.batch(t)
        opt.param_groups[0]["lr"] = m["lrs"][t]
        model.train_step(model.stage(to_torch_batch(b)), torch.from_numpy(b["y"]).float().cuda(), opt,
                         global_step=t + 1, seed=m["seeds"][t])
        model.sync()
        out[f"s{t}/gnorm"] = opt.norm_out.cpu().numpy()
        for k in keys:
            out[f"s{t}/p/{k}"] = model.arena.views[k].cpu().numpy()
            out[f"s{t}/m/{k}"] = model.arena._view(opt.m, k).cpu().numpy()
            out[f"s{t}/v/{k}"] = model.arena._view(opt.v, k).cpu().numpy()
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(REPO, "gpurun_out", f"parity_dump_{case}.npz"), **out)


if __name__ == "__main__":
    main()
