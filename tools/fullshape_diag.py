"""Which bf16 component moves a full-shape step away from fp32: the step of tests/test_gpu_fullshape.py (golden_util
full_shape_case) run once in fp32 and in amp bf16 with single components switched back to their fp32 kernels through
the engine's flags, each compared with the fp32 oracle's gradients (oracle.model.TrainState.grads) on the dense
parameters: the clip's global norm and the per-tensor norm-wise deviation of the gradient (m = 0.1 coef g).
Not part of the product.

    python tools/fullshape_diag.py [cfg4] [variants: fp32,bf16,attn32,ffn32,proj32,gemm32]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "toss-next-ctr-prediction_amd"), os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from golden_util import FULL_SHAPE_DSEED, FULL_SHAPE_PSEED, full_shape_case, to_torch_batch  # noqa: E402

LR, WD, CLIP = 3e-4, 1e-4, 0.5


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "cfg4"
    variants = (sys.argv[2] if len(sys.argv) > 2 else "fp32,bf16,attn32,ffn32,proj32,gemm32").split(",")
    from oracle.model import TrainState
    from oracle.synth import reference_init
    torch.set_num_threads(16)
    cfg, cards, cols, A, B, L, vocab, Fn, b = full_shape_case(name)
    P0 = {k: torch.from_numpy(v) for k, v in reference_init(A, FULL_SHAPE_PSEED).items()}
    st = TrainState(P0, A, LR, WD, CLIP, ema_cfg=None)
    loss, _, grads = st.grads(to_torch_batch(b), torch.from_numpy(b["y"]).float(), FULL_SHAPE_DSEED)
    gn = float(torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g) for g in grads.values()])))
    tables = {"dare.emb_att.weight", "dare.emb_rep.weight"} | {f"cat_embs.{c}.weight" for c in cols}
    gref = {k: g.double().numpy().ravel() for k, g in grads.items() if k not in tables}
    del st, grads
    print(f"{name} B={B}: oracle loss {float(loss):.7f} gnorm {gn:.6f}", flush=True)
    from tossctr import CTRModel, FusedAdamW, build_ema
    for var in variants:
        c = dict(cfg, amp="none" if var == "fp32" else "bf16")
        model = CTRModel(c, vocab, Fn, Fn, cards, cols, device="cuda:0")
        model.load_state_dict(P0)
        eng = model.engine
        if var == "attn32":
            eng.attn_bf = eng.attn_layer = eng.attn_oproj = False
        elif var == "ffn32":
            eng.ffn_flags = 0
        elif var == "proj32":
            eng.rowgemm_bf = False
            eng.rowgemm = False
            eng.gemm_flags = 0
        elif var == "gemm32":
            eng.gemm_flags = 0
        ema = build_ema(model, c)
        opt = FusedAdamW(model, lr=LR, weight_decay=WD, max_grad_norm=CLIP, ema=ema, lazy=True)
        model.train()
        lh = float(model.train_step(model.stage(to_torch_batch(b)), torch.from_numpy(b["y"]).float().cuda(), opt,
                                    global_step=1, seed=FULL_SHAPE_DSEED).item())
        gh, coef = float(opt.norm_out[0].item()), float(opt.norm_out[1].item())
        ar = model.arena
        devs = []
        for k, gr in gref.items():
            m = ar._view(opt.m, k).double().cpu().numpy().ravel()
            g = m / (0.1 * coef)
            devs.append((np.linalg.norm(g - gr) / max(np.linalg.norm(gr), 1e-300), k, np.linalg.norm(gr)))
        devs.sort(reverse=True)
        print(f"[{var}] loss {lh:.7f} ({(lh - float(loss)) / float(loss):+.2e}) gnorm {gh:.6f} ({(gh - gn) / gn:+.3e})")
        for d, k, n in devs[:8]:
            print(f"    {k:42s} {d:.3e}  |g| {n:.3e}")
        del model, opt, ema
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
