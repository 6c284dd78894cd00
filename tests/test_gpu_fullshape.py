"""One training step at the bench's FULL shape against the CPU oracle.

BASELINE config 2 exactly as bench.py runs it (tossctr.configs.dare_qnn_next: D = 32, L = 100, K = 60, 3
encoder layers, 82 + 82 + 35 features, MLP 7552-512-256; B = 4096; DARE tables 10,000,000 x 32, hashed tables
1,000,000 x d_c) from the reference's own initialisation (oracle.synth.reference_init, pinned bitwise against
the reference by tests/golden/gen_golden.py), the yaml's lr 3e-4, clip 0.5, EMA 0.999.  Every grid-size- and
batch-size-dependent code path runs at its production size here: the XCD-aware attention grid over 4096
samples, the persistent FFN row walk over 245,760 rows, the rocPRIM sorts of 409,600 top-K keys and 143,360
categorical keys, the lazy touch / update class lists.

The HIP step runs in fp32 (amp none: the oracle is fp32) and is compared with oracle.model.TrainState.step on
the same batch and dropout seed (north star: 1e-4 rtol on fp32 logits / grads):
  * loss (1e-5 relative), logits (norm-wise 1e-4), the clip's global grad norm (1e-4 relative);
  * top-K: the token in every slot exactly, the position wherever the score is not tied;
  * both Adam moments after the step -- m = 0.1 * clip_coef * g and v = 0.001 * (clip_coef * g)^2 pin the
    gradient of every dense parameter and of every touched table row (norm-wise 2e-4 / 4e-4, the moment
    tolerances of golden_util.Fixture.check_moment);
  * the parameter update p1 - p0 and the EMA shadow's on the dense parameters and the touched rows (norm-wise
    1e-4 + 2 fp32 ulps, elementwise within one lr; well-conditioned elements as in test_gpu_shard.py);
  * untouched table rows (a sample of 4096 per table): the decay-only step p0 (1 - lr wd) and its EMA,
    within 1 fp32 ulp.
The oracle takes ~30 s and ~35 GB of host memory on the GPU box's 16 threads."""
import zlib

import numpy as np
import pytest
import torch

from golden_util import close_enough, to_torch_batch

pytestmark = pytest.mark.gpu

LR, WD, CLIP = 3e-4, 1e-4, 0.5


def _touched(b, cols):
    out = {"dare.emb_att.weight": np.unique(b["seq"]), "dare.emb_rep.weight": np.unique(b["seq"])}
    for i, c in enumerate(cols):
        out[f"cat_embs.{c}.weight"] = np.unique(b["X_cat"][:, i])
    return out


@pytest.mark.timeout(900)
def test_cfg2_full_shape_step_matches_oracle():
    from oracle.model import TrainState, make_arch
    from oracle.synth import make_batch, reference_init
    from tossctr import CTRModel, FusedAdamW, build_ema
    from tossctr.configs import N_NUM_NEXT, cat_cardinals, dare_qnn_next

    torch.set_num_threads(16)
    cfg = dare_qnn_next()
    cfg["amp"] = "none"
    cards = cat_cardinals(cfg)
    cols = list(cards)
    vocab, B, L, Fn = 10_000_000, 4096, 100, N_NUM_NEXT
    A = make_arch(cfg, vocab, Fn, Fn, cards, cols)
    P0 = {k: torch.from_numpy(v) for k, v in reference_init(A, 2024).items()}
    b = make_batch(B, Fn, Fn, list(cards.values()), L, vocab, seed=31337, pos_rate=0.019)
    seed = (777 << 32) | 1

    # ---- the HIP step (fused path: compact table grads, exact lazy AdamW / EMA)
    model = CTRModel(cfg, vocab, Fn, Fn, cards, cols, device="cuda:0")
    model.load_state_dict(P0)
    ema = build_ema(model, cfg)
    opt = FusedAdamW(model, lr=LR, weight_decay=WD, max_grad_norm=CLIP, ema=ema, lazy=True)
    model.train()
    loss_g = float(model.train_step(model.stage(to_torch_batch(b)), torch.from_numpy(b["y"]).float().cuda(), opt,
                                    global_step=1, seed=seed).item())
    sv = model.engine.last
    logits_g = sv["logits"].double().cpu().numpy()
    idx_g = sv["idx"].cpu().numpy().astype(np.int64)
    gnorm_g = float(opt.norm_out[0].item())
    model.sync()
    touched = _touched(b, cols)
    ar = model.arena
    got = {}
    for k in ar.order:
        views = {n: ar._view(buf, k) for n, buf in (("p", ar.buf), ("m", opt.m), ("v", opt.v), ("e", ema.shadow))}
        if ar.kind[k] == "table":
            rows = torch.from_numpy(touched[k]).cuda()
            got[k] = {n: v[rows].double().cpu() for n, v in views.items()}
            r = np.random.default_rng(zlib.crc32(k.encode()))
            free = np.setdiff1d(r.choice(views["p"].shape[0], 4096, replace=False), touched[k])
            got[k]["free"] = free
            got[k]["p_free"] = views["p"][torch.from_numpy(free).cuda()].cpu()
            got[k]["e_free"] = views["e"][torch.from_numpy(free).cuda()].cpu()
        else:
            got[k] = {n: v.double().cpu() for n, v in views.items()}
    del model, opt, ema
    torch.cuda.empty_cache()

    # ---- the oracle (reference semantics, fp32 CPU)
    st = TrainState(P0, A, LR, WD, CLIP, ema_cfg=cfg["ema"])
    rec = {}
    loss_r, (logits_r, _, _), grads = st.grads(to_torch_batch(b), torch.from_numpy(b["y"]).float(), seed, record=rec)
    for p in st.P.values():      # host memory: the dense table grads exist once (TrainState.step clones them)
        p.grad = None
    gnorm_r = st.apply(grads, LR)
    del grads
    assert abs(loss_g - float(loss_r)) <= 1e-5 * max(1.0, abs(float(loss_r))), (loss_g, float(loss_r))
    close_enough(logits_g, logits_r.detach().double().numpy(), 1e-4, 1e-5, "logits")
    assert abs(gnorm_g - float(gnorm_r)) <= 1e-4 * float(gnorm_r), (gnorm_g, float(gnorm_r))

    idx_r = rec["topk_idx"].numpy().astype(np.int64)
    vals_r = rec["topk_vals"].detach().double().numpy()
    seq = b["seq"].astype(np.int64)
    tok_g, tok_r = np.take_along_axis(seq, idx_g, 1), np.take_along_axis(seq, idx_r, 1)
    assert np.array_equal(tok_g, tok_r), np.argwhere(tok_g != tok_r)[:5]
    tied = np.zeros(idx_r.shape, bool)
    for i in range(B):
        _, inv, cnt = np.unique(vals_r[i], return_inverse=True, return_counts=True)
        tied[i] = cnt[inv] > 1
    sel = (tok_r != A.pad_id) & ~tied
    assert np.array_equal(idx_g[sel], idx_r[sel])

    for k in A.param_shapes():
        k = k[0]
        p0 = P0[k]
        g = got[k]
        if k in touched:
            rows = torch.from_numpy(touched[k])
            p0k, ref_p, ref_e = p0[rows], st.P[k].detach()[rows], st.shadow[k][rows]
            ref_m = st.m[k][rows] if k in st.m else None
            ref_v = st.v[k][rows] if k in st.v else None
            # untouched rows take the decay-only step (a zero gradient) and the EMA of it
            free = torch.from_numpy(g["free"])
            assert torch.allclose(g["p_free"], st.P[k].detach()[free], rtol=1.2e-7, atol=0), k
            assert torch.allclose(g["e_free"], st.shadow[k][free], rtol=2.4e-7, atol=0), k
        else:
            p0k, ref_p, ref_e = p0, st.P[k].detach(), st.shadow[k]
            ref_m, ref_v = st.m.get(k), st.v.get(k)
        if ref_m is not None:
            close_enough(g["m"].numpy().ravel(), ref_m.double().numpy().ravel(), 2e-4, 0.0, f"m:{k}")
            close_enough(g["v"].numpy().ravel(), ref_v.double().numpy().ravel(), 4e-4, 0.0, f"v:{k}")
        base = p0k.double().numpy().ravel()
        dg = g["p"].numpy().ravel() - base
        dr = ref_p.double().numpy().ravel() - base
        assert np.abs(dg - dr).max(initial=0) <= LR, k
        if ref_v is not None:
            good = np.sqrt(ref_v.double().numpy().ravel() / (1 - 0.999)) >= 100 * 1e-8
            ulp = 2.0 * np.spacing(np.abs(base + dr).astype(np.float32)).astype(np.float64)
            close_enough(dg[good], dr[good], 1e-4, 0.0, f"dp:{k}", ulp[good], elem_rtol=1e-2)
        eg = g["e"].numpy().ravel() - base
        er = ref_e.double().numpy().ravel() - base
        assert np.abs(eg - er).max(initial=0) <= 0.01 * LR + 1e-6, k
