"""amp bf16 parity margins: for every tensor the bf16 fused-step test checks (tests/test_gpu_amp.py), the
ratio of the build's deviation to the reference's own bf16-vs-fp32 band (|got - ref_bf16| / band and
|got - ref_fp32| / band) and to the test's tolerance, worst first.  GPU only; prints one line per tensor.

    python tools/amp_band_report.py [case ...]      (default: every golden_util.BF16_CASES case)
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for _p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "toss-next-ctr-prediction_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import golden_util as gu  # noqa: E402


def main():
    from tossctr import CTRModel, FusedAdamW, build_ema
    cases = sys.argv[1:] or gu.BF16_CASES
    for case in cases:
        f16 = gu.Fixture(case)
        f32 = gu.Fixture(f16.meta["twin"])
        m, tr = f16.meta, f16.meta["train"]
        model = CTRModel(m["cfg"], m["vocab"], m["Fn"], m["Fm"], f16.cat_cards, f16.cat_cols, device="cuda:0")
        model.load_state_dict({k: torch.from_numpy(v) for k, v in f16.params0().items()})
        ema = build_ema(model, m["cfg"])
        opt = FusedAdamW(model, lr=tr["lr"], weight_decay=tr["wd"], max_grad_norm=tr["clip"], ema=ema, lazy=True)
        p0 = {k: torch.from_numpy(v).double() for k, v in f16.params0().items()}
        for t in range(m["steps"]):
            b = f16.batch(t)
            opt.param_groups[0]["lr"] = m["lrs"][t]
            loss = model.train_step(model.stage(gu.to_torch_batch(b)), torch.from_numpy(b["y"]).float().cuda(), opt,
                                    global_step=t + 1, seed=m["seeds"][t])
            print(f"{case} step {t}: loss {loss.item():.7f} ref16 {float(f16.z[f'out{t}/loss']):.7f} "
                  f"ref32 {float(f32.z[f'out{t}/loss']):.7f}")
        rows = []
        real = gu.check_bf16_band
        gu.BF16_BAND_SAVE = gu.BF16_BAND

        def probe(name, got, **kw):
            gu.BF16_BAND = 1e30        # never fails: only the margins are reported
            try:
                e16, e32, band = real(f16, f32, name, got, **kw)
            finally:
                gu.BF16_BAND = gu.BF16_BAND_SAVE
            rows.append((max(e16, e32) / max(band, 1e-30), e16 / max(band, 1e-30), e32 / max(band, 1e-30), name))

        sd = model.state_dict()
        for k, v in sd.items():
            probe(f"dT/{k}", v.double().cpu() - p0[k], update=True, p0=p0[k])
        ar = model.arena
        for k in m["grad_keys"]:
            probe(f"mT/{k}", ar._view(opt.m, k))
            probe(f"vT/{k}", ar._view(opt.v, k))
        rows.sort(reverse=True)
        for r in rows[:25]:
            print(f"{case} {r[3]:60s} max/band {r[0]:7.2f}  e16/band {r[1]:7.2f}  e32/band {r[2]:7.2f}")
        # where the worst tensor's deviation sits: concentrated on a few elements (AdamW sign flips after step 0:
        # an element whose step-0 gradient is within rounding noise of 0 moves by +-lr either way) or spread
        worst = rows[0][3]
        kind, key = worst.split("/", 1)
        if kind in ("mT", "vT"):
            got = (ar._view(opt.m if kind == "mT" else opt.v, key)).detach().cpu().double().numpy().ravel()
            idx, r16 = gu._exact_subset(f16, worst)
            idx32, r32 = gu._exact_subset(f32, worst)
            if idx is not None:
                pos = {int(i): j for j, i in enumerate(idx32)}
                sel = [pos[int(i)] for i in idx]
                r32 = r32[sel]
                got = got[idx]
            for lab, d in (("ours-ref32", got - r32), ("ours-ref16", got - r16), ("ref16-ref32", r16 - r32)):
                e = np.sort(d * d)[::-1]
                tot = e.sum() + 1e-300
                print(f"{case} {worst} {lab}: n={e.size} top1 {e[0] / tot:.2f} top10 {e[:10].sum() / tot:.2f} "
                      f"top1% {e[:max(1, e.size // 100)].sum() / tot:.2f} top10% {e[:max(1, e.size // 10)].sum() / tot:.2f}")


if __name__ == "__main__":
    main()
