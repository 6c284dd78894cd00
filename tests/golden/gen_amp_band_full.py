"""The reference's own bf16-vs-fp32 deviation AT THE FULL-SHAPE TESTS' OWN STEP, as constants for them.

tests/test_gpu_fullshape.py holds the bf16 build's full-shape step against the fp32 oracle within AMP_BAND_K x the
deviation the REFERENCE itself shows between its bf16-autocast and its fp32 run of the same step.  Until round 5 that
band came from a B = 16 fixture (gen_amp_band.py); this script measures it on exactly the step the test runs: the
BASELINE config at its production batch (golden_util.FULL_SHAPE: cfg2 / cfg3 at B = 4096, cfg4 at B = 1024), the
reference's own initialisation (torch.manual_seed(2024) before CTRModel, which oracle.synth.reference_init restates;
the dense parameters are asserted bitwise here), the same synthetic batch and dropout masks (the build's counter masks
injected through gen_golden.DropPatch in the reference's call order).

What runs is the REFERENCE (never copied into the repo): src.models.wrapper.CTRModel forward / backward, bce_wll_style
exec'd from src/train.py:71-90, nn.utils.clip_grad_norm_ as src/train.py:189,194 -- once in fp32 and once with the
forward and the loss inside torch.autocast(bfloat16) (src/train.py:158-168, CPU autocast here: no GPU in this
container).  For each quantity q of the step

    delta[q] = || q_bf16 - q_fp32 || / || q_fp32 ||

for the loss, the clip's global grad norm, the logits and aux logits, and every parameter's raw gradient (the tables
over the rows the batch reads; every other row's gradient is exactly zero in both runs), written to
tests/golden/amp_band_full_<cfg>.json.

    python tests/golden/gen_amp_band_full.py cfg2 [cfg3 cfg4]        # build container only (needs /root/reference)
"""
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, os.path.join(REPO, "tests"), REPO, os.path.join(REPO, "toss-next-ctr-prediction_amd")]

from gen_golden import DropPatch, load_ref  # noqa: E402
from golden_util import (FULL_SHAPE_DSEED, FULL_SHAPE_PSEED, full_shape_case, full_shape_touched,  # noqa: E402
                         to_torch_batch)


def rel(a, b):
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def run(name):
    CTRModel, _, _, _, bce_wll_style = load_ref()
    cfg, cards, cols, A, B, L, vocab, Fn, b = full_shape_case(name)
    touched = full_shape_touched(b, cols)
    torch.manual_seed(FULL_SHAPE_PSEED)
    model = CTRModel(cfg, vocab, Fn, Fn, dict(cards), cols)
    # the dense parameters against oracle.synth.reference_init (the tables follow the same generator stream: a
    # mismatch anywhere before a dense parameter would show in it); the tables are checked at the batch's rows
    from oracle.synth import reference_init
    P0 = reference_init(A, FULL_SHAPE_PSEED)
    for k, p in model.state_dict().items():
        if k in touched:
            r = touched[k]
            assert np.array_equal(p.numpy()[r], P0[k][r]), k
        else:
            assert np.array_equal(p.numpy(), P0[k]), k
    del P0
    aux_w = float(cfg["model"]["qnn_alpha"].get("aux_head_weight", 0.0))
    batch = to_torch_batch(b)
    y = torch.from_numpy(b["y"]).float()
    res = {}
    for amp in ("none", "bf16"):
        t0 = time.time()
        model.train()
        model.zero_grad(set_to_none=True)
        patch = DropPatch(A)
        patch.seed, patch.calls = FULL_SHAPE_DSEED, 0
        ctx = torch.autocast("cpu", dtype=torch.bfloat16) if amp == "bf16" else torch.autocast("cpu", enabled=False)
        with patch, ctx:
            logits, _, aux = model(batch)
            loss = bce_wll_style(logits, y)
            if aux_w > 0:
                loss = loss + aux_w * bce_wll_style(aux, y)
        assert patch.calls == len(patch.sites), (patch.calls, patch.sites)
        loss.backward()
        grads = {}
        for k, p in model.named_parameters():
            if p.grad is None:
                continue
            g = p.grad.detach()
            grads[k] = (g[torch.from_numpy(touched[k])] if k in touched else g).double().numpy().copy()
        gnorm = float(nn.utils.clip_grad_norm_(model.parameters(), float(cfg["train"]["grad_clip_norm"])))
        res[amp] = {"loss": float(loss.item()), "gnorm": gnorm, "logits": logits.detach().double().numpy(),
                    "aux": aux.detach().double().numpy(), "grads": grads}
        print(f"{name} {amp}: loss {res[amp]['loss']:.6f} gnorm {gnorm:.6f} ({time.time() - t0:.1f} s)", flush=True)
    f32, f16 = res["none"], res["bf16"]
    assert set(f32["grads"]) == set(f16["grads"])
    out = {"source": f"the reference's step at the full-shape test's own inputs ({name}: B = {B}, L = {L}, "
                     f"reference init seed {FULL_SHAPE_PSEED}) under autocast(bf16) vs fp32 (gen_amp_band_full.py)",
           "B": B, "L": L,
           "scalars": {q: rel(f16[q], f32[q]) for q in ("loss", "gnorm")},
           "outputs": {q: rel(f16[q], f32[q]) for q in ("logits", "aux")},
           "grads": {k: rel(f16["grads"][k], f32["grads"][k]) for k in sorted(f32["grads"])},
           "fp32": {"loss": f32["loss"], "gnorm": f32["gnorm"]}}
    path = os.path.join(HERE, f"amp_band_full_{name}.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    g = np.array(list(out["grads"].values()))
    print(f"wrote {path}: logits {out['outputs']['logits']:.3e}, loss {out['scalars']['loss']:.3e}, gnorm "
          f"{out['scalars']['gnorm']:.3e}; grads median {np.median(g):.3e}, min {g.min():.3e}, max {g.max():.3e}",
          flush=True)


if __name__ == "__main__":
    torch.set_num_threads(8)
    for n in sys.argv[1:] or ["cfg2", "cfg3", "cfg4"]:
        run(n)
