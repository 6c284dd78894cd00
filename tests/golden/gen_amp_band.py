"""The reference's own bf16-vs-fp32 deviation at the cfg2 widths, as constants for the full-shape amp test.

tests/golden/cfg2_ref.npz and cfg2_ref_bf16.npz are the REFERENCE run here (gen_golden.gen_cfg2_ref: BASELINE
config 2's widths -- D = 32, L = 100, K = 60, 3 layers, 82 + 82 + 35 features, QNN 6 x 16 x 192, MLP 7552-512-256
-- from the reference's own init, B = 16) once in fp32 and once under torch.autocast(bfloat16) (src/train.py:158-168
with CPU autocast) on the same inputs, seeds and parameters.  For each step-0 quantity q this writes

    delta[q] = || q_bf16 - q_fp32 || / || q_fp32 ||

(norms over the whole tensor when the fixture stores it in full, else over its exact sampled elements and touched
rows -- golden_util._exact_subset, the same subset for both runs), for the logits, the aux logits, the loss, the
clip's global grad norm and every parameter's raw gradient, to tests/golden/amp_band_cfg2.json.  The GPU test
tests/test_gpu_fullshape.py::test_cfg2_full_shape_bf16_step holds the bf16 build at the bench's full shape
against the fp32 oracle within AMP_BAND_K x these deviations.

    python tests/golden/gen_amp_band.py        # reads the two fixtures only (no reference import)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.dirname(os.path.dirname(HERE))]

from golden_util import Fixture, _exact_subset  # noqa: E402

OUT = os.path.join(HERE, "amp_band_cfg2.json")


def rel(a, b):
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def main():
    f16, f32 = Fixture("cfg2_ref_bf16"), Fixture("cfg2_ref")
    assert f16.meta["twin"] == "cfg2_ref"
    out = {"source": "tests/golden/cfg2_ref_bf16.npz vs cfg2_ref.npz (reference under autocast(bf16) vs fp32, step 0, "
                     f"B = {f32.meta['B']})",
           "scalars": {}, "outputs": {}, "grads": {}}
    for q in ("loss", "gnorm"):
        out["scalars"][q] = rel(f16.z[f"out0/{q}"], f32.z[f"out0/{q}"])
    for q in ("logits", "aux"):
        out["outputs"][q] = rel(f16.z[f"out0/{q}"], f32.z[f"out0/{q}"])
    for k in f32.meta["grad_keys"]:
        i16, r16 = _exact_subset(f16, f"grad0/{k}")
        i32, r32 = _exact_subset(f32, f"grad0/{k}")
        assert (i16 is None) == (i32 is None) and (i16 is None or np.array_equal(i16, i32)), k
        out["grads"][k] = rel(r16, r32)
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    g = np.array(list(out["grads"].values()))
    print(f"wrote {OUT}: logits {out['outputs']['logits']:.3e}, loss {out['scalars']['loss']:.3e}, gnorm "
          f"{out['scalars']['gnorm']:.3e}; grads median {np.median(g):.3e}, min {g.min():.3e}, max {g.max():.3e}")


if __name__ == "__main__":
    main()
