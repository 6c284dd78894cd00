"""Where does the world-2 same-batch sharded-vs-single eval-logit gap come from (tests/test_gpu_shard.py::_compare)?

Runs tests/dist_shard_worker.py (single, replicated, sharded; same batch on both ranks; tiny fp32 config) for 1..4
steps and prints, per run length: the eval logits' norm-wise gap, the samples whose logits differ most with
whether their DARE top-K selections (tokens) agree, and the parameters with the largest relative gaps.

    python tools/shard_logit_diag.py [--steps 4] [--out gpurun_out/shard_diag]
"""
import argparse
import os
import subprocess
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(REPO, "tests", "dist_shard_worker.py")


def run(mode, steps, out, *extra):
    path = os.path.join(out, f"{mode}_{steps}{'_'.join(extra)}.pt")
    r = subprocess.run([sys.executable, WORKER, "--mode", mode, "--same-batch", "1", "--steps", str(steps), "--out",
                        path, *extra], capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        print(r.stdout[-2000:], r.stderr[-2000:])
        raise SystemExit(r.returncode)
    if "--eval-check" in extra:
        print(r.stdout[-3000:])
    return torch.load(path, weights_only=True)


def oracle_swap(got, single, mode):
    """The eval forward of the CPU oracle (fp32) on each run's final parameters: is the logit gap a property of the
    parameters, and which ones?  Parameters of the sharded run are swapped for the single run's one group at a time."""
    sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "toss-next-ctr-prediction_amd")]
    from golden_util import to_torch_batch
    from oracle.model import Dropper, forward, make_arch
    from oracle.synth import make_batch
    cards = single["cards"]
    A = make_arch(single["cfg"], single["vocab"], single["Fn"], single["Fm"], cards, list(cards))
    eb = to_torch_batch(make_batch(single["B"], single["Fn"], single["Fm"], list(cards.values()), single["L"],
                                   single["vocab"], seed=4242))

    def ev(sd):
        with torch.no_grad():
            return forward({k: v.float() for k, v in sd.items()}, eb, A, Dropper(0, training=False))[0].double().numpy()

    z1, z2 = ev(single["sd"]), ev(got["sd"])
    n = np.linalg.norm
    print(f"    oracle eval: single-params vs {mode}-params gap {n(z2 - z1) / n(z1):.3e}; GPU single vs oracle single "
          f"{n(single['logits'].double().numpy() - z1) / n(z1):.3e}; GPU {mode} vs oracle {mode} "
          f"{n(got['logits'].double().numpy() - z2) / n(z2):.3e}")
    D = A.D
    for label, keys, sl in (("in_proj_bias q", "mha.in_proj_bias", slice(0, D)),
                            ("in_proj_bias k", "mha.in_proj_bias", slice(D, 2 * D)),
                            ("in_proj_bias v", "mha.in_proj_bias", slice(2 * D, 3 * D)),
                            ("all in_proj_bias", "mha.in_proj_bias", slice(None)),
                            ("everything but in_proj_bias", None, None)):
        sd = {k: v.clone() for k, v in got["sd"].items()}
        for k in sd:
            if keys is None:
                if not k.endswith("mha.in_proj_bias"):
                    sd[k] = single["sd"][k].clone()
            elif k.endswith(keys):
                sd[k][sl] = single["sd"][k][sl]
        z = ev(sd)
        print(f"    swap {label:28s}: gap to single {n(z - z1) / n(z1):.3e}")
    for k, v in got["sd"].items():
        if k.endswith("mha.in_proj_bias"):
            d = (v - single["sd"][k]).double()
            print(f"    {k}: max |diff| q {float(d[:D].abs().max()):.2e} k {float(d[D:2 * D].abs().max()):.2e} "
                  f"v {float(d[2 * D:].abs().max()):.2e}; |b_k| max {float(v[D:2 * D].abs().max()):.2e}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--out", default="/tmp/shard_diag")
    ap.add_argument("--quick", action="store_true", help="only the last run length")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    for steps in range(args.steps if args.quick else 1, args.steps + 1):
        single = run("single", steps, args.out)
        for mode in ("replicated", "sharded"):
            got = run(mode, steps, args.out)
            za, zb = got["logits"].double().numpy(), single["logits"].double().numpy()
            gap = np.linalg.norm(za - zb) / np.linalg.norm(zb)
            # sharded top-K rows carry fetched-row ids (1 + unique index), not tokens: compare the selected scores
            same = (np.sort(got["eval_vals"].numpy(), 1) == np.sort(single["eval_vals"].numpy(), 1)).all(1)
            samegap = np.linalg.norm((za - zb)[same]) / np.linalg.norm(zb[same])
            print(f"steps {steps} {mode:10s}: logits gap {gap:.3e}; top-K differs on {int((~same).sum())} of "
                  f"{len(same)} samples; gap over the agreeing samples {samegap:.3e}; losses "
                  f"{np.max(np.abs(np.array(got['losses']) - np.array(single['losses']))):.3e}")
            ia, ib = got["eval_idx"].numpy(), single["eval_idx"].numpy()
            same_idx = (ia == ib).all(1)
            print(f"    top-K positions differ (in slot order) on {int((~same_idx).sum())} samples; logits gap over the "
                  f"others {np.linalg.norm((za - zb)[same_idx]) / np.linalg.norm(zb[same_idx]):.3e}")
            for i in np.where(~same_idx)[0][:6]:
                k = int(np.argmax(ia[i] != ib[i]))
                va = single["eval_vals"][i].numpy()
                print(f"      sample {i}: first differing slot {k}: positions {ia[i][k:k + 2]} vs {ib[i][k:k + 2]}, scores "
                      f"{va[k]:.7f} {va[k + 1] if k + 1 < len(va) else float('nan'):.7f}; |dz| {abs(za[i] - zb[i]):.3e}")
            d = np.abs(za - zb)
            for i in np.argsort(-d)[:3]:
                va, vb = got["eval_vals"][i].numpy(), single["eval_vals"][i].numpy()
                print(f"    sample {i}: |dz| {d[i]:.3e} (z {zb[i]:+.4f}), top-K same {bool(same[i])}, "
                      f"max |d score| {np.abs(np.sort(va) - np.sort(vb)).max():.3e}")
            worst = []
            for k in single["sd"]:
                a, b = got["sd"][k].double().numpy().ravel(), single["sd"][k].double().numpy().ravel()
                worst.append((np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30), k))
            worst.sort(reverse=True)
            print("    params: " + ", ".join(f"{k} {r:.2e}" for r, k in worst[:4]))
            if steps == args.steps:
                oracle_swap(got, single, mode)
    # the evaluation forwards' workspaces, buffer by buffer in allocation (= forward) order: the first that differs
    a = run("single", args.steps, args.out, "--dump-ws", "1")
    b = run("sharded", args.steps, args.out, "--dump-ws", "1")
    wa = torch.load(os.path.join(args.out, f"single_{args.steps}--dump-ws_1.pt.ws"), weights_only=True)
    wb = torch.load(os.path.join(args.out, f"sharded_{args.steps}--dump-ws_1.pt.ws"), weights_only=True)
    for k, va in wa.items():
        vb = wb.get(k)
        if vb is None or vb.shape != va.shape or not va.is_floating_point():
            continue
        d = float((va.double() - vb.double()).abs().max())
        print(f"    ws {k:16s} {tuple(va.shape)}: max |single - sharded| {d:.3e}")
    del a, b
    # the sharded run's evaluation with the dense optimizer stream / with every row flushed before it
    for extra in (("--lazy", "0"), ("--sync-eval", "1"), ("--eval-check", "1")):
        got = run("sharded", args.steps, args.out, *extra)
        za, zb = got["logits"].double().numpy(), single["logits"].double().numpy()
        print(f"steps {args.steps} sharded {' '.join(extra)}: eval logits gap to single "
              f"{np.linalg.norm(za - zb) / np.linalg.norm(zb):.3e}")


if __name__ == "__main__":
    main()
