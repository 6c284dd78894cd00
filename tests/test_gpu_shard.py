"""Row-sharded embedding tables (tossctr/shard.py, csrc/shard.hip) vs replicated tables, world 2.

Each configuration runs as a child process (tests/dist_shard_worker.py) whose two ranks share cuda:0
over gloo.  Checks:
  * world 2 with the SAME batch on both ranks = the single-GPU run (DDP mean of equal grads);
  * sharded = replicated with DIFFERENT batches per rank: losses, eval logits, every parameter (full
    tables gathered from the shards) and the EMA shadow -- equal up to the summation order of the
    global grad norm (per-owner partial sums vs one sum);
  * sharded lazy = sharded dense optimizer stream, bit for bit;
  * each rank holds ceil(vocab / 2) rows of a sequence table.
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from golden_util import close_enough

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
_cache = {}


def _run(tmp_path_factory, mode, same, lazy=1, steps=4, config="tiny", nccl=0, prefetch=1, sync_check=0,
         interleave=0, short_last=0, autograd=0):
    key = (mode, same, lazy, steps, config, nccl, prefetch, sync_check, interleave, short_last, autograd)
    if key not in _cache:
        out = str(tmp_path_factory.mktemp("shard") / ("_".join(map(str, key)) + ".pt"))
        r = subprocess.run([sys.executable, os.path.join(HERE, "dist_shard_worker.py"), "--mode", mode,
                            "--same-batch", str(same), "--lazy", str(lazy), "--steps", str(steps), "--config", config,
                            "--nccl", str(nccl), "--prefetch", str(prefetch), "--sync-check", str(sync_check),
                            "--interleave-eval", str(interleave), "--short-last", str(short_last), "--autograd", str(autograd),
                            "--out", out], capture_output=True, text=True, timeout=250)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        if config in ("tiny", "cfg5w"):
            _cache[key] = torch.load(out, weights_only=True)
        else:
            ranks = 1 if mode == "single" else 2
            _cache[key] = [torch.load(f"{out}.rank{r}", weights_only=True) for r in range(ranks)]
    return _cache[key]


def _compare(a, b, rtol, atol=1e-6, what=""):
    close_enough(np.asarray(a["losses"], np.float64), np.asarray(b["losses"], np.float64), rtol, atol, what + "loss")
    # the eval logits after the last step, at rtol -- unless the evaluation's DARE top-K put two candidates in a
    # different slot order.  The runs' parameters agree to ~1e-8 (the clip norm's cross-rank summation order moves
    # the clip coefficient by an ulp), so the selection scores agree to a few fp32 ulps; two candidates of one sample
    # whose scores tie to that precision can swap slots (measured, tools/shard_logit_diag.py: scores -1.0807130 /
    # -1.0807132 at positions 28 / 31, the tiny config after 4 steps).  The encoder sees the slot order (its
    # positional bias), so that sample's logit moves (9.8e-4), and the SE gate's batch mean carries a share of it to
    # every other sample (~2e-5).  Every slot-order difference must be such a tie (the same positions, scores within
    # 8 ulps); only then are the logits held to 1e-3.
    ia, ib = a["eval_idx"].numpy(), b["eval_idx"].numpy()
    flip = ~(ia == ib).all(1)
    lt = rtol
    if flip.any():
        va = a["eval_vals"].numpy()
        for i in np.where(flip)[0]:
            d = ia[i] != ib[i]
            assert sorted(ia[i][d]) == sorted(ib[i][d]), (what, i, ia[i], ib[i])
            sc = va[i][d]
            assert sc.max() - sc.min() <= 8 * np.spacing(np.float32(np.abs(sc).max())), (what, i, sc)
        lt = max(rtol, 1e-3)
    close_enough(a["logits"].double().numpy(), b["logits"].double().numpy(), lt, atol, what + "logits")
    assert a["sd"].keys() == b["sd"].keys()
    for k in a["sd"]:
        assert a["sd"][k].shape == b["sd"][k].shape, k
        # the MHA key bias's exact gradient is 0 (softmax shift invariance): what it receives is rounding
        # noise that AdamW normalises into lr-sized steps, so any change of summation order anywhere (e.g.
        # the clip norm's cross-rank sum) moves it -- compared at the north-star 1e-4 instead
        rt = max(rtol, 1e-4) if k.endswith("mha.in_proj_bias") else rtol
        close_enough(a["sd"][k].double().numpy().ravel(), b["sd"][k].double().numpy().ravel(), rt, atol, what + k)
        close_enough(a["ema"][k].double().numpy().ravel(), b["ema"][k].double().numpy().ravel(), rt, atol,
                     what + "ema:" + k)


def test_world2_same_batch_matches_single(tmp_path_factory):
    single = _run(tmp_path_factory, "single", 1)
    rep = _run(tmp_path_factory, "replicated", 1)
    sh = _run(tmp_path_factory, "sharded", 1)
    _compare(rep, single, 1e-5, what="replicated vs single: ")
    _compare(sh, single, 1e-5, what="sharded vs single: ")


def test_sharded_matches_replicated(tmp_path_factory):
    rep = _run(tmp_path_factory, "replicated", 0)
    sh = _run(tmp_path_factory, "sharded", 0)
    assert sh["local_rows"] == (sh["vocab"] + 1) // 2 and rep["local_rows"] == rep["vocab"]
    _compare(sh, rep, 1e-5, what="sharded vs replicated: ")


def test_sharded_lazy_equals_dense_stream(tmp_path_factory):
    lazy = _run(tmp_path_factory, "sharded", 0, 1)
    dense = _run(tmp_path_factory, "sharded", 0, 0)
    assert lazy["losses"] == dense["losses"]
    for k in lazy["sd"]:
        assert torch.equal(lazy["sd"][k], dense["sd"][k]), k
        assert torch.equal(lazy["ema"][k], dense["ema"][k]), k


@pytest.mark.parametrize("mode,config", [("replicated", "tiny"), ("sharded", "tiny"), ("sharded", "cfg5w")])
def test_data_parallel_step_matches_oracle(tmp_path_factory, mode, config):
    """world 2 with a different batch per rank against the CPU restatement applied per
    replica (oracle.model.TrainState.step_data_parallel: each rank's grads on its own batch -- its own SE
    batch mean and loss class counts -- averaged as DDP does, then one clip -> AdamW -> EMA).  After one
    step from zero moments m = (1 - b1) * clip_coef * mean grad and v = (1 - b2) (clip_coef * mean grad)^2,
    so both moments pin the averaged gradient of every parameter, tables included (rows routed to and
    merged on their owners when sharded); checked norm-wise at 2e-4 / 4e-4 (moment tolerances,
    golden_util.Fixture.check_moment).  The update pT - p0 is checked norm-wise at 1e-4 (+ 2 fp32 ulps)
    on the elements whose AdamW step is well conditioned (sqrt(v_hat) >= 100 eps), and everywhere
    elementwise within one lr.

    config "cfg5w": BASELINE config 5's widths through the row-sharded exchange (D = 64, the yaml's 35 d_c,
    K = 100, S1, 3 layers, 82 + 82 features; small tables), from the reference's own init at the yaml's lr 3e-4
    (tests/dist_shard_worker.py)."""
    from golden_util import to_torch_batch
    from oracle.model import TrainState, make_arch
    from oracle.synth import make_batch, make_params, reference_init
    res = _run(tmp_path_factory, mode, 0, steps=1, config=config)
    cards = res["cards"]
    cols = list(cards)
    vocab = res["vocab"]
    A = make_arch(res["cfg"], vocab, res["Fn"], res["Fm"], cards, cols)
    P0 = reference_init(A, 5) if res["init"] == "reference" else make_params(A.param_shapes(), 5, A.pad_id)
    P0 = {k: torch.from_numpy(v) for k, v in P0.items()}
    lr = res["lr0"]
    st = TrainState(P0, A, lr, 0.05, res["clip"], ema_cfg={"enabled": True, "decay": 0.9})
    bs = [make_batch(res["B"], res["Fn"], res["Fm"], list(cards.values()), res["L"], vocab, seed=1000 + 100 * r)
          for r in range(2)]
    losses, _, gnorm = st.step_data_parallel([to_torch_batch(b) for b in bs],
                                             [torch.from_numpy(b["y"]).float() for b in bs], lr, [(9 << 32)] * 2)
    assert abs(res["losses"][0] - float(losses[0])) <= 1e-5 * max(1.0, abs(float(losses[0])))
    assert abs(res["gnorm"] - float(gnorm)) <= 1e-4 * float(gnorm), (res["gnorm"], float(gnorm))
    for k in st.grad_keys:
        close_enough(res["m"][k].double().numpy().ravel(), st.m[k].double().numpy().ravel(), 2e-4, 0.0, f"{mode} m:{k}")
        close_enough(res["v"][k].double().numpy().ravel(), st.v[k].double().numpy().ravel(), 4e-4, 0.0, f"{mode} v:{k}")
    for k in P0:
        p0 = P0[k].double().numpy().ravel()
        got = res["sd"][k].double().numpy().ravel() - p0
        ref = st.P[k].detach().double().numpy().ravel() - p0
        assert np.abs(got - ref).max(initial=0) <= lr, k
        if k in st.grad_keys:
            good = np.sqrt(st.v[k].double().numpy().ravel() / (1 - 0.999)) >= 100 * 1e-8
            ulp = 2.0 * np.spacing(np.abs(p0 + ref).astype(np.float32)).astype(np.float64)
            close_enough(got[good], ref[good], 1e-4, 0.0, f"{mode} dp:{k}", ulp[good], elem_rtol=1e-2)
        ge = res["ema"][k].double().numpy().ravel() - p0
        re = st.shadow[k].double().numpy().ravel() - p0
        assert np.abs(ge - re).max(initial=0) <= 0.1 * lr + 1e-6, k


def test_cfg5_reduced_sharded_matches_single(tmp_path_factory):
    """BASELINE config 5 at reduced scale (tests/dist_shard_worker.py --config cfg5r: D = 64, the yaml's
    d_c, 35 hashed tables of 4M rows + the 10M-row DARE tables, 28-bit owner-major keys at world 2):
    two row-sharded ranks on the same batch = the single-GPU step, over two steps -- every touched row's
    parameters, both moments and EMA shadow (gathered from their owners) and every dense parameter."""
    single = _run(tmp_path_factory, "single", 1, steps=2, config="cfg5r")[0]
    shards = _run(tmp_path_factory, "sharded", 1, steps=2, config="cfg5r")
    close_enough(np.asarray(shards[0]["losses"]), np.asarray(single["losses"]), 1e-5, 1e-6, "cfg5r loss")
    lr = 3e-3

    def cmp(got, ref, label):
        """m, v: norm-wise + elementwise 1e-5 -- they pin each step's routed / merged gradient.  p, EMA:
        norm-wise 1e-5 (+ 2 ulp) and elementwise within one lr: the global-norm summation order differs
        (per-owner partials), which moves the clip coefficient by an ulp, and AdamW amplifies that where a
        step's sqrt(v_hat) is near eps (that can be step 1 of an element whose final v is large)."""
        g = {n: got[n].double().numpy().ravel() for n in ("p", "m", "v", "e")}
        r = {n: ref[n].double().numpy().ravel() for n in ("p", "m", "v", "e")}
        rt = 1e-4 if label.endswith("mha.in_proj_bias") else 1e-5
        close_enough(g["m"], r["m"], rt, 0.0, f"cfg5r m:{label}")
        close_enough(g["v"], r["v"], 2 * rt, 0.0, f"cfg5r v:{label}")
        for n in ("p", "e"):
            assert np.abs(g[n] - r[n]).max(initial=0) <= lr, (label, n)
            ulp = 2.0 * np.spacing(np.abs(r[n]).astype(np.float32)).astype(np.float64)
            err, nrm = np.linalg.norm(g[n] - r[n]), np.linalg.norm(r[n])
            assert err <= rt * nrm + np.linalg.norm(ulp), (label, n, err / nrm)

    for k, d in single["dense"].items():
        if float(d["v"].abs().max()) == 0.0:          # no gradient (e.g. ctx_mlp in S1 mode): p, e only
            for n in ("p", "e"):
                close_enough(shards[0]["dense"][k][n].double().numpy().ravel(), d[n].double().numpy().ravel(),
                             1e-6, 0.0, f"cfg5r {n}:{k}")
            continue
        cmp(shards[0]["dense"][k], d, k)
    for k, d in single["rows"].items():
        ids = np.concatenate([s["rows"][k]["ids"].numpy() for s in shards])
        order = np.argsort(ids)
        assert np.array_equal(ids[order], d["ids"].numpy()), k
        got = {n: torch.cat([s["rows"][k][n] for s in shards])[torch.from_numpy(order)] for n in ("p", "m", "v", "e")}
        cmp(got, d, k)


@pytest.mark.parametrize("mode", ["replicated", "sharded"])
def test_rccl_world1_equals_single(tmp_path_factory, mode):
    """The RCCL (nccl backend) code path on one card: world 1 over RCCL -- the head bucket's all-reduce
    started mid-backward on the process group's stream and waited for before the clip, the sharded
    exchange's all-to-alls -- gives the single-process step: bitwise with replicated tables (a world-1
    sum is the identity); sharded sums the clip norm's table partials separately (1e-5, as above)."""
    single = _run(tmp_path_factory, "single", 1)
    got = _run(tmp_path_factory, mode, 1, nccl=1)
    if mode == "sharded":
        _compare(got, single, 1e-5, what="RCCL world-1 sharded vs single: ")
        return
    assert got["losses"] == single["losses"]
    for k in single["sd"]:
        assert torch.equal(got["sd"][k], single["sd"][k]), k
        assert torch.equal(got["ema"][k], single["ema"][k]), k


@pytest.mark.parametrize("interleave", [0, 1], ids=["prefetched", "eval_in_between"])
def test_sharded_prefetch_equals_in_place_plan(tmp_path_factory, interleave):
    """The next batch's exchange planned beside the step (a plan stream, two plan slots) = planned in place at
    the step's fetch: bit for bit, world 2 with different batches per rank.  The worker asserts that every
    step after the first consumed its prefetched plan (TableShards.prefetch_hits), so the overlap is really
    exercised.  ``eval_in_between``: an evaluation forward between step 1 and step 2 fetches another batch, so
    the plan made for step 2 is dropped (ordered behind on the fetching stream) and step 2 plans in place --
    still the same bits, and exactly one miss."""
    pre = _run(tmp_path_factory, "sharded", 0, interleave=interleave)
    inplace = _run(tmp_path_factory, "sharded", 0, prefetch=0)
    assert pre["losses"] == inplace["losses"]
    for k in pre["sd"]:
        assert torch.equal(pre["sd"][k], inplace["sd"][k]), k
        assert torch.equal(pre["ema"][k], inplace["ema"][k]), k


@pytest.mark.parametrize("mode", ["replicated", "sharded"])
def test_short_last_step_matches_single(tmp_path_factory, mode):
    """An epoch's short last step (tossctr.train.rank_slice: a rank without rows): world 2 on the same batches,
    where on the last step rank 1 runs train_step(contribute=False) and both ranks average over
    contributors=1 -- equal to the single-GPU run of the same batches (1e-5: the clip norm's cross-rank sum)."""
    single = _run(tmp_path_factory, "single", 1)
    got = _run(tmp_path_factory, mode, 1, short_last=1)
    _compare(got, single, 1e-5, what=f"{mode} short last step vs single: ")


def test_rccl_sharded_step_never_blocks_the_host(tmp_path_factory):
    """The row-sharded step over RCCL issues without a host synchronisation: steps 2-5 of a world-1 run run
    under torch.cuda.set_sync_debug_mode("error") (the exchange sizes come from counts planned beside the
    previous step, read from pinned memory), and the run still equals the single-GPU one."""
    single = _run(tmp_path_factory, "single", 1, steps=6)
    got = _run(tmp_path_factory, "sharded", 1, steps=6, nccl=1, sync_check=1)
    _compare(got, single, 1e-5, what="RCCL world-1 sharded (sync-checked) vs single: ")


def test_sharded_autograd_loop_matches_fused_step(tmp_path_factory):
    """The reference loop (src/train.py:185-195) on row-sharded tables, world 2, different batches per rank:
    ``model(batch)``, ``loss.backward()`` -- collective: the dense grads averaged over the ranks, every table row
    grad sent to its owner and averaged, a table's ``.grad`` its local shard's -- ``model.clip_grad_norm_`` (the
    global norm, FSDP-style) and ``torch.optim.AdamW`` on the local parameters.  It must land where the fused
    sharded step does (``train_step``: the same DDP mean, global clip and AdamW; FusedAdamW's hardware sqrt /
    reciprocal differ from torch's by a few ulp of the update term): losses, and every parameter with the full
    tables gathered from the shards, after 4 steps."""
    a = _run(tmp_path_factory, "sharded", 0, autograd=1)
    b = _run(tmp_path_factory, "sharded", 0)
    # the optimizer step's replica check ran after every backward (and found the dense grads identical)
    assert a["replica_checks"] == 4, a["replica_checks"]
    close_enough(np.asarray(a["losses"], np.float64), np.asarray(b["losses"], np.float64), 1e-5, 1e-6, "loss")
    assert a["sd"].keys() == b["sd"].keys()
    for k in a["sd"]:
        assert a["sd"][k].shape == b["sd"][k].shape, k
        close_enough(a["sd"][k].double().numpy().ravel(), b["sd"][k].double().numpy().ravel(), 1e-4, 1e-6, k)


def test_sharded_autograd_fused_optimizer_matches_fused_step(tmp_path_factory):
    """``loss.backward()`` followed by ``FusedAdamW.step()`` on row-sharded tables (world 2, different batches per
    rank): the backward leaves the table grads compact (``.grad`` None), ``step()`` all-reduces the dense grads,
    routes the row grads to their owners and clips on the global norm -- it must land where ``train_step`` does
    (the loss gradient comes from torch's autograd of the loss instead of the fused loss kernel: ulps)."""
    a = _run(tmp_path_factory, "sharded", 0, autograd=3)
    b = _run(tmp_path_factory, "sharded", 0)
    close_enough(np.asarray(a["losses"], np.float64), np.asarray(b["losses"], np.float64), 1e-5, 1e-6, "loss")
    for k in b["sd"]:
        # as the torch.optim loop above (1e-4: the MHA key bias's exact gradient is 0, so its rounding noise takes
        # +-lr AdamW steps of either sign; its moments are left out of the comparison)
        close_enough(a["sd"][k].double().numpy().ravel(), b["sd"][k].double().numpy().ravel(), 1e-4, 1e-6, k)
        ma, mb = a["m"][k].double().numpy().ravel(), b["m"][k].double().numpy().ravel()
        if k.endswith("mha.in_proj_bias"):
            D = ma.size // 3
            ma, mb = np.delete(ma, np.s_[D:2 * D]), np.delete(mb, np.s_[D:2 * D])
        close_enough(ma, mb, 1e-4, 1e-9, "m:" + k)


def test_sharded_autograd_reference_clip_is_refused(tmp_path_factory):
    """The reference's own ``nn.utils.clip_grad_norm_(model.parameters(), clip)`` on row-sharded tables takes each
    rank's LOCAL shard norm, so the ranks would scale their replicated dense grads differently and drift apart;
    the optimizer step after such a backward raises on every rank (the check is collective) at the first step."""
    out = str(tmp_path_factory.mktemp("shard") / "refclip.pt")
    r = subprocess.run([sys.executable, os.path.join(HERE, "dist_shard_worker.py"), "--mode", "sharded",
                        "--same-batch", "0", "--steps", "2", "--autograd", "2", "--out", out],
                       capture_output=True, text=True, timeout=250)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    for rank in range(2):
        with open(f"{out}.raised{rank}") as fh:
            msg = fh.read()
        assert "model.clip_grad_norm_" in msg, (rank, msg)
