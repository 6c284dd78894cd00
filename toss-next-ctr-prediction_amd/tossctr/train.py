"""K-fold training loop -- drop-in for src/train.py (``main(cfg_path)``, ``train_one_fold``) on MI355X.

Same control flow as the reference (src/train.py:92-366): StratifiedGroupKFold(max(5, n_splits)),
fold-level resume (skip a fold whose ckpt exists), per-step lr = cosine_warmup_lr, the step
forward -> bce_wll_style (+aux_w * aux) -> backward -> clip -> AdamW -> EMA, per-epoch validation with
EMA weights, AP/WLL/Score, temperature calibration, early stopping, ``torch.save({"state", "score"})``.

MI355X differences (same results, different mechanics):
  * batches come from HBM-resident shards (data.DeviceShards) gathered by the fold's permuted index,
    not DataLoader worker processes;
  * the step is the fused device step (CTRModel.train_step + optim.FusedAdamW): no per-step host
    sync -- the reference's ``float(loss.cpu())`` each step (src/train.py:202) becomes an on-device sum;
  * ``best_state["model"]`` is a detached copy (the reference stores live references, so its "best"
    checkpoint is really the last epoch's weights);
  * optional data parallelism: run under torchrun, every rank takes its own stride of each epoch's
    permutation; dense grads are all-reduced and the embedding tables row-sharded over the ranks
    (tossctr/shard.py; ``dist: {shard_tables: false}`` in the yaml keeps them replicated); validation
    batches are spread over the ranks and their logits all-gathered;
  * or fold parallelism (``dist: {mode: folds}``): rank r trains folds r, r + W, ... of the
    same StratifiedGroupKFold split, each exactly as a single-GPU run would (no collective while training),
    and writes those folds' checkpoints; the scores are gathered once at the end.
"""
from __future__ import annotations

import argparse
import copy
import gc
import json
import math
import os

import numpy as np
import torch


def cosine_warmup_lr(epoch, step, steps_per_epoch, base_lr, warmup_epochs=1, total_epochs=10):
    """Per-step linear warmup then cosine decay (src/utils/sched.py:3-11)."""
    gstep = epoch * steps_per_epoch + step
    warmup_steps = warmup_epochs * steps_per_epoch
    total_steps = total_epochs * steps_per_epoch
    if gstep < warmup_steps:
        return base_lr * (gstep + 1) / max(1, warmup_steps)
    progress = (gstep - warmup_steps) / max(1, total_steps - warmup_steps)
    return 0.5 * base_lr * (1.0 + math.cos(math.pi * progress))


def set_seed(seed: int, deterministic: bool = True):
    """src/utils/seed.py:3-17 (the HIP kernels are deterministic by construction)."""
    import random
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def check_supported(cfg):
    """Refuse configuration the fused path does not implement instead of silently training something
    else: ``sampler.type: balanced`` (src/train.py:95-106; no reference yaml enables it) and an ``amp``
    mode other than none/bf16 (fp16 + GradScaler, src/train.py:133-139,185-190)."""
    amp = str(cfg.get("amp", "none") or "none").lower()
    if amp not in ("none", "bf16"):
        raise NotImplementedError(f"amp: {cfg.get('amp')!r} -- the fused MI355X step runs fp32 or bf16 (amp: bf16)")
    if str((cfg.get("sampler", {}) or {}).get("type", "") or "").lower() == "balanced":
        raise NotImplementedError("sampler.type: balanced is not supported (no reference config enables it)")


_FOLD_LOCAL = False      # set by main() in fold-parallel mode: training runs with no process group


def _dist():
    import torch.distributed as dist
    if _FOLD_LOCAL:
        return None
    return dist if dist.is_available() and dist.is_initialized() else None


def fold_owner(fold: int, world: int) -> int:
    """Fold-parallel mode: the rank that trains ``fold`` (folds dealt round-robin over the ranks)."""
    return fold % world


def _cardinals(cfg, cat_cols):
    d = cfg["data"]
    return {c: int(d["hash_buckets"].get(c, 1000003)) + int(d.get("hash_buckets_margin", 0)) for c in cat_cols}


def _feature_dims(manifest_path):
    with open(manifest_path) as f:
        man = json.load(f)
    first = man["shards"][0]
    return (int(np.load(first["X_num"]["path"], mmap_mode="r").shape[1]),
            int(np.load(first["X_mask"]["path"], mmap_mode="r").shape[1]))


def _cal_state(cal):
    """The fitted calibrator as plain data (temperature, isotonic thresholds) for the checkpoint;
    tossctr.infer applies it on device."""
    out = {"method": cal.method, "temperature": None if cal.temperature is None else float(cal.temperature)}
    if cal.iso is not None:
        out["iso_x"] = [float(v) for v in cal.iso.X_thresholds_]
        out["iso_y"] = [float(v) for v in cal.iso.y_thresholds_]
    return out


@torch.no_grad()
def predict_logits(model, store, idx_np, bs, as_tensor=False):
    """Eval-mode forward over rows idx (src/train.py:211-225); returns logits (numpy, or the float32 device
    tensor with ``as_tensor``).

    The batches are the reference's (consecutive bs-row slices of idx, which matters: the SE gate uses
    the batch mean).  Data parallel: rank r runs batches r, r + world, ... and the logits are
    all-gathered, so every rank returns all of them; ranks short of a batch re-run their last one
    (row-sharded tables make every forward collective) and drop the result."""
    model.eval()
    dev = store.device
    dist = _dist()
    world = dist.get_world_size() if dist else 1
    rank = dist.get_rank() if dist else 0
    idx_all = torch.from_numpy(np.asarray(idx_np, dtype=np.int64)).to(dev)
    n = idx_all.numel()
    nb = (n + bs - 1) // bs
    if nb == 0:
        return torch.zeros(0, dtype=torch.float32, device=dev) if as_tensor else np.zeros(0, np.float32)
    per_rank = (nb + world - 1) // world
    mine = torch.zeros(per_rank * bs, dtype=torch.float32, device=dev)
    for i in range(per_rank):
        j = min(i * world + rank, nb - 1)
        sl = idx_all[j * bs:(j + 1) * bs]
        inputs, _ = store.batch(sl, slot=1)
        logits, _, _, _ = model.engine.forward(*inputs, training=False, seed=0, save=False)
        mine[i * bs:i * bs + sl.numel()] = logits
    if world == 1:
        return mine[:n] if as_tensor else mine[:n].cpu().numpy()
    from . import dist as D
    allr = torch.empty(world * per_rank * bs, dtype=torch.float32, device=dev)
    D.all_gather_into(allr, mine, dist.group.WORLD)
    out = allr.view(world, per_rank, bs).transpose(0, 1).reshape(-1)     # batch j = (i, r), j = i*world + r
    return out[:n].contiguous() if as_tensor else out[:n].cpu().numpy()


def release(model, opt, ema):
    """Break the model <-> optimizer / EMA reference cycle (model._fused_opt, opt.model, engine.lazy,
    shards.lazy, ema.model) so the fold's arena, moments and EMA shadow are freed when the last
    reference goes, not at some later gen-2 collection (src/train.py:280-316 _free_fold)."""
    model.__dict__.pop("_fused_opt", None)
    model.engine.lazy = None
    model.engine.grad_ready = None
    model.engine.last = None
    if model.shards is not None:
        model.shards.lazy = None
    if opt is not None:
        opt.model = opt.engine = opt.shards = None
    if ema is not None:
        ema.model = None


def rank_slice(n, bs, world, rank, step):
    """(start, rows) of rank ``rank``'s batch at ``step`` of an epoch over n permuted rows: every full
    step gives each rank bs consecutive rows (rank-major); the epoch's last, short step splits its
    remainder as evenly as possible (the first remainder % world ranks take one row more), so no row
    is seen twice in an epoch (single GPU: the reference's ceil(n / bs) batches, the last one short)."""
    g = bs * world
    lo = step * g
    rem = min(g, n - lo)
    if rem >= g:
        return lo + rank * bs, bs
    base, extra = divmod(max(0, rem), world)
    return lo + rank * base + min(rank, extra), base + (1 if rank < extra else 0)


def step_contributors(n, bs, world, step):
    """How many ranks hold rows at ``step`` (rank_slice): all of them except on a short last step with
    fewer rows than ranks.  The all-reduced gradient is averaged over these."""
    return max(1, min(world, n - step * bs * world))


def train_one_fold(cfg, fold, idx_tr, idx_va, manifest_path, logger, store=None, device=None):
    """src/train.py:92-317 (same signature + optional pre-staged ``store``). Returns (best_state, best_score)."""
    from .configs import cat_cardinals  # noqa: F401
    from .data import DeviceShards
    from .metrics import Calibrator, DeviceMetrics, final_score
    from .optim import FusedAdamW, build_ema
    from .wrapper import CTRModel
    dist = _dist()
    world = dist.get_world_size() if dist else 1
    rank = dist.get_rank() if dist else 0
    device = device or torch.device("cuda", torch.cuda.current_device())
    check_supported(cfg)
    bs, epochs, warmup = cfg["train"]["batch_size"], cfg["train"]["epochs"], cfg["train"]["warmup_epochs"]
    cat_cols = cfg["data"]["cat_cols"]
    store = store or DeviceShards(manifest_path, device)
    seq_vocab = int(cfg.get("seq_vocab", 10_000_000))              # src/train.py:116
    cards = _cardinals(cfg, cat_cols)
    n_num, n_mask = _feature_dims(manifest_path)
    # data parallel: embedding tables row-sharded over the ranks unless dist.shard_tables is false
    shard = bool(dist) and world > 1 and bool(cfg.get("dist", {}).get("shard_tables", True))
    model = CTRModel(cfg, seq_vocab, n_num, n_mask, cards, cat_cols, device=device,
                     process_group=dist.group.WORLD if dist else None, shard_tables=shard)
    model.reset_parameters(torch.Generator(device=device).manual_seed(int(cfg.get("seed", 777)) + fold))
    ema = build_ema(model, cfg)
    opt = FusedAdamW(model, lr=cfg["train"]["lr"], weight_decay=cfg["train"]["weight_decay"],
                     max_grad_norm=cfg["train"].get("grad_clip_norm", 0.0), ema=ema,
                     process_group=dist.group.WORLD if dist else None)
    y_host = store.t["y"].view(-1).cpu().numpy()
    idx_tr = np.asarray(idx_tr, dtype=np.int64)
    steps_per_epoch = math.ceil(len(idx_tr) / (bs * world))
    gen = torch.Generator(device=device).manual_seed(int(cfg.get("seed", 777)) * 1000 + fold)
    idx_tr_dev = torch.from_numpy(idx_tr).to(device)
    global_step, best_score, best_state, wait = 0, -1e9, None, 0
    dmet = DeviceMetrics(device)
    for epoch in range(1, epochs + 1):
        model.train()
        perm = idx_tr_dev[torch.randperm(len(idx_tr), generator=gen, device=device)]
        loss_sum = torch.zeros((), device=device)
        def batch_at(step):
            lo, n_rows = rank_slice(len(idx_tr), bs, world, rank, step)
            # a rank left without rows on the last step still joins the step's collectives with one
            # row whose loss gradient is zeroed: it adds nothing to the averaged gradient
            idx = perm[lo:lo + n_rows] if n_rows else perm[:1]
            # row-sharded tables: batches alternate between two gather slots so the next one can be staged
            # (and its exchange planned, tossctr/shard.py) while this step runs
            return store.batch(idx, slot=step % 2 if shard else 0), n_rows

        nxt = batch_at(0) if shard else None
        for step in range(steps_per_epoch):
            global_step += 1
            (inputs, y), n_rows = nxt if nxt is not None else batch_at(step)
            nxt = batch_at(step + 1) if shard and step + 1 < steps_per_epoch else None
            opt.param_groups[0]["lr"] = cosine_warmup_lr(epoch - 1, step, steps_per_epoch, cfg["train"]["lr"], warmup,
                                                         epochs)
            # DDP semantics per replica: the mean of the per-rank gradients over the ranks that
            # hold rows -- on the short last step a rank without rows does not dilute the average
            n_contrib = step_contributors(len(idx_tr), bs, world, step)
            loss_sum += model.train_step(inputs, y, opt, global_step=global_step, contribute=n_rows > 0,
                                         contributors=n_contrib if n_contrib < world else None,
                                         next_inputs=nxt[0][0] if nxt is not None else None)[0]
        tr_loss = float(loss_sum.item()) / max(1, steps_per_epoch)
        use_ema_eval = ema is not None and cfg["ema"].get("eval_with_ema", True)
        if use_ema_eval:
            ema.store(model)
            ema.copy_to(model)
        # validation metrics and the temperature fit on device (csrc/metrics.hip): the logits stay in HBM
        z_dev = predict_logits(model, store, idx_va, bs, as_tensor=True)
        y_true = y_host[np.asarray(idx_va, dtype=np.int64)].astype(np.int64)
        y_dev = torch.from_numpy(y_true.astype(np.float32)).to(device)
        ap, wll, score = dmet.final_score(z_dev, y_dev)
        cal, score_cal = None, None
        if cfg.get("calibration", {}).get("enabled", False):
            cc = cfg["calibration"]
            z_raw = z_dev.cpu().numpy()
            cal = Calibrator(method=cc.get("method", "temperature"), lr=float(cc.get("lr", 0.05)),
                             iters=int(cc.get("iters", 200))).fit(z_raw, y_true, device_metrics=dmet,
                                                                  z_dev=z_dev, y_dev=y_dev)
            if cal.iso is None:
                # predict_proba clips even when neither a temperature nor an isotonic map was fitted
                # (isotonic fallback below min_iso_nodes): score the clipped path with T = 1 then
                T = cal.temperature if cal.temperature is not None else 1.0
                ap_cal, wll_cal, score_cal = dmet.final_score(z_dev, y_dev, T=T)
            else:                       # isotonic map: host (sklearn), as the reference
                ap_cal, wll_cal, score_cal = final_score(y_true, cal.predict_proba(z_raw))
        if rank == 0:
            K, tau = cfg["sequence"]["top_k"], cfg["sequence"]["recency_tau"]
            lr = opt.param_groups[0]["lr"]
            logger.row(fold=fold, epoch=epoch, split="val", loss=round(tr_loss, 6), AP=round(ap, 6),
                       WLL=round(wll, 6), Score=round(score, 6), lr=lr, bs=bs, K=K, tau=tau)
            logger.csv(fold=fold, epoch=epoch, split="val", loss=tr_loss, AP=ap, WLL=wll, Score=score, lr=lr, bs=bs,
                       K=K, tau=tau)
            logger.scalars(f"fold{fold}", epoch, train_loss=tr_loss, val_AP=ap, val_WLL=wll, val_Score=score)
            if score_cal is not None:
                logger.row(fold=fold, epoch=epoch, split="val_cal", loss="--", AP=round(ap_cal, 6),
                           WLL=round(wll_cal, 6), Score=round(score_cal, 6), lr=lr, bs=bs, K=K, tau=tau)
        if use_ema_eval:
            ema.restore(model)
        cur = score_cal if score_cal is not None else score
        if cur > best_score:
            best_score = cur
            best_state = {"model": {k: v.detach().cpu().clone() for k, v in model.state_dict().items()},
                          "cfg": cfg, "best_score": float(best_score), "epoch": int(epoch),
                          "calibrator": (_cal_state(cal) if cal else None),
                          "ema": (ema.state_dict() if ema is not None else None), "global_step": global_step}
            wait = 0
        else:
            wait += 1
            if wait >= cfg["train"]["early_stop_patience"]:
                break
    release(model, opt, ema)
    del model, opt, ema
    gc.collect()                    # src/train.py:312
    torch.cuda.empty_cache()
    return best_state, best_score


def main(cfg_path_or_dict):
    """src/train.py:319-352.  Under torchrun: data parallel within each fold (default), or fold parallel with
    ``dist: {mode: folds}`` (every rank trains its own folds, fold_owner)."""
    global _FOLD_LOCAL
    from sklearn.model_selection import StratifiedGroupKFold
    from .data import DeviceShards, load_labels_groups_for_split
    from .metrics import Logger
    if isinstance(cfg_path_or_dict, dict):
        cfg = copy.deepcopy(cfg_path_or_dict)
    else:
        import yaml
        with open(cfg_path_or_dict) as f:
            cfg = yaml.safe_load(f)
    os.makedirs(cfg["logging"]["log_dir"], exist_ok=True)
    set_seed(cfg["seed"], deterministic=cfg.get("deterministic", True))
    dist = _dist()
    rank = dist.get_rank() if dist else 0
    world = dist.get_world_size() if dist else 1
    mode = str((cfg.get("dist", {}) or {}).get("mode", "data")).lower()
    if mode not in ("data", "folds"):
        raise ValueError(f"dist.mode must be 'data' or 'folds', got {mode!r}")
    folds_mode = mode == "folds" and world > 1
    device = torch.device("cuda", torch.cuda.current_device())
    out_dir = os.path.join(cfg["logging"]["log_dir"], cfg["exp_name"])
    # fold parallel: every rank logs the folds it trains (rank > 0 to a CSV of its own: no shared appends)
    logger = Logger(out_dir, tb=cfg["logging"].get("tb", False), csv_log=cfg["logging"].get("csv_log", True),
                    quiet=rank != 0 and not folds_mode,
                    csv_name="train_log.csv" if rank == 0 or not folds_mode else f"train_log_rank{rank}.csv")
    manifest_path = cfg["data"]["manifest_train"]
    y, groups = load_labels_groups_for_split(manifest_path)
    n_splits = int(cfg["cv"]["n_splits"])
    sgkf = StratifiedGroupKFold(n_splits=max(5, n_splits), shuffle=True, random_state=cfg["seed"])
    store = DeviceShards(manifest_path, device)
    results = {}
    _FOLD_LOCAL = folds_mode
    try:
        for fold, (tr, va) in enumerate(sgkf.split(np.zeros_like(y), y, groups)):
            if n_splits == 1 and fold > 0:
                break
            if folds_mode and fold_owner(fold, world) != rank:
                continue
            ckpt = os.path.join(out_dir, f"ckpt_folds_{fold}.pt")
            if os.path.exists(ckpt):
                continue
            state, score = train_one_fold(cfg, fold, tr, va, manifest_path, logger, store=store, device=device)
            if rank == 0 or folds_mode:
                os.makedirs(out_dir, exist_ok=True)
                torch.save({"state": state, "score": float(score)}, ckpt)
            results[fold] = score
    finally:
        _FOLD_LOCAL = False
    if folds_mode:       # every rank returns every fold's score (the run's only collective)
        parts = [None] * world
        dist.all_gather_object(parts, {int(k): float(v) for k, v in results.items()})
        results = {k: v for p in parts for k, v in p.items()}
        results = dict(sorted(results.items()))
    return results


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", required=True)
    args = ap.parse_args()
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch.distributed as _d
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
        _d.init_process_group(os.environ.get("CTR_DIST_BACKEND", "nccl"))
    main(args.cfg)
