"""The K-fold loop (tossctr.train.main, drop-in for src/train.py) end to end on a tiny synthetic cache."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def tiny_run_cfg(tmp, man, query_mode="concat", qnn=True, tb=True, ema=True):
    cols = ["c0", "c1", "c2", "c3"]
    return {
        "exp_name": "tiny", "seed": 777, "device": "cuda", "seq_vocab": 3000,
        "data": {"cat_cols": cols, "hash_buckets": {c: 200 for c in cols}, "hash_buckets_margin": 3,
                 "manifest_train": man},
        "sequence": {"max_len": 24, "pad_id": 0, "top_k": 12, "recency_tau": 16, "query_mode": query_mode,
                     "query_key": "c1", "transformer_block": tb,
                     "tfm": {"n_layers": 2, "n_heads": 4, "mha_dropout": 0.1, "ffn_hidden": 32, "ffn_dropout": 0.1,
                             "norm": "rms", "gating": "softmax", "add_positional_bias": True}},
        "model": {"emb_dim": 16, "dare_dropout": 0.2, "cat_embedding_dims": {"c0": 8, "c1": 12, "c2": 4, "c3": 16},
                  "qnn_alpha": {"enabled": qnn, "feature_embed_dim": 8, "heads": 2, "rank": 4, "proj_dim": 16,
                                "mlp_hidden": [32, 16], "dropout": 0.2, "use_se": True, "se_reduction": 4,
                                "use_residual": True, "norm": "rms", "pair_grouping": "all", "aux_head_weight": 0.1}},
        "train": {"batch_size": 256, "epochs": 2, "lr": 1e-3, "weight_decay": 1e-4, "warmup_epochs": 1,
                  "early_stop_patience": 3, "grad_clip_norm": 0.5},
        "cv": {"n_splits": 1},
        "calibration": {"enabled": True, "method": "temperature", "lr": 0.05, "iters": 50},
        "logging": {"log_dir": os.path.join(tmp, "runs"), "tb": False, "csv_log": True},
        "ema": {"enabled": ema, "decay": 0.99, "eval_with_ema": True},
    }


@pytest.mark.parametrize("variant", ["qnn_concat", "fc_s1"])
def test_kfold_loop_end_to_end(tmp_path, variant):
    from tossctr import CTRModel
    from tossctr.data import synth_rows, write_shard_cache
    from tossctr.train import main
    arr = synth_rows(3000, 6, 6, [203, 203, 203, 203], 24, 3000, seed=5, pos_rate=0.2)
    man = write_shard_cache(str(tmp_path / "cache"), arr, shard_rows=1100, num_cols=[f"n{i}" for i in range(6)],
                            cat_cols=["c0", "c1", "c2", "c3"], group_key="c0")
    if variant == "qnn_concat":
        cfg = tiny_run_cfg(str(tmp_path), man)
    else:
        cfg = tiny_run_cfg(str(tmp_path), man, query_mode="S1", qnn=False, tb=False, ema=False)
    res = main(cfg)
    assert list(res) == [0] and np.isfinite(res[0])
    ckpt = os.path.join(cfg["logging"]["log_dir"], "tiny", "ckpt_folds_0.pt")
    assert os.path.exists(ckpt)
    st = torch.load(ckpt, weights_only=True)
    assert set(st) == {"state", "score"} and set(st["state"]) >= {"model", "cfg", "best_score", "epoch", "ema"}
    cards = {c: 203 for c in ["c0", "c1", "c2", "c3"]}
    m = CTRModel(cfg, 3000, 6, 6, cards, ["c0", "c1", "c2", "c3"], device="cuda:0")
    m.load_state_dict(st["state"]["model"], strict=True)
    csv_path = os.path.join(cfg["logging"]["log_dir"], "tiny", "train_log.csv")
    assert sum(1 for _ in open(csv_path)) >= 2
    # resume: a second main() skips the finished fold
    assert main(cfg) == {}


def test_kfold_loop_world2_sharded_tables(tmp_path):
    """main() under two ranks (gloo on one card, tables row-sharded): the checkpoint holds full tables,
    and its recorded validation score is what a single-GPU evaluation of those weights gives (the DP
    validation spreads batches over the ranks and all-gathers the logits)."""
    import json
    import subprocess
    import sys
    from sklearn.model_selection import StratifiedGroupKFold
    from tossctr import CTRModel
    from tossctr.data import DeviceShards, load_labels_groups_for_split, synth_rows, write_shard_cache
    from tossctr.metrics import final_score
    from tossctr.train import predict_logits
    cols = ["c0", "c1", "c2", "c3"]
    arr = synth_rows(3000, 6, 6, [203] * 4, 24, 3000, seed=6, pos_rate=0.2)
    man = write_shard_cache(str(tmp_path / "cache"), arr, shard_rows=1100, num_cols=[f"n{i}" for i in range(6)],
                            cat_cols=cols, group_key="c0")
    cfg = tiny_run_cfg(str(tmp_path), man, ema=False)
    cfg["calibration"]["enabled"] = False
    cfg["train"]["epochs"] = 1
    cfg_path, out = str(tmp_path / "cfg.json"), str(tmp_path / "res.json")
    with open(cfg_path, "w") as f:
        json.dump(cfg, f)
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "dist_train_worker.py"), cfg_path, out],
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    with open(out) as f:
        score = json.load(f)["0"]
    st = torch.load(os.path.join(cfg["logging"]["log_dir"], "tiny", "ckpt_folds_0.pt"), weights_only=True)
    assert st["state"]["model"]["dare.emb_att.weight"].shape == (3000, 16)
    m = CTRModel(cfg, 3000, 6, 6, {c: 203 for c in cols}, cols, device="cuda:0")
    m.load_state_dict(st["state"]["model"], strict=True)
    y, groups = load_labels_groups_for_split(man)
    _, va = next(StratifiedGroupKFold(n_splits=5, shuffle=True, random_state=cfg["seed"]).split(
        np.zeros_like(y), y, groups))
    store = DeviceShards(man, torch.device("cuda", 0))
    z = predict_logits(m, store, va, cfg["train"]["batch_size"])
    _, _, ref = final_score(y[va].astype(np.int64), 1.0 / (1.0 + np.exp(-z.astype(np.float64))))
    assert abs(ref - score) < 1e-6 * max(1.0, abs(ref)), (ref, score)


def test_kfold_fold_parallel_world2_equals_single(tmp_path):
    """dist: {mode: folds} (src/train.py:334-346): two ranks (gloo on one card) train the five
    folds round-robin (rank 0: folds 0, 2, 4; rank 1: folds 1, 3) with no collective while training, each
    writing its folds' checkpoints -- every fold's score and weights equal a single-process run of main(), bit
    for bit (fold-local seeds, deterministic kernels)."""
    import json
    import subprocess
    import sys
    from tossctr.data import synth_rows, write_shard_cache
    from tossctr.train import main
    cols = ["c0", "c1", "c2", "c3"]
    arr = synth_rows(2000, 6, 6, [203] * 4, 24, 3000, seed=8, pos_rate=0.2)
    man = write_shard_cache(str(tmp_path / "cache"), arr, shard_rows=700, num_cols=[f"n{i}" for i in range(6)],
                            cat_cols=cols, group_key="c0")
    cfg = tiny_run_cfg(str(tmp_path / "folds"), man)
    cfg["cv"]["n_splits"] = 5
    cfg["train"]["epochs"] = 1
    cfg["dist"] = {"mode": "folds"}
    cfg_path, out = str(tmp_path / "cfg.json"), str(tmp_path / "res.json")
    with open(cfg_path, "w") as f:
        json.dump(cfg, f)
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "dist_train_worker.py"), cfg_path, out],
                       capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    with open(out) as f:
        got = {int(k): v for k, v in json.load(f).items()}
    single = dict(cfg, logging=dict(cfg["logging"], log_dir=str(tmp_path / "single" / "runs")))
    ref = main(single)
    assert sorted(got) == sorted(ref) == [0, 1, 2, 3, 4]
    for fold in ref:
        assert got[fold] == ref[fold], (fold, got[fold], ref[fold])
        a = torch.load(os.path.join(cfg["logging"]["log_dir"], "tiny", f"ckpt_folds_{fold}.pt"), weights_only=True)
        b = torch.load(os.path.join(single["logging"]["log_dir"], "tiny", f"ckpt_folds_{fold}.pt"), weights_only=True)
        for k, v in b["state"]["model"].items():
            assert torch.equal(a["state"]["model"][k], v), (fold, k)
    assert os.path.exists(os.path.join(cfg["logging"]["log_dir"], "tiny", "train_log_rank1.csv"))


def test_fold_teardown_frees_device_memory(tmp_path):
    """train_one_fold releases its arena, moments, EMA shadow and workspaces before returning (the
    model <-> optimizer cycle is broken and collected, src/train.py:280-316): two folds in a row end at
    the same allocated bytes.  Tables of 2 x 2M x 16 fp32 make any leak ~0.5 GB."""
    import gc
    from tossctr.data import DeviceShards, synth_rows, write_shard_cache
    from tossctr.train import train_one_fold

    class Quiet:
        def row(self, *a, **kw):
            pass
        csv = scalars = row

    arr = synth_rows(1200, 6, 6, [203] * 4, 24, 3000, seed=7, pos_rate=0.2)
    man = write_shard_cache(str(tmp_path / "cache"), arr, shard_rows=600, num_cols=[f"n{i}" for i in range(6)],
                            cat_cols=["c0", "c1", "c2", "c3"], group_key="c0")
    cfg = tiny_run_cfg(str(tmp_path), man)
    cfg["seq_vocab"] = 2_000_000
    cfg["train"]["epochs"] = 1
    dev = torch.device("cuda", 0)
    store = DeviceShards(man, dev)
    idx = np.arange(1200)
    torch.cuda.synchronize()
    gc.collect()
    base = torch.cuda.memory_allocated(dev)
    for fold in range(2):
        train_one_fold(cfg, fold, idx[:1000], idx[1000:], man, Quiet(), store=store, device=dev)
        torch.cuda.synchronize()
        assert torch.cuda.memory_allocated(dev) - base < 8 << 20, (fold, torch.cuda.memory_allocated(dev) - base)
