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
    st = torch.load(ckpt, weights_only=False)
    assert set(st) == {"state", "score"} and set(st["state"]) >= {"model", "cfg", "best_score", "epoch", "ema"}
    cards = {c: 203 for c in ["c0", "c1", "c2", "c3"]}
    m = CTRModel(cfg, 3000, 6, 6, cards, ["c0", "c1", "c2", "c3"], device="cuda:0")
    m.load_state_dict(st["state"]["model"], strict=True)
    csv_path = os.path.join(cfg["logging"]["log_dir"], "tiny", "train_log.csv")
    assert sum(1 for _ in open(csv_path)) >= 2
    # resume: a second main() skips the finished fold
    assert main(cfg) == {}
