"""The BASELINE.json benchmark configurations as cfg dicts.

``/root/reference`` (and its yamls) does not exist on the GPU box, so the values the hot path reads
are restated here with their yaml line citations.  ``load_yaml`` accepts the reference's own yaml
files unchanged when they are available.
"""
from __future__ import annotations

import copy

# cfgs/dare_qnn_next.yaml:17-51 (cat_cols) and :198-233 (cat_embedding_dims)
CAT_DIMS_NEXT = {
    "gender": 8, "age_group": 8, "inventory_id": 16, "day_of_week": 8, "hour": 8,
    "l_feat_1": 8, "l_feat_2": 8, "l_feat_3": 8, "l_feat_4": 8, "l_feat_5": 33, "l_feat_6": 30,
    "l_feat_7": 18, "l_feat_8": 8, "l_feat_9": 22, "l_feat_10": 17, "l_feat_11": 40, "l_feat_12": 64,
    "l_feat_13": 8, "l_feat_14": 57, "l_feat_15": 51, "l_feat_16": 8, "l_feat_17": 22, "l_feat_18": 8,
    "l_feat_19": 8, "l_feat_20": 8, "l_feat_21": 8, "l_feat_22": 8, "l_feat_23": 8, "l_feat_24": 8,
    "l_feat_25": 43, "l_feat_26": 8, "l_feat_27": 8, "feat_a_2": 8, "feat_a_8": 8, "feat_a_9": 8,
}
N_NUM_NEXT = 82   # cfgs/dare_qnn_next.yaml:52-134 num_cols_explicit (82 columns) -> X_num / X_mask width


def dare_base(**over):
    """BASELINE config 1: cfgs/dare_base.yaml (DARE only: S1 query on inventory_id, no encoder block, fc
    head, emb_dim 64, L = 400, K = 80), restated value for value; ``over`` replaces top-level sections."""
    cfg = {
        "exp_name": "dare_base", "seed": 777, "device": "cuda", "deterministic": True, "amp": "none",   # l.1-5
        "use_compile": False,
        "data": {"train_path": "/path/to/train.parquet", "test_path": "/path/to/test.parquet",          # l.8-24
                 "cache_dir": "./cache/dare_base", "use_cache": True, "chunked_build": True, "add_isna_mask": True,
                 "impute_strategy": "median",
                 "cat_cols": ["gender", "age_group", "inventory_id", "day_of_week", "hour", "l_feat_14"],
                 "hash_buckets": {"gender": 16, "age_group": 64, "day_of_week": 8, "hour": 32,
                                  "inventory_id": 2_000_000, "l_feat_14": 1_000_000},
                 "num_patterns": ["feat_*", "history_*", "l_feat_*"]},
        "sequence": {"col": "seq", "max_len": 400, "pad_id": 0, "top_k": 80, "recency_tau": 256,         # l.26-34
                     "query_mode": "S1", "query_key": "inventory_id", "transformer_block": False},
        "model": {"emb_dim": 64, "dare_dropout": 0.1, "qnn_alpha": {"enabled": False}},                # l.36-40
        "train": {"batch_size": 16384, "epochs": 10, "optimizer": "adamw", "lr": 0.001, "weight_decay": 0.0001,
                  "warmup_epochs": 1, "cosine": True, "early_stop_patience": 3, "grad_clip_norm": 1.0},  # l.42-51
        "cv": {"n_splits": 5, "group_key": "inventory_id", "stratify_target": "clicked"},              # l.53-56
        "eval": {"monitor": "score", "maximize": True},                                                # l.58-60
        "calibration": {"enabled": True, "method": "temperature", "lr": 0.05, "iters": 200},           # l.62-66
        "logging": {"log_dir": "./runs", "tb": True, "csv_log": True, "verbose_steps": 100},           # l.68-72
    }
    for k, v in over.items():
        if isinstance(v, dict) and isinstance(cfg.get(k), dict):
            cfg[k] = {**cfg[k], **v}
        else:
            cfg[k] = v
    return cfg


def dare_qnn_next(emb_dim=32, max_len=100, batch_size=4096, hash_buckets=1_000_000):
    """BASELINE config 2: cfgs/dare_qnn_next.yaml with hash_buckets=1e6, emb_dim=32, seq_len=100, bs=4096."""
    cat_cols = list(CAT_DIMS_NEXT)
    return {
        "exp_name": "dare_qnn_next", "seed": 777, "device": "cuda", "deterministic": True, "amp": "none",
        "use_compile": False,
        "data": {"cat_cols": cat_cols, "hash_buckets": {c: hash_buckets for c in cat_cols},
                 "hash_buckets_margin": 0},
        "sequence": {"col": "seq", "max_len": max_len, "pad_id": 0, "top_k": 60, "recency_tau": 512,
                     "query_mode": "concat", "query_key": "inventory_id", "transformer_block": True,
                     "tfm": {"n_layers": 3, "n_heads": 8, "mha_dropout": 0.1, "ffn_hidden": 384, "ffn_dropout": 0.1,
                             "norm": "rms", "gating": "softmax", "add_positional_bias": True}},   # yaml l.177-193
        "model": {"emb_dim": emb_dim, "dare_dropout": 0.2, "cat_embedding_dims": dict(CAT_DIMS_NEXT),
                  "qnn_alpha": {"enabled": True, "feature_embed_dim": 32, "heads": 6, "rank": 16, "proj_dim": 192,
                                "mlp_hidden": [512, 256], "dropout": 0.2, "use_se": True, "se_reduction": 8,
                                "use_residual": True, "norm": "rms", "pair_grouping": "all",
                                "aux_head_weight": 0.1}},                                         # yaml l.234-249
        "train": {"batch_size": batch_size, "epochs": 8, "optimizer": "adamw", "lr": 3e-4, "weight_decay": 1e-4,
                  "warmup_epochs": 2, "cosine": True, "early_stop_patience": 3, "grad_clip_norm": 0.5},  # l.250-259
        "cv": {"n_splits": 5, "group_key": "inventory_id"},
        "calibration": {"enabled": True, "method": "temperature", "lr": 0.05, "iters": 200},
        "logging": {"log_dir": "./runs", "tb": False, "csv_log": True},
        "ema": {"enabled": True, "decay": 0.999, "eval_with_ema": True, "start_epoch": 1},       # l.288-292
    }


def dare_qnn_next_k100_s1(**kw):
    """BASELINE config 3: cfgs/dare_qnn_next_k100_s1.yaml (K=100, query S1) at the cfg2 overrides."""
    cfg = dare_qnn_next(**kw)
    cfg["exp_name"] = "dare_qnn_next_k100_s1"
    cfg["sequence"]["top_k"] = 100
    cfg["sequence"]["query_mode"] = "S1"
    return cfg


# cfgs/v3_k148_s1.yaml:137-171 (hash_buckets; margin 500 at l.172)
HB_V3 = {
    "gender": 1005, "age_group": 1011, "day_of_week": 1009, "hour": 1026, "inventory_id": 1020, "l_feat_1": 1004,
    "l_feat_2": 1005, "l_feat_3": 1005, "l_feat_4": 1028, "l_feat_5": 2078, "l_feat_6": 1902, "l_feat_7": 1315,
    "l_feat_8": 1005, "l_feat_9": 1478, "l_feat_10": 1264, "l_feat_11": 2526, "l_feat_12": 6052, "l_feat_13": 1004,
    "l_feat_14": 4239, "l_feat_15": 3584, "l_feat_16": 1004, "l_feat_17": 1478, "l_feat_18": 1010, "l_feat_19": 1005,
    "l_feat_20": 1004, "l_feat_21": 1005, "l_feat_22": 1005, "l_feat_23": 1004, "l_feat_24": 1005, "l_feat_25": 2790,
    "l_feat_26": 1020, "l_feat_27": 1007, "feat_a_2": 1008, "feat_a_8": 1010, "feat_a_9": 1012,
}


def v3_k148_s1(batch_size=4096, max_len=400):
    """BASELINE config 4: cfgs/v3_k148_s1.yaml as-is -- D=64 (l.199), L=400, K=148, S1 (l.181-184),
    4 layers x 8 heads, ffn 384, ffn dropout 0.15 (l.186-194), dare dropout 0.25 (l.200),
    inventory_id dim 32 (l.205), EMA off (l.294), buckets l.137-172."""
    cfg = dare_qnn_next(emb_dim=64, max_len=max_len, batch_size=batch_size)
    cfg["exp_name"] = "v3_k132_s1"
    cfg["data"]["hash_buckets"] = dict(HB_V3)
    cfg["data"]["hash_buckets_margin"] = 500
    sq = cfg["sequence"]
    sq.update(top_k=148, query_mode="S1")
    sq["tfm"].update(n_layers=4, ffn_dropout=0.15)
    cfg["model"]["dare_dropout"] = 0.25
    cfg["model"]["cat_embedding_dims"]["inventory_id"] = 32
    cfg["ema"]["enabled"] = False
    return cfg


def hb1e8_d64(**kw):
    """BASELINE config 5: the k100_s1 shape with every hash_buckets = 1e8 and emb_dim = 64 (tables of
    60 B parameters: row-sharded over 8 GPUs)."""
    kw.setdefault("emb_dim", 64)
    kw.setdefault("hash_buckets", 100_000_000)
    cfg = dare_qnn_next_k100_s1(**kw)
    cfg["exp_name"] = "hb1e8_d64"
    return cfg


BENCH_CONFIGS = {"cfg2": dare_qnn_next, "cfg3": dare_qnn_next_k100_s1, "cfg4": v3_k148_s1, "cfg5": hb1e8_d64}


def cat_cardinals(cfg):
    """src/train.py:119: hash_buckets.get(c, 1000003) + hash_buckets_margin."""
    d = cfg["data"]
    return {c: int(d["hash_buckets"].get(c, 1000003)) + int(d.get("hash_buckets_margin", 0)) for c in d["cat_cols"]}


def load_yaml(path, **overrides):
    import yaml
    with open(path) as f:
        cfg = yaml.safe_load(f)
    cfg = copy.deepcopy(cfg)
    for k, v in overrides.items():
        cfg[k] = v
    return cfg
