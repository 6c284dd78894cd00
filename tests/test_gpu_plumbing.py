"""BASELINE config 1, the literal plumbing run: cfgs/dare_base.yaml (tossctr.configs.dare_base, pinned to the
yaml by tests/test_configs_cpu.py) on a synthetic 10k-row Parquet -> tossctr.build_cache (drop-in for
src/data/build_cache_v1.py) -> tossctr.train.main for 1 fold and 1 epoch at bs=256 (src/train.py:319-352)
-> the checkpoint loaded with torch.load(weights_only=True) -> eval logits of the HIP model vs the CPU
oracle forward (oracle/model.py) on the same rows, norm-wise 1e-4 -> tossctr.infer.main on the test cache.
Everything else is the yaml's: seq_vocab 10M (src/train.py:116), emb_dim 64, L = 400, K = 80, S1 query,
fc head, hash buckets up to 2M."""
import os
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
pa = pytest.importorskip("pyarrow")
pq = pytest.importorskip("pyarrow.parquet")


def _parquet(path, n, seed, train):
    """The dare_base schema: its six categoricals, numeric feat_* / history_* / l_feat_* columns (nulls,
    NaN, inf), a comma-joined ``seq`` (empty / null / over-long rows) and, for train, ``clicked``."""
    rng = np.random.default_rng(seed)
    r = random.Random(seed)
    cols = {"ID": pa.array([f"{'TRAIN' if train else 'TEST'}_{i:07d}" for i in range(n)])}
    if train:
        cols["clicked"] = pa.array((rng.random(n) < 0.1).astype(np.int64))
    cols["gender"] = pa.array([None if i % 31 == 0 else r.choice(["1.0", "2.0"]) for i in range(n)])
    cols["age_group"] = pa.array(rng.integers(1, 9, n).astype(np.int64))
    cols["inventory_id"] = pa.array([None if i % 53 == 0 else int(v) for i, v in enumerate(rng.integers(0, 90, n))])
    cols["day_of_week"] = pa.array(rng.integers(1, 8, n).astype(np.int64))
    cols["hour"] = pa.array(rng.integers(0, 24, n).astype(np.int64))
    for j in (1, 2, 3, 14):
        v = rng.standard_normal(n)
        v[rng.random(n) < 0.05] = np.nan
        if j == 2:
            v[3], v[4] = np.inf, -np.inf
        cols[f"l_feat_{j}"] = pa.array([None if (i + j) % 41 == 0 else float(x) for i, x in enumerate(v)])
    for j in (1, 2):
        cols[f"feat_a_{j}"] = pa.array([None if i % 17 == j else int(x) for i, x in enumerate(rng.integers(-5, 5, n))])
    cols["history_a_1"] = pa.array(rng.random(n).astype(np.float32))
    seqs = []
    for i in range(n):
        k = int(rng.integers(0, 450))
        s = ",".join(str(int(t)) for t in rng.integers(1, 5000, k))
        seqs.append(None if i % 23 == 0 else s)
    cols["seq"] = pa.array(seqs)
    pq.write_table(pa.table(cols), path)


@pytest.mark.timeout(600)
def test_dare_base_plumbing(tmp_path):
    from oracle.model import Dropper, forward as oracle_forward, make_arch
    from tossctr import CTRModel
    from tossctr.build_cache import build_train_and_test
    from tossctr.configs import dare_base
    from tossctr.data import ShardedDataset, collate_sharded
    from tossctr.infer import main as infer_main
    from tossctr.train import _feature_dims, main
    tr_path, te_path = str(tmp_path / "train.parquet"), str(tmp_path / "test.parquet")
    _parquet(tr_path, 10_000, 1, True)
    _parquet(te_path, 1_500, 2, False)
    cfg = dare_base(data={"train_path": tr_path, "test_path": te_path, "cache_dir": str(tmp_path / "cache")},
                    train={"batch_size": 256, "epochs": 1}, cv={"n_splits": 1},
                    logging={"log_dir": str(tmp_path / "runs"), "tb": False})
    mp_train, mp_test = build_train_and_test(cfg)
    cfg["data"]["manifest_train"], cfg["data"]["manifest_test"] = mp_train, mp_test
    res = main(cfg)
    assert list(res) == [0] and np.isfinite(res[0])
    ckpt = os.path.join(cfg["logging"]["log_dir"], "dare_base", "ckpt_folds_0.pt")
    st = torch.load(ckpt, weights_only=True)
    state = st["state"]
    assert abs(float(st["score"]) - float(res[0])) < 1e-12
    sd = state["model"]
    assert sd["dare.emb_att.weight"].shape == (10_000_000, 64)
    # the checkpoint's weights: HIP eval forward vs the CPU oracle on 512 rows of the train cache
    cat_cols = cfg["data"]["cat_cols"]
    cards = {c: int(cfg["data"]["hash_buckets"][c]) for c in cat_cols}
    n_num, n_mask = _feature_dims(mp_train)
    model = CTRModel(cfg, 10_000_000, n_num, n_mask, cards, cat_cols, device="cuda:0")
    model.load_state_dict(sd, strict=True)
    model.eval()
    rows = np.arange(0, 10_000, 10_000 // 512)[:512]
    batch = collate_sharded([ShardedDataset(mp_train, rows, True, cat_cols)[i] for i in range(len(rows))])
    with torch.no_grad():
        z, p, a = model(batch)
    A = make_arch(cfg, 10_000_000, n_num, n_mask, cards, cat_cols)
    P = {k: v.float() for k, v in sd.items()}
    with torch.no_grad():
        zr, pr, ar = oracle_forward(P, {k: batch[k] for k in ("X_num", "X_mask", "X_cat", "seq")}, A,
                                    Dropper(0, training=False))
    for got, ref, name in ((z, zr, "logits"), (a, ar, "aux")):
        got, ref = got.cpu().double(), ref.double()
        assert float((got - ref).norm() / (ref.norm() + 1e-30)) < 1e-4, name
    del model
    # inference on the test cache: one probability per test row, in (0, 1), calibrated as trained
    sub = infer_main(cfg)
    lines = open(sub).read().strip().split("\n")
    assert lines[0] == "ID,clicked" and len(lines) == 1 + 1_500
    probs = np.array([float(x.split(",")[1]) for x in lines[1:]])
    assert np.all((probs > 0) & (probs < 1))
