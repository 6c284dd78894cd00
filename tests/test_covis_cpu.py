"""Co-visitation features, host side (tossctr/covis.py; drop-in for src/features/covis.py): the native seq
explode (csrc/hostio.cpp) against the plain-Python restatement (oracle/covis.py), the restatement itself
against a hand-worked example, fold assignment, and the build_cache_v2-style covis join of the shard builder.
Parity vs polars is unpinned (polars is not installed; see oracle/covis.py)."""
import json
import math
import os
import random

import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")
pq = pytest.importorskip("pyarrow.parquet")

from oracle import covis as ocv


def _seq_strings(rng, n, vocab=30):
    out = []
    for i in range(n):
        k = rng.randrange(0, 12)
        if i % 17 == 0:
            out.append(None)
        elif i % 19 == 0:
            out.append("")
        else:
            toks = [str(rng.randrange(-3, vocab)) for _ in range(k + 1)]
            if i % 7 == 0:
                toks.insert(rng.randrange(0, len(toks) + 1), rng.choice(["", "x", " 4", "2147483648", "+9", "-0"]))
            out.append(",".join(toks))
    return out


@pytest.mark.parametrize("top_k", [1, 3, 8, 120])
def test_native_explode_matches_restatement(top_k):
    from tossctr.covis import explode_seq
    rng = random.Random(top_k)
    vals = _seq_strings(rng, 400) + [",,", "1,", ",1", "2147483647,-2147483648", "007", "1,x,2,,3"]
    row_ptr, tok, pos, ok = explode_seq(pa.array(vals, pa.string()), top_k)
    ref = ocv.explode(vals, top_k, 512.0)
    assert row_ptr[-1] == len(ref) == len(tok)
    rows = np.repeat(np.arange(len(vals)), np.diff(row_ptr))
    assert [r for (r, _, _, _) in ref] == rows.tolist()
    assert [t is not None for (_, t, _, _) in ref] == ok.astype(bool).tolist()
    assert [0 if t is None else t for (_, t, _, _) in ref] == tok.tolist()
    assert [p for (_, _, p, _) in ref] == pos.tolist()


def test_restatement_hand_example():
    """Three rows worked by hand (covis.py:155-292 semantics)."""
    seqs = ["1,2", "2", None]
    tgt = ["A", "A", "A"]
    tb = [0, 0, 0]
    clicked = [1, 0, 0]
    tau = 4.0
    ex = ocv.explode(seqs, 120, tau)
    assert [(r, t, p) for (r, t, p, _) in ex] == [(0, 1, 0), (0, 2, 1), (1, 2, 0), (2, None, -1)]
    table, p0 = ocv.pair_stats(ex, tgt, tb, clicked, [1, 1, 1], S=2, ctr_clip=(1e-3, 0.999), min_impr=2)
    assert p0 == 0.5                          # two clicked elements of four exploded (null included)
    g1, g2 = table[(1, "A", 0)], table[(2, "A", 0)]
    assert (g1["impr"], g1["clicks"], g2["impr"], g2["clicks"]) == (1, 1, 2, 1)
    assert g1["ctr"] == (1 + 1) / (1 + 1 + 1) and g2["ctr"] == (1 + 1) / (2 + 1 + 1)
    assert g1["is_lowcount"] and not g2["is_lowcount"]
    assert g2["w_rec_sum"] == math.exp(-1 / tau) + 1.0 and g2["max_pos"] == 1
    f = ocv.row_features(ex, [0, 1, 2], tgt, tb, table, topn=3)
    w1 = math.exp(-1 / tau)
    assert f[0] == pytest.approx([7 / 6, 7 / 12, 2 / 3, 7 / 12, (2 / 3 + 0.5 * w1) / (1 + w1), 3.0, 2.0,
                                  math.sqrt((4 / 9 + 1 / 4) / 2)], rel=1e-15)
    assert f[1] == pytest.approx([0.5, 0.5, 0.5, 0.5, 0.5, 2.0, 2.0, 0.5], rel=1e-15)
    assert f[2] == [0.0] * 8                  # only the null token: every aggregate null -> 0


def test_restatement_topn_nulls_first():
    """ctr.sort(descending=True).head(n): polars sorts nulls first, so unmatched tokens fill head slots."""
    ex = ocv.explode(["1,9,2,8"], 120, 512.0)
    table = {(1, "A", 0): {"ctr": 0.3, "impr": 5}, (2, "A", 0): {"ctr": 0.1, "impr": 1}}
    f = ocv.row_features(ex, [0], ["A"], [0], table, topn=3)[0]
    assert f[3] == pytest.approx(0.3)          # [null, null, 0.3] -> mean 0.3
    f = ocv.row_features(ex, [0], ["A"], [0], table, topn=2)[0]
    assert f[3] == 0.0                         # [null, null] -> null -> 0


def test_make_folds_round_robin_over_sorted_hashes():
    from tossctr.covis import CoVisCfg, make_folds
    rng = np.random.default_rng(0)
    inv = pa.array([None if i % 11 == 0 else int(v) for i, v in enumerate(rng.integers(0, 40, 500))])
    dow = pa.array([int(v) for v in rng.integers(0, 7, 500)])
    tbl = pa.table({"inventory_id": inv, "day_of_week": dow})
    cfg = CoVisCfg(train_path="", test_path="", n_folds=5)
    rid, fold = make_folds(cfg, tbl)
    from tossctr.build_cache import hash_strings
    import pyarrow.compute as pc
    g = hash_strings(pc.binary_join_element_wise(pc.fill_null(pc.cast(inv, pa.string()), "NA"),
                                                 pc.fill_null(pc.cast(dow, pa.string()), "NA"), "\x1f"))
    assert np.array_equal(fold, ocv.make_folds(g, 5))
    assert np.array_equal(rid, np.arange(500))
    # every group lands in exactly one fold
    for gv in np.unique(g):
        assert len(np.unique(fold[g == gv])) == 1


def test_time_bins_and_codes():
    from tossctr.covis import CoVisCfg, _tb_codes, encode_codes, time_bin_values
    tbl = pa.table({"day_of_week": pa.array([1, None, 3, 6]), "hour": pa.array([5, 2, None, 23])})
    for mode in ("day_of_week", "hour", "day_of_week_hour"):
        cfg = CoVisCfg(train_path="", test_path="", time_bin=mode)
        got = time_bin_values(tbl, cfg)
        ref = ocv.time_bins([1, None, 3, 6], [5, 2, None, 23], mode)
        assert got.tolist() == [-1 if r is None else r for r in ref]
    (a, b), vals, bits = _tb_codes(np.array([5, -1, 9]), np.array([9, 2]))
    assert vals.tolist() == [2, 5, 9] and bits == 2 and a.tolist() == [1, -1, 2] and b.tolist() == [2, 0]
    (x, y), d = encode_codes(pa.array(["a", None, "b"]), pa.array(["b", "c"]))
    assert x.tolist() == [0, -1, 1] and y.tolist() == [1, 2] and d.to_pylist() == ["a", "b", "c"]


def test_build_cache_joins_covis_features(tmp_path):
    """build_cache_v2.py:208-287: features left-joined on the global rid (train) / ID (test), nulls -> 0."""
    from tossctr.build_cache import build_sharded_cache
    n = 37
    rng = np.random.default_rng(1)
    tr = pa.table({"clicked": pa.array(rng.integers(0, 2, n)), "seq": pa.array(["1,2"] * n),
                   "inventory_id": pa.array(rng.integers(0, 5, n)), "feat_a": pa.array(rng.normal(size=n)),
                   "ID": pa.array([f"TR_{i}" for i in range(n)])})
    te = tr.drop_columns(["clicked"])
    pq.write_table(tr, tmp_path / "train.parquet")
    pq.write_table(te, tmp_path / "test.parquet")
    cv = tmp_path / "covis"
    cv.mkdir()
    rid = np.array([3, 0, 36, 17, 5])
    pq.write_table(pa.table({"rid": pa.array(rid), "inventory_id_sum_ctr": pa.array(rid * 0.5),
                             "inventory_id_max_impr": pa.array(rid.astype(np.int64) * 2)}),
                   cv / "rowfeat_oof_all.parquet")
    pq.write_table(pa.table({"inventory_id_sum_ctr": pa.array([1.5, 2.5]), "inventory_id_max_impr": pa.array([7, 8]),
                             "ID": pa.array(["TR_4", "TR_30"])}), cv / "rowfeat_test.parquet")
    common = dict(target_col="clicked", seq_col="seq", cat_cols=["inventory_id"], hash_buckets={},
                  hash_buckets_margin=0, num_patterns=["feat_*"], max_len=4, pad_id=0, group_key="inventory_id",
                  shard_rows=10, batch_size=8, covis_enabled=True, covis_dir=str(cv))
    for split, is_train in (("train", True), ("test", False)):
        mp = build_sharded_cache(str(tmp_path / f"{split}.parquet"), str(tmp_path / "cache" / split),
                                 is_train=is_train, **common)
        man = json.load(open(mp))
        assert man["num_cols"] == ["feat_a", "inventory_id_sum_ctr", "inventory_id_max_impr"]
        X = np.concatenate([np.load(s["X_num"]["path"]) for s in man["shards"]])
        M = np.concatenate([np.load(s["X_mask"]["path"]) for s in man["shards"]])
        exp_sum, exp_imp = np.zeros(n), np.zeros(n)
        if is_train:
            exp_sum[rid], exp_imp[rid] = rid * 0.5, rid * 2
        else:
            exp_sum[[4, 30]], exp_imp[[4, 30]] = [1.5, 2.5], [7, 8]
        assert np.array_equal(X[:, 1], exp_sum.astype(np.float32))
        assert np.array_equal(X[:, 2], exp_imp.astype(np.float32))
        assert not M[:, 1:].any()
