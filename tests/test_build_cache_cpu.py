"""Parquet -> NPY shard cache builder (tossctr/build_cache.py, drop-in for src/data/build_cache_v1.py) vs
the plain-Python restatement of the reference (oracle/cache_builder.py): numeric selection, median
imputation + masks + nan_to_num, hashed categoricals / groups (XXH64 replacement of polars' hash, checked
against the xxhash package), ids, the right-aligned seq matrix, shard cuts and manifest.  CPU only (the
native helpers are host code in libctrhip.so)."""
import json
import os
import random

import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")
pq = pytest.importorskip("pyarrow.parquet")
xxhash = pytest.importorskip("xxhash")


def _strings(rng, n):
    alpha = "abcxyz0123456789,;-_ ÄéΩ😀"
    return ["".join(rng.choice(alpha) for _ in range(rng.randrange(0, 90))) for _ in range(n)]


def test_native_xxh64_matches_xxhash_package():
    from tossctr.build_cache import hash_strings
    rng = random.Random(5)
    vals = _strings(rng, 500) + ["", "NA", "a" * 31, "b" * 32, "c" * 33, "d" * 64, "é" * 40]
    got = hash_strings(pa.array(vals))
    ref = np.array([xxhash.xxh64_intdigest(v.encode("utf-8"), seed=2025) for v in vals], dtype=np.uint64)
    assert np.array_equal(got, ref)
    # nulls hash as "NA"; non-string columns through their string form
    got = hash_strings(pa.array([None, 17, -3], type=pa.int64()))
    assert list(got) == [xxhash.xxh64_intdigest(s.encode(), seed=2025) for s in ("NA", "17", "-3")]


def test_parse_seq_matches_reference_loop():
    from tossctr.build_cache import parse_seq
    from oracle.cache_builder import process_rows
    vals = ["", None, "1,2,3", ",,5,,", " 7, 8", "-4,9", ",".join(str(i) for i in range(40)), "11", "2147483647"]
    got = parse_seq(pa.array(vals), 16, 0)
    ref = process_rows({"seq": vals}, len(vals), is_train=False, target_col=None, seq_col="seq", cat_cols=[],
                       hash_buckets={}, margin=0, num_cols=[], med_map={}, max_len=16, pad_id=0, group_key="g",
                       batch_starts=[0])["seq"]
    assert np.array_equal(got, ref)
    with pytest.raises(ValueError):
        parse_seq(pa.array(["1,x,2"]), 4, 0)
    with pytest.raises(ValueError):
        parse_seq(pa.array(["1, ,2"]), 4, 0)        # int(" ") raises in the reference
    with pytest.raises(ValueError):
        parse_seq(pa.array(["3000000000"]), 4, 0)   # np.int32 overflow in the reference


def _make_parquet(path, n, seed, with_id=True):
    rng = np.random.default_rng(seed)
    r = random.Random(seed)
    cols = {}
    if with_id:
        cols["ID"] = pa.array([None if i % 97 == 5 else f"TRAIN_{i:07d}" for i in range(n)])
    cols["clicked"] = pa.array(rng.integers(0, 2, n).astype(np.int64))
    cols["inventory_id"] = pa.array([None if i % 53 == 0 else int(v) for i, v in enumerate(rng.integers(0, 40, n))])
    cols["gender"] = pa.array([None if i % 31 == 0 else r.choice(["1.0", "2.0", "M", "F"]) for i in range(n)])
    cols["age_group"] = pa.array(rng.integers(1, 9, n).astype(np.int64))
    for j in range(3):
        v = rng.standard_normal(n)
        v[rng.random(n) < 0.05] = np.nan
        if j == 1:
            v[3] = np.inf
            v[4] = -np.inf
        cols[f"l_feat_{j + 1}"] = pa.array([None if (i + j) % 41 == 0 else float(x) for i, x in enumerate(v)])
    cols["feat_a_1"] = pa.array([None if i % 17 == 0 else int(x) for i, x in enumerate(rng.integers(-5, 5, n))])
    cols["history_a_1"] = pa.array(rng.random(n).astype(np.float32))
    seqs = []
    for i in range(n):
        k = int(rng.integers(0, 30))
        s = ",".join(str(int(t)) for t in rng.integers(1, 5000, k))
        if i % 23 == 0:
            s = None
        elif i % 29 == 0:
            s = "," + (s or "") + ",,"
        seqs.append(s)
    cols["seq"] = pa.array(seqs)
    cols["junk"] = pa.array(rng.random(n))
    pq.write_table(pa.table(cols), path, row_group_size=300)


CFG = dict(seq_col="seq", cat_cols=["gender", "age_group", "inventory_id", "missing_col"],
           hash_buckets={"gender": 7, "age_group": 11, "inventory_id": 1000}, hash_buckets_margin=3,
           num_patterns=["l_feat_*", "feat_*", "history_*", "junk"], max_len=20, pad_id=0, group_key="inventory_id",
           impute_strategy="median", remove_cols=["junk"])


@pytest.mark.parametrize("with_id", [True, False])
def test_build_sharded_cache_matches_reference_restatement(tmp_path, with_id):
    import pyarrow.dataset as ds
    from tossctr.build_cache import build_sharded_cache
    from oracle import cache_builder as ocb
    n = 1037
    path = str(tmp_path / "train.parquet")
    _make_parquet(path, n, seed=3 + with_id, with_id=with_id)
    man_path = build_sharded_cache(path, str(tmp_path / "cache"), is_train=True, target_col="clicked",
                                   shard_rows=400, batch_size=256, **CFG)
    with open(man_path) as f:
        man = json.load(f)
    assert man["rows"] == n and [s["rows"] for s in man["shards"]] == [400, 400, 237]
    assert [(s["start"], s["end"]) for s in man["shards"]] == [(0, 400), (400, 800), (800, 1037)]
    assert man["cat_cols"] == CFG["cat_cols"] and man["group_key"] == "inventory_id" and man["seq_col"] == "seq"
    assert man["num_cols"] == ["feat_a_1", "history_a_1", "l_feat_1", "l_feat_2", "l_feat_3"]   # junk removed
    got = {k: np.concatenate([np.load(s[k]["path"]) for s in man["shards"]]) for k in
           ["X_num", "X_mask", "X_cat", "seq", "y", "groups", "ids"]}
    for s in man["shards"]:
        assert list(s)[:7] == ["X_num", "X_mask", "X_cat", "seq", "y", "groups", "ids"]
        assert s["X_num"]["dtype"] == "float32" and s["seq"]["dtype"] == "int32" and s["ids"]["dtype"] == "<U64"
    # oracle over the same rows, record-batch starts from the same scanner
    tbl = pq.read_table(path)
    rows = {c: tbl.column(c).to_pylist() for c in tbl.schema.names if c != "junk"}
    starts, pos = [], 0
    for rb in ds.dataset(path, format="parquet").scanner(batch_size=256).to_batches():
        starts.append(pos)
        pos += rb.num_rows
    num_cols, med = ocb.num_cols_and_medians(rows, list(rows), "clicked", "seq", CFG["cat_cols"],
                                             CFG["num_patterns"], "inventory_id", "median")
    assert num_cols == man["num_cols"]
    ref = ocb.process_rows(rows, n, is_train=True, target_col="clicked", seq_col="seq", cat_cols=CFG["cat_cols"],
                           hash_buckets=CFG["hash_buckets"], margin=3, num_cols=num_cols, med_map=med, max_len=20,
                           pad_id=0, group_key="inventory_id", batch_starts=starts)
    for k in ["X_mask", "X_cat", "seq", "y", "groups", "ids"]:
        assert got[k].dtype == ref[k].dtype and np.array_equal(got[k], ref[k]), k
    assert np.array_equal(got["X_num"], ref["X_num"])
    assert got["X_mask"].sum() > 0 and (got["seq"] == 0).all(axis=1).sum() > 0


def test_cache_feeds_the_shard_readers(tmp_path):
    """The builder's output is what tossctr.data's readers (and the K-fold loop) consume."""
    from tossctr.build_cache import build_sharded_cache
    from tossctr.data import load_labels_groups_for_split
    path = str(tmp_path / "t.parquet")
    _make_parquet(path, 300, seed=9)
    man_path = build_sharded_cache(path, str(tmp_path / "c"), is_train=True, target_col="clicked", shard_rows=128,
                                   **CFG)
    y, groups = load_labels_groups_for_split(man_path)
    assert y.shape == (300,) and groups.shape == (300,) and set(np.unique(y)) <= {0, 1}
