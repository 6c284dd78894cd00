"""Parquet -> NPY shard cache + manifest.json -- drop-in for src/data/build_cache_v1.py.

Same entry points, arguments and on-disk result as the reference (``build_sharded_cache``,
``build_train_and_test``, ``analyze_schema_and_stats``; build_cache_v1.py:31-355): streaming Arrow record
batches (``batch_size=200_000``), per-column global medians for imputation, hashed categoricals, the
right-aligned ``seq`` matrix, shards cut at exactly ``shard_rows`` rows, ``shard_XXX/<name>.npy`` +
``manifest.json`` with the reference's keys.  The output is what ``tossctr.data`` (and the reference's
own ``src/data/dataset.py``) read.

MI355X-build differences (the reference runs on polars, which this environment does not have):
  * the frame engine is pyarrow; the two host hot loops (string hashing, the per-row seq split/parse of
    build_cache_v1.py:149-156) run natively in libctrhip.so (csrc/hostio.cpp) over the Arrow buffers;
  * the hash: polars' ``Series.hash(seed=2025, seed_1=0)`` is polars-version specific and cannot be
    reproduced without polars.  The build uses XXH64(utf8(value), seed=2025) -- stable, documented, and
    checked against the ``xxhash`` package.  Bucket assignment (``% (hash_buckets + margin)``), the "NA"
    null fill, the ``% (2**31 - 1)`` group ids and everything downstream follow the reference; the ids
    themselves differ from a polars build (parity "unpinned" for the hash).  Composite
    groups hash ``group + "\\x1f" + time`` instead of polars' struct hash;
  * medians: exact, over non-null non-NaN values (``np.nanmedian``); polars' median on a column holding
    float NaN values orders NaN above every number.
"""
from __future__ import annotations

import json
import os
import re
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _lib

HASH_SEED = 2025
ARRAYS = ["X_num", "X_mask", "X_cat", "seq", "y", "groups", "ids"]


def _pa():
    import pyarrow as pa
    import pyarrow.compute as pc
    import pyarrow.dataset as ds
    return pa, pc, ds


def match_patterns(cols: List[str], patterns: List[str]) -> List[str]:
    """build_cache_v1.py:11-16: '*' globs anchored at both ends, matches in pattern order, deduplicated, sorted."""
    out = []
    for p in patterns:
        regex = re.compile("^" + p.replace("*", ".*") + "$")
        out += [c for c in cols if regex.match(c)]
    return sorted(list(dict.fromkeys(out)))


# ------------------------------------------------------------------------------ native string helpers
def _string_buffers(arr):
    """(offsets int32 (n+1), data uint8, valid uint8 or None) of an Arrow string array."""
    pa, pc, _ = _pa()
    if isinstance(arr, pa.ChunkedArray):
        arr = arr.combine_chunks() if arr.num_chunks != 1 else arr.chunk(0)
    if arr.type != pa.string():
        arr = pc.cast(arr, pa.string())
    bufs = arr.buffers()
    n = len(arr)
    off = np.frombuffer(bufs[1], dtype=np.int32, count=arr.offset + n + 1)[arr.offset:] if n else \
        np.zeros(1, np.int32)
    data = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None and bufs[2].size else np.zeros(1, np.uint8)
    valid = None
    if arr.null_count:
        valid = np.asarray(arr.is_valid().to_numpy(zero_copy_only=False), dtype=np.uint8)
    return np.ascontiguousarray(off), data, valid


def hash_strings(arr, seed: int = HASH_SEED) -> np.ndarray:
    """XXH64 of each value's string form, nulls as "NA" (the reference's ``cast(Utf8).fill_null("NA")``)."""
    pa, pc, _ = _pa()
    arr = pc.fill_null(pc.cast(arr, pa.string()), "NA")
    off, data, _ = _string_buffers(arr)
    n = len(off) - 1
    out = np.empty(max(n, 1), dtype=np.uint64)
    rc = _lib.query("ctr_hash_utf8", off.ctypes.data, data.ctypes.data, n, int(seed), out.ctypes.data)
    if rc != 0:
        raise ValueError("ctr_hash_utf8: malformed string buffers")
    return out[:n]


def parse_seq(arr, max_len: int, pad_id: int) -> np.ndarray:
    """build_cache_v1.py:149-156 over an Arrow string column (nulls -> all pad)."""
    off, data, valid = _string_buffers(arr)
    n = len(off) - 1
    out = np.empty((max(n, 1), max_len), dtype=np.int32)
    rc = _lib.query("ctr_parse_seq", off.ctypes.data, data.ctypes.data,
                    valid.ctypes.data if valid is not None else None, n, int(max_len), int(pad_id), out.ctypes.data)
    if rc != 0:
        row = -rc - 2
        raise ValueError(f"seq row {row}: a token is not an int32 integer (int() would reject it)")
    return out[:n]


# ------------------------------------------------------------------------------ schema / statistics
def analyze_schema_and_stats(parquet_path: str, target_col: Optional[str], seq_col: str, cat_cols: List[str],
                             num_patterns: List[str], group_key: str, impute_strategy: str,
                             num_cols_explicit: List[str] | None = None,
                             remove_cols: List[str] | None = None) -> Dict:
    """build_cache_v1.py:31-75: column list, numeric columns (explicit list or patterns), global medians
    for imputation (0.0 where undefined), row count."""
    _, _, ds = _pa()
    dataset = ds.dataset(parquet_path, format="parquet")
    cols = list(dataset.schema.names)
    if num_cols_explicit:
        num_cols = [c for c in num_cols_explicit if c in cols]
    else:
        num_cols = [c for c in match_patterns(cols, num_patterns)
                    if c not in cat_cols and c not in [target_col, seq_col, group_key, "ID"] and c in cols]
    if remove_cols:
        num_cols = [c for c in num_cols if c not in remove_cols]
    med_map = {c: 0.0 for c in num_cols}
    if impute_strategy == "median":
        for c in num_cols:
            v = _column_f64(dataset.to_table(columns=[c]).column(c))
            v = v[~np.isnan(v)]
            med_map[c] = float(np.median(v)) if v.size else 0.0
    return {"all_cols": cols, "num_cols": num_cols, "med_map": med_map, "n_rows": int(dataset.count_rows())}


def _column_f64(col) -> np.ndarray:
    pa, pc, _ = _pa()
    col = pc.cast(col, pa.float64())
    if isinstance(col, pa.ChunkedArray):
        col = col.combine_chunks() if col.num_chunks != 1 else col.chunk(0)
    return np.asarray(col.to_numpy(zero_copy_only=False), dtype=np.float64)   # nulls -> NaN


# ------------------------------------------------------------------------------ one record batch
def process_batch(tbl, *, is_train: bool, target_col: Optional[str], seq_col: str, cat_cols: List[str],
                  hash_buckets: Dict[str, int], hash_buckets_margin: int, num_cols: List[str],
                  med_map: Dict[str, float], max_len: int, pad_id: int, group_key: str,
                  time_key: Optional[str] = None, composite_group: bool = False) -> Dict[str, np.ndarray]:
    """build_cache_v1.py:79-166 for one Arrow table/record batch."""
    pa, pc, _ = _pa()
    cols = tbl.schema.names
    n = tbl.num_rows
    y = None
    if is_train and target_col in cols:
        y = np.asarray(pc.cast(tbl.column(target_col), pa.int8()).to_numpy(zero_copy_only=False), dtype=np.int8)
    if composite_group and group_key in cols and time_key is not None and time_key in cols:
        gs = pc.fill_null(pc.cast(tbl.column(group_key), pa.string()), "NA")
        ts = pc.fill_null(pc.cast(tbl.column(time_key), pa.string()), "NA")
        g = hash_strings(pc.binary_join_element_wise(gs, ts, "\x1f"))
    elif group_key in cols:
        g = hash_strings(tbl.column(group_key))
    else:
        g = np.zeros(n, dtype=np.uint64)
    groups = (g % np.uint64(2**31 - 1)).astype(np.int64)
    if "ID" in cols:
        ids = np.asarray(pc.fill_null(pc.cast(tbl.column("ID"), pa.string()), "").to_numpy(zero_copy_only=False),
                         dtype="U64")
    else:
        ids = np.asarray(np.arange(n, dtype=np.int64).astype(str), dtype="U64")
    xc = []
    for c in cat_cols:
        hb = int(hash_buckets.get(c, 1000003)) + int(hash_buckets_margin)
        if c in cols:
            xc.append((hash_strings(tbl.column(c)) % np.uint64(hb)).astype(np.int32))
        else:
            xc.append(np.zeros((n,), np.int32))
    X_cat = np.stack(xc, axis=1).astype(np.int32) if xc else np.zeros((n, 0), np.int32)
    if num_cols:
        X_num = np.stack([_column_f64(tbl.column(c)) for c in num_cols], axis=1).astype(np.float32)
        mask = np.isnan(X_num).astype(np.uint8)
        for j, c in enumerate(num_cols):
            if mask[:, j].any():
                X_num[mask[:, j].astype(bool), j] = med_map.get(c, 0.0)
        np.nan_to_num(X_num, copy=False, nan=0.0, posinf=1e6, neginf=-1e6)
    else:
        X_num = np.zeros((n, 0), np.float32)
        mask = np.zeros((n, 0), np.uint8)
    if seq_col in cols:
        seq = parse_seq(tbl.column(seq_col), max_len, pad_id)
    else:
        seq = np.full((n, max_len), pad_id, dtype=np.int32)
    return {"X_num": X_num, "X_mask": mask, "X_cat": X_cat, "seq": seq,
            "y": (y if y is not None else np.zeros((n,), np.int8)), "groups": groups, "ids": ids}


# ------------------------------------------------------------------------------ shards
def _save_shard(shard_dir: str, arrays: Dict[str, np.ndarray]) -> Dict:
    os.makedirs(shard_dir, exist_ok=True)
    meta = {}
    for k in ARRAYS:
        v = arrays[k]
        path = os.path.join(shard_dir, f"{k}.npy")
        np.save(path, v)
        meta[k] = {"path": path, "shape": list(v.shape), "dtype": str(v.dtype)}
    meta["rows"] = arrays["seq"].shape[0]
    return meta


def _join_covis(rb, covis, row_cursor):
    """build_cache_v2.py:270-287: left join of the covis row features (global rid / ID), nulls -> 0.0."""
    pa, pc, _ = _pa()
    key, kcol, vals = covis
    if key == "rid":
        probe = pa.array(np.arange(row_cursor, row_cursor + rb.num_rows, dtype=np.int64))
        kcol = pc.cast(kcol, pa.int64())
    else:
        if "ID" not in rb.schema.names:
            return rb
        probe = pc.cast(rb.column("ID"), pa.string())
        kcol = pc.cast(kcol, pa.string())
    pos = pc.index_in(probe, value_set=kcol)
    valid = np.asarray(pc.is_valid(pos).to_numpy(zero_copy_only=False), bool)
    idx = np.asarray(pc.fill_null(pos, 0).to_numpy(zero_copy_only=False), np.int64)
    tbl = pa.Table.from_batches([rb])
    for c, v in vals.items():
        col = np.where(valid, v[idx] if len(v) else 0.0, 0.0)
        col = np.nan_to_num(col, nan=0.0)
        if c in tbl.schema.names:
            tbl = tbl.drop_columns([c])
        tbl = tbl.append_column(c, pa.array(col))
    return tbl


def build_sharded_cache(parquet_path: str, out_dir: str, *, is_train: bool, target_col: Optional[str],
                        seq_col: str, cat_cols: List[str], hash_buckets: Dict[str, int], hash_buckets_margin: int,
                        num_patterns: List[str], max_len: int, pad_id: int, group_key: str,
                        time_key: Optional[str] = None, composite_group: bool = False,
                        shard_rows: int = 2_000_000, impute_strategy: str = "median",
                        num_cols_explicit: List[str] | None = None, remove_cols: List[str] | None = None,
                        batch_size: int = 200_000, covis_enabled: bool = False,
                        covis_dir: str = "./cache/covis") -> str:
    """build_cache_v1.py:169-307 (build_cache_v2.py:177-347 with ``covis_enabled``: the co-visitation row
    features of tossctr.covis left-joined on the global row id (train) or ``ID`` (test), nulls -> 0.0,
    appended to the numeric columns with median 0.0).  Returns the manifest path."""
    pa, pc, ds = _pa()
    os.makedirs(out_dir, exist_ok=True)
    schema = analyze_schema_and_stats(parquet_path, target_col, seq_col, cat_cols, num_patterns, group_key,
                                      impute_strategy, num_cols_explicit, remove_cols)
    num_cols, med_map = schema["num_cols"], schema["med_map"]
    covis = None
    if covis_enabled:
        import pyarrow.parquet as pq
        cv = pq.read_table(os.path.join(covis_dir, "rowfeat_oof_all.parquet" if is_train else "rowfeat_test.parquet"))
        key = "rid" if is_train else "ID"
        covis_cols = [c for c in cv.schema.names if c not in ("rid", "ID") and
                      (pa.types.is_floating(cv.schema.field(c).type) or pa.types.is_integer(cv.schema.field(c).type))]
        for c in covis_cols:
            if c not in num_cols:
                num_cols.append(c)
                med_map[c] = 0.0
        covis = (key, cv.column(key), {c: _column_f64(cv.column(c)) for c in covis_cols})
    manifest = {"parquet": parquet_path, "is_train": is_train, "rows": 0, "shards": [],
                "num_cols": num_cols, "cat_cols": cat_cols, "group_key": group_key, "seq_col": seq_col}
    acc = {k: [] for k in ARRAYS}
    row_buf = 0

    def emit(arrays):
        idx = len(manifest["shards"])
        meta = _save_shard(os.path.join(out_dir, f"shard_{idx:03d}"), arrays)
        meta["index"] = idx
        meta["start"] = manifest["rows"]
        meta["end"] = manifest["rows"] + meta["rows"]
        manifest["shards"].append(meta)
        manifest["rows"] += meta["rows"]

    row_cursor = 0
    keep = None
    if remove_cols:
        keep = [c for c in ds.dataset(parquet_path, format="parquet").schema.names if c not in remove_cols]
    for rb in ds.dataset(parquet_path, format="parquet").scanner(columns=keep, batch_size=batch_size).to_batches():
        if rb.num_rows == 0:
            continue
        if covis is not None:
            rb = _join_covis(rb, covis, row_cursor)
        row_cursor += rb.num_rows
        batch = process_batch(rb, is_train=is_train, target_col=target_col, seq_col=seq_col, cat_cols=cat_cols,
                              hash_buckets=hash_buckets, hash_buckets_margin=hash_buckets_margin,
                              num_cols=num_cols, med_map=med_map, max_len=max_len, pad_id=pad_id,
                              group_key=group_key, time_key=time_key, composite_group=composite_group)
        for k in ARRAYS:
            acc[k].append(batch[k])
        row_buf += rb.num_rows
        while row_buf >= shard_rows:                      # cut exactly shard_rows, carry the tail
            cat = {k: np.concatenate(acc[k], axis=0) for k in ARRAYS}
            emit({k: v[:shard_rows] for k, v in cat.items()})
            acc = {k: [v[shard_rows:]] for k, v in cat.items()}
            row_buf = acc["seq"][0].shape[0]
    if row_buf:
        emit({k: np.concatenate(acc[k], axis=0) for k in ARRAYS})
    man_path = os.path.join(out_dir, "manifest.json")
    with open(man_path, "w") as f:
        json.dump(manifest, f, indent=2)
    return man_path


def build_train_and_test(cfg: dict, covis_enabled: bool = False) -> Tuple[str, str]:
    """build_cache_v1.py:310-351 / build_cache_v2.py:350-389.  The reference's v2 helper never passes
    ``covis_enabled`` (so its caches carry no covis columns); ``covis_enabled=True`` joins the features built
    by tossctr.covis from ``cfg["features"]["covis"]["work_dir"]``."""
    common = dict(seq_col=cfg["sequence"]["col"], cat_cols=cfg["data"]["cat_cols"],
                  hash_buckets=cfg["data"]["hash_buckets"],
                  hash_buckets_margin=cfg["data"].get("hash_buckets_margin", 0),
                  num_patterns=cfg["data"]["num_patterns"], num_cols_explicit=cfg["data"].get("num_cols_explicit"),
                  max_len=cfg["sequence"]["max_len"], pad_id=cfg["sequence"]["pad_id"],
                  group_key=cfg["cv"]["group_key"], time_key=cfg["cv"].get("time_key"),
                  composite_group=bool(cfg["cv"].get("composite_group", False)),
                  shard_rows=cfg["data"].get("shard_rows", 2_000_000),
                  impute_strategy=cfg["data"]["impute_strategy"], remove_cols=cfg["data"].get("remove_cols"))
    if covis_enabled:
        common.update(covis_enabled=True,
                      covis_dir=cfg.get("features", {}).get("covis", {}).get("work_dir", "./cache/covis"))
    mp_train = build_sharded_cache(cfg["data"]["train_path"], os.path.join(cfg["data"]["cache_dir"], "train"),
                                   is_train=True, target_col="clicked", **common)
    mp_test = build_sharded_cache(cfg["data"]["test_path"], os.path.join(cfg["data"]["cache_dir"], "test"),
                                  is_train=False, target_col=None, **common)
    return mp_train, mp_test


if __name__ == "__main__":
    import argparse

    import yaml
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", required=True)
    with open(ap.parse_args().cfg) as fh:
        print(build_train_and_test(yaml.safe_load(fh)))
