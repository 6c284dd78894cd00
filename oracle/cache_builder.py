"""Plain-Python restatement of the reference's Parquet -> NPY shard builder for checking
``tossctr.build_cache``.

TEST INFRASTRUCTURE (see oracle/__init__.py): imported only by tests/.

Follows src/data/build_cache_v1.py row by row on Python lists (``pyarrow`` only reads the file):
  * numeric columns: _match_patterns (:11-16) / explicit list, exclusions (:47-54), global median
    imputation (:56-66), isnan mask, nan_to_num(0, 1e6, -1e6) (:134-146);
  * categoricals: str(value) or "NA" for null, hashed, ``% (hash_buckets.get(c, 1000003) + margin)`` (:124-132);
  * groups: hash(str(group) or "NA") % (2**31 - 1) (:96-113); ids: str(ID) or "" / per-batch arange (:115-123);
  * seq: the :149-156 loop verbatim (split(","), `if x`, int(), last max_len, right-aligned over pad_id);
  * shards: cut at exactly shard_rows, manifest keys and order (:169-307).
The hash is the build's documented replacement for polars' Series.hash: XXH64(utf8, seed=2025) from the
``xxhash`` package (3.x; its published algorithm), independent of csrc/hostio.cpp's restatement.
"""
from __future__ import annotations

import re

import numpy as np


def xxh64(s: str, seed: int = 2025) -> int:
    import xxhash
    return xxhash.xxh64_intdigest(s.encode("utf-8"), seed=seed)


def match_patterns(cols, patterns):
    out = []
    for p in patterns:
        regex = re.compile("^" + p.replace("*", ".*") + "$")
        out += [c for c in cols if regex.match(c)]
    return sorted(list(dict.fromkeys(out)))


def num_cols_and_medians(rows, cols, target_col, seq_col, cat_cols, num_patterns, group_key, impute_strategy):
    """rows: {col: python list}.  (num_cols, med_map)."""
    num_cols = [c for c in match_patterns(cols, num_patterns)
                if c not in cat_cols and c not in [target_col, seq_col, group_key, "ID"] and c in cols]
    med = {}
    for c in num_cols:
        vals = [float(v) for v in rows[c] if v is not None and not (isinstance(v, float) and v != v)]
        med[c] = float(np.median(vals)) if (vals and impute_strategy == "median") else 0.0
    return num_cols, med


def process_rows(rows, n, *, is_train, target_col, seq_col, cat_cols, hash_buckets, margin, num_cols, med_map,
                 max_len, pad_id, group_key, batch_starts):
    """All rows at once; ``batch_starts`` = first row of each Arrow record batch (ids restart per batch)."""
    y = np.array([int(v) for v in rows[target_col]], np.int8) if (is_train and target_col in rows) else \
        np.zeros(n, np.int8)
    if group_key in rows:
        groups = np.array([xxh64("NA" if v is None else str(v)) % (2**31 - 1) for v in rows[group_key]], np.int64)
    else:
        groups = np.zeros(n, np.int64)
    if "ID" in rows:
        ids = np.array(["" if v is None else str(v) for v in rows["ID"]], dtype="U64")
    else:
        ids = np.empty(n, dtype="U64")
        bounds = list(batch_starts) + [n]
        for a, b in zip(bounds[:-1], bounds[1:]):
            ids[a:b] = np.arange(b - a).astype(str)
    xc = []
    for c in cat_cols:
        hb = hash_buckets.get(c, 1000003) + margin
        if c in rows:
            xc.append([xxh64("NA" if v is None else str(v)) % hb for v in rows[c]])
        else:
            xc.append([0] * n)
    X_cat = np.array(xc, dtype=np.int64).T.astype(np.int32) if cat_cols else np.zeros((n, 0), np.int32)
    X_num = np.array([[np.nan if v is None else float(v) for v in rows[c]] for c in num_cols],
                     dtype=np.float64).T.astype(np.float32) if num_cols else np.zeros((n, 0), np.float32)
    mask = np.isnan(X_num).astype(np.uint8)
    for j, c in enumerate(num_cols):
        X_num[mask[:, j] == 1, j] = med_map.get(c, 0.0)
    np.nan_to_num(X_num, copy=False, nan=0.0, posinf=1e6, neginf=-1e6)
    s = [("" if v is None else v) for v in rows[seq_col]] if seq_col in rows else [""] * n
    seq = np.full((n, max_len), pad_id, dtype=np.int32)
    for i, st in enumerate(s):
        if not st:
            continue
        toks = [int(x) for x in str(st).split(",") if x]
        toks = toks[-max_len:]
        if toks:
            seq[i, -len(toks):] = np.asarray(toks, dtype=np.int32)
    return {"X_num": X_num, "X_mask": mask, "X_cat": X_cat, "seq": seq, "y": y, "groups": groups, "ids": ids}
