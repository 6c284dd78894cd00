"""Plain-Python restatement of the reference's co-visitation feature builder, for checking
``tossctr.covis`` (csrc/covis.hip + the explode parser in csrc/hostio.cpp).

TEST INFRASTRUCTURE (see oracle/__init__.py): imported only by tests/.

Follows src/features/covis.py (polars lazy frames) on Python lists:
  * seq parse (_parse_seq_topk, :60-80): ``str.split(",")`` (empty pieces kept), per-piece non-strict Int32
    cast (a piece that is not [+-]digits within int32 is null), the LAST ``seq_top_k`` pieces; a null seq is
    the empty list;
  * explode (:174-183, :236-243): an empty list explodes to one null token; ``pos = cum_count() - 1`` over
    the row, where cum_count counts non-null tokens (polars >= 1.0); ``w_rec = exp(-pos / tau)``;
  * time_bin (_make_timebin_expr, :97-103): the configured column cast to Int32, or day_of_week*24 + hour;
  * pair stats (_pair_stats_from_scan, :155-213): group_by (token, target[, time_bin]) -> impr = len,
    clicks = sum(clicked), w_rec_sum, max_pos; p0 = mean(clicked) over the EXPLODED rows (:199-201);
    ctr = beta-smoothed (clicks + p0 S) / (impr + p0 S + (1-p0) S) clipped to [1e-9, 1-1e-9]
    (_beta_smooth_ctr, :106-109), then to ctr_clip; is_lowcount = impr < min_impr;
  * row features (_row_features_from_pair_tbl, :233-292): left join of the exploded rows on the pair keys
    (nulls never match), per row: sum / mean / max of ctr, the top-n mean of ``ctr.sort(descending=True)``
    (polars sorts nulls FIRST, so unmatched tokens take top-n slots), (ctr*w).sum() / w.sum(), sum / max of
    impr (null -> 0), sqrt(mean(ctr^2)); fill_null(0);
  * folds (make_folds, :113-150): sorted distinct group hashes dealt round-robin over n_folds.

PARITY UNPINNED: polars (the reference's engine, Series/struct ``hash``) is not installed here and the
reference pipeline does not run under its own pinned polars (``clip_min`` was removed in polars 1.0,
``DataFrame.set_index`` does not exist, ``with_row_index("rid")`` twice on one frame) -- no fixture or
golden output of it exists.  This file restates the evident intent line by line; the hash is the build's
XXH64 replacement (``xxhash`` package) as in oracle/cache_builder.py.
"""
from __future__ import annotations

import math
import re

import numpy as np

_INT = re.compile(r"^[+-]?[0-9]+$")


def cast_int32(piece: str):
    """polars Utf8 -> Int32, strict=False: null unless the piece is an int32 decimal literal."""
    if not _INT.match(piece):
        return None
    v = int(piece)
    return v if -2**31 <= v < 2**31 else None


def parse_seq_topk(s, top_k: int):
    """covis.py:60-80: list of the last top_k pieces (None for unparsable ones); null seq -> []."""
    if s is None:
        return []
    toks = [cast_int32(p) for p in s.split(",")]
    return toks[-top_k:] if top_k > 0 else []


def explode(seqs, top_k: int, tau: float):
    """covis.py:174-183: [(row, token|None, pos, w_rec)] in row order."""
    out = []
    for r, s in enumerate(seqs):
        toks = parse_seq_topk(s, top_k) or [None]          # explode of [] -> one null
        cnt = 0
        for t in toks:
            if t is not None:
                cnt += 1
            pos = cnt - 1
            out.append((r, t, pos, math.exp(-pos / float(tau))))
    return out


def time_bins(dow, hour, mode: str):
    """covis.py:97-103; None where an input is null."""
    if mode == "day_of_week_hour":
        return [None if d is None or h is None else int(d) * 24 + int(h) for d, h in zip(dow, hour)]
    src = dow if mode == "day_of_week" else hour
    return [None if v is None else int(v) for v in src]


def beta_smooth(clicks, impr, p0, S):
    alpha = p0 * S
    beta = (1.0 - p0) * S
    return min(max((clicks + alpha) / (impr + alpha + beta), 1e-9), 1 - 1e-9)


def pair_stats(ex, target, tbin, clicked, keep, S, ctr_clip, min_impr):
    """covis.py:155-213 over the exploded rows of the kept source rows.  Returns (table, p0) with
    table = {(token, target, tbin): dict(impr, clicks, w_rec_sum, max_pos, ctr, is_lowcount)}, including
    groups with null key parts (they exist in the reference table but can never match the join)."""
    grp = {}
    n = c = 0
    for (r, t, pos, w) in ex:
        if not keep[r]:
            continue
        n += 1
        c += int(clicked[r])
        k = (t, target[r], tbin[r] if tbin is not None else 0)
        g = grp.get(k)
        if g is None:
            grp[k] = g = {"impr": 0, "clicks": 0, "w_rec_sum": 0.0, "max_pos": pos}
        g["impr"] += 1
        g["clicks"] += int(clicked[r])
        g["w_rec_sum"] += w
        g["max_pos"] = max(g["max_pos"], pos)
    p0 = c / n if n else 0.019
    for g in grp.values():
        v = beta_smooth(g["clicks"], g["impr"], p0, S)
        g["ctr"] = min(max(v, ctr_clip[0]), ctr_clip[1])
        g["is_lowcount"] = g["impr"] < min_impr
    return grp, p0


AGG_ORDER = ("sum_ctr", "mean_ctr", "max_ctr", "top_mean_ctr", "wmean_ctr", "sum_impr", "max_impr", "pnorm_ctr")


def row_features(ex, rows, target, tbin, table, topn):
    """covis.py:233-292 for the source rows in ``rows``: {row: [8 values in AGG_ORDER]}."""
    want = set(rows)
    per = {}
    for (r, t, pos, w) in ex:
        if r in want:
            per.setdefault(r, []).append((t, w))
    out = {}
    for r in rows:
        ctrs, imprs, wsum, wnum = [], [], 0.0, 0.0
        for (t, w) in per[r]:
            tb = tbin[r] if tbin is not None else 0
            g = None if (t is None or target[r] is None or tb is None) else table.get((t, target[r], tb))
            ctr = None if g is None else g["ctr"]
            imprs.append(0 if g is None else g["impr"])
            ctrs.append(ctr)
            wsum += w
            if ctr is not None:
                wnum += ctr * w
        vals = [v for v in ctrs if v is not None]
        n = len(vals)
        nulls = len(ctrs) - n
        head = sorted(vals, reverse=True)[:max(0, topn - nulls)]     # nulls first, then descending
        s = 0.0
        for v in vals:
            s += v
        ss = 0.0
        for v in vals:
            ss += v * v
        hs = 0.0
        for v in head:
            hs += v
        out[r] = [s, s / n if n else 0.0, max(vals) if n else 0.0, hs / len(head) if head else 0.0,
                  wnum / wsum, float(sum(imprs)), float(max(imprs)), math.sqrt(ss / n) if n else 0.0]
    return out


def make_folds(group_hash, n_folds):
    """covis.py:113-150: fold of each row from the rank of its group hash among the sorted distinct ones."""
    uniq = sorted(set(int(g) for g in group_hash))
    rank = {g: i for i, g in enumerate(uniq)}
    return np.array([rank[int(g)] % n_folds for g in group_hash], dtype=np.int64)
