"""Co-visitation features (drop-in for src/features/covis.py + src/tools/build_covis_features.py).

The reference builds, with polars on the host, (token, target[, time_bin]) statistics of the exploded
``seq`` column -- impressions, clicks, recency-weighted counts and a beta-smoothed CTR -- for the full
train set and out-of-fold per fold, then left-joins every row's recent tokens on them and aggregates the
matches into numeric columns that build_cache_v2 appends to X_num.  Here:

  * the seq column is exploded once per split on the host, natively (csrc/hostio.cpp
    ``ctr_covis_explode``: split / non-strict Int32 cast / last ``seq_top_k`` / cum_count positions), and
    staged in HBM;
  * the group-by is a device radix sort of packed u64 pair keys + run-length groups
    (csrc/covis.hip ``ctr_covis_pair_stats``), re-run per fold with a row keep-mask -- the exploded
    arrays stay resident across the 5 OOF passes and the full pass;
  * the join + aggregation is one thread per row binary-searching the sorted pair keys
    (``ctr_covis_row_features``).

Files written (same names as the reference): folds.parquet, pair_full_<tgt>.parquet,
pair_oof_f<f>_<tgt>.parquet, rowfeat_oof_f<f>.parquet (global train ``rid``), rowfeat_test.parquet
(``ID``), rowfeat_oof_all.parquet.  ``tossctr.build_cache.build_sharded_cache(covis_enabled=True)`` joins
them the way build_cache_v2.py:208-287 does.

Deviations (the reference does not run under its own pinned polars >= 1.5; parity
with the restatement in oracle/covis.py):
  * group hashes use the build's XXH64 replacement of polars' hash (as tossctr/build_cache.py);
  * the wmean column is named ``<tgt>_wmean_ctr`` (the reference's ``.alias`` binds to the denominator, so
    polars would name it ``ctr_<tgt>``);
  * pair-table groups with a null key part are not written (the join can never match them);
  * ``rid`` in the OOF row features is the global train row index, the key build_cache_v2 joins on.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _lib

AGG_INDEX = {"sum_ctr": 0, "mean_ctr": 1, "max_ctr": 2, "top3_mean_ctr": 3, "wmean_ctr": 4, "sum_impr": 5,
             "max_impr": 6, "pnorm_ctr": 7}


@dataclass
class CoVisCfg:
    """covis.py:10-45 (same fields and defaults)."""
    train_path: str
    test_path: str
    seq_col: str = "seq"
    id_col_test: str = "ID"
    target_keys: List[str] = None
    use_time_bin: bool = True
    time_bin: str = "day_of_week"
    seq_top_k: int = 120
    recency_tau: int = 512
    min_impr: int = 10
    prior_strength: int = 50
    ctr_clip: Tuple[float, float] = (1e-3, 0.999)
    backoff: List[str] = None
    agg_topn: int = 3
    agg_outputs: List[str] = None
    n_folds: int = 5
    group_key: str = "inventory_id"
    time_key: Optional[str] = "day_of_week"
    composite_group: bool = True
    work_dir: str = "./cache/covis"

    def __post_init__(self):
        if self.target_keys is None:
            self.target_keys = ["inventory_id"]
        if self.backoff is None:
            self.backoff = ["pair", "token", "target", "global"]
        if self.agg_outputs is None:
            self.agg_outputs = ["sum_ctr", "mean_ctr", "max_ctr", "top3_mean_ctr", "wmean_ctr", "sum_impr",
                                "max_impr", "pnorm_ctr"]


def _pa():
    import pyarrow as pa
    import pyarrow.compute as pc
    import pyarrow.parquet as pq
    return pa, pc, pq


# ------------------------------------------------------------------------------ host side
def explode_seq(arr, top_k: int):
    """covis.py:60-80 + :174-183 over an Arrow string column -> (row_ptr int64 (n+1), tok, pos int32, ok u8)."""
    from .build_cache import _string_buffers
    pa, pc, _ = _pa()
    if isinstance(arr, pa.ChunkedArray):
        arr = arr.combine_chunks() if arr.num_chunks != 1 else arr.chunk(0)
    off, data, valid = _string_buffers(arr)
    n = len(off) - 1
    row_ptr = np.empty(n + 1, dtype=np.int64)
    total = _lib.query("ctr_covis_explode_count", off.ctypes.data, data.ctypes.data,
                       valid.ctypes.data if valid is not None else None, n, int(top_k), row_ptr.ctypes.data)
    if total < 0:
        raise ValueError("ctr_covis_explode_count: malformed string buffers")
    tok = np.empty(max(total, 1), np.int32)
    pos = np.empty(max(total, 1), np.int32)
    ok = np.empty(max(total, 1), np.uint8)
    rc = _lib.query("ctr_covis_explode", off.ctypes.data, data.ctypes.data,
                    valid.ctypes.data if valid is not None else None, n, int(top_k), row_ptr.ctypes.data,
                    tok.ctypes.data, pos.ctypes.data, ok.ctypes.data)
    if rc != 0:
        raise ValueError("ctr_covis_explode failed")
    return row_ptr, tok[:total], pos[:total], ok[:total]


def time_bin_values(tbl, cfg: CoVisCfg) -> np.ndarray:
    """_make_timebin_expr (covis.py:97-103): int64 per row, -1 for null (all 0 without time bins)."""
    pa, pc, _ = _pa()
    n = tbl.num_rows
    if not cfg.use_time_bin:
        return np.zeros(n, np.int64)

    def col(name):
        c = pc.cast(tbl.column(name), pa.int32())
        return (np.asarray(pc.fill_null(c, 0).to_numpy(zero_copy_only=False), np.int64),
                np.asarray(pc.is_null(c).to_numpy(zero_copy_only=False), bool))
    if cfg.time_bin == "day_of_week_hour":
        (d, dn), (h, hn) = col("day_of_week"), col("hour")
        v, nul = d * 24 + h, dn | hn
    else:
        v, nul = col(cfg.time_bin)
    return np.where(nul, -1, v)


def encode_codes(*cols):
    """Dense codes over the union of several Arrow columns (nulls -> -1) and the values per code."""
    pa, pc, _ = _pa()
    chunks = []
    for c in cols:
        chunks += c.chunks if isinstance(c, pa.ChunkedArray) else [c]
    typ = chunks[0].type
    ca = pa.chunked_array([ch.cast(typ) for ch in chunks], type=typ).combine_chunks()
    d = pc.dictionary_encode(ca)
    idx = np.asarray(pc.fill_null(d.indices, -1).to_numpy(zero_copy_only=False), np.int64)
    out, o = [], 0
    for c in cols:
        out.append(idx[o:o + len(c)].astype(np.int32))
        o += len(c)
    return out, d.dictionary


def _tb_codes(*tbs):
    vals = np.unique(np.concatenate([t[t >= 0] for t in tbs])) if any((t >= 0).any() for t in tbs) else \
        np.zeros(0, np.int64)
    bits = max(1, int(math.ceil(math.log2(max(len(vals), 2)))))
    codes = [np.where(t >= 0, np.searchsorted(vals, np.where(t >= 0, t, vals[0] if len(vals) else 0)), -1)
             .astype(np.int32) for t in tbs]
    return codes, vals, bits


# ------------------------------------------------------------------------------ device side
class ExplodedSplit:
    """One split's exploded seq column resident in HBM, plus per-row codes per target."""

    def __init__(self, row_ptr, tok, pos, ok, device):
        import torch
        self.device = torch.device(device)
        self.n_rows = len(row_ptr) - 1
        self.n = int(row_ptr[-1])
        if self.n >= 2**32:
            raise ValueError("covis: more than 2^32 exploded tokens in one split")
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.device)
        self.row_ptr = t(row_ptr)
        self.tok, self.pos, self.ok = t(tok), t(pos), t(ok)
        self.erow = torch.repeat_interleave(torch.arange(self.n_rows, dtype=torch.int32, device=self.device),
                                            t(np.diff(row_ptr)), output_size=self.n)


class PairTable:
    def __init__(self, keys, impr, clicks, w_rec_sum, max_pos, ctr, lowcount, n_pairs, p0):
        self.keys, self.impr, self.clicks, self.w_rec_sum = keys, impr, clicks, w_rec_sum
        self.max_pos, self.ctr, self.lowcount, self.n_pairs_dev, self.p0_dev = max_pos, ctr, lowcount, n_pairs, p0

    @property
    def n_pairs(self):
        return int(self.n_pairs_dev.item())

    @property
    def p0(self):
        return float(self.p0_dev.item())

    def to_host(self, tb_bits):
        """dict of numpy columns: token, tgt code, tb code, impr, clicks, w_rec_sum, max_pos, ctr, is_lowcount."""
        n = self.n_pairs
        k = self.keys[:n].cpu().numpy().view(np.uint64)
        tok = ((k >> np.uint64(32)).astype(np.uint32) ^ np.uint32(0x80000000)).view(np.int32)
        low = (k & np.uint64(0xFFFFFFFF)).astype(np.uint64)
        return {"token": tok, "tgt": (low >> np.uint64(tb_bits)).astype(np.int64),
                "tb": (low & np.uint64((1 << tb_bits) - 1)).astype(np.int64),
                "impr": self.impr[:n].cpu().numpy().astype(np.uint32), "clicks": self.clicks[:n].cpu().numpy(),
                "w_rec_sum": self.w_rec_sum[:n].cpu().numpy(), "max_pos": self.max_pos[:n].cpu().numpy().astype(np.int64),
                "ctr": self.ctr[:n].cpu().numpy(), "is_lowcount": self.lowcount[:n].cpu().numpy().astype(bool)}


def _stream(dev):
    import torch
    return torch.cuda.current_stream(dev).cuda_stream


def pair_stats(ex: ExplodedSplit, tgt, tb, click, keep, tb_bits: int, cfg: CoVisCfg, ws=None) -> PairTable:
    """_pair_stats_from_scan (covis.py:155-213) on device.  tgt / tb: int32 codes per row (-1 null) as device
    tensors; click: uint8; keep: uint8 per row or None (all rows)."""
    import torch
    d = ex.device
    cap = max(ex.n, 1)
    need = int(_lib.query("ctr_covis_ws_size", ex.n))
    if ws is None or ws.numel() < need:
        ws = torch.empty(need, dtype=torch.uint8, device=d)
    e = lambda dt: torch.empty(cap, dtype=dt, device=d)
    pt = PairTable(e(torch.int64), e(torch.int32), e(torch.int64), e(torch.float64), e(torch.int32),
                   e(torch.float64), e(torch.uint8), torch.zeros(1, dtype=torch.int64, device=d),
                   torch.zeros(1, dtype=torch.float64, device=d))
    lo, hi = cfg.ctr_clip
    _lib.call("ctr_covis_pair_stats", ex.tok.data_ptr(), ex.pos.data_ptr(), ex.ok.data_ptr(), ex.erow.data_ptr(),
              ex.n, tgt.data_ptr(), tb.data_ptr(), click.data_ptr(), keep.data_ptr() if keep is not None else None,
              int(tb_bits), float(cfg.recency_tau), float(cfg.prior_strength), float(lo), float(hi), int(cfg.min_impr),
              pt.keys.data_ptr(), pt.impr.data_ptr(), pt.clicks.data_ptr(), pt.w_rec_sum.data_ptr(),
              pt.max_pos.data_ptr(), pt.ctr.data_ptr(), pt.lowcount.data_ptr(), pt.n_pairs_dev.data_ptr(),
              pt.p0_dev.data_ptr(), ws.data_ptr(), ws.numel(), _stream(d))
    pt.ws = ws
    return pt


def row_features(ex: ExplodedSplit, rows, tgt, tb, tb_bits: int, pt: PairTable, cfg: CoVisCfg):
    """_row_features_from_pair_tbl (covis.py:233-292) for source rows ``rows`` (int64 device tensor) ->
    (len(rows), 8) float64 device tensor in AGG_INDEX order."""
    import torch
    nq = rows.numel()
    out = torch.empty((max(nq, 1), 8), dtype=torch.float64, device=ex.device)
    _lib.call("ctr_covis_row_features", rows.data_ptr(), nq, ex.row_ptr.data_ptr(), ex.tok.data_ptr(),
              ex.pos.data_ptr(), ex.ok.data_ptr(), tgt.data_ptr(), tb.data_ptr(), int(tb_bits),
              float(cfg.recency_tau), pt.keys.data_ptr(), pt.ctr.data_ptr(), pt.impr.data_ptr(),
              pt.n_pairs_dev.data_ptr(), int(cfg.agg_topn), out.data_ptr(), _stream(ex.device))
    return out[:nq]


# ------------------------------------------------------------------------------ pipeline
def make_folds(cfg: CoVisCfg, tbl=None):
    """covis.py:113-150: (rid, fold) with folds dealt round-robin over the sorted distinct group hashes."""
    from .build_cache import hash_strings
    pa, pc, pq = _pa()
    if tbl is None:
        cols = [cfg.group_key] + ([cfg.time_key] if cfg.composite_group and cfg.time_key else [])
        tbl = pq.read_table(cfg.train_path, columns=cols)
    gs = pc.fill_null(pc.cast(tbl.column(cfg.group_key), pa.string()), "NA")
    if cfg.composite_group and cfg.time_key is not None:
        ts = pc.fill_null(pc.cast(tbl.column(cfg.time_key), pa.string()), "NA")
        g = hash_strings(pc.binary_join_element_wise(gs, ts, "\x1f"))
    else:
        g = hash_strings(gs)
    uniq, inv = np.unique(g, return_inverse=True)
    return np.arange(len(g), dtype=np.int64), (inv % cfg.n_folds).astype(np.int64)


def _feature_names(cfg: CoVisCfg, tgt: str):
    names = []
    for a in cfg.agg_outputs:
        if a not in AGG_INDEX:
            raise ValueError(f"covis: unknown agg output {a!r}")
        names.append(f"{tgt}_top{cfg.agg_topn}_mean_ctr" if a == "top3_mean_ctr" else f"{tgt}_{a}")
    return names


class _Split:
    def __init__(self, tbl, cfg, device, tgt_codes, tb_codes):
        import torch
        rp, tok, pos, ok = explode_seq(tbl.column(cfg.seq_col), cfg.seq_top_k)
        self.ex = ExplodedSplit(rp, tok, pos, ok, device)
        self.tgt = {k: torch.from_numpy(v).to(device) for k, v in tgt_codes.items()}
        self.tb = torch.from_numpy(tb_codes).to(device)


def _pair_table_arrow(host, tgt, tgt_dict, tb_vals, cfg):
    pa, pc, _ = _pa()
    cols = {"token": pa.array(host["token"], pa.int32()),
            tgt: pc.take(tgt_dict, pa.array(host["tgt"]))}
    if cfg.use_time_bin:
        cols["time_bin"] = pa.array(tb_vals[host["tb"]].astype(np.int32) if len(tb_vals) else
                                    np.zeros(len(host["tb"]), np.int32))
    for k in ("impr", "clicks", "w_rec_sum", "max_pos", "ctr", "is_lowcount"):
        cols[k] = pa.array(host[k])
    return pa.table(cols)


def build_all(cfg: CoVisCfg, device="cuda", write_pairs: bool = True):
    """build_covis_features.py main: folds, pair stats (full + OOF), row features (OOF + test) and
    rowfeat_oof_all.  Returns the work_dir."""
    import torch
    pa, pc, pq = _pa()
    os.makedirs(cfg.work_dir, exist_ok=True)
    dev = torch.device(device)
    tcols = {cfg.seq_col, "clicked", *cfg.target_keys}
    if cfg.use_time_bin:
        tcols |= {"day_of_week", "hour"} if cfg.time_bin == "day_of_week_hour" else {cfg.time_bin}
    tr = pq.read_table(cfg.train_path, columns=sorted(tcols))
    te_cols = sorted((tcols - {"clicked"}) | {cfg.id_col_test})
    te = pq.read_table(cfg.test_path, columns=te_cols)

    rid, fold = make_folds(cfg)
    pq.write_table(pa.table({"rid": pa.array(rid.astype(np.uint32)), "fold": pa.array(fold)}),
                   os.path.join(cfg.work_dir, "folds.parquet"))

    tgt_tr, tgt_te, tgt_dict = {}, {}, {}
    for k in cfg.target_keys:
        (a, b), dic = encode_codes(tr.column(k), te.column(k))
        tgt_tr[k], tgt_te[k], tgt_dict[k] = a, b, dic
    (tb_tr, tb_te), tb_vals, tb_bits = _tb_codes(time_bin_values(tr, cfg), time_bin_values(te, cfg))
    for k in cfg.target_keys:
        if len(tgt_dict[k]) >= (1 << (32 - tb_bits)) - 1:
            raise ValueError(f"covis: target {k!r} has too many distinct values for the packed pair key")
    S_tr = _Split(tr, cfg, dev, tgt_tr, tb_tr)
    click = torch.from_numpy(np.array(pc.fill_null(pc.cast(tr.column("clicked"), pa.uint8()), 0)
                                      .to_numpy(zero_copy_only=False), np.uint8)).to(dev)
    fold_d = torch.from_numpy(fold).to(dev)
    ws = None
    feats = []
    for f in range(cfg.n_folds):
        keep = (fold_d != f).to(torch.uint8)
        val = torch.nonzero(fold_d == f).flatten().to(torch.int64)
        cols = {"rid": pa.array(val.cpu().numpy())}
        for k in cfg.target_keys:
            pt = pair_stats(S_tr.ex, S_tr.tgt[k], S_tr.tb, click, keep, tb_bits, cfg, ws)
            ws = pt.ws
            if write_pairs:
                pq.write_table(_pair_table_arrow(pt.to_host(tb_bits), k, tgt_dict[k], tb_vals, cfg),
                               os.path.join(cfg.work_dir, f"pair_oof_f{f}_{k}.parquet"))
            F = row_features(S_tr.ex, val, S_tr.tgt[k], S_tr.tb, tb_bits, pt, cfg).cpu().numpy()
            for name, a in zip(_feature_names(cfg, k), cfg.agg_outputs):
                cols[name] = pa.array(F[:, AGG_INDEX[a]])
        t = pa.table(cols)
        pq.write_table(t, os.path.join(cfg.work_dir, f"rowfeat_oof_f{f}.parquet"))
        feats.append(t)
    pq.write_table(pa.concat_tables(feats), os.path.join(cfg.work_dir, "rowfeat_oof_all.parquet"))

    # test rows against the full-train pair tables
    S_te = _Split(te, cfg, dev, tgt_te, tb_te)
    rows = torch.arange(S_te.ex.n_rows, dtype=torch.int64, device=dev)
    cols = {}
    for k in cfg.target_keys:
        pt = pair_stats(S_tr.ex, S_tr.tgt[k], S_tr.tb, click, None, tb_bits, cfg, ws)
        ws = pt.ws
        if write_pairs:
            pq.write_table(_pair_table_arrow(pt.to_host(tb_bits), k, tgt_dict[k], tb_vals, cfg),
                           os.path.join(cfg.work_dir, f"pair_full_{k}.parquet"))
        F = row_features(S_te.ex, rows, S_te.tgt[k], S_te.tb, tb_bits, pt, cfg).cpu().numpy()
        for name, a in zip(_feature_names(cfg, k), cfg.agg_outputs):
            cols[name] = pa.array(F[:, AGG_INDEX[a]])
    ids = pc.cast(te.column(cfg.id_col_test), pa.string())
    pq.write_table(pa.table({**cols, "ID": ids}), os.path.join(cfg.work_dir, "rowfeat_test.parquet"))
    return cfg.work_dir


def cfg_from_yaml(cfg: dict) -> CoVisCfg:
    """src/tools/build_covis_features.py:6-31."""
    d, s, fc = cfg["data"], cfg["sequence"], cfg["features"]["covis"]
    return CoVisCfg(train_path=d["train_path"], test_path=d["test_path"], seq_col=s["col"], id_col_test="ID",
                    target_keys=fc["target_keys"], use_time_bin=fc["use_time_bin"], time_bin=fc["time_bin"],
                    seq_top_k=fc["seq_top_k"], recency_tau=fc["recency_tau"], min_impr=fc["min_impr"],
                    prior_strength=fc["prior_strength"], ctr_clip=tuple(fc["ctr_clip"]), backoff=fc["backoff"],
                    agg_topn=int(fc["agg"]["topn"]), agg_outputs=fc["agg"]["outputs"],
                    n_folds=cfg["cv"]["n_splits"], group_key=cfg["cv"]["group_key"],
                    time_key=cfg["cv"].get("time_key"), composite_group=bool(cfg["cv"].get("composite_group", False)),
                    work_dir=fc["work_dir"])


def main(cfg_path: str, device="cuda"):
    import yaml
    with open(cfg_path) as fh:
        cfg = yaml.safe_load(fh)
    out = build_all(cfg_from_yaml(cfg), device=device)
    print("[ok] CoVis features built:", out)


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=str, required=True)
    main(ap.parse_args().cfg)
