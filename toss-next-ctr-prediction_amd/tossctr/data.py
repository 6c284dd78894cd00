"""NPY shard cache + manifest (the on-disk format of src/data/build_cache_v1.py:169-307) and its readers.

Host-side mirror of src/data/dataset.py (ShardedDataset / load_labels_groups_for_split /
collate_sharded) for drop-in use, plus ``DeviceShards``: the MI355X input path.  The reference feeds
the GPU through a per-row Python ``__getitem__`` + ``np.stack`` collate in DataLoader workers (~33 k
rows/s measured in the survey); here every shard column is staged ONCE into HBM (a 1 M-row cfg2 shard
is ~1 GB, tiny against 288 GB) and a batch is assembled on device by ``ctr_gather_rows`` from the fold's
permuted index -- no host round trip per step.
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from . import _lib

ARRAYS = ["X_num", "X_mask", "X_cat", "seq", "y", "groups", "ids"]


# ---------------------------------------------------------------------------- writer
def write_shard_cache(out_dir, arrays, shard_rows=2_000_000, *, num_cols=None, cat_cols=None, group_key="",
                      seq_col="seq", is_train=True, parquet=""):
    """Write arrays {X_num f32 (N,Fn), X_mask u8, X_cat i32, seq i32 (N,L), y i8, groups i64, ids} as
    shard_XXX/<name>.npy + manifest.json, exactly the reference layout (build_cache_v1.py:169-177,
    223-238, 273-307).  Returns the manifest path."""
    os.makedirs(out_dir, exist_ok=True)
    n = arrays["seq"].shape[0]
    man = {"parquet": parquet, "is_train": is_train, "rows": 0, "shards": [], "num_cols": list(num_cols or []),
           "cat_cols": list(cat_cols or []), "group_key": group_key, "seq_col": seq_col}
    for si, s0 in enumerate(range(0, max(n, 1), shard_rows)):
        s1 = min(n, s0 + shard_rows)
        sdir = os.path.join(out_dir, f"shard_{si:03d}")
        os.makedirs(sdir, exist_ok=True)
        meta = {}
        for k in ARRAYS:
            v = arrays[k][s0:s1]
            path = os.path.join(sdir, f"{k}.npy")
            np.save(path, v)
            meta[k] = {"path": path, "shape": list(v.shape), "dtype": str(v.dtype)}
        meta["rows"] = s1 - s0
        meta["index"] = si
        meta["start"] = man["rows"]
        meta["end"] = man["rows"] + meta["rows"]
        man["shards"].append(meta)
        man["rows"] += meta["rows"]
    path = os.path.join(out_dir, "manifest.json")
    with open(path, "w") as f:
        json.dump(man, f, indent=2)
    return path


def synth_rows(n, Fn, Fm, cards, L, vocab, seed, pos_rate=0.019, pad_id=0):
    """SURVEY §8(d) synthetic rows in the reference's on-disk dtypes."""
    r = np.random.default_rng(seed)
    X_mask = (r.random((n, Fm)) < 0.1).astype(np.uint8)
    X_num = r.standard_normal((n, Fn)).astype(np.float32)
    if Fn == Fm:
        X_num[X_mask.astype(bool)] = 0.0
    X_cat = np.stack([r.integers(0, c, n) for c in cards], axis=1).astype(np.int32)
    lens = r.integers(0, L + 1, n)
    toks = r.integers(1, vocab, (n, L)).astype(np.int32)
    seq = np.where(np.arange(L)[None, :] >= (L - lens)[:, None], toks, pad_id).astype(np.int32)
    y = (r.random(n) < pos_rate).astype(np.int8)
    groups = r.integers(0, 2**31 - 1, n).astype(np.int64)
    ids = np.array([f"ID_{i:08d}" for i in range(n)])
    return dict(X_num=X_num, X_mask=X_mask, X_cat=X_cat, seq=seq, y=y, groups=groups, ids=ids)


# ---------------------------------------------------------------------------- host readers (compat)
class ShardedNPY:
    """src/data/dataset.py:8-43: lazily mmap one shard's arrays."""

    def __init__(self, meta):
        self.paths = {k: meta[k]["path"] for k in ARRAYS}
        self.rows = meta["rows"]
        self.arrs = {}

    def open(self):
        for k, p in self.paths.items():
            if os.path.exists(p):
                self.arrs[k] = np.load(p, allow_pickle=False) if k == "ids" else np.load(p, mmap_mode="r")
            else:
                self.arrs[k] = None

    def get_row(self, i, train):
        if not self.arrs:
            self.open()
        out = {k: self.arrs[k][i] for k in ("X_num", "X_mask", "X_cat", "seq", "groups")}
        if not train and self.arrs.get("ids") is not None:
            out["ids"] = self.arrs["ids"][i]
        if train:
            out["y"] = self.arrs["y"][i]
        return out


class ShardedDataset(torch.utils.data.Dataset):
    """src/data/dataset.py:45-80 (same signature): global index -> (shard, local row)."""

    def __init__(self, manifest_path, index, train, cat_cols):
        with open(manifest_path) as f:
            self.manifest = json.load(f)
        self.index = np.asarray(index).astype(np.int64)
        self.train = train
        self.cat_cols = cat_cols
        self.shards = [ShardedNPY(m) for m in self.manifest["shards"]]
        b = np.array([(m["start"], m["end"]) for m in self.manifest["shards"]], dtype=np.int64).reshape(-1, 2)
        self.starts, self.ends = b[:, 0], b[:, 1]

    def __len__(self):
        return self.index.shape[0]

    def _locate(self, g):
        s = int(np.searchsorted(self.ends, g, side="right"))
        return s, int(g - self.starts[s])

    def __getitem__(self, i):
        sid, li = self._locate(int(self.index[i]))
        return self.shards[sid].get_row(li, self.train)


def load_labels_groups_for_split(manifest_path):
    """src/data/dataset.py:82-96."""
    with open(manifest_path) as f:
        man = json.load(f)
    ys = [np.asarray(np.load(m["y"]["path"], mmap_mode="r")) for m in man["shards"]]
    gs = [np.asarray(np.load(m["groups"]["path"], mmap_mode="r")) for m in man["shards"]]
    return np.concatenate(ys), np.concatenate(gs)


def collate_sharded(batch):
    """src/data/dataset.py:98-124."""
    keys = batch[0].keys()

    def st(name, dtype):
        return torch.from_numpy(np.ascontiguousarray(np.stack([b[name] for b in batch], 0)).astype(dtype, copy=False))

    out = {"X_num": st("X_num", np.float32), "X_mask": st("X_mask", np.float32), "X_cat": st("X_cat", np.int64),
           "seq": st("seq", np.int64)}
    if "y" in keys:
        out["y"] = torch.from_numpy(np.asarray([b["y"] for b in batch], dtype=np.float32))
    if "ids" in keys:
        out["ids"] = np.asarray([b["ids"] for b in batch])
    if "groups" in keys:
        out["groups"] = torch.from_numpy(np.asarray([b["groups"] for b in batch], dtype=np.int64))
    return out


# ---------------------------------------------------------------------------- device path
class DeviceShards:
    """All rows of a manifest staged in HBM in the kernels' dtypes (X_num f32, X_mask f32, X_cat i32,
    seq i32, y f32); ``batch(idx)`` gathers rows on device (ctr_gather_rows)."""

    def __init__(self, manifest_path, device):
        with open(manifest_path) as f:
            man = json.load(f)
        self.device = torch.device(device)
        cols = {"X_num": np.float32, "X_mask": np.float32, "X_cat": np.int32, "seq": np.int32, "y": np.float32}
        self.t = {}
        for k, dt in cols.items():
            parts = []
            for m in man["shards"]:
                a = np.load(m[k]["path"], mmap_mode="r")
                # a read-only mmap stays read-only through astype(copy=False): copy it (it is staged to the
                # device right after, so the host copy is transient)
                parts.append(torch.from_numpy(np.array(a, dtype=dt, copy=True)))
            host = torch.cat(parts) if parts else torch.zeros(0)
            if host.dim() == 1:
                host = host[:, None]
            self.t[k] = host.to(self.device).contiguous()
        self.rows = int(man["rows"])
        self._out = {}

    def _get(self, name, shape, dtype):
        t = self._out.get(name)
        if t is None or tuple(t.shape) != tuple(shape):
            t = torch.empty(shape, dtype=dtype, device=self.device)
            self._out[name] = t
        return t

    def batch(self, idx: torch.Tensor, slot=0):
        """idx: int64 device tensor of global row ids.  Returns ((X_num, X_mask, X_cat, seq), y)."""
        n = int(idx.numel())
        st = torch.cuda.current_stream(self.device).cuda_stream
        out = []
        for k in ("X_num", "X_mask", "X_cat", "seq", "y"):
            src = self.t[k]
            dst = self._get(f"{k}{slot}", (n, src.shape[1]), src.dtype)
            _lib.call("ctr_gather_rows", src.data_ptr(), src.shape[1], idx.data_ptr(), n, dst.data_ptr(), st)
            out.append(dst)
        return tuple(out[:4]), out[4].view(-1)
