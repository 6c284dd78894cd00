"""Co-visitation feature build cost at the reference's data scale: device pair statistics (one full-train
pass and one out-of-fold pass) and row features (csrc/covis.hip) over N rows x ~top_k exploded tokens, vs a
vectorised numpy group-by + join on a bounded sample of the same rows on the host (polars, the reference's
engine, is not installed here).  Not part of the product.

    python tools/covis_bench.py [--rows 10700000] [--mean-len 100]
"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "toss-next-ctr-prediction_amd"))

import torch  # noqa: E402

from tossctr.covis import CoVisCfg, ExplodedSplit, pair_stats, row_features  # noqa: E402


def synth(rows, mean_len, top_k, vocab, seed):
    rng = np.random.default_rng(seed)
    lens = np.clip(rng.poisson(mean_len, rows), 0, top_k).astype(np.int64)
    lens = np.maximum(lens, 1)                              # an empty seq explodes to one null
    row_ptr = np.zeros(rows + 1, np.int64)
    np.cumsum(lens, out=row_ptr[1:])
    n = int(row_ptr[-1])
    tok = (rng.zipf(1.3, n) % vocab).astype(np.int32)       # skewed token popularity
    ok = np.ones(n, np.uint8)
    starts = np.repeat(row_ptr[:-1], lens)
    pos = (np.arange(n, dtype=np.int64) - starts).astype(np.int32)
    tgt = rng.integers(0, 2000, rows).astype(np.int32)      # ~inventory_id cardinality
    tb = rng.integers(0, 7, rows).astype(np.int32)          # day_of_week
    click = (rng.random(rows) < 0.019).astype(np.uint8)
    return row_ptr, tok, pos, ok, tgt, tb, click


def host_numpy(row_ptr, tok, tgt, tb, click, pos, tau, S, clip):
    """numpy group-by (unique over packed keys) + join (searchsorted) + per-row sums: the same work."""
    lens = np.diff(row_ptr)
    erow = np.repeat(np.arange(len(lens)), lens)
    key = ((tok.astype(np.int64) + 2**31) << 32) | (tgt[erow].astype(np.int64) << 3) | tb[erow]
    uk, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    clk = np.bincount(inv, weights=click[erow], minlength=len(uk))
    w = np.exp(-pos / tau)
    wsum = np.bincount(inv, weights=w, minlength=len(uk))
    p0 = click[erow].mean()
    ctr = np.clip(np.clip((clk + p0 * S) / (cnt + S), 1e-9, 1 - 1e-9), *clip)
    j = np.searchsorted(uk, key)
    c = ctr[j]
    feats = np.add.reduceat(c, row_ptr[:-1]), np.add.reduceat(c * w, row_ptr[:-1]), wsum
    return feats


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_700_000)
    ap.add_argument("--mean-len", type=float, default=100.0)
    ap.add_argument("--vocab", type=int, default=1_000_000)
    ap.add_argument("--host-rows", type=int, default=400_000)
    args = ap.parse_args()
    cfg = CoVisCfg(train_path="", test_path="")
    t0 = time.perf_counter()
    row_ptr, tok, pos, ok, tgt, tb, click = synth(args.rows, args.mean_len, cfg.seq_top_k, args.vocab, 0)
    n = int(row_ptr[-1])
    print(f"rows {args.rows}, exploded {n} ({time.perf_counter() - t0:.1f} s to synthesise)", flush=True)
    dev = torch.device("cuda")
    ex = ExplodedSplit(row_ptr, tok, pos, ok, dev)
    tg, tbd, ck = (torch.from_numpy(a).to(dev) for a in (tgt, tb, click))
    keep = (torch.arange(args.rows, device=dev) % 5 != 0).to(torch.uint8)
    rows = torch.arange(args.rows, device=dev, dtype=torch.int64)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    pt = pair_stats(ex, tg, tbd, ck, None, 3, cfg)          # warm-up (workspace allocation)
    F = row_features(ex, rows, tg, tbd, 3, pt, cfg)
    torch.cuda.synchronize()
    ev[0].record()
    pt = pair_stats(ex, tg, tbd, ck, None, 3, cfg, pt.ws)
    ev[1].record()
    pt2 = pair_stats(ex, tg, tbd, ck, keep, 3, cfg, pt.ws)
    ev[2].record()
    F = row_features(ex, rows, tg, tbd, 3, pt, cfg)
    ev[3].record()
    torch.cuda.synchronize()
    t_full, t_oof, t_rows = (ev[i].elapsed_time(ev[i + 1]) for i in range(3))
    print(f"device: pair stats (full) {t_full:.1f} ms = {n / t_full / 1e6:.2f} G exploded/s, "
          f"{pt.n_pairs} pairs; OOF pass {t_oof:.1f} ms ({pt2.n_pairs} pairs); row features {t_rows:.1f} ms = "
          f"{args.rows / t_rows / 1e3:.1f} M rows/s ({n / t_rows / 1e6:.2f} G exploded/s)", flush=True)
    per_fold = t_oof + t_rows / 5
    print(f"device: 5 folds + full + test-sized rows ~ {5 * per_fold + t_full + t_rows:.0f} ms per target key")
    hr = min(args.host_rows, args.rows)
    h_ptr = row_ptr[:hr + 1]
    hn = int(h_ptr[-1])
    t0 = time.perf_counter()
    host_numpy(h_ptr, tok[:hn], tgt[:hr], tb[:hr], click[:hr], pos[:hn], cfg.recency_tau, cfg.prior_strength,
               cfg.ctr_clip)
    th = time.perf_counter() - t0
    print(f"host numpy (1 thread, sample of {hr} rows / {hn} exploded): group-by + join {th * 1e3:.0f} ms = "
          f"{hn / th / 1e6:.2f} M exploded/s -> full pass at this rate ~{n / (hn / th):.0f} s")


if __name__ == "__main__":
    main()
