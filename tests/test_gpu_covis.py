"""Co-visitation pair statistics and row features on device (csrc/covis.hip through the C ABI) against the
plain-Python restatement of src/features/covis.py (oracle/covis.py): every pair group (integer columns
exact, f64 columns within 1e-12 relative -- the device and host exp differ by an ulp), every row aggregate,
out-of-fold keep masks, null targets / time bins / tokens, then the whole build_covis_features pipeline on
Parquet files and the shard builder's join.  Parity vs polars: unpinned (see oracle/covis.py)."""
import random

import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")
pq = pytest.importorskip("pyarrow.parquet")

from oracle import covis as ocv

pytestmark = pytest.mark.gpu

RTOL = 1e-12


def _data(n, seed, vocab=40, junk=("", "bad")):
    rng = random.Random(seed)
    seqs = []
    for i in range(n):
        if i % 23 == 0:
            seqs.append(None)
            continue
        toks = [str(rng.randrange(1, vocab)) for _ in range(rng.randrange(1, 30))]
        if i % 9 == 0:
            toks.insert(rng.randrange(0, len(toks)), rng.choice(junk))
        seqs.append(",".join(toks))
    tgt = [None if i % 29 == 0 else rng.choice(["a", "b", "c", "d"]) for i in range(n)]
    dow = [None if i % 31 == 0 else rng.randrange(0, 7) for i in range(n)]
    hour = [rng.randrange(0, 24) for _ in range(n)]
    clicked = [int(rng.random() < 0.2) for _ in range(n)]
    return seqs, tgt, dow, hour, clicked


def _setup(seqs, tgt, dow, hour, cfg):
    import torch
    from tossctr.covis import ExplodedSplit, _tb_codes, encode_codes, explode_seq, time_bin_values
    rp, tok, pos, ok = explode_seq(pa.array(seqs, pa.string()), cfg.seq_top_k)
    ex = ExplodedSplit(rp, tok, pos, ok, "cuda")
    (codes,), dic = encode_codes(pa.array(tgt, pa.string()))
    tbl = pa.table({"day_of_week": pa.array(dow, pa.int64()), "hour": pa.array(hour, pa.int64())})
    (tbc,), vals, bits = _tb_codes(time_bin_values(tbl, cfg))
    return ex, torch.from_numpy(codes).cuda(), torch.from_numpy(tbc).cuda(), bits


@pytest.mark.parametrize("time_bin,top_k,topn,use_tb", [("day_of_week", 120, 3, True), ("day_of_week_hour", 7, 3, True),
                                                     ("hour", 3, 5, True), ("day_of_week", 10, 1, False)])
def test_pair_stats_and_row_features_match_restatement(time_bin, top_k, topn, use_tb):
    import torch
    from tossctr.covis import CoVisCfg, encode_codes, pair_stats, row_features
    n = 1500
    seqs, tgt, dow, hour, clicked = _data(n, seed=top_k + topn)
    cfg = CoVisCfg(train_path="", test_path="", time_bin=time_bin, seq_top_k=top_k, recency_tau=64,
                   min_impr=3, prior_strength=20, agg_topn=topn, use_time_bin=use_tb)
    ex, tg, tb, bits = _setup(seqs, tgt, dow, hour, cfg)
    click = torch.tensor(clicked, dtype=torch.uint8, device="cuda")
    fold = np.arange(n) % 4
    tbins = ocv.time_bins(dow, hour, time_bin) if use_tb else None
    oex = ocv.explode(seqs, top_k, float(cfg.recency_tau))
    for f in (None, 1):
        keep_h = [1] * n if f is None else (fold != f).astype(int).tolist()
        keep = None if f is None else torch.tensor(keep_h, dtype=torch.uint8, device="cuda")
        pt = pair_stats(ex, tg, tb, click, keep, bits, cfg)
        table, p0 = ocv.pair_stats(oex, tgt, tbins, clicked, keep_h, cfg.prior_strength, cfg.ctr_clip, cfg.min_impr)
        assert pt.p0 == p0
        h = pt.to_host(bits)
        ref = {k: v for k, v in table.items() if None not in k}
        assert len(h["token"]) == len(ref)
        dic = encode_codes(pa.array(tgt, pa.string()))[1].to_pylist()
        tbv = sorted(set(v for v in tbins if v is not None)) if use_tb else [0]
        prev = None
        for i in range(len(h["token"])):
            key = (int(h["token"][i]), dic[h["tgt"][i]], tbv[h["tb"][i]] if use_tb else 0)
            assert prev is None or key != prev
            prev = key
            g = ref[key]
            assert (int(h["impr"][i]), int(h["clicks"][i]), int(h["max_pos"][i]), bool(h["is_lowcount"][i])) == \
                (g["impr"], g["clicks"], g["max_pos"], g["is_lowcount"])
            assert h["ctr"][i] == pytest.approx(g["ctr"], rel=RTOL)
            assert h["w_rec_sum"][i] == pytest.approx(g["w_rec_sum"], rel=RTOL)
        # sorted ascending by (token, target code, time-bin code)
        assert list(zip(h["token"], h["tgt"], h["tb"])) == sorted(zip(h["token"], h["tgt"], h["tb"]))
        rows = np.arange(n) if f is None else np.nonzero(fold == f)[0]
        F = row_features(ex, torch.from_numpy(rows).cuda(), tg, tb, bits, pt, cfg).cpu().numpy()
        rf = ocv.row_features(oex, rows.tolist(), tgt, tbins, table, topn)
        R = np.array([rf[r] for r in rows.tolist()])
        np.testing.assert_array_equal(F[:, [5, 6]], R[:, [5, 6]])
        np.testing.assert_allclose(F, R, rtol=RTOL, atol=0)


def test_empty_and_degenerate_inputs():
    import torch
    from tossctr.covis import CoVisCfg, pair_stats, row_features
    cfg = CoVisCfg(train_path="", test_path="", agg_topn=3)
    seqs = [None, "", ",", "x"]
    ex, tg, tb, bits = _setup(seqs, ["a"] * 4, [1] * 4, [0] * 4, cfg)
    click = torch.ones(4, dtype=torch.uint8, device="cuda")
    pt = pair_stats(ex, tg, tb, click, None, bits, cfg)
    assert pt.n_pairs == 0 and pt.p0 == 1.0            # 5 exploded nulls, all clicked
    F = row_features(ex, torch.arange(4, device="cuda"), tg, tb, bits, pt, cfg).cpu().numpy()
    assert (F == 0).all()
    keep = torch.zeros(4, dtype=torch.uint8, device="cuda")
    pt = pair_stats(ex, tg, tb, click, keep, bits, cfg)
    assert pt.n_pairs == 0 and pt.p0 == 0.019          # no kept rows: the reference's fallback p0


def test_build_all_pipeline_matches_restatement(tmp_path):
    """build_covis_features.py end to end: folds, OOF + full pair tables, row features, oof_all, test; then
    the shard builder appends them to X_num."""
    from tossctr.build_cache import build_sharded_cache
    from tossctr.covis import CoVisCfg, build_all, make_folds
    n_tr, n_te = 900, 300
    seqs, tgt, dow, hour, clicked = _data(n_tr + n_te, seed=7, junk=("",))   # the shard builder int()s
    inv = [None if t is None else {"a": 11, "b": 12, "c": 13, "d": 14}[t] for t in tgt]
    ad = [(i * 7) % 5 for i in range(n_tr + n_te)]
    cols = lambda s: {"seq": pa.array(seqs[s], pa.string()), "inventory_id": pa.array(inv[s], pa.int64()),
                      "l_feat_14": pa.array(ad[s], pa.int64()), "day_of_week": pa.array(dow[s], pa.int64()),
                      "hour": pa.array(hour[s], pa.int64())}
    tr = slice(0, n_tr)
    te = slice(n_tr, n_tr + n_te)
    pq.write_table(pa.table({**cols(tr), "clicked": pa.array(clicked[tr], pa.int64()),
                             "feat_a": pa.array(np.arange(n_tr, dtype=np.float64))}), tmp_path / "train.parquet")
    pq.write_table(pa.table({**cols(te), "ID": pa.array([f"TEST_{i}" for i in range(n_te)]),
                             "feat_a": pa.array(np.arange(n_te, dtype=np.float64))}), tmp_path / "test.parquet")
    cfg = CoVisCfg(train_path=str(tmp_path / "train.parquet"), test_path=str(tmp_path / "test.parquet"),
                   target_keys=["inventory_id", "l_feat_14"], seq_top_k=12, recency_tau=32, min_impr=2,
                   prior_strength=10, work_dir=str(tmp_path / "covis"))
    build_all(cfg, device="cuda")
    _, fold = make_folds(cfg)
    oex_tr = ocv.explode(seqs[tr], cfg.seq_top_k, float(cfg.recency_tau))
    oex_te = ocv.explode(seqs[te], cfg.seq_top_k, float(cfg.recency_tau))
    tb_tr = ocv.time_bins(dow[tr], hour[tr], cfg.time_bin)
    tb_te = ocv.time_bins(dow[te], hour[te], cfg.time_bin)
    oof = pq.read_table(tmp_path / "covis" / "rowfeat_oof_all.parquet").to_pydict()
    assert sorted(oof["rid"]) == list(range(n_tr))
    names = ["sum_ctr", "mean_ctr", "max_ctr", "top3_mean_ctr", "wmean_ctr", "sum_impr", "max_impr", "pnorm_ctr"]
    for key, vals in (("inventory_id", inv), ("l_feat_14", ad)):
        for f in range(cfg.n_folds):
            keep = (fold != f).astype(int).tolist()
            table, _ = ocv.pair_stats(oex_tr, vals[tr], tb_tr, clicked[tr], keep, cfg.prior_strength, cfg.ctr_clip,
                                      cfg.min_impr)
            rows = np.nonzero(fold == f)[0].tolist()
            rf = ocv.row_features(oex_tr, rows, vals[tr], tb_tr, table, cfg.agg_topn)
            at = {r: i for i, r in enumerate(oof["rid"])}
            for j, nm in enumerate(names):
                got = [oof[f"{key}_{nm}"][at[r]] for r in rows]
                np.testing.assert_allclose(got, [rf[r][j] for r in rows], rtol=RTOL, atol=0)
        table, _ = ocv.pair_stats(oex_tr, vals[tr], tb_tr, clicked[tr], [1] * n_tr, cfg.prior_strength,
                                  cfg.ctr_clip, cfg.min_impr)
        full = pq.read_table(tmp_path / "covis" / f"pair_full_{key}.parquet").to_pydict()
        assert len(full["token"]) == len([k for k in table if None not in k])
        for i in range(len(full["token"])):
            g = table[(full["token"][i], full[key][i], full["time_bin"][i])]
            assert full["impr"][i] == g["impr"] and full["clicks"][i] == g["clicks"]
        rte = pq.read_table(tmp_path / "covis" / "rowfeat_test.parquet").to_pydict()
        assert rte["ID"] == [f"TEST_{i}" for i in range(n_te)]
        # test rows may have targets never seen in train: those match nothing
        tv = [v for v in vals[te]]
        rf = ocv.row_features(oex_te, list(range(n_te)), tv, tb_te, table, cfg.agg_topn)
        for j, nm in enumerate(names):
            np.testing.assert_allclose(rte[f"{key}_{nm}"], [rf[r][j] for r in range(n_te)], rtol=RTOL, atol=0)
    # the shard builder appends the 16 covis columns after the numeric ones
    mp = build_sharded_cache(cfg.train_path, str(tmp_path / "cache" / "train"), is_train=True, target_col="clicked",
                             seq_col="seq", cat_cols=["inventory_id"], hash_buckets={}, hash_buckets_margin=0,
                             num_patterns=["feat_*"], max_len=8, pad_id=0, group_key="inventory_id",
                             covis_enabled=True, covis_dir=cfg.work_dir)
    import json
    man = json.load(open(mp))
    assert len(man["num_cols"]) == 1 + 16
    X = np.concatenate([np.load(s["X_num"]["path"]) for s in man["shards"]])
    at = {r: i for i, r in enumerate(oof["rid"])}
    c = man["num_cols"].index("inventory_id_wmean_ctr")
    np.testing.assert_array_equal(X[:, c], np.array([oof["inventory_id_wmean_ctr"][at[r]] for r in range(n_tr)],
                                                    dtype=np.float32))
