"""Exact lazy table update (csrc/lazy.hip) vs the dense AdamW/EMA stream (csrc/optim.hip): after any
sequence of training ticks, EMA-only ticks, evaluation reads and mid-run flushes, the flushed lazy
state (parameters, both Adam moments, EMA shadow) must equal the dense state BIT FOR BIT.

Tables are made much larger than what a batch touches (vocab x40, hashed cardinalities x50) so most
rows skip most ticks, and the learning rate changes every tick (cosine warm-up), so a replay that
used the wrong tick's scalars would show."""
import math

import numpy as np
import pytest
import torch

from golden_util import Fixture, to_torch_batch
from oracle.synth import make_batch

pytestmark = pytest.mark.gpu


def _models(fx, vocab, cards):
    from tossctr import CTRModel
    m = fx.meta
    a = CTRModel(m["cfg"], vocab, m["Fn"], m["Fm"], cards, list(cards), device="cuda:0")
    g = torch.Generator(device="cuda:0")
    g.manual_seed(123)
    a.reset_parameters(generator=g)
    b = CTRModel(m["cfg"], vocab, m["Fn"], m["Fm"], cards, list(cards), device="cuda:0")
    b.load_state_dict(a.state_dict())
    return a, b


@pytest.mark.parametrize("case", ["tiny_concat", "tiny_s2"])
def test_lazy_matches_dense_bitwise(case):
    from tossctr import ArenaEMA, FusedAdamW
    fx = Fixture(case)
    m, tr = fx.meta, fx.meta["train"]
    vocab = int(m["vocab"]) * 40
    cards = {k: v * 50 for k, v in fx.cat_cards.items()}
    md, ml = _models(fx, vocab, cards)
    ema_d = ArenaEMA(md, base_decay=0.99, warmup_steps=5, warmup_type="cosine")
    ema_l = ArenaEMA(ml, base_decay=0.99, warmup_steps=5, warmup_type="cosine")
    od = FusedAdamW(md, lr=1e-3, weight_decay=tr["wd"], max_grad_norm=tr["clip"], ema=ema_d, lazy=False)
    ol = FusedAdamW(ml, lr=1e-3, weight_decay=tr["wd"], max_grad_norm=tr["clip"], ema=ema_l, lazy=True)
    B, L = 48, int(m["L"])
    steps = 14
    for t in range(steps):
        b = make_batch(B, m["Fn"], m["Fm"], list(cards.values()), L, vocab, seed=1000 + t)
        lr = 1e-3 * 0.5 * (1 + math.cos(math.pi * t / steps)) + 1e-5
        for model, opt in ((md, od), (ml, ol)):
            opt.param_groups[0]["lr"] = lr
            inputs = model.stage(to_torch_batch(b))
            y = torch.from_numpy(b["y"]).float().cuda()
            model.train()
            model.train_step(inputs, y, opt, global_step=t + 1, seed=(7 << 32) | t)
            if t == 4:       # an EMA-only tick
                opt.ema.update(model, global_step=t + 1)
            if t == 6:       # an evaluation read between ticks (touches rows, no tick)
                model.eval()
                with torch.no_grad():
                    model(to_torch_batch(make_batch(B, m["Fn"], m["Fm"], list(cards.values()), L, vocab, seed=7)))
        if t == 9:
            ml.sync()        # a mid-run flush, then more lazy ticks
        # the step outputs of the two paths agree exactly at every tick
        assert torch.equal(od.norm_out, ol.norm_out), t
    ml.sync()
    assert ol.tick == steps + 1
    assert torch.equal(md.arena.buf, ml.arena.buf)
    assert torch.equal(od.m, ol.m)
    assert torch.equal(od.v, ol.v)
    assert torch.equal(ema_d.shadow, ema_l.shadow)
    # sanity: the test exercised both untouched and touched rows of a large table
    ar = ml.arena
    ta = ar._view(ol.m, "dare.emb_att.weight")
    touched = (ta != 0).any(dim=1)
    assert 0 < int(touched.sum()) < ta.shape[0] // 2


def _pooled_batch(B, m, cards, L, vocab, seed, pool_seq, pool_cat):
    """make_batch with half of the history tokens and of the categorical ids drawn from small pools spread
    over the tables, so rows recur after gaps of every length (a token of the 4000-row pool returns every
    few ticks, a uniform one almost never): the replay of 1 .. T missed ticks is exercised row by row."""
    b = make_batch(B, m["Fn"], m["Fm"], list(cards.values()), L, vocab, seed=seed)
    r = np.random.default_rng(seed + 17)
    seq = b["seq"]
    sel = (seq != 0) & (r.random(seq.shape) < 0.5)
    seq[sel] = pool_seq[r.integers(0, pool_seq.size, int(sel.sum()))]
    xc = b["X_cat"]
    for c in range(xc.shape[1]):
        s = r.random(B) < 0.5
        xc[s, c] = pool_cat[c][r.integers(0, pool_cat[c].size, int(s.sum()))]
    return b


@pytest.mark.parametrize("case,vocab,card", [("cfg2_dims", 2_000_000, 60_000), ("cfg4_full", 5_000_000, 60_000)],
                         ids=["D32_cfg2", "D64_cfg4"])
def test_lazy_matches_dense_bitwise_at_cfg_widths(case, vocab, card):
    """Lazy = dense, bit for bit, at the widths the bench runs: cfg2 (D = 32: lazy_*_pair*<32>, 35 tables of
    the yaml's d_c) and cfg4 (D = 64, L = 400, K = 148, 4 layers: lazy_*_pair*<64>), over 32 ticks with a
    changing lr, an EMA-only tick, an evaluation read and two mid-run flushes; tables >= 40x the rows the run
    touches, and pooled ids (_pooled_batch), so rows replay gaps of every length up to the whole run."""
    from tossctr import ArenaEMA, FusedAdamW
    fx = Fixture(case)
    m, tr = fx.meta, fx.meta["train"]
    cards = {k: card for k in fx.cat_cards}
    md, ml = _models(fx, vocab, cards)
    ema_d = ArenaEMA(md, base_decay=0.99, warmup_steps=5, warmup_type="cosine")
    ema_l = ArenaEMA(ml, base_decay=0.99, warmup_steps=5, warmup_type="cosine")
    od = FusedAdamW(md, lr=1e-3, weight_decay=1e-4, max_grad_norm=0.5, ema=ema_d, lazy=False)
    ol = FusedAdamW(ml, lr=1e-3, weight_decay=1e-4, max_grad_norm=0.5, ema=ema_l, lazy=True)
    B, L = (48, int(m["L"])) if case == "cfg2_dims" else (24, int(m["L"]))
    steps = 32
    r = np.random.default_rng(9)
    pool_seq = r.choice(np.arange(1, vocab), 4000, replace=False).astype(np.int32)
    pool_cat = [r.choice(card, 200, replace=False).astype(np.int32) for _ in cards]
    seen_seq, seen_cat = set(), [set() for _ in cards]
    for t in range(steps):
        b = _pooled_batch(B, m, cards, L, vocab, 2000 + t, pool_seq, pool_cat)
        seen_seq.update(np.unique(b["seq"]).tolist())
        for c, s in enumerate(seen_cat):
            s.update(np.unique(b["X_cat"][:, c]).tolist())
        lr = 1e-3 * 0.5 * (1 + math.cos(math.pi * t / steps)) + 1e-5
        for model, opt in ((md, od), (ml, ol)):
            opt.param_groups[0]["lr"] = lr
            model.train()
            model.train_step(model.stage(to_torch_batch(b)), torch.from_numpy(b["y"]).float().cuda(), opt,
                             global_step=t + 1, seed=(5 << 32) | t)
            if t == 4:
                opt.ema.update(model, global_step=t + 1)
            if t == 6:
                model.eval()
                with torch.no_grad():
                    model(to_torch_batch(_pooled_batch(B, m, cards, L, vocab, 77, pool_seq, pool_cat)))
        if t in (11, 23):
            ml.sync()
        assert torch.equal(od.norm_out, ol.norm_out), t
    assert vocab >= 40 * len(seen_seq) and all(card >= 40 * len(s) for s in seen_cat)
    ml.sync()
    assert ol.tick == steps + 1
    assert torch.equal(md.arena.buf, ml.arena.buf)
    assert torch.equal(od.m, ol.m)
    assert torch.equal(od.v, ol.v)
    assert torch.equal(ema_d.shadow, ema_l.shadow)


def test_lazy_state_dict_flushes():
    from tossctr import FusedAdamW
    fx = Fixture("tiny_concat")
    m, tr = fx.meta, fx.meta["train"]
    cards = dict(fx.cat_cards)
    md, ml = _models(fx, int(m["vocab"]), cards)
    od = FusedAdamW(md, lr=1e-2, weight_decay=0.1, lazy=False)
    ol = FusedAdamW(ml, lr=1e-2, weight_decay=0.1, lazy=True)
    b = fx.batch(0)
    for model, opt in ((md, od), (ml, ol)):
        for t in range(3):
            model.train_step(model.stage(to_torch_batch(b)), torch.from_numpy(b["y"]).float().cuda(), opt, t + 1,
                             seed=t)
    sd_d, sd_l = md.state_dict(), ml.state_dict()
    for k in sd_d:
        assert torch.equal(sd_d[k], sd_l[k]), k
    assert ol._flushed_tick == ol.tick == 3
    np.testing.assert_array_equal(ol.last.cpu().numpy() & 0x7FFFFFFF, 3)    # bit 31: row took a grad tick


def test_touch_first_chunk_full_class_plus_hot_row():
    """lazy_touch_pair_cls_kernel's first chunk of TOUCH_CH = 256 token positions: all 256 distinct rows
    claimed into one class list (rows that took a gradient tick) while the hot (padding) row joins the same
    class -- 257 entries.  The padding row's state word is given the has-grad bit by hand (its moments are
    zero, so the full replay is bit-identical to the short one).  Lazy must still equal dense bitwise."""
    from tossctr import FusedAdamW
    fx = Fixture("tiny_concat")
    m, tr = fx.meta, fx.meta["train"]
    vocab = int(m["vocab"]) * 4
    cards = dict(fx.cat_cards)
    md, ml = _models(fx, vocab, cards)
    od = FusedAdamW(md, lr=1e-3, weight_decay=tr["wd"], max_grad_norm=tr["clip"], lazy=False)
    ol = FusedAdamW(ml, lr=1e-3, weight_decay=tr["wd"], max_grad_norm=tr["clip"], lazy=True)
    L = int(m["L"])
    assert 8 * L == 256
    toks = np.random.default_rng(5).choice(np.arange(1, vocab), 8 * L, replace=False).astype(np.int32)
    batches = []
    for t in range(4):
        b = make_batch(16, m["Fn"], m["Fm"], list(cards.values()), L, vocab, seed=300 + t)
        if t in (0, 2):            # tick 1 steps the 256 tokens (every history position takes an att grad);
            b["seq"][:8] = toks.reshape(8, L)     # tick 3 reads them again first: 256 distinct class-1 rows
        batches.append(b)
    for t, b in enumerate(batches):
        for model, opt in ((md, od), (ml, ol)):
            if t == 2 and opt is ol:
                ol.last[0] |= np.int32(-2 ** 31)      # the hot row in the has-grad class as well
            model.train_step(model.stage(to_torch_batch(b)), torch.from_numpy(b["y"]).float().cuda(), opt, t + 1,
                             seed=(3 << 32) | t)
    ml.sync()
    assert torch.equal(md.arena.buf, ml.arena.buf)
    assert torch.equal(od.m, ol.m) and torch.equal(od.v, ol.v)


@pytest.mark.parametrize("ema", [True, False])
def test_cat_flush_classified_equals_touch_replay(ema):
    """ctr_lazy_flush (lazy_flush_cls_kernel: classified row lists, four elements per lane, the next chunk's state
    words loaded during the current chunk's replay) against an independent replay of the same rows: ctr_lazy_touch
    over EVERY key (lazy_touch_kernel: an 8-lane group per row, replay_rows_wave; itself checked bitwise against
    the dense stream through the model tests above), on a synthetic state over every lane layout: widths 1..64
    with rows that are and are not 16-byte aligned, rows current / never stepped / stepped at random ticks, ticks
    without the AdamW step or without the EMA.  Bitwise."""
    from tossctr import _lib
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device=dev).manual_seed(11)
    T = 23
    hist = torch.zeros((T + 2) * _lib.query("ctr_opt_hist_entry_bytes"), dtype=torch.uint8, device=dev)
    for t in range(1, T + 1):
        _lib.call("ctr_opt_hist_record", hist.data_ptr(), t, 3e-3 * min(1.0, t / 7), 0.05, 0.9, 0.999, 1e-8, t,
                  0.99, 0 if t == 9 else 1, 1 if (ema and t != 14) else 0, st)
    widths = [1, 3, 4, 5, 7, 8, 9, 12, 16, 17, 22, 30, 33, 43, 51, 57, 64]
    rows = [2500 + 97 * i for i in range(len(widths))]
    n = sum(r * w for r, w in zip(rows, widths))
    nrows = sum(rows)
    u = torch.rand(nrows, generator=g, device=dev)
    last0 = torch.zeros(nrows, dtype=torch.int32, device=dev)
    nz = u < 0.3
    last0[nz] = torch.randint(1, T, (int(nz.sum()),), generator=g, device=dev, dtype=torch.int32) | -2 ** 31
    mid = (u >= 0.3) & (u < 0.6)
    last0[mid] = torch.randint(1, T, (int(mid.sum()),), generator=g, device=dev, dtype=torch.int32)
    last0[(u >= 0.6) & (u < 0.65)] = T
    row_nz = torch.cat([(last0[o:o + r] < 0).float().repeat_interleave(w)
                        for o, r, w in zip(np.cumsum([0] + rows[:-1]).tolist(), rows, widths)])
    P0 = torch.randn(n, generator=g, device=dev)
    M0 = torch.randn(n, generator=g, device=dev) * 1e-3 * row_nz
    V0 = torch.rand(n, generator=g, device=dev) * 1e-6 * row_nz
    E0 = P0 + 0.01 * torch.randn(n, generator=g, device=dev)
    last = torch.empty_like(last0)
    arr = (_lib.LazyTab * len(widths))()
    po = ro = 0
    for i, (r, w) in enumerate(zip(rows, widths)):
        arr[i].p_off, arr[i].rows, arr[i].width, arr[i].key_base, arr[i].last = po, r, w, ro, last.data_ptr() + 4 * ro
        po += r * w
        ro += r
    tabs = torch.from_numpy(np.frombuffer(bytes(arr), dtype=np.uint8).copy()).to(dev)
    keys = torch.arange(nrows, dtype=torch.int32, device=dev)

    def run(flush):
        last.copy_(last0)
        P, M, V, E = P0.clone(), M0.clone(), V0.clone(), E0.clone() if ema else None
        args = (P.data_ptr(), M.data_ptr(), V.data_ptr(), E.data_ptr() if ema else None, hist.data_ptr(), T, st)
        if flush:
            _lib.call("ctr_lazy_flush", tabs.data_ptr(), len(widths), max(rows), *args)
        else:
            _lib.call("ctr_lazy_touch", tabs.data_ptr(), len(widths), keys.data_ptr(), nrows, 1, 2, *args)
        torch.cuda.synchronize()
        return P, M, V, E, last.clone()

    ref = run(False)
    got = run(True)
    for name, a, b in zip("PMVE", ref[:4], got[:4]):
        if a is not None:
            assert torch.equal(a.view(torch.int32), b.view(torch.int32)), (name, int((a != b).sum()))
    assert torch.equal(ref[4], got[4])
    assert bool(((ref[4] & 0x7FFFFFFF) == T).all())


def test_adamw_ema_hist_one_launch_equals_two_kernel_form():
    """ctr_adamw_ema_hist runs as ONE launch (the tick's history record and the sparse chunks' key-range searches
    inside adamw_ema_kernel<true>): on the dense optimizer's full chunk list -- sparse table chunks included, which
    the lazy step never hands it -- it writes bit for bit what ctr_adamw_ema (chunk_key_range_kernel + adamw_ema_kernel)
    writes, and records the tick's scalars."""
    from tossctr import ArenaEMA, FusedAdamW
    from tossctr._lib import call
    from tossctr.engine import ptr
    fx = Fixture("tiny_concat")
    m, tr = fx.meta, fx.meta["train"]
    vocab = int(m["vocab"]) * 40
    cards = {k: v * 50 for k, v in fx.cat_cards.items()}
    md, _ = _models(fx, vocab, cards)
    ema = ArenaEMA(md, base_decay=0.99, warmup_steps=5, warmup_type="cosine")
    od = FusedAdamW(md, lr=1e-3, weight_decay=tr["wd"], max_grad_norm=tr["clip"], ema=ema, lazy=False)
    b = make_batch(48, m["Fn"], m["Fm"], list(cards.values()), int(m["L"]), vocab, seed=77)
    md.train()
    md.train_step(md.stage(to_torch_batch(b)), torch.from_numpy(b["y"]).float().cuda(), od, global_step=1, seed=5)
    tg = md.engine.tg
    segs = od._segs_device(tg)
    chunks, n = od._chunks_dev["all"]
    st = torch.cuda.current_stream().cuda_stream
    outs = []
    for form in ("two", "one"):
        P, M, V, E = md.arena.buf.clone(), od.m.clone(), od.v.clone(), ema.shadow.clone()
        krange = torch.full((2 * n,), -1, dtype=torch.int32, device="cuda")
        hist = torch.zeros(64 * 64, dtype=torch.uint8, device="cuda")
        args = (ptr(chunks), n, ptr(segs), ptr(krange), ptr(P), ptr(M), ptr(V), ptr(E), ptr(md.arena.grad),
                ptr(od.norm_out, 1), 1e-3, float(tr["wd"]), 0.9, 0.999, 1e-8, 2, 0.97)
        if form == "two":
            call("ctr_adamw_ema", *args, 1, 1, st)
        else:
            call("ctr_adamw_ema_hist", *args, 1, ptr(hist), 3, st)
        outs.append((P, M, V, E, hist))
    torch.cuda.synchronize()
    for a, c in zip(outs[0][:4], outs[1][:4]):
        assert torch.equal(a, c)
    assert not torch.equal(outs[0][0], md.arena.buf)                 # the launch stepped something
    from tossctr import _lib
    hb = _lib.query("ctr_opt_hist_entry_bytes")
    h = outs[1][4]
    assert int(h[:3 * hb].sum()) == 0 and int(h[3 * hb:4 * hb].sum()) != 0 and int(h[4 * hb:].sum()) == 0   # tick 3 only
    kinds = {int(s["kind"]) for s in od._segments(tg)}
    assert 1 in kinds                                                  # sparse table chunks were in the list
