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
