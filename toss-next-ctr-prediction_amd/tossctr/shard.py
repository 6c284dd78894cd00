"""Row-sharded embedding tables across the data-parallel ranks (BASELINE config 5).

Replicated tables (tossctr/optim.py ``FusedAdamW.exchange``) all-gather every rank's row grads and
repeat the table optimizer work on every GPU; with ``hash_buckets=1e8, emb_dim=64`` the tables alone
(60 B params, 240 GB fp32 before Adam moments) do not fit one GPU at all.  Here row r of a table lives
on rank ``r % world`` at local row ``r // world`` (tables, moments, EMA shadow and lazy-update state
are all 1/world per GPU), and a step exchanges only the rows a batch uses:

  forward  ``fetch``:  plan (dedup the batch's ids, owner-major) -> all-to-all of requested keys ->
           owners bring the rows current (exact lazy AdamW) and gather them -> all-to-all of rows back.
           The batch is remapped to fetched-row ids, so the forward kernels read a compact table.
  backward ``route``:  the row-grad dedup runs on fetched-row ids; its sorted unique ids map back to
           owner runs -> all-to-all of (local key, grad row) -> the owner's second dedup merges the
           ranks' contributions in rank order (deterministic) -> clip / AdamW / EMA on local rows.

Per rank and step that is the batch's unique rows twice (rows out, grads back; categorical rows at their
table's width d_c) instead of world x (all ranks' grads) for the replicated all-gather.  Four all-to-alls per
step: per-owner counts (3 numbers per peer), requested keys (both table groups in one buffer), rows back
(att, rep and packed categorical rows in one buffer), grads to the owners (the same three in one buffer,
along the forward's splits).  RCCL needs the splits on the host: the counts of batch t+1 are planned on a
stream of their own while step t runs (``prefetch``, issued by ``CTRModel.train_step(next_inputs=...)``)
and copied to pinned memory, so the host's read at step t+1 waits on nothing in flight.  Without a
prefetch the plan runs in place and the read waits for it.

The pad token's rows are never fetched: fetched row 0 is zero, which is what ``padding_idx`` keeps
the pad rows at (zero init, zero grad, so AdamW/EMA leave them at zero).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from . import dist as D
from ._lib import call

INVALID = 0xFFFFFFFF


def _ptr(t, elems=0):
    return t.data_ptr() + elems * t.element_size() if t is not None else None


def shard_rows(rows: int, world: int) -> int:
    """Local rows of a table of ``rows`` rows: ceil(rows / world) (the last ranks may own one fewer)."""
    return (int(rows) + world - 1) // world


def full_to_local(full: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    """Rows ``rank, rank + world, ...`` of a full table, padded to shard_rows() rows."""
    n = shard_rows(full.shape[0], world)
    out = full.new_zeros((n,) + tuple(full.shape[1:]))
    loc = full[rank::world]
    out[:loc.shape[0]] = loc
    return out


def locals_to_full(parts: torch.Tensor, rows: int) -> torch.Tensor:
    """parts (world, local_rows, width) of every rank -> the full (rows, width) table."""
    w, n = parts.shape[0], parts.shape[1]
    return parts.transpose(0, 1).reshape(n * w, *parts.shape[2:])[:rows]


class _Grow:
    """Device buffers that only grow (exchange sizes vary per step)."""

    def __init__(self, device):
        self.device = device
        self.t = {}

    def get(self, name, n, width=None, dtype=torch.float32, zero=False):
        shape = (n,) if width is None else (n, width)
        t = self.t.get(name)
        if t is None or t.shape[0] < n or t.dtype != dtype or (width is not None and t.shape[1] != width):
            cap = max(n, 1) if t is None else max(n, int(t.shape[0] * 1.25))
            cshape = (cap,) if width is None else (cap, width)
            t = torch.zeros(cshape, dtype=dtype, device=self.device) if zero else \
                torch.empty(cshape, dtype=dtype, device=self.device)
            self.t[name] = t
        return t[:n] if width is None else t[:n]


class _Plan:
    """One batch's exchange plan: its sorted owner-major unique keys, the batch remapped to fetched-row ids, the
    categorical wire offsets, and the per-peer counts (device, then pinned host once ``event`` completes)."""


class TableShards:
    """Owner map, fetch (forward) and grad routing (backward) for one CTRModel's tables."""

    CAT_LD = 64    # fetched categorical rows are zero-padded to 64 floats in HBM (d_c <= 64); packed on the wire

    def __init__(self, arch, group, rank: int, world: int, device):
        self.a = arch
        self.group = group
        self.rank, self.world = int(rank), int(world)
        self.device = device
        W = self.world
        obits = (W - 1).bit_length()
        # sequence tokens: local key = token // W
        self.seq_rows = shard_rows(arch.seq_vocab, W)
        self.seq_lbits = self.seq_rows.bit_length()           # local keys < 2^lbits - 1
        self.seq_kbits = self.seq_lbits + obits
        # hashed categoricals: local key = lbase[c] + x // W
        loc = [shard_rows(c, W) for c in arch.cat_cards]
        self.cat_local_rows = loc
        self.cat_lbase_np = np.concatenate([[0], np.cumsum(loc)[:-1]]).astype(np.uint32)
        total = int(sum(loc))
        self.cat_lbits = total.bit_length()
        self.cat_kbits = self.cat_lbits + obits
        if self.seq_kbits > 32 or self.cat_kbits > 32:
            raise ValueError(f"row-sharded keys need {max(self.seq_kbits, self.cat_kbits)} bits (> 32): "
                             f"use more ranks per table or smaller tables")
        self.cat_lbase = torch.from_numpy(self.cat_lbase_np.view(np.int32)).to(device)
        self.cat_zero_off = torch.zeros(arch.Fc, dtype=torch.int64, device=device)
        self.cat_zero_base = torch.zeros(arch.Fc, dtype=torch.int32, device=device)
        self.cat_dims = torch.tensor(arch.cat_dims, dtype=torch.int32, device=device)
        self.buf = _Grow(device)
        self.lazy = None        # FusedAdamW (lazy) bound by the optimizer: owners bring rows current
        self.tabs_seq = None    # device ctr_lazy_tab_t arrays of the local shards (set by the engine)
        self.tabs_cat = None
        self.arena_buf = None   # the rank's parameter arena (local table shards)
        self._slot = 0          # plan buffer slot of the next plan (alternates)
        self._plan_stream = None
        self._pending = None    # the plan prefetch() issued for the next fetch()
        self._host = {}         # pinned count buffers per slot
        self.prefetch_hits = 0      # fetches that consumed the plan prefetch() made for them
        self.prefetch_misses = 0    # prefetched plans dropped because another batch was fetched first

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def _mask(bits):
        return (1 << bits) - 1

    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def _plan(self, name, X, ncols, mode):
        n = X.numel()
        uniq = self.buf.get(f"{name}_uniq", n, dtype=torch.int32)
        nu = self.buf.get(f"{name}_nu", 1, dtype=torch.int32)
        remap = self.buf.get(f"{name}_remap", n, dtype=torch.int32)
        cnt = self.buf.get(f"{name}_cnt", self.world, dtype=torch.int64)
        wsz = _lib.query("ctr_shard_plan_ws_size", n)
        ws = self.buf.get(f"{name}_ws", wsz, dtype=torch.uint8)
        if mode == 0:
            call("ctr_shard_plan", _ptr(X), n, 1, 0, self.a.pad_id, None, self.world, self.seq_lbits, self.seq_kbits,
                 _ptr(uniq), _ptr(nu), _ptr(remap), _ptr(cnt), _ptr(ws), wsz, self._stream())
        else:
            call("ctr_shard_plan", _ptr(X), n, ncols, 1, 0, _ptr(self.cat_lbase), self.world, self.cat_lbits,
                 self.cat_kbits, _ptr(uniq), _ptr(nu), _ptr(remap), _ptr(cnt), _ptr(ws), wsz, self._stream())
        return uniq, nu, remap.view(X.shape), cnt

    def _offsets(self, name, keys, n_ptr, n, cap, counts=None):
        """Offsets of categorical keys' rows at their table widths (and per-owner float counts)."""
        off = self.buf.get(f"{name}_off", cap + 1, dtype=torch.int32)
        wsz = _lib.query("ctr_shard_offsets_ws_size", cap)
        ws = self.buf.get(f"{name}_off_ws", wsz, dtype=torch.uint8)
        call("ctr_shard_offsets", _ptr(keys), _ptr(n_ptr), n, cap, self._mask(self.cat_lbits), _ptr(self.cat_lbase),
             _ptr(self.cat_dims), self.a.Fc, _ptr(off), self.world, self.cat_lbits, _ptr(counts), _ptr(ws), wsz,
             self._stream())
        return off

    # ------------------------------------------------------------------ plan (ids -> owners; no host read)
    def _issue_plan(self, X_cat, seq):
        """Dedup + owner-major keys of one batch, the per-owner counts all-to-all, and an asynchronous copy of
        the counts into pinned host memory, all on the current stream.  Plans alternate between two buffer
        slots, so a prefetched plan never writes what the step in flight reads."""
        W, slot = self.world, self._slot
        self._slot ^= 1
        pl = _Plan()
        pl.X_cat, pl.seq = X_cat, seq
        pl.uniq_s, _, pl.seq_c, cnt_s = self._plan(f"seq{slot}", seq, 1, 0)
        pl.uniq_c, nu_c, pl.xcat_c, cnt_c = self._plan(f"cat{slot}", X_cat, X_cat.shape[1], 1)
        fcnt = self.buf.get(f"fcnt{slot}", W, dtype=torch.int64)
        pl.off_c = self._offsets(f"req{slot}", pl.uniq_c, nu_c, 0, X_cat.numel(), fcnt)
        send = self.buf.get(f"csend{slot}", 3 * W, dtype=torch.int64).view(W, 3)
        for j, v in enumerate((cnt_s, cnt_c, fcnt)):
            send[:, j].copy_(v)
        recv = self.buf.get(f"crecv{slot}", 3 * W, dtype=torch.int64)
        D.all_to_all_var(recv, send.view(-1), [3] * W, [3] * W, self.group)
        host = self._host.get(slot)
        if host is None:
            host = self._host[slot] = torch.empty(6 * W, dtype=torch.int64, pin_memory=True)
        host[:3 * W].copy_(send.view(-1), non_blocking=True)
        host[3 * W:].copy_(recv, non_blocking=True)
        pl.host = host
        pl.event = torch.cuda.Event()
        pl.event.record(torch.cuda.current_stream(self.device))
        return pl

    def prefetch(self, X_cat, seq):
        """Plan the NEXT batch's exchange now, on a stream of its own: it runs beside the current step, so the
        next fetch() finds its counts on the host without waiting.  Its buffers are written only after
        everything queued so far on the current stream (the step in flight may still read the other slot)."""
        cur = torch.cuda.current_stream(self.device)
        if self._plan_stream is None:
            self._plan_stream = torch.cuda.Stream(device=self.device)
        ev = torch.cuda.Event()
        ev.record(cur)
        self._plan_stream.wait_event(ev)
        with torch.cuda.stream(self._plan_stream):
            self._pending = self._issue_plan(X_cat, seq)

    def _take_plan(self, X_cat, seq):
        pl, self._pending = self._pending, None
        cur = torch.cuda.current_stream(self.device)
        if pl is not None and pl.X_cat is X_cat and pl.seq is seq:
            cur.wait_event(pl.event)
            self.prefetch_hits += 1
        else:
            if pl is not None:
                # a prefetched plan for another batch (e.g. an evaluation forward came in between): it is
                # dropped, but its device writes and its copy into the pinned counts of its slot may still be
                # running on the plan stream -- order everything after it, or the next in-place plan that reuses
                # that slot on this stream could race with it
                cur.wait_event(pl.event)
                self.prefetch_misses += 1
            pl = self._issue_plan(X_cat, seq)
        # the host's only wait of the step: on counts computed beside the previous step when prefetched
        pl.event.synchronize()
        W = self.world
        h = pl.host.tolist()
        pl.send = [h[j:3 * W:3] for j in range(3)]
        pl.recv = [h[3 * W + j::3] for j in range(3)]
        return pl

    # ------------------------------------------------------------------ one buffer per exchange
    def _wire(self, counts, widths):
        """Per-peer segments of several 4-byte arrays in one all-to-all buffer: peer w's segment holds, for
        each array b, its counts[b][w] rows of widths[b] words (the arrays' rows are grouped by peer in rank
        order).  Returns the pieces (array, word offset in the array, word offset in the wire, words), the
        words per peer and the total."""
        pieces, per_peer, off = [], [], 0
        pref = [0] * len(counts)
        for w in range(self.world):
            start = off
            for b, (c, wd) in enumerate(zip(counts, widths)):
                n = int(c[w]) * wd
                if n:
                    pieces.append((b, pref[b] * wd, off, n))
                off += n
                pref[b] += int(c[w])
            per_peer.append(off - start)
        return pieces, per_peer, off

    def _copy(self, pieces, arrays, wire, to_wire):
        segs = (_lib.Seg * max(1, len(pieces)))()
        wp = wire.data_ptr()
        for i, (b, aoff, woff, n) in enumerate(pieces):
            ap = arrays[b].data_ptr() + 4 * aoff
            segs[i].src, segs[i].dst = (ap, wp + 4 * woff) if to_wire else (wp + 4 * woff, ap)
            segs[i].n = n
        call("ctr_copy_segments", segs, len(pieces), self._stream())

    def _exchange(self, name, send_arrays, recv_arrays, send_counts, recv_counts, widths, dtype):
        """ONE all-to-all for several arrays: gather their per-peer pieces into a wire buffer, exchange,
        scatter the received pieces into the receive arrays."""
        sp, s_peer, s_tot = self._wire(send_counts, widths)
        rp, r_peer, r_tot = self._wire(recv_counts, widths)
        ws = self.buf.get(f"{name}_wsend", s_tot, dtype=dtype)
        wr = self.buf.get(f"{name}_wrecv", r_tot, dtype=dtype)
        self._copy(sp, send_arrays, ws, True)
        D.all_to_all_var(wr, ws, r_peer, s_peer, self.group)
        self._copy(rp, recv_arrays, wr, False)

    # ------------------------------------------------------------------ forward
    def fetch(self, X_cat, seq):
        """Rows the batch reads, fetched from their owners.  Returns the remapped batch (fetched-row
        ids; 0 = pad) and the compact tables: att/rep (1 + n_uniq, D) with row 0 zero, cat (1 + n, 64).
        Categorical rows travel at their table's width d_c (packed), not as 64-float rows.  Two all-to-alls:
        the requested keys of both table groups, then the att, rep and categorical rows in one buffer."""
        a, st = self.a, self._stream()
        Dm, LD = a.D, self.CAT_LD
        pl = self._take_plan(X_cat, seq)
        (send_s, send_c, send_f), (recv_s, recv_c, recv_f) = pl.send, pl.recv
        ns, nc = sum(send_s), sum(send_c)
        rs, rc = sum(recv_s), sum(recv_c)
        # requested keys -> owners (sequence and categorical keys in one exchange)
        req_s = self.buf.get("req_s", rs, dtype=torch.int32)
        req_c = self.buf.get("req_c", rc, dtype=torch.int32)
        self._exchange("keys", (pl.uniq_s, pl.uniq_c), (req_s, req_c), (send_s, send_c), (recv_s, recv_c), (1, 1),
                       torch.int32)
        # owner side: local keys, rows brought current, rows gathered (categorical ones packed at d_c)
        loc_s = self.buf.get("loc_s", rs, dtype=torch.int32)
        loc_c = self.buf.get("loc_c", rc, dtype=torch.int32)
        call("ctr_shard_strip", _ptr(req_s), rs, self._mask(self.seq_lbits), _ptr(loc_s), st)
        call("ctr_shard_strip", _ptr(req_c), rc, self._mask(self.cat_lbits), _ptr(loc_c), st)
        if self.lazy is not None:
            self.lazy.touch_local(loc_s, loc_c)
        arena = self.arena_buf
        out_att = self.buf.get("out_att", rs, Dm)
        out_rep = self.buf.get("out_rep", rs, Dm)
        out_cat = self.buf.get("out_cat", rc, LD)
        tabs, nt = self.tabs_seq
        call("ctr_shard_gather", _ptr(loc_s), rs, 0, _ptr(tabs), nt, _ptr(arena), _ptr(out_att), _ptr(out_rep), Dm, st)
        tabs, nt = self.tabs_cat
        call("ctr_shard_gather", _ptr(loc_c), rc, 1, _ptr(tabs), nt, _ptr(arena), _ptr(out_cat), None, LD, st)
        off_o = self._offsets("own", req_c, None, rc, rc)
        pk_o = self.buf.get("cat_pk_o", sum(recv_f))
        call("ctr_shard_pack", _ptr(out_cat), LD, rc, _ptr(off_o), _ptr(pk_o), st)
        # rows back, in the requester's unique-key order (fetched row u + 1 = unique key u).  Row 0 (pad) of
        # att / rep / cat is zeroed once when the buffer is allocated and never written.
        att = self.buf.get("att", 1 + seq.numel(), Dm, zero=True)
        rep = self.buf.get("rep", 1 + seq.numel(), Dm, zero=True)
        cat = self.buf.get("cat", 1 + X_cat.numel(), LD, zero=True)
        pk_r = self.buf.get("cat_pk_r", sum(send_f))
        self._exchange("rows", (out_att, out_rep, pk_o), (att[1:], rep[1:], pk_r), (recv_s, recv_s, recv_f),
                       (send_s, send_s, send_f), (Dm, Dm, 1), torch.float32)
        call("ctr_shard_unpack", _ptr(pk_r), _ptr(pl.off_c), nc, _ptr(cat, LD), LD, st)
        return dict(seq=pl.seq_c, xcat=pl.xcat_c, att=att, rep=rep, cat=cat, n_seq=seq.numel(), n_cat=X_cat.numel(),
                    splits=(send_s, recv_s, send_c, recv_c, send_f, recv_f), loc_s=loc_s, loc_c=loc_c,
                    off_c=pl.off_c, off_o=off_o)

    # ------------------------------------------------------------------ backward
    def _rowgrad(self, name, keys, rows, n, width, bits):
        uk = self.buf.get(f"{name}_uk", n, dtype=torch.int32)
        ug = self.buf.get(f"{name}_ug", n, width)
        nu = self.buf.get(f"{name}_nu", 1, dtype=torch.int32)
        wsz = _lib.query("ctr_rowgrad_ws_size", n)
        ws = self.buf.get("rowgrad_ws", wsz, dtype=torch.uint8)
        call("ctr_rowgrad", _ptr(keys), _ptr(rows), n, width, width, bits, _ptr(uk), _ptr(ug), _ptr(nu), _ptr(ws), wsz,
             self._stream())
        return dict(keys=uk, G=ug, n_uniq=nu, width=width, n=n)

    def _rowgrad2(self, name, keys, rows_a, rows_b, n, width, bits):
        """Owner-side merge of the att and rep grads, which share their keys: one sort for both."""
        uk = self.buf.get(f"{name}_uk", n, dtype=torch.int32)
        ua = self.buf.get(f"{name}_ua", n, width)
        ub = self.buf.get(f"{name}_ub", n, width)
        nu = self.buf.get(f"{name}_nu", 1, dtype=torch.int32)
        wsz = _lib.query("ctr_rowgrad_ws_size", n)
        ws = self.buf.get("rowgrad_ws", wsz, dtype=torch.uint8)
        call("ctr_rowgrad2", _ptr(keys), _ptr(rows_a), _ptr(rows_b), n, width, width, bits, _ptr(uk), _ptr(ua),
             _ptr(ub), _ptr(nu), _ptr(ws), wsz, self._stream())
        return (dict(keys=uk, G=ua, n_uniq=nu, width=width, n=n), dict(keys=uk, G=ub, n_uniq=nu, width=width, n=n))

    def route(self, tg, fx):
        """Compact grads on fetched-row ids (tg from Engine.backward) -> the owners' merged grads on
        local keys: {"att", "rep", "cat"} in the layout the optimizer consumes.

        The grads are scattered to the fetched-row order first (a fetched row without a gradient -- a
        token outside every top-K -- stays 0, which AdamW steps exactly like an untouched row), so they
        go back along the forward's request splits: no second count exchange, no host read."""
        st = self._stream()
        LD = self.CAT_LD
        ta, tr, tc = tg["att"], tg["rep"], tg["cat"]
        send_s, recv_s, send_c, recv_c, send_f, recv_f = fx["splits"]
        ns, nc, rs, rc = sum(send_s), sum(send_c), sum(recv_s), sum(recv_c)
        Dm = ta["width"]
        ga = self.buf.get("dg_att", ns, Dm)
        gr = self.buf.get("dg_rep", ns, Dm)
        gc = self.buf.get("dg_cat", nc, LD)
        for dst, t, w in ((ga, ta, Dm), (gr, tr, Dm), (gc, tc, LD)):
            dst.zero_()
            call("ctr_scatter_rows", _ptr(t["keys"]), _ptr(t["G"]), _ptr(t["n_uniq"]), t["n"], w, t["G"].shape[1], 1,
                 dst.shape[0], _ptr(dst), st)
        pk = self.buf.get("dg_cat_pk", sum(send_f))
        call("ctr_shard_pack", _ptr(gc), LD, nc, _ptr(fx["off_c"]), _ptr(pk), st)
        rg_a = self.buf.get("ga_s", rs, Dm)
        rg_r = self.buf.get("gr_s", rs, Dm)
        rg_p = self.buf.get("gc_pk", sum(recv_f))
        self._exchange("grads", (ga, gr, pk), (rg_a, rg_r, rg_p), (send_s, send_s, send_f), (recv_s, recv_s, recv_f),
                       (Dm, Dm, 1), torch.float32)
        rg_c = self.buf.get("gc_c", rc, LD)
        call("ctr_shard_unpack", _ptr(rg_p), _ptr(fx["off_o"]), rc, _ptr(rg_c), LD, st)
        att, rep = self._rowgrad2("sh_seq", fx["loc_s"], rg_a, rg_r, rs, Dm, self.seq_lbits)
        return {"att": att, "rep": rep, "cat": self._rowgrad("sh_cat", fx["loc_c"], rg_c, rc, LD, self.cat_lbits)}

    # ------------------------------------------------------------------ full-table views (checkpoints)
    def gather_full(self, local: torch.Tensor, rows: int) -> torch.Tensor:
        """Every rank's shard of one table -> the full table (collective; result on this device)."""
        parts = torch.empty((self.world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
        D.all_gather_into(parts.view(-1), local.contiguous().view(-1), self.group)
        return locals_to_full(parts, rows)

