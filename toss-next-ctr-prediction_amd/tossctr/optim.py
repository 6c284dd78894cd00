"""Fused clip_grad_norm_ + AdamW + EMA for the CTRModel parameter arena.

Drop-in for the reference step tail (src/train.py:133-139 construction, :185-199 per step):
    nn.utils.clip_grad_norm_(model.parameters(), c); opt.step(); ema.update(model, global_step)
Semantics are torch's dense ones (every element decays / moves each step, untouched table rows see
grad 0).  Dense parameters are ONE pass over (p, m, v, ema) by csrc/optim.hip; the embedding tables
(1.24 B of the 1.25 B elements at the benchmark config) take the exact lazy path of csrc/lazy.hip:
a row is replayed to the current tick when read, when it gets a gradient, or at flush() --
bit-identical to the dense stream, which stays available as lazy=False.  No dense table gradient is
ever written.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib
from ._lib import OptChunk, OptSeg, call
from .engine import ptr

INVALID_KEY = 0xFFFFFFFF


def ema_decay_at(base, warmup_steps, warmup_type, n_updates):
    """ModelEMA._decay_at (src/utils/ema.py:72-88)."""
    if warmup_steps <= 0 or warmup_type == "none":
        return base
    t = min(1.0, (n_updates + 1) / warmup_steps)
    if warmup_type == "linear":
        d = 1.0 - (1.0 - base) * t
    elif warmup_type == "cosine":
        d = 1.0 - (1.0 - base) * (0.5 * (1 + math.cos(math.pi * (1 - t))))
    else:
        d = base
    return float(max(0.0, min(1.0, d)))


class ArenaEMA:
    """ModelEMA (src/utils/ema.py:11-198) over the arena: fp32 shadow of every parameter."""

    def __init__(self, model, base_decay=0.999, warmup_steps=0, warmup_type="linear", update_after_step=0,
                 update_interval=1, ema_on_buffers="copy", offload_to_cpu=False, pin_memory=False, param_filter=None):
        if offload_to_cpu:
            raise NotImplementedError("offload_to_cpu EMA is not supported on the fused path")
        if param_filter:
            raise NotImplementedError("param_filter is not supported on the fused path")
        self.model = model
        self.base_decay = float(base_decay)
        self.warmup_steps = int(max(0, warmup_steps))
        self.warmup_type = warmup_type
        self.update_after_step = int(max(0, update_after_step))
        self.update_interval = int(max(1, update_interval))
        self.ema_on_buffers = ema_on_buffers
        self.offload_to_cpu = False
        self.pin_memory = bool(pin_memory)
        self.param_filter = set()
        self.num_updates = 0
        model.sync()
        self.shadow = model.arena.buf.clone()
        self._saved = None

    def wants_update(self, global_step):
        if global_step < self.update_after_step:
            return False
        return (global_step - self.update_after_step) % self.update_interval == 0

    def next_decay(self):
        return ema_decay_at(self.base_decay, self.warmup_steps, self.warmup_type, self.num_updates)

    def update(self, model, global_step):
        """Standalone update (when not fused into FusedAdamW.step)."""
        opt = getattr(model, "_fused_opt", None)
        if opt is None:
            raise RuntimeError("ArenaEMA.update needs a FusedAdamW bound to the model")
        opt.ema_only(self, global_step)

    @torch.no_grad()
    def store(self, model):
        model.sync()
        self._saved = model.arena.buf.clone()

    @torch.no_grad()
    def copy_to(self, model):
        model.sync()
        model.arena.buf.copy_(self.shadow)

    @torch.no_grad()
    def restore(self, model):
        if self._saved is None:
            return
        model.arena.buf.copy_(self._saved)
        self._saved = None

    def shadow_params(self):
        """{key: shadow tensor}; row-sharded tables come back whole (collective)."""
        self.model.sync()
        ar = self.model.arena
        return {k: self.model.full_table(self.shadow, k) for k in ar.order}

    def state_dict(self):
        return {"base_decay": self.base_decay, "warmup_steps": self.warmup_steps, "warmup_type": self.warmup_type,
                "update_after_step": self.update_after_step, "update_interval": self.update_interval,
                "ema_on_buffers": self.ema_on_buffers, "offload_to_cpu": False, "pin_memory": self.pin_memory,
                "param_filter": [], "num_updates": self.num_updates,
                "shadow_params": {k: v.detach().cpu().clone() for k, v in self.shadow_params().items()},
                "shadow_buffers": {}}

    def load_state_dict(self, state):
        self.base_decay = float(state["base_decay"])
        self.warmup_steps = int(state["warmup_steps"])
        self.warmup_type = state["warmup_type"]
        self.update_after_step = int(state["update_after_step"])
        self.update_interval = int(state["update_interval"])
        self.num_updates = int(state.get("num_updates", 0))
        self.model.sync()
        ar, sh = self.model.arena, self.model.shards
        for k in ar.order:
            src = torch.as_tensor(state["shadow_params"][k])
            if sh is not None and ar.kind[k] == "table":
                from .shard import full_to_local
                src = full_to_local(src, sh.rank, sh.world)
            ar._view(self.shadow, k).copy_(src)


def build_ema(model, cfg):
    """src/utils/ema.py:200-216."""
    if not cfg.get("ema", {}).get("enabled", False):
        return None
    ec = cfg["ema"]
    return ArenaEMA(model, base_decay=float(ec.get("decay", 0.999)), warmup_steps=int(ec.get("warmup_steps", 0)),
                    warmup_type=str(ec.get("warmup_type", "linear")),
                    update_after_step=int(ec.get("update_after_step", 0)),
                    update_interval=int(ec.get("update_interval", 1)),
                    ema_on_buffers=str(ec.get("ema_on_buffers", "copy")),
                    offload_to_cpu=bool(ec.get("offload_to_cpu", False)),
                    pin_memory=bool(ec.get("pin_memory", False)), param_filter=ec.get("param_filter", []))


class FusedAdamW:
    """torch.optim.AdamW(model.parameters(), lr, weight_decay) + clip + EMA as one arena stream."""

    def __init__(self, model, lr, weight_decay=1e-2, betas=(0.9, 0.999), eps=1e-8, max_grad_norm=0.0, ema=None,
                 process_group=None, lazy=True):
        self.model = model
        self.arena = ar = model.arena
        self.engine = model.engine
        self.param_groups = [{"lr": float(lr), "weight_decay": float(weight_decay), "betas": betas, "eps": eps}]
        self.max_grad_norm = float(max_grad_norm)
        self.ema = ema
        self.pg = process_group
        self.world = 1
        self.contributors = None    # ranks contributing to the current step's gradient (None: all)
        if process_group is not None:
            import torch.distributed as dist
            self.world = dist.get_world_size(process_group)
        self._timing = False
        self._events = []
        dev = ar.device
        self.m = torch.zeros(ar.total, dtype=torch.float32, device=dev)
        self.v = torch.zeros(ar.total, dtype=torch.float32, device=dev)
        self.step_count = 0
        self.norm_out = torch.zeros(2, dtype=torch.float32, device=dev)     # [global norm, clip coef]
        self.nparts_call = _lib.query("ctr_norm_nparts_per_call")
        self.norm_parts = torch.zeros(4 * self.nparts_call, dtype=torch.float32, device=dev)
        self._seg_key = None
        self._segs_dev = None
        self._norm_key = None
        self._norm_arr = None
        self._build_chunks()
        # exact lazy table update (csrc/lazy.hip): tables leave the dense stream; rows are replayed to
        # the current tick when read, when they get a gradient, or at flush()
        self.lazy = bool(lazy)
        self.tick = 0
        self._flushed_tick = 0
        if self.lazy:
            self._init_lazy()
        object.__setattr__(model, "_fused_opt", self)
        self.engine.lazy = self if self.lazy else None
        self.shards = self.engine.shards
        # data parallel: the dense grads are all-reduced in two buckets -- the head (qnn.* / fc.*: the last
        # dense params of the arena and ~98 % of their bytes at cfg2), started by the engine as soon as
        # the head's backward is done and overlapped with the DARE backward, then the rest
        self._early, self._early_started = None, False
        self._head_lo = self._head_offset()
        if process_group is not None and self._head_lo is not None:
            self.engine.grad_ready = self._head_ready
        if self.shards is not None:
            if process_group is None:
                raise ValueError("row-sharded tables need the process_group they are sharded over")
            self.shards.lazy = self if self.lazy else None

    def _head_offset(self):
        ar = self.arena
        offs = [ar.offsets[k] for k in ar.order if ar.kind[k] == "dense" and k.split(".")[0] in ("qnn", "fc")
                and ar.offsets[k] < ar.n_dense_grad]
        return min(offs) if offs else None

    def _head_ready(self):
        from . import dist as D
        self._early_started = True
        self._early = D.allreduce_sum_async(self.arena.grad[self._head_lo:self.arena.n_dense_grad], self.pg)

    def _reduce_dense(self):
        """Sum the dense grads over the ranks: the head bucket was started during the backward (when the
        engine reached that point), the rest now; the current stream then waits for both."""
        from . import dist as D
        g, n = self.arena.grad, self.arena.n_dense_grad
        started, work = self._early_started, self._early
        self._early_started, self._early = False, None
        lo = self._head_lo if started else n
        D.allreduce_sum_(g[:lo], self.pg)
        if work is not None:
            work.wait()

    # -------------------------------------------------------------- layout
    def _segments(self, tg):
        """Segment table: dense-grad region, no-grad region, then one sparse segment per table."""
        ar, eng, a = self.arena, self.engine, self.engine.a
        segs = []
        if ar.n_dense_grad > 0:
            segs.append(dict(p_off=0, n=ar.n_dense_grad, width=1, kind=0, g_off=0))
        lo, hi = ar.nograd_range
        if hi > lo:
            segs.append(dict(p_off=lo, n=hi - lo, width=1, kind=2, g_off=0))
        for key in ["dare.emb_att.weight", "dare.emb_rep.weight"] + [f"cat_embs.{c}.weight" for c in a.cat_names]:
            shp = ar.shapes[key]
            if key == "dare.emb_att.weight":
                name, base = "att", 0
            elif key == "dare.emb_rep.weight":
                name, base = "rep", 0
            else:
                name, base = "cat", int(eng.cat_row_base_np[a.cat_names.index(key[9:-7])])
            t = tg.get(name) if tg else None
            segs.append(dict(p_off=ar.offsets[key], n=int(np.prod(shp)), width=shp[1], kind=1, g_off=0,
                             keys=ptr(t["keys"]) if t else None, G=ptr(t["G"]) if t else None,
                             n_uniq=ptr(t["n_uniq"]) if t else None, g_ld=t["G"].shape[1] if t else 0,
                             key_base=base, name=name))
        return segs

    def _build_chunks(self):
        segs = self._segments(None)
        CH = _lib.query("ctr_opt_chunk_elems")
        lists = {"all": [], "adam": [], "all_dense": [], "adam_dense": []}
        for si, sg in enumerate(segs):
            n4 = (sg["n"] + 3) // 4 * 4     # stream whole float4s; the tail sits in the 64-element padding
            for e0 in range(0, n4, CH):
                c = (si, e0, min(n4, e0 + CH))
                lists["all"].append(c)
                if sg["kind"] != 2:
                    lists["adam"].append(c)
                if sg["kind"] != 1:
                    lists["all_dense"].append(c)
                if sg["kind"] == 0:
                    lists["adam_dense"].append(c)
        self._chunk_all = lists["all"]
        self._chunks_dev = {}
        for name, lst in lists.items():
            arr = (OptChunk * max(1, len(lst)))()
            for i, (si, e0, e1) in enumerate(lst):
                arr[i].seg, arr[i].pad, arr[i].e0, arr[i].e1 = si, 0, e0, e1
            raw = np.frombuffer(bytes(arr), dtype=np.uint8).copy()
            self._chunks_dev[name] = (torch.from_numpy(raw).to(self.arena.device), len(lst))
        self.krange = torch.zeros(2 * max(1, len(self._chunk_all)), dtype=torch.int32, device=self.arena.device)

    def _init_lazy(self):
        ar, eng, a = self.arena, self.engine, self.engine.a
        dev = ar.device
        keys = ["dare.emb_att.weight", "dare.emb_rep.weight"] + [f"cat_embs.{c}.weight" for c in a.cat_names]
        total = sum(ar.shapes[k][0] for k in keys)
        self.last = torch.zeros(total, dtype=torch.int32, device=dev)
        tabs, r0 = {}, 0
        for k in keys:
            rows, width = ar.shapes[k]
            base = int(eng.cat_row_base_np[a.cat_names.index(k[9:-7])]) if k.startswith("cat_embs.") else 0
            tabs[k] = (ar.offsets[k], rows, width, base, ptr(self.last, r0))
            r0 += rows
        self._lazy_max_rows = max(t[1] for t in tabs.values())

        def dev_tabs(names):
            arr = (_lib.LazyTab * len(names))()
            for i, k in enumerate(names):
                arr[i].p_off, arr[i].rows, arr[i].width, arr[i].key_base, arr[i].last = tabs[k]
            raw = np.frombuffer(bytes(arr), dtype=np.uint8).copy()
            return torch.from_numpy(raw).to(dev), len(names)

        cat = [f"cat_embs.{c}.weight" for c in a.cat_names]     # key_base ascending = X_cat column order
        self._lazy_tabs = {"att": dev_tabs(keys[:1]), "rep": dev_tabs(keys[1:2]), "seq": dev_tabs(keys[:2]),
                           "cat": dev_tabs(cat), "all": dev_tabs(keys)}
        self._seq_width = ar.shapes[keys[0]][1]
        self._seq_rows = ar.shapes[keys[0]][0]
        self._hist_entry = _lib.query("ctr_opt_hist_entry_bytes")
        self.hist = torch.zeros(1024 * self._hist_entry, dtype=torch.uint8, device=dev)

    def _hist_for(self, tick):
        if (tick + 1) * self._hist_entry > self.hist.numel():
            h = torch.zeros(2 * self.hist.numel(), dtype=torch.uint8, device=self.arena.device)
            h[:self.hist.numel()].copy_(self.hist)
            self.hist = h
        return self.hist

    def _ema_ptr(self):
        return ptr(self.ema.shadow) if self.ema is not None else None

    def touch_rows(self, X, group):
        """Bring the table rows a batch reads up to the current tick (called by Engine.forward):
        group "cat": X = X_cat (B, Fc), column c indexes table c; "seq": X = seq (B, L), each token a
        row of both DARE tables."""
        if self.tick == self._flushed_tick:
            return
        if group == "seq":      # both DARE tables of each token (lazy.hip, pair kernels); the padding token,
            # which most left-padded histories hold, is claimed once
            call("ctr_lazy_touch_pair_hot", ptr(self._lazy_tabs["seq"][0]), self._seq_width, ptr(X), X.numel(),
                 int(self.engine.a.pad_id), ptr(self.arena.buf), ptr(self.m), ptr(self.v), self._ema_ptr(),
                 ptr(self.hist), self.tick, self.engine.s())
            return
        tabs, n = self._lazy_tabs[group]
        call("ctr_lazy_touch", ptr(tabs), n, ptr(X), X.shape[0], X.shape[1], 1,
             ptr(self.arena.buf), ptr(self.m), ptr(self.v), self._ema_ptr(), ptr(self.hist), self.tick,
             self.engine.s())

    def touch_local(self, loc_seq, loc_cat):
        """Row-sharded tables: bring the local rows other ranks requested this step current (owner side
        of TableShards.fetch): loc_seq rows of both DARE shards, loc_cat local categorical keys."""
        if self.tick == self._flushed_tick:
            return
        st = self.engine.s()
        if loc_seq.numel():
            call("ctr_lazy_touch_pair", ptr(self._lazy_tabs["seq"][0]), self._seq_width, ptr(loc_seq),
                 loc_seq.numel(), ptr(self.arena.buf), ptr(self.m), ptr(self.v), self._ema_ptr(), ptr(self.hist),
                 self.tick, st)
        if loc_cat.numel():
            tabs, n = self._lazy_tabs["cat"]
            call("ctr_lazy_touch", ptr(tabs), n, ptr(loc_cat), loc_cat.numel(), 1, 2, ptr(self.arena.buf),
                 ptr(self.m), ptr(self.v), self._ema_ptr(), ptr(self.hist), self.tick, st)

    @torch.no_grad()
    def flush(self):
        """Replay every table row to the current tick: afterwards arena, moments and EMA shadow hold
        exactly what the dense stream would (call before reading them as a whole)."""
        if not self.lazy or self.tick == self._flushed_tick:
            return
        # the DARE pair and the categorical tables are disjoint rows: their flushes run side by side (both
        # are bound by memory latency and replay issue, neither fills the chip alone)
        with self.engine.side():
            call("ctr_lazy_flush_pair", ptr(self._lazy_tabs["seq"][0]), self._seq_width, self._seq_rows,
                 ptr(self.arena.buf), ptr(self.m), ptr(self.v), self._ema_ptr(), ptr(self.hist), self.tick,
                 self.engine.s())
        tabs, n = self._lazy_tabs["cat"]
        call("ctr_lazy_flush", ptr(tabs), n, self._lazy_max_rows, ptr(self.arena.buf), ptr(self.m), ptr(self.v),
             self._ema_ptr(), ptr(self.hist), self.tick, self.engine.s())
        self.engine.join()
        self._flushed_tick = self.tick

    def _segs_device(self, tg):
        # the table segments only change when the compact grad buffers do: key on their pointers (building
        # the segment list every step cost ~0.25 ms of host time, exposed when the host is behind)
        key = tuple((ptr(t["keys"]), ptr(t["G"]), ptr(t["n_uniq"]), t["G"].shape[1])
                    for t in (tg.get(n) for n in ("att", "rep", "cat")) if t) if tg else None
        if key != self._seg_key or self._segs_dev is None:
            segs = self._segments(tg)
            arr = (OptSeg * len(segs))()
            for i, s in enumerate(segs):
                o = arr[i]
                o.p_off, o.n, o.width, o.kind, o.g_off = s["p_off"], s["n"], s["width"], s["kind"], s["g_off"]
                o.keys, o.G, o.n_uniq = s.get("keys"), s.get("G"), s.get("n_uniq")
                o.g_ld, o.key_base = s.get("g_ld", 0), s.get("key_base", 0)
            raw = np.frombuffer(bytes(arr), dtype=np.uint8).copy()
            # pinned + non-blocking: a rebuild (row-sharded exchange buffers that grew) must not stall the host
            # on the device (the host allocator keeps the pinned block until the copy has run)
            self._segs_dev = torch.from_numpy(raw).pin_memory().to(self.arena.device, non_blocking=True)
            self._seg_key = key
        return self._segs_dev

    # -------------------------------------------------------------- step
    def _norm_rows(self, tg):
        """The three compact row-grad tables as ctr_sqnorm_all's host array (rebuilt only when the buffers move)."""
        ts = [tg[name] for name in ("att", "rep", "cat")]
        key = tuple((ptr(t["keys"]), ptr(t["G"]), ptr(t["n_uniq"]), t["width"], t["G"].shape[1]) for t in ts)
        if key != self._norm_key:
            arr = (_lib.SqnormRows * len(key))()
            for o, k in zip(arr, key):
                o.keys, o.G, o.n_uniq, o.width, o.ld = k
            self._norm_arr, self._norm_key = arr, key
        return self._norm_arr

    def clip(self, tg, rows=None):
        """Global grad L2 norm over dense grads + deduplicated table rows -> (norm, coef) on device."""
        st = self.engine.s()
        parts = self.norm_parts
        n = self.nparts_call
        # dense + the three tables' partials in one launch (the bits of ctr_sqnorm_dense + 3 ctr_sqnorm_rows)
        rows = rows if rows is not None else self._norm_rows(tg)
        call("ctr_sqnorm_all", ptr(self.arena.grad), self.arena.n_dense_grad, rows, len(rows), INVALID_KEY,
             ptr(parts, 0), st)
        if self.shards is not None:     # each rank holds its own rows' grads: sum the table partials
            from . import dist as D
            D.allreduce_sum_(parts[n:], self.pg)
        # the DDP mean over the ranks that hold rows this step (all of them except on an epoch's short last
        # step, where tossctr.train.rank_slice leaves some ranks empty: their zero gradients do not count)
        div = self.world if self.contributors is None else self.contributors
        call("ctr_clip_finalize", ptr(parts), 4 * n, self.max_grad_norm, 1.0 / div, ptr(self.norm_out), st)
        return self.norm_out

    # -------------------------------------------------------------- data parallel
    def exchange(self, tg):
        """DDP semantics over RCCL: dense grads all-reduced (summed; the 1/world mean is folded into the
        clip multiplier), each table's compact (keys, rows) all-gathered and re-deduplicated so every
        rank applies the same global row grads (replicated tables stay bitwise identical)."""
        from . import dist as D
        eng = self.engine
        self._reduce_dense()
        out = {}
        st = eng.s()
        W = eng.ws(-1, -1)
        for name in ("att", "cat"):
            t = tg[name]
            n, w = t["n"], t["width"]
            keys = W.get(f"dp_{name}_keys", (self.world * n,), torch.int32)
            rows = W.get(f"dp_{name}_rows", (self.world * n, w))
            cnt = W.get(f"dp_{name}_cnt", (self.world,), torch.int32)
            D.gather_compact(t["keys"][:n], t["G"][:n], t["n_uniq"], keys, rows, cnt, self.pg)
            call("ctr_mask_tail_keys", ptr(keys), n, self.world, ptr(cnt), st)
            if name == "cat":
                out[name] = eng._rowgrad(W, "dp_cat", keys, rows, self.world * n, w, w, eng.cat_key_bits)
                continue
            # rep grads share att's keys (ctr_rowgrad2 in the backward): gather their rows in the same
            # slot order and merge both with one sort
            rrows = W.get("dp_rep_rows", (self.world * n, w))
            D.all_gather_into(rrows, tg["rep"]["G"][:n], self.pg)
            out["att"], out["rep"] = eng._rowgrad2(W, keys, rows, rrows, self.world * n, w, eng.seq_key_bits,
                                                   name="dp_seq")
        return out

    def time_kernels(self, on):
        """Bracket each fused-optimizer launch with HIP events on the stream it runs on."""
        self._timing = bool(on)
        if on:
            self._events = []

    def kernel_ms(self):
        torch.cuda.synchronize()
        if not self._events:
            return float("nan")
        return sum(a.elapsed_time(b) for a, b in self._events) / len(self._events)

    def step(self, tg=None, global_step=None):
        """clip (if max_grad_norm > 0) -> AdamW -> EMA (if bound and due at global_step)."""
        tg = tg if tg is not None else self.engine.tg
        if self.shards is not None:
            self._reduce_dense()
            tg = self.shards.route(tg, tg["fx"])
            self.engine.tg = tg
        elif self.pg is not None:
            tg = self.exchange(tg)
            self.engine.tg = tg
        g = self.param_groups[0]
        # everything the update launches need is put together BEFORE the clip is issued: the clip's kernels are short
        # and the device drains them faster than the host issues them, so host work between the clip and the update
        # sat in the trace as an idle gap (24 us a step, profiles/r06/gaps_final.md); issued here it overlaps the
        # backward's long kernels instead
        do_ema = 0
        decay = 0.0
        if self.ema is not None and global_step is not None and self.ema.wants_update(global_step):
            do_ema = 1
            decay = self.ema.next_decay()
        segs = self._segs_device(tg)
        chunks, n = self._chunks_dev[("all" if do_ema else "adam") + ("_dense" if self.lazy else "")]
        b1, b2 = g["betas"]
        shadow = ptr(self.ema.shadow) if self.ema is not None else ptr(self.arena.buf)
        tick = self.tick + 1 if self.lazy else self.tick
        head = (ptr(chunks), n, ptr(segs), ptr(self.krange), ptr(self.arena.buf), ptr(self.m), ptr(self.v), shadow,
                ptr(self.arena.grad), ptr(self.norm_out, 1), float(g["lr"]), float(g["weight_decay"]), float(b1),
                float(b2), float(g["eps"]), self.step_count + 1, float(decay))
        rows = self._norm_rows(tg)
        updates = []
        if self.lazy:
            hist = ptr(self._hist_for(tick))
            ta, tr, tc = tg["att"], tg["rep"], tg["cat"]
            if ta["keys"] is tr["keys"] and ta["G"].shape[1] == tr["G"].shape[1]:
                # att and rep grads share their keys: one wave per key updates both rows
                updates.append(("ctr_lazy_update_pair", ptr(self._lazy_tabs["seq"][0]), self._seq_width,
                                ptr(ta["keys"]), ptr(ta["G"]), ptr(tr["G"]), ta["G"].shape[1], ptr(ta["n_uniq"]),
                                ta["n"], ptr(self.norm_out, 1), ptr(self.arena.buf), ptr(self.m), ptr(self.v),
                                self._ema_ptr(), hist, tick))
                names = ("cat",)
            else:
                names = ("att", "rep", "cat")
            for name in names:
                t = tg[name]
                tabs, nt = self._lazy_tabs[name]
                updates.append(("ctr_lazy_update", ptr(tabs), nt, ptr(t["keys"]), ptr(t["G"]), t["G"].shape[1],
                                ptr(t["n_uniq"]), t["n"], ptr(self.norm_out, 1), ptr(self.arena.buf), ptr(self.m),
                                ptr(self.v), self._ema_ptr(), hist, tick))
        self.clip(tg, rows)
        self.step_count += 1
        st = self.engine.s()
        if self._timing:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        if self.lazy:
            # the tick's scalars go to the lazy tables' history in the same launches as the dense update
            self.tick = tick
            call("ctr_adamw_ema_hist", *head, do_ema, hist, tick, st)
        else:
            call("ctr_adamw_ema", *head, 1, do_ema, st)
        for u in updates:
            call(*u, st)
        if self._timing:
            ev[1].record()
            self._events.append(ev)
        if do_ema:
            self.ema.num_updates += 1

    def ema_only(self, ema, global_step):
        if not ema.wants_update(global_step):
            return
        decay = ema.next_decay()
        segs = self._segs_device(None)
        chunks, n = self._chunks_dev["all_dense" if self.lazy else "all"]
        g = self.param_groups[0]
        if self.lazy:
            if ema is not self.ema:
                raise RuntimeError("lazy FusedAdamW: the EMA must be the one bound at construction")
            self.tick += 1
            call("ctr_opt_hist_record", ptr(self._hist_for(self.tick)), self.tick, float(g["lr"]),
                 float(g["weight_decay"]), 0.9, 0.999, 1e-8, max(1, self.step_count), float(decay), 0, 1,
                 self.engine.s())
        call("ctr_adamw_ema", ptr(chunks), n, ptr(segs), ptr(self.krange), ptr(self.arena.buf), ptr(self.m),
             ptr(self.v), ptr(ema.shadow), ptr(self.arena.grad), None, float(g["lr"]), float(g["weight_decay"]), 0.9, 0.999,
             1e-8, max(1, self.step_count), float(decay), 0, 1, self.engine.s())
        ema.num_updates += 1

    def zero_grad(self, set_to_none=True):
        pass   # grads are overwritten every backward
