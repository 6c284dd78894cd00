"""Step engine: drives the HIP kernels (libctrhip.so) for CTRModel forward / backward.

The reference computes this with eager torch ops under autograd (src/models/*.py); here every
arithmetic op is a hand-written gfx950 kernel and torch is used only for device memory, streams and
(in tossctr/dist.py) collectives.  Activations live in per-(B, L) preallocated buffers, so a step
does no allocation and is graph-capturable.

Buffer names follow the reference's tensors (see the call-stack comments in each method).
"""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np
import torch

from . import _lib
from ._lib import GemmEpi, call
from .arch import QUERY_MODES, Arch
# Side-stream issue order: the main stream's next product is queued before the side stream's grads (its
# event wait then resolves behind queued main-stream work; 4.82 -> 4.79 ms/step).

from .rng import (SITE_DARE, SITE_EMB, SITE_FC, SITE_FFN0, SITE_MLP0, SITE_QNN, SITE_ATTN0, drop_args)

F32 = 4
INVALID_KEY = 0xFFFFFFFF


_raw_stream = torch._C._cuda_getCurrentRawStream


def ptr(t, elems=0):
    return t.data_ptr() + elems * t.element_size() if t is not None else None


def _align(n, a=64):
    return (n + a - 1) // a * a


def _key_bits(n_keys: int) -> int:
    return max(1, int(n_keys).bit_length())


class ParamArena:
    """All parameters in ONE flat fp32 device buffer (so clip + AdamW + EMA is a single stream).

    Layout: [dense params that get grads][dense params without grads][embedding tables]; every
    param starts on a 64-element boundary.  ``views[key]`` are the tensors the nn.Module exposes.
    The dense-with-grad region is mirrored 1:1 by the dense grad buffer ``grad``.
    """

    def __init__(self, arch: Arch, device, shards=None):
        shapes = arch.param_shapes()
        if shards is not None:     # row-sharded tables: this rank's rows only (tossctr/shard.py)
            local = {"dare.emb_att.weight": shards.seq_rows, "dare.emb_rep.weight": shards.seq_rows}
            local.update({f"cat_embs.{c}.weight": r for c, r in zip(arch.cat_names, shards.cat_local_rows)})
            shapes = [(k, (local[k],) + tuple(shp[1:]) if kind == "table" else shp, kind) for k, shp, kind in shapes]
        ng = arch.no_grad_keys()
        groups = ([x for x in shapes if x[2] == "dense" and x[0] not in ng],
                  [x for x in shapes if x[2] == "dense" and x[0] in ng],
                  [x for x in shapes if x[2] == "table"])
        self.offsets, self.shapes, self.kind = {}, {}, {}
        off = 0
        bounds = []
        for g in groups:
            start = off
            for k, shp, kind in g:
                self.offsets[k] = off
                self.shapes[k] = tuple(shp)
                self.kind[k] = kind
                off = _align(off + int(np.prod(shp)))
            bounds.append((start, off))
        self.n_dense_grad = bounds[0][1]
        self.nograd_range = bounds[1]
        self.table_range = bounds[2]
        self.total = off
        self.device = device
        self.buf = torch.zeros(self.total, dtype=torch.float32, device=device)
        # dense grads for every dense param (the no-grad ones are only written on the autograd-compat
        # path); the optimizer / clip read just [0, n_dense_grad)
        self.grad = torch.zeros(max(1, self.nograd_range[1]), dtype=torch.float32, device=device)
        self.order = [k for k, _, _ in shapes]
        self.views = {k: self._view(self.buf, k) for k in self.order}
        self.grad_views = {k: self._view(self.grad, k) for k in self.order if self.kind[k] == "dense"}

    def _view(self, buf, k):
        o, s = self.offsets[k], self.shapes[k]
        return buf[o:o + int(np.prod(s))].view(s)

    def numel(self, k):
        return int(np.prod(self.shapes[k]))


class Workspace:
    """Named, reusable device buffers for one (B, L)."""

    def __init__(self, device):
        self.device = device
        self.t = {}

    def get(self, name, shape, dtype=torch.float32):
        shape = tuple(int(s) for s in shape)
        t = self.t.get(name)
        if t is None or t.shape != shape or t.dtype != dtype:
            t = torch.empty(shape, dtype=dtype, device=self.device)
            self.t[name] = t
        return t

    def get_zeroed(self, name, shape, dtype=torch.float32):
        """Like get(), zero-filled when (re)allocated: for buffers whose unwritten entries must read 0."""
        shape = tuple(int(s) for s in shape)
        t = self.t.get(name)
        if t is None or t.shape != shape or t.dtype != dtype:
            t = torch.zeros(shape, dtype=dtype, device=self.device)
            self.t[name] = t
        return t


class Engine:
    def __init__(self, arch: Arch, arena: ParamArena, shards=None):
        self.a = arch
        self.arena = arena
        self.shards = shards
        self.P = arena.views
        self.G = arena.grad_views
        self.device = arena.device
        self._dev_index = torch.device(self.device).index or 0
        self._pending_cs = None        # deferred column sums (colsum(defer=True)) while a backward collects them
        _lib.load()
        a = arch
        dev = self.device
        # categorical metadata (device arrays)
        self.cat_tab_off = torch.tensor([arena.offsets[f"cat_embs.{c}.weight"] for c in a.cat_names],
                                        dtype=torch.int64, device=dev)
        self.cat_proj_off = torch.tensor([arena.offsets[f"cat_proj.{c}.weight"] for c in a.cat_names],
                                         dtype=torch.int64, device=dev)
        self.cat_dims_t = torch.tensor(a.cat_dims, dtype=torch.int32, device=dev)
        base = np.cumsum([0] + a.cat_cards[:-1]).astype(np.uint64)
        assert int(sum(a.cat_cards)) < 2**32 - 1, "categorical rows exceed 32-bit keys"
        self.cat_row_base_np = base.astype(np.uint32)
        self.cat_row_base = torch.from_numpy(self.cat_row_base_np.view(np.int32)).to(dev)
        self.cat_key_bits = _key_bits(int(sum(a.cat_cards)))
        self.seq_key_bits = _key_bits(a.seq_vocab)
        if shards is not None:
            # the optimizer addresses table rows by LOCAL keys; the forward/backward by fetched-row ids
            self.cat_row_base_np = shards.cat_lbase_np.copy()
            shards.arena_buf = arena.buf
            shards.tabs_seq = self._tab_array(["dare.emb_att.weight", "dare.emb_rep.weight"], [0, 0])
            shards.tabs_cat = self._tab_array([f"cat_embs.{c}.weight" for c in a.cat_names],
                                              [int(x) for x in shards.cat_lbase_np])
        # query column index in the X_cat column order (src/models/wrapper.py:130)
        self.qi = a.cat_cols.index(a.query_key) if a.query_mode != "S2" else 0
        # column order of X_cat = cat_cols; tables are in cardinals order -> must coincide
        if list(a.cat_cols) != list(a.cat_names):
            raise NotImplementedError("cat_cols_order must match the cat_cardinals order")
        self._decay = {}
        self._ws = {}
        self._splitk = {}
        self._gen = 0
        # backward side stream: weight / bias grads whose inputs are final run beside the input-grad chain
        # (one stream per engine; joined before the optimizer and before a data-parallel bucket hand-off)
        self._side = None
        self.side_stream = True      # False: everything on the current stream (A/B experiments)
        self.stream = None
        self.last = None
        self.grad_ready = None   # data parallel: called once the head's dense grads are final (bucket 1)
        # amp: bf16 (src/train.py:133-139,158-164, torch.autocast(bfloat16)): every GEMM-shaped product on the
        # gemm kernel takes bf16-rounded operands on bf16 MFMA with fp32 accumulation; parameters, optimizer
        # state, tables and the element-wise math stay fp32
        self.bf16 = a.amp == "bf16"
        self.gemm_flags = 1 if self.bf16 else 0     # CTR_GEMM_BF16
        self.lazy = None     # a lazy FusedAdamW: table rows are brought current before they are read
        # fused FFN kernels (ffn.hip) when the shape allows; the GEMM path otherwise
        # row-streaming in/out-projection kernels (rowgemm.hip) for the D they are built for
        self.rowgemm = a.n_layers > 0 and all(bool(_lib.query("ctr_rowgemm_supported", k, n))
                                              for k, n in ((a.D, 3 * a.D), (a.D, a.D), (3 * a.D, a.D)))
        # amp: bf16 at the widths the fp32 row kernels do not cover (D = 64): their bf16-operand forms
        # (rowgemm_bf.hip), as the reference's autocast F.linear
        self.rowgemm_bf = bool(self.bf16 and a.n_layers > 0 and not self.rowgemm and
                               all(bool(_lib.query("ctr_rowgemm_bf_supported", k, n))
                                   for k, n in ((a.D, 3 * a.D), (a.D, a.D), (3 * a.D, a.D))))
        self.rowgemm = self.rowgemm or self.rowgemm_bf
        # LayerNorm encoder layers (norm != "rms", layernorm.hip) take the unfused forms: the fused kernels carry
        # RMSNorm in their epilogues
        self.ln = a.layer_norm
        self.ffn_fused = a.n_layers > 0 and not self.ln and \
            bool(_lib.query("ctr_ffn_supported", a.D, a.ffn_hidden, 0)) and self._ffn_contiguous()
        # amp: bf16 -> the fused FFN's bf16-MFMA kernels where their shape constraints hold (D in {32, 64},
        # FF % 32 == 0); other shapes keep the fp32 kernels (more precise than the reference's bf16)
        self.ffn_flags = 1 if (self.bf16 and self.ffn_fused and
                               _lib.query("ctr_ffn_supported", a.D, a.ffn_hidden, 1)) else 0   # CTR_FFN_BF16
        # amp: bf16 -> the attention core on bf16 MFMA (attn_mf.hip: K <= 64, head dim 4 or 8), as the
        # reference's autocast baddbmm / bmm; other shapes keep the fp32 kernels
        self.attn_bf = bool(self.bf16 and a.n_layers > 0 and _lib.query("ctr_attn_bf_ok", a.top_k, a.H, a.D))
        # ... and the layer's in_proj -> attention -> out_proj + residual + RMSNorm in one launch where it fits
        # (attn_mf.hip: K <= 64, D = 32; the same bits as the three launches)
        self.attn_layer = bool(self.attn_bf and self.rowgemm and not self.ln and
                               _lib.query("ctr_attn_layer_fwd_ok", a.top_k, a.H, a.D))
        # ... and in the backward the out-projection's input grad dO = dh1 W_out inside the attention backward
        # (ctr_attn_bwd_bf_oproj: same bits, dO never written)
        self.attn_oproj = bool(self.attn_bf and self.rowgemm and
                               _lib.query("ctr_attn_bwd_bf_oproj_ok", a.top_k, a.H, a.D))
        # ... and with both: qkv and its grad saved in bf16 (the staged operands / the reference's autocast dtype),
        # the in-projection's backward reading the bf16 grad (ctr_rowgemm_a16 / ctr_rowgemm_wgrad_y16)
        # (-67 us a step at cfg2, profiles/r06/ab_qkv16.log)
        self.qkv16 = bool(self.attn_layer and self.attn_oproj and not self.rowgemm_bf)
        # ... and, opt-in (CTR_ATTN_LAYER_BWD=1), the in-projection's input grad + residual inside the attention
        # backward too (ctr_attn_bwd_bf_layer16: ctr_rowgemm_a16's bits).  Not the default: it needs every head of a
        # sample in one 8-wave workgroup, and that form of the attention backward ran 124 -> 173 us a launch, more
        # than the 26 us in_proj launch and its boundary it removes (step +20 us, profiles/r06/ab_attn_layer_bwd.log)
        self.attn_layer_bwd = bool(self.qkv16 and os.environ.get("CTR_ATTN_LAYER_BWD", "0") == "1" and
                                   _lib.query("ctr_attn_bwd_bf_layer_ok", a.top_k, a.H, a.D))

    def _tab_array(self, keys, bases):
        """Device ctr_lazy_tab_t array (no lazy state) describing arena tables."""
        arr = (_lib.LazyTab * len(keys))()
        for i, (k, kb) in enumerate(zip(keys, bases)):
            rows, width = self.arena.shapes[k]
            arr[i].p_off, arr[i].rows, arr[i].width, arr[i].key_base, arr[i].last = \
                self.arena.offsets[k], rows, width, kb, None
        raw = np.frombuffer(bytes(arr), dtype=np.uint8).copy()
        return torch.from_numpy(raw).to(self.device), len(keys)

    def _ffn_contiguous(self):
        """The fused FFN backward colsums its [d norm1.w | dW1 | db1 | dW2 | db2 | d norm2.w] slab straight
        into the grad arena: the six must be dense and in that order."""
        off = self.arena.offsets
        keys = ("norm1.w", "ffn.0.weight", "ffn.0.bias", "ffn.3.weight", "ffn.3.bias", "norm2.w")
        for li in range(self.a.n_layers):
            p = f"dare.layers.{li}."
            o = [off[p + k] for k in keys]
            if o != sorted(o) or any(self.arena.kind[p + k] != "dense" for k in keys):
                return False
        return True

    # ------------------------------------------------------------------ helpers
    def s(self):
        # the raw handle of torch's current stream on this device (torch.cuda.current_stream() builds a
        # Stream object per call: ~5 us of host time, ~130 calls per step)
        return _raw_stream(self._dev_index)

    def ws(self, B, L):
        key = (B, L)
        if key not in self._ws:
            self._ws[key] = Workspace(self.device)
        return self._ws[key]

    def decay_log(self, L):
        # log(exp(-(L-1-l)/max(1,tau)) + 1e-8) evaluated with torch fp32 ops on the host exactly as
        # src/models/dare.py:126-130 does, then uploaded once per L
        if L not in self._decay:
            pos = torch.arange(L)
            d = torch.exp(-(L - 1 - pos).float() / max(1.0, float(self.a.tau)))
            self._decay[L] = torch.log(d + 1e-8).to(self.device)
        return self._decay[L]

    def splitk_ws(self, nfloats):
        """Split-K / colsum scratch, one buffer per stream (the side stream's kernels run concurrently)."""
        st = self.s()
        buf = self._splitk.get(st)
        if buf is None or buf.numel() < nfloats:
            buf = torch.empty(max(nfloats, 1 << 20), dtype=torch.float32, device=self.device)
            self._splitk[st] = buf
        return buf

    class _Side:
        def __init__(self, eng, after=None):
            self.eng = eng
            self.after = after

        def __enter__(self):
            e = self.eng
            if not e.side_stream:
                return self
            if e._side is None:
                e._side = torch.cuda.Stream(device=e.device)
            self.main = torch.cuda.current_stream(e.device)
            ev = self.after
            if ev is None:
                ev = e._event()
                ev.record(self.main)
            e._side.wait_event(ev)
            self.ctx = torch.cuda.stream(e._side)
            self.ctx.__enter__()
            e._side_used = True
            return self

        def __exit__(self, *exc):
            if self.eng.side_stream:
                self.ctx.__exit__(*exc)
            return False

    def _event(self):
        """An event from a reused ring (a wait enqueued on an event binds to the record before it, so a later
        re-record of the same event does not disturb it); saves an event create/destroy per side() / join()."""
        ring = self.__dict__.setdefault("_ev_ring", [])
        if len(ring) < 64:
            ring.append(torch.cuda.Event())
            return ring[-1]
        self._ev_i = (getattr(self, "_ev_i", -1) + 1) % len(ring)
        return ring[self._ev_i]

    def side(self, after=None):
        """Context: the enclosed launches go to the side stream, after everything issued so far on the
        current stream (or, with ``after``, after the point that event marks: see mark()).  Their inputs must
        not be overwritten by later main-stream work before join()."""
        return Engine._Side(self, after)

    def mark(self):
        """An event recorded on the current stream now: side(after=mark) launched later in host order still
        starts behind only the work issued before the mark -- so a long host-side launch sequence (the rocPRIM
        sort's ~20 dispatches) can be issued after the main stream's next kernels are already queued."""
        if not self.side_stream:
            return None
        ev = self._event()
        ev.record(torch.cuda.current_stream(self.device))
        return ev

    def join(self):
        """Current stream waits for the side stream's work."""
        if self._side is not None and getattr(self, "_side_used", False):
            ev = self._event()
            ev.record(self._side)
            torch.cuda.current_stream(self.device).wait_event(ev)
            self._side_used = False

    @staticmethod
    def _tiles(M, N):
        """Workgroup tiles of ctr_gemm's dispatch before split-K (128x128 tiles)."""
        bn = 32 if N <= 32 else 64 if N <= 64 else 96 if N <= 96 else 128
        bm = 64 if (M <= 64 and bn == 128) else 128
        return math.ceil(M / bm) * math.ceil(N / bn)

    def gemm(self, M, N, K, A, lda, ta, Bm, ldb, tb, Cm, ldc, epi=None, splits=1, seg=None):
        """C = op(A) op(B) (+ epilogue); A/B/C are raw pointers.  A grid too small to fill the 256 CUs
        with a deep K (e.g. the QNN MLP's first layer, 32x4 tiles over K = 6400) is split along K."""
        if splits == 1 and K >= 512 and not (epi is not None and epi.norm_w) and self._tiles(M, N) < 256:
            splits = self._split_factor(M, N, K, 256)
        wsp = None
        if splits > 1:
            wsp = ptr(self.splitk_ws(splits * M * N))
        call("ctr_gemm_ex", M, N, K, A, lda, ta, Bm, ldb, tb, Cm, ldc, epi, splits, wsp, seg, self.gemm_flags,
             self.s())

    def bf_image(self, W, name, src, ld, rows, cols, out=None, off=0, ld_out=None):
        """bf16 (RNE) image of a fp32 (rows, cols) operand for ctr_gemm_bf16 (workspace buffer `name`)."""
        ld_out = ld_out or cols
        if out is None:
            out = W.get(name, (rows, ld_out), torch.bfloat16)
        call("ctr_to_bf16", src, ld, rows, cols, ptr(out, off), ld_out, self.s())
        return out

    def gemm_bf(self, M, N, K, A, lda, ta, Bm, ldb, tb, Cm, ldc, epi=None, seg=None, out_bf16=False):
        """C = op(A) op(B) on bf16 operand images (ctr_gemm_bf16, amp: bf16); split-K so that the
        (tiles x splits) grid stays within one wave of 2 workgroups per CU.  ``out_bf16``: C (and the C2
        segment) bf16, the output dtype autocast gives the reference's matmul (no split-K)."""
        tiles = math.ceil(M / 128) * math.ceil(N / 128)
        splits = 1 if out_bf16 else max(1, min(512 // max(tiles, 1), K // 512))
        wsp = ptr(self.splitk_ws(splits * M * N)) if splits > 1 else None
        call("ctr_gemm_bf16_ex", M, N, K, A, lda, ta, Bm, ldb, tb, Cm, ldc, epi, splits, wsp, seg,
             1 if out_bf16 else 0, self.s())     # CTR_GEMM_OUT_BF16

    def bf_ok(self, M, N, K, lda, ta, ldb, tb):
        return self.bf16 and bool(_lib.query("ctr_gemm_bf16_ok", M, N, K, lda, ta, ldb, tb, 1))

    @staticmethod
    def _split_factor(M, N, K, min_depth):
        """Split-K factor: ~1024 workgroups (4 resident per CU), at most 8 splits once the grid has >= 32
        tiles and 32 below 64k-deep K, each split >= min_depth deep (tools/kbench.py --which gemm sweeps,
        profiles/r01/microbench_gemm.log)."""
        tiles = Engine._tiles(M, N)
        s = math.ceil(1024 / tiles)
        s = min(s, 8 if tiles >= 32 else 32 if K < 65536 else s)
        return int(max(1, min(s, K // min_depth)))

    @staticmethod
    def wgrad_splits(M, N, K):
        """Split-K factor for weight-gradient GEMMs (tiny M x N, huge K = rows), splits >= 64 rows deep."""
        return Engine._split_factor(M, N, K, 64)

    def _ln_fwd(self, h, M, N, name, y, mu, rs, ybf=None, ldybf=0):
        """y = LayerNorm(h) with weight / bias ``name``.weight / .bias (nn.LayerNorm, eps 1e-5); the row mean and
        rstd saved for the backward; ybf: y's bf16 image too (row stride ldybf)."""
        call("ctr_layernorm_fwd", ptr(h), N, M, N, ptr(self.P[name + ".weight"]), ptr(self.P[name + ".bias"]), 1e-5,
             ptr(y), N, ptr(mu), ptr(rs), ptr(ybf) if ybf is not None else None, ldybf, self.s())

    def _ln_bwd(self, W, dy, h, mu, rs, M, N, name, dh):
        """LayerNorm backward: dh, and the weight / bias grads of ``name`` through per-block partial rows."""
        npart = _lib.query("ctr_layernorm_bwd_nparts", M, N)
        dwp = W.get(f"ln_dw_part{N}", (npart, N))
        dbp = W.get(f"ln_db_part{N}", (npart, N))
        call("ctr_layernorm_bwd", ptr(dy), N, ptr(h), N, ptr(mu), ptr(rs), ptr(self.P[name + ".weight"]), M, N,
             ptr(dh), N, None, 0, ptr(dwp), ptr(dbp), self.s())
        self.colsum(ptr(dwp), N, npart, N, ptr(self.G[name + ".weight"]))
        self.colsum(ptr(dbp), N, npart, N, ptr(self.G[name + ".bias"]))

    def rowgemm_call(self, M, K, N, A, W, tb, C, bias=None, add=None, resid=None, norm_w=None, norm_h=None,
                     norm_r=None):
        """C (M, N) = A (M, K) W^T (tb) or A W, + bias / + add / residual + RMSNorm (rowgemm.hip; amp at
        D = 64: rowgemm_bf.hip)."""
        call("ctr_rowgemm_bf" if self.rowgemm_bf else "ctr_rowgemm", M, K, N, A, K, W, tb, C, N, bias, add,
             N if add else 0, resid, N if resid else 0, norm_w, norm_h, norm_r, 1e-6, self.s())

    def wgrad_rows(self, W, dY, X, M, n_out, n_in, wkey, bkey, tag="", defer=False, y16=False):
        """dW = dY^T X and db = colsum(dY) of one nn.Linear in one pass (rowgemm.hip): per-wave partial
        slab rows laid out like the grad arena from the weight on, reduced by one fixed-order colsum.
        ``y16``: dY in bf16 (ctr_rowgemm_wgrad_y16)."""
        o0 = self.arena.offsets[wkey]
        o_db = self.arena.offsets[bkey] - o0
        n_sl = o_db + n_out
        ld = (n_sl + 3) // 4 * 4
        bf = "_bf" if self.rowgemm_bf else ""
        rows = _lib.query(f"ctr_rowgemm{bf}_wgrad_rows", M)
        slab = W.get_zeroed(f"wg_slab_{n_out}x{n_in}_{tag}", (rows, ld))     # padding columns stay zero
        call("ctr_rowgemm_wgrad_y16" if y16 else f"ctr_rowgemm{bf}_wgrad", dY, n_out, X, n_in, M, n_out, n_in,
             ptr(slab), ld, o_db, self.s())
        self.colsum(ptr(slab), ld, rows, n_sl, ptr(self.arena.grad, o0), defer=defer)

    def colsum(self, X, ld, M, N, out, div=1.0, defer=False):
        """out = colsum(X) / div.  ``defer``: X is a buffer nothing overwrites before the end of the encoder
        backward (per-layer slabs) -- queue it for the one ctr_colsum_multi launch pair that sums all of them
        (flush_colsums) instead of two launches of its own."""
        if defer and self._pending_cs is not None:
            seg = _lib.ColsumSeg(X, ld, M, N, out, float(div), 0)
            if _lib.query("ctr_colsum_multi_ok", C.byref(seg)) and len(self._pending_cs) < _lib.COLSUM_MAXSEG:
                self._pending_cs.append(seg)
                return
        w = self.splitk_ws(_lib.query("ctr_colsum_ws_size", M, N) // 4 + 1)
        call("ctr_colsum", X, ld, M, N, float(div), out, ptr(w), self.s())

    def flush_colsums(self):
        """The deferred column sums, in one launch pair on the current stream (callers: the side stream, after
        the last producer of the slabs was issued)."""
        segs, self._pending_cs = self._pending_cs, None
        if not segs:
            return
        arr = (_lib.ColsumSeg * len(segs))(*segs)
        nb = _lib.query("ctr_colsum_multi_ws_size", arr, len(segs))
        w = self.splitk_ws(nb // 4 + 1)
        call("ctr_colsum_multi", arr, len(segs), ptr(w), w.numel() * 4, self.s())

    def wgrad(self, dY, ldy, X, ldx, M_rows, n_out, n_in, dW, lddw=None, bias_grad=None):
        """dW[n_out, n_in] = dY^T X over M_rows rows (+ db = colsum(dY))."""
        sp = self.wgrad_splits(n_out, n_in, M_rows)
        self.gemm(n_out, n_in, M_rows, dY, ldy, 1, X, ldx, 0, dW, lddw or n_in, None, sp)
        if bias_grad is not None:
            self.colsum(dY, ldy, M_rows, n_out, bias_grad)

    # ------------------------------------------------------------------ forward
    def forward(self, X_num, X_mask, X_cat, seq, training: bool, seed: int, save: bool, prefetch=None):
        """CTRModel.forward (src/models/wrapper.py:138-176). Inputs are device tensors:
        X_num f32 (B,Fn), X_mask f32 (B,Fm), X_cat int32 (B,Fc), seq int32 (B,L).
        ``prefetch`` = the next batch's (X_cat, seq): row-sharded tables plan its exchange beside this step.
        Returns (logits, prob, aux) views into workspace buffers, and the saved context."""
        a, P = self.a, self.P
        B, L = int(X_cat.shape[0]), int(seq.shape[1])
        K, D = a.K_eff(L), a.D
        F = a.F
        FD = F * D
        W = self.ws(B, L)
        st = self.s()
        sv = {"B": B, "L": L, "K": K, "training": training, "seed": seed, "X_num": X_num, "X_mask": X_mask,
              "X_cat": X_cat, "seq": seq}
        xF = W.get("xF", (B, FD))
        num_off, mask_off, cat_off = D, D + a.Fn * D, D + (a.Fn + a.Fm) * D
        # table rows brought current first (the DARE pair's on the side stream: joined before the top-K select)
        tv = self._table_views(X_cat, seq)
        sv["tv"] = tv
        # ---- numeric / binary embeddings straight into their xF slots (feature_embed.py:19-27,42-48)
        if a.Fn > 0 and a.Fm > 0:      # both groups in one launch
            call("ctr_feat_embed_fwd2", ptr(X_num), a.Fn, ptr(P["num_embed.weight"]), ptr(P["num_embed.bias"]),
                 ptr(P["num_embed.out_proj.weight"]), ptr(xF, num_off), ptr(X_mask), a.Fm, ptr(P["mask_embed.weight"]),
                 None, ptr(P["mask_embed.out_proj.weight"]), ptr(xF, mask_off), B, a.f_embed, D, FD, st)
        elif a.Fn > 0:
            call("ctr_feat_embed_fwd", ptr(X_num), B, a.Fn, ptr(P["num_embed.weight"]), ptr(P["num_embed.bias"]),
                 ptr(P["num_embed.out_proj.weight"]), a.f_embed, D, ptr(xF, num_off), FD, st)
        elif a.Fm > 0:
            call("ctr_feat_embed_fwd", ptr(X_mask), B, a.Fm, ptr(P["mask_embed.weight"]), None,
                 ptr(P["mask_embed.out_proj.weight"]), a.f_embed, D, ptr(xF, mask_off), FD, st)
        # ---- hashed categorical gather + projection (+ emb dropout into xF) (wrapper.py:106-112,149-150)
        cat_e = W.get("cat_e", (B, a.Fc, D))
        if prefetch is not None and self.shards is not None:
            self.shards.prefetch(*prefetch)
        dk = drop_args(seed, SITE_EMB, a.p_emb, training)
        call("ctr_cat_embed_fwd", ptr(tv["xcat"]), B, a.Fc, ptr(self.arena.buf), tv["cat_tab"], tv["cat_off"],
             ptr(self.cat_proj_off), ptr(self.cat_dims_t), tv["cat_ld"], D, ptr(cat_e), ptr(xF, cat_off), FD, *dk, st)
        # ---- context + query (wrapper.py:114-136)
        ctx = W.get("ctx", (B, a.nctx * D))
        hq = W.get("hq", (B, D))
        query = W.get("query", (B, D))
        mode = QUERY_MODES[a.query_mode]
        call("ctr_context_fwd", ptr(xF, num_off), FD, a.Fn, ptr(xF, mask_off), FD, a.Fm, ptr(cat_e), a.Fc, D, B,
             mode, self.qi, ptr(P["ctx_mlp.0.weight"]), ptr(P["ctx_mlp.0.bias"]), ptr(ctx), ptr(hq), ptr(query), st)
        # ---- DARE top-K (dare.py:116-138)
        idx = W.get("topk_idx", (B, K), torch.int32)
        tok = W.get("topk_tok", (B, K), torch.int32)
        vals = W.get("topk_vals", (B, K))
        xs = [W.get("x0", (B, K, D))]
        self.join()                     # the DARE rows' touch (side stream, _table_views)
        call("ctr_dare_topk_fwd", ptr(tv["seq"]), B, L, ptr(query), tv["att"], tv["rep"], D, ptr(self.decay_log(L)), K,
             tv["pad"], ptr(idx), ptr(tok), ptr(vals), ptr(xs[0]), st)
        # ---- encoder layers (dare.py:53-70)
        layers = []
        M = B * K
        scale = float(np.float32(math.sqrt(1.0 / float(D // a.H)))) if a.n_layers else 1.0
        for li in range(a.n_layers):
            pre = f"dare.layers.{li}."
            Ls = {}
            x = xs[-1]
            qkv = W.get(f"qkv{li}", (M, 3 * D), torch.bfloat16 if self.qkv16 else torch.float32)
            relmean = None
            if a.add_pos:
                relmean = W.get(f"relmean{li}", (2 * a.top_k + 1,))
                if not self.attn_layer:      # (the fused layer forward forms the head mean itself)
                    call("ctr_pos_bias_mean", ptr(P[pre + "pbias.rel.weight"]), a.H, 2 * a.top_k + 1, ptr(relmean), st)
            o = W.get(f"o{li}", (M, D))
            mrow = W.get(f"mrow{li}", (B * a.H * K,))
            lrow = W.get(f"lrow{li}", (B * a.H * K,))
            da = drop_args(seed, SITE_ATTN0 + 2 * li, a.mha_p, training)
            amask = W.get(f"amask{li}", (_lib.query("ctr_attn_mask_words", B, K, a.H),), torch.int32) \
                if da[1] else None
            h1 = W.get(f"h1_{li}", (M, D))
            r1 = W.get(f"r1_{li}", (M,))
            x1 = W.get(f"x1_{li}", (M, D))
            if self.attn_layer:
                # in_proj -> attention -> out_proj + residual + RMSNorm in one launch (attn_mf.hip)
                call("ctr_attn_layer_fwd_bf16" if self.qkv16 else "ctr_attn_layer_fwd_bf", ptr(x), B, K, a.H, D,
                     ptr(P[pre + "mha.in_proj_weight"]),
                     ptr(P[pre + "mha.in_proj_bias"]), ptr(P[pre + "pbias.rel.weight"]) if a.add_pos else None,
                     ptr(relmean), a.top_k, scale, *da, ptr(amask),
                     ptr(P[pre + "mha.out_proj.weight"]), ptr(P[pre + "mha.out_proj.bias"]), ptr(P[pre + "norm1.w"]),
                     1e-6, ptr(qkv), ptr(o), ptr(mrow), ptr(lrow), ptr(h1), ptr(r1), ptr(x1), st)
            else:
                if self.rowgemm:
                    self.rowgemm_call(M, D, 3 * D, ptr(x), ptr(P[pre + "mha.in_proj_weight"]), 1, ptr(qkv),
                                      bias=ptr(P[pre + "mha.in_proj_bias"]))
                else:
                    self.gemm(M, 3 * D, D, ptr(x), D, 0, ptr(P[pre + "mha.in_proj_weight"]), D, 1, ptr(qkv), 3 * D,
                              GemmEpi(bias=ptr(P[pre + "mha.in_proj_bias"])))
                call("ctr_attn_fwd_bf" if self.attn_bf else "ctr_attn_fwd", ptr(qkv), B, K, a.H, D, ptr(relmean),
                     a.top_k, scale, *da, ptr(amask), ptr(o), ptr(mrow), ptr(lrow), st)
                if self.ln:     # h1 = x + out_proj(o), then x1 = LayerNorm(h1)
                    if self.rowgemm:
                        self.rowgemm_call(M, D, D, ptr(o), ptr(P[pre + "mha.out_proj.weight"]), 1, ptr(h1),
                                          bias=ptr(P[pre + "mha.out_proj.bias"]), add=ptr(x))
                    else:
                        self.gemm(M, D, D, ptr(o), D, 0, ptr(P[pre + "mha.out_proj.weight"]), D, 1, ptr(h1), D,
                                  GemmEpi(bias=ptr(P[pre + "mha.out_proj.bias"]), add=ptr(x), ld_add=D))
                    self._ln_fwd(h1, M, D, pre + "norm1", x1, W.get(f"mu1_{li}", (M,)), r1)
                elif self.rowgemm:
                    self.rowgemm_call(M, D, D, ptr(o), ptr(P[pre + "mha.out_proj.weight"]), 1, ptr(x1),
                                      bias=ptr(P[pre + "mha.out_proj.bias"]), resid=ptr(x),
                                      norm_w=ptr(P[pre + "norm1.w"]), norm_h=ptr(h1), norm_r=ptr(r1))
                else:
                    self.gemm(M, D, D, ptr(o), D, 0, ptr(P[pre + "mha.out_proj.weight"]), D, 1, ptr(x1), D,
                              GemmEpi(bias=ptr(P[pre + "mha.out_proj.bias"]), resid=ptr(x), ld_resid=D,
                                      norm_w=ptr(P[pre + "norm1.w"]), norm_h=ptr(h1), norm_r=ptr(r1), norm_eps=1e-6))
            FF = a.ffn_hidden
            dfk = drop_args(seed, SITE_FFN0 + 2 * li, a.ffn_p, training)
            h2 = W.get(f"h2_{li}", (M, D))
            r2 = W.get(f"r2_{li}", (M,))
            x2 = W.get(f"x{li + 1}", (B, K, D))
            act = fo = fmask = None
            if self.ffn_fused:
                # Linear -> GELU -> Dropout -> Linear -> +x1 -> RMSNorm in one kernel (ffn.hip)
                fmask = W.get(f"fmask{li}", (_lib.query("ctr_ffn_mask_words", M, FF),), torch.int32) \
                    if dfk[1] else None
                # bf16 weight images for the bf16 backward (W1 | W2^T | W1^T), written by the forward
                fwbf = W.get(f"fwbf{li}", (3 * FF * D,), torch.bfloat16) if self.ffn_flags else None
                call("ctr_ffn_fwd", ptr(x1), M, D, FF, ptr(P[pre + "ffn.0.weight"]), ptr(P[pre + "ffn.0.bias"]),
                     ptr(P[pre + "ffn.3.weight"]), ptr(P[pre + "ffn.3.bias"]), ptr(P[pre + "norm2.w"]), 1e-6, *dfk,
                     ptr(fmask), ptr(x2), ptr(h2), ptr(r2), ptr(fwbf), self.ffn_flags, st)
            else:
                act = W.get(f"ffa{li}", (M, FF))
                fo = W.get(f"ffo{li}", (M, FF))
                self.gemm(M, FF, D, ptr(x1), D, 0, ptr(P[pre + "ffn.0.weight"]), D, 1, ptr(fo), FF,
                          GemmEpi(bias=ptr(P[pre + "ffn.0.bias"]), act=2, pre=ptr(act), drop_key=dfk[0],
                                  drop_thresh=dfk[1], drop_scale=dfk[2]))
                if self.ln:     # h2 = x1 + ffn(x1), then x2 = LayerNorm(h2)
                    self.gemm(M, D, FF, ptr(fo), FF, 0, ptr(P[pre + "ffn.3.weight"]), FF, 1, ptr(h2), D,
                              GemmEpi(bias=ptr(P[pre + "ffn.3.bias"]), add=ptr(x1), ld_add=D))
                    self._ln_fwd(h2, M, D, pre + "norm2", x2, W.get(f"mu2_{li}", (M,)), r2)
                else:
                    self.gemm(M, D, FF, ptr(fo), FF, 0, ptr(P[pre + "ffn.3.weight"]), FF, 1, ptr(x2), D,
                              GemmEpi(bias=ptr(P[pre + "ffn.3.bias"]), resid=ptr(x1), ld_resid=D,
                                      norm_w=ptr(P[pre + "norm2.w"]), norm_h=ptr(h2), norm_r=ptr(r2), norm_eps=1e-6))
            Ls.update(qkv=qkv, relmean=relmean, o=o, mrow=mrow, lrow=lrow, amask=amask, h1=h1, r1=r1, x1=x1,
                      act=act, fo=fo, fmask=fmask, fwbf=fwbf if self.ffn_fused else None,
                      h2=h2, r2=r2)
            layers.append(Ls)
            xs.append(x2)
        # ---- gating pool + aux head (dare.py:150-162)
        w = W.get("pool_w", (B, K))
        u = W.get("u", (B, D))
        aux = W.get("aux", (B,))
        ddr = drop_args(seed, SITE_DARE, a.p_dare, training)
        fcin = None
        if a.use_qnn:
            xf_u, xf_ld = ptr(xF), FD
        else:
            nfc = 1 + (a.Fn > 0) + (a.Fm > 0) + a.Fc
            fcin = W.get("fcin", (B, nfc * D))
            xf_u, xf_ld = ptr(fcin), nfc * D
        call("ctr_pool_fwd", ptr(xs[-1]), ptr(vals), B, K, D, 0 if a.gating == "softmax" else 1, *ddr,
             ptr(P["dare.aux_head.weight"]), ptr(P["dare.aux_head.bias"]), ptr(w), ptr(u), xf_u, xf_ld, ptr(aux), st)
        logits = W.get("logits", (B,))
        if a.use_qnn:
            q = self._qnn_forward(W, xF, B, seed, training, logits)
        else:
            q = self._fc_forward(W, fcin, ctx, cat_e, B, seed, training, logits)
        prob = W.get("prob", (B,))
        call("ctr_sigmoid", ptr(logits), B, ptr(prob), st)
        if save:
            self._gen += 1
            sv.update(gen=self._gen, xF=xF, cat_e=cat_e, ctx=ctx, hq=hq, query=query, idx=idx, tok=tok, vals=vals,
                      xs=xs, layers=layers, w=w, u=u, aux=aux, logits=logits, prob=prob, fcin=fcin, qnn=q, W=W)
            self.last = sv      # the most recent training forward's saved tensors (top-K indices etc.)
        return logits, prob, aux, (sv if save else None)

    def _table_views(self, X_cat, seq):
        """Where the forward / backward read table rows.  Replicated tables: the arena, indexed by the
        batch ids (lazy rows brought current first).  Row-sharded tables: the rows fetched from their
        owners (tossctr/shard.py), indexed by the batch remapped to fetched-row ids (0 = pad)."""
        a, P = self.a, self.P
        if self.shards is None:
            if self.lazy is not None:
                self.lazy.touch_rows(X_cat, "cat")
                # the DARE rows' catch-up (the longest touch, latency-bound) on the side stream beside the
                # embedding / categorical / context forward; the main stream joins it before the top-K select
                with self.side():
                    self.lazy.touch_rows(seq, "seq")
            return dict(fx=None, xcat=X_cat, seq=seq, pad=a.pad_id, cat_tab=None, cat_off=ptr(self.cat_tab_off),
                        cat_ld=0, att=ptr(P["dare.emb_att.weight"]), rep=ptr(P["dare.emb_rep.weight"]),
                        row_base=ptr(self.cat_row_base), seq_bits=self.seq_key_bits, cat_bits=self.cat_key_bits)
        fx = self.shards.fetch(X_cat, seq)
        return dict(fx=fx, xcat=fx["xcat"], seq=fx["seq"], pad=0, cat_tab=ptr(fx["cat"]),
                    cat_off=ptr(self.shards.cat_zero_off), cat_ld=self.shards.CAT_LD, att=ptr(fx["att"]),
                    rep=ptr(fx["rep"]), row_base=ptr(self.shards.cat_zero_base),
                    seq_bits=_key_bits(1 + fx["n_seq"]), cat_bits=_key_bits(1 + fx["n_cat"]))

    def _qnn_forward(self, W, xF, B, seed, training, logits):
        """QNNAlphaDetailed.forward (qnn_alpha.py:109-130)."""
        a, P, st = self.a, self.P, self.s()
        D, F = a.D, a.F
        FD, C, QR = F * D, a.C, a.qh * a.qr
        z = W.get("z", (B, FD))
        rq = W.get("rq", (B,))
        H0 = a.mlp_hidden[0] if a.mlp_hidden else 1
        din = FD + C
        # amp: the MLP's first GEMM runs on a bf16 image of [z | inter], written by z's and inter's producers
        zi_bf = W.get("zi_bf", (B, din), torch.bfloat16) if (self.bf_ok(B, H0, din, din, 0, din, 1) and
                                                              FD % 8 == 0 and FD % 4 == 0) else None
        # amp: the pair interaction reads the same bf16 image (z as the reference's autocast A = z @ U_h takes it,
        # qnn.hip ctr_qnn_gram_*_zbf); with the MLP weight grad on the image too, nothing reads the fp32 z
        # (D = 32: -67 us a step at cfg2, profiles/r06/ab_gram_zbf.log; D = 64 keeps the fp32-z products, whose
        # bf16 form left cfg4's full-shape step outside the reference's band, gputest_gram_zbf.log)
        gram_zbf = bool(zi_bf is not None and D == 32 and self.bf_ok(H0, din, B, H0, 1, din, 0))
        if a.qnn_layer_norm:
            self._ln_fwd(xF, B, FD, "qnn.pre_norm", z, W.get("muq", (B,)), rq, ybf=zi_bf, ldybf=din)
        elif zi_bf is not None:
            call("ctr_rmsnorm_fwd_bf", ptr(xF), FD, B, FD, ptr(P["qnn.pre_norm.w"]), 1e-6,
                 None if gram_zbf else ptr(z), FD, ptr(rq), ptr(zi_bf), din, st)
        else:
            call("ctr_rmsnorm_fwd", ptr(xF), FD, B, FD, ptr(P["qnn.pre_norm.w"]), 1e-6, ptr(z), FD, ptr(rq), st)
        ucat = W.get("ucat", (D, QR))
        call("ctr_qnn_ucat", ptr(P["qnn.U"]), a.qh, D, a.qr, ptr(ucat), 0, st)
        # pair interaction through per-sample Gram matrices: A = z @ Ucat is never formed (qnn.hip)
        blocks = a.qnn_blocks()
        nb = max(1, len(blocks))
        zsum = W.get("qzsum", (nb, B, D))
        gram = W.get("qgram", (B, D * D))
        S = W.get("qS", (nb, B, QR))
        quad = W.get("qquad", (B, QR))
        if gram_zbf:
            for i, (f0, f1) in enumerate(blocks or [(0, F)]):
                call("ctr_qnn_gram_fwd_zbf", ptr(zi_bf, f0 * D), din, B, f1 - f0, D, ptr(ucat), QR, ptr(zsum[i]),
                     ptr(gram), ptr(S[i]), ptr(quad), int(i > 0), st)
        elif blocks:     # pair_grouping 'block' (qnn_alpha.py:99-108): quad and G summed over the blocks
            for i, (f0, f1) in enumerate(blocks):
                call("ctr_qnn_gram_fwd_ex", ptr(z, f0 * D), FD, B, f1 - f0, D, ptr(ucat), QR, ptr(zsum[i]), ptr(gram),
                     ptr(S[i]), ptr(quad), int(i > 0), st)
        else:
            call("ctr_qnn_gram_fwd", ptr(z), B, F, D, ptr(ucat), QR, ptr(zsum), ptr(gram), ptr(S), ptr(quad), st)
        vfull = W.get("qvfull", (QR, C))
        call("ctr_qnn_vfull", ptr(P["qnn.V"]), a.qh, a.qr, a.qP, ptr(vfull), 0, st)
        inter_pre = W.get("inter_pre", (B, C))
        self.gemm(B, C, QR, ptr(quad), QR, 0, ptr(vfull), C, 0, ptr(inter_pre), C)
        gate = g1 = mean = None
        if a.use_se:
            mean = W.get("se_mean", (C,))
            self.colsum(ptr(inter_pre), C, B, C, ptr(mean), div=float(B))
            Cr = C // a.se_r
            g1 = W.get("se_g1", (Cr,))
            gate = W.get("se_gate", (C,))
            call("ctr_se_fwd_gate", ptr(mean), C, Cr, ptr(P["qnn.se.fc.0.weight"]), ptr(P["qnn.se.fc.0.bias"]),
                 ptr(P["qnn.se.fc.2.weight"]), ptr(P["qnn.se.fc.2.bias"]), ptr(g1), ptr(gate), st)
        inter = W.get("inter", (B, C))
        dq_ = drop_args(seed, SITE_QNN, a.qnn_p, training)
        if zi_bf is not None:
            call("ctr_scale_drop_bf", ptr(inter_pre), B, C, ptr(gate), *dq_, ptr(inter), C, ptr(zi_bf, FD), din, st)
        else:
            call("ctr_scale_drop", ptr(inter_pre), B, C, ptr(gate), *dq_, ptr(inter), C, st)
        # MLP on cat[z, inter] without materialising the concat: W0 = [W0a | W0b]
        hs, acts = [], []
        W0 = P["qnn.mlp.0.weight"]
        nh = len(a.mlp_hidden)
        for j in range(nh + 1):
            last = j == nh
            wkey, bkey = f"qnn.mlp.{3 * j}.weight", f"qnn.mlp.{3 * j}.bias"
            n_out = 1 if last else a.mlp_hidden[j]
            out = logits if last else W.get(f"mlp_h{j}", (B, n_out))
            pre = None if last else W.get(f"mlp_a{j}", (B, n_out))
            dm = (0, 0, 1.0) if last else drop_args(seed, SITE_MLP0 + j, a.qnn_p, training)
            epi = GemmEpi(bias=ptr(P[bkey]), act=0 if last else 1, pre=ptr(pre), drop_key=dm[0], drop_thresh=dm[1],
                          drop_scale=dm[2])
            if j == 0 and zi_bf is not None:
                # amp: the bf16 image of [z | inter] (one (B, FD + C) buffer, also the weight grad's operand)
                # and of W0; the bf16-operand GEMM (glds-staged MFMA tiles)
                w0_bf = self.bf_image(W, "w0_bf", ptr(W0), din, n_out, din)
                self.gemm_bf(B, n_out, din, ptr(zi_bf), din, 0, ptr(w0_bf), din, 1, ptr(out), n_out, epi)
            elif j == 0:
                # input [z | inter] (qnn_alpha.py:120-124): one GEMM over both K segments
                self.gemm(B, n_out, FD + C, ptr(z), FD, 0, ptr(W0), din, 1, ptr(out), n_out, epi,
                          seg=_lib.GemmSeg(A2=ptr(inter), lda2=C, ka=FD))
            else:
                kin = a.mlp_hidden[j - 1]
                self.gemm(B, n_out, kin, ptr(hs[-1]), kin, 0, ptr(P[wkey]), kin, 1, ptr(out), n_out, epi)
            if not last:
                hs.append(out)
                acts.append(pre)
        return dict(z=z, rq=rq, ucat=ucat, zsum=zsum, gram=gram, vfull=vfull, S=S, quad=quad, inter_pre=inter_pre,
                    mean=mean, g1=g1, gate=gate, inter=inter, hs=hs, acts=acts,
                    zi_bf=zi_bf, w0_bf=W.t.get("w0_bf") if zi_bf is not None else None, gram_zbf=gram_zbf)

    def _fc_forward(self, W, fcin, ctx, cat_e, B, seed, training, logits):
        """QNN disabled: fc head on [u, mean(num_e), mean(mask_e), cat_embs] (wrapper.py:95-100,167-173)."""
        a, P, st = self.a, self.P, self.s()
        D = a.D
        nfc = fcin.shape[1] // D
        col = 1
        nctx_parts = (a.Fn > 0) + (a.Fm > 0)
        if nctx_parts:   # the ctx buffer holds [num_mean, mask_mean, cat_mean]
            call("ctr_copy2d", ptr(ctx), a.nctx * D, ptr(fcin, D), nfc * D, B, nctx_parts * D, st)
            col += nctx_parts
        call("ctr_copy2d", ptr(cat_e), a.Fc * D, ptr(fcin, col * D), nfc * D, B, a.Fc * D, st)
        fa = W.get("fc_a", (B, 512))
        fh = W.get("fc_h", (B, 512))
        dfk = drop_args(seed, SITE_FC, 0.1, training)
        self.gemm(B, 512, nfc * D, ptr(fcin), nfc * D, 0, ptr(P["fc.0.weight"]), nfc * D, 1, ptr(fh), 512,
                  GemmEpi(bias=ptr(P["fc.0.bias"]), act=1, pre=ptr(fa), drop_key=dfk[0], drop_thresh=dfk[1],
                          drop_scale=dfk[2]))
        self.gemm(B, 1, 512, ptr(fh), 512, 0, ptr(P["fc.3.weight"]), 512, 1, ptr(logits), 1,
                  GemmEpi(bias=ptr(P["fc.3.bias"])))
        return dict(fa=fa, fh=fh)

    # ------------------------------------------------------------------ loss
    def loss(self, sv, y):
        """bce_wll_style(logits, y) + aux_w * bce_wll_style(aux, y) and its grads (src/train.py:71-90,165-168)."""
        W, B = sv["W"], sv["B"]
        out = W.get("loss", (1,))
        dz = W.get("dlogits", (B,))
        dza = W.get("daux", (B,))
        call("ctr_loss", ptr(sv["logits"]), ptr(sv["aux"]), ptr(y), B, float(self.a.aux_w), ptr(out), ptr(dz),
             ptr(dza), self.s())
        return out, dz, (dza if self.a.aux_w > 0 else None)

    # ------------------------------------------------------------------ backward
    def backward(self, sv, dlogits, daux, overlap=True):
        """Backward of the whole model.  Dense grads -> arena.grad; table grads -> compact
        (sorted unique keys, summed rows, count) in self.tg for the optimizer stream.  ``overlap``: let a
        data-parallel optimizer start the head bucket's all-reduce mid-backward (grad_ready)."""
        if sv["gen"] != self._gen:
            raise RuntimeError("backward() must follow the most recent training forward (buffers are reused)")
        a, P, G, st = self.a, self.P, self.G, self.s()
        B, L, K, D = sv["B"], sv["L"], sv["K"], a.D
        W = sv["W"]
        F = a.F
        FD = F * D
        M = B * K
        seed, training = sv["seed"], sv["training"]
        xF = sv["xF"]
        num_off, mask_off, cat_off = D, D + a.Fn * D, D + (a.Fn + a.Fm) * D
        call("ctr_zero_f32", ptr(self.arena.grad), self.arena.grad.numel(), st)
        dxF = W.get("dxF", (B, FD))
        dfc = None
        # ---------------- head
        if a.use_qnn:
            self._qnn_backward(sv, dlogits, dxF)
            du_ptr, du_ld = ptr(dxF), FD
        else:
            dxF.zero_()
            dfc = self._fc_backward(sv, dlogits)
            du_ptr, du_ld = ptr(dfc), dfc.shape[1]
        if overlap and self.grad_ready is not None:
            # the head's grads (the last dense params of the arena: qnn.* / fc.*) are final: their
            # all-reduce runs beside the rest of the backward
            self.join()
            self.grad_ready()
        # ---------------- pool + aux head
        dx = W.get("dx_a", (B, K, D))
        dvals = W.get("dvals", (B, K))
        ddr = drop_args(seed, SITE_DARE, a.p_dare, training)
        call("ctr_pool_bwd", ptr(sv["xs"][-1]), ptr(sv["vals"]), ptr(sv["w"]), B, K, D,
             0 if a.gating == "softmax" else 1, *ddr, ptr(P["dare.aux_head.weight"]), du_ptr, du_ld,
             ptr(daux), ptr(dx), ptr(dvals), st)
        if daux is not None:
            self.gemm(1, D, B, ptr(daux), 1, 1, ptr(sv["u"]), D, 0, ptr(G["dare.aux_head.weight"]), D, None,
                      self.wgrad_splits(1, D, B))
            self.colsum(ptr(daux), 1, B, 1, ptr(G["dare.aux_head.bias"]))
        # ---------------- encoder layers, last to first
        dx_other = W.get("dx_b", (B, K, D))
        self._pending_cs = []          # the layers' slab column sums: one launch pair after the last layer
        for li in reversed(range(a.n_layers)):
            dx, dx_other = self._layer_backward(sv, li, dx, dx_other), dx
        with self.side():
            self.flush_colsums()
        # ---------------- top-K select -> dq, table row contributions
        tg = self.tg = {}
        dq = W.get("dq", (B, D))
        att_c = W.get("att_contrib", (M, D))
        att_k = W.get("att_keys", (M,), torch.int32)
        rep_k = W.get("rep_keys", (M,), torch.int32)
        tv = sv["tv"]
        tg["fx"] = tv["fx"]
        call("ctr_dare_topk_bwd", ptr(sv["tok"]), B, K, ptr(sv["query"]), tv["att"], D, ptr(dvals), tv["pad"], ptr(dq),
             ptr(att_c), ptr(att_k), ptr(rep_k), st)
        # att and rep contributions share their keys (the top-K tokens): one sort for both, on the side stream
        # beside the context / embedding backward (its own sort workspace), issued below
        # ---------------- context / query
        mode = QUERY_MODES[a.query_mode]
        dcat = W.get("dcat", (B, a.Fc, D))
        dpre = W.get("dpre", (B, D))
        dk = drop_args(seed, SITE_EMB, a.p_emb, training)
        call("ctr_context_bwd", ptr(xF, num_off), FD, a.Fn, ptr(xF, mask_off), FD, a.Fm, ptr(sv["cat_e"]), a.Fc, D,
             B, mode, self.qi, ptr(P["ctx_mlp.0.weight"]), ptr(sv["hq"]), ptr(dq),
             ptr(dxF, cat_off) if a.use_qnn else None, FD, *dk, ptr(dfc), dfc.shape[1] if dfc is not None else 0,
             ptr(dxF, num_off), ptr(dxF, mask_off), ptr(dcat), ptr(dpre), st)
        # the DARE rows' dedupe runs on the side stream from here (its inputs are final); its ~20 launches are
        # issued after the main stream's embedding backward is queued (step time unchanged in A/B either way:
        # the two branches meet at the join)
        seq_ready = self.mark()
        if mode != 0:
            self.wgrad(ptr(dpre), D, ptr(sv["ctx"]), a.nctx * D, B, D, a.nctx * D, ptr(G["ctx_mlp.0.weight"]),
                       bias_grad=ptr(G["ctx_mlp.0.bias"]))
        # ---------------- numeric / binary embeddings
        if a.Fn > 0 and a.Fm > 0:      # both groups in one launch per kernel
            fwn = W.get("fe_ws_num", (_lib.query("ctr_feat_embed_bwd_ws", B, a.Fn, D) // 4 + 1,))
            fwm = W.get("fe_ws_mask", (_lib.query("ctr_feat_embed_bwd_ws", B, a.Fm, D) // 4 + 1,))
            call("ctr_feat_embed_bwd2", ptr(sv["X_num"]), a.Fn, ptr(P["num_embed.weight"]), ptr(P["num_embed.bias"]),
                 ptr(P["num_embed.out_proj.weight"]), ptr(dxF, num_off), ptr(G["num_embed.weight"]),
                 ptr(G["num_embed.bias"]), ptr(G["num_embed.out_proj.weight"]), ptr(fwn),
                 ptr(sv["X_mask"]), a.Fm, ptr(P["mask_embed.weight"]), None, ptr(P["mask_embed.out_proj.weight"]),
                 ptr(dxF, mask_off), ptr(G["mask_embed.weight"]), None, ptr(G["mask_embed.out_proj.weight"]),
                 ptr(fwm), B, a.f_embed, D, FD, st)
        elif a.Fn > 0:
            wsz = _lib.query("ctr_feat_embed_bwd_ws", B, a.Fn, D)
            fw = W.get("fe_ws_num", (wsz // 4 + 1,))
            call("ctr_feat_embed_bwd", ptr(sv["X_num"]), B, a.Fn, ptr(P["num_embed.weight"]),
                 ptr(P["num_embed.bias"]), ptr(P["num_embed.out_proj.weight"]), a.f_embed, D, ptr(dxF, num_off), FD,
                 ptr(G["num_embed.weight"]), ptr(G["num_embed.bias"]), ptr(G["num_embed.out_proj.weight"]), ptr(fw),
                 st)
        elif a.Fm > 0:
            wsz = _lib.query("ctr_feat_embed_bwd_ws", B, a.Fm, D)
            fw = W.get("fe_ws_mask", (wsz // 4 + 1,))
            call("ctr_feat_embed_bwd", ptr(sv["X_mask"]), B, a.Fm, ptr(P["mask_embed.weight"]), None,
                 ptr(P["mask_embed.out_proj.weight"]), a.f_embed, D, ptr(dxF, mask_off), FD,
                 ptr(G["mask_embed.weight"]), None, ptr(G["mask_embed.out_proj.weight"]), ptr(fw), st)
        # ---------------- categorical tables + projections
        n_cat = B * a.Fc
        cat_c = W.get_zeroed("cat_contrib", (n_cat, 64))     # columns past a table's d_c: zero, never written
        cat_k = W.get("cat_keys", (n_cat,), torch.int32)
        cws = W.get("cat_ws", (_lib.query("ctr_cat_embed_bwd_ws", B, a.Fc) // 4 + 1,))
        call("ctr_cat_embed_bwd", ptr(tv["xcat"]), B, a.Fc, ptr(self.arena.buf), tv["cat_tab"], tv["cat_off"],
             ptr(self.cat_proj_off), ptr(self.cat_dims_t), tv["cat_ld"], D, ptr(dcat), tv["row_base"], ptr(cat_c),
             ptr(cat_k), ptr(self.arena.grad), ptr(self.cat_proj_off), ptr(cws), st)
        with self.side(after=seq_ready):
            tg["att"], tg["rep"] = self._rowgrad2(W, att_k, att_c, dx, M, D, tv["seq_bits"], ws="rowgrad_ws_side")
        tg["cat"] = self._rowgrad(W, "cat", cat_k, cat_c, n_cat, 64, 64, tv["cat_bits"])
        self.join()
        return tg

    def _rowgrad(self, W, name, keys, contrib, n, width, ld, key_bits):
        uk = W.get(f"{name}_uk", (n,), torch.int32)
        ug = W.get(f"{name}_ug", (n, width))
        nu = W.get(f"{name}_nu", (1,), torch.int32)
        wsz = _lib.query("ctr_rowgrad_ws_size", n)
        rws = W.get("rowgrad_ws", (max(wsz, W.t["rowgrad_ws"].numel() if "rowgrad_ws" in W.t else 0),),
                    torch.uint8)
        call("ctr_rowgrad", ptr(keys), ptr(contrib), n, width, ld, key_bits, ptr(uk), ptr(ug), ptr(nu), ptr(rws),
             rws.numel(), self.s())
        return dict(keys=uk, G=ug, n_uniq=nu, width=width, n=n)

    def _rowgrad2(self, W, keys, contrib_a, contrib_b, n, width, key_bits, name="seq", ws="rowgrad_ws"):
        uk = W.get(f"{name}_uk", (n,), torch.int32)
        ua = W.get(f"{name}_ug_a", (n, width))
        ub = W.get(f"{name}_ug_b", (n, width))
        nu = W.get(f"{name}_nu", (1,), torch.int32)
        wsz = _lib.query("ctr_rowgrad_ws_size", n)
        rws = W.get(ws, (max(wsz, W.t[ws].numel() if ws in W.t else 0),), torch.uint8)
        call("ctr_rowgrad2", ptr(keys), ptr(contrib_a), ptr(contrib_b), n, width, width, key_bits, ptr(uk), ptr(ua),
             ptr(ub), ptr(nu), ptr(rws), rws.numel(), self.s())
        return (dict(keys=uk, G=ua, n_uniq=nu, width=width, n=n), dict(keys=uk, G=ub, n_uniq=nu, width=width, n=n))

    def _layer_backward(self, sv, li, dx2, dout_buf):
        """DAREEncoderLayer backward (dare.py:53-70). dx2: grad wrt layer output. Returns grad wrt input."""
        a, P, G, st = self.a, self.P, self.G, self.s()
        B, K, D = sv["B"], sv["K"], a.D
        M, FF = B * K, a.ffn_hidden
        W = sv["W"]
        Ls = sv["layers"][li]
        pre = f"dare.layers.{li}."
        seed, training = sv["seed"], sv["training"]
        dfk = drop_args(seed, SITE_FFN0 + 2 * li, a.ffn_p, training)
        if self.ffn_fused:
            # one kernel for norm2 backward -> FFN backward (+ residual) -> norm1 backward: recompute
            # pre/GELU/dropout from x1, per-workgroup slabs [d norm1.w | dW1 | db1 | dW2 | db2 | d norm2.w]
            # laid out like the grad arena from norm1.w on -> one colsum lands all six
            off = self.arena.offsets
            o0 = off[pre + "norm1.w"]
            o = [off[pre + k] - o0 for k in ("norm1.w", "ffn.0.weight", "ffn.0.bias", "ffn.3.weight", "ffn.3.bias",
                                             "norm2.w")]
            n_sl = o[5] + D
            ld_sl = (n_sl + 3) // 4 * 4
            nb = _lib.query("ctr_ffn_slab_rows", M, D, FF, self.ffn_flags)
            slab = W.get_zeroed(f"ffn_slab{li}", (nb, ld_sl))
            dh1 = W.get(f"dh1_{li}", (M, D))
            call("ctr_ffn_bwd_norms", ptr(Ls["x1"]), ptr(dx2), ptr(Ls["h2"]), ptr(Ls["r2"]), ptr(P[pre + "norm2.w"]),
                 ptr(Ls["h1"]), ptr(Ls["r1"]), ptr(P[pre + "norm1.w"]), M, D, FF, ptr(P[pre + "ffn.0.weight"]),
                 ptr(P[pre + "ffn.0.bias"]), ptr(P[pre + "ffn.3.weight"]), *dfk, ptr(Ls["fmask"]), ptr(dh1),
                 ptr(slab), ld_sl, *o, ptr(Ls["fwbf"]), self.ffn_flags, st)
            slab_sum = (ptr(slab), ld_sl, nb, n_sl, ptr(self.arena.grad, o0))
        else:
            slab_sum = None
            # x2 = norm2(x1 + ffn(x1))
            dh2 = W.get("dh2", (M, D))
            if self.ln:
                self._ln_bwd(W, dx2, Ls["h2"], W.get(f"mu2_{li}", (M,)), Ls["r2"], M, D, pre + "norm2", dh2)
            else:
                npart = _lib.query("ctr_rmsnorm_bwd_nparts", M, D)
                dwp = W.get("dw_part", (npart, D))
                call("ctr_rmsnorm_bwd", ptr(dx2), D, ptr(Ls["h2"]), D, ptr(Ls["r2"]), ptr(P[pre + "norm2.w"]), M, D,
                     ptr(dh2), D, None, 0, ptr(dwp), st)
                self.colsum(ptr(dwp), D, npart, D, ptr(G[pre + "norm2.w"]))
            dx1 = W.get("dx1", (M, D))
            # ffn.3: f @ W2^T + b2
            self.wgrad(ptr(dh2), D, ptr(Ls["fo"]), FF, M, D, FF, ptr(G[pre + "ffn.3.weight"]),
                       bias_grad=ptr(G[pre + "ffn.3.bias"]))
            dact = W.get("dffa", (M, FF))
            self.gemm(M, FF, D, ptr(dh2), D, 0, ptr(P[pre + "ffn.3.weight"]), FF, 0, ptr(dact), FF,
                      GemmEpi(dact=2, aux=ptr(Ls["act"]), drop_key=dfk[0], drop_thresh=dfk[1], drop_scale=dfk[2]))
            # ffn.0: x1 @ W1^T + b1
            self.wgrad(ptr(dact), FF, ptr(Ls["x1"]), D, M, FF, D, ptr(G[pre + "ffn.0.weight"]),
                       bias_grad=ptr(G[pre + "ffn.0.bias"]))
            self.gemm(M, D, FF, ptr(dact), FF, 0, ptr(P[pre + "ffn.0.weight"]), D, 0, ptr(dx1), D,
                      GemmEpi(add=ptr(dh2), ld_add=D))
            # x1 = norm1(x + attn(x)); per layer: the side stream's out_proj weight grad reads it while the
            # next layer's backward runs on the main stream
            dh1 = W.get(f"dh1_{li}", (M, D))
            if self.ln:
                self._ln_bwd(W, dx1, Ls["h1"], W.get(f"mu1_{li}", (M,)), Ls["r1"], M, D, pre + "norm1", dh1)
            else:
                call("ctr_rmsnorm_bwd", ptr(dx1), D, ptr(Ls["h1"]), D, ptr(Ls["r1"]), ptr(P[pre + "norm1.w"]), M, D,
                     ptr(dh1), D, None, 0, ptr(dwp), st)
                self.colsum(ptr(dwp), D, npart, D, ptr(G[pre + "norm1.w"]))
        # out_proj
        do = W.get("do", (M, D))
        # dO formed inside the attention backward below (attn_oproj): the FFN slab sums and out_proj's weight grad go to
        # the side stream together with the attention backward's side work -- one fork (event record + wait) per
        # layer instead of two, a boundary fewer on the main stream (3.260 -> 3.222 ms a step over four same-box
        # pairs, profiles/r06/ab_merge_fork.log)
        oproj_side = self.attn_oproj
        if oproj_side:
            pass
        elif self.rowgemm:
            if slab_sum is not None:     # main-stream product first, then the side stream's slab sums
                self.rowgemm_call(M, D, D, ptr(dh1), ptr(P[pre + "mha.out_proj.weight"]), 0, ptr(do))
                with self.side():
                    self.colsum(*slab_sum, defer=True)
                    self.wgrad_rows(W, ptr(dh1), ptr(Ls["o"]), M, D, D, pre + "mha.out_proj.weight",
                                    pre + "mha.out_proj.bias", tag=li, defer=True)
            else:
                with self.side():
                    self.wgrad_rows(W, ptr(dh1), ptr(Ls["o"]), M, D, D, pre + "mha.out_proj.weight",
                                    pre + "mha.out_proj.bias", tag=li, defer=True)
                self.rowgemm_call(M, D, D, ptr(dh1), ptr(P[pre + "mha.out_proj.weight"]), 0, ptr(do))
        else:
            if slab_sum is not None:
                with self.side():
                    self.colsum(*slab_sum, defer=True)
            self.wgrad(ptr(dh1), D, ptr(Ls["o"]), D, M, D, D, ptr(G[pre + "mha.out_proj.weight"]),
                       bias_grad=ptr(G[pre + "mha.out_proj.bias"]))
            self.gemm(M, D, D, ptr(dh1), D, 0, ptr(P[pre + "mha.out_proj.weight"]), D, 0, ptr(do), D)
        # attention core
        dqkv = W.get(f"dqkv{li}", (M, 3 * D), torch.bfloat16 if self.qkv16 else torch.float32)
        nparts = (1 if self.attn_layer_bwd else _lib.query("ctr_attn_bwd_bf_nparts", a.H) if self.attn_bf else
                  _lib.query("ctr_attn_bwd_nparts", a.H, K, D)) * B
        nrel = 2 * a.top_k + 1
        drp = W.get(f"drel_part{li}", (nparts, nrel))
        da = drop_args(seed, SITE_ATTN0 + 2 * li, a.mha_p, training)
        scale = float(np.float32(math.sqrt(1.0 / float(D // a.H))))
        if self.attn_layer_bwd:          # + dout = dqkv W_in + dh1 (the in_proj launch below is not needed)
            call("ctr_attn_bwd_bf_layer16", ptr(Ls["qkv"]), ptr(Ls["o"]), ptr(dh1), ptr(P[pre + "mha.out_proj.weight"]),
                 ptr(P[pre + "mha.in_proj_weight"]), B, K, a.H, D, ptr(Ls["relmean"]), a.top_k, scale, *da,
                 ptr(Ls["amask"]), ptr(Ls["mrow"]), ptr(Ls["lrow"]), ptr(dqkv), ptr(drp), ptr(dout_buf), st)
        elif self.attn_oproj:
            call("ctr_attn_bwd_bf_oproj16" if self.qkv16 else "ctr_attn_bwd_bf_oproj", ptr(Ls["qkv"]), ptr(Ls["o"]), ptr(dh1), ptr(P[pre + "mha.out_proj.weight"]),
                 B, K, a.H, D, ptr(Ls["relmean"]), a.top_k, scale, *da, ptr(Ls["amask"]), ptr(Ls["mrow"]),
                 ptr(Ls["lrow"]), ptr(dqkv), ptr(drp), st)
        else:
            call("ctr_attn_bwd_bf" if self.attn_bf else "ctr_attn_bwd", ptr(Ls["qkv"]), ptr(Ls["o"]), ptr(do), B, K,
                 a.H, D, ptr(Ls["relmean"]), a.top_k, scale, *da, ptr(Ls["amask"]), ptr(Ls["mrow"]), ptr(Ls["lrow"]),
                 ptr(dqkv), ptr(drp), st)
        x_in = sv["xs"][li]
        # (here the side work goes first: queuing the in_proj input grad ahead of it measured 0.02 ms/step slower)
        with self.side():
            if oproj_side:
                if slab_sum is not None:
                    self.colsum(*slab_sum, defer=True)
                self.wgrad_rows(W, ptr(dh1), ptr(Ls["o"]), M, D, D, pre + "mha.out_proj.weight",
                                pre + "mha.out_proj.bias", tag=li, defer=True)
            if a.add_pos:
                call("ctr_pos_bias_grad", ptr(drp), nparts, a.H, nrel, ptr(G[pre + "pbias.rel.weight"]), self.s())
            if self.rowgemm:
                self.wgrad_rows(W, ptr(dqkv), ptr(x_in), M, 3 * D, D, pre + "mha.in_proj_weight",
                                pre + "mha.in_proj_bias", tag=li, defer=True, y16=self.qkv16)
        # in_proj
        if self.attn_layer_bwd:
            pass
        elif self.qkv16:
            call("ctr_rowgemm_a16", M, 3 * D, D, ptr(dqkv), 3 * D, ptr(P[pre + "mha.in_proj_weight"]), 0,
                 ptr(dout_buf), D, None, ptr(dh1), D, st)
        elif self.rowgemm:
            self.rowgemm_call(M, 3 * D, D, ptr(dqkv), ptr(P[pre + "mha.in_proj_weight"]), 0, ptr(dout_buf),
                              add=ptr(dh1))
        else:
            self.wgrad(ptr(dqkv), 3 * D, ptr(x_in), D, M, 3 * D, D, ptr(G[pre + "mha.in_proj_weight"]),
                       bias_grad=ptr(G[pre + "mha.in_proj_bias"]))
            self.gemm(M, D, 3 * D, ptr(dqkv), 3 * D, 0, ptr(P[pre + "mha.in_proj_weight"]), D, 0, ptr(dout_buf), D,
                      GemmEpi(add=ptr(dh1), ld_add=D))
        return dout_buf

    def _qnn_backward(self, sv, dlogits, dxF):
        a, P, G, st = self.a, self.P, self.G, self.s()
        B, D, W = sv["B"], a.D, sv["W"]
        q = sv["qnn"]
        F = a.F
        FD, C, QR = F * D, a.C, a.qh * a.qr
        din = FD + C
        seed, training = sv["seed"], sv["training"]
        nh = len(a.mlp_hidden)
        # MLP, last layer first; dact epilogues fold relu' and the dropout mask in
        dcur, ncur = dlogits, 1
        dcur_bf = None
        for j in reversed(range(nh + 1)):
            wkey, bkey = f"qnn.mlp.{3 * j}.weight", f"qnn.mlp.{3 * j}.bias"
            if j > 0:
                kin = a.mlp_hidden[j - 1]
                with self.side():
                    self.wgrad(ptr(dcur), ncur, ptr(q["hs"][j - 1]), kin, B, ncur, kin, ptr(G[wkey]),
                               bias_grad=ptr(G[bkey]))
                dprev = W.get(f"dmlp_a{j - 1}", (B, kin))
                dm = drop_args(seed, SITE_MLP0 + j - 1, a.qnn_p, training)
                self.gemm(B, kin, ncur, ptr(dcur), ncur, 0, ptr(P[wkey]), kin, 0, ptr(dprev), kin,
                          GemmEpi(dact=1, aux=ptr(q["acts"][j - 1]), drop_key=dm[0], drop_thresh=dm[1],
                                  drop_scale=dm[2]))
                dcur, ncur = dprev, kin
            elif q.get("zi_bf") is not None and self.bf_ok(ncur, din, B, ncur, 1, din, 0):
                # amp: dW0 = dcur^T [z | inter] on the forward's bf16 image (both operands k-major)
                dcur_bf = self.bf_image(W, "dcur_bf", ptr(dcur), ncur, B, ncur)
                with self.side():
                    self.gemm_bf(ncur, din, B, ptr(dcur_bf), ncur, 1, ptr(q["zi_bf"]), din, 0, ptr(G[wkey]), din)
                    self.colsum(ptr(dcur), ncur, B, ncur, ptr(G[bkey]))
            else:
                # first layer: W0 = [W0a (over z) | W0b (over inter)]
                with self.side():
                    self.gemm(ncur, FD + C, B, ptr(dcur), ncur, 1, ptr(q["z"]), FD, 0, ptr(G[wkey]), din, None,
                              self.wgrad_splits(ncur, FD + C, B), seg=_lib.GemmSeg(B2=ptr(q["inter"]), ldb2=C, nb=FD))
                    self.colsum(ptr(dcur), ncur, B, ncur, ptr(G[bkey]))
        W0 = P["qnn.mlp.0.weight"]
        bf_da = q.get("w0_bf") is not None and dcur_bf is not None and self.bf_ok(B, din, ncur, ncur, 0, din, 0)
        dz_bf = a.use_residual and bf_da
        dinter = W.get("dinter_bf" if dz_bf else "dinter", (B, C), torch.bfloat16 if dz_bf else torch.float32)
        dz_mlp = W.get("dz_mlp_bf" if dz_bf else "dz_mlp", (B, FD), torch.bfloat16 if dz_bf else torch.float32)
        if dz_bf:   # amp: [dz | dinter] = dcur W0 on bf16 images (W0 k-major: transposed reads), bf16 out as
            # autocast's matmul returns it (the input grad the reference's cat backward splits is bf16)
            self.gemm_bf(B, din, ncur, ptr(dcur_bf), ncur, 0, ptr(q["w0_bf"]), din, 0, ptr(dz_mlp), FD,
                         seg=_lib.GemmSeg(C2=ptr(dinter), ldc2=C, nc=FD), out_bf16=True)
        elif a.use_residual:     # [dz | dinter] = dcur W0: one GEMM, output split at column FD
            self.gemm(B, FD + C, ncur, ptr(dcur), ncur, 0, ptr(W0), din, 0, ptr(dz_mlp), FD,
                      seg=_lib.GemmSeg(C2=ptr(dinter), ldc2=C, nc=FD))
        else:
            self.gemm(B, C, ncur, ptr(dcur), ncur, 0, ptr(W0, FD), din, 0, ptr(dinter), C)
        # SE + dropout
        dinter_pre = W.get("dinter_pre", (B, C))
        dq_ = drop_args(seed, SITE_QNN, a.qnn_p, training)
        Cr = C // a.se_r if a.use_se else 1
        sws = W.get("se_ws", (_lib.query("ctr_se_bwd_ws", B, C) // 4 + 1,))
        call("ctr_se_bwd", ptr(dinter), C, int(dz_bf), ptr(q["inter_pre"]), B, C, Cr, ptr(q["gate"]), ptr(q["g1"]),
             ptr(q["mean"]), ptr(P.get("qnn.se.fc.0.weight")), ptr(P.get("qnn.se.fc.2.weight")), *dq_, ptr(dinter_pre),
             ptr(G.get("qnn.se.fc.0.weight")), ptr(G.get("qnn.se.fc.0.bias")), ptr(G.get("qnn.se.fc.2.weight")),
             ptr(G.get("qnn.se.fc.2.bias")), ptr(sws), st)
        # pair interaction (Gram form, qnn.hip): dquad = dinter Vfull^T; dV = blockdiag(quad^T dinter)
        dquad = W.get("qdquad", (B, QR))
        self.gemm(B, QR, C, ptr(dinter_pre), C, 0, ptr(q["vfull"]), C, 1, ptr(dquad), QR)
        dvfull = W.get("qdvfull", (QR, C))
        with self.side():
            self.gemm(QR, C, B, ptr(q["quad"]), QR, 1, ptr(dinter_pre), C, 0, ptr(dvfull), C, None,
                      self.wgrad_splits(QR, C, B))
            call("ctr_qnn_vfull", ptr(dvfull), a.qh, a.qr, a.qP, ptr(G["qnn.V"]), 1, self.s())
        dz = W.get("dz", (B, FD))
        blocks = a.qnn_blocks()
        DS = W.get("qDS", (max(1, len(blocks)), B, QR))
        dadd = dz_mlp if a.use_residual else None
        if blocks:
            # the features of no block take no interaction grad: dz = the MLP's input grad there
            f_prev = 0
            for f0, f1 in blocks + [(F, F)]:
                if f0 > f_prev:
                    call("ctr_qnn_passthrough", ptr(dadd, f_prev * D), int(dz_bf), FD, B, (f0 - f_prev) * D,
                         ptr(dz, f_prev * D), FD, st)
                f_prev = f1
            for i, (f0, f1) in enumerate(blocks):
                if q["gram_zbf"]:
                    call("ctr_qnn_gram_bwd_zbf", ptr(q["zi_bf"], f0 * D), din, FD, B, f1 - f0, D, ptr(q["ucat"]), QR,
                         ptr(q["S"][i]), ptr(dquad), ptr(dadd, f0 * D), int(dz_bf), ptr(dz, f0 * D), ptr(DS[i]), st)
                else:
                    call("ctr_qnn_gram_bwd_ex", ptr(q["z"], f0 * D), FD, B, f1 - f0, D, ptr(q["ucat"]), QR,
                         ptr(q["S"][i]), ptr(dquad), ptr(dadd, f0 * D), int(dz_bf), ptr(dz, f0 * D), ptr(DS[i]), st)
        elif q["gram_zbf"]:
            call("ctr_qnn_gram_bwd_zbf", ptr(q["zi_bf"]), din, FD, B, F, D, ptr(q["ucat"]), QR, ptr(q["S"]),
                 ptr(dquad), ptr(dadd), int(dz_bf), ptr(dz), ptr(DS), st)
        else:
            call("ctr_qnn_gram_bwd", ptr(q["z"]), B, F, D, ptr(q["ucat"]), QR, ptr(q["S"]), ptr(dquad),
                 ptr(dadd), int(dz_bf), ptr(dz), ptr(DS), st)
        # dUcat = 2 (zsum^T DS - sum_b G_b Ucat diag(dquad_b)); the block form sums zsum_k^T DS_k over the blocks
        T1 = W.get("qT1", (D, QR))
        T = W.get("qT", (D * D, QR))
        ducat = W.get("ducat", (D, QR))
        with self.side():
            for i in range(max(1, len(blocks))):
                self.gemm(D, QR, B, ptr(q["zsum"][i]), D, 1, ptr(DS[i]), QR, 0, ptr(T1), QR,
                          GemmEpi(add=ptr(T1), ld_add=QR) if i > 0 else None, self.wgrad_splits(D, QR, B))
            self.gemm(D * D, QR, B, ptr(q["gram"]), D * D, 1, ptr(dquad), QR, 0, ptr(T), QR, None,
                      self.wgrad_splits(D * D, QR, B))
            call("ctr_qnn_du_combine", ptr(T1), ptr(T), ptr(q["ucat"]), D, QR, ptr(ducat), self.s())
            call("ctr_qnn_ucat", ptr(ducat), a.qh, D, a.qr, ptr(G["qnn.U"]), 1, self.s())
        # pre-norm
        if a.qnn_layer_norm:
            self._ln_bwd(W, dz, sv["xF"], W.get("muq", (B,)), q["rq"], B, FD, "qnn.pre_norm", dxF)
            return
        npart = _lib.query("ctr_rmsnorm_bwd_nparts", B, FD)
        dwp = W.get("dwq_part", (npart, FD))
        call("ctr_rmsnorm_bwd", ptr(dz), FD, ptr(sv["xF"]), FD, ptr(q["rq"]), ptr(P["qnn.pre_norm.w"]), B, FD,
             ptr(dxF), FD, None, 0, ptr(dwp), st)
        with self.side():
            self.colsum(ptr(dwp), FD, npart, FD, ptr(G["qnn.pre_norm.w"]))

    def _fc_backward(self, sv, dlogits):
        a, P, G, st = self.a, self.P, self.G, self.s()
        B, W = sv["B"], sv["W"]
        fcin = sv["fcin"]
        q = sv["qnn"]
        nin = fcin.shape[1]
        self.wgrad(ptr(dlogits), 1, ptr(q["fh"]), 512, B, 1, 512, ptr(G["fc.3.weight"]), bias_grad=ptr(G["fc.3.bias"]))
        dfa = W.get("dfc_a", (B, 512))
        dfk = drop_args(sv["seed"], SITE_FC, 0.1, sv["training"])
        self.gemm(B, 512, 1, ptr(dlogits), 1, 0, ptr(P["fc.3.weight"]), 512, 0, ptr(dfa), 512,
                  GemmEpi(dact=1, aux=ptr(q["fa"]), drop_key=dfk[0], drop_thresh=dfk[1], drop_scale=dfk[2]))
        self.wgrad(ptr(dfa), 512, ptr(fcin), nin, B, 512, nin, ptr(G["fc.0.weight"]), bias_grad=ptr(G["fc.0.bias"]))
        dfcin = W.get("dfcin", (B, nin))
        self.gemm(B, nin, 512, ptr(dfa), 512, 0, ptr(P["fc.0.weight"]), nin, 0, ptr(dfcin), nin)
        return dfcin

    # ------------------------------------------------------------------ compat: dense table grads
    def dense_table_grad(self, key, tg=None, scale=1.0):
        """Materialise the dense gradient of one embedding table from the compact rows (autograd path).
        Row-sharded tables: ``tg`` = the grads routed to this rank's rows (TableShards.route: local keys, the
        local row bases), the result this rank's shard, times ``scale``."""
        if self.shards is not None and tg is None:
            raise RuntimeError("row-sharded tables: pass the routed grads (CTRModel._reduce_sharded_grads)")
        tg = self.tg if tg is None else tg
        a = self.a
        shp = self.arena.shapes[key]
        out = torch.zeros(shp, dtype=torch.float32, device=self.device)
        if key == "dare.emb_att.weight":
            t, base = tg["att"], 0
        elif key == "dare.emb_rep.weight":
            t, base = tg["rep"], 0
        else:
            c = a.cat_names.index(key[len("cat_embs."):-len(".weight")])
            t, base = tg["cat"], int(self.cat_row_base_np[c])
        call("ctr_scatter_rows", ptr(t["keys"]), ptr(t["G"]), ptr(t["n_uniq"]), t["n"], shp[1], t["G"].shape[1],
             base, shp[0], ptr(out), self.s())
        if scale != 1.0:
            out.mul_(scale)
        return out
