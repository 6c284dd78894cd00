"""ctypes binding of libctrhip.so (the C ABI in include/ctr_hip.h).

The product path has NO fallback: if the library is missing or fails to load this module raises,
and every op that needs it fails loudly.  Build with ``make -C toss-next-ctr-prediction_amd``
(or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# CTR_LIB_PATH: an alternative build of the same library (kernel A/B experiments, tools/ only)
LIB_PATH = os.environ.get("CTR_LIB_PATH") or os.path.join(_HERE, "libctrhip.so")

p, i, l, f, u, z = C.c_void_p, C.c_int, C.c_long, C.c_float, C.c_uint32, C.c_size_t
COLSUM_MAXSEG = 16      # CTR_COLSUM_MAXSEG


class GemmEpi(C.Structure):
    _fields_ = [("bias", p), ("add", p), ("ld_add", i), ("act", i), ("pre", p), ("dact", i), ("aux", p),
                ("drop_key", u), ("drop_thresh", u), ("drop_scale", f), ("resid", p), ("ld_resid", i),
                ("norm_w", p), ("norm_h", p), ("norm_r", p), ("norm_eps", f)]


class GemmSeg(C.Structure):
    _fields_ = [("A2", p), ("lda2", i), ("ka", i), ("B2", p), ("ldb2", i), ("nb", i), ("C2", p), ("ldc2", i),
                ("nc", i)]


class OptSeg(C.Structure):
    _fields_ = [("p_off", C.c_int64), ("n", C.c_int64), ("width", C.c_int32), ("kind", C.c_int32),
                ("g_off", C.c_int64), ("keys", p), ("G", p), ("n_uniq", p), ("g_ld", C.c_int32),
                ("key_base", C.c_uint32)]


class SqnormRows(C.Structure):
    _fields_ = [("keys", p), ("G", p), ("n_uniq", p), ("width", i), ("ld", i)]


class OptChunk(C.Structure):
    _fields_ = [("seg", C.c_int32), ("pad", C.c_int32), ("e0", C.c_int64), ("e1", C.c_int64)]


class ColsumSeg(C.Structure):
    _fields_ = [("X", p), ("ld", C.c_long), ("M", i), ("N", i), ("out", p), ("div", f), ("pad", i)]


class Seg(C.Structure):
    _fields_ = [("src", p), ("dst", p), ("n", C.c_longlong)]


class LazyTab(C.Structure):
    _fields_ = [("p_off", C.c_int64), ("rows", C.c_int64), ("width", C.c_int32), ("key_base", C.c_uint32),
                ("last", p)]


# name: (restype, argtypes) -- keep in the order of include/ctr_hip.h
SIGS = {
    "ctr_last_error": (C.c_char_p, []),
    "ctr_abi_version": (i, []),
    "ctr_gemm_ws_size": (z, [i, i, i]),
    "ctr_gemm": (i, [i, i, i, p, i, i, p, i, i, p, i, C.POINTER(GemmEpi), i, p, p]),
    "ctr_gemm_seg": (i, [i, i, i, p, i, i, p, i, i, p, i, C.POINTER(GemmEpi), i, p, C.POINTER(GemmSeg), p]),
    "ctr_gemm_ex": (i, [i, i, i, p, i, i, p, i, i, p, i, C.POINTER(GemmEpi), i, p, C.POINTER(GemmSeg), i, p]),
    "ctr_gemm_bf16_ok": (i, [i, i, i, i, i, i, i, i]),
    "ctr_gemm_bf16": (i, [i, i, i, p, i, i, p, i, i, p, i, C.POINTER(GemmEpi), i, p, C.POINTER(GemmSeg), p]),
    "ctr_gemm_bf16_ex": (i, [i, i, i, p, i, i, p, i, i, p, i, C.POINTER(GemmEpi), i, p, C.POINTER(GemmSeg), i, p]),
    "ctr_to_bf16": (i, [p, l, i, i, p, l, p]),
    "ctr_rowgemm_supported": (i, [i, i]),
    "ctr_rowgemm": (i, [i, i, i, p, i, p, i, p, i, p, p, i, p, i, p, p, p, f, p]),
    "ctr_rowgemm_wgrad_rows": (i, [i]),
    "ctr_rowgemm_wgrad": (i, [p, i, p, i, i, i, i, p, l, i, p]),
    "ctr_rowgemm_a16": (i, [i, i, i, p, i, p, i, p, i, p, p, i, p]),
    "ctr_rowgemm_wgrad_y16": (i, [p, i, p, i, i, i, i, p, l, i, p]),
    "ctr_rowgemm_bf_supported": (i, [i, i]),
    "ctr_rowgemm_bf": (i, [i, i, i, p, i, p, i, p, i, p, p, i, p, i, p, p, p, f, p]),
    "ctr_rowgemm_bf_wgrad_rows": (i, [i]),
    "ctr_rowgemm_bf_wgrad": (i, [p, i, p, i, i, i, i, p, l, i, p]),
    "ctr_feat_embed_fwd": (i, [p, i, i, p, p, p, i, i, p, l, p]),
    "ctr_feat_embed_bwd_ws": (z, [i, i, i]),
    "ctr_feat_embed_bwd": (i, [p, i, i, p, p, p, i, i, p, l, p, p, p, p, p]),
    "ctr_feat_embed_fwd2": (i, [p, i, p, p, p, p, p, i, p, p, p, p, i, i, i, l, p]),
    "ctr_feat_embed_bwd2": (i, [p, i, p, p, p, p, p, p, p, p, p, i, p, p, p, p, p, p, p, p, i, i, i, l, p]),
    "ctr_cat_embed_fwd": (i, [p, i, i, p, p, p, p, p, i, i, p, p, l, u, u, f, p]),
    "ctr_cat_embed_bwd_ws": (z, [i, i]),
    "ctr_cat_embed_bwd": (i, [p, i, i, p, p, p, p, p, i, i, p, p, p, p, p, p, p, p]),
    "ctr_context_fwd": (i, [p, l, i, p, l, i, p, i, i, i, i, i, p, p, p, p, p, p]),
    "ctr_context_bwd": (i, [p, l, i, p, l, i, p, i, i, i, i, i, p, p, p, p, l, u, u, f, p, l, p, p, p, p, p]),
    "ctr_dare_topk_fwd": (i, [p, i, i, p, p, p, i, p, i, i, p, p, p, p, p]),
    "ctr_dare_topk_bwd": (i, [p, i, i, p, p, i, p, i, p, p, p, p, p]),
    "ctr_pool_fwd": (i, [p, p, i, i, i, i, u, u, f, p, p, p, p, p, l, p, p]),
    "ctr_pool_bwd": (i, [p, p, p, i, i, i, i, u, u, f, p, p, l, p, p, p, p]),
    "ctr_pos_bias_mean": (i, [p, i, i, p, p]),
    "ctr_pos_bias_grad": (i, [p, i, i, i, p, p]),
    "ctr_attn_mask_words": (i, [i, i, i]),
    "ctr_attn_set_generic": (None, [i]),
    "ctr_gemm_bf16_set_variant": (None, [i]),
    "ctr_attn_fwd": (i, [p, i, i, i, i, p, i, f, u, u, f, p, p, p, p, p]),
    "ctr_attn_bwd_nparts": (i, [i, i, i]),
    "ctr_attn_bwd": (i, [p, p, p, i, i, i, i, p, i, f, u, u, f, p, p, p, p, p, p]),
    "ctr_attn_bf_ok": (i, [i, i, i]),
    "ctr_attn_fwd_bf": (i, [p, i, i, i, i, p, i, f, u, u, f, p, p, p, p, p]),
    "ctr_attn_bwd_bf_oproj_ok": (i, [i, i, i]),
    "ctr_attn_bwd_bf_oproj": (i, [p, p, p, p, i, i, i, i, p, i, f, u, u, f, p, p, p, p, p, p]),
    "ctr_attn_bwd_bf_oproj16": (i, [p, p, p, p, i, i, i, i, p, i, f, u, u, f, p, p, p, p, p, p]),
    "ctr_attn_bwd_bf_layer_ok": (i, [i, i, i]),
    "ctr_attn_bwd_bf_layer16": (i, [p, p, p, p, p, i, i, i, i, p, i, f, u, u, f, p, p, p, p, p, p, p]),
    "ctr_attn_layer_fwd_ok": (i, [i, i, i]),
    "ctr_attn_layer_fwd_bf": (i, [p, i, i, i, i, p, p, p, p, i, f, u, u, f, p, p, p, p, f, p, p, p, p, p, p, p, p]),
    "ctr_attn_layer_fwd_bf16": (i, [p, i, i, i, i, p, p, p, p, i, f, u, u, f, p, p, p, p, f, p, p, p, p, p, p, p, p]),
    "ctr_attn_bwd_bf_nparts": (i, [i]),
    "ctr_attn_bwd_bf": (i, [p, p, p, i, i, i, i, p, i, f, u, u, f, p, p, p, p, p, p]),
    "ctr_ffn_supported": (i, [i, i, i]),
    "ctr_ffn_slab_rows": (i, [i, i, i, i]),
    "ctr_ffn_mask_words": (i, [i, i]),
    "ctr_ffn_fwd": (i, [p, i, i, i, p, p, p, p, p, f, u, u, f, p, p, p, p, p, i, p]),
    "ctr_ffn_bwd": (i, [p, p, i, i, i, p, p, p, u, u, f, p, p, p, l, i, i, p, i, p]),
    "ctr_ffn_bwd_norms": (i, [p, p, p, p, p, p, p, p, i, i, i, p, p, p, u, u, f, p, p, p, l,
                              i, i, i, i, i, i, p, i, p]),
    "ctr_rmsnorm_fwd": (i, [p, l, i, i, p, f, p, l, p, p]),
    "ctr_rmsnorm_fwd_bf": (i, [p, l, i, i, p, f, p, l, p, p, l, p]),
    "ctr_rmsnorm_bwd_nparts": (i, [i, i]),
    "ctr_rmsnorm_bwd": (i, [p, l, p, l, p, p, i, i, p, l, p, l, p, p]),
    "ctr_layernorm_fwd": (i, [p, l, i, i, p, p, f, p, l, p, p, p, l, p]),
    "ctr_layernorm_bwd_nparts": (i, [i, i]),
    "ctr_layernorm_bwd": (i, [p, l, p, l, p, p, p, i, i, p, l, p, l, p, p, p]),
    "ctr_colsum_ws_size": (z, [i, i]),
    "ctr_colsum": (i, [p, l, i, i, f, p, p, p]),
    "ctr_colsum_multi_ok": (i, [C.POINTER(ColsumSeg)]),
    "ctr_colsum_multi_ws_size": (z, [C.POINTER(ColsumSeg), i]),
    "ctr_colsum_multi": (i, [C.POINTER(ColsumSeg), i, p, z, p]),
    "ctr_loss": (i, [p, p, p, i, f, p, p, p, p]),
    "ctr_qnn_ucat": (i, [p, i, i, i, p, i, p]),
    "ctr_qnn_vfull": (i, [p, i, i, i, p, i, p]),
    "ctr_qnn_gram_fwd_ex": (i, [p, l, i, i, i, p, i, p, p, p, p, i, p]),
    "ctr_qnn_gram_bwd_ex": (i, [p, l, i, i, i, p, i, p, p, p, i, p, p, p]),
    "ctr_qnn_passthrough": (i, [p, i, l, i, i, p, l, p]),
    "ctr_qnn_gram_fwd": (i, [p, i, i, i, p, i, p, p, p, p, p]),
    "ctr_qnn_gram_bwd": (i, [p, i, i, i, p, i, p, p, p, i, p, p, p]),
    "ctr_qnn_gram_fwd_zbf": (i, [p, l, i, i, i, p, i, p, p, p, p, i, p]),
    "ctr_qnn_gram_bwd_zbf": (i, [p, l, l, i, i, i, p, i, p, p, p, i, p, p, p]),
    "ctr_qnn_du_combine": (i, [p, p, p, i, i, p, p]),
    "ctr_se_fwd_gate": (i, [p, i, i, p, p, p, p, p, p, p]),
    "ctr_scale_drop": (i, [p, i, i, p, u, u, f, p, l, p]),
    "ctr_scale_drop_bf": (i, [p, i, i, p, u, u, f, p, l, p, l, p]),
    "ctr_se_bwd_ws": (z, [i, i]),
    "ctr_se_bwd": (i, [p, l, i, p, i, i, i, p, p, p, p, p, u, u, f, p, p, p, p, p, p, p]),
    "ctr_rowgrad_ws_size": (z, [i]),
    "ctr_rowgrad": (i, [p, p, i, i, i, i, p, p, p, p, z, p]),
    "ctr_rowgrad2": (i, [p, p, p, i, i, i, i, p, p, p, p, p, z, p]),
    "ctr_opt_chunk_elems": (i, []),
    "ctr_adamw_ema": (i, [p, i, p, p, p, p, p, p, p, p, f, f, f, f, f, i, f, i, i, p]),
    "ctr_adamw_ema_hist": (i, [p, i, p, p, p, p, p, p, p, p, f, f, f, f, f, i, f, i, p, i, p]),
    "ctr_norm_nparts_per_call": (i, []),
    "ctr_sqnorm_dense": (i, [p, l, p, p]),
    "ctr_sqnorm_rows": (i, [p, p, p, i, i, u, p, p]),
    "ctr_sqnorm_all": (i, [p, l, C.POINTER(SqnormRows), i, u, p, p]),
    "ctr_clip_finalize": (i, [p, i, f, f, p, p]),
    "ctr_mask_tail_keys": (i, [p, i, i, p, p]),
    "ctr_opt_hist_entry_bytes": (i, []),
    "ctr_opt_hist_record": (i, [p, i, f, f, f, f, f, i, f, i, i, p]),
    "ctr_lazy_touch": (i, [p, i, p, l, i, i, p, p, p, p, p, i, p]),
    "ctr_lazy_update": (i, [p, i, p, p, i, p, l, p, p, p, p, p, p, i, p]),
    "ctr_lazy_flush": (i, [p, i, l, p, p, p, p, p, i, p]),
    "ctr_lazy_touch_pair": (i, [p, i, p, l, p, p, p, p, p, i, p]),
    "ctr_lazy_touch_pair_hot": (i, [p, i, p, l, i, p, p, p, p, p, i, p]),
    "ctr_lazy_update_pair": (i, [p, i, p, p, p, i, p, l, p, p, p, p, p, p, i, p]),
    "ctr_lazy_flush_pair": (i, [p, i, l, p, p, p, p, p, i, p]),
    "ctr_shard_plan_ws_size": (z, [l]),
    "ctr_shard_plan": (i, [p, l, i, i, i, p, i, i, i, p, p, p, p, p, z, p]),
    "ctr_shard_strip": (i, [p, l, u, p, p]),
    "ctr_shard_gather": (i, [p, l, i, p, i, p, p, p, i, p]),
    "ctr_shard_offsets_ws_size": (z, [l]),
    "ctr_shard_offsets": (i, [p, p, l, l, u, p, p, i, p, i, i, p, p, z, p]),
    "ctr_shard_pack": (i, [p, i, l, p, p, p]),
    "ctr_shard_unpack": (i, [p, p, l, p, i, p]),
    "ctr_copy_segments": (i, [C.POINTER(Seg), i, p]),
    "ctr_calibrate": (i, [p, i, f, i, p, p, i, p, p]),
    "ctr_ensemble": (i, [p, i, i, i, p, i, p, p]),
    "ctr_sigmoid": (i, [p, i, p, p]),
    "ctr_copy2d": (i, [p, l, p, l, i, i, p]),
    "ctr_zero_f32": (i, [p, l, p]),
    "ctr_step_marker": (i, [i, p]),
    "ctr_gather_rows": (i, [p, l, p, i, p, p]),
    "ctr_scatter_rows": (i, [p, p, p, i, i, i, u, l, p, p]),
    "ctr_val_prob": (i, [p, i, f, i, p, p]),
    "ctr_metrics_ws_size": (z, [i]),
    "ctr_ap_wll": (i, [p, p, i, p, p, z, p]),
    "ctr_temp_nll": (i, [p, p, i, f, p, p, z, p]),
    "ctr_hash_utf8": (i, [p, p, l, C.c_uint64, p]),
    "ctr_parse_seq": (l, [p, p, p, l, i, i, p]),
    "ctr_covis_explode_count": (l, [p, p, p, l, i, p]),
    "ctr_covis_explode": (i, [p, p, p, l, i, p, p, p, p]),
    "ctr_covis_ws_size": (z, [l]),
    "ctr_covis_pair_stats": (i, [p, p, p, p, l, p, p, p, p, i, C.c_double, C.c_double, C.c_double, C.c_double, i,
                                 p, p, p, p, p, p, p, p, p, p, z, p]),
    "ctr_covis_row_features": (i, [p, l, p, p, p, p, p, p, i, C.c_double, p, p, p, p, i, p, p]),
}

_lib = None


def load():
    """Load libctrhip.so (raises if it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"HIP kernel library not built: {LIB_PATH} (run `make -C {os.path.dirname(_HERE)}`)")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class CtrError(RuntimeError):
    pass


_timed = {}     # entry name -> (list of (start, end, key) torch.cuda.Event pairs, shape keys to bracket or None = all)
_every = [1, {}]   # bracket one call in `every` of each entry (per-entry call counters): the rest run unbracketed
# entry points reported per call shape: one entry serves launches of different shapes (the three QNN MLP products)
_TIME_KEY = {"ctr_gemm_bf16_ex": lambda a: f"ctr_gemm_bf16_ex@{a[0]}x{a[1]}x{a[2]}" + ("b" if a[15] else "")}


def time_calls(names, every=1):
    """Bracket every call of the named entry points with HIP events on the current stream (the stream
    the library launches on); ``timed_ms()`` reads the per-call averages.  ``time_calls(())`` stops.
    A name may carry a shape key (``ctr_gemm_bf16_ex@MxNxK``): only the entry's calls of that shape are bracketed
    (the bench times just the dominant launch; events around the entry's other shapes would cost step time).
    ``every`` > 1: one call in each group of ``every`` calls of an entry is bracketed, position (group index mod
    every) in the group -- the layers' launches sampled in turn (an event record between two kernels costs a
    boundary of its own); timed_ms() averages per bracketed call."""
    _timed.clear()
    _every[0] = max(1, int(every))
    _every[1] = {}
    for n in names:
        base = n.split("@")[0]
        evs, keys = _timed.setdefault(base, ([], set()))
        if keys is not None:
            if "@" in n:
                keys.add(n)
            else:
                _timed[base] = (evs, None)


def timed_ms():
    """{key: (calls, average ms per call)} of the calls bracketed since time_calls(); the key is the entry name, or
    the name and the call's shape for the entries of _TIME_KEY."""
    import torch
    torch.cuda.synchronize()
    out = {}
    for evs, _ in _timed.values():
        acc = {}
        for a, b, key in evs:
            acc.setdefault(key, []).append(a.elapsed_time(b))
        for key, ts in acc.items():
            out[key] = (len(ts), sum(ts) / len(ts))
    return out


_fns = {}      # name -> bound ctypes function (one dict lookup per call on the launch path)


def call(name, *args):
    fn = _fns.get(name)
    if fn is None:
        fn = _fns[name] = getattr(load(), name)
    ent = _timed.get(name) if _timed else None
    key = None
    if ent is not None:
        kf = _TIME_KEY.get(name)
        key = kf(args) if kf else name
        if ent[1] is not None and key not in ent[1]:
            ent = None
        elif _every[0] > 1:      # one call in each group of `every`, the phase rotating group to group (every
            k = _every[1].get(key, 0)     # position -- e.g. every encoder layer's launch -- is sampled in turn)
            _every[1][key] = k + 1
            e = _every[0]
            if k % e != (k // e) % e:
                ent = None
    if ent is not None:
        import torch
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        rc = fn(*args)
        ev[1].record()
        ent[0].append((ev[0], ev[1], key))
    else:
        rc = fn(*args)
    if rc != 0:
        raise CtrError(f"{name} failed ({rc}): {_lib.ctr_last_error().decode()}")
    return rc


def query(name, *args):
    return getattr(load(), name)(*args)
