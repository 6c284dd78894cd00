"""Data-parallel collectives for the fused step (one process per GPU, torch.distributed).

backend "nccl" is RCCL on ROCm (xGMI between the GPUs of a node).  The same calls run under "gloo"
(CPU tests, or several ranks sharing one GPU in tests): device tensors are then staged through host
memory, because gloo's all-gather works on CPU tensors.

What crosses the wire per step (cfg2, per rank): the dense grad buffer (4.48 M fp32 = 18 MB, all-reduced)
and, per embedding table group, the rank's compact deduplicated row grads (fixed-size buffers of n
slots + the valid count, all-gathered; n = B*K for the DARE tables, B*Fc for the hashed tables).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def _needs_host_staging(group, t):
    return t.is_cuda and dist.get_backend(group) == "gloo"


def allreduce_sum_(t: torch.Tensor, group=None):
    """In-place sum across ranks."""
    if _needs_host_staging(group, t):
        h = t.cpu()
        dist.all_reduce(h, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, group=group)
    return t


def allreduce_max_(t: torch.Tensor, group=None):
    """In-place elementwise max across ranks."""
    if _needs_host_staging(group, t):
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.MAX, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t


def allreduce_sum_async(t: torch.Tensor, group=None):
    """Start an in-place sum across ranks and return its handle (``wait()`` makes the current stream wait
    for it; None when it already completed).  Under RCCL the collective runs on the process group's own
    stream after everything queued so far on the current stream, i.e. beside the kernels issued after
    this call -- the bucketed overlap of DDP.  gloo (host-staged) completes it here."""
    if _needs_host_staging(group, t):
        allreduce_sum_(t, group)
        return None
    return dist.all_reduce(t, group=group, async_op=True)


def all_gather_into(out: torch.Tensor, inp: torch.Tensor, group=None):
    """out = concat over ranks (rank order) of inp; out.numel() == world * inp.numel()."""
    if _needs_host_staging(group, inp):
        ho = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(ho, inp.cpu().contiguous(), group=group)
        out.copy_(ho)
    else:
        dist.all_gather_into_tensor(out, inp.contiguous(), group=group)
    return out


def gather_compact(keys, rows, count, keys_out, rows_out, count_out, group=None):
    """All-gather one table group's compact grads: keys (n,), rows (n, w), count (1,) per rank ->
    keys_out (world*n,), rows_out (world*n, w), count_out (world,).  Slots >= count of each rank are
    garbage; the caller invalidates them (ctr_mask_tail_keys) before re-deduplicating."""
    all_gather_into(keys_out, keys, group)
    all_gather_into(rows_out, rows, group)
    all_gather_into(count_out, count, group)


def all_to_all_var(out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, group=None):
    """out = concat over source ranks of what each sent here; inp's first in_splits[w] rows (dim 0) go
    to rank w.  Splits are host lists (the row-sharded exchange reads its counts back once per phase)."""
    if _needs_host_staging(group, inp):
        ho = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(ho, inp.cpu().contiguous(), list(out_splits), list(in_splits), group=group)
        out.copy_(ho)
    else:
        dist.all_to_all_single(out, inp.contiguous(), list(out_splits), list(in_splits), group=group)
    return out
