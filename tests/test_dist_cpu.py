"""world_size-2 gloo test (CPU) of the data-parallel exchange: dense all-reduce + compact table-grad
all-gather, merged the way FusedAdamW.exchange merges them (invalidate tail slots, global dedup)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_SLOTS, WIDTH = 50, 6


def rank_data(r):
    g = np.random.default_rng(100 + r)
    cnt = int(g.integers(10, N_SLOTS))
    keys = np.sort(g.choice(200, cnt, replace=False)).astype(np.int32)
    keys = np.concatenate([keys, g.integers(0, 1000, N_SLOTS - cnt).astype(np.int32)])   # garbage tail
    rows = g.standard_normal((N_SLOTS, WIDTH)).astype(np.float32)
    dense = g.standard_normal(37).astype(np.float32)
    return keys, rows, cnt, dense


def merge(keys_all, rows_all, counts, world):
    """numpy restatement of ctr_mask_tail_keys + ctr_rowgrad (stable order of contributions)."""
    acc = {}
    for r in range(world):
        for i in range(counts[r]):
            k = int(keys_all[r * N_SLOTS + i])
            acc[k] = acc.get(k, 0) + rows_all[r * N_SLOTS + i].astype(np.float64)
    ks = sorted(acc)
    return np.array(ks), np.stack([acc[k] for k in ks])


def worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tossctr import dist as D
    keys, rows, cnt, dense = rank_data(rank)
    kt, rt = torch.from_numpy(keys), torch.from_numpy(rows)
    ct = torch.tensor([cnt], dtype=torch.int32)
    ko = torch.empty(world * N_SLOTS, dtype=torch.int32)
    ro = torch.empty(world * N_SLOTS, WIDTH)
    co = torch.empty(world, dtype=torch.int32)
    D.gather_compact(kt, rt, ct, ko, ro, co, None)
    dt = torch.from_numpy(dense.copy())
    D.allreduce_sum_(dt, None)
    out[rank] = (ko.numpy().copy(), ro.numpy().copy(), co.numpy().copy(), dt.numpy().copy())
    dist.destroy_process_group()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_dp_exchange_gloo_world2():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(worker, args=(world, free_port(), out), nprocs=world, join=True)
    datas = [rank_data(r) for r in range(world)]
    exp_dense = sum(d[3].astype(np.float64) for d in datas)
    exp_counts = np.array([d[2] for d in datas])
    for r in range(world):
        ko, ro, co, dt = out[r]
        assert np.array_equal(co, exp_counts)
        for q in range(world):   # rank order of the gathered blocks
            assert np.array_equal(ko[q * N_SLOTS:(q + 1) * N_SLOTS], datas[q][0])
        assert np.allclose(dt, exp_dense, atol=1e-5)
    k0, g0 = merge(*out[0][:3], world)
    k1, g1 = merge(*out[1][:3], world)
    assert np.array_equal(k0, k1) and np.array_equal(g0, g1)      # replicas apply identical row grads
    # union of both ranks' valid keys, summed where they overlap
    allk = sorted(set(datas[0][0][:datas[0][2]]) | set(datas[1][0][:datas[1][2]]))
    assert list(k0) == allk
