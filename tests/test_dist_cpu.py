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


# ---------------------------------------------------------------- row-sharded tables (tossctr/shard.py)
def a2a_worker(rank, world, port, out):
    """Each rank requests a ragged set of rows from every owner and receives them back: the two
    all-to-alls of TableShards.fetch (keys out, rows back) with host-known split sizes."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tossctr import dist as D
    from tossctr.shard import full_to_local
    table = torch.arange(40 * 3, dtype=torch.float32).view(40, 3)      # full table, row r owned by r % world
    local = full_to_local(table, rank, world)
    g = np.random.default_rng(7 + rank)
    want = np.unique(g.integers(0, 40, 17))
    owner = want % world
    order = np.lexsort((want // world, owner))                         # owner-major, as ctr_shard_plan sorts
    want, owner = want[order], owner[order]
    send = [int((owner == w).sum()) for w in range(world)]
    cnt = torch.empty(world, dtype=torch.int64)
    D.all_to_all_var(cnt, torch.tensor(send, dtype=torch.int64), [1] * world, [1] * world)
    recv = cnt.tolist()
    req = torch.empty(sum(recv), dtype=torch.int32)
    D.all_to_all_var(req, torch.from_numpy((want // world).astype(np.int32)), recv, send)
    rows = local[req.long()]                                           # owner gathers its local rows
    back = torch.empty(len(want), 3)
    D.all_to_all_var(back, rows, send, recv)
    out[rank] = (want, back.numpy().copy(), table.numpy())
    dist.destroy_process_group()


def test_shard_all_to_all_roundtrip_gloo_world2():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(a2a_worker, args=(world, free_port(), out), nprocs=world, join=True)
    for r in range(world):
        want, back, table = out[r]
        np.testing.assert_array_equal(back, table[want])


def test_shard_layout_helpers_and_cfg5_key_widths():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "toss-next-ctr-prediction_amd"))
    from tossctr.arch import Arch
    from tossctr.configs import N_NUM_NEXT, cat_cardinals, dare_qnn_next_k100_s1
    from tossctr.shard import TableShards, full_to_local, locals_to_full, shard_rows
    full = torch.randn(23, 5)
    for world in (1, 2, 3, 8):
        parts = torch.stack([full_to_local(full, r, world) for r in range(world)])
        assert parts.shape == (world, shard_rows(23, world), 5)
        assert torch.equal(locals_to_full(parts, 23), full)
    # BASELINE config 5: every hash_buckets = 1e8, emb_dim 64, 8 ranks -> owner-major keys fit 32 bits
    cfg = dare_qnn_next_k100_s1(emb_dim=64, hash_buckets=100_000_000)
    cards = cat_cardinals(cfg)
    arch = Arch.from_cfg(cfg, 10_000_000, N_NUM_NEXT, N_NUM_NEXT, cards, list(cfg["data"]["cat_cols"]))
    for world in (2, 4, 8):
        sh = TableShards(arch, None, 0, world, torch.device("cpu"))
        assert sh.seq_kbits <= 32 and sh.cat_kbits <= 32
        assert sum(sh.cat_local_rows) * world >= sum(cards.values())
        # every valid owner-major key stays below the INVALID sentinel's truncated value
        top = ((world - 1) << sh.cat_lbits) | (sum(sh.cat_local_rows) - 1)
        assert top < (1 << sh.cat_kbits) - 1
        top = ((world - 1) << sh.seq_lbits) | (sh.seq_rows - 1)
        assert top < (1 << sh.seq_kbits) - 1


def test_fold_parallel_assignment():
    """dist: {mode: folds}: every fold of the K-fold split is trained by exactly one rank, round-robin."""
    from tossctr.train import fold_owner
    for world in (2, 3, 5, 8):
        for n in (5, 7, 10):
            owners = [fold_owner(f, world) for f in range(n)]
            assert all(0 <= o < world for o in owners)
            counts = [owners.count(r) for r in range(world)]
            assert max(counts) - min(counts) <= 1 and sum(counts) == n
