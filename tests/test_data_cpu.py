"""CPU tests of the shard cache format and host readers (src/data/dataset.py, build_cache_v1.py layout)."""
import json

import numpy as np
import pytest
import torch

from tossctr.data import (ShardedDataset, collate_sharded, load_labels_groups_for_split, synth_rows,
                          write_shard_cache)


def test_shard_cache_roundtrip_and_collate(tmp_path):
    arr = synth_rows(1000, 5, 5, [50, 60, 70], 12, 300, seed=3)
    man = write_shard_cache(str(tmp_path), arr, shard_rows=300, num_cols=[f"n{i}" for i in range(5)],
                            cat_cols=["a", "b", "c"], group_key="a")
    m = json.load(open(man))
    assert m["rows"] == 1000 and len(m["shards"]) == 4
    assert [s["start"] for s in m["shards"]] == [0, 300, 600, 900]
    assert m["shards"][3]["end"] == 1000
    for k in ("X_num", "X_mask", "X_cat", "seq", "y", "groups", "ids"):
        assert k in m["shards"][0] and "path" in m["shards"][0][k]
    y, g = load_labels_groups_for_split(man)
    assert np.array_equal(y, arr["y"]) and np.array_equal(g, arr["groups"])
    idx = np.array([5, 299, 300, 999, 601])
    ds = ShardedDataset(man, idx, train=True, cat_cols=["a", "b", "c"])
    assert len(ds) == 5
    b = collate_sharded([ds[i] for i in range(len(ds))])
    assert b["X_num"].dtype == torch.float32 and b["X_mask"].dtype == torch.float32
    assert b["X_cat"].dtype == torch.int64 and b["seq"].dtype == torch.int64 and b["y"].dtype == torch.float32
    assert np.array_equal(b["seq"].numpy(), arr["seq"][idx])
    assert np.array_equal(b["X_mask"].numpy(), arr["X_mask"][idx].astype(np.float32))
    assert np.allclose(b["X_num"].numpy(), arr["X_num"][idx])


def test_synth_rows_layout():
    a = synth_rows(500, 4, 4, [10, 20], 30, 100, seed=1)
    seq = a["seq"]
    # right-aligned histories, left padded with pad_id 0 (build_cache_v1.py:150-156)
    for row in seq:
        nz = np.nonzero(row)[0]
        if len(nz):
            assert nz[-1] == 29 and np.all(row[nz[0]:] != 0)
    assert (a["X_num"][a["X_mask"].astype(bool)] == 0).all()
    assert a["X_cat"][:, 0].max() < 10 and a["X_cat"][:, 1].max() < 20


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("n", [1, 7, 96, 100, 257])
def test_rank_slices_cover_epoch_once(n, world):
    """Data-parallel epoch split (tossctr.train.rank_slice): every row of the permutation is trained
    exactly once per epoch, full steps give each rank bs rows, the last step's remainder is spread over
    the ranks; at world 1 the batches are the reference's (ceil(n / bs) of bs rows, the last short)."""
    import math
    from tossctr.train import rank_slice
    bs = 16
    steps = math.ceil(n / (bs * world))
    seen = []
    for step in range(steps):
        sizes = []
        for r in range(world):
            lo, k = rank_slice(n, bs, world, r, step)
            seen.extend(range(lo, lo + k))
            sizes.append(k)
        assert max(sizes) - min(sizes) <= (0 if step < steps - 1 else 1) or step == steps - 1
        if step < steps - 1:
            assert sizes == [bs] * world
    assert sorted(seen) == list(range(n))
    # the gradient average of each step runs over exactly the ranks that hold rows
    from tossctr.train import step_contributors
    for step in range(steps):
        assert step_contributors(n, bs, world, step) == sum(rank_slice(n, bs, world, r, step)[1] > 0
                                                            for r in range(world))
    if world == 1:
        assert [rank_slice(n, bs, 1, 0, s) for s in range(steps)] == \
            [(s * bs, min(bs, n - s * bs)) for s in range(steps)]


def test_unsupported_options_raise():
    from tossctr.train import check_supported
    check_supported({"amp": "none"})
    check_supported({"amp": "bf16", "sampler": {"type": "None"}})
    with pytest.raises(NotImplementedError):
        check_supported({"amp": "fp16"})
    with pytest.raises(NotImplementedError):
        check_supported({"amp": "none", "sampler": {"type": "balanced"}})
