"""World-2 K-fold training run (tossctr.train.main) for tests/test_gpu_train.py, started as a child
process; both ranks share cuda:0 over gloo, tables row-sharded.

    python tests/dist_train_worker.py CFG_JSON OUT_JSON
"""
import json
import os
import socket
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for _p in (HERE, REPO, os.path.join(REPO, "toss-next-ctr-prediction_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def run(rank, world, port, cfg_path, out_path):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from tossctr.train import main
    with open(cfg_path) as f:
        cfg = json.load(f)
    res = main(cfg)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump({str(k): v for k, v in res.items()}, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(run, args=(2, port, sys.argv[1], sys.argv[2]), nprocs=2, join=True)
