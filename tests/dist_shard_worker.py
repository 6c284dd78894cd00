"""Data-parallel training run for tests/test_gpu_shard.py, started as a child process (it spawns its
ranks before anything in it touches the GPU).  World-2 runs put both ranks on cuda:0 and use gloo
(host-staged): the same collective sequence the RCCL run issues, on one card.

    python tests/dist_shard_worker.py --mode {single,replicated,sharded} --same-batch {0,1}
                                      --lazy {0,1} --out FILE
"""
import argparse
import os
import socket
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for _p in (HERE, REPO, os.path.join(REPO, "toss-next-ctr-prediction_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

CASE, STEPS, B = "tiny_concat", 4, 40


def run(rank, world, port, args):
    import torch
    import torch.distributed as dist
    from golden_util import Fixture, to_torch_batch
    from oracle.model import make_arch
    from oracle.synth import make_batch, make_params
    from tossctr import ArenaEMA, CTRModel, FusedAdamW

    pg = None
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pg = dist.group.WORLD
    torch.cuda.set_device(0)
    fx = Fixture(CASE)
    m, tr = fx.meta, fx.meta["train"]
    vocab = int(m["vocab"]) * 8                 # sparse tables: most rows skip most ticks
    cards = {k: v * 4 + 1 for k, v in fx.cat_cards.items()}
    cols = list(cards)
    arch = make_arch(m["cfg"], vocab, m["Fn"], m["Fm"], cards, cols)
    params = {k: torch.from_numpy(v) for k, v in make_params(arch.param_shapes(), 5, arch.pad_id).items()}
    model = CTRModel(m["cfg"], vocab, m["Fn"], m["Fm"], cards, cols, device="cuda:0", process_group=pg,
                     shard_tables=args.mode == "sharded")
    model.load_state_dict(params)
    ema = ArenaEMA(model, base_decay=0.9)
    opt = FusedAdamW(model, lr=3e-3, weight_decay=0.05, max_grad_norm=tr["clip"] or 1.0, ema=ema, process_group=pg,
                     lazy=bool(args.lazy))
    L = int(m["L"])
    losses = []
    for t in range(STEPS):
        bseed = 1000 + t + (0 if args.same_batch else 100 * rank)
        b = make_batch(B, m["Fn"], m["Fm"], list(cards.values()), L, vocab, seed=bseed)
        opt.param_groups[0]["lr"] = 3e-3 * (1.0 - 0.2 * t)
        inputs = model.stage(to_torch_batch(b))
        y = torch.from_numpy(b["y"]).float().cuda()
        model.train()
        loss = model.train_step(inputs, y, opt, global_step=t + 1, seed=(9 << 32) | t)
        losses.append(float(loss.item()))
    model.eval()
    eb = make_batch(B, m["Fn"], m["Fm"], list(cards.values()), L, vocab, seed=4242 + 7 * rank)
    with torch.no_grad():
        logits = model(to_torch_batch(eb), seed=1)[0].cpu()
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    shadow = {k: v.detach().cpu() for k, v in ema.state_dict()["shadow_params"].items()}
    local_rows = int(model.arena.shapes["dare.emb_att.weight"][0])
    if rank == 0:
        torch.save({"sd": sd, "ema": shadow, "losses": losses, "logits": logits, "gnorm": float(opt.norm_out[0]),
                    "local_rows": local_rows, "vocab": vocab}, args.out)
    if pg is not None:
        dist.barrier()
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=("single", "replicated", "sharded"), required=True)
    ap.add_argument("--same-batch", type=int, default=0)
    ap.add_argument("--lazy", type=int, default=1)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    if args.mode == "single":
        run(0, 1, 0, args)
        return
    import torch.multiprocessing as mp
    mp.spawn(run, args=(2, _free_port(), args), nprocs=2, join=True)


if __name__ == "__main__":
    main()
