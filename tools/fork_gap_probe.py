"""Does a side-stream fork (event record on the main stream + wait on the side stream) cost a boundary on the
main stream?  Three patterns, 20 repetitions each, under rocprofv3 --kernel-trace (tools/fork_gap_summary.py):
  plain: A -> B on the main stream
  fork:  A -> [record ev on main; side waits ev; side runs S] -> B on main
  fork0: A -> [record ev on main; side waits ev] -> B on main (no side kernel)
A writes 400 MB (a fill), B and S are small fills.  The gap is start(B) - end(A) in the trace."""
import torch

dev = torch.device("cuda", 0)
big = torch.empty(100 << 20, device=dev)
small = torch.empty(1 << 16, device=dev)
side_buf = torch.empty(1 << 16, device=dev)
side = torch.cuda.Stream(device=dev)
main = torch.cuda.current_stream(dev)
evs = [torch.cuda.Event() for _ in range(64)]


def pattern(kind, i):
    big.fill_(1.0 + i)                                   # A
    if kind != "plain":
        ev = evs[i % 64]
        ev.record(main)
        side.wait_event(ev)
        if kind == "fork":
            with torch.cuda.stream(side):
                side_buf.fill_(2.0)                      # S
    small.fill_(3.0 + (kind == "fork") + 2 * (kind == "fork0"))   # B (value tags the pattern)


for _ in range(3):
    for k in ("plain", "fork", "fork0"):
        pattern(k, 0)
torch.cuda.synchronize()
for k in ("plain", "fork", "fork0"):
    for i in range(20):
        pattern(k, i)
    torch.cuda.synchronize()
print("done")
