"""Instruction mix of a kernel's MFMA loop from hipcc -S output (static count per iteration).

usage: python tools/isa_mix.py file.s mangled_kernel_name
The loop is the outermost `Loop Header` block whose back edge encloses v_mfma instructions."""
import collections
import re
import sys


def loop_mix(asm, name):
    i = asm.index(name + ":")
    body = asm[i:asm.index(".Lfunc_end", i)].splitlines()
    heads = {m.group(1): n for n, l in enumerate(body) if (m := re.match(r"^(\.LBB\w+):.*Loop Header", l))}
    best = None
    for n, l in enumerate(body):
        m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if m and m.group(1) in heads and heads[m.group(1)] < n:
            lo = heads[m.group(1)]
            seg = body[lo:n + 1]
            if any("v_mfma" in x for x in seg) and (best is None or n + 1 - lo > best[1] - best[0]):
                best = (lo, n + 1)
    seg = body[best[0]:best[1]] if best else body
    cnt, ops = collections.Counter(), collections.Counter()
    for l in seg:
        t = l.strip().split()
        if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
            continue
        op = t[0]
        k = ("mfma" if op.startswith("v_mfma") else "valu" if op.startswith("v_") else "lds" if op.startswith("ds_")
             else "vmem" if op.startswith(("global_", "buffer_")) else "salu" if op.startswith("s_") else op)
        cnt[k] += 1
        if k == "valu":
            ops[op] += 1
    return cnt, ops


if __name__ == "__main__":
    c, o = loop_mix(open(sys.argv[1]).read(), sys.argv[2])
    print(dict(c))
    print(o.most_common(25))
