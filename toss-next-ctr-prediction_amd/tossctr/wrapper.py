"""CTRModel -- drop-in for src/models/wrapper.py:7-176 on MI355X.

Same constructor signature, same ``forward(batch) -> (logits, prob, aux_logit)`` and the same
``state_dict`` keys/shapes/order as the reference (parameters are views into one device arena, see
engine.ParamArena).  The compute is libctrhip.so; there is no torch/CPU fallback.

Two training paths:
  * reference-style: ``logits, prob, aux = model(batch); loss = f(...); loss.backward()`` works --
    a custom autograd.Function runs the HIP backward and hands torch ordinary dense ``.grad`` tensors
    (tables included; fine for tests / small vocabularies).  With row-sharded tables the backward is
    collective (dense grads averaged over the ranks, row grads sent to their owners; a table's ``.grad``
    is its local shard's) and ``model.clip_grad_norm_`` replaces ``nn.utils.clip_grad_norm_`` (global norm):
    the reference's own call would clip each rank by its local norm, and the next optimizer step raises
    (``_check_replicated_grads``) rather than let the replicas drift; with FusedAdamW bound the table grads stay
    compact and its ``step()`` routes and clips them on the global norm;
  * fused (what tossctr.train and bench.py use): ``model.train_step(...)`` via tossctr.optim --
    table grads stay compact (sorted unique rows) and clip + AdamW + EMA run as one HBM stream.
"""
from __future__ import annotations

import weakref

import torch
import torch.nn as nn

from .arch import Arch
from .engine import Engine, ParamArena, ptr
from . import _lib

# Row-sharded models whose autograd backward left replicated dense grads that the next optimizer step must find still
# identical on every rank (CTRModel._check_replicated_grads).  The reference loop clips with
# nn.utils.clip_grad_norm_(model.parameters()) (src/train.py:189,194): on row-sharded tables that norm is per rank
# (a table's .grad is the local shard's), each rank would scale its replicated dense grads by its own coefficient
# and the replicas would drift apart silently.  The check turns that into an error at the step.
_PENDING_CHECK = weakref.WeakSet()
_STEP_HOOK = None


def _step_pre_hook(optimizer, args, kwargs):
    for model in list(_PENDING_CHECK):
        _PENDING_CHECK.discard(model)
        model._check_replicated_grads()


def _arm_step_check(model):
    global _STEP_HOOK
    if _STEP_HOOK is None:
        from torch.optim.optimizer import register_optimizer_step_pre_hook
        _STEP_HOOK = register_optimizer_step_pre_hook(_step_pre_hook)
    _PENDING_CHECK.add(model)


def _tree_module(root: nn.Module, key: str) -> tuple:
    parts = key.split(".")
    mod = root
    for name in parts[:-1]:
        if name not in mod._modules:
            mod.add_module(name, nn.Module())
        mod = mod._modules[name]
    return mod, parts[-1]


class _Query:
    """`.dare.query_mode` is read by the reference wrapper (src/models/wrapper.py:154)."""


class _CTRFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, inputs, seed, *params):
        logits, prob, aux, sv = model.engine.forward(*inputs, training=True, seed=seed, save=True)
        ctx.model, ctx.sv = model, sv
        ctx.set_materialize_grads(False)
        return logits.clone(), prob.clone(), aux.clone()

    @staticmethod
    def backward(ctx, g_logits, g_prob, g_aux):
        model, sv = ctx.model, ctx.sv
        eng = model.engine
        B = sv["B"]
        dz = torch.zeros(B, device=eng.device) if g_logits is None else g_logits.float().contiguous().clone()
        if g_prob is not None:   # prob = sigmoid(logits): dz += dprob * p * (1 - p)
            p = sv["prob"]
            dz = dz + g_prob * p * (1 - p)
        daux = None if g_aux is None else g_aux.float().contiguous()
        eng.backward(sv, dz, daux, overlap=False)     # torch reads the grads right after: no async reduce
        sh, routed = model.shards, None
        fused = model.__dict__.get("_fused_opt")
        if sh is not None and fused is None:
            # row-sharded tables under a plain torch optimizer: DDP semantics here, in the backward -- the dense
            # grads all-reduced and averaged, each table's row grads sent to their owners (the fused step's
            # exchange, tossctr/shard.py route) and averaged; .grad of a table is then its local shard's
            routed = model._reduce_sharded_grads()
            _arm_step_check(model)
        grads = []
        for k in model.arena.order:
            if model.arena.kind[k] == "table":
                if sh is None:
                    grads.append(eng.dense_table_grad(k))
                elif routed is None:
                    # FusedAdamW bound: its step() routes the engine's compact row grads and clips on the global
                    # norm itself, so no dense shard grad is materialised
                    grads.append(None)
                else:
                    grads.append(eng.dense_table_grad(k, routed, 1.0 / model._contributors()))
            elif k in model.no_grad and not (k.startswith("dare.aux_head") and daux is not None):
                grads.append(None)
            else:
                grads.append(eng.G[k].clone())
        return (None, None, None, *grads)


class CTRModel(nn.Module):
    def __init__(self, cfg, seq_vocab: int, num_feat_dim: int, mask_feat_dim: int, cat_cardinals: dict,
                 cat_cols_order: list, device=None, process_group=None, shard_tables=False):
        """Reference constructor (src/models/wrapper.py:8-9) plus MI355X placement: ``device`` (default:
        the current HIP device) and, for data parallelism, ``shard_tables=True`` with ``process_group``:
        every embedding table is row-sharded over the group's ranks (tossctr/shard.py) -- each rank
        holds rows r with r % world == rank.  Collective from then on: every rank runs forward /
        train_step / state_dict / load_state_dict together."""
        super().__init__()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else None
        if device is None or torch.device(device).type != "cuda":
            raise RuntimeError("tossctr.CTRModel runs only on an MI355X (HIP) device; no CPU fallback")
        _lib.load()
        self.cfg = cfg
        self.arch = Arch.from_cfg(cfg, seq_vocab, num_feat_dim, mask_feat_dim, cat_cardinals, cat_cols_order)
        self.cat_cols_order = list(cat_cols_order)
        self.num_dim, self.mask_dim, self.D = num_feat_dim, mask_feat_dim, self.arch.D
        self.query_key = self.arch.query_key
        self.aux_weight = self.arch.aux_w
        self.use_qnn = self.arch.use_qnn
        shards = None
        if shard_tables:
            import torch.distributed as dist
            from .shard import TableShards
            if process_group is None:
                process_group = dist.group.WORLD
            shards = TableShards(self.arch, process_group, dist.get_rank(process_group),
                                 dist.get_world_size(process_group), torch.device(device))
        object.__setattr__(self, "shards", shards)
        object.__setattr__(self, "arena", ParamArena(self.arch, torch.device(device), shards))
        object.__setattr__(self, "engine", Engine(self.arch, self.arena, shards))
        self.no_grad = self.arch.no_grad_keys()
        for k in self.arena.order:
            mod, name = _tree_module(self, k)
            mod.register_parameter(name, nn.Parameter(self.arena.views[k], requires_grad=True))
        self.dare.query_mode = self.arch.query_mode
        self.seed = int(cfg.get("seed", 777))
        self._step = 0
        self.reset_parameters()

    def sync(self):
        """Bring lazily-updated table rows (FusedAdamW(lazy=True)) up to the current optimizer tick."""
        opt = self.__dict__.get("_fused_opt")
        if opt is not None:
            opt.flush()

    def state_dict(self, *args, **kwargs):
        self.sync()
        sd = super().state_dict(*args, **kwargs)
        if self.shards is not None:     # full tables, as the reference's state_dict has them (collective)
            prefix = kwargs.get("prefix", args[1] if len(args) > 1 else "")
            for k in self.arena.order:
                if self.arena.kind[k] == "table":
                    sd[prefix + k] = self.full_table(self.arena.buf, k)
        return sd

    def load_state_dict(self, state_dict, strict=True, assign=False):
        self.sync()     # moments / EMA of lagging rows must be current before their params change
        if self.shards is not None:     # full tables in, this rank's rows kept
            from .shard import full_to_local
            sh = self.shards
            state_dict = dict(state_dict)
            for k in self.arena.order:
                if self.arena.kind[k] == "table" and k in state_dict:
                    state_dict[k] = full_to_local(torch.as_tensor(state_dict[k]), sh.rank, sh.world)
        return super().load_state_dict(state_dict, strict=strict, assign=assign)

    def full_table(self, buf, key):
        """Parameter ``key`` viewed in an arena-layout buffer (parameters, a moment, the EMA shadow);
        row-sharded tables are gathered from every rank (collective)."""
        v = self.arena._view(buf, key)
        if self.shards is None or self.arena.kind[key] != "table":
            return v
        return self.shards.gather_full(v, self.arch_rows(key))

    def arch_rows(self, key):
        for k, shp, _ in self.arch.param_shapes():
            if k == key:
                return shp[0]
        raise KeyError(key)

    # the arena is not an nn.Module buffer: keep .to()/.cuda() from re-allocating parameters
    def _apply(self, fn, recurse=True):
        return self

    @torch.no_grad()
    def reset_parameters(self, generator=None):
        """Reference default init: nn.Embedding N(0,1) (pad row 0), nn.Linear kaiming-uniform /
        U(+-1/sqrt(fan_in)) biases, RMSNorm w = 1 (LayerNorm weight 1, bias 0), feature slopes N(0, 0.02^2),
        U/V N(0, 0.02^2)."""
        a = self.arch
        g = generator
        gt = g     # row-sharded tables: every rank draws its own rows (dense params stay identical)
        if self.shards is not None:
            base = g.initial_seed() if g is not None else torch.initial_seed()
            gt = torch.Generator(device=self.arena.device).manual_seed(
                (base * 1000003 + 7919 * (self.shards.rank + 1)) % (1 << 63))
        for k in self.arena.order:
            t = self.arena.views[k]
            if k.endswith(".w") or k.endswith(("norm1.weight", "norm2.weight", "pre_norm.weight")):
                t.fill_(1.0)          # RMSNorm w / nn.LayerNorm weight
            elif k.endswith(("norm1.bias", "norm2.bias", "pre_norm.bias")):
                t.zero_()
            elif ".emb_" in k or k.startswith("cat_embs."):
                t.normal_(0.0, 1.0, generator=gt)
                if ".emb_" in k:
                    if self.shards is None:
                        t[a.pad_id].zero_()
                    elif a.pad_id % self.shards.world == self.shards.rank:
                        t[a.pad_id // self.shards.world].zero_()
            elif "pbias.rel" in k:
                t.normal_(0.0, 1.0, generator=g)
            elif k in ("num_embed.weight", "mask_embed.weight", "qnn.U", "qnn.V"):
                t.normal_(0.0, 0.02, generator=g)
            elif k == "num_embed.bias":
                t.zero_()
            else:
                fan_in = t.shape[-1] if t.dim() > 1 else self._fan_in_of_bias(k)
                bound = 1.0 / max(1, fan_in) ** 0.5
                t.uniform_(-bound, bound, generator=g)

    def _fan_in_of_bias(self, k):
        wk = k[: -len("bias")] + "weight"
        if k.endswith("in_proj_bias"):
            return self.D
        if wk in self.arena.shapes:
            return self.arena.shapes[wk][-1]
        return 1

    # ------------------------------------------------------------------ forward
    def _stage(self, batch):
        """X_num/X_mask -> f32, X_cat/seq -> int32 on the model device (src/models/wrapper.py:139-143)."""
        dev = self.arena.device
        X_num = batch["X_num"].to(dev, non_blocking=True).float().contiguous()
        X_mask = batch["X_mask"].to(dev, non_blocking=True).float().contiguous()
        X_cat = batch["X_cat"].to(dev, non_blocking=True).to(torch.int32).contiguous()
        seq = batch["seq"].to(dev, non_blocking=True).to(torch.int32).contiguous()
        return X_num, X_mask, X_cat, seq

    def next_seed(self):
        self._step += 1
        return ((self.seed & 0xFFFFFFFF) << 32) | (self._step & 0xFFFFFFFF)

    def forward(self, batch, seed=None):
        inputs = self._stage(batch)
        if self.training and torch.is_grad_enabled():
            seed = self.next_seed() if seed is None else seed
            return _CTRFunction.apply(self, inputs, seed, *[getattr(*_tree_module(self, k)) for k in self.arena.order])
        logits, prob, aux, _ = self.engine.forward(*inputs, training=self.training,
                                                   seed=self.next_seed() if seed is None else seed, save=False)
        return logits.clone(), prob.clone(), aux.clone()

    # ------------------------------------------------------------------ row-sharded tables, autograd path
    # ranks holding rows in the current step (row-sharded autograd path; None: every rank), as train_step's
    # ``contributors``: an epoch's short last step leaves some ranks without rows (tossctr.train.rank_slice), their
    # zero gradients do not count in the mean
    contributors = None

    def _reduce_sharded_grads(self):
        """Collective (every rank, in the backward): dense grads all-reduced and divided by the number of
        contributing ranks (DDP's mean; ``self.contributors``, default the world size), the compact table row grads
        routed to their owners; returns the routed grads (the caller scales them by the same 1 / contributors)."""
        from . import dist as D
        sh, ar = self.shards, self.arena
        n = ar.n_dense_grad
        D.allreduce_sum_(ar.grad[:n], sh.group)
        ar.grad[:n].mul_(1.0 / self._contributors())
        return sh.route(self.engine.tg, self.engine.tg["fx"])

    def _contributors(self):
        return self.shards.world if self.contributors is None else int(self.contributors)

    @torch.no_grad()
    def _check_replicated_grads(self):
        """Collective, before the optimizer step that follows a row-sharded autograd backward: the dense grads are
        replicas (all-reduced in the backward), so any per-rank rescaling since -- above all
        ``nn.utils.clip_grad_norm_(model.parameters())``, whose norm on row-sharded tables is the local one -- shows
        as ranks disagreeing on them.  Raises instead of letting the replicas drift apart."""
        from . import dist as D
        self.__dict__["replica_checks"] = self.__dict__.get("replica_checks", 0) + 1
        gs = [p.grad for k, p in self.named_parameters() if self.arena.kind[k] != "table" and p.grad is not None]
        s = torch.stack([g.double().sum() for g in gs]).sum() if gs else torch.zeros((), dtype=torch.float64,
                                                                                   device=self.arena.device)
        t = torch.stack([s, -s])
        D.allreduce_max_(t, self.shards.group)
        if bool(t[0] != -t[1]):
            raise RuntimeError(
                "row-sharded tables: the replicated dense gradients differ between ranks at the optimizer step. "
                "nn.utils.clip_grad_norm_(model.parameters(), ...) takes each rank's LOCAL table shards' norm here; "
                "clip with model.clip_grad_norm_(max_norm) (the global norm over all shards, collective) instead")

    @torch.no_grad()
    def clip_grad_norm_(self, max_norm: float, norm_type: float = 2.0):
        """``torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm)`` over the WHOLE model when its tables
        are row-sharded (collective; as FSDP's ``clip_grad_norm_``): the dense grads are replicated, each rank
        holds its shards' grads, so the squared norm is the dense part plus the all-reduced table parts.  Same
        coefficient as torch (``max_norm / (norm + 1e-6)``, clamped to 1, always multiplied).  Without sharded
        tables it is torch's own function.  Returns the total norm."""
        params = [p for p in self.parameters() if p.grad is not None]
        if self.shards is None:
            return torch.nn.utils.clip_grad_norm_(params, max_norm, norm_type)
        if float(norm_type) != 2.0:
            raise NotImplementedError("row-sharded clip_grad_norm_: norm_type 2 only")
        from . import dist as D
        tab = {id(v) for k, v in self.named_parameters() if self.arena.kind[k] == "table"}
        sq = torch.zeros(2, dtype=torch.float32, device=self.arena.device)
        for p in params:
            sq[1 if id(p) in tab else 0] += p.grad.float().pow(2).sum()
        D.allreduce_sum_(sq[1:], self.shards.group)
        total = sq.sum().sqrt()
        coef = (max_norm / (total + 1e-6)).clamp(max=1.0)
        for p in params:
            p.grad.mul_(coef)
        return total

    # ------------------------------------------------------------------ fused training step
    def train_step(self, inputs, y, opt, global_step, seed=None, contribute=True, contributors=None,
                   next_inputs=None):
        """One reference step (src/train.py:152-199): forward -> bce_wll_style(+aux) -> backward ->
        clip -> AdamW -> EMA, all on device, no host sync.  ``inputs`` = staged (X_num, X_mask, X_cat,
        seq) device tensors (see ``stage``), ``y`` float labels on device.  Returns the loss (device).
        ``contribute=False`` (data parallel: a rank without rows on an epoch's last step) runs the step
        with a zero loss gradient, so the rank joins the collectives but adds nothing to the gradient;
        ``contributors`` = how many ranks hold rows this step (the all-reduced gradient is averaged over those,
        not over the whole world; None: every rank).  ``next_inputs`` = the next step's staged inputs, if
        known: row-sharded tables plan that batch's exchange beside this step (tossctr/shard.py), so the
        next step's host read of the exchange sizes waits on nothing; they must stay unchanged until then."""
        seed = self.next_seed() if seed is None else seed
        eng = self.engine
        pf = (next_inputs[2], next_inputs[3]) if next_inputs is not None else None
        _, _, _, sv = eng.forward(*inputs, training=True, seed=seed, save=True, prefetch=pf)
        loss, dz, daux = eng.loss(sv, y)
        if not contribute:
            loss.zero_()
            dz.zero_()
            if daux is not None:
                daux.zero_()
        tg = eng.backward(sv, dz, daux)
        opt.contributors = contributors
        try:
            opt.step(tg, global_step)
        finally:
            opt.contributors = None
        return loss

    def stage(self, batch):
        return self._stage(batch)
