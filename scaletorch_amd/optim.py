"""Optimizers over flat parameter arenas + global gradient clipping.

Reference: ``create_optimizer`` (scaletorch/trainer/model_builder.py:103-162:
adamw[fused] / adam / sgd(m=0.9) / lamb->adamw) and ``clip_gradients``
(scaletorch/trainer/train_step.py:122-136, a LOCAL clip_grad_norm_).

* ``ArenaAdamW``: fp32 master weights + fp32 (or, ``state_dtype="bf16"``, bf16 --
  the reference's own state precision: 22 instead of 30 B/param per step and
  4 B/param less memory) exp_avg / exp_avg_sq per arena;
  on GPU one fused HIP kernel (csrc/adamw.hip) per arena updates master, m, v
  and writes the bf16 model copy -- the whole step is 1-2 launches.  The
  reference kept bf16 params AND bf16 optimizer states (no master weights).
* the clip coefficient is computed on device from the GLOBAL norm (squared
  norms all-reduced over the model-parallel group with TP/EP replicas counted
  once, data_parallel.py ``grad_sumsq_segments``) and read by the kernel from
  device memory: no host sync unless the norm is logged.
* overlap (GPU, ``ST_OVERLAP_OPT=1`` default): the update is enqueued bucket by
  bucket, in FORWARD order, on the model's side stream (data_parallel.py); each
  module of the next forward waits only for the buckets holding its own weights,
  so the HBM-bound AdamW pass (~30 B/param) runs under the next step's MFMA-bound
  GEMMs instead of between steps.  Under ZeRO-1 the bucket's parameter all-gather
  is issued right behind its update on the same stream.  The squared gradient
  norm is likewise accumulated per bucket on that stream during backward
  (world size 1), so clipping costs one scalar reduction after backward.
* ``ArenaSGD`` / ``ArenaAdam`` / ``ArenaLAMB`` cover the other reference choices.
Each subclasses ``torch.optim.Optimizer`` so torch LR schedulers drive ``lr``.
"""
from __future__ import annotations

import math

import os

import torch

from .dist import collectives as C
from .dist import trace
from .ops import _lib



# ---------------------------------------------------------------- bf16 moments: stochastic rounding
# Mirror of csrc/adamw.hip ``sr_bf16`` (bit-for-bit): a 16-bit offset hashed from (element
# index, step, launch length, moment) is added to the fp32 bits, which are then truncated,
# so a stored bf16 moment is an UNBIASED estimate of its fp32 value.  Round-to-nearest
# froze exp_avg_sq at beta2 = 0.999 (its 0.1 % per-step change is below bf16's half-ulp).
_M32 = 0xFFFFFFFF


def _mix32_int(x: int) -> int:
    x &= _M32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & _M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & _M32
    x ^= x >> 16
    return x


def _mix32(x: torch.Tensor) -> torch.Tensor:
    """lowbias32 on an int64 tensor of uint32 values (wrapping products masked to 32 bits)."""
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def sr_key(step: int) -> int:
    """Key of one optimizer step."""
    return _mix32_int((int(step) * 0x9E3779B9) & _M32)


def sr_offsets(n: int, key: int, base: int = 0, device=None) -> tuple[torch.Tensor, torch.Tensor]:
    """The kernel's 16-bit rounding offsets of arena elements base .. base + n - 1: (exp_avg,
    exp_avg_sq) = (low, high) half of mix32(lo32(i) ^ mix32(hi32(i) ^ key))."""
    idx = torch.arange(base, base + n, dtype=torch.int64, device=device)
    h = _mix32((idx & _M32) ^ _mix32((idx >> 32) ^ key))
    return h & 0xFFFF, h >> 16


def sr_round_bf16(x: torch.Tensor, r16: torch.Tensor) -> torch.Tensor:
    """fp32 ``x`` -> bf16 by stochastic rounding with per-element offsets ``r16`` (flat order),
    bit-for-bit as csrc/adamw.hip ``sr_bf16``."""
    xf = x.reshape(-1).float()
    u = xf.view(torch.int32).to(torch.int64) & _M32
    bits = ((u + r16.reshape(-1)) >> 16) & 0xFFFF
    out = (bits - (bits >= 0x8000).to(torch.int64) * 0x10000).to(torch.int16).view(torch.bfloat16)
    special = (u & 0x7F800000) == 0x7F800000
    if bool(special.any()):
        out = torch.where(special, xf.to(torch.bfloat16), out)
    return out


class _ArenaOptimizer(torch.optim.Optimizer):
    """Base: per-arena optimizer state over the arena's SEGMENTS -- the whole
    arena, or under ZeRO-1 (data_parallel.GradArena ``zero1``) this rank's
    shard of every bucket, with state tensors sized to the shard."""

    def __init__(self, dp_model, lr: float, defaults: dict):
        self.dp = dp_model
        arenas = dp_model.arenas
        params = [a.param_flat for a in arenas]
        super().__init__([{"params": [p]} for p in params], dict(lr=lr, **defaults))
        self.arenas = arenas
        self._step = 0
        for a in arenas:
            if a.param_flat.dtype == torch.float32:
                a.master = None
            elif a.zero1:
                a.master = torch.cat([a.param_flat[lo:hi].float() for lo, hi, _ in a.segments()])
            else:
                a.master = a.param_flat.detach().float().clone()
        self.clip_coef = None
        self.last_grad_norm = None
        self.side_stream = getattr(dp_model, "side_stream", None)

    @property
    def sharded(self) -> bool:
        return any(a.zero1 for a in self.arenas)

    def _views(self, a, states: tuple):
        """Yield (param_seg, grad_seg, master_seg, *state_segs) for every segment."""
        for lo, hi, so in a.segments():
            n = hi - lo
            master = a.master[so: so + n] if a.master is not None else a.param_flat[lo:hi]
            yield (a.param_flat[lo:hi], a.grad_flat[lo:hi], master) + tuple(s[so: so + n] for s in states)

    @torch.no_grad()
    def reload_masters(self) -> None:
        """Re-read the fp32 master copy from the (externally overwritten) bf16 params,
        e.g. after an HF weight import into a model whose optimizer already exists."""
        from .ops.grad import invalidate_wt

        self.sync()
        for a in self.arenas:
            invalidate_wt(a.params)
            if a.master is None:
                continue
            a.wait_params()
            for lo, hi, so in a.segments():
                a.master[so: so + hi - lo].copy_(a.param_flat[lo:hi])

    def _finish_step(self) -> None:
        for a in self.arenas:
            a.gather_params()

    def zero_grad(self, set_to_none: bool = False) -> None:  # noqa: ARG002
        self.dp.zero_grad()

    # ---------------------------------------------------------------- clipping
    def _zero_unwritten(self) -> None:
        for a in self.arenas:  # normally a no-op: the DP sync already zeroed untouched grads
            a.zero_fresh()

    def grad_norm(self, mp_group=None) -> torch.Tensor:
        """Global L2 norm of the gradients (device scalar, fp32)."""
        self._zero_unwritten()
        if _lib.probe_env("ST_NORM_PROBE_SKIP"):
            # timing probe of the diagnostic library only (no clipping, norm reported as 0)
            for a in self.arenas:
                a.sq_count = 0
            return torch.zeros(1, dtype=torch.float32, device=self.arenas[0].grad_flat.device)
        pre = [a.take_sumsq() for a in self.arenas]
        if pre and all(x is not None for x in pre) and C.get_world_size() <= 1:
            total = pre[0].clone()  # accumulated on the side stream during backward
            for x in pre[1:]:
                total += x
            return total.sqrt()
        segs = self.dp.grad_sumsq_segments()
        dev = segs[0][0].device
        total = torch.zeros(1, dtype=torch.float32, device=dev)
        for t, w in segs:
            if t.numel() == 0:
                continue
            if _lib.use_native(t) and t.numel() % 4 == 0:
                part = torch.zeros(1, dtype=torch.float32, device=dev)
                _lib.ops().sumsq_(t, part)
                total += part * w
            else:
                total += t.float().pow(2).sum() * w
        if self.sharded:  # shard shares sum over every rank (grad_sumsq_segments)
            if C.get_world_size() > 1:
                C.all_reduce(total)
        elif mp_group is not None and C.get_world_size(mp_group) > 1:
            C.all_reduce(total, group=mp_group)
        return total.sqrt()

    def clip_grad_norm_(self, max_norm: float | None, mp_group=None) -> torch.Tensor:
        norm = self.grad_norm(mp_group)
        self.last_grad_norm = norm
        if max_norm is not None and max_norm > 0:
            self.clip_coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
        else:
            self.clip_coef = None
        return norm

    # ---------------------------------------------------------------- state
    def sync(self) -> None:
        """Join the side-stream update (before reading master / states on the host)."""
        if self.side_stream is not None:
            torch.cuda.current_stream().wait_stream(self.side_stream)

    def state_dict(self):
        self.sync()
        return {
            "step": self._step,
            "param_groups": [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups],
            "arenas": [self._arena_state(a) for a in self.arenas],
        }

    def _arena_state(self, a) -> dict:
        return {"master": None if a.master is None else a.master.detach().cpu()}

    def load_state_dict(self, sd):
        self.sync()
        self._step = sd["step"]
        for g, s in zip(self.param_groups, sd["param_groups"]):
            g.update(s)
        for a, s in zip(self.arenas, sd["arenas"]):
            self._load_arena_state(a, s)

    def _load_arena_state(self, a, s) -> None:
        from .ops.grad import invalidate_wt

        invalidate_wt(a.params)
        if s.get("master") is not None and a.master is not None:
            a.master.copy_(s["master"].to(a.master.device))
            for lo, hi, so in a.segments():
                a.param_flat[lo:hi].copy_(a.master[so: so + hi - lo])
            a.gather_params()
            a.wait_params()


class ArenaAdamW(_ArenaOptimizer):
    def __init__(self, dp_model, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, fused: bool = True, decoupled: bool = True, state_dtype: str = "fp32"):
        super().__init__(dp_model, lr, dict(betas=tuple(betas), eps=eps, weight_decay=weight_decay))
        self.fused = fused
        self.decoupled = decoupled
        sd = {"fp32": torch.float32, "bf16": torch.bfloat16}[state_dtype]
        for a in self.arenas:
            a.exp_avg = torch.zeros(a.state_numel, dtype=sd, device=a.param_flat.device)
            a.exp_avg_sq = torch.zeros_like(a.exp_avg)

    def _native(self, a) -> bool:
        return (self.fused and self.decoupled and _lib.use_native(a.param_flat) and a.master is not None
                and a.param_flat.dtype == torch.bfloat16)

    def _step_overlapped(self, t: int) -> None:
        """Enqueue every bucket's fused update on the side stream in forward order
        (first-used bucket first); record per-bucket completion for the forward
        pre-hooks, or chain the ZeRO-1 all-gather of the bucket behind it."""
        import torch.distributed as dist

        ev = torch.cuda.Event()
        ev.record()  # gradients final + clip coefficient computed
        st = self.side_stream
        if self.clip_coef is not None:
            self.clip_coef.record_stream(st)
        # timing probe of the diagnostic library only (WRONG training: the weights never change):
        # ST_OPT_PROBE_SKIP=1 skips every update kernel, so an A/B prices the side-stream AdamW
        skip = _lib.probe_env("ST_OPT_PROBE_SKIP") is not None
        fuse_wt = os.environ.get("ST_ADAMW_WT", "1") == "1"
        with torch.cuda.stream(st):
            st.wait_event(ev)
            for g, a in zip(self.param_groups, self.arenas):
                lr, (b1, b2), eps, wd = g["lr"], g["betas"], g["eps"], g["weight_decay"]
                for b in reversed(a.buckets):
                    lo, hi, so = b.shard_lo, b.shard_hi, b.state_lo
                    n = hi - lo
                    fused = []
                    if n and not skip:
                        plan = self._wt_plan(a, b) if fuse_wt and not a.zero1 else [("flat", lo, hi, None)]
                        for kind, plo, phi, w in plan:
                            if kind == "flat":
                                s0 = so + plo - lo
                                _lib.ops().adamw_step_(a.master[s0: s0 + phi - plo], a.exp_avg[s0: s0 + phi - plo],
                                                       a.exp_avg_sq[s0: s0 + phi - plo], a.grad_flat[plo:phi],
                                                       a.param_flat[plo:phi], self.clip_coef, lr, b1, b2, eps, wd, t,
                                                       plo)
                            else:
                                s0 = so + plo - lo
                                _lib.ops().adamw_wt_step_(a.master[s0: s0 + phi - plo], a.exp_avg[s0: s0 + phi - plo],
                                                          a.exp_avg_sq[s0: s0 + phi - plo], a.grad_flat[plo:phi],
                                                          a.param_flat[plo:phi].view(w.shape), w._st_wt,
                                                          self.clip_coef, lr, b1, b2, eps, wd, t, plo)
                                fused.append(w)
                    if a.zero1:
                        trace.record("dp.all_gather", a.param_flat[b.start: b.end], group_size=a.world, arena=a.name)
                        b.ag_handle = dist.all_gather_into_tensor(a.param_flat[b.start: b.end],
                                                                  a.param_flat[b.shard_lo: b.shard_hi],
                                                                  group=a.group, async_op=True)
                    else:
                        b.opt_event = torch.cuda.Event()
                        b.opt_event.record(st)
                        for w in fused:
                            w._st_wt_pending = b.opt_event

    def _wt_plan(self, a, b) -> list:
        """The bucket's update as launches: ("wt", lo, hi, w) for every weight that keeps a
        W^T copy for its data-gradient GEMM (ops/grad.py) -- updated by the kernel that
        also writes W^T -- and ("flat", lo, hi, None) for the runs between them."""
        from .ops.grad import _wt_enabled

        offs = getattr(a, "_st_off_of", None)
        if offs is None:
            offs = a._st_off_of = {id(p): o for p, o in zip(a.params, a.offsets)}
        runs = []
        for w in b.params:
            wt = getattr(w, "_st_wt", None)
            if wt is not None and _wt_enabled(w) and wt.shape == (w.shape[1], w.shape[0]):
                o = offs[id(w)]
                runs.append((o, o + w.numel(), w))
        runs.sort(key=lambda r: r[0])
        plan, cur = [], b.shard_lo
        for o, e, w in runs:
            if o > cur:
                plan.append(("flat", cur, o, None))
            plan.append(("wt", o, e, w))
            cur = e
        if cur < b.shard_hi:
            plan.append(("flat", cur, b.shard_hi, None))
        return plan

    @torch.no_grad()
    def step(self, closure=None):  # noqa: ARG002
        self._zero_unwritten()
        self._step += 1
        t = self._step
        if self.side_stream is not None and all(self._native(a) for a in self.arenas):
            self._step_overlapped(t)
            return
        for g, a in zip(self.param_groups, self.arenas):
            lr, (b1, b2), eps, wd = g["lr"], g["betas"], g["eps"], g["weight_decay"]
            native = (self.fused and self.decoupled and _lib.use_native(a.param_flat) and a.master is not None
                      and a.param_flat.dtype == torch.bfloat16)
            for (param, gseg, master, m, v), base in zip(self._views(a, (a.exp_avg, a.exp_avg_sq)),
                                                         (lo for lo, _, _ in a.segments())):
                if native:
                    _lib.ops().adamw_step_(master, m, v, gseg, param, self.clip_coef, lr, b1, b2, eps, wd, t, base)
                    continue
                grad = gseg.float()
                if self.clip_coef is not None:
                    grad = grad * self.clip_coef
                if not self.decoupled and wd:
                    grad = grad + wd * master
                m_st, v_st = m, v
                if m.dtype != torch.float32:  # bf16 moments: fp32 math, one stochastic rounding per step
                    m, v = m.float(), v.float()
                m.mul_(b1).add_(grad, alpha=1 - b1)
                v.mul_(b2).addcmul_(grad, grad, value=1 - b2)
                if m_st is not m:
                    rm, rv = sr_offsets(m.numel(), sr_key(t), base, m.device)
                    m_st.copy_(sr_round_bf16(m, rm).view_as(m_st))
                    v_st.copy_(sr_round_bf16(v, rv).view_as(v_st))
                bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
                denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
                if self.decoupled and wd:
                    master.mul_(1 - lr * wd)
                master.addcdiv_(m, denom, value=-lr / bc1)
                if a.master is not None:
                    param.copy_(master)
        self._finish_step()

    def _arena_state(self, a) -> dict:
        d = super()._arena_state(a)
        d.update(exp_avg=a.exp_avg.detach().cpu(), exp_avg_sq=a.exp_avg_sq.detach().cpu())
        return d

    def _load_arena_state(self, a, s) -> None:
        super()._load_arena_state(a, s)
        # copy_ converts: an fp32-state checkpoint resumes into bf16 states and vice versa
        a.exp_avg.copy_(s["exp_avg"].to(a.exp_avg.device))
        a.exp_avg_sq.copy_(s["exp_avg_sq"].to(a.exp_avg_sq.device))


class ArenaAdam(ArenaAdamW):
    """Adam with L2 (coupled) weight decay."""

    def __init__(self, dp_model, **kw):
        kw.pop("fused", None)
        super().__init__(dp_model, fused=False, decoupled=False, **kw)


class ArenaSGD(_ArenaOptimizer):
    def __init__(self, dp_model, lr: float = 1e-3, momentum: float = 0.9, weight_decay: float = 0.0):
        super().__init__(dp_model, lr, dict(momentum=momentum, weight_decay=weight_decay))
        for a in self.arenas:
            a.momentum_buf = torch.zeros(a.state_numel, dtype=torch.float32, device=a.param_flat.device)

    @torch.no_grad()
    def step(self, closure=None):  # noqa: ARG002
        self._zero_unwritten()
        self._step += 1
        for g, a in zip(self.param_groups, self.arenas):
            for param, gseg, master, mom in self._views(a, (a.momentum_buf,)):
                grad = gseg.float()
                if self.clip_coef is not None:
                    grad = grad * self.clip_coef
                if g["weight_decay"]:
                    grad = grad + g["weight_decay"] * master
                mom.mul_(g["momentum"]).add_(grad)
                master.add_(mom, alpha=-g["lr"])
                if a.master is not None:
                    param.copy_(master)
        self._finish_step()

    def _arena_state(self, a) -> dict:
        d = super()._arena_state(a)
        d["momentum"] = a.momentum_buf.detach().cpu()
        return d

    def _load_arena_state(self, a, s) -> None:
        super()._load_arena_state(a, s)
        a.momentum_buf.copy_(s["momentum"].to(a.momentum_buf.device))


class ArenaLAMB(ArenaAdamW):
    """LAMB: AdamW update rescaled per parameter by ||w|| / ||update|| (trust ratio)."""

    def __init__(self, dp_model, **kw):
        kw.pop("fused", None)
        if any(a.zero1 for a in dp_model.arenas):
            raise ValueError("LAMB needs whole-parameter norms; use it without zero1")
        super().__init__(dp_model, fused=False, **kw)

    @torch.no_grad()
    def step(self, closure=None):  # noqa: ARG002
        self._zero_unwritten()
        self._step += 1
        t = self._step
        for g, a in zip(self.param_groups, self.arenas):
            lr, (b1, b2), eps, wd = g["lr"], g["betas"], g["eps"], g["weight_decay"]
            master = a.master if a.master is not None else a.param_flat
            grad = a.grad_flat.float()
            if self.clip_coef is not None:
                grad = grad * self.clip_coef
            m, v = a.exp_avg.float(), a.exp_avg_sq.float()
            m.mul_(b1).add_(grad, alpha=1 - b1)
            v.mul_(b2).addcmul_(grad, grad, value=1 - b2)
            if m is not a.exp_avg:
                a.exp_avg.copy_(m)
                a.exp_avg_sq.copy_(v)
            upd = (m / (1 - b1 ** t)) / ((v / (1 - b2 ** t)).sqrt() + eps)
            if wd:
                upd.add_(master, alpha=wd)
            for p, o in zip(a.params, a.offsets):
                n = p.numel()
                w, u = master[o: o + n], upd[o: o + n]
                wn, un = w.norm(), u.norm()
                ratio = torch.where((wn > 0) & (un > 0), wn / un, torch.ones_like(wn))
                w.add_(u * ratio, alpha=-lr)
            if a.master is not None:
                a.param_flat.copy_(master)


def create_optimizer(dp_model, optimizer_type: str = "adamw", lr: float = 1e-3, weight_decay: float = 0.0,
                     betas=(0.9, 0.999), eps: float = 1e-8, use_fused_adam: bool = True, state_dtype: str = "fp32"):
    t = optimizer_type.lower()
    if t == "adamw":
        return ArenaAdamW(dp_model, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, fused=use_fused_adam,
                          state_dtype=state_dtype)
    if t == "adam":
        return ArenaAdam(dp_model, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, state_dtype=state_dtype)
    if t == "sgd":
        return ArenaSGD(dp_model, lr=lr, momentum=0.9, weight_decay=weight_decay)
    if t == "lamb":
        return ArenaLAMB(dp_model, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
    raise ValueError(f"unknown optimizer_type {optimizer_type!r}")
