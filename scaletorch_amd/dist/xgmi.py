"""Intra-node custom collectives over xGMI peer memory (csrc/xgmi_allreduce.hip):
all-reduce, all-gather and reduce-scatter on one IPC buffer + flag protocol.

The reference sends every tensor-parallel all-reduce through NCCL/HCCL
(scaletorch/parallel/tensor_parallel/tp_comms.py:117-166, :229-320; SURVEY.md
§2.2 "custom transport").  On one MI355X node every GPU has a direct xGMI link to
each of the others, so a TP group can all-reduce by READING its peers' buffers:

* each rank allocates one IPC-shareable buffer (accessed with system-coherent
  loads/stores only); the 64-byte IPC
  handles are exchanged once over the process group and every rank maps the
  others (``hipIpcOpenMemHandle``);
* ``all_reduce(t)``: one-shot (copy in, per-block cross-rank flag handshake, sum
  the slice from all W buffers) for messages up to ``oneshot_max`` bytes,
  two-shot (reduce-scatter into a result area, handshake, all-gather) above it;
  fp32 accumulation in a fixed rank order, so every rank gets bitwise the same
  result; anything that does not fit (size, dtype, alignment) goes to RCCL;
* ``all_gather(t)`` / ``reduce_scatter(t)``: every rank publishes its input once,
  then block b of every rank pulls slice b of ALL peers' data at once (all 7
  links busy) -- the sequence-parallel activation gather / gradient scatter;
* up to 256 workgroups (one per CU) pull at once, sized by message;
* ``all_to_all(t)``: equal-split exchange by PUSH -- every rank writes chunk d
  straight into rank d's buffer (all 7 links, posted writes), one handshake, a local
  copy out: the EP token dispatch/combine (reference ep_comms.py:14-38, RCCL
  all_to_all_single there);
* ``pair_all_gather`` / ``pair_reduce_scatter``: a 2-rank group (TP = 2) has ONE
  direct link; these split the message over the direct link AND 2-hop paths through
  the memory of every other GPU of the node (the relay GPU runs nothing), so all 7
  links of each partner carry a share.  The communicator spans the node; only the
  pair calls it (``XgmiComm(node_group)``, any disjoint pairs at once);
* every wait is bounded (``ST_XGMI_TIMEOUT_S``, default 60 s): a peer that never
  arrives sets an error word instead of hanging the GPU; ``check()`` (polled by the
  trainer at every logging step, tensor_parallel.check_xgmi) turns it into an
  exception so the job exits non-zero and a torchrun restart can resume.

Use: ``XgmiAllReduce(group)`` collectively on every rank of ``group`` (all ranks
on ONE node, one GPU each), then ``comm.all_reduce(t)`` in the same order on all
ranks.  ``tensor_parallel.set_tp_comm("xgmi")`` routes the TP all-reduces here.
"""
from __future__ import annotations

import socket

import torch
import torch.distributed as dist

from ..ops import _lib


def _ops():
    if not _lib.load():
        raise RuntimeError(f"xgmi all-reduce needs the HIP kernel library: {_lib.load_error()}")
    return _lib.ops()


def _blocks_for(nbytes: int) -> int:
    """Workgroups per rank: ~64 KiB of message per block, 8..256 blocks (one per CU
    at most, so every block of the grid is co-resident)."""
    return int(min(256, max(8, nbytes // (64 << 10))))


def _ep_blocks(area_rows: int, x: torch.Tensor, world: int) -> int:
    """Workgroups of an EP exchange: sized by the HOST bound of the rows moved (identical on
    every rank -- the per-block handshake pairs block b of every rank), one per ~64 KiB of
    a rank's share, 8..256; every block of every rank must be co-resident for the barrier."""
    return _blocks_for(area_rows * x.shape[1] * x.element_size() // max(1, world))


def _default_timeout() -> str:
    """Peer-arrival bound of every spin wait.  It guards against a dead peer, not a slow one:
    ranks legitimately drift apart by seconds (first-call GEMM tuning, a checkpoint write on
    one rank, gloo's host staging), and a kernel that gives up leaves its output unwritten.
    Round 6's 8-rank one-GPU Mixtral rehearsal hit the old 2-s bound in the EP exchange,
    and the unwritten rows turned the weights non-finite by step 2.  60 s, or 300 s when
    ranks time-share one GPU (ST_GPU_OVERSUBSCRIBE=1)."""
    import os

    return "300" if os.environ.get("ST_GPU_OVERSUBSCRIBE", "0") == "1" else "60"


_MODES = {"oneshot": 0, "twoshot": 1, "all_gather": 2, "reduce_scatter": 3, "all_to_all": 4,
          "pair_all_gather": 5, "pair_reduce_scatter": 6}


class XgmiAllReduce:
    """Custom all-reduce for one process group whose ranks share a node."""

    # communicators created so far in this process; creation is collective, so the
    # count (-> epoch base) is identical on every rank of a group
    _serial = 0

    @classmethod
    def _next_base(cls) -> int:
        cls._serial += 1
        return (cls._serial % 255) << 24

    def __init__(self, group=None, max_bytes: int = 64 << 20, oneshot_max: int = 512 << 10, _sim=None,
                 timeout_s: float | None = None):
        import os

        self.group = group
        self.oneshot_max = oneshot_max
        self.cap = (max_bytes + 255) // 256 * 256
        self.timeout_s = float(timeout_s if timeout_s is not None else os.environ.get("ST_XGMI_TIMEOUT_S", _default_timeout()))
        if _sim is not None:  # in-process simulation (tests): (rank, world, epoch base)
            self.rank, self.world, base = _sim
            self.id = int(_ops().xgmi_create(self.rank, self.world, self.cap, base))
            _ops().xgmi_set_timeout(self.id, self.timeout_s)
            return
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > 8:
            raise ValueError("xgmi all-reduce spans at most the 8 GPUs of one node")
        where = [None] * self.world
        dist.all_gather_object(where, (socket.gethostname(), torch.cuda.current_device()), group=group)
        shared_ok = os.environ.get("ST_GPU_OVERSUBSCRIBE", "0") == "1"  # 1-GPU multi-rank rehearsals / tests
        if len({h for h, _ in where}) != 1 or (len({d for _, d in where}) != self.world and not shared_ok):
            raise ValueError(f"xgmi all-reduce needs one GPU per rank on one node, got {where}")
        self.id = int(_ops().xgmi_create(self.rank, self.world, self.cap, self._next_base()))
        _ops().xgmi_set_timeout(self.id, self.timeout_s)
        mine = _ops().xgmi_handle(self.id).tolist()
        handles = [None] * self.world
        dist.all_gather_object(handles, mine, group=group)
        for r, h in enumerate(handles):
            if r != self.rank:
                _ops().xgmi_open(self.id, r, torch.tensor(h, dtype=torch.uint8))
        dist.barrier(group=group)

    @classmethod
    def simulate(cls, world: int, max_bytes: int = 8 << 20, oneshot_max: int = 512 << 10,
                 timeout_s: float | None = None):
        """``world`` communicators in THIS process wired to each other's buffers
        (one GPU), for tests: ``all_reduce_sim`` runs every rank's job in ONE launch
        (rank = blockIdx.y), exercising the kernels and the cross-rank flag protocol
        without IPC.  (Separate streams per simulated rank are not enough: HIP maps
        a process's streams onto a few shared hardware queues, and two spinning
        kernels on one queue serialise.)"""
        base = cls._next_base()
        comms = [cls(max_bytes=max_bytes, oneshot_max=oneshot_max, _sim=(r, world, base), timeout_s=timeout_s)
                 for r in range(world)]
        for c in comms:
            for r, p in enumerate(comms):
                _ops().xgmi_set_peer(c.id, r, p.id)
        return comms

    def supports(self, t: torch.Tensor, scale: int = 1) -> bool:
        """``t`` can go through the kernels; ``scale`` = data-area multiple the op needs
        (reduce-scatter publishes world x its output)."""
        return (t.is_cuda and t.dtype in (torch.bfloat16, torch.float32) and t.is_contiguous()
                and t.numel() % 8 == 0 and t.numel() * t.element_size() * scale <= self.cap
                and t.data_ptr() % 16 == 0)

    def all_gather(self, t: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """[n] per rank -> [world * n] in rank order (RCCL when the kernels do not apply)."""
        if out is None:
            out = torch.empty((self.world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        if not self.supports(t) or out.data_ptr() % 16:
            dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
            return out
        _ops().xgmi_all_reduce(self.id, t, out, _MODES["all_gather"], _blocks_for(t.numel() * t.element_size()))
        return out

    def reduce_scatter(self, t: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """[world * n] per rank -> this rank's [n] of the sum (fp32 accumulation, fixed order)."""
        if out is None:
            out = torch.empty((t.shape[0] // self.world,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        if not self.supports(out, scale=self.world) or not self.supports(t) or out.data_ptr() % 16:
            dist.reduce_scatter_tensor(out, t.contiguous(), group=self.group)
            return out
        _ops().xgmi_all_reduce(self.id, t, out, _MODES["reduce_scatter"],
                               _blocks_for(out.numel() * out.element_size()))
        return out

    @staticmethod
    def collective_sim(comms, ins, outs, op: str, partners: list[int] | None = None) -> None:
        """Simulation of ``op`` (all_gather | reduce_scatter | all_to_all | pair_all_gather |
        pair_reduce_scatter; pairs: ``partners[r]``) across ``comms`` in ONE launch."""
        world = len(comms)
        if op in ("all_gather", "pair_all_gather"):
            nbytes = ins[0].numel() * ins[0].element_size()
        elif op == "all_to_all":
            nbytes = ins[0].numel() * ins[0].element_size() // world
        else:
            nbytes = outs[0].numel() * outs[0].element_size()
        _ops().xgmi_all_reduce_sim([c.id for c in comms], ins, outs, _MODES[op], _blocks_for(nbytes), partners)

    def all_to_all(self, t: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """Equal-split all-to-all of dim 0 ([world * n] per rank: chunk d goes to rank d;
        out[r-th chunk] came from rank r) -- RCCL when the kernels do not apply."""
        if out is None:
            out = torch.empty_like(t)
        if not self.supports(t) or out.data_ptr() % 16 or t.shape[0] % self.world:
            dist.all_to_all_single(out, t.contiguous(), group=self.group)
            return out
        _ops().xgmi_all_reduce(self.id, t, out, _MODES["all_to_all"],
                               _blocks_for(t.numel() * t.element_size() // self.world))
        return out

    # ---- expert-parallel exchange with device-side counts (dropless, no host sync)
    def ep_counts(self, counts: torch.Tensor) -> torch.Tensor:
        """All-gather this rank's per-expert row counts (int32 [E], device) into the
        [world, E] matrix every rank needs for the exchange -- a bitwise copy through the
        all-gather kernel (int32 viewed as fp32, padded to 8 words)."""
        E = counts.numel()
        E8 = (E + 7) // 8 * 8
        src = torch.zeros(E8, dtype=torch.int32, device=counts.device)
        src[:E] = counts.to(torch.int32)
        out = torch.empty(self.world * E8, dtype=torch.int32, device=counts.device)
        _ops().xgmi_all_reduce(self.id, src.view(torch.float32), out.view(torch.float32), _MODES["all_gather"],
                               _blocks_for(E8 * 4))
        return out.view(self.world, E8)[:, :E].contiguous()

    def ep_fits(self, rows: int, t: torch.Tensor) -> bool:
        """``rows`` rows of ``t``'s width fit one data area (the host bound of an exchange)."""
        return (t.is_cuda and t.dtype in (torch.bfloat16, torch.float32) and t.dim() == 2 and t.shape[1] % 8 == 0
                and rows * t.shape[1] * t.element_size() <= self.cap)

    def ep_exchange(self, x: torch.Tensor, M: torch.Tensor, El: int, direction: int, out_rows: int,
                    area_rows: int) -> torch.Tensor:
        """Dispatch (direction 0: ``x`` = this rank's rows sorted by global expert ->
        [out_rows, h] of its local experts' rows, expert-major, the first sum(M[:, mine])
        rows valid) or combine (direction 1: the reverse, out_rows = this rank's sorted
        rows).  ``M`` [world, E] int32 device counts (``ep_counts``); ``area_rows`` the
        host bound of rows landing in one rank's buffer.  No host sync."""
        out = torch.empty(out_rows, x.shape[1], dtype=x.dtype, device=x.device)
        _ops().xgmi_ep_exchange(self.id, x.contiguous(), out, M, El, direction, area_rows,
                                _ep_blocks(area_rows, x, self.world))
        return out

    @staticmethod
    def ep_exchange_sim(comms, xs, M, El: int, direction: int, out_rows: int, area_rows: int):
        outs = [torch.empty(out_rows, x.shape[1], dtype=x.dtype, device=x.device) for x in xs]
        _ops().xgmi_ep_exchange_sim([c.id for c in comms], xs, outs, M, El, direction, area_rows,
                                    _ep_blocks(area_rows, xs[0], len(comms)))
        return outs

    def _pair_ok(self, n_elems: int, t: torch.Tensor) -> bool:
        # a relay holds a path's share of the message in a slot of cap / 8 bytes
        return (t.is_cuda and t.dtype in (torch.bfloat16, torch.float32) and t.is_contiguous()
                and n_elems % 8 == 0 and n_elems * t.element_size() * 8 <= self.cap and t.data_ptr() % 16 == 0)

    def pair_all_gather(self, t: torch.Tensor, partner: int, out: torch.Tensor | None = None) -> torch.Tensor:
        """2-rank all-gather with ``partner`` (a rank of this communicator's group) over
        the direct link + 2-hop relays: out = [lower rank's t | higher rank's t]."""
        if out is None:
            out = torch.empty((2 * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        if not self._pair_ok(t.numel(), t) or out.data_ptr() % 16:
            raise ValueError("pair_all_gather: message does not fit the kernels (use the pair's RCCL group)")
        _ops().xgmi_pair(self.id, t, out, _MODES["pair_all_gather"], partner, _blocks_for(t.numel() * t.element_size()))
        return out

    def pair_reduce_scatter(self, t: torch.Tensor, partner: int, out: torch.Tensor | None = None) -> torch.Tensor:
        """2-rank reduce-scatter with ``partner``: t = [chunk of the lower rank | chunk of the
        higher rank]; out = this rank's chunk summed over the pair (fp32, fixed order)."""
        if out is None:
            out = torch.empty((t.shape[0] // 2,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        if not self._pair_ok(out.numel(), t) or out.data_ptr() % 16:
            raise ValueError("pair_reduce_scatter: message does not fit the kernels (use the pair's RCCL group)")
        _ops().xgmi_pair(self.id, t, out, _MODES["pair_reduce_scatter"], partner,
                         _blocks_for(out.numel() * out.element_size()))
        return out

    def all_reduce(self, t: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """Sum of ``t`` over the group into ``out`` (default: in place)."""
        out = t if out is None else out
        if not self.supports(t):
            if out is not t:
                out.copy_(t)
            dist.all_reduce(out, group=self.group)
            return out
        nbytes = t.numel() * t.element_size()
        mode = 0 if nbytes <= self.oneshot_max else 1
        _ops().xgmi_all_reduce(self.id, t, out, mode, _blocks_for(nbytes))
        return out

    @staticmethod
    def all_reduce_sim(comms, ins, outs) -> None:
        nbytes = ins[0].numel() * ins[0].element_size()
        mode = 0 if nbytes <= comms[0].oneshot_max else 1
        _ops().xgmi_all_reduce_sim([c.id for c in comms], ins, outs, mode, _blocks_for(nbytes))

    def check(self) -> None:
        """Raise if any collective of this communicator timed out (host sync)."""
        if int(_ops().xgmi_error(self.id)):
            raise RuntimeError(f"xgmi collective: a peer did not arrive within {self.timeout_s:g} s (rank died or "
                               "call order differs); outputs since then are invalid")

    def close(self) -> None:
        if getattr(self, "id", None) is not None:
            _ops().xgmi_destroy(self.id)
            self.id = None


XgmiComm = XgmiAllReduce  # the communicator carries all three collectives


def _max_bytes_default(kind: str = "pair") -> int:
    """IPC data area per rank (ST_XGMI_MAX_MB for the node communicator behind the tp = 2 pair
    path, ST_XGMI_EP_MAX_MB for the dropless EP exchange; 512 MiB each).  The pair path's
    relay slots are an eighth of it (``_pair_ok``), so 512 MiB takes messages up to 64 MiB
    -- the SP sub-chunks at S = 4096 (16-32 MiB) and the start-up self-test (32 MiB); the
    EP area holds one rank's landing rows at the host bound (268 MiB for Mixtral EP 8 at
    4096 tokens).  Two processes sharing ONE GPU (rehearsals / tests) hung opening a peer's
    512 MiB area (hipIpcOpenMemHandle) while 16 MiB opened at once (tests/test_xgmi_gpu.py
    SP pair-path test): such runs set the variables low."""
    import os

    if kind == "ep":
        return int(float(os.environ.get("ST_XGMI_EP_MAX_MB", "512")) * (1 << 20))
    return int(float(os.environ.get("ST_XGMI_MAX_MB", "512")) * (1 << 20))


def area_bytes(max_bytes: int) -> int:
    """Device memory one communicator allocates (csrc/xgmi_allreduce.hip: a 16 KiB flag
    header + 4 data areas: two collectives in flight x two epoch parities)."""
    return 16384 + 4 * ((int(max_bytes) + 255) // 256 * 256)


def planned_ipc_bytes(tp: int = 1, ep: int = 1, tp_msg_bytes: int | None = None,
                      moe_dropless: bool = False, ep_area: int | None = None) -> int:
    """Upper bound of the IPC areas a rank holds when the start-up self-tests keep xGMI
    (losers are closed): tp = 2 -> the node communicator of the pair path + the 2-rank one;
    tp > 2 -> one TP-group communicator sized by the message; EP dropless -> the push area."""
    from ..parallel.tensor_parallel import _tp_area_bytes

    total = 0
    if tp == 2:
        total += area_bytes(_max_bytes_default()) + area_bytes(64 << 20)
    elif tp > 2:
        total += area_bytes(_tp_area_bytes(tp_msg_bytes))
    if ep > 1:
        import os

        use = ep_area if (ep_area and not os.environ.get("ST_XGMI_EP_MAX_MB")) else _max_bytes_default("ep")
        total += area_bytes(use)
    return total


def node_group():
    """The process group of the ranks on this node (collective over the WORLD: every rank
    creates every node's group, in the same order)."""
    world = dist.get_world_size()
    hosts = [None] * world
    dist.all_gather_object(hosts, socket.gethostname())
    mine = None
    for h in sorted(set(hosts)):
        ranks = [r for r in range(world) if hosts[r] == h]
        g = dist.new_group(ranks=ranks)
        if h == socket.gethostname():
            mine = (g, ranks)
    return mine


class PairPath:
    """A 2-rank group's multipath transport: the node-wide communicator plus this rank's
    partner (its node-group rank) -- ``all_gather`` / ``reduce_scatter`` in the 2-rank
    group's rank order over the direct link and 2-hop relays."""

    def __init__(self, comm: XgmiAllReduce, partner: int, lower: bool):
        self.comm, self.partner, self.lower = comm, partner, lower

    def fits(self, n_elems: int, t: torch.Tensor) -> bool:
        return self.comm._pair_ok(n_elems, t)

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        return self.comm.pair_all_gather(t, self.partner)

    def reduce_scatter(self, t: torch.Tensor) -> torch.Tensor:
        return self.comm.pair_reduce_scatter(t, self.partner)


def setup_pair_path(pair_group) -> PairPath | None:
    """Collective over the WORLD (call on every rank, at start-up): the node communicator
    and, for ranks whose ``pair_group`` has 2 ranks on this node with group rank order =
    node rank order, their PairPath (else None)."""
    ng, ranks = node_group()
    comm = XgmiAllReduce(ng, max_bytes=_max_bytes_default())
    if pair_group is None or dist.get_world_size(pair_group) != 2:
        return None
    me = dist.get_rank()
    other = dist.get_global_rank(pair_group, 1 - dist.get_rank(pair_group))
    if other not in ranks:
        return None
    lower = me < other
    if lower != (dist.get_rank(pair_group) == 0):  # the pair ops order by node rank
        return None
    return PairPath(comm, ranks.index(other), lower)
