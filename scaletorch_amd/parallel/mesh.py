"""5-D process mesh ``[DP, PP, CP, EP, TP]`` (TP fastest-varying).

Same rank arithmetic as the reference ProcessGroupManager
(scaletorch/parallel/process_group.py:88-102) so a checkpoint's
``tp_rank``/``pp_rank`` mean the same thing, with these MI355X-first changes:

* groups are created with ``torch.distributed.new_group`` per family, in the
  same deterministic order on every rank (RCCL communicators are created
  lazily on first use, so unused families cost nothing);
* TP is the fastest axis, so a TP group is always a set of consecutive local
  GPUs: on one 8-GPU xGMI node every pair is one direct link, and across nodes
  TP never leaves a node for tp <= 8;
* EP is carved out of data parallelism (Megatron style): samples differ across
  EP ranks (the loader shards data over DP x EP), dense parameters are reduced
  over ``dense_dp_group`` = DP x CP x EP and expert parameters over
  ``expert_dp_group`` = DP x CP.  The reference reduced dense weights over DP
  only and fed EP peers identical samples;
* a global proxy (``pgm``) mirrors the reference's ``process_group_manager``.
"""
from __future__ import annotations

import logging
import os

import torch

from ..dist import collectives as C

logger = logging.getLogger(__name__)

AXES = ("dp", "pp", "cp", "ep", "tp")


class ProcessGroupManager:
    def __init__(self, tp_size: int = 1, cp_size: int = 1, pp_size: int = 1, dp_size: int = 1,
                 ep_size: int = 1, rank: int | None = None, world_size: int | None = None,
                 create_groups: bool = True):
        for n, v in (("tp_size", tp_size), ("cp_size", cp_size), ("pp_size", pp_size),
                     ("dp_size", dp_size), ("ep_size", ep_size)):
            if v <= 0:
                raise ValueError(f"{n} must be positive, got {v}")
        self.global_rank = C.get_rank() if rank is None else rank
        self.world_size = C.get_world_size() if world_size is None else world_size
        self.local_rank = int(os.environ.get("LOCAL_RANK", self.global_rank % max(1, self.world_size)))
        expected = tp_size * cp_size * pp_size * dp_size * ep_size
        if self.world_size != expected:
            raise ValueError(
                f"World size ({self.world_size}) != TP ({tp_size}) * CP ({cp_size}) * PP ({pp_size}) * "
                f"DP ({dp_size}) * EP ({ep_size}) = {expected}")
        self.sizes = dict(dp=dp_size, pp=pp_size, cp=cp_size, ep=ep_size, tp=tp_size)
        self.grid = torch.arange(self.world_size).view(dp_size, pp_size, cp_size, ep_size, tp_size)
        r = self.global_rank
        self.tp_rank = r % tp_size
        r //= tp_size
        self.ep_rank = r % ep_size
        r //= ep_size
        self.cp_rank = r % cp_size
        r //= cp_size
        self.pp_rank = r % pp_size
        self.dp_rank = r // pp_size
        self.coords = dict(dp=self.dp_rank, pp=self.pp_rank, cp=self.cp_rank, ep=self.ep_rank, tp=self.tp_rank)
        self._all_groups = []
        self._create_groups = create_groups and C.is_distributed()
        self._build()

    # ------------------------------------------------------------------ groups
    def group_ranks(self, varying: tuple[str, ...]) -> list[list[int]]:
        """All rank lists of the family whose members differ only along ``varying`` axes."""
        fixed = [a for a in AXES if a not in varying]
        out = []
        import itertools

        for combo in itertools.product(*[range(self.sizes[a]) for a in fixed]):
            idx = []
            fc = dict(zip(fixed, combo))
            for a in AXES:
                idx.append(slice(None) if a in varying else fc[a])
            out.append(self.grid[tuple(idx)].flatten().tolist())
        return out

    def my_ranks(self, varying: tuple[str, ...]) -> list[int]:
        idx = tuple(slice(None) if a in varying else self.coords[a] for a in AXES)
        return self.grid[idx].flatten().tolist()

    def _family(self, varying: tuple[str, ...], channel: str = "model"):
        """Create (collectively, same order on every rank) the groups of one family.

        Trivial families (size 1) get the ``SINGLE`` sentinel instead of a
        communicator -- every collective wrapper treats it as a no-op -- and a
        family with the same rank lists as an earlier one OF THE SAME CHANNEL
        reuses its groups.  Channels keep communicators apart whose collectives
        are issued from different places: the gradient buckets ("grad") fire
        from post-accumulate hooks whose timing relative to the autograd-driven
        model collectives (EP all-to-all, TP/CP) may differ across ranks, so
        they must never share an RCCL communicator (one ordered queue) with them.
        """
        mine = self.my_ranks(varying)
        if len(mine) == 1:
            return C.SINGLE, mine
        if not self._create_groups:
            return None, mine
        lists = self.group_ranks(varying)
        key = (channel,) + tuple(tuple(x) for x in lists)
        cache = self.__dict__.setdefault("_family_cache", {})
        if key not in cache:
            groups = []
            for ranks in lists:
                g = C.new_group(ranks=ranks)
                self._all_groups.append(g)
                groups.append(g)
            cache[key] = groups
        return cache[key][lists.index(mine)], mine

    def _pp_channels(self) -> dict:
        """{(kind, i): communicator or None} for every directed pipeline channel this
        rank is an end of (created collectively, same order on every rank)."""
        P = self.sizes["pp"]
        if P == 1:
            return {}
        import itertools

        fixed = [a for a in AXES if a != "pp"]
        out = {}
        for kind in ("fwd", "bwd"):
            for i in range(P):
                a, b = (i, (i + 1) % P) if kind == "fwd" else ((i + 1) % P, i)  # (sender, receiver)
                for combo in itertools.product(*[range(self.sizes[x]) for x in fixed]):
                    fc = dict(zip(fixed, combo))
                    ranks = [int(self.grid[tuple(s if x == "pp" else fc[x] for x in AXES)]) for s in (a, b)]
                    g = None
                    if self._create_groups:
                        g = C.new_group(ranks=sorted(ranks))
                        self._all_groups.append(g)
                    if self.global_rank in ranks:
                        out[(kind, i)] = g
        return out

    def pp_channel(self, kind: str, i: int):
        """Communicator of directed pipeline channel (kind, i mod P); the whole-pipeline
        group when groups are not created (single-process simulation)."""
        return self.pp_channels.get((kind, i % self.pp_world_size)) or self.pp_group

    def _build(self) -> None:
        self.tp_group, self.tp_group_ids = self._family(("tp",))
        self.cp_group, self.cp_group_ids = self._family(("cp",))
        self.pp_group, self.pp_group_ids = self._family(("pp",))
        # pipeline p2p: ONE 2-rank communicator per directed channel -- activations
        # stage i -> i+1 on ("fwd", i), gradients stage i+1 -> i on ("bwd", i), the
        # interleaved ring seam being i = P-1.  A batched p2p op (batch_isend_irecv) runs
        # on its communicator's single RCCL stream; on a whole-pipeline communicator a
        # middle stage's receive posted ahead from r-1 would queue in front of its send
        # to r+1 and close a wait cycle at pp >= 3 (parallel/interleaved.py
        # ``simulate_streams`` replays both layouts).  Each stream here carries one
        # direction between one pair of ranks, so a posted receive only ever waits for
        # its own sender.
        self.pp_channels = self._pp_channels()
        self.ep_group, self.ep_group_ids = self._family(("ep",))
        self.dp_group, self.dp_group_ids = self._family(("dp",))
        self.cp_dp_group, self.cp_dp_group_ids = self._family(("dp", "cp"))
        self.pp_dp_group, self.pp_dp_group_ids = self._family(("dp", "pp"))
        # gradient-reduction groups (EP carved out of DP)
        self.dense_dp_group, self.dense_dp_group_ids = self._family(("dp", "cp", "ep"), channel="grad")
        self.expert_dp_group, self.expert_dp_group_ids = self._family(("dp", "cp"), channel="grad")
        # model-parallel group for global grad-norm (everything but data replicas)
        self.mp_group, self.mp_group_ids = self._family(("pp", "tp", "ep"))

        self.tp_world_size = len(self.tp_group_ids)
        self.cp_world_size = len(self.cp_group_ids)
        self.pp_world_size = len(self.pp_group_ids)
        self.ep_world_size = len(self.ep_group_ids)
        self.dp_world_size = len(self.dp_group_ids)
        self.cp_dp_world_size = len(self.cp_dp_group_ids)
        self.pp_dp_world_size = len(self.pp_dp_group_ids)
        self.dense_dp_world_size = len(self.dense_dp_group_ids)
        self.tp_first_rank, self.tp_last_rank = self.tp_group_ids[0], self.tp_group_ids[-1]
        self.cp_first_rank, self.cp_last_rank = self.cp_group_ids[0], self.cp_group_ids[-1]
        self.pp_first_rank, self.pp_last_rank = self.pp_group_ids[0], self.pp_group_ids[-1]
        self.ep_first_rank, self.ep_last_rank = self.ep_group_ids[0], self.ep_group_ids[-1]
        self.dp_first_rank, self.dp_last_rank = self.dp_group_ids[0], self.dp_group_ids[-1]
        self.cp_send_rank = self.cp_group_ids[(self.cp_rank + 1) % self.cp_world_size]
        self.cp_recv_rank = self.cp_group_ids[(self.cp_rank - 1) % self.cp_world_size]
        self.pp_is_first_stage = self.pp_rank == 0
        self.pp_is_last_stage = self.pp_rank == self.pp_world_size - 1
        self.pp_next_rank = None if self.pp_is_last_stage else self.pp_group_ids[self.pp_rank + 1]
        self.pp_prev_rank = None if self.pp_is_first_stage else self.pp_group_ids[self.pp_rank - 1]
        # data shard index: DP x EP replicas see different samples
        self.data_rank = self.dp_rank * self.ep_world_size + self.ep_rank
        self.data_world_size = self.dp_world_size * self.ep_world_size

    # ------------------------------------------------------------------ misc
    def get_info(self) -> str:
        return (f"rank {self.global_rank}: DP={self.dp_rank}/{self.dp_world_size} PP={self.pp_rank}/"
                f"{self.pp_world_size} CP={self.cp_rank}/{self.cp_world_size} EP={self.ep_rank}/"
                f"{self.ep_world_size} TP={self.tp_rank}/{self.tp_world_size}")

    def __str__(self) -> str:
        return (f"TP({self.tp_world_size})-CP({self.cp_world_size})-PP({self.pp_world_size})-"
                f"EP({self.ep_world_size})-DP({self.dp_world_size})-Rank({self.global_rank})")

    def cleanup(self) -> None:
        for g in self._all_groups:
            try:
                C.destroy_group(g)
            except Exception:
                logger.warning("failed to destroy group", exc_info=True)
        self._all_groups = []


class _Proxy:
    """Truthy only once a manager is installed (reference: process_group.py:359-384)."""

    _instance: ProcessGroupManager | None = None

    def __getattr__(self, name):
        inst = type(self)._instance
        if inst is None:
            raise AttributeError(f"process group manager not initialised (accessing .{name})")
        return getattr(inst, name)

    def __bool__(self) -> bool:
        return type(self)._instance is not None


pgm = _Proxy()
process_group_manager = pgm


def setup_process_group_manager(tp_size: int = 1, cp_size: int = 1, pp_size: int = 1, dp_size: int = 1,
                                ep_size: int = 1) -> ProcessGroupManager:
    inst = ProcessGroupManager(tp_size, cp_size, pp_size, dp_size, ep_size)
    _Proxy._instance = inst
    return inst


def reset_process_group_manager() -> None:
    if _Proxy._instance is not None:
        _Proxy._instance = None


def get_process_group_manager() -> ProcessGroupManager | None:
    return _Proxy._instance


# ------------------------------------------------------------------ convenience accessors
def tp_size() -> int:
    return pgm.tp_world_size if pgm else 1


def tp_rank() -> int:
    return pgm.tp_rank if pgm else 0


def tp_group():
    return pgm.tp_group if pgm else None


def cp_size() -> int:
    return pgm.cp_world_size if pgm else 1


def cp_rank() -> int:
    return pgm.cp_rank if pgm else 0


def ep_size() -> int:
    return pgm.ep_world_size if pgm else 1


def ep_rank() -> int:
    return pgm.ep_rank if pgm else 0


def pp_size() -> int:
    return pgm.pp_world_size if pgm else 1
