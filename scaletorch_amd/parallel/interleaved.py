"""Interleaved 1F1B pipeline schedule (virtual pipeline stages).

Each of the P pipeline ranks holds V model chunks: the L layers are split evenly
into P*V chunks and global chunk c = v*P + r lives on rank r as its local chunk v
(the embedding on rank 0 chunk 0, the final norm + LM head on rank P-1 chunk
V-1).  A micro-batch therefore visits the ring of ranks V times, and the
pipeline bubble shrinks from (P-1)/(M+P-1) to (P-1)/(V*M+P-1) of the step for M
micro-batches (Narayanan et al., "Efficient Large-Scale Language Model Training
on GPU Clusters", 2021).  The reference has AFAB and plain 1F1B only
(scaletorch/parallel/pipeline_parallel/pipeline_parallel.py:457-671).

Step numbering (identical on every rank, M a multiple of P):
  forward step k  -> chunk  (k mod P*V) // P,          micro-batch (k // (P*V))*P + k mod P
  backward step k -> chunk  V-1 - (k mod P*V) // P,    same micro-batch formula
so a forward message produced at step k is consumed by the next rank at ITS step
k, except across the ring seam (rank P-1 -> rank 0, next chunk), where it is step
k + P; backward messages mirror this.  ``build_schedule`` returns, per rank, the
ordered list of compute steps and batched exchanges; ``simulate`` replays all
ranks under RCCL semantics (one ordered p2p stream per rank: a batch starts once
the previous one has completed; an op completes when its partner's current batch
holds the matching op) and proves the schedule deadlock-free and order-matched.
"""
from __future__ import annotations

from dataclasses import dataclass, field


def fwd_chunk(k: int, P: int, V: int) -> int:
    return (k % (P * V)) // P


def bwd_chunk(k: int, P: int, V: int) -> int:
    return V - 1 - (k % (P * V)) // P


def micro_batch(k: int, P: int, V: int) -> int:
    return (k // (P * V)) * P + k % P


def num_warmup(P: int, V: int, M: int, r: int) -> int:
    return min((P - r - 1) * 2 + (V - 1) * P, M * V)


@dataclass
class Exchange:
    """One batched p2p exchange: entries are ("fwd" | "bwd", step) -- a forward
    message carries the output of forward step `step`, a backward message the
    input gradient of backward step `step` (the sender's numbering)."""
    send: list = field(default_factory=list)
    recv: list = field(default_factory=list)  # ("fwd", k): input of OUR fwd step k; ("bwd", k): grad for OUR bwd step k


def build_schedule(P: int, V: int, M: int, r: int) -> list:
    """Ordered actions of rank r: ("F", k), ("B", k) and Exchange objects."""
    if M % P:
        raise ValueError(f"interleaved 1F1B needs micro-batches ({M}) divisible by pipeline size ({P})")
    T = M * V
    W = num_warmup(P, V, M, r)
    first, last = r == 0, r == P - 1

    def send_fwd(k):
        return not (last and fwd_chunk(k, P, V) == V - 1)

    def recv_fwd(k):  # input of forward step k comes over the wire
        return k < T and not (first and fwd_chunk(k, P, V) == 0)

    def send_bwd(k):
        return not (first and bwd_chunk(k, P, V) == 0)

    def recv_bwd(k):
        return k < T and not (last and bwd_chunk(k, P, V) == V - 1)

    acts = []
    if recv_fwd(0):
        acts.append(Exchange(recv=[("fwd", 0)]))
    for k in range(W):
        acts.append(("F", k))
        ex = Exchange()
        if send_fwd(k):
            ex.send.append(("fwd", k))
        if recv_fwd(k + 1) and k + 1 < T:
            ex.recv.append(("fwd", k + 1))
        if k == W - 1 and W < T and recv_bwd(0):
            ex.recv.append(("bwd", 0))
        if ex.send or ex.recv:
            acts.append(ex)
    for j in range(T - W):
        fk, bk = W + j, j
        acts.append(("F", fk))
        acts.append(("B", bk))
        ex = Exchange()
        if send_fwd(fk):
            ex.send.append(("fwd", fk))
        if send_bwd(bk):
            ex.send.append(("bwd", bk))
        if fk + 1 < T and recv_fwd(fk + 1):
            ex.recv.append(("fwd", fk + 1))
        if recv_bwd(bk + 1):
            ex.recv.append(("bwd", bk + 1))
        if ex.send or ex.recv:
            acts.append(ex)
    if W == T and recv_bwd(0):  # all-warmup rank: the first gradient arrives on its own
        acts.append(Exchange(recv=[("bwd", 0)]))
    for bk in range(T - W, T):
        acts.append(("B", bk))
        ex = Exchange()
        if send_bwd(bk):
            ex.send.append(("bwd", bk))
        if recv_bwd(bk + 1):
            ex.recv.append(("bwd", bk + 1))
        if ex.send or ex.recv:
            acts.append(ex)
    return acts


def _peer_and_key(P: int, r: int, kind: str, k: int, sending: bool):
    """(peer rank, message key) of a message; the key names the message the same way
    on both ends: (kind, receiver's step)."""
    if kind == "fwd":
        if sending:
            dst = (r + 1) % P
            return dst, ("fwd", k + P if r == P - 1 else k)
        return (r - 1) % P, ("fwd", k)
    if sending:
        dst = (r - 1) % P
        return dst, ("bwd", k + P if r == 0 else k)
    return (r + 1) % P, ("bwd", k)


def simulate(P: int, V: int, M: int) -> None:
    """Replay every rank's schedule under ordered-stream p2p semantics; raises on a
    deadlock, an unmatched message or a compute step whose input never arrived."""
    scheds = [build_schedule(P, V, M, r) for r in range(P)]
    pos = [0] * P
    pending = [None] * P   # rank -> list of (peer, key, is_send) still open in its current batch
    have_fwd = [set() for _ in range(P)]
    have_bwd = [set() for _ in range(P)]
    T = M * V

    def load(r):
        while pos[r] < len(scheds[r]) and pending[r] is None:
            a = scheds[r][pos[r]]
            if isinstance(a, Exchange):
                ops = [(*_peer_and_key(P, r, kd, k, True), True) for kd, k in a.send]
                ops += [(*_peer_and_key(P, r, kd, k, False), False) for kd, k in a.recv]
                pending[r] = ops
            else:
                kind, k = a
                if kind == "F":
                    if not ((r == 0 and fwd_chunk(k, P, V) == 0) or k in have_fwd[r]):
                        raise AssertionError(f"rank {r}: forward step {k} without its input")
                else:
                    if not ((r == P - 1 and bwd_chunk(k, P, V) == V - 1) or k in have_bwd[r]):
                        raise AssertionError(f"rank {r}: backward step {k} without its output grad")
                pos[r] += 1

    for r in range(P):
        load(r)
    while True:
        progressed = False
        for r in range(P):
            if not pending[r]:
                continue
            for op in list(pending[r]):
                peer, key, is_send = op
                if pending[peer] is None:
                    continue
                match = (r, key, not is_send)
                if match in pending[peer]:
                    pending[r].remove(op)
                    pending[peer].remove(match)
                    recv_rank = peer if is_send else r
                    (have_fwd if key[0] == "fwd" else have_bwd)[recv_rank].add(key[1])
                    progressed = True
            for q in range(P):
                if pending[q] == []:
                    pending[q] = None
                    pos[q] += 1
                    load(q)
        if all(pos[r] >= len(scheds[r]) and pending[r] is None for r in range(P)):
            break
        if not progressed:
            state = {r: (pos[r], pending[r]) for r in range(P)}
            raise AssertionError(f"p2p deadlock (P={P}, V={V}, M={M}): {state}")
    for r in range(P):
        nb = sum(1 for a in scheds[r] if not isinstance(a, Exchange) and a[0] == "B")
        nf = sum(1 for a in scheds[r] if not isinstance(a, Exchange) and a[0] == "F")
        if nf != T or nb != T:
            raise AssertionError(f"rank {r}: {nf} forward / {nb} backward steps, expected {T}")


def simulate_channels(P: int, V: int, M: int, depth: int = 2) -> None:
    """Replay every rank's schedule as the engine runs it (pipeline_parallel.py): each
    message travels on a CHANNEL = (direction, ring seam or not), i.e. one direction
    between one pair of ranks on its own communicator, whose stream runs that rank's ops
    on the channel in issue order; receives are posted ``depth`` ahead of their use in
    schedule order; a send is issued after the compute step that produced its tensor;
    each rank's compute steps run in schedule order, a step waiting for its input.
    Raises on a deadlock.  (``simulate`` proves the stricter one-ordered-stream model.)"""
    scheds = [build_schedule(P, V, M, r) for r in range(P)]
    T = M * V

    def chan(kind, sender):
        seam = (kind == "fwd" and sender == P - 1) or (kind == "bwd" and sender == 0)
        return (kind, seam, sender)

    # per rank: the compute steps in order, and the sends each step releases
    steps, sends_after, recv_order = [], [], []
    for r in range(P):
        st, rel, ro = [], {}, {"fwd": [], "bwd": []}
        last_step = None
        for a in scheds[r]:
            if isinstance(a, Exchange):
                for kd, k in a.send:
                    rel.setdefault(last_step, []).append((kd, k))
                for kd, k in a.recv:
                    ro[kd].append(k)
            else:
                st.append(a)
                last_step = a
        steps.append(st)
        sends_after.append(rel)
        recv_order.append(ro)
    # channel queues: sender side (issued sends), receiver side (posted receives)
    sq: dict = {}
    rq: dict = {}
    posted = [{"fwd": 0, "bwd": 0} for _ in range(P)]
    delivered = [set() for _ in range(P)]  # (kind, receiver step) that arrived

    def post(r):
        for kd in ("fwd", "bwd"):
            sender = (r - 1) % P if kd == "fwd" else (r + 1) % P
            c = chan(kd, sender)
            used = sum(1 for key in delivered[r] if key[0] == kd)
            while posted[r][kd] < len(recv_order[r][kd]) and posted[r][kd] < used + depth:
                rq.setdefault(c, []).append(recv_order[r][kd][posted[r][kd]])
                posted[r][kd] += 1

    pos = [0] * P
    for r in range(P):
        post(r)
    while True:
        progressed = False
        for r in range(P):  # compute steps whose input has arrived
            while pos[r] < len(steps[r]):
                kind, k = steps[r][pos[r]]
                need = None
                if kind == "F" and not (r == 0 and fwd_chunk(k, P, V) == 0):
                    need = ("fwd", k)
                if kind == "B" and not (r == P - 1 and bwd_chunk(k, P, V) == V - 1):
                    need = ("bwd", k)
                if need is not None and need not in delivered[r]:
                    break
                for kd, kk in sends_after[r].get((kind, k), []):
                    _, key = _peer_and_key(P, r, kd, kk, True)
                    sq.setdefault(chan(kd, r), []).append(key[1])
                pos[r] += 1
                progressed = True
        for c in list(sq):  # deliver matched channel heads
            kd, _, sender = c
            recv_rank = (sender + 1) % P if kd == "fwd" else (sender - 1) % P
            while sq.get(c) and rq.get(c) and sq[c][0] == rq[c][0]:
                delivered[recv_rank].add((kd, sq[c].pop(0)))
                rq[c].pop(0)
                progressed = True
            if sq.get(c) and rq.get(c) and sq[c][0] != rq[c][0]:
                raise AssertionError(f"channel {c}: send {sq[c][0]} meets receive {rq[c][0]} (order mismatch)")
        for r in range(P):
            post(r)
        if all(pos[r] == len(steps[r]) for r in range(P)):
            break
        if not progressed:
            raise AssertionError(f"channel deadlock (P={P}, V={V}, M={M}): steps at {pos}")
    for r in range(P):
        if len(steps[r]) != 2 * T:
            raise AssertionError(f"rank {r}: {len(steps[r])} compute steps, expected {2 * T}")


# ---------------------------------------------------------------------------
# Stream-level replay of the engine (pipeline_parallel.PipelineEngine) on RCCL
# ---------------------------------------------------------------------------
def channel_layout(kind: str, sender: int, receiver: int, P: int):
    """Communicator of a message in the engine's layout: one 2-rank communicator per
    directed stage pair (mesh.ProcessGroupManager._pp_channels)."""
    return (kind, sender, receiver)


def shared_layout(kind: str, sender: int, receiver: int, P: int):
    """The round-3 layout: one whole-pipeline communicator per direction (plus the
    interleaved ring seam on two more) -- a middle stage's activation receive and
    its activation send share one RCCL stream."""
    seam = (kind == "fwd" and sender == P - 1) or (kind == "bwd" and sender == 0)
    return (kind, "seam" if seam else "pipe")


def engine_programs(P: int, V: int, M: int, schedule: str = "1f1b", depth: int = 2, layout=channel_layout):
    """Per-rank event lists in the engine's HOST issue order:
    ("post", comm, peer, key) an irecv, ("send", comm, peer, key) an isend,
    ("wait", key) the compute stream waiting for a received message.  Message keys
    are (kind, receiving rank, receiver's step / micro-batch)."""
    progs = []
    for r in range(P):
        ev = []
        if schedule == "interleaved":
            sched = build_schedule(P, V, M, r)
            order = {"fwd": [], "bwd": []}
            for a in sched:
                if isinstance(a, Exchange):
                    for kd, k in a.recv:
                        order[kd].append(k)
            src = {"fwd": (r - 1) % P, "bwd": (r + 1) % P}
        else:
            order = {"fwd": list(range(M)) if r > 0 else [], "bwd": list(range(M)) if r < P - 1 else []}
            src = {"fwd": r - 1, "bwd": r + 1}
        posted = {"fwd": 0, "bwd": 0}

        def fill(kd):
            while posted[kd] < len(order[kd]) and posted[kd] - taken[kd] < depth:
                k = order[kd][posted[kd]]
                ev.append(("post", layout(kd, src[kd], r, P), src[kd], (kd, r, k)))
                posted[kd] += 1

        taken = {"fwd": 0, "bwd": 0}

        def take(kd):
            taken[kd] += 1
            fill(kd)

        def send(kd, dst, k):
            ev.append(("send", layout(kd, r, dst, P), dst, (kd, dst, k)))

        fill("fwd")
        fill("bwd")
        if schedule == "interleaved":
            for a in build_schedule(P, V, M, r):
                if isinstance(a, Exchange):
                    for kd, k in a.send:
                        dst, key = _peer_and_key(P, r, kd, k, True)
                        send(kd, dst, key[1])
                    for kd, _k in a.recv:
                        take(kd)
                    continue
                kind, k = a
                if kind == "F" and not (r == 0 and fwd_chunk(k, P, V) == 0):
                    ev.append(("wait", ("fwd", r, k)))
                if kind == "B" and not (r == P - 1 and bwd_chunk(k, P, V) == V - 1):
                    ev.append(("wait", ("bwd", r, k)))
        else:
            def fwd(m):
                if r > 0:
                    take("fwd")
                    ev.append(("wait", ("fwd", r, m)))
                if r < P - 1:
                    send("fwd", r + 1, m)

            def bwd(m):
                if r < P - 1:
                    take("bwd")
                    ev.append(("wait", ("bwd", r, m)))
                if r > 0:
                    send("bwd", r - 1, m)

            if schedule == "afab":
                for m in range(M):
                    fwd(m)
                for m in range(M):
                    bwd(m)
            else:
                warm = min(P - r - 1, M)
                for m in range(warm):
                    fwd(m)
                for j in range(M - warm):
                    fwd(warm + j)
                    bwd(j)
                for j in range(M - warm, M):
                    bwd(j)
        progs.append(ev)
    return progs


def simulate_streams(progs) -> None:
    """Replay per-rank programs under RCCL semantics: the host never blocks; the
    compute stream runs the program in order and stalls at a "wait" until that
    message has arrived; every p2p op is enqueued on the stream of (rank, its
    communicator) and becomes runnable once the compute stream has reached its issue
    point (ProcessGroupNCCL fences the comm stream on the current stream); each such
    stream runs its ops strictly in order, and a send and its receive complete
    together when both are at the heads of their streams.  Raises on a deadlock or
    on two heads of one communicator that pair up in the wrong order."""
    P = len(progs)
    cpos = [0] * P
    queues: dict = {}
    arrived = set()
    while True:
        progressed = False
        for r in range(P):
            while cpos[r] < len(progs[r]):
                e = progs[r][cpos[r]]
                if e[0] == "wait":
                    if e[1] not in arrived:
                        break
                else:
                    queues.setdefault((r, e[1]), []).append(e)
                cpos[r] += 1
                progressed = True
        for (r, comm), q in list(queues.items()):
            while q:
                op, _, peer, key = q[0]
                if op != "send":
                    break
                pq = queues.get((peer, comm))
                if not pq:
                    break
                pop, _, ppeer, pkey = pq[0]
                if pop != "post" or ppeer != r:
                    break
                if pkey != key:
                    raise AssertionError(f"communicator {comm}: send {key} meets receive {pkey}")
                q.pop(0)
                pq.pop(0)
                arrived.add(key)
                progressed = True
        if all(cpos[r] == len(progs[r]) for r in range(P)) and not any(queues.values()):
            return
        if not progressed:
            heads = {k: q[0] for k, q in queues.items() if q}
            raise AssertionError(f"p2p stream deadlock: compute at {cpos}, stream heads {heads}")
