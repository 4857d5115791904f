"""Checkpoint save / resume in the reference layout + HF safetensors import.

Reference: CheckpointManager and init helpers in scaletorch/utils/checkpoint.py:23-560.
Layout (kept byte-for-byte so tooling and resume scripts carry over):
  {work_dir}/{step}/weights_tp_rank_world_size={tp}_{tpws}_pp_rank_world_size={pp}_{ppws}.pth
  {work_dir}/{step}/scheduler.pt
with ``{"model", "optimizer", "trained_steps", "trained_tokens"}`` per file and
model keys in the reference naming (``reference_state_dict``).  Additions:
``_ep_rank_world_size={ep}_{epws}`` is appended only when EP > 1 (the
reference's EP shards overwrote each other); writes can run on a background
thread after a device->host copy so the training loop does not stall on disk;
``latest_checkpoint`` enables torchrun auto-resume.  Loading always uses
``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import glob
import json
import logging
import os
import re
import threading
from pathlib import Path

import torch

from ..dist import collectives as C
from ..parallel import mesh

logger = logging.getLogger(__name__)


def checkpoint_filename(tp_rank: int, tp_ws: int, pp_rank: int, pp_ws: int, ep_rank: int = 0, ep_ws: int = 1) -> str:
    name = f"weights_tp_rank_world_size={tp_rank}_{tp_ws}_pp_rank_world_size={pp_rank}_{pp_ws}"
    if ep_ws > 1:
        name += f"_ep_rank_world_size={ep_rank}_{ep_ws}"
    return name + ".pth"


def _shard_filename() -> str:
    return f"optimizer_shard_rank_world_size={C.get_rank()}_{C.get_world_size()}.pth"


def _coords():
    pg = mesh.pgm
    if not pg:
        return 0, 1, 0, 1, 0, 1, 0, 0
    return (pg.tp_rank, pg.tp_world_size, pg.pp_rank, pg.pp_world_size, pg.ep_rank, pg.ep_world_size,
            pg.dp_rank, pg.cp_rank)


def _to_cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().to("cpu", copy=True)
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


_DONE = "complete_rank_world_size={}_{}"
_STARTED = "started_rank_world_size={}_{}"


def _has_markers(step_dir: str) -> bool:
    return bool(glob.glob(os.path.join(step_dir, "complete_rank_world_size=*"))
                or glob.glob(os.path.join(step_dir, "started_rank_world_size=*")))


def is_complete(step_dir: str) -> bool:
    """Every rank of the job that wrote ``step_dir`` finished its files: each rank
    drops ``started_rank_world_size={r}_{W}`` BEFORE its first file and
    ``complete_rank_world_size={r}_{W}`` after its last one (incl. ZeRO-1 optimizer
    shards); a directory from a crash mid-save lacks some completion markers.

    A directory with neither kind of marker predates them (legacy layout).  It
    counts as complete only with ``ST_CKPT_ACCEPT_UNMARKED=1`` (the default) AND
    when no OLDER sibling step directory carries markers: once the current code has
    saved (marked) step N, an unmarked step M > N can only be its crash before the
    first marker.  Unmarked directories older than every marked one are legacy
    saves and stay valid, so a crash during the first marked save after resuming
    from a legacy step falls back to that step, not to step 0."""
    marks = glob.glob(os.path.join(step_dir, "complete_rank_world_size=*"))
    if not marks:
        if glob.glob(os.path.join(step_dir, "started_rank_world_size=*")):
            return False  # a save began and never finished
        if os.environ.get("ST_CKPT_ACCEPT_UNMARKED", "1") != "1":
            logger.warning("skipping checkpoint %s: no completion markers", step_dir)
            return False
        parent = os.path.dirname(os.path.abspath(step_dir))
        me = os.path.basename(os.path.abspath(step_dir))
        for sib in glob.glob(os.path.join(parent, "*")):
            b = os.path.basename(sib)
            if b.isdigit() and me.isdigit() and int(b) < int(me) and _has_markers(sib):
                logger.warning("skipping unmarked checkpoint %s: older sibling %s has save markers "
                               "(a crash before this save's first marker)", step_dir, sib)
                return False
        logger.warning("checkpoint %s has no completion markers (legacy layout); treating it as complete "
                       "(ST_CKPT_ACCEPT_UNMARKED=0 skips such directories)", step_dir)
        return True
    worlds = {m.rsplit("_", 1)[-1] for m in marks}
    if len(worlds) != 1:
        return False
    return len(marks) == int(worlds.pop())


def latest_checkpoint(work_dir: str) -> str | None:
    """Newest COMPLETE step directory under ``work_dir`` (auto-resume)."""
    steps = []
    for d in glob.glob(os.path.join(work_dir, "*")):
        b = os.path.basename(d)
        if b.isdigit() and glob.glob(os.path.join(d, "weights_*.pth")) and is_complete(d):
            steps.append(int(b))
    return os.path.join(work_dir, str(max(steps))) if steps else None


class CheckpointManager:
    def __init__(self, work_dir: str = "./work_dir", async_save: bool = True):
        self.work_dir = work_dir
        self.async_save = async_save
        self._thread: threading.Thread | None = None

    def wait(self) -> None:
        if self._thread is not None:
            self._thread.join()
            self._thread = None

    def save_checkpoint(self, model, optimizer, trained_steps: int, trained_tokens: int, out_dir: str | None = None,
                        lr_scheduler=None) -> str:
        tp, tpws, pp, ppws, ep, epws, dp, cp = _coords()
        out_dir = out_dir or os.path.join(self.work_dir, str(trained_steps))
        path = os.path.join(out_dir, checkpoint_filename(tp, tpws, pp, ppws, ep, epws))
        raw = getattr(model, "module", model)
        if hasattr(model, "wait_params"):  # ZeRO-1: parameter all-gathers may still be in flight
            model.wait_params()
        writer = dp == 0 and cp == 0  # one copy per (tp, pp, ep) shard
        sharded = bool(getattr(optimizer, "sharded", False))
        writes = []
        if writer:
            sd = raw.reference_state_dict() if hasattr(raw, "reference_state_dict") else raw.state_dict()
            opt = {"zero1_sharded": True, "world": C.get_world_size()} if sharded else _to_cpu(optimizer.state_dict())
            payload = {"model": _to_cpu(sd), "optimizer": opt,
                       "trained_steps": trained_steps, "trained_tokens": trained_tokens}
            writes.append((path, payload))
        if sharded:  # ZeRO-1: every rank owns a distinct optimizer shard
            writes.append((os.path.join(out_dir, _shard_filename()), _to_cpu(optimizer.state_dict())))
        os.makedirs(out_dir, exist_ok=True)
        sched = _to_cpu(lr_scheduler.state_dict()) if (lr_scheduler is not None and writer) else None
        self.wait()
        done = os.path.join(out_dir, _DONE.format(C.get_rank(), C.get_world_size()))
        # before any file of this rank lands: a crash from here on leaves a directory
        # that is_complete() recognises as a partial save
        with open(os.path.join(out_dir, _STARTED.format(C.get_rank(), C.get_world_size())), "w") as f:
            f.write("started\n")

        def _write():
            for pth, obj in writes:
                tmp = pth + ".tmp"
                torch.save(obj, tmp, _use_new_zipfile_serialization=True)
                os.replace(tmp, pth)
            if sched is not None and tp == 0 and pp == 0 and ep == 0:
                torch.save(sched, os.path.join(out_dir, "scheduler.pt"))
            with open(done, "w") as f:  # last: this rank's part of the step directory is on disk
                f.write("ok\n")

        if self.async_save:
            self._thread = threading.Thread(target=_write, daemon=False)
            self._thread.start()
        else:
            _write()
        return path

    def load_checkpoint(self, model, optimizer, resume_path: str, lr_scheduler=None, strict: bool = True):
        """Returns (trained_steps, trained_tokens)."""
        tp, tpws, pp, ppws, ep, epws, _, _ = _coords()
        path = os.path.join(resume_path, checkpoint_filename(tp, tpws, pp, ppws, ep, epws))
        if not os.path.exists(path):
            raise FileNotFoundError(f"checkpoint {path} not found")
        ck = torch.load(path, map_location="cpu", weights_only=True)
        for k in ("model", "optimizer", "trained_steps", "trained_tokens"):
            if k not in ck:
                raise KeyError(f"checkpoint {path} missing key {k!r}")
        raw = getattr(model, "module", model)
        with torch.no_grad():
            if hasattr(raw, "load_reference_state_dict"):
                raw.load_reference_state_dict(ck["model"], strict=strict)
            else:
                raw.load_state_dict(ck["model"], strict=strict)
        if optimizer is not None:
            opt = ck["optimizer"]
            if isinstance(opt, dict) and opt.get("zero1_sharded"):
                if opt.get("world") != C.get_world_size():
                    raise ValueError("ZeRO-1 checkpoint was written with a different world size")
                opt = torch.load(os.path.join(resume_path, _shard_filename()), map_location="cpu", weights_only=True)
            optimizer.load_state_dict(opt)
        sp = os.path.join(resume_path, "scheduler.pt")
        if lr_scheduler is not None and os.path.exists(sp):
            lr_scheduler.load_state_dict(torch.load(sp, weights_only=True))
        return int(ck["trained_steps"]), int(ck["trained_tokens"])


# ------------------------------------------------------------------ HF safetensors import
_HF_MAP = [
    (r"^model\.embed_tokens\.weight$", "embedding.weight"),
    (r"^model\.norm\.weight$", "final_norm.weight"),
    (r"^lm_head\.weight$", "final_proj.weight"),
    (r"^model\.layers\.(\d+)\.self_attn\.o_proj\.", r"decoder_layers.\1.attention.out_proj."),
    (r"^model\.layers\.(\d+)\.self_attn\.([qkv])_proj\.", r"decoder_layers.\1.attention.\2_proj."),
    (r"^model\.layers\.(\d+)\.self_attn\.([qk])_norm\.", r"decoder_layers.\1.attention.\2_norm."),
    (r"^model\.layers\.(\d+)\.mlp\.gate\.weight$", r"decoder_layers.\1.moe.router.gate.weight"),
    (r"^model\.layers\.(\d+)\.block_sparse_moe\.gate\.weight$", r"decoder_layers.\1.moe.router.gate.weight"),
    (r"^model\.layers\.(\d+)\.mlp\.experts\.(\d+)\.(gate|up|down)_proj\.", r"decoder_layers.\1.moe.experts.experts.\2.\3_proj."),
    (r"^model\.layers\.(\d+)\.block_sparse_moe\.experts\.(\d+)\.w1\.", r"decoder_layers.\1.moe.experts.experts.\2.gate_proj."),
    (r"^model\.layers\.(\d+)\.block_sparse_moe\.experts\.(\d+)\.w3\.", r"decoder_layers.\1.moe.experts.experts.\2.up_proj."),
    (r"^model\.layers\.(\d+)\.block_sparse_moe\.experts\.(\d+)\.w2\.", r"decoder_layers.\1.moe.experts.experts.\2.down_proj."),
    (r"^model\.layers\.(\d+)\.mlp\.(gate|up|down)_proj\.", r"decoder_layers.\1.mlp.\2_proj."),
    (r"^model\.layers\.(\d+)\.(input_layernorm|post_attention_layernorm)\.", r"decoder_layers.\1.\2."),
]


def hf_to_internal_name(name: str) -> str | None:
    for pat, rep in _HF_MAP:
        if re.search(pat, name):
            return re.sub(pat, rep, name)
    return None


def _tp_split_dim(name: str) -> int | None:
    """Dimension a reference-named weight is split along under TP (None = replicated):
    column-parallel (q/k/v, gate/up incl. experts, LM head, vocab embedding) on the
    output rows, row-parallel (o, down incl. experts) on the input columns
    (reference InitializationManager, scaletorch/utils/checkpoint.py:339-423)."""
    if any(s in name for s in ("out_proj", "down_proj")):
        return 1
    if any(s in name for s in ("q_proj", "k_proj", "v_proj", "gate_proj", "up_proj", "final_proj", "embedding")):
        return 0
    return None


def _tp_slice(name: str, t: torch.Tensor, tp: int, rank: int) -> torch.Tensor:
    d = _tp_split_dim(name) if tp > 1 else None
    return t if d is None else t.chunk(tp, d)[rank]


def _read_tp_shard(fh, name: str, iname: str, tp: int, rank: int) -> torch.Tensor:
    """Read only this TP rank's slice of tensor ``name`` (safetensors slices the
    memory-mapped file, so an 8B shard never materialises the full matrix)."""
    d = _tp_split_dim(iname) if tp > 1 else None
    if d is None:
        return fh.get_tensor(name)
    sl = fh.get_slice(name)
    n = sl.get_shape()[d]
    if n % tp:
        raise ValueError(f"{name}: dim {d} of size {n} does not split over tp={tp}")
    lo, hi = rank * (n // tp), (rank + 1) * (n // tp)
    return sl[lo:hi] if d == 0 else sl[:, lo:hi]


def hf_weight_files(path: str) -> list[str]:
    """The safetensors files of an HF checkpoint directory: the shards named by
    ``model.safetensors.index.json`` when present (reference _load_sharded_checkpoint,
    scaletorch/utils/checkpoint.py:145-187), else every ``*.safetensors``."""
    if not path or not os.path.isdir(path):
        return []
    idx = os.path.join(path, "model.safetensors.index.json")
    if os.path.exists(idx):
        with open(idx) as f:
            shards = sorted(set(json.load(f)["weight_map"].values()))
        missing = [s for s in shards if not os.path.exists(os.path.join(path, s))]
        if missing:
            raise FileNotFoundError(f"{idx} names shards that are not present: {missing}")
        return [os.path.join(path, s) for s in shards]
    return sorted(glob.glob(os.path.join(path, "*.safetensors")))


def load_hf_safetensors(model, path: str, strict: bool = False, optimizer=None) -> list[str]:
    """Load this rank's shard of an HF checkpoint dir (single file or sharded index) into ``model``.

    Only the tensors of this PP stage / EP shard are read, and of those only this TP
    rank's slice (safetensors memory-maps the files).  HF names map to the internal ones
    through ``_HF_MAP`` (Llama / Qwen3 / Qwen3-MoE / Mixtral ``w1/w2/w3``); tied
    embeddings fill the LM head from ``embed_tokens``.  The bf16 parameters may be
    views into the DP arena, so the copy lands there; when an arena optimizer already
    exists pass it as ``optimizer`` so its fp32 master copy is refreshed (otherwise
    its first step would write the stale masters back).

    Raises when the files hold none of this rank's tensors (a wrong directory must
    not silently train from random weights) and, with ``strict``, when any of them is
    missing.  Returns the sorted internal names loaded.
    """
    from safetensors import safe_open

    raw = getattr(model, "module", model)
    tp = mesh.tp_size()
    tpr = mesh.tp_rank()
    ep, epr = mesh.ep_size(), mesh.ep_rank()
    files = hf_weight_files(path)
    if not files:
        raise FileNotFoundError(f"no *.safetensors under {path}")
    wanted = set(raw.reference_state_dict().keys())
    sd = {}
    for f in files:
        with safe_open(f, framework="pt") as fh:
            for name in fh.keys():
                iname = hf_to_internal_name(name)
                if iname is None:
                    continue
                m = re.match(r"(.*moe\.experts\.experts\.)(\d+)(\..*)", iname)
                if m and ep > 1:
                    e = int(m.group(2))
                    per = raw.config.num_experts // ep
                    if e // per != epr:
                        continue
                    iname = f"{m.group(1)}{e % per}{m.group(3)}"
                if iname not in wanted and not (iname == "embedding.weight" and "final_proj.weight" in wanted):
                    continue
                sd[iname] = _read_tp_shard(fh, name, iname, tp, tpr)
    if raw.config.tie_word_embeddings and "final_proj.weight" in wanted and "final_proj.weight" not in sd \
            and "embedding.weight" in sd:
        sd["final_proj.weight"] = sd["embedding.weight"]
    if not sd:
        raise ValueError(f"{path}: {len(files)} safetensors file(s) but none of their tensors maps onto this "
                         f"rank's {len(wanted)} parameters (wrong architecture or naming?)")
    missing = sorted(wanted - set(sd))
    if missing:
        msg = f"{path}: {len(missing)} of {len(wanted)} parameters not in the checkpoint, e.g. {missing[:4]}"
        if strict:
            raise KeyError(msg)
        logger.warning("%s: they keep their random init", msg)
    dtype = next(raw.parameters()).dtype
    with torch.no_grad():
        raw.load_reference_state_dict({k: v.to(dtype) for k, v in sd.items()}, strict=False)
    if optimizer is not None and hasattr(optimizer, "reload_masters"):
        optimizer.reload_masters()
    return sorted(sd)


def maybe_load_hf_weights(model, name_or_path: str, mode: str = "auto", optimizer=None) -> int:
    """Model-build hook (reference model_builder.py:82-84 -> init_model_with_materialized_weights):
    ``auto`` loads when ``name_or_path`` is a directory holding safetensors, ``required``
    fails without them, ``off`` keeps the random init.  Returns the tensor count loaded
    on this rank (0 = random init) and logs it."""
    if mode == "off":
        return 0
    files = hf_weight_files(name_or_path)
    if not files:
        if mode == "required":
            raise FileNotFoundError(f"--hf_weights required but {name_or_path!r} holds no *.safetensors")
        return 0
    names = load_hf_safetensors(model, name_or_path, strict=(mode == "required"), optimizer=optimizer)
    logger.info("loaded %d tensors from %d safetensors file(s) under %s (tp %d/%d, pp stage %d, ep %d/%d)",
                len(names), len(files), name_or_path, mesh.tp_rank(), mesh.tp_size(),
                mesh.pgm.pp_rank if mesh.pgm else 0, mesh.ep_rank(), mesh.ep_size())
    return len(names)
