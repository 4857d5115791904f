#!/usr/bin/env python3
"""2-D FSDP2 x TP Llama with PyTorch DTensor: tensor parallel (+ sequence parallel)
inside a node, FSDP2 across the data-parallel dimension, ``loss_parallel`` cross
entropy on vocab-sharded logits, DCP (sharded) checkpoints with resume, and an
optional FSDP2 CPU-offload mode.

Reference: examples/FSDP2/fsdp2_tp_llama2_main.py:91-507 (2-D mesh, SP-style TP plan,
loss_parallel, DCP resume) and examples/FSDP2/fsdp2_llama2_main.py (CPU offload).
MI355X side: the attention core of every layer is the framework's gfx950 flash
kernel (``scaletorch_amd.ops.flash_attn``, GQA-native) running on each TP rank's
local heads; collectives are RCCL over xGMI (gloo on CPU).

  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/fsdp2/fsdp2_tp_llama.py --tp 2 --steps 10
  torchrun --nproc-per-node 4 --master-addr 127.0.0.1 examples/fsdp2/fsdp2_tp_llama.py --cpu --tp 2   # gloo
  ... --cpu-offload     # FSDP2 parameters + optimizer states on the host (fsdp2_llama2_main.py)
  ... --resume          # continue from the DCP checkpoint in --ckpt-dir
"""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.realpath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402

PRESETS = {  # (dim, layers, heads, kv_heads, ffn, vocab); reference examples/FSDP2/llama2.py:25-54
    "debug": (256, 2, 8, 4, 512, 512),
    "llama2-small": (1024, 8, 16, 8, 2816, 32000),
    "llama3-8b": (4096, 32, 32, 8, 14336, 128256),
}


class Attention(nn.Module):
    def __init__(self, dim, heads, kv_heads):
        super().__init__()
        self.n_heads, self.n_kv, self.hd = heads, kv_heads, dim // heads
        self.wq = nn.Linear(dim, heads * self.hd, bias=False)
        self.wk = nn.Linear(dim, kv_heads * self.hd, bias=False)
        self.wv = nn.Linear(dim, kv_heads * self.hd, bias=False)
        self.wo = nn.Linear(heads * self.hd, dim, bias=False)

    def forward(self, x, cos, sin):
        from scaletorch_amd import ops

        B, S = x.shape[0], x.shape[1]
        # after ColwiseParallel (use_local_output) these are this rank's local heads
        q = self.wq(x).view(B, S, -1, self.hd)
        k = self.wk(x).view(B, S, -1, self.hd)
        v = self.wv(x).view(B, S, -1, self.hd)
        q = ops.apply_rope(q, cos, sin, None)
        k = ops.apply_rope(k, cos, sin, None)
        o = ops.flash_attn(q, k, v, causal=True)  # HIP flash kernel on GPU, fp32 reference on CPU
        return self.wo(o.reshape(B, S, -1))


class FeedForward(nn.Module):
    def __init__(self, dim, ffn):
        super().__init__()
        self.w1 = nn.Linear(dim, ffn, bias=False)
        self.w3 = nn.Linear(dim, ffn, bias=False)
        self.w2 = nn.Linear(ffn, dim, bias=False)

    def forward(self, x):
        return self.w2(F.silu(self.w1(x)) * self.w3(x))


class Block(nn.Module):
    def __init__(self, dim, heads, kv_heads, ffn):
        super().__init__()
        self.attention_norm = nn.RMSNorm(dim, eps=1e-5)
        self.attention = Attention(dim, heads, kv_heads)
        self.ffn_norm = nn.RMSNorm(dim, eps=1e-5)
        self.feed_forward = FeedForward(dim, ffn)

    def forward(self, x, cos, sin):
        x = x + self.attention(self.attention_norm(x), cos, sin)
        return x + self.feed_forward(self.ffn_norm(x))


class Llama(nn.Module):
    def __init__(self, dim, layers, heads, kv_heads, ffn, vocab, max_seq=8192):
        super().__init__()
        from scaletorch_amd import ops

        self.tok_embeddings = nn.Embedding(vocab, dim)
        self.layers = nn.ModuleDict({str(i): Block(dim, heads, kv_heads, ffn) for i in range(layers)})
        self.norm = nn.RMSNorm(dim, eps=1e-5)
        self.output = nn.Linear(dim, vocab, bias=False)
        cos, sin = ops.rope_tables(max_seq, dim // heads, 500000.0)
        self.register_buffer("cos", cos, persistent=False)
        self.register_buffer("sin", sin, persistent=False)

    def forward(self, ids):
        h = self.tok_embeddings(ids)
        S = ids.shape[1]
        for layer in self.layers.values():
            h = layer(h, self.cos[:S], self.sin[:S])
        return self.output(self.norm(h))


def tp_plan_and_shard(model: Llama, tp_mesh) -> None:
    """SP-style TP plan (reference fsdp2_tp_llama2_main.py:154-204)."""
    from torch.distributed.tensor import Replicate, Shard
    from torch.distributed.tensor.parallel import (ColwiseParallel, PrepareModuleInput, RowwiseParallel,
                                                   SequenceParallel, parallelize_module)

    parallelize_module(model, tp_mesh, {
        "tok_embeddings": RowwiseParallel(input_layouts=Replicate(), output_layouts=Shard(1)),
        "norm": SequenceParallel(),
        "output": ColwiseParallel(input_layouts=Shard(1), output_layouts=Shard(-1), use_local_output=False),
    })
    for block in model.layers.values():
        parallelize_module(block, tp_mesh, {
            "attention_norm": SequenceParallel(),
            "attention": PrepareModuleInput(input_layouts=(Shard(1), None, None),
                                            desired_input_layouts=(Replicate(), None, None)),
            "attention.wq": ColwiseParallel(),
            "attention.wk": ColwiseParallel(),
            "attention.wv": ColwiseParallel(),
            "attention.wo": RowwiseParallel(output_layouts=Shard(1)),
            "ffn_norm": SequenceParallel(),
            "feed_forward": PrepareModuleInput(input_layouts=(Shard(1),), desired_input_layouts=(Replicate(),)),
            "feed_forward.w1": ColwiseParallel(),
            "feed_forward.w3": ColwiseParallel(),
            "feed_forward.w2": RowwiseParallel(output_layouts=Shard(1)),
        })


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="debug", choices=sorted(PRESETS))
    ap.add_argument("--tp", type=int, default=2)
    ap.add_argument("--seq", type=int, default=64)
    ap.add_argument("--mbs", type=int, default=2)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--lr", type=float, default=3e-3)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--cpu-offload", action="store_true", help="FSDP2 CPUOffloadPolicy (params/grads/optim on host)")
    ap.add_argument("--ckpt-dir", default="")
    ap.add_argument("--resume", action="store_true")
    return ap.parse_args(argv)


def main(argv=None) -> dict:
    args = parse(argv)
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.fsdp import CPUOffloadPolicy, MixedPrecisionPolicy, fully_shard
    from torch.distributed.tensor.parallel import loss_parallel

    from scaletorch_amd.dist.launch import init_dist

    rank, local_rank, world = init_dist(backend="gloo" if args.cpu else None, use_cpu=args.cpu)
    if world % args.tp:
        raise SystemExit(f"world {world} not divisible by tp {args.tp}")
    dev = torch.device("cpu") if (args.cpu or not torch.cuda.is_available()) else torch.device("cuda", local_rank)
    mesh = init_device_mesh(dev.type, (world // args.tp, args.tp), mesh_dim_names=("dp", "tp"))
    dp_mesh, tp_mesh = mesh["dp"], mesh["tp"]
    dim, layers, heads, kv, ffn, vocab = PRESETS[args.preset]
    if (heads % args.tp) or (kv % args.tp):
        raise SystemExit("heads and kv_heads must be divisible by tp")
    torch.manual_seed(0)  # identical init everywhere; TP/FSDP take their shards of it
    with torch.device(dev):
        model = Llama(dim, layers, heads, kv, ffn, vocab, max_seq=max(args.seq, 128))
    tp_plan_and_shard(model, tp_mesh)
    mp = MixedPrecisionPolicy(param_dtype=torch.bfloat16, reduce_dtype=torch.float32) if dev.type == "cuda" \
        else MixedPrecisionPolicy()
    kw = dict(mesh=dp_mesh, mp_policy=mp)
    if args.cpu_offload:
        kw["offload_policy"] = CPUOffloadPolicy(pin_memory=dev.type == "cuda")
    for block in model.layers.values():
        fully_shard(block, **kw)
    fully_shard(model, **kw)
    opt = torch.optim.AdamW(model.parameters(), lr=args.lr, foreach=dev.type == "cuda" and not args.cpu_offload)
    ckpt = args.ckpt_dir or os.path.join(ROOT, "work_dir", "fsdp2_tp_ckpt")
    start = load(model, opt, ckpt) if args.resume else 0
    # every TP rank of a dp replica sees the same batch; replicas see different batches
    g = torch.Generator().manual_seed(4321 + dp_mesh.get_local_rank())
    for _ in range(start):
        torch.randint(0, vocab, (args.mbs, args.seq + 1), generator=g)
    losses = []
    t0 = time.perf_counter()
    for step in range(start, start + args.steps):
        ids = torch.randint(0, vocab, (args.mbs, args.seq + 1), generator=g).to(dev)
        logits = model(ids[:, :-1])  # DTensor sharded on the vocab dim
        with loss_parallel():  # CE on vocab-sharded logits: no all-gather of [B, S, V]
            loss = F.cross_entropy(logits.flatten(0, 1), ids[:, 1:].flatten())
            loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        opt.zero_grad()
        lv = loss.full_tensor() if hasattr(loss, "full_tensor") else loss
        losses.append(float(lv.detach().float()))
        if rank == 0:
            print(f"step {step} loss {losses[-1]:.4f}", flush=True)
    dt = time.perf_counter() - t0
    save(model, opt, ckpt, start + args.steps)
    if rank == 0:
        tok = args.steps * args.mbs * args.seq * (world // args.tp)
        print(f"fsdp2xtp done: dp{world // args.tp} tp{args.tp} {tok / dt:.0f} tokens/s, final loss {losses[-1]:.4f}",
              flush=True)
    return {"losses": losses}


def save(model, opt, path: str, step: int) -> None:
    import torch.distributed.checkpoint as dcp
    from torch.distributed.checkpoint.state_dict import get_state_dict

    msd, osd = get_state_dict(model, opt)
    dcp.save({"model": msd, "optim": osd, "step": torch.tensor(step)}, checkpoint_id=path)


def load(model, opt, path: str) -> int:
    import torch.distributed.checkpoint as dcp
    from torch.distributed.checkpoint.state_dict import get_state_dict, set_state_dict

    msd, osd = get_state_dict(model, opt)
    state = {"model": msd, "optim": osd, "step": torch.tensor(0)}
    dcp.load(state, checkpoint_id=path)
    set_state_dict(model, opt, model_state_dict=state["model"], optim_state_dict=state["optim"])
    return int(state["step"])


if __name__ == "__main__":
    main()
    if dist.is_initialized():
        dist.destroy_process_group()
