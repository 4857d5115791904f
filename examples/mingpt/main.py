#!/usr/bin/env python3
"""minGPT character-level training with scaletorch_amd data parallelism.

Reference: examples/torch_examples/minigpt/{main,trainer,model,char_dataset}.py
(torch DDP + Hydra + epoch snapshots).  Here the GPT is
``scaletorch_amd.models.gpt.GPT``, data parallelism is the framework's
bucketed arena DataParallel (RCCL on GPUs, gloo on CPU -- the reference passed
``device_ids`` to DDP and could not run on CPU), config is plain YAML
(``yaml.safe_load``), and snapshots resume at epoch granularity.

  torchrun --nproc-per-node 2 --master-addr 127.0.0.1 examples/mingpt/main.py \
      --config examples/mingpt/gpt2_train_cfg.yaml --cpu
"""
from __future__ import annotations

import argparse
import math
import os
import sys
from dataclasses import dataclass

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.realpath(__file__))))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402
import yaml  # noqa: E402
from torch.utils.data import DataLoader, Dataset, DistributedSampler  # noqa: E402

from scaletorch_amd.dist import collectives as C  # noqa: E402
from scaletorch_amd.dist.launch import cleanup_dist, init_dist  # noqa: E402
from scaletorch_amd.models.gpt import GPT, GPTConfig  # noqa: E402
from scaletorch_amd.parallel.data_parallel import DataParallel  # noqa: E402


class CharDataset(Dataset):
    """Character-level next-char prediction over one text file (reference char_dataset.py:127-180)."""

    def __init__(self, text: str, block_size: int, chars: list[str] | None = None):
        self.chars = chars or sorted(set(text))
        self.stoi = {c: i for i, c in enumerate(self.chars)}
        self.itos = dict(enumerate(self.chars))
        self.block_size = block_size
        self.data = torch.tensor([self.stoi[c] for c in text if c in self.stoi], dtype=torch.long)

    @property
    def vocab_size(self) -> int:
        return len(self.chars)

    def __len__(self) -> int:
        return max(0, len(self.data) - self.block_size - 1)

    def __getitem__(self, i: int):
        chunk = self.data[i: i + self.block_size + 1]
        return chunk[:-1], chunk[1:]


@dataclass
class Snapshot:
    model_state: dict
    optimizer_state: dict
    finished_epoch: int


def load_text(path: str, truncate: float) -> str:
    if not os.path.exists(path):  # no network: synthesise a deterministic corpus
        words = ["alpha", "beta", "gamma", "delta", "epsilon", "zeta", "eta", "theta", "the", "of", "and"]
        g = torch.Generator().manual_seed(0)
        idx = torch.randint(0, len(words), (20000,), generator=g).tolist()
        text = " ".join(words[i] for i in idx)
    else:
        with open(path) as f:
            text = f.read()
    return text[: max(1, int(len(text) * truncate))] if 0 < truncate < 1 else text


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default=os.path.join(os.path.dirname(__file__), "gpt2_train_cfg.yaml"))
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--max_iters", type=int, default=None)
    ap.add_argument("--max_epochs", type=int, default=None)
    ap.add_argument("--snapshot_path", default=None)
    args = ap.parse_args(argv)
    with open(args.config) as f:
        cfg = yaml.safe_load(f)
    dc, gc, tc, oc = cfg["data_config"], cfg["gpt_config"], cfg["trainer_config"], cfg["optimizer_config"]
    if args.max_epochs is not None:
        tc["max_epochs"] = args.max_epochs
    if args.snapshot_path is not None:
        tc["snapshot_path"] = args.snapshot_path
    max_iters = args.max_iters or tc.get("max_iters")

    rank, local_rank, world = init_dist(use_cpu=args.cpu)
    device = torch.device("cuda", local_rank) if torch.cuda.is_available() and not args.cpu else torch.device("cpu")
    torch.manual_seed(1234)

    text = load_text(os.path.join(ROOT, dc["path"]) if not os.path.isabs(dc["path"]) else dc["path"], dc["truncate"])
    full = CharDataset(text, dc["block_size"])
    n_train = int(len(full.data) * dc["train_split"])
    train = CharDataset(text[:n_train], dc["block_size"], full.chars)
    test = CharDataset(text[n_train:], dc["block_size"], full.chars)
    model = GPT(GPTConfig(vocab_size=full.vocab_size, block_size=dc["block_size"], **gc)).to(device)
    ddp = DataParallel(model, bucket_size=1 << 20, expose_grads=True)
    opt = model.configure_optimizers(oc["weight_decay"], oc["learning_rate"], (0.9, 0.95), device.type)

    start_epoch = 0
    snap = tc.get("snapshot_path")
    if snap and os.path.exists(snap):
        s = torch.load(snap, map_location="cpu", weights_only=True)
        model.load_state_dict(s["model_state"])
        opt.load_state_dict(s["optimizer_state"])
        start_epoch = int(s["finished_epoch"])
        if rank == 0:
            print(f"resumed from {snap} at epoch {start_epoch}", flush=True)

    sampler = DistributedSampler(train, num_replicas=world, rank=rank, shuffle=True)
    loader = DataLoader(train, batch_size=tc["batch_size"], sampler=sampler, num_workers=tc["data_loader_workers"])
    use_amp = tc.get("use_amp", False) and device.type == "cuda"
    it = 0
    last = None
    for epoch in range(start_epoch, tc["max_epochs"]):
        sampler.set_epoch(epoch)
        model.train()
        for x, y in loader:
            x, y = x.to(device), y.to(device)
            ddp.zero_grad()
            with torch.autocast(device.type, dtype=torch.bfloat16, enabled=use_amp):
                _, loss = ddp(x, y)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(model.parameters(), tc["grad_norm_clip"])
            opt.step()
            it += 1
            last = loss.detach()
            if rank == 0 and it % 20 == 0:
                print(f"[GPU{rank}] Epoch {epoch} | Iter {it} | Train Loss {last.item():.5f}", flush=True)
            if max_iters and it >= max_iters:
                break
        if snap and rank == 0 and (epoch + 1) % tc["save_every"] == 0:
            os.makedirs(os.path.dirname(snap) or ".", exist_ok=True)
            torch.save({"model_state": model.state_dict(), "optimizer_state": opt.state_dict(),
                        "finished_epoch": epoch + 1}, snap)
        if max_iters and it >= max_iters:
            break
    # evaluation on the held-out split
    model.eval()
    with torch.no_grad():
        tl = DataLoader(test, batch_size=tc["batch_size"])
        losses = []
        for i, (x, y) in enumerate(tl):
            losses.append(model(x.to(device), y.to(device))[1].float())
            if i >= 4:
                break
        val = torch.stack(losses).mean() if losses else torch.tensor(float("nan"))
        C.all_reduce(val, op="mean")
    if rank == 0:
        print(f"final train loss {float(last) if last is not None else float('nan'):.4f} val loss {val.item():.4f}",
              flush=True)
    cleanup_dist()
    return 0


if __name__ == "__main__":
    sys.exit(main())
