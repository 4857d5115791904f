#!/usr/bin/env python3
"""ImageNet-style ResNet training with DDP (reference:
examples/torch_examples/imagenet/dist_train.py -- torchvision ResNet, DDP,
``--dummy`` data, top-1/top-5 meters).

torchvision is not installed here, so the ResNet family is defined below
(BasicBlock / Bottleneck, resnet18 ... resnet101).  On MI355X: one rank per
GPU, bf16 autocast, channels_last (MIOpen NHWC kernels), gradients reduced by
torch DDP or by scaletorch_amd's arena DataParallel (``--dp arena``).

  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/imagenet/resnet_ddp.py --arch resnet50 --dummy
  torchrun --nproc-per-node 2 --master-addr 127.0.0.1 examples/imagenet/resnet_ddp.py --cpu --arch resnet18 \
      --dummy --image-size 64 --steps 4
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


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, c, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, c, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(c)
        self.conv2 = nn.Conv2d(c, c, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(c)
        self.down = None
        if stride != 1 or cin != c:
            self.down = nn.Sequential(nn.Conv2d(cin, c, 1, stride, bias=False), nn.BatchNorm2d(c))

    def forward(self, x):
        idt = x if self.down is None else self.down(x)
        y = F.relu(self.bn1(self.conv1(x)))
        return F.relu(self.bn2(self.conv2(y)) + idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, c, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, c, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(c)
        self.conv2 = nn.Conv2d(c, c, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(c)
        self.conv3 = nn.Conv2d(c, 4 * c, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(4 * c)
        nn.init.zeros_(self.bn3.weight)  # zero-init residual branch
        self.down = None
        if stride != 1 or cin != 4 * c:
            self.down = nn.Sequential(nn.Conv2d(cin, 4 * c, 1, stride, bias=False), nn.BatchNorm2d(4 * c))

    def forward(self, x):
        idt = x if self.down is None else self.down(x)
        y = F.relu(self.bn1(self.conv1(x)))
        y = F.relu(self.bn2(self.conv2(y)))
        return F.relu(self.bn3(self.conv3(y)) + idt)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
                                  nn.MaxPool2d(3, 2, 1))
        cin, stages = 64, []
        for i, n in enumerate(layers):
            c = 64 * 2 ** i
            blocks = []
            for j in range(n):
                blocks.append(block(cin, c, 2 if (j == 0 and i > 0) else 1))
                cin = c * block.expansion
            stages.append(nn.Sequential(*blocks))
        self.stages = nn.Sequential(*stages)
        self.fc = nn.Linear(cin, num_classes)

    def forward(self, x):
        x = self.stages(self.stem(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


ARCHS = {"resnet18": (BasicBlock, [2, 2, 2, 2]), "resnet34": (BasicBlock, [3, 4, 6, 3]),
         "resnet50": (Bottleneck, [3, 4, 6, 3]), "resnet101": (Bottleneck, [3, 4, 23, 3])}


def accuracy(logits, y, ks=(1, 5)):
    top = logits.topk(max(ks), 1).indices
    hit = top.eq(y[:, None])
    return [hit[:, :k].any(1).float().mean().item() * 100 for k in ks]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet50", choices=sorted(ARCHS))
    ap.add_argument("--batch-size", type=int, default=128, help="per rank")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--dummy", action="store_true", help="synthetic images (no dataset needed)")
    ap.add_argument("--dp", default="ddp", choices=["ddp", "arena"])
    ap.add_argument("--cpu", action="store_true")
    return ap.parse_args(argv)


def main(argv=None) -> dict:
    args = parse(argv)
    from scaletorch_amd.dist.launch import init_dist
    from scaletorch_amd.parallel.data_parallel import DataParallel

    rank, local_rank, world = init_dist(backend="gloo" if args.cpu else None, use_cpu=args.cpu)
    gpu = torch.cuda.is_available() and not args.cpu
    dev = torch.device("cuda", local_rank) if gpu else torch.device("cpu")
    if not args.dummy:
        raise SystemExit("no ImageNet here: pass --dummy (synthetic data)")
    torch.manual_seed(0)
    block, layers = ARCHS[args.arch]
    model = ResNet(block, layers, args.classes).to(dev)
    if gpu:
        model = model.to(memory_format=torch.channels_last)
    if world > 1:
        model = (nn.SyncBatchNorm.convert_sync_batchnorm(model) if gpu else model)
        if args.dp == "arena":
            model = DataParallel(model, bucket_size=32 << 20, expose_grads=True)
        else:
            model = nn.parallel.DistributedDataParallel(model, device_ids=[local_rank] if gpu else None)
    opt = torch.optim.SGD(model.parameters(), lr=args.lr * world * args.batch_size / 256, momentum=0.9,
                          weight_decay=1e-4)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=max(1, args.steps))
    g = torch.Generator().manual_seed(100 + rank)
    # a fixed synthetic batch pool (class-dependent mean) so the loss can actually fall
    means = torch.randn(args.classes, 3, 1, 1, generator=torch.Generator().manual_seed(5))
    t0, imgs = time.perf_counter(), 0
    for step in range(args.steps):
        y = torch.randint(0, args.classes, (args.batch_size,), generator=g)
        x = means[y] + torch.randn(args.batch_size, 3, args.image_size, args.image_size, generator=g)
        x, y = x.to(dev, non_blocking=True), y.to(dev, non_blocking=True)
        if gpu:
            x = x.contiguous(memory_format=torch.channels_last)
        if args.dp == "arena" and world > 1:
            model.zero_grad()
        opt.zero_grad(set_to_none=True)
        with torch.autocast(dev.type, dtype=torch.bfloat16, enabled=gpu):
            logits = model(x)
            loss = F.cross_entropy(logits.float(), y)
        loss.backward()
        opt.step()
        sched.step()
        imgs += args.batch_size * world
        if rank == 0 and (step % 10 == 0 or step == args.steps - 1):
            top1, top5 = accuracy(logits.float(), y)
            print(f"step {step} loss {loss.item():.4f} acc@1 {top1:.1f} acc@5 {top5:.1f}", flush=True)
    if gpu:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if rank == 0:
        print(f"{args.arch} {world} ranks: {imgs / dt:.1f} images/s", flush=True)
    return {"loss": float(loss.item()), "images_per_s": imgs / dt}


if __name__ == "__main__":
    main()
    if dist.is_initialized():
        dist.destroy_process_group()
