#!/usr/bin/env python3
"""Load / forward / backward sanity for every registered model family.

Reference: tools/verify_qwen3.py:28-97 (build Qwen3 0.6B-8B, forward + backward,
finite loss).  Here for any registry name (Llama 2/3/3.1/3.2, Qwen3 dense and
MoE, Mixtral, tiny-*), with the layer count optionally cut for speed:

  * parameter count of the built model == the analytic count of its config;
  * initial loss ~ ln(V) (random init predicts ~uniformly);
  * every trainable parameter receives a finite, non-zero gradient;
  * reference-layout state dict (q_proj/k_proj/v_proj, gate_proj/up_proj,
    experts.N.*) round-trips through load_reference_state_dict bit-exactly.

  python tools/verify_model.py --models llama3-8b,qwen3-8b,qwen3-30b-a3b --layers 2
  python tools/verify_model.py --models tiny-llama,tiny-qwen3,tiny-moe,tiny-mixtral --device cpu
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def verify(name: str, layers: int | None, device: str, seq: int = 128, batch: int = 2) -> dict:
    import torch

    from scaletorch_amd.models import build_model, get_model_config
    from scaletorch_amd.ops import cross_entropy

    cfg = get_model_config(name, num_hidden_layers=layers)
    dev = torch.device(device)
    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    torch.manual_seed(0)
    with torch.device(dev):
        prev = torch.get_default_dtype()
        torch.set_default_dtype(dtype)
        try:
            model = build_model(cfg)
        finally:
            torch.set_default_dtype(prev)
    model.cos, model.sin = model.cos.float(), model.sin.float()
    n_built = sum(p.numel() for p in model.parameters())
    n_cfg = cfg.num_params()
    ids = torch.randint(0, cfg.vocab_size, (batch, seq + 1), device=dev)
    pos = torch.arange(seq, device=dev).expand(batch, seq)
    logits = model(input_ids=ids[:, :-1], position_ids=pos)
    loss = cross_entropy(logits, ids[:, 1:].contiguous())
    aux = model.aux_loss() if cfg.is_moe else None
    total = loss + (aux if aux is not None else 0)
    total.backward()
    lnv = math.log(cfg.vocab_size)
    no_grad = [n for n, p in model.named_parameters() if p.requires_grad and (p.grad is None)]
    bad_grad = [n for n, p in model.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
    zero_grad = [n for n, p in model.named_parameters() if p.grad is not None and p.grad.abs().sum() == 0]
    ref = {k: v.detach().clone() for k, v in model.reference_state_dict().items()}
    names = sorted(ref)
    has_ref_names = any("q_proj" in k for k in names) and any(("gate_proj" in k) for k in names)
    before = {k: v.clone() for k, v in model.state_dict().items()}
    with torch.no_grad():
        for p in model.parameters():
            p.zero_()
    model.load_reference_state_dict(ref, strict=False)
    after = model.state_dict()
    roundtrip = all(torch.equal(before[k], after[k]) for k in before if k in after)
    res = {
        "model": name, "layers": cfg.num_hidden_layers, "device": device, "dtype": str(dtype).split(".")[-1],
        "params_built": n_built, "params_config": n_cfg, "params_match": n_built == n_cfg,
        "loss": round(float(loss.detach()), 4), "ln_vocab": round(lnv, 4), "loss_near_ln_vocab": abs(float(loss.detach()) - lnv) < 0.15 * lnv,
        "aux_loss": None if aux is None else round(float(aux), 5),
        "params_without_grad": no_grad, "non_finite_grads": bad_grad, "zero_grads": zero_grad[:5],
        "reference_names": has_ref_names, "reference_roundtrip": roundtrip,
    }
    res["ok"] = bool(res["params_match"] and res["loss_near_ln_vocab"] and not no_grad and not bad_grad
                     and has_ref_names and roundtrip)
    return res


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="tiny-llama,tiny-qwen3,tiny-moe,tiny-mixtral")
    ap.add_argument("--layers", type=int, default=None, help="override num_hidden_layers (speed)")
    ap.add_argument("--device", default=None)
    ap.add_argument("--seq", type=int, default=128)
    args = ap.parse_args()
    import torch

    device = args.device or ("cuda" if torch.cuda.is_available() else "cpu")
    ok = True
    for m in args.models.split(","):
        r = verify(m, args.layers, device, args.seq)
        ok &= r["ok"]
        print(json.dumps(r), flush=True)
        if device == "cuda":
            torch.cuda.empty_cache()
    print("ALL OK" if ok else "FAILURES")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
