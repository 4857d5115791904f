"""Fused chunked LM head + cross-entropy (ops/fused_head.py) against the plain
fp32 ``F.cross_entropy(x @ W^T)`` reference: loss, dX and dW, with chunking,
ignored rows, an upstream gradient scale and the DP ``main_grad`` accumulation."""
import pytest
import torch
import torch.nn.functional as F

from scaletorch_amd.ops.fused_head import fused_linear_cross_entropy


def _ref(x, w, t, ignore=-100):
    x = x.detach().float().requires_grad_(True)
    w = w.detach().float().requires_grad_(True)
    loss = F.cross_entropy(x @ w.t(), t, ignore_index=ignore)
    return loss, x, w


@pytest.mark.parametrize("chunk", [7, 16, 1000])
def test_fused_head_matches_reference(chunk):
    torch.manual_seed(0)
    N, h, V = 37, 24, 50
    x = torch.randn(N, h, requires_grad=True)
    w = torch.randn(V, h, requires_grad=True)
    t = torch.randint(0, V, (N,))
    t[3] = -100
    t[20] = -100
    loss = fused_linear_cross_entropy(x, w, t, chunk=chunk)
    (loss * 0.25).backward()
    rl, rx, rw = _ref(x, w, t)
    (rl * 0.25).backward()
    assert torch.allclose(loss, rl, rtol=1e-5, atol=1e-5)
    assert torch.allclose(x.grad, rx.grad, rtol=1e-4, atol=1e-6)
    assert torch.allclose(w.grad, rw.grad, rtol=1e-4, atol=1e-6)


def test_fused_head_vocab_shards_sum_to_full():
    """Vocab-parallel pieces (shard + vocab_start) combine to the full-vocab loss:
    each shard's target logit is 0 unless the target falls inside it."""
    from scaletorch_amd.ops import fused_head as fh

    torch.manual_seed(1)
    N, h, V = 12, 8, 20
    x, w = torch.randn(N, h), torch.randn(V, h)
    t = torch.randint(0, V, (N,))
    parts = []
    for r in range(2):
        lse, tl = fh._chunk_stats(x @ w[10 * r:10 * (r + 1)].t(), t, 10 * r, native=False)
        parts.append((lse, tl))
    lse = torch.logsumexp(torch.stack([p[0] for p in parts]), 0)
    tl = parts[0][1] + parts[1][1]
    assert torch.allclose((lse - tl).mean(), F.cross_entropy(x @ w.t(), t), atol=1e-5)


def test_fused_head_main_grad_accumulates():
    """Arena mode: dW lands in ``main_grad`` (fresh -> overwritten, then accumulated)
    scaled by the upstream gradient, and autograd sees no .grad."""
    torch.manual_seed(2)
    N, h, V = 16, 8, 32
    x = torch.randn(N, h, requires_grad=True)
    w = torch.nn.Parameter(torch.randn(V, h))
    w.main_grad = torch.full((V, h), 123.0)
    w._st_fresh = True
    seen = []
    w._st_grad_ready = lambda p: seen.append(p)
    t = torch.randint(0, V, (N,))
    (fused_linear_cross_entropy(x, w, t, chunk=5) / 2).backward()
    (fused_linear_cross_entropy(x, w, t, chunk=5) / 2).backward()
    rl, rx, rw = _ref(x, w, t)
    rl.backward()
    assert w.grad is None
    assert torch.allclose(w.main_grad, rw.grad, rtol=1e-4, atol=1e-6)
    assert len(seen) == 2


def test_fused_head_no_grad_is_loss_only():
    torch.manual_seed(3)
    x, w = torch.randn(9, 4), torch.randn(6, 4)
    t = torch.randint(0, 6, (9,))
    with torch.no_grad():
        loss = fused_linear_cross_entropy(x, w, t, chunk=4)
    assert torch.allclose(loss, F.cross_entropy(x @ w.t(), t), atol=1e-6)


def test_model_fused_head_equals_logits_path():
    """Transformer(labels=...) returns the same loss and gradients as logits + CE."""
    from scaletorch_amd.models import TransformerLM, get_model_config

    torch.manual_seed(4)
    cfg = get_model_config("tiny-llama")
    m = TransformerLM(cfg)
    ids = torch.randint(0, cfg.vocab_size, (2, 16))
    tgt = torch.randint(0, cfg.vocab_size, (2, 16))
    loss = m(input_ids=ids, labels=tgt, lm_head_chunk=10)
    loss.backward()
    g1 = {n: p.grad.clone() for n, p in m.named_parameters()}
    m.zero_grad()
    ref = F.cross_entropy(m(input_ids=ids).float().flatten(0, 1), tgt.flatten())
    ref.backward()
    assert torch.allclose(loss, ref, rtol=1e-5, atol=1e-5)
    for n, p in m.named_parameters():
        assert torch.allclose(g1[n], p.grad, rtol=1e-3, atol=1e-5), n


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [256, 4096])
def test_fused_head_gpu_native(chunk):
    """HIP path (csrc/xent.hip in place, TN dgrad on the W^T copy, fp32 wgrad GEMM)
    against the fp32 reference on bf16 inputs; arena mode (main_grad) included."""
    from scaletorch_amd.ops import _lib
    from scaletorch_amd.ops.grad import bump_weight_epoch

    assert _lib.load(), _lib.load_error()
    torch.manual_seed(5)
    N, h, V = 1000, 256, 32000
    x = (torch.randn(N, h, device="cuda") * 0.5).bfloat16().requires_grad_(True)
    w = torch.nn.Parameter((torch.randn(V, h, device="cuda") * 0.05).bfloat16())
    w.main_grad = torch.zeros(V, h, device="cuda")
    w._st_fresh = True
    bump_weight_epoch()
    t = torch.randint(0, V, (N,), device="cuda")
    t[::7] = -100
    loss = fused_linear_cross_entropy(x, w, t, chunk=chunk)
    (loss / 4).backward()
    rl, rx, rw = _ref(x, w, t)
    (rl / 4).backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - rl.item()) < 2e-3 * rl.item()
    rel = lambda a, b: ((a.float() - b).norm() / b.norm()).item()  # noqa: E731
    assert rel(x.grad, rx.grad) < 1e-2
    assert rel(w.main_grad, rw.grad) < 1e-2


def test_fused_head_direct_main_grad_mode():
    """grad_scale (the trainer's 1/GA): dW is written into main_grad during the
    forward, pre-scaled; the promised upstream gradient gives the exact result, a
    different one still yields the exact dX and is reported by check_grad_scale."""
    from scaletorch_amd.ops import fused_head as fh

    torch.manual_seed(6)
    N, h, V = 20, 8, 40
    w = torch.nn.Parameter(torch.randn(V, h))
    t = torch.randint(0, V, (N,))
    fh._SCALE_MISMATCH.clear()
    w.main_grad = torch.full((V, h), 9.0)
    w._st_fresh = True
    xs = [torch.randn(N, h, requires_grad=True) for _ in range(2)]
    for x in xs:
        (fused_linear_cross_entropy(x, w, t, chunk=7, grad_scale=0.5) * 0.5).backward()
    ref_w = torch.zeros(V, h)
    for x in xs:
        rl, rx, rw = _ref(x, w, t)
        (rl * 0.5).backward()
        ref_w += rw.grad
        assert torch.allclose(x.grad, rx.grad, rtol=1e-4, atol=1e-6)
    assert w.grad is None
    assert torch.allclose(w.main_grad, ref_w, rtol=1e-4, atol=1e-6)
    fh.check_grad_scale()  # promise kept: no error
    x = torch.randn(N, h, requires_grad=True)
    (fused_linear_cross_entropy(x, w, t, grad_scale=0.5) * 0.25).backward()
    rl, rx, _ = _ref(x, w, t)
    (rl * 0.25).backward()
    assert torch.allclose(x.grad, rx.grad, rtol=1e-4, atol=1e-6)
    with pytest.raises(RuntimeError, match="grad_scale"):
        fh.check_grad_scale()
    fh._SCALE_MISMATCH.clear()
