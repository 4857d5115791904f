"""Numerics of every HIP kernel vs a plain PyTorch fp32 reference of the same op (GPU only)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from scaletorch_amd import ops  # noqa: E402
from scaletorch_amd.ops import _lib  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _native():
    assert _lib.load(), f"HIP kernel library not loaded: {_lib.load_error()}"


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("h", [256, 4096, 5120])
@pytest.mark.parametrize("with_res", [False, True])
def test_rmsnorm(h, with_res):
    torch.manual_seed(0)
    x = torch.randn(3, 77, h, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn_like(x, requires_grad=True) if with_res else None
    w = (1 + 0.1 * torch.randn(h, device="cuda")).to(torch.bfloat16).requires_grad_(True)
    if with_res:
        y, s = ops.add_rms_norm(x, r, w, 1e-5)
        gy, gs = torch.randn_like(y), torch.randn_like(s)
        (y.float() * gy.float()).sum().add((s.float() * gs.float()).sum()).backward()
    else:
        y = ops.rms_norm(x, w, 1e-5)
        gy = torch.randn_like(y)
        (y.float() * gy.float()).sum().backward()
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True) if with_res else None
    sr = xr + rr if with_res else xr
    yr = sr * torch.rsqrt(sr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    loss = (yr * gy.float()).sum()
    if with_res:
        loss = loss + (sr * gs.float()).sum()
    loss.backward()
    assert rel(y, yr) < 1e-2
    assert rel(x.grad, xr.grad) < 2e-2
    assert rel(w.grad, wr.grad) < 2e-2
    if with_res:
        assert rel(r.grad, rr.grad) < 2e-2


def test_rmsnorm_dweight_bitwise_repeatable():
    """The dweight column sum has no atomics (csrc/rmsnorm.hip colsum_kernel): many
    rows (256 partial blocks) give bitwise-identical weight gradients run to run."""
    torch.manual_seed(0)
    h = 4096
    x = torch.randn(8192, h, device="cuda", dtype=torch.bfloat16)
    w = (1 + 0.1 * torch.randn(h, device="cuda")).to(torch.bfloat16)
    gy = torch.randn(8192, h, device="cuda", dtype=torch.bfloat16)
    grads = []
    for _ in range(3):
        wi = w.clone().requires_grad_(True)
        y = ops.rms_norm(x, wi, 1e-5)
        y.backward(gy)
        grads.append(wi.grad.clone())
    wr = w.float().requires_grad_(True)
    xf = x.float()
    (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * wr).backward(gy.float())
    assert rel(grads[0], wr.grad) < 2e-2
    assert torch.equal(grads[0], grads[1]) and torch.equal(grads[0], grads[2])


@pytest.mark.parametrize("D", [64, 128])
def test_rope_inplace(D):
    torch.manual_seed(0)
    B, S, NH = 2, 100, 6
    cos, sin = ops.rope_tables(512, D, 10000.0, device="cuda")
    base = torch.randn(B, S, NH + 3, D, device="cuda", dtype=torch.bfloat16)
    x = base.clone()
    view = x[:, :, :NH]
    pos = torch.randint(0, 512, (B, S), device="cuda")
    _lib.ops().rope_(view, cos, sin, pos, 0, False)
    ref = ops.apply_rope_ref(base[:, :, :NH].float(), cos, sin, pos).float()
    assert rel(view, ref) < 1e-2
    assert torch.equal(x[:, :, NH:], base[:, :, NH:])  # untouched tail
    _lib.ops().rope_(view, cos, sin, pos, 0, True)  # inverse
    assert rel(view, base[:, :, :NH]) < 1e-2


def test_host_pointer_rejected_before_launch():
    """A CPU tensor handed to a kernel must raise on the host, never reach the device."""
    cos, sin = ops.rope_tables(64, 64, 10000.0, device="cpu")
    x = torch.randn(1, 8, 2, 64, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        _lib.ops().rope_(x, cos, sin, None, 0, False)
    with pytest.raises(RuntimeError):
        _lib.ops().xent_fwd(torch.randn(4, 64, device="cuda", dtype=torch.bfloat16), torch.zeros(4, dtype=torch.long), 0)


@pytest.mark.parametrize("I", [384, 8 * 1100])  # one-vector and two-vector-per-lane paths, ragged tail
def test_swiglu(I):
    torch.manual_seed(0)
    gu = torch.randn(5, 33, 2 * I, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    y = ops.swiglu(gu)
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    gr = gu.detach().float().requires_grad_(True)
    a, b = gr.chunk(2, -1)
    yr = torch.nn.functional.silu(a) * b
    (yr * g.float()).sum().backward()
    assert rel(y, yr) < 1e-2
    assert rel(gu.grad, gr.grad) < 2e-2


def test_adamw_and_sumsq():
    torch.manual_seed(0)
    n = 4096 * 33
    master = torch.randn(n, device="cuda")
    m, v = torch.randn(n, device="cuda") * 0.01, torch.rand(n, device="cuda") * 0.01
    g = torch.randn(n, device="cuda")
    p = master.to(torch.bfloat16)
    clip = torch.tensor([0.5], device="cuda")
    mr, vr, wr = m.clone(), v.clone(), master.clone()
    lr, b1, b2, eps, wd, t = 1e-3, 0.9, 0.95, 1e-8, 0.1, 7
    _lib.ops().adamw_step_(master, m, v, g, p, clip, lr, b1, b2, eps, wd, t)
    gg = g * 0.5
    mr.mul_(b1).add_(gg, alpha=1 - b1)
    vr.mul_(b2).addcmul_(gg, gg, value=1 - b2)
    wr.mul_(1 - lr * wd)
    wr.addcdiv_(mr / (1 - b1 ** t), (vr / (1 - b2 ** t)).sqrt() + eps, value=-lr)
    assert rel(m, mr) < 1e-6 and rel(v, vr) < 1e-6
    assert (master - wr).abs().max().item() < 1e-6
    assert rel(p, wr) < 1e-2
    out = torch.zeros(1, device="cuda")
    _lib.ops().sumsq_(g, out)
    assert abs(out.item() - g.double().pow(2).sum().item()) / g.double().pow(2).sum().item() < 1e-5
    gb = g.to(torch.bfloat16)
    out.zero_()
    _lib.ops().sumsq_(gb, out)
    ref = gb.double().pow(2).sum().item()
    assert abs(out.item() - ref) / ref < 1e-5


def test_adamw_bf16_moments():
    """bf16 exp_avg / exp_avg_sq (optimizer_state_dtype="bf16"): fp32 math on the
    widened moments, the update uses the unrounded fp32 moments, one STOCHASTIC bf16
    rounding per stored moment (csrc/adamw.hip sr_bf16) -- checked against an fp32
    PyTorch reference and the bit-exact torch mirror (optim.sr_round_bf16)."""
    from scaletorch_amd.optim import sr_key, sr_offsets, sr_round_bf16

    torch.manual_seed(0)
    n = 4096 * 33 + 8
    master = torch.randn(n, device="cuda")
    m = (torch.randn(n, device="cuda") * 0.01).to(torch.bfloat16)
    v = (torch.rand(n, device="cuda") * 0.01).to(torch.bfloat16)
    g = torch.randn(n, device="cuda")
    p = master.to(torch.bfloat16)
    mr, vr, wr = m.float(), v.float(), master.clone()
    lr, b1, b2, eps, wd, t = 1e-3, 0.9, 0.95, 1e-8, 0.1, 3
    _lib.ops().adamw_step_(master, m, v, g, p, None, lr, b1, b2, eps, wd, t)
    mr.mul_(b1).add_(g, alpha=1 - b1)
    vr.mul_(b2).addcmul_(g, g, value=1 - b2)
    wr.mul_(1 - lr * wd)
    wr.addcdiv_(mr / (1 - b1 ** t), (vr / (1 - b2 ** t)).sqrt() + eps, value=-lr)
    # one stochastic rounding: |err| < 1 ulp = 2^-7 |x| (+ slack for the fp32 fma-vs-mul/add
    # order where b1*m and (1-b1)*g nearly cancel); almost every element equals the mirror's
    offsets = sr_offsets(n, sr_key(t), 0, "cuda")
    for which, (got, want) in enumerate(((m, mr), (v, vr))):
        err = (got.float() - want).abs()
        assert err.le(want.abs() * 2 ** -7 + 1e-7).all(), (err - want.abs() * 2 ** -7).max().item()
        mirror = sr_round_bf16(want, offsets[which])
        assert (got == mirror).float().mean().item() > 0.99
    assert (master - wr).abs().max().item() < 1e-6
    assert rel(p, wr) < 1e-2


def test_adamw_bf16_second_moment_tracks_fp32_over_2000_steps():
    """The kernel's bf16 exp_avg_sq at beta2 = 0.999 over 2,000 steps of a unit-variance
    gradient stream stays within 2 % (mean over elements) of the fp32-moment kernel's:
    stochastic rounding keeps it unbiased where nearest rounding stalled."""
    n = 1 << 16
    gen = torch.Generator(device="cuda").manual_seed(11)
    st = {}
    for sd in (torch.float32, torch.bfloat16):
        st[sd] = [torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda", dtype=sd),
                  torch.zeros(n, device="cuda", dtype=sd)]
    for t in range(1, 2001):
        g = torch.randn(n, device="cuda", generator=gen)
        for sd, (w, m, v) in st.items():
            _lib.ops().adamw_step_(w, m, v, g, None, None, 1e-4, 0.9, 0.999, 1e-8, 0.0, t)
    v32, v16 = st[torch.float32][2], st[torch.bfloat16][2].float()
    assert abs(v16.mean().item() / v32.mean().item() - 1) < 0.02
    assert ((v16 - v32).abs() / v32).median().item() < 0.04
    m32, m16 = st[torch.float32][1], st[torch.bfloat16][1].float()
    assert (m16 - m32).abs().mean().item() < 0.02 * m32.abs().mean().item()


@pytest.mark.parametrize("sd", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("RC", [(192, 320), (1024, 64)])
def test_adamw_wt_matches_flat_update_and_transpose(sd, RC):
    """The fused AdamW + W^T pass (csrc/adamw.hip adamw_wt_kernel) == the flat AdamW
    kernel followed by a transpose, bitwise (same per-element math), for fp32 and bf16
    moments, a non-square weight and a one-tile-wide one."""
    torch.manual_seed(0)
    R, C = RC
    n = R * C
    master = torch.randn(n, device="cuda")
    m = (torch.randn(n, device="cuda") * 0.01).to(sd)
    v = (torch.rand(n, device="cuda") * 0.01).to(sd)
    g = torch.randn(n, device="cuda")
    p = master.to(torch.bfloat16).view(R, C)
    wt = torch.empty(C, R, device="cuda", dtype=torch.bfloat16)
    clip = torch.tensor([0.7], device="cuda")
    ref = [x.clone() for x in (master, m, v, p)]
    args = (1e-3, 0.9, 0.95, 1e-8, 0.1, 5)
    _lib.ops().adamw_step_(ref[0], ref[1], ref[2], g, ref[3].view(-1), clip, *args)
    _lib.ops().adamw_wt_step_(master, m, v, g, p, wt, clip, *args)
    assert torch.equal(master, ref[0]) and torch.equal(m, ref[1]) and torch.equal(v, ref[2])
    assert torch.equal(p, ref[3])
    assert torch.equal(wt, ref[3].t())
    with pytest.raises(RuntimeError):
        _lib.ops().adamw_wt_step_(master, m, v, g, p, wt.t(), clip, *args)  # wt must be [C, R] contiguous


@pytest.mark.parametrize("V", [512, 32000])
def test_cross_entropy(V):
    torch.manual_seed(0)
    N = 300
    logits = (3 * torch.randn(N, V, device="cuda")).to(torch.bfloat16).requires_grad_(True)
    tgt = torch.randint(0, V, (N,), device="cuda")
    tgt[::17] = -100
    loss = ops.cross_entropy(logits, tgt)
    loss.backward()
    lr = logits.detach().float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(lr, tgt, ignore_index=-100)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-3 * max(1.0, ref.item())
    assert rel(logits.grad, lr.grad) < 2e-2


FLASH_CASES = [
    # B, Sq, Sk, H, Hkv, D, causal
    (2, 256, 256, 4, 4, 128, True),
    (1, 333, 333, 8, 2, 128, True),
    (2, 200, 320, 4, 1, 128, False),
    (1, 128, 128, 4, 4, 64, True),
    (2, 257, 257, 4, 2, 64, False),
    (1, 1024, 1024, 8, 2, 128, True),
    (1, 64, 1000, 4, 1, 128, True),     # short query block at the end of a long key range
    (1, 300, 300, 8, 1, 128, True),     # GQA group of 8 summed in one dK/dV workgroup
    (1, 2048, 2048, 4, 1, 64, True),
    (2, 96, 96, 2, 2, 128, False),
]


@pytest.mark.parametrize("B,Sq,Sk,H,Hkv,D,causal", FLASH_CASES)
def test_flash_fwd_bwd(B, Sq, Sk, H, Hkv, D, causal):
    # these short grids take the dK/dV query-range split (auto: up to 8 ranges, some
    # of them empty for the short query ranges)
    _flash_case(B, Sq, Sk, H, Hkv, D, causal, 1.0)


@pytest.mark.parametrize("split", ["1", "3"])
@pytest.mark.parametrize("kernel", ["DKDV", "DQ"])
@pytest.mark.parametrize("B,Sq,Sk,H,Hkv,D,causal", [FLASH_CASES[1], FLASH_CASES[2], FLASH_CASES[6], FLASH_CASES[8]])
def test_flash_bwd_split_forced(B, Sq, Sk, H, Hkv, D, causal, kernel, split, monkeypatch):
    """The dK/dV (query ranges) and dQ (key ranges) kernels unsplit -- the long-grid path --
    and cut into 3 ranges whose fp32 partials are reduced in order."""
    monkeypatch.setenv(f"ST_FLASH_{kernel}_SPLIT", split)
    _flash_case(B, Sq, Sk, H, Hkv, D, causal, 1.0)



@pytest.mark.parametrize("B,Sq,Sk,H,Hkv,D,causal", FLASH_CASES)
def test_flash_bwd_recompute_path(B, Sq, Sk, H, Hkv, D, causal, monkeypatch):
    """The dQ kernel that recomputes S / dP itself (ST_FLASH_BWD_DS=0) -- the default
    path above stores dS from the dK/dV kernel and derives dQ from it."""
    monkeypatch.setenv("ST_FLASH_BWD_DS", "0")
    _flash_case(B, Sq, Sk, H, Hkv, D, causal, 1.0)


@pytest.mark.parametrize("ds", ["0", "1"])
@pytest.mark.parametrize("q_off,k_off", [(32, 0), (0, 32), (96, 160), (300, 0), (0, 0), (1000, 0)])
def test_flash_bwd_unaligned_offsets(q_off, k_off, ds, monkeypatch):
    """Causal blocks at global offsets that are not multiples of the 64-row tiles (ring /
    zig-zag CP blocks): the dS workspace must cover every (query tile, key block) pair the
    dQ kernel reads, including query blocks the dK/dV kernel would otherwise skip."""
    monkeypatch.setenv("ST_FLASH_BWD_DS", ds)
    torch.manual_seed(0)
    B, Sq, Sk, H, Hkv, D = 1, 320, 384, 4, 2, 128
    q = torch.randn(B, Sq, H, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, Sk, Hkv, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, Sk, Hkv, D, device="cuda", dtype=torch.bfloat16)
    scale = 1 / math.sqrt(D)
    out, lse = ops.flash_attn_fwd(q, k, v, scale, True, q_off, k_off)
    dout = torch.randn_like(out)
    dq, dk, dv = ops.flash_attn_bwd(dout, q, k, v, out, lse, scale, True, q_off, k_off)
    rq, rk, rv = ops.attention.flash_bwd_ref(dout, q, k, v, out, lse, scale, True, q_off, k_off)
    assert torch.isfinite(dq.float()).all() and torch.isfinite(dk.float()).all()
    assert rel(dq, rq) < 2e-2 and rel(dk, rk) < 2e-2 and rel(dv, rv) < 2e-2


def test_flash_bwd_ds_bitwise_repeatable():
    """The dS-materialising backward has no atomics: two runs agree bitwise."""
    torch.manual_seed(0)
    B, S, H, Hkv, D = 2, 1024, 8, 2, 128
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    out, lse = ops.flash_attn_fwd(q, k, v, 1 / math.sqrt(D), True)
    dout = torch.randn_like(out)
    a = ops.flash_attn_bwd(dout, q, k, v, out, lse, 1 / math.sqrt(D), True)
    b = ops.flash_attn_bwd(dout, q, k, v, out, lse, 1 / math.sqrt(D), True)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("qscale", [6.0, 30.0])
def test_flash_large_logits(qscale):
    """Peaked softmax: exercises the deferred (thresholded) O rescale."""
    _flash_case(1, 700, 700, 4, 2, 128, True, qscale)


def _flash_case(B, Sq, Sk, H, Hkv, D, causal, qscale):
    torch.manual_seed(0)
    q = (torch.randn(B, Sq, H, D, device="cuda") * qscale).to(torch.bfloat16)
    k = torch.randn(B, Sk, Hkv, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, Sk, Hkv, D, device="cuda", dtype=torch.bfloat16)
    scale = 1 / math.sqrt(D)
    off = Sk - Sq if causal else 0  # bottom-right aligned causal when Sq != Sk
    out, lse = ops.flash_attn_fwd(q, k, v, scale, causal, off, 0)
    ref_out, ref_lse = ops.sdpa_ref(q, k, v, causal, scale, off, 0)
    assert rel(out, ref_out) < 1e-2
    assert (lse - ref_lse).abs().max().item() < 1e-2
    dout = torch.randn_like(out)
    dq, dk, dv = ops.flash_attn_bwd(dout, q, k, v, out, lse, scale, causal, off, 0)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    o2, _ = ops.attention._sdpa_fp32(qr, kr, vr, causal, scale, off, 0)
    o2.backward(dout.float())
    assert rel(dq, qr.grad) < 2e-2
    assert rel(dk, kr.grad) < 2e-2
    assert rel(dv, vr.grad) < 2e-2


def test_flash_offsets_blockwise_equals_full():
    """Ring-attention building block: attention split into K/V blocks with global
    offsets and merged by lse_merge_ equals full causal attention."""
    torch.manual_seed(0)
    B, S, H, Hkv, D = 1, 512, 4, 2, 128
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    scale = 1 / math.sqrt(D)
    full, full_lse = ops.flash_attn_fwd(q, k, v, scale, True)
    qs = q[:, 256:]  # second half of queries, global offset 256
    acc = torch.zeros(B, 256, H, D, device="cuda")
    lse = torch.full((B, H, 256), float("-inf"), device="cuda")
    for kb in range(2):
        ks, vs = k[:, kb * 256:(kb + 1) * 256], v[:, kb * 256:(kb + 1) * 256]
        bo, bl = ops.flash_attn_fwd(qs, ks, vs, scale, True, 256, kb * 256)
        _lib.ops().lse_merge_(acc, lse, bo, bl)
    assert rel(acc, full[:, 256:]) < 1e-2
    assert (lse - full_lse[:, :, 256:]).abs().max().item() < 1e-2


def test_flash_bwd_block_with_global_lse():
    """Ring-attention backward building block: one K/V block, global (merged) out/lse."""
    torch.manual_seed(0)
    B, S, H, Hkv, D = 2, 256, 4, 2, 128
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, 2 * S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, 2 * S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    scale = 1 / math.sqrt(D)
    out, lse = ops.flash_attn_fwd(q, k, v, scale, True, S, 0)  # queries at global [S, 2S)
    dout = torch.randn_like(out)
    for kb in range(2):
        ks, vs = k[:, kb * S:(kb + 1) * S], v[:, kb * S:(kb + 1) * S]
        dq, dk, dv = ops.flash_attn_bwd(dout, q, ks, vs, out, lse, scale, True, S, kb * S)
        rq, rk, rv = ops.attention.flash_bwd_ref(dout, q, ks, vs, out, lse, scale, True, S, kb * S)
        assert rel(dq, rq) < 2e-2 and rel(dk, rk) < 2e-2 and rel(dv, rv) < 2e-2


def test_rope_attention_autograd_matches_reference():
    torch.manual_seed(0)
    B, S, H, Hkv, D = 2, 192, 4, 2, 128
    cos, sin = ops.rope_tables(1024, D, 500000.0, device="cuda")
    qkv = torch.randn(B, S, (H + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    out = ops.rope_attention(qkv.clone(), cos, sin, None, H, Hkv, D)
    g = torch.randn_like(out)
    (out.float() * g.float()).sum().backward()
    gq = qkv.grad.clone()
    qkv.grad = None
    import os

    os.environ["ST_DISABLE_NATIVE"] = "1"
    try:
        qf = qkv.detach().float().requires_grad_(True)
        ref = ops.rope_attention(qf, cos, sin, None, H, Hkv, D)
        (ref * g.float()).sum().backward()
    finally:
        os.environ["ST_DISABLE_NATIVE"] = "0"
    assert rel(out, ref) < 2e-2
    assert rel(gq, qf.grad) < 3e-2


@pytest.mark.parametrize("T,E,k,renorm", [(3000, 8, 2, True), (2500, 128, 8, True), (700, 60, 4, False)])
def test_moe_router_topk(T, E, k, renorm):
    from scaletorch_amd.ops import moe

    torch.manual_seed(0)
    logits = torch.randn(T, E, device="cuda") * 2
    probs, topw, topi = moe.router_topk(logits, k, renorm)
    rp, rw, ri = moe._router_ref(logits, k, renorm)
    assert torch.allclose(probs, rp, atol=1e-6, rtol=1e-5)
    assert torch.equal(topi.long().sort(-1).values, ri.long().sort(-1).values)
    assert torch.allclose(topw, rw, atol=1e-6, rtol=1e-5)
    # gradients: topw and the aux-loss path through probs
    lg = logits.clone().requires_grad_(True)
    p, w, _ = moe.router_topk(lg, k, renorm)
    gw, gp = torch.randn_like(w), torch.randn_like(p)
    ((w * gw).sum() + (p * gp).sum()).backward()
    lr = logits.clone().requires_grad_(True)
    p2, w2, _ = moe._router_ref(lr, k, renorm)
    ((w2 * gw).sum() + (p2 * gp).sum()).backward()
    assert rel(lg.grad, lr.grad) < 1e-5


@pytest.mark.parametrize("T,E,k,h", [(3000, 8, 2, 256), (1500, 128, 8, 512), (5, 64, 4, 64)])
def test_moe_permute_gather_combine(T, E, k, h):
    from scaletorch_amd.ops import moe

    torch.manual_seed(0)
    topi = torch.randint(0, E, (T, k), device="cuda", dtype=torch.int32)
    perm = moe.permutation(topi, E)
    order = torch.argsort(topi.reshape(-1).long(), stable=True)
    assert torch.equal(perm.sorted_entry.long(), order)
    assert torch.equal(perm.counts.long(), torch.bincount(topi.reshape(-1).long(), minlength=E))
    assert torch.equal(perm.pos.long()[order], torch.arange(T * k, device="cuda"))
    x = torch.randn(T, h, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    xs = moe.gather_rows(x, perm)
    assert torch.equal(xs, x.detach().index_select(0, order // k))
    w = torch.rand(T, k, device="cuda", requires_grad=True)
    y = (xs.float() * 1.5).to(torch.bfloat16)  # an "expert"
    out = moe.combine(y, w, perm)
    ref_y = y.detach().float().requires_grad_(True)
    ref_w = w.detach().clone().requires_grad_(True)
    ref = (ref_y.index_select(0, perm.pos.long()).view(T, k, h) * ref_w.unsqueeze(-1)).sum(1)
    assert rel(out, ref) < 1e-2
    g = torch.randn(T, h, device="cuda", dtype=torch.bfloat16)
    out.backward(g)
    ref.backward(g.float())
    assert rel(w.grad, ref_w.grad) < 1e-2
    # dx: every token receives sum over its slots of 1.5 * w * g
    exp_dx = 1.5 * (ref_w.detach().sum(-1, keepdim=True) * g.float())
    assert rel(x.grad, exp_dx) < 2e-2


@pytest.mark.parametrize("bn", ["auto", "128", "256"])
@pytest.mark.parametrize("T,M,N,beta", [(64, 256, 256, 0), (512, 512, 768, 1), (1024, 768, 512, 0), (96, 256, 512, 1),
                                        (160, 512, 384, 1)])
def test_wgrad_gemm(T, M, N, beta, bn, monkeypatch):
    if bn != "auto":
        monkeypatch.setenv("ST_WGRAD_BN", bn)
    """dW (+)= dY^T X with token-major operands (csrc/wgrad_gemm.hip) vs fp32 reference;
    strided operands (column slices of wider activations) and asymmetric data."""
    torch.manual_seed(0)
    dy_full = torch.randn(T, M + 64, device="cuda", dtype=torch.bfloat16)
    x_full = torch.randn(T, N + 128, device="cuda", dtype=torch.bfloat16)
    dy, x = dy_full[:, 32: 32 + M], x_full[:, 64: 64 + N]
    ramp = torch.arange(M, device="cuda", dtype=torch.float32)[:, None] * 1e-3
    out = torch.randn(M, N, device="cuda") + ramp
    ref = dy.float().t() @ x.float() + (out if beta else 0)
    if bn == "256" and N % 256:
        assert not _lib.ops().wgrad_gemm_(out, dy, x, beta)
        return
    assert _lib.ops().wgrad_gemm_(out, dy, x, beta)
    torch.cuda.synchronize()
    assert rel(out, ref) < 1e-5


@pytest.mark.parametrize("T,M,N,beta", [(64, 256, 256, 0), (192, 512, 768, 1), (4096, 512, 1024, 1), (1024, 768, 512, 0)])
def test_wgrad_gemm_8phase(T, M, N, beta, monkeypatch):
    """The 8-phase 256x256 kernel (ST_WGRAD_P8=1): single, odd (tail) and long K-tile
    counts, strided operands, beta = 0/1, vs the fp32 reference."""
    monkeypatch.setenv("ST_WGRAD_P8", "1")
    torch.manual_seed(1)
    dy_full = torch.randn(T, M + 64, device="cuda", dtype=torch.bfloat16)
    x_full = torch.randn(T, N + 128, device="cuda", dtype=torch.bfloat16)
    dy, x = dy_full[:, 32: 32 + M], x_full[:, 64: 64 + N]
    ramp = torch.arange(N, device="cuda", dtype=torch.float32)[None, :] * 1e-3
    out = torch.randn(M, N, device="cuda") + ramp
    ref = dy.float().t() @ x.float() + (out if beta else 0)
    assert _lib.ops().wgrad_gemm_(out, dy, x, beta)
    torch.cuda.synchronize()
    assert rel(out, ref) < 1e-5


@pytest.mark.parametrize("variant,bn", [(1, "256"), (1, "128"), (2, "auto")])
@pytest.mark.parametrize("split", ["auto", "2", "4"])
@pytest.mark.parametrize("T,M,N,beta", [(512, 6144, 4096, 1), (256, 4096, 1792 * 2, 0), (512, 512, 1024, 1)])
def test_wgrad_gemm_tail_split(T, M, N, beta, split, variant, bn, monkeypatch):
    """Tail split (csrc/wgrad_gemm.hip): whole tiles for the full rounds of 256 CUs, the
    last partial round cut into token ranges whose fp32 partials are added in order --
    qkv-like 384 tiles (256 whole + 128 split), down-like 896, and a sub-round grid;
    vs the fp32 reference, and bitwise repeatable."""
    if split != "auto":
        monkeypatch.setenv("ST_WGRAD_SPLIT", split)
    if bn != "auto":
        monkeypatch.setenv("ST_WGRAD_BN", bn)
    torch.manual_seed(2)
    dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    ramp = torch.arange(N, device="cuda", dtype=torch.float32)[None, :] * 1e-3
    out0 = torch.randn(M, N, device="cuda") + ramp
    ref = dy.float().t() @ x.float() + (out0 if beta else 0)
    outs = []
    for _ in range(2):
        out = out0.clone()
        assert _lib.ops().wgrad_gemm_(out, dy, x, beta, variant)
        outs.append(out)
    torch.cuda.synchronize()
    assert rel(outs[0], ref) < 1e-5
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("split", ["1", "auto"])
@pytest.mark.parametrize("T,M,N", [(512, 4096, 4352), (512, 6144, 4096), (256, 512, 1024), (1024, 256, 256),
                                   (256, 768, 1280)])
def test_wgrad4_matches_fp32(T, M, N, split, monkeypatch):
    """csrc/wgrad4.hip (variant 6): persistent one-wave-per-SIMD tiles, several per workgroup;
    qkv-like 384 tiles (the last 128 split along K, the partials of ranges 1.. added in order by
    the tail reduce), sub-round grids; beta 0 over garbage then beta 1 accumulate, on a strided
    (ldc > N) output as well; bitwise repeatable."""
    if split != "auto":
        monkeypatch.setenv("ST_WGRAD4_SPLIT", split)
    torch.manual_seed(4)
    dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    ref = dy.float().t() @ x.float()
    for ldc in (N, N + 256):
        big = torch.full((M, ldc), 7.0, device="cuda")
        out = big[:, :N]
        assert _lib.ops().wgrad_gemm_(out, dy, x, 0, 6)
        torch.cuda.synchronize()
        assert rel(out, ref) < 1e-5
        assert _lib.ops().wgrad_gemm_(out, dy, x, 1, 6)
        torch.cuda.synchronize()
        assert rel(out, 2 * ref) < 1e-5
        if ldc > N:
            assert torch.all(big[:, N:] == 7.0)
        again = torch.zeros(M, N, device="cuda")
        assert _lib.ops().wgrad_gemm_(again, dy, x, 0, 6)
        assert _lib.ops().wgrad_gemm_(again, dy, x, 1, 6)
        assert torch.equal(again, out)


@pytest.mark.parametrize("variant", [1, 2, 6])
@pytest.mark.parametrize("T", [1, 37, 100, 1000, 2047, 2100])
def test_wgrad_gemm_ragged_tokens(T, variant):
    """Token counts that are not a multiple of the K-tile (MoE experts): the last tile's
    rows past T come from the buffer descriptor's zero fill; strided operands, beta = 1."""
    torch.manual_seed(3)
    M, N = 512, 768 if variant == 1 else 512
    dy = torch.randn(T, M + 64, device="cuda", dtype=torch.bfloat16)[:, 32: 32 + M]
    x = torch.randn(T, N + 128, device="cuda", dtype=torch.bfloat16)[:, 64: 64 + N]
    out = torch.randn(M, N, device="cuda")
    ref = dy.float().t() @ x.float() + out
    assert _lib.ops().wgrad_gemm_(out, dy, x, 1, variant)
    torch.cuda.synchronize()
    assert rel(out, ref) < 1e-5


def test_wgrad_gemm_unsupported_shape_declines():
    dy = torch.randn(64, 200, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(64, 192, device="cuda", dtype=torch.bfloat16)
    out = torch.zeros(200, 192, device="cuda")
    assert not _lib.ops().wgrad_gemm_(out, dy, x, 0)
    assert out.abs().sum().item() == 0


@pytest.mark.parametrize("D,with_pos", [(128, False), (128, True), (64, True)])
def test_qknorm_rope_attention_matches_unfused(D, with_pos):
    """Fused per-head QK-norm + RoPE + flash attention (csrc/qknorm_rope.hip) vs the
    fp32 reference chain (RMSNorm per head -> RoPE -> SDPA): output, dQKV and both
    norm-weight gradients."""
    from scaletorch_amd.ops.attention import apply_rope_ref, rope_tables, sdpa_ref
    from scaletorch_amd.ops.norm import rms_norm_ref

    torch.manual_seed(0)
    B, S, H, Hkv = 2, 192, 4, 2
    qkv = torch.randn(B, S, (H + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16) * 2
    wq = torch.nn.Parameter(1 + 0.3 * torch.randn(D, device="cuda", dtype=torch.bfloat16))
    wk = torch.nn.Parameter(1 + 0.3 * torch.randn(D, device="cuda", dtype=torch.bfloat16))
    cos, sin = rope_tables(1024, D, 10000.0, device="cuda")
    pos = (torch.randperm(1024, device="cuda")[:S].sort().values.expand(B, S).contiguous() if with_pos else None)
    x = qkv.clone().requires_grad_(True)
    out = ops.qknorm_rope_attention(x, wq, wk, 1e-6, cos, sin, pos, H, Hkv, D)
    g = torch.randn_like(out)
    out.backward(g)
    # fp32 reference
    xr = qkv.float().clone().requires_grad_(True)
    wqr, wkr = wq.detach().float().requires_grad_(True), wk.detach().float().requires_grad_(True)
    x4 = xr.view(B, S, H + 2 * Hkv, D)
    q = rms_norm_ref(x4[:, :, :H], wqr, 1e-6)
    k = rms_norm_ref(x4[:, :, H: H + Hkv], wkr, 1e-6)
    q = apply_rope_ref(q, cos, sin, pos)
    k = apply_rope_ref(k, cos, sin, pos)
    ref = sdpa_ref(q, k, x4[:, :, H + Hkv:], True, 1.0 / math.sqrt(D))[0].reshape(B, S, H * D)
    ref.backward(g.float())
    assert rel(out, ref) < 2e-2
    assert rel(x.grad, xr.grad) < 3e-2
    assert rel(wq.grad, wqr.grad) < 3e-2 and rel(wk.grad, wkr.grad) < 3e-2


@pytest.mark.parametrize("shape", [(64, 64), (128, 192), (4096, 1024), (6144, 4096)])
def test_transpose_bf16(shape):
    from scaletorch_amd.ops import _lib

    R, C = shape
    src = torch.randn(R, C, device="cuda", dtype=torch.bfloat16)
    dst = torch.empty(C, R, device="cuda", dtype=torch.bfloat16)
    _lib.ops().transpose_(src, dst)
    assert torch.equal(dst, src.t().contiguous())


def _attn_rows_ref(q, k, v, rows, scale, q_offset=0):
    """fp32 causal attention for the query rows ``rows`` (global position q_offset + row)
    against keys [0, position]; GQA by head groups.  Returns (out [B,n,H,D], lse [B,H,n])."""
    B, _, H, D = q.shape
    g = H // k.shape[2]
    qs = q[:, rows].float()  # [B, n, H, D]
    kf = k.float().repeat_interleave(g, dim=2)
    vf = v.float().repeat_interleave(g, dim=2)
    s = torch.einsum("bnhd,bkhd->bhnk", qs, kf) * scale
    pos = torch.as_tensor(rows, device=q.device) + q_offset
    mask = torch.arange(k.shape[1], device=q.device)[None, :] > pos[:, None]
    s = s.masked_fill(mask[None, None], float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    out = torch.einsum("bhnk,bkhd->bnhd", torch.softmax(s, dim=-1), vf)
    return out, lse


@pytest.mark.parametrize("S", [4096, 8192, 32768])
@pytest.mark.parametrize("pp", ["1", "0"])
def test_flash_long_sequence_sampled_rows(S, pp, monkeypatch):
    """Long causal sequences (the bench's 4K, 8K and the CP8@32K global length):
    the kernel's output and lse on sampled query rows (start, middle, end) against
    an fp32 reference over every visible key; both forward kernels (8-wave ping-pong,
    ST_FLASH_PP=1, and the 4-wave one)."""
    monkeypatch.setenv("ST_FLASH_PP", pp)
    torch.manual_seed(0)
    B, H, Hkv, D = 1, 4, 2, 128
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    scale = 1 / math.sqrt(D)
    out, lse = ops.flash_attn_fwd(q, k, v, scale, True, 0, 0)
    for start in (0, S // 2 - 100, S - 256):
        rows = list(range(start, start + 256))
        ro, rl = _attn_rows_ref(q, k, v, rows, scale)
        assert rel(out[:, rows], ro) < 1e-2, start
        assert (lse[:, :, rows] - rl).abs().max().item() < 1e-2, start


@pytest.mark.parametrize("kernel", ["default", "pp"])
def test_flash_fwd_rescale_spikes(kernel, monkeypatch):
    """The deferred O rescale (running max grown by > 2^8 after P of earlier tiles is already
    in O) fires only on data that spikes late: key rows with 6x the norm at several positions
    deep into the sequence (cdna_hip_programming.md T13 / rule 26), vs the fp32 reference."""
    monkeypatch.setenv("ST_FLASH_PP", "1" if kernel == "pp" else "0")
    torch.manual_seed(21)
    B, S, H, Hkv, D = 2, 2048, 4, 2, 128
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    for t in (300, 301, 700, 1333, 1900):
        k[:, t] = (k[:, t].float() * 6).to(torch.bfloat16)
    scale = 1 / math.sqrt(D)
    out, lse = ops.flash_attn_fwd(q, k, v, scale, True, 0, 0)
    ref_o, ref_l = ops.sdpa_ref(q, k, v, True, scale, 0, 0)
    assert rel(out, ref_o) < 1e-2
    assert (lse - ref_l).abs().max().item() < 2e-2


@pytest.mark.parametrize("q_off", [0, 12288, 28672])
def test_flash_cp_chunk_at_global_offset(q_off):
    """The CP8@32K building block: a 4096-query chunk at global offset q_off against
    every key before it (Sk = q_off + 4096), forward AND backward, vs fp32."""
    torch.manual_seed(1)
    B, H, Hkv, D, n = 1, 4, 2, 128, 4096
    Sk = q_off + n
    q = torch.randn(B, n, H, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, Sk, Hkv, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, Sk, Hkv, D, device="cuda", dtype=torch.bfloat16)
    scale = 1 / math.sqrt(D)
    out, lse = ops.flash_attn_fwd(q, k, v, scale, True, q_off, 0)
    ref_out, ref_lse = ops.sdpa_ref(q, k, v, True, scale, q_off, 0)
    assert rel(out, ref_out) < 1e-2
    assert (lse - ref_lse).abs().max().item() < 1e-2
    dout = torch.randn_like(out)
    dq, dk, dv = ops.flash_attn_bwd(dout, q, k, v, out, lse, scale, True, q_off, 0)
    rq, rk, rv = ops.attention.flash_bwd_ref(dout, q, k, v, out, lse, scale, True, q_off, 0)
    assert rel(dq, rq) < 2e-2 and rel(dk, rk) < 2e-2 and rel(dv, rv) < 2e-2


def test_embedding_bwd_deterministic():
    """Sorted-segment embedding backward (csrc/embedding.hip): equals the fp64
    index_add reference, accumulates into existing rows, and is bitwise identical
    run to run (the atomics path it replaces is not)."""
    from scaletorch_amd.parallel.embedding import embedding

    torch.manual_seed(3)
    V, H, T = 300, 256, 5000
    w = torch.nn.Parameter(torch.randn(V, H, device="cuda").bfloat16())
    ids = torch.randint(0, V, (2, T // 2), device="cuda")
    ids[0, :400] = 7  # one long run
    dy = torch.randn(2, T // 2, H, device="cuda", dtype=torch.bfloat16)
    ref = torch.zeros(V, H, dtype=torch.float64, device="cuda").index_add_(0, ids.reshape(-1),
                                                                          dy.reshape(-1, H).double())
    outs = []
    for _ in range(2):
        w.main_grad = torch.full((V, H), 0.5, device="cuda")
        w._st_fresh = False  # accumulate into the existing 0.5
        embedding(ids, w).backward(dy)
        outs.append(w.main_grad.clone())
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    assert ((outs[0].double() - 0.5) - ref).abs().max().item() < 1e-3


@pytest.mark.gpu
def test_embedding_bwd_long_runs_and_masked_ids():
    """Long runs split across workgroups (csrc/embedding.hip): two long runs meeting
    inside one 64-position block, a pad-like run of 20K tokens, and -1 (TP out-of-shard)
    ids that must be skipped -- exact vs fp64, bitwise identical run to run."""
    from scaletorch_amd.parallel.embedding import embedding

    torch.manual_seed(5)
    V, H = 257, 512
    parts = [torch.full((3000,), -1), torch.full((101,), 3), torch.full((130,), 4), torch.randint(0, V, (777,)),
             torch.full((20000,), 0), torch.tensor([5]), torch.full((65,), 6)]
    ids = torch.cat(parts)[torch.randperm(sum(p.numel() for p in parts))].cuda().reshape(1, -1)
    T = ids.numel()
    w = torch.nn.Parameter(torch.randn(V, H, device="cuda").bfloat16())
    dy = torch.randn(1, T, H, device="cuda", dtype=torch.bfloat16)
    keep = ids.reshape(-1) >= 0
    ref = torch.zeros(V, H, dtype=torch.float64, device="cuda").index_add_(
        0, ids.reshape(-1)[keep], dy.reshape(-1, H)[keep].double())
    outs = []
    for _ in range(2):
        w.main_grad = torch.zeros(V, H, device="cuda")
        w._st_fresh = False
        embedding(ids.clamp(min=0), w, ids).backward(dy)
        outs.append(w.main_grad.clone())
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    err = (outs[0].double() - ref).abs().max().item()
    assert err < 5e-3 * max(1.0, ref.abs().max().item() / 100), err


@pytest.mark.parametrize("impl", ["wgrad4", "4stage"])
@pytest.mark.parametrize("N", [256, 384])
@pytest.mark.parametrize("beta", [0, 1])
def test_wgrad_grouped_matches_per_expert(N, beta, impl, monkeypatch):
    """One-launch grouped weight gradient (csrc/wgrad_gemm.hip st_wgrad_grouped; csrc/wgrad4.hip
    st_wgrad4_grouped where it tiles the shape, N % 256 == 0): expert row ranges from device
    offsets (empty experts, ragged counts, one > 1 K-tile), beta 0 overwrites / 1 accumulates
    (an empty expert with beta 0 is zeroed)."""
    monkeypatch.setenv("ST_WGRAD_GROUPED4", "1" if impl == "wgrad4" else "0")
    torch.manual_seed(4)
    M = 512
    counts = torch.tensor([37, 0, 300, 1, 64, 0, 1000], device="cuda", dtype=torch.int32)
    T = int(counts.sum())
    offs = torch.cumsum(counts, 0, dtype=torch.int32)
    dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    out = torch.randn(counts.numel(), M, N, device="cuda")
    ref = out.clone() if beta else torch.zeros_like(out)
    off = 0
    for e, n in enumerate(counts.tolist()):
        ref[e] += dy[off:off + n].float().t() @ x[off:off + n].float()
        off += n
    assert _lib.ops().wgrad_grouped_(out, dy, x, offs, beta)
    torch.cuda.synchronize()
    assert rel(out, ref) < 1e-5


@pytest.mark.parametrize("N,K", [(256, 512), (384, 256), (1536, 2048)])
@pytest.mark.parametrize("wn", [False, True])
def test_grouped_gemm_matches_per_expert(N, K, wn):
    """One-launch grouped expert GEMM (csrc/grouped_gemm.hip) vs an fp32 per-expert reference:
    empty experts, 1-row, ragged and > 256-row groups, both weight layouts ([G,N,K]: x w^T;
    [G,K,N]: x w), a strided x, BN 256 and 128.  Rows past the last offset stay untouched."""
    torch.manual_seed(6)
    counts = torch.tensor([37, 0, 300, 1, 256, 0, 513], device="cuda", dtype=torch.int32)
    G, T = counts.numel(), int(counts.sum())
    offs = torch.cumsum(counts, 0, dtype=torch.int32)
    xb = torch.randn(T + 5, K + 64, device="cuda", dtype=torch.bfloat16)
    x = xb[:, 32: 32 + K]
    w = torch.randn(G, K, N, device="cuda", dtype=torch.bfloat16) if wn else \
        torch.randn(G, N, K, device="cuda", dtype=torch.bfloat16)
    y = _lib.ops().grouped_gemm(x, w, offs, wn)
    torch.cuda.synchronize()
    off = 0
    for e, n in enumerate(counts.tolist()):
        ref = x[off:off + n].float() @ (w[e].float() if wn else w[e].float().t())
        if n:
            assert rel(y[off:off + n].float(), ref) < 1e-2, (e, n)
        off += n


@pytest.mark.parametrize("T,K,I", [(300, 192, 128), (1000, 1024, 384), (5000, 128, 4096)])  # last: 320 tiles, KT 2
def test_gemm_swiglu_matches_fp32(T, K, I):
    """Dense gate|up GEMM with the SwiGLU epilogue (csrc/gemm4w.hip ``st_gemm4w_swiglu``) vs
    fp32: gu = x [W_gate; W_up]^T (one bf16 rounding) and h = silu(gate) * up of the stored
    bf16 gate / up (what csrc/swiglu.hip computes from gu); partial last row tile, strided x."""
    torch.manual_seed(13)
    xb = torch.randn(T, K + 64, device="cuda", dtype=torch.bfloat16)
    x = xb[:, :K]
    w = torch.randn(2 * I, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5
    gu, h = _lib.ops().gemm_swiglu(x, w)
    torch.cuda.synchronize()
    ref = x.float() @ w.float().t()
    assert rel(gu.float(), ref) < 1e-2
    g, u = gu[:, :I].float(), gu[:, I:].float()
    assert rel(h.float(), torch.nn.functional.silu(g) * u) < 1e-2
    assert torch.equal(h, _lib.ops().swiglu_fwd(gu))


def test_gemm4w_swiglu_grouped_matches_fp32():
    """Grouped gate|up GEMM + SwiGLU epilogue on the one-wave-per-SIMD kernel (the long-K MoE
    forward, models/moe.py ``_gmm_swiglu``): per-expert fp32 references, an empty expert, a
    ragged tail, R_max padding rows untouched by the check."""
    torch.manual_seed(15)
    counts = [300, 0, 513, 77]
    G, K, I = len(counts), 4096, 256
    offs = torch.cumsum(torch.tensor(counts, device="cuda", dtype=torch.int32), 0, dtype=torch.int32)
    T = sum(counts) + 40
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(G, 2 * I, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5
    gu, h = _lib.ops().gemm4w_swiglu_grouped(x, w, offs)
    torch.cuda.synchronize()
    off = 0
    for e, n in enumerate(counts):
        if n:
            ref = x[off:off + n].float() @ w[e].float().t()
            assert rel(gu[off:off + n].float(), ref) < 1e-2, e
            assert torch.equal(h[off:off + n], _lib.ops().swiglu_fwd(gu[off:off + n].contiguous())), e
        off += n


def test_expert_ffn_gemm4w_matches_grouped():
    """_ExpertFFNFn at K 4,096 (Mixtral-like: the forward GEMMs take csrc/gemm4w.hip) equals the
    8-phase grouped-kernel path (ST_MOE_GEMM4W=0) on outputs, dx and both fp32 weight grads."""
    import os

    from scaletorch_amd.models.moe import _ExpertFFNFn

    G, K, I = 3, 4096, 256
    counts = [300, 0, 529]
    offs = torch.cumsum(torch.tensor(counts, device="cuda", dtype=torch.int32), 0, dtype=torch.int32)
    T = sum(counts) + 17
    res = {}
    for on in ("1", "0"):
        os.environ["ST_MOE_GEMM4W"] = on
        try:
            torch.manual_seed(16)
            x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16, requires_grad=True)
            w_gu = torch.nn.Parameter(torch.randn(G, 2 * I, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5)
            w_dn = torch.nn.Parameter(torch.randn(G, K, I, device="cuda", dtype=torch.bfloat16) / I ** 0.5)
            for w in (w_gu, w_dn):
                w.main_grad = torch.zeros(w.shape, device="cuda")
                w._st_fresh = True
            xin = x * 1
            xin._st_padded = True
            y = _ExpertFFNFn.apply(xin, offs, w_gu, w_dn)
            y.backward(torch.randn(y.shape, device="cuda", generator=torch.Generator("cuda").manual_seed(4)).to(y.dtype))
            v = sum(counts)
            res[on] = (y[:v].float(), x.grad[:v].float(), w_gu.main_grad.clone(), w_dn.main_grad.clone())
        finally:
            os.environ.pop("ST_MOE_GEMM4W", None)
    for a, b in zip(res["1"], res["0"]):
        assert rel(a, b) < 2e-2


def test_mlp_fused_swiglu_matches_unfused():
    """The Llama MLP with the fused gate|up + SwiGLU kernel (ops.mlp.gate_up_swiglu,
    ST_MLP_FUSED_SWIGLU=1) equals the unfused path (hipBLASLt GEMM + swiglu kernel) on the
    output, the input gradient and both fp32 main_grad weight gradients."""
    import os

    from scaletorch_amd.models.config import get_model_config
    from scaletorch_amd.models.transformer import MLP

    cfg = get_model_config("tiny-llama", hidden_size=256, intermediate_size=384)
    res = {}
    for fused in ("1", "0"):
        os.environ["ST_MLP_FUSED_SWIGLU"] = fused
        try:
            torch.manual_seed(14)
            mlp = MLP(cfg).cuda().to(torch.bfloat16)
            for p in mlp.parameters():
                p.main_grad = torch.zeros(p.shape, device="cuda")
                p._st_fresh = True
            x = torch.randn(2, 300, 256, device="cuda", dtype=torch.bfloat16, requires_grad=True)
            y = mlp(x)
            y.backward(torch.randn(y.shape, device="cuda", generator=torch.Generator("cuda").manual_seed(5)).to(y.dtype))
            torch.cuda.synchronize()
            res[fused] = (y.float(), x.grad.float(), mlp.gate_up_proj.weight.main_grad.clone(),
                          mlp.down_proj.weight.main_grad.clone())
        finally:
            os.environ.pop("ST_MLP_FUSED_SWIGLU", None)
    for a, b in zip(res["1"], res["0"]):
        assert rel(a, b) < 2e-2


@pytest.mark.parametrize("persist", ["1", "0"])
def test_gemm4w_matches_fp32(persist, monkeypatch):
    """The one-wave-per-SIMD grouped GEMM (csrc/gemm4w.hip: MoE long-K experts), persistent
    grid and one tile per workgroup, vs an fp32 per-group reference: empty / 1-row / partial /
    multi-tile groups, strided x, K = 192 (three 64-k tiles) and K = 1024."""
    monkeypatch.setenv("ST_GEMM4W_PERSIST", persist)
    kind = "5"
    torch.manual_seed(11)
    # the last case has 320 tiles: a persistent workgroup (kinds 5, 6) walks several of them
    for K, counts, N in ((192, [37, 0, 300, 1, 513], 512), (1024, [256, 700], 512), (192, [3000, 0, 1999, 1], 4096)):
        c = torch.tensor(counts, device="cuda", dtype=torch.int32)
        G, T = c.numel(), int(c.sum())
        offs = torch.cumsum(c, 0, dtype=torch.int32)
        xb = torch.randn(T, K + 64, device="cuda", dtype=torch.bfloat16)
        x = xb[:, 32:32 + K]
        w = torch.randn(G, N, K, device="cuda", dtype=torch.bfloat16)
        y = _lib.ops().gemm4w(x, w, offs)
        torch.cuda.synchronize()
        off = 0
        for e, n in enumerate(counts):
            if n:
                ref = x[off:off + n].float() @ w[e].float().t()
                assert rel(y[off:off + n].float(), ref) < 1e-2, (kind, K, e, n)
            off += n


@pytest.mark.parametrize("I,K", [(256, 512), (384, 1024)])
def test_grouped_gemm_swiglu_epilogues_match_fp32(I, K):
    """Grouped gate|up GEMM with the SwiGLU epilogue (EPI 1) and the down-projection
    data gradient with the SwiGLU-backward epilogue (EPI 2) vs fp32 per-expert references:
    gu = x [W_gate; W_up]^T, a = silu(gate) * up; dgu = [dy W_dn * up * silu'(gate) |
    dy W_dn * silu(gate)].  Empty experts, ragged / 1-row / > 256-row groups, rows past
    the last offset (R_max padding) untouched."""
    torch.manual_seed(9)
    counts = torch.tensor([37, 0, 300, 1, 256, 513], device="cuda", dtype=torch.int32)
    G, T = counts.numel(), int(counts.sum())
    offs = torch.cumsum(counts, 0, dtype=torch.int32)
    pad = 40  # R_max padding rows
    x = torch.randn(T + pad, K, device="cuda", dtype=torch.bfloat16)
    w_gu = torch.randn(G, 2 * I, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5
    w_dn = torch.randn(G, K, I, device="cuda", dtype=torch.bfloat16) / I ** 0.5
    gu, a = _lib.ops().grouped_gemm_swiglu(x, w_gu, offs)
    dy = torch.randn(T + pad, K, device="cuda", dtype=torch.bfloat16)
    dgu = _lib.ops().grouped_gemm_dswiglu(dy, w_dn, offs, gu)
    torch.cuda.synchronize()
    off = 0
    for e, n in enumerate(counts.tolist()):
        if n:
            ref_gu = x[off:off + n].float() @ w_gu[e].float().t()
            assert rel(gu[off:off + n].float(), ref_gu) < 1e-2, ("gu", e)
            g, u = ref_gu[:, :I], ref_gu[:, I:]
            assert rel(a[off:off + n].float(), torch.nn.functional.silu(g) * u) < 2e-2, ("a", e)
            gq, uq = gu[off:off + n, :I].float(), gu[off:off + n, I:].float()  # what the backward reads
            da = dy[off:off + n].float() @ w_dn[e].float()
            sg = torch.sigmoid(gq)
            ref_dg = da * uq * (sg + gq * sg * (1 - sg))
            ref_du = da * gq * sg
            assert rel(dgu[off:off + n, :I].float(), ref_dg) < 2e-2, ("dgate", e)
            assert rel(dgu[off:off + n, I:].float(), ref_du) < 2e-2, ("dup", e)
        off += n


def test_expert_ffn_fused_matches_unfused():
    """_ExpertFFNFn forward/backward with the fused SwiGLU epilogues equals the unfused
    path (GEMM + swiglu kernels) within bf16 rounding, on outputs, input gradient and
    fp32 weight gradients, for a padded (R_max) buffer with the activation recomputed."""
    import os

    from scaletorch_amd.models.moe import _ExpertFFNFn

    torch.manual_seed(10)
    G, K, I = 4, 512, 384
    counts = torch.tensor([100, 0, 257, 60], device="cuda", dtype=torch.int32)
    offs = torch.cumsum(counts, 0, dtype=torch.int32)
    T = int(counts.sum()) + 31
    res = {}
    for fused in ("1", "0"):
        os.environ["ST_MOE_FUSED_SWIGLU"] = fused
        try:
            torch.manual_seed(10)
            x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16, requires_grad=True)
            w_gu = torch.nn.Parameter(torch.randn(G, 2 * I, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5)
            w_dn = torch.nn.Parameter(torch.randn(G, K, I, device="cuda", dtype=torch.bfloat16) / I ** 0.5)
            for w in (w_gu, w_dn):
                w.main_grad = torch.zeros(w.shape, device="cuda")
                w._st_fresh = True
            xin = x * 1
            xin._st_padded = True
            y = _ExpertFFNFn.apply(xin, offs, w_gu, w_dn)
            dy = torch.randn_like(y)
            y.backward(dy)
            v = int(offs[-1])
            res[fused] = (y[:v].float(), x.grad[:v].float(), w_gu.main_grad.clone(), w_dn.main_grad.clone())
        finally:
            os.environ.pop("ST_MOE_FUSED_SWIGLU", None)
    for a, b in zip(res["1"], res["0"]):
        assert rel(a, b) < 2e-2


def test_expert_ffn_vendor_gemms_match_grouped():
    """_ExpertFFNFn with host-known counts (one hipBLASLt GEMM per expert,
    ``ST_MOE_VENDOR_GEMM``) equals the one-launch grouped-kernel path on outputs, input
    gradient and fp32 weight gradients (empty expert, ragged groups, R_max padding rows)."""
    from scaletorch_amd.models.moe import _ExpertFFNFn

    G, K, I = 4, 512, 384
    counts = [100, 0, 257, 60]
    offs = torch.cumsum(torch.tensor(counts, device="cuda", dtype=torch.int32), 0, dtype=torch.int32)
    T = sum(counts) + 31
    res = {}
    for host in (True, False):
        torch.manual_seed(12)
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        w_gu = torch.nn.Parameter(torch.randn(G, 2 * I, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5)
        w_dn = torch.nn.Parameter(torch.randn(G, K, I, device="cuda", dtype=torch.bfloat16) / I ** 0.5)
        for w in (w_gu, w_dn):
            w.main_grad = torch.zeros(w.shape, device="cuda")
            w._st_fresh = True
        xin = x * 1
        xin._st_padded = True
        y = _ExpertFFNFn.apply(xin, offs, w_gu, w_dn, counts if host else None)
        y.backward(torch.randn(y.shape, device="cuda", generator=torch.Generator("cuda").manual_seed(3)).to(y.dtype))
        v = sum(counts)
        res[host] = (y[:v].float(), x.grad[:v].float(), w_gu.main_grad.clone(), w_dn.main_grad.clone())
    for a, b in zip(res[True], res[False]):
        assert rel(a, b) < 2e-2


@pytest.mark.parametrize("wn", [False, True])
@pytest.mark.parametrize("M", [4096 + 352, 8192 + 1536, 8192 - 300])
def test_gmm_tail_split_matches_fp32(M, wn):
    """The narrow (N = 4,096) one-expert GEMM split into whole 4,096-row waves on the grouped /
    gemm4w kernel plus a hipBLASLt tail (models/moe.py ``_gmm_tail_split``) equals the fp32
    product, for a tail it splits (352, 1,536 rows) and one it leaves whole (3,796)."""
    from scaletorch_amd.models.moe import _gmm_tail_split

    torch.manual_seed(5)
    K, N = 4096, 4096  # K >= 4096: the wn=False bands run on gemm4w
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn((1, K, N) if wn else (1, N, K), device="cuda", dtype=torch.bfloat16) / K ** 0.5)
    offs = torch.tensor([M], device="cuda", dtype=torch.int32)
    y = _gmm_tail_split(x, w, offs, wn, False)
    ref = x.float() @ (w[0].float() if wn else w[0].float().t())
    assert y.shape == (M, N)
    assert rel(y.float(), ref) < 1e-2


@pytest.mark.parametrize("cp,rank", [(4, 1), (8, 3)])
def test_cp_two_phase_backward_at_zigzag_offsets(cp, rank):
    """The CP all-gather backward's two phases (parallel/context_parallel.py ``_CPAttnFn``):
    per zig-zag chunk the dK/dV kernel with the dS workspace (``flash_bwd_kv``), then, while
    the dK/dV reduce-scatter would be in flight, dQ = dS K (``flash_bwd_q_ds``) -- checked
    per chunk at the rank's global offsets against the fp32 ``flash_bwd_ref``."""
    from scaletorch_amd.parallel.context_parallel import zigzag_chunk_starts

    torch.manual_seed(0)
    S, H, Hkv, D = 128 * 2 * cp, 4, 2, 128
    a, b, c = zigzag_chunk_starts(S, cp, rank)
    kf = torch.randn(1, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    vf = torch.randn(1, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    scale = 1 / math.sqrt(D)
    for g0 in (a, b):
        q = torch.randn(1, c, H, D, device="cuda", dtype=torch.bfloat16)
        k, v = kf[:, :g0 + c], vf[:, :g0 + c]
        out, lse = ops.flash_attn_fwd(q, k, v, scale, True, g0, 0)
        dout = torch.randn_like(out)
        dk, dv, ws = _lib.ops().flash_bwd_kv(dout, q, k, v, out, lse, scale, True, g0, 0, None, None)
        if ws.numel() == 0:
            pytest.skip("the dS path did not take the CP chunk shape (one-shot backward covers it)")
        dq = torch.empty_like(q)
        _lib.ops().flash_bwd_q_ds(q, k, ws, scale, True, g0, 0, dq)
        rq, rk, rv = ops.attention.flash_bwd_ref(dout, q, k, v, out, lse, scale, True, g0, 0)
        assert rel(dq, rq) < 2e-2 and rel(dk, rk) < 2e-2 and rel(dv, rv) < 2e-2, g0
