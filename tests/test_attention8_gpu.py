"""MFMA attention for 8-wide heads (``csrc/attention8.hip``) against a float64 torch
reference of the same segment-masked multi-head softmax attention: forward output and
the gradients of q, k and v, for batch scope (one segment plus a padding segment) and
graph scope (many small segments), at row counts that are and are not multiples of 16
for the single-launch v2 kernels (splits <= 0: in-workgroup key/query split, one-pass
deferred-rescale softmax; variants -1..-4 are other (row tiles, waves) shapes) and for
forced grid split counts (splits > 0: the combine and partial-sum paths)."""
import math

import pytest
import torch

from hydragnn_amd import _native
from hydragnn_amd.ops.attention import attention_reference, make_segments

pytestmark = pytest.mark.gpu


def _segments(N, scope, dev):
    if scope == "batch":
        return make_segments(N, "batch", num_valid=N - N // 9, device=dev)
    sizes, ptr = [], [0]
    g = torch.Generator().manual_seed(N)
    while ptr[-1] < N:
        ptr.append(min(N, ptr[-1] + int(torch.randint(5, 90, (1,), generator=g))))
    return make_segments(N, "graph", ptr=torch.tensor(ptr), device=dev)


@pytest.mark.parametrize("N", [37, 300, 2560])
@pytest.mark.parametrize("scope", ["batch", "graph"])
@pytest.mark.parametrize("splits", [0, -2, -3, -5, -8, 1, 3])
def test_attn8_matches_reference(N, scope, splits):
    torch.manual_seed(N + splits)
    dev = torch.device("cuda")
    H = 8
    ops = _native.ops()
    qkv = (torch.randn(N, 24 * H, device=dev) * 1.5).contiguous()
    sid, sptr = _segments(N, scope, dev)
    sc = 1.0 / math.sqrt(8)
    Qp, Qq, Kp, Kq, Vp, Vq = ops.attn8_pack(qkv, H)
    O, L2 = ops.attn8_fwd(Qp, Kp, Vq, sid, sptr, N, sc, splits)
    x = qkv.double().cpu().requires_grad_()
    ref = attention_reference(x, H, sid.cpu(), sc)
    torch.testing.assert_close(O.double().cpu(), ref.detach(), rtol=2e-5, atol=2e-5)
    dO = torch.randn(N, 8 * H, device=dev)
    ref.backward(dO.double().cpu())
    dqkv = ops.attn8_bwd(dO, O, L2, Qp, Qq, Kp, Kq, Vp, sid, sptr, sc, splits)
    torch.testing.assert_close(dqkv.double().cpu(), x.grad, rtol=1e-4, atol=1e-4)


def test_attn8_v2_large_scores_rescale():
    """Scores that grow along the key order force the deferred-rescale path many times
    (every row's reference moves by > 8 log2 units several times within one wave's slice)."""
    torch.manual_seed(7)
    dev = torch.device("cuda")
    N, H = 700, 8
    ops = _native.ops()
    qkv = torch.randn(N, 24 * H, device=dev)
    ramp = torch.linspace(0.0, 12.0, N, device=dev).unsqueeze(1)
    qkv[:, 8 * H:16 * H] *= ramp  # keys grow with their index
    qkv[:, :8 * H] = qkv[:, :8 * H].abs() + 1.0
    qkv[:, 8 * H:16 * H] = qkv[:, 8 * H:16 * H].abs()
    sid, sptr = make_segments(N, "batch", num_valid=N - 3, device=dev)
    sc = 1.0 / math.sqrt(8)
    Qp, Qq, Kp, Kq, Vp, Vq = ops.attn8_pack(qkv, H)
    O, L2 = ops.attn8_fwd(Qp, Kp, Vq, sid, sptr, N, sc, 0)
    x = qkv.double().cpu().requires_grad_()
    ref = attention_reference(x, H, sid.cpu(), sc)
    torch.testing.assert_close(O.double().cpu(), ref.detach(), rtol=2e-5, atol=2e-5)
    dO = torch.randn(N, 8 * H, device=dev)
    ref.backward(dO.double().cpu())
    dqkv = ops.attn8_bwd(dO, O, L2, Qp, Qq, Kp, Kq, Vp, sid, sptr, sc, 0)
    torch.testing.assert_close(dqkv.double().cpu(), x.grad, rtol=1e-4, atol=2e-4)


@pytest.mark.parametrize("N", [37, 300, 2560])
@pytest.mark.parametrize("scope", ["batch", "graph"])
def test_attn8_bf16_mfma_close_to_reference(N, scope):
    """bf16 MFMA mode of the v2 kernels (precision "bf16": operands rounded to bf16, fp32
    accumulate and softmax): forward output and q / k / v gradients within bf16 rounding of
    the float64 reference (relative to each tensor's scale)."""
    torch.manual_seed(N + 7)
    dev = torch.device("cuda")
    H = 8
    ops = _native.ops()
    qkv = (torch.randn(N, 24 * H, device=dev) * 1.5).contiguous()
    sid, sptr = _segments(N, scope, dev)
    sc = 1.0 / math.sqrt(8)
    Qp, Qq, Kp, Kq, Vp, Vq = ops.attn8_pack(qkv, H)
    O, L2 = ops.attn8_fwd(Qp, Kp, Vq, sid, sptr, N, sc, 0, True)
    x = qkv.double().cpu().requires_grad_()
    ref = attention_reference(x, H, sid.cpu(), sc)
    err = (O.double().cpu() - ref.detach()).abs().max().item()
    assert err < 3e-2 * ref.abs().max().item(), err
    dO = torch.randn(N, 8 * H, device=dev)
    ref.backward(dO.double().cpu())
    # the packed backward operands (-delta, dO in the pair / quad layouts), as gf_att_bwd writes them
    Nq = Qp.shape[1]
    dOp, dOq = ops.attn8_pack(torch.cat([dO, dO, dO], 1).contiguous(), H)[:2]
    nd = torch.zeros(H, Nq, device=dev)
    nd[:, :N] = -(dO * O).view(N, H, 8).sum(-1).t()
    dqkv = ops.attn8_bwd_packed(nd, dOp, dOq, L2, Qp, Qq, Kp, Kq, Vp, sid, sptr, N, sc, True)
    g = x.grad
    for blk in range(3):
        a, b = dqkv[:, blk * 8 * H:(blk + 1) * 8 * H].double().cpu(), g[:, blk * 8 * H:(blk + 1) * 8 * H]
        err = (a - b).abs().max().item()
        assert err < 4e-2 * b.abs().max().item(), (blk, err, b.abs().max().item())
    # the fp32 mode of the same packed entry point matches the reference tightly
    O32, L32 = ops.attn8_fwd(Qp, Kp, Vq, sid, sptr, N, sc, 0)
    nd32 = torch.zeros(H, Nq, device=dev)
    nd32[:, :N] = -(dO * O32).view(N, H, 8).sum(-1).t()
    dq32 = ops.attn8_bwd_packed(nd32, dOp, dOq, L32, Qp, Qq, Kp, Kq, Vp, sid, sptr, N, sc)
    torch.testing.assert_close(dq32.double().cpu(), g, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("N,nv,H", [(1, 1, 1), (16, 16, 8), (33, 20, 2), (700, 700, 8), (700, 0, 1),
                                    (2311, 2311, 8), (2528, 2311, 8), (2560, 2400, 4), (4100, 3000, 8)])
def test_attn8_v3_persistent_batch_scope(N, nv, H):
    """v3 (one 16-wave workgroup per CU, units dealt by cost, wave pieces merged in LDS):
    batch-scope layouts with and without a padding segment, row counts on and off the
    16-row grid, against the float64 reference; bitwise deterministic across launches."""
    torch.manual_seed(N + nv + H)
    dev = torch.device("cuda")
    ops = _native.ops()
    qkv = (torch.randn(N, 24 * H, device=dev) * 1.5).contiguous()
    sid, sptr = make_segments(N, "batch", num_valid=nv if nv < N else None, device=dev)
    sc = 1.0 / math.sqrt(8)
    Qp, Qq, Kp, Kq, Vp, Vq = ops.attn8_pack(qkv, H)
    O, L2 = ops.attn8_fwd(Qp, Kp, Vq, sid, sptr, N, sc, 0)
    O2, L22 = ops.attn8_fwd(Qp, Kp, Vq, sid, sptr, N, sc, 0)
    assert torch.equal(O, O2) and torch.equal(L2, L22)
    Nq = Qp.shape[1]
    if Nq > N:
        assert torch.all(L2[:, N:] == 0)
    x = qkv.double().cpu().requires_grad_()
    ref = attention_reference(x, H, sid.cpu(), sc)
    torch.testing.assert_close(O.double().cpu(), ref.detach(), rtol=2e-5, atol=2e-5)
    dO = torch.randn(N, 8 * H, device=dev)
    ref.backward(dO.double().cpu())
    dqkv = ops.attn8_bwd(dO, O, L2, Qp, Qq, Kp, Kq, Vp, sid, sptr, sc, 0)
    dqkv2 = ops.attn8_bwd(dO, O, L2, Qp, Qq, Kp, Kq, Vp, sid, sptr, sc, 0)
    assert torch.equal(dqkv, dqkv2)
    torch.testing.assert_close(dqkv.double().cpu(), x.grad, rtol=1e-4, atol=1e-4)
