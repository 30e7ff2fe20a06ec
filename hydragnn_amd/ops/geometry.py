"""Edge geometry and radial bases (reference ``hydragnn/utils/model/operations.py:21-36``,
PyG DimeNet ``BesselBasisLayer``/``Envelope``, SchNet ``GaussianSmearing``,
PAINN ``sinc_expansion``/``cosine_cutoff`` (``PAINNStack.py:322-343``)).

All functions are composed of differentiable torch ops on gathered rows so
that forces (double backward through positions) work; gathers use the CSR
segment ops so their backward is deterministic.
"""
import math

import torch

from . import segment as seg


def edge_vectors_and_lengths(pos, dst_si, src_si, shifts=None, normalize=False, eps=1e-9):
    """vec = pos[receiver] - pos[sender] + shift (receiver = edge_index[1])."""
    vec = seg.gather(pos, dst_si) - seg.gather(pos, src_si)
    if shifts is not None:
        vec = vec + shifts
    length = torch.linalg.vector_norm(vec, dim=-1, keepdim=True)
    if normalize:
        vec = vec / (length + eps)
    return vec, length


def get_edge_vectors_and_lengths(positions, edge_index, shifts, normalize=False, eps=1e-9):
    """Index-based variant with the reference signature."""
    sender, receiver = edge_index[0], edge_index[1]
    vec = positions[receiver] - positions[sender] + shifts
    length = torch.linalg.vector_norm(vec, dim=-1, keepdim=True)
    if normalize:
        vec = vec / (length + eps)
    return vec, length


class Envelope(torch.nn.Module):
    """DimeNet polynomial envelope u(d) with exponent p+1."""

    def __init__(self, exponent):
        super().__init__()
        self.p = exponent + 1
        self.a = -(self.p + 1) * (self.p + 2) / 2
        self.b = self.p * (self.p + 2)
        self.c = -self.p * (self.p + 1) / 2

    def forward(self, x):
        p, a, b, c = self.p, self.a, self.b, self.c
        x_p0 = x.pow(p - 1)
        x_p1 = x_p0 * x
        x_p2 = x_p1 * x
        return (1.0 / x + a * x_p0 + b * x_p1 + c * x_p2) * (x < 1.0).to(x.dtype)


class BesselBasis(torch.nn.Module):
    """rbf_k(d) = u(d/c) * sin(k*pi*d/c) with learnable frequencies (PyG BesselBasisLayer)."""

    def __init__(self, num_radial, cutoff=5.0, envelope_exponent=5):
        super().__init__()
        self.cutoff = float(cutoff)
        self.envelope = Envelope(envelope_exponent)
        self.freq = torch.nn.Parameter(torch.empty(num_radial))
        self.reset_parameters()

    def reset_parameters(self):
        with torch.no_grad():
            self.freq.copy_(torch.arange(1, self.freq.numel() + 1, dtype=torch.float32) * math.pi)

    def forward(self, dist):
        d = dist.unsqueeze(-1) / self.cutoff
        return self.envelope(d) * torch.sin(self.freq * d)


class _EdgeBasis(torch.autograd.Function):
    """One-launch radial bases (csrc/edge_basis.hip); first derivative native, higher orders
    via the composite path (``composite_mode``)."""

    @staticmethod
    def forward(ctx, d, off, K, kind, a, b, masked):
        from .. import _native

        ctx.save_for_backward(d, off)
        ctx.cfg = (K, kind, a, b, masked)
        return _native.ops().edge_basis_fwd(d, off, K, kind, a, b, masked)

    @staticmethod
    def backward(ctx, g):
        from .. import _native

        d, off = ctx.saved_tensors
        K, kind, a, b, masked = ctx.cfg
        dd = _native.ops().edge_basis_bwd(g, d, off, K, kind, a, b, masked).view(d.shape)
        return dd, None, None, None, None, None, None


def _basis_native(d):
    from .pna import fused

    return d.is_cuda and d.dtype == torch.float32 and fused("radial")


class GaussianSmearing(torch.nn.Module):
    def __init__(self, start=0.0, stop=5.0, num_gaussians=50):
        super().__init__()
        offset = torch.linspace(start, stop, num_gaussians)
        self.coeff = -0.5 / (offset[1] - offset[0]).item() ** 2 if num_gaussians > 1 else -0.5
        self.register_buffer("offset", offset)

    def forward(self, dist):
        if _basis_native(dist) and self.offset.dtype == torch.float32:
            return _EdgeBasis.apply(dist.reshape(-1), self.offset, self.offset.numel(), 0, float(self.coeff), 0.0,
                                    False)
        dist = dist.view(-1, 1) - self.offset.view(1, -1)
        return torch.exp(self.coeff * dist.pow(2))


def sinc_expansion(edge_dist, edge_size, cutoff):
    """sin(n*pi*d/c)/d, n=1..edge_size (PAINN)."""
    if _basis_native(edge_dist) and edge_dist.dim() == 1:
        return _EdgeBasis.apply(edge_dist, None, int(edge_size), 1, math.pi / cutoff, 0.0, False)
    n = torch.arange(edge_size, device=edge_dist.device, dtype=edge_dist.dtype) + 1
    return torch.sin(edge_dist.unsqueeze(-1) * n * math.pi / cutoff) / edge_dist.unsqueeze(-1)


def cosine_cutoff(edge_dist, cutoff, masked=True):
    """0.5 (cos(pi d / c) + 1), zero beyond the cutoff when ``masked`` (PAINN); SchNet's
    CFConv uses the unmasked form."""
    if _basis_native(edge_dist):
        return _EdgeBasis.apply(edge_dist.reshape(-1), None, 1, 2, math.pi / cutoff, float(cutoff),
                                bool(masked)).view(edge_dist.shape)
    if not masked:
        return 0.5 * (torch.cos(edge_dist * math.pi / cutoff) + 1.0)
    return torch.where(edge_dist < cutoff, 0.5 * (torch.cos(math.pi * edge_dist / cutoff) + 1),
                       torch.zeros_like(edge_dist))
