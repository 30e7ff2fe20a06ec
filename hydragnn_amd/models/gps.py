"""GPS layer: local MPNN + global multi-head attention + MLP (reference
``hydragnn/globalAtt/gps.py:32-159``).

    h_loc = BN1(dropout(conv(x)) + x)
    h_att = BN2(dropout(MHA(x)) + x)          (MHA over the attention scope)
    out   = BN3((h_loc + h_att) + MLP(h_loc + h_att)),  MLP = Lin(F,2F)-act-drop-Lin(2F,F)-drop

Attention runs on the HIP flash kernel (``ops/attention.py``).  Parameter
names follow ``torch.nn.MultiheadAttention`` (``attn.in_proj_weight``,
``attn.in_proj_bias``, ``attn.out_proj.*``) and PyG ``BatchNorm``
(``norm1.module.*``) so state dicts keep the reference layout.
"""
import math
import os

import torch
import torch.nn.functional as F
from torch import nn

from ..ops.attention import segment_attention
from ..ops.linear import ACT_RELU, linear
from ..ops.norm import norm_add
from ..ops.rng import dropout as rng_dropout, new_salt
from ..ops.streams import Fork

_GPS_FORK = os.environ.get("HYDRA_GPS_FORK", "1") == "1"  # attention branch on a side stream
from .layers import BatchNorm, Linear


class MultiheadAttention(nn.Module):
    def __init__(self, embed_dim, num_heads, bias=True):
        super().__init__()
        assert embed_dim % num_heads == 0, "hidden_dim must be divisible by global_attn_heads"
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.in_proj_bias = nn.Parameter(torch.empty(3 * embed_dim)) if bias else None
        self.out_proj = Linear(embed_dim, embed_dim, bias=bias)
        self._reset_parameters()

    def _reset_parameters(self):
        nn.init.xavier_uniform_(self.in_proj_weight)
        if self.in_proj_bias is not None:
            nn.init.zeros_(self.in_proj_bias)
            nn.init.zeros_(self.out_proj.bias)

    def forward(self, x, seg_id, seg_ptr):
        qkv = linear(x, self.in_proj_weight, self.in_proj_bias)
        o = segment_attention(qkv, self.num_heads, seg_id, seg_ptr)
        return self.out_proj(o)


class PerformerAttention(nn.Module):
    """Linear-complexity FAVOR+ attention (``attn_type="performer"``, gps.py:62-67).

    Random-feature softmax-kernel approximation restricted to the same
    segments as the exact kernel (segment sums via CSR ops).
    """

    def __init__(self, channels, heads, head_channels=64, kernel=None, qkv_bias=False, attn_out_bias=True,
                 dropout=0.0, num_features=None):
        super().__init__()
        self.heads = heads
        self.head_channels = head_channels
        inner = heads * head_channels
        self.q = Linear(channels, inner, bias=qkv_bias)
        self.k = Linear(channels, inner, bias=qkv_bias)
        self.v = Linear(channels, inner, bias=qkv_bias)
        self.attn_out = Linear(inner, channels, bias=attn_out_bias)
        m = num_features or max(1, int(head_channels * math.log(head_channels)))
        self.register_buffer("proj", torch.randn(m, head_channels))

    def forward(self, x, seg_id, seg_ptr):
        from ..ops import segment as seg

        N = x.shape[0]
        H, D = self.heads, self.head_channels
        q = self.q(x).view(N, H, D) * D ** -0.25
        k = self.k(x).view(N, H, D) * D ** -0.25
        v = self.v(x).view(N, H, D)

        def phi(t):
            proj = t @ self.proj.t()
            return torch.exp(proj - t.pow(2).sum(-1, keepdim=True) / 2) / math.sqrt(self.proj.shape[0])

        qf, kf = phi(q), phi(k)  # [N, H, M]
        S = int(seg_ptr.numel() - 1)
        si = seg.SegIndex(seg_id, seg_ptr, None, S)
        kv = seg.segment_sum((kf.unsqueeze(-1) * v.unsqueeze(-2)).reshape(N, -1), si).view(S, H, -1, D)
        ksum = seg.segment_sum(kf.reshape(N, -1), si).view(S, H, -1)
        kv_n = seg.gather(kv.reshape(S, -1), si).view(N, H, -1, D)
        ks_n = seg.gather(ksum.reshape(S, -1), si).view(N, H, -1)
        num = torch.einsum("nhm,nhmd->nhd", qf, kv_n)
        den = (qf * ks_n).sum(-1, keepdim=True) + 1e-6
        return self.attn_out((num / den).reshape(N, H * D))


class GPSConv(nn.Module):
    def __init__(self, channels, conv, heads=1, dropout=0.0, act="relu", attn_type="multihead", norm=True):
        super().__init__()
        self.channels = channels
        self.conv = conv
        self.heads = heads
        self.dropout = dropout
        self.attn_type = attn_type or "multihead"
        if self.attn_type == "multihead":
            self.attn = MultiheadAttention(channels, heads)
        elif self.attn_type == "performer":
            self.attn = PerformerAttention(channels, heads)
        else:
            raise ValueError(f"{attn_type} is not supported")
        self.mlp = nn.Sequential(
            Linear(channels, channels * 2),
            nn.ReLU() if act == "relu" else act,
            nn.Dropout(dropout),
            Linear(channels * 2, channels),
            nn.Dropout(dropout),
        )
        self.norm1 = BatchNorm(channels) if norm else None
        self.norm2 = BatchNorm(channels) if norm else None
        self.norm3 = BatchNorm(channels) if norm else None

        # dropout call-site ids for the counter-hash dropout (ops/rng.py)
        self._salts = [new_salt() for _ in range(4)]

    def forward(self, inv, equiv, ctx):
        nv = ctx.get("num_valid")
        tr = self.training
        hs = []
        # the attention branch runs on a side stream, concurrently with the local MPNN
        # (forward AND backward; ops/streams.py)
        with Fork(inv, ctx.attn_seg_id, ctx.attn_seg_ptr, enable=_GPS_FORK) as fork:
            h = self.attn(inv, ctx.attn_seg_id, ctx.attn_seg_ptr)
            h_att = norm_add(h, self.norm2, nv, residual=inv, p=self.dropout, salt=self._salts[1], training=tr)
        if self.conv is not None:
            h, equiv = self.conv(inv, equiv, ctx)
            # BN1(dropout(h) + x): one fused launch each way on the GPU
            hs.append(norm_add(h, self.norm1, nv, residual=inv, p=self.dropout, salt=self._salts[0], training=tr))
        hs.append(fork.join(h_att))
        out = hs[0] if len(hs) == 1 else hs[0] + hs[1]
        lin1, act, _, lin2, _ = self.mlp
        if isinstance(act, nn.ReLU):  # bias + ReLU in the GEMM epilogue
            h = linear(out, lin1.weight, lin1.bias, act=ACT_RELU)
        else:
            h = act(lin1(out))
        m = rng_dropout(h, self.dropout, tr, self._salts[2])
        out = norm_add(lin2(m), self.norm3, nv, residual=out, p=self.dropout, salt=self._salts[3], training=tr)
        return out, equiv

    def __repr__(self):
        return f"GPSConv({self.channels}, conv={self.conv}, heads={self.heads}, attn_type={self.attn_type})"
