// Fused GATv2 segment-softmax attention + aggregation (gfx950).
//
// Reference: PyG GATv2Conv as used by hydragnn/models/GATStack.py:175-205 (heads=6,
// negative_slope=0.05, add_self_loops=True).  Per destination node i and head h:
//     g_ij = xl[j] + xr[i] (+ ge_ij)          s_ij = att_h . leaky_relu(g_ij)
//     a_ij = softmax_{j in N(i) + {i}} s_ij   (self term g_ii = xl[i] + xr[i] (+ gself_i))
//     out_i = sum_j dropout(a_ij) xl[j]
// The torch composite needs ~20 launches and several [E, H*C] temporaries per layer
// (gathers, leaky_relu, head sums, segment max / exp / sum / normalise, weighted gather,
// segment sum).  Here: ONE forward launch (online softmax over the node's CSR segment,
// the self loop folded in as one extra element, no [E, *] tensor materialised) and ONE
// backward launch producing every per-edge / per-node gradient, plus one CSR
// segment-sum by source for dxl (deterministic, no atomics).
//
// Mapping: one thread per (node, head); the C channels of that head live in registers
// (register width CM = 8 / 16 / 32 >= C; wider heads use the composite path).  Edges of node i: [rowptr[i], rowptr[i+1]) in the
// by-destination CSR, src[e] = source node.  Dropout on the attention coefficients uses
// the same counter hash as ops/rng.py (element index e*H + h; self loop: i*H + h with
// salt + 1000003), so the fused and composite paths draw identical masks.
#include "common.h"
#include "dropout.h"

namespace hy {

struct GatArgs {
  const float* xl;
  const float* xr;
  const float* ge;     // [E, H*C] edge term or nullptr
  const float* gself;  // [N, H*C] self-loop edge term or nullptr
  const float* att;    // [H*C]
  const int* rowptr;   // [N+1]
  const int* src;      // [E]
  int ldl, ldr;        // row strides of xl / xr
  int N, H, C;  // C: channels per head (<= the kernel's register width CM)
  float slope;
  int self_loop;
};

__device__ __forceinline__ float lrelu(float v, float s) { return v > 0.f ? v : v * s; }

template <int CM>
__device__ __forceinline__ float gat_score(const GatArgs& a, const float* __restrict__ xlj,
                                           const float (&xr)[CM], const float* __restrict__ gext,
                                           const float (&att)[CM], float (&g)[CM]) {
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CM; ++c) {
    if (c < a.C) {
      g[c] = xlj[c] + xr[c] + (gext != nullptr ? gext[c] : 0.f);
      s = fmaf(att[c], lrelu(g[c], a.slope), s);
    }
  }
  return s;
}

// out [N, H*C], ml [N, H, 2] = (running max, sum of exp) saved for the backward
template <int CM>
__global__ void __launch_bounds__(256) gat_fwd_kernel(GatArgs a, const int64_t* __restrict__ rng, int64_t salt,
                                                      float p, float* __restrict__ out, float* __restrict__ ml) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.N * a.H) return;
  const int i = t / a.H, h = t - i * a.H;
  const int C = a.C;
  const int HC = a.H * C;
  const DropCfg d1 = drop_cfg(rng, salt, p), d2 = drop_cfg(rng, salt + 1000003, p);
  float xr[CM], att[CM], acc[CM], g[CM];
#pragma unroll
  for (int c = 0; c < CM; ++c) {
    xr[c] = c < C ? a.xr[(int64_t)i * a.ldr + h * C + c] : 0.f;
    att[c] = c < C ? a.att[h * C + c] : 0.f;
    acc[c] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  const int e0 = a.rowptr[i], e1 = a.rowptr[i + 1];
  const int total = e1 - e0 + (a.self_loop ? 1 : 0);
  for (int k = 0; k < total; ++k) {
    const bool self = k == e1 - e0;
    const int e = e0 + k;
    const int j = self ? i : a.src[e];
    const float* xlj = a.xl + (int64_t)j * a.ldl + h * C;
    const float* gext = self ? (a.gself != nullptr ? a.gself + (int64_t)i * HC + h * C : nullptr)
                             : (a.ge != nullptr ? a.ge + (int64_t)e * HC + h * C : nullptr);
    const float s = gat_score<CM>(a, xlj, xr, gext, att, g);
    if (s > m) {
      const float al = __expf(m - s);  // m = -inf -> 0
      l *= al;
#pragma unroll
      for (int c = 0; c < CM; ++c) acc[c] *= al;
      m = s;
    }
    const float pe = __expf(s - m);
    l += pe;
    float w = pe;
    if (self ? d2.on : d1.on) {
      const DropCfg& dc = self ? d2 : d1;
      const uint32_t idx = (uint32_t)((self ? (int64_t)i : (int64_t)e) * a.H + h);
      w = keep_elem(dc.seed, idx, dc.thresh) ? w * dc.scale : 0.f;
    }
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < C) acc[c] = fmaf(w, xlj[c], acc[c]);
  }
  const float inv = 1.f / (l + 1e-16f);
#pragma unroll
  for (int c = 0; c < CM; ++c)
    if (c < C) out[(int64_t)i * HC + h * C + c] = acc[c] * inv;
  ml[2 * t] = m;
  ml[2 * t + 1] = l;
}

// Backward.  For node i, head h with a_k = exp(s_k - m) / (l + 1e-16), dropout multiplier
// w_k, da_k = w_k * (dout_i . v_k), D = sum_k a_k da_k:
//   ds_k = a_k (da_k - D);  dg_k = ds_k * att (.) lrelu'(g_k)
//   P[e]      = dg_e + a_e w_e dout_i          (summed by source j -> dxl_j)
//   dge[e]    = dg_e                            (edge term)
//   dxr_i     = sum_k dg_k ;   dxl_self_i = dg_self + a_self w_self dout_i ; dgself_i = dg_self
//   datt_part[i, h] = sum_k ds_k lrelu(g_k)     (reduced over nodes afterwards)
template <int CM>
__global__ void __launch_bounds__(256) gat_bwd_kernel(GatArgs a, const int64_t* __restrict__ rng, int64_t salt,
                                                      float p, const float* __restrict__ dout,
                                                      const float* __restrict__ ml, float* __restrict__ P,
                                                      float* __restrict__ dge, float* __restrict__ dxr,
                                                      float* __restrict__ dxl_self, float* __restrict__ dgself,
                                                      float* __restrict__ datt_part) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.N * a.H) return;
  const int i = t / a.H, h = t - i * a.H;
  const int C = a.C;
  const int HC = a.H * C;
  const DropCfg d1 = drop_cfg(rng, salt, p), d2 = drop_cfg(rng, salt + 1000003, p);
  float xr[CM], att[CM], go[CM], g[CM], accr[CM], acct[CM];
#pragma unroll
  for (int c = 0; c < CM; ++c) {
    xr[c] = c < C ? a.xr[(int64_t)i * a.ldr + h * C + c] : 0.f;
    att[c] = c < C ? a.att[h * C + c] : 0.f;
    go[c] = c < C ? dout[(int64_t)i * HC + h * C + c] : 0.f;
    accr[c] = 0.f;
    acct[c] = 0.f;
  }
  const float m = ml[2 * t], inv = 1.f / (ml[2 * t + 1] + 1e-16f);
  const int e0 = a.rowptr[i], e1 = a.rowptr[i + 1];
  const int total = e1 - e0 + (a.self_loop ? 1 : 0);
  auto mult = [&](bool self, int e) {
    const DropCfg& dc = self ? d2 : d1;
    if (!dc.on) return 1.f;
    const uint32_t idx = (uint32_t)((self ? (int64_t)i : (int64_t)e) * a.H + h);
    return keep_elem(dc.seed, idx, dc.thresh) ? dc.scale : 0.f;
  };
  // pass 1: D = sum_k a_k da_k
  float D = 0.f;
  for (int k = 0; k < total; ++k) {
    const bool self = k == e1 - e0;
    const int e = e0 + k;
    const int j = self ? i : a.src[e];
    const float* xlj = a.xl + (int64_t)j * a.ldl + h * C;
    const float* gext = self ? (a.gself != nullptr ? a.gself + (int64_t)i * HC + h * C : nullptr)
                             : (a.ge != nullptr ? a.ge + (int64_t)e * HC + h * C : nullptr);
    const float s = gat_score<CM>(a, xlj, xr, gext, att, g);
    const float ak = __expf(s - m) * inv;
    float dv = 0.f;
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < C) dv = fmaf(go[c], xlj[c], dv);
    D = fmaf(ak, dv * mult(self, e), D);
  }
  // pass 2: per-element gradients
  for (int k = 0; k < total; ++k) {
    const bool self = k == e1 - e0;
    const int e = e0 + k;
    const int j = self ? i : a.src[e];
    const float* xlj = a.xl + (int64_t)j * a.ldl + h * C;
    const float* gext = self ? (a.gself != nullptr ? a.gself + (int64_t)i * HC + h * C : nullptr)
                             : (a.ge != nullptr ? a.ge + (int64_t)e * HC + h * C : nullptr);
    const float s = gat_score<CM>(a, xlj, xr, gext, att, g);
    const float ak = __expf(s - m) * inv;
    const float wk = mult(self, e);
    float dv = 0.f;
#pragma unroll
    for (int c = 0; c < CM; ++c)
      if (c < C) dv = fmaf(go[c], xlj[c], dv);
    const float ds = ak * (dv * wk - D);
    const float aw = ak * wk;
    float* pr = self ? dxl_self + (int64_t)i * HC + h * C : P + (int64_t)e * HC + h * C;
    float* gr = self ? (dgself != nullptr ? dgself + (int64_t)i * HC + h * C : nullptr)
                     : (dge != nullptr ? dge + (int64_t)e * HC + h * C : nullptr);
#pragma unroll
    for (int c = 0; c < CM; ++c) {
      if (c >= C) continue;
      const float lr = lrelu(g[c], a.slope);
      const float dg = ds * att[c] * (g[c] > 0.f ? 1.f : a.slope);
      accr[c] += dg;
      acct[c] = fmaf(ds, lr, acct[c]);
      pr[c] = dg + aw * go[c];
      if (gr != nullptr) gr[c] = dg;
    }
  }
  if (!a.self_loop) {
    for (int c = 0; c < C; ++c) dxl_self[(int64_t)i * HC + h * C + c] = 0.f;
  }
#pragma unroll
  for (int c = 0; c < CM; ++c) {
    if (c < C) {
      dxr[(int64_t)i * HC + h * C + c] = accr[c];
      datt_part[(int64_t)i * HC + h * C + c] = acct[c];
    }
  }
}

static GatArgs gat_args(const at::Tensor& xl, const at::Tensor& xr, const c10::optional<at::Tensor>& ge,
                        const c10::optional<at::Tensor>& gself, const at::Tensor& att, const at::Tensor& rowptr,
                        const at::Tensor& src, int64_t H, double slope, bool self_loop, int C) {
  HY_CHECK_CUDA(xl);
  HY_CHECK_F32(xl);
  HY_CHECK_F32(xr);
  HY_CHECK_I32(rowptr);
  HY_CHECK_I32(src);
  const int64_t N = xl.size(0);
  HY_CHECK(xl.dim() == 2 && xr.dim() == 2 && xr.size(0) == N && xl.size(1) == H * C && xr.size(1) == H * C &&
               xl.stride(1) == 1 && xr.stride(1) == 1,
           "gat: xl / xr must be [N, H*C] with unit column stride");
  HY_CHECK(att.is_contiguous() && att.numel() == H * C && att.scalar_type() == at::kFloat, "gat: att [H*C]");
  HY_CHECK(rowptr.numel() == N + 1, "gat: rowptr [N+1]");
  GatArgs a{};
  a.xl = xl.data_ptr<float>();
  a.xr = xr.data_ptr<float>();
  a.ge = nullptr;
  a.gself = nullptr;
  if (ge.has_value() && ge->defined()) {
    HY_CHECK(ge->is_contiguous() && ge->size(0) == src.numel() && ge->numel() == src.numel() * H * C,
             "gat: edge term [E, H*C]");
    a.ge = ge->data_ptr<float>();
  }
  if (gself.has_value() && gself->defined()) {
    HY_CHECK(gself->is_contiguous() && gself->numel() == N * H * C, "gat: self-loop term [N, H*C]");
    a.gself = gself->data_ptr<float>();
  }
  a.att = att.data_ptr<float>();
  a.rowptr = rowptr.data_ptr<int>();
  a.src = src.data_ptr<int>();
  a.ldl = (int)xl.stride(0);
  a.ldr = (int)xr.stride(0);
  a.N = (int)N;
  a.H = (int)H;
  a.C = C;
  a.slope = (float)slope;
  a.self_loop = self_loop ? 1 : 0;
  return a;
}

// register width: the smallest of 8 / 16 / 32 holding C (C > 32 would spill: composite path)
#define HY_GAT_DISPATCH(C, ...)                                                  \
  if ((C) <= 8) { constexpr int kC = 8; __VA_ARGS__; }                           \
  else if ((C) <= 16) { constexpr int kC = 16; __VA_ARGS__; }                    \
  else if ((C) <= 32) { constexpr int kC = 32; __VA_ARGS__; }                    \
  else HY_CHECK(false, "gat: at most 32 channels per head on the fused path");

std::tuple<at::Tensor, at::Tensor> gat_fwd(const at::Tensor& xl, const at::Tensor& xr,
                                           const c10::optional<at::Tensor>& ge,
                                           const c10::optional<at::Tensor>& gself, const at::Tensor& att,
                                           const at::Tensor& rowptr, const at::Tensor& src, int64_t H, double slope,
                                           bool self_loop, const c10::optional<at::Tensor>& rng, int64_t salt,
                                           double p) {
  const int C = (int)(att.numel() / H);
  GatArgs a = gat_args(xl, xr, ge, gself, att, rowptr, src, H, slope, self_loop, C);
  const int64_t N = xl.size(0);
  auto out = at::empty({N, H * C}, xl.options());
  auto ml = at::empty({N, H, 2}, xl.options());
  if (N == 0) return {out, ml};
  const int64_t* rp = rng.has_value() && rng->defined() ? rng->data_ptr<int64_t>() : nullptr;
  HY_GAT_DISPATCH(C, gat_fwd_kernel<kC><<<ceil_div(N * H, 256), 256, 0, stream()>>>(
                         a, rp, salt, (float)p, out.data_ptr<float>(), ml.data_ptr<float>()));
  return {out, ml};
}

// returns (P [E, H*C], dge [E, H*C] or empty, dxr, dxl_self, dgself or empty, datt_part [N, H*C])
std::vector<at::Tensor> gat_bwd(const at::Tensor& dout_, const at::Tensor& xl, const at::Tensor& xr,
                                const c10::optional<at::Tensor>& ge, const c10::optional<at::Tensor>& gself,
                                const at::Tensor& att, const at::Tensor& rowptr, const at::Tensor& src,
                                const at::Tensor& ml, int64_t H, double slope, bool self_loop,
                                const c10::optional<at::Tensor>& rng, int64_t salt, double p) {
  const int C = (int)(att.numel() / H);
  GatArgs a = gat_args(xl, xr, ge, gself, att, rowptr, src, H, slope, self_loop, C);
  auto dout = dout_.contiguous();
  const int64_t N = xl.size(0), E = src.numel();
  HY_CHECK(dout.sizes() == at::IntArrayRef({N, H * C}) && ml.numel() == N * H * 2, "gat_bwd: shapes");
  auto o = xl.options();
  auto P = at::empty({E, H * C}, o);
  auto dge = a.ge != nullptr ? at::empty({E, H * C}, o) : at::empty({0}, o);
  auto dxr = at::empty({N, H * C}, o);
  auto dxl_self = at::empty({N, H * C}, o);
  auto dgself = a.gself != nullptr ? at::empty({N, H * C}, o) : at::empty({0}, o);
  auto datt = at::empty({N, H * C}, o);
  if (N > 0) {
    const int64_t* rp = rng.has_value() && rng->defined() ? rng->data_ptr<int64_t>() : nullptr;
    HY_GAT_DISPATCH(C, gat_bwd_kernel<kC><<<ceil_div(N * H, 256), 256, 0, stream()>>>(
                           a, rp, salt, (float)p, dout.data_ptr<float>(), ml.data_ptr<float>(), P.data_ptr<float>(),
                           a.ge != nullptr ? dge.data_ptr<float>() : nullptr, dxr.data_ptr<float>(),
                           dxl_self.data_ptr<float>(), a.gself != nullptr ? dgself.data_ptr<float>() : nullptr,
                           datt.data_ptr<float>()));
  }
  return {P, dge, dxr, dxl_self, dgself, datt};
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def(
      "gat_fwd(Tensor xl, Tensor xr, Tensor? ge, Tensor? gself, Tensor att, Tensor rowptr, Tensor src, int H, "
      "float slope, bool self_loop, Tensor? rng, int salt, float p) -> (Tensor, Tensor)");
  m.def(
      "gat_bwd(Tensor dout, Tensor xl, Tensor xr, Tensor? ge, Tensor? gself, Tensor att, Tensor rowptr, Tensor src, "
      "Tensor ml, int H, float slope, bool self_loop, Tensor? rng, int salt, float p) -> Tensor[]");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("gat_fwd", hy::gat_fwd);
  m.impl("gat_bwd", hy::gat_bwd);
}
