// CSR segment reductions, row gathers and arg-scatters (gfx950).
//
// These are the atomic-free replacements for torch_scatter / PyG aggregation
// used by every message-passing stack (reference: torch_scatter calls at
// hydragnn/models/Base.py:599, EGCLStack.py:292-298, PAINNStack.py:256-257,
// mace_utils/modules/blocks.py:380-382, and PyG MessagePassing aggr="add"/"mean"/
// "min"/"max").  Because batches are CSR-sorted by destination once in the
// collator, every reduction reads a contiguous edge range per node: results are
// bitwise deterministic and need no float atomics.
//
// Backward duality (used by ops/segment.py to get arbitrary-order derivatives):
//   seg_sum(x, rowptr)             <->  gather_rows(g, seg_id)
//   gather_rows(x, idx)            <->  seg_sum(g, idx_rowptr, idx_perm)
//   seg_minmax(x) -> (out, arg)    <->  scatter_arg(g, arg)  /  gather_arg(x, arg)
#include "common.h"

namespace hy {

template <int VEC>
struct VecT;
template <>
struct VecT<4> {
  using T = float4;
  static __device__ __forceinline__ T zero() { return f4zero(); }
  static __device__ __forceinline__ T add(T a, T b) { return f4add(a, b); }
};
template <>
struct VecT<2> {
  using T = float2;
  static __device__ __forceinline__ T zero() { return make_float2(0.f, 0.f); }
  static __device__ __forceinline__ T add(T a, T b) { return make_float2(a.x + b.x, a.y + b.y); }
};
template <>
struct VecT<1> {
  using T = float;
  static __device__ __forceinline__ T zero() { return 0.f; }
  static __device__ __forceinline__ T add(T a, T b) { return a + b; }
};

template <typename T>
__device__ __forceinline__ T shfl_xor_t(T v, int o);
template <>
__device__ __forceinline__ float shfl_xor_t<float>(float v, int o) { return __shfl_xor(v, o, 64); }
template <>
__device__ __forceinline__ float2 shfl_xor_t<float2>(float2 v, int o) {
  return make_float2(__shfl_xor(v.x, o, 64), __shfl_xor(v.y, o, 64));
}
template <>
__device__ __forceinline__ float4 shfl_xor_t<float4>(float4 v, int o) {
  return make_float4(__shfl_xor(v.x, o, 64), __shfl_xor(v.y, o, 64), __shfl_xor(v.z, o, 64), __shfl_xor(v.w, o, 64));
}

// out[n, :] = sum_{e in [rowptr[n], rowptr[n+1])} x[perm ? perm[e] : e, :] * (scale? 1/deg : 1)
// Load balance: a segment is served by KS x tpr threads of one wave — KS
// interleaved row streams per column group, folded by a fixed xor butterfly (deterministic)
// — so a hub node with 70 in-edges (torch_cluster "index" caps make low-index atoms the
// source of every neighbourhood) costs ~70/KS dependent loads instead of 70.
//
// GM = true: gather-multiply-sum  out[n] = sum_e w[row] * x[gidx[row]] (row = perm[e] or e),
// the CFConv / continuous-filter message + aggregation in one pass (no [E, F] message
// tensor): x is the node table, w the per-edge filter rows.
template <typename T>
__device__ __forceinline__ T vmul(T a, T b);
template <>
__device__ __forceinline__ float4 vmul<float4>(float4 a, float4 b) {
  return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w);
}
template <>
__device__ __forceinline__ float2 vmul<float2>(float2 a, float2 b) { return make_float2(a.x * b.x, a.y * b.y); }
template <>
__device__ __forceinline__ float vmul<float>(float a, float b) { return a * b; }

template <int VEC, bool MEAN, int KS, bool GM = false>
__global__ void __launch_bounds__(256) seg_sum_kernel(const float* __restrict__ x,
                                                      const int* __restrict__ rowptr,
                                                      const int* __restrict__ perm,
                                                      float* __restrict__ out, int N, int F,
                                                      int tpr, int rpb,
                                                      const float* __restrict__ w = nullptr,
                                                      const int* __restrict__ gidx = nullptr, int ldo = 0,
                                                      const int* __restrict__ row_limit = nullptr) {
  using V = VecT<VEC>;
  using T = typename V::T;
  const int tg = tpr * KS;
  const int r = blockIdx.x * rpb + threadIdx.x / tg;
  const int lt = threadIdx.x % tg;
  const int c = lt % tpr, k = lt / tpr;
  if (r >= N) return;
  // row_limit (device scalar, e.g. the padded batch's valid-node count): rows past it are
  // padding; the padding graph's long tail segment is then empty instead of serial work
  const int end = row_limit ? min(rowptr[r + 1], *row_limit) : rowptr[r + 1];
  const int beg = min(rowptr[r], end);
  const int nv = F / VEC;
  const float inv = MEAN ? 1.f / (float)max(end - beg, 1) : 1.f;
  for (int v = c; v < nv; v += tpr) {
    T a0 = V::zero(), a1 = V::zero();
    // this stream's rows e = beg + k, + KS, ... alternate between a0 and a1; U row pairs per
    // batch with every index load, then every row load, in flight together (one pair at a
    // time paid the perm -> row dependent latency per pair).  Rows past the segment are
    // clamped loads that are never added: the fold order is the pairwise one regardless.
    constexpr int U = VEC == 4 ? 2 : 4;
    for (int e = beg + k; e < end; e += 2 * KS * U) {
      int i0[U], i1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int ea = min(e + 2 * KS * u, end - 1), eb = min(e + 2 * KS * u + KS, end - 1);
        i0[u] = perm ? perm[ea] : ea;
        i1[u] = perm ? perm[eb] : eb;
      }
      T x0[U], x1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if constexpr (GM) {
          x0[u] = vmul(reinterpret_cast<const T*>(w + (int64_t)i0[u] * F)[v],
                       reinterpret_cast<const T*>(x + (int64_t)gidx[i0[u]] * F)[v]);
          x1[u] = vmul(reinterpret_cast<const T*>(w + (int64_t)i1[u] * F)[v],
                       reinterpret_cast<const T*>(x + (int64_t)gidx[i1[u]] * F)[v]);
        } else {
          x0[u] = reinterpret_cast<const T*>(x + (int64_t)i0[u] * F)[v];
          x1[u] = reinterpret_cast<const T*>(x + (int64_t)i1[u] * F)[v];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int ea = e + 2 * KS * u;
        if (ea < end) a0 = V::add(a0, x0[u]);
        if (ea + KS < end) a1 = V::add(a1, x1[u]);
      }
    }
    T a = V::add(a0, a1);
#pragma unroll
    for (int o = 1; o < KS; o <<= 1) a = V::add(a, shfl_xor_t<T>(a, o * tpr));
    if (k != 0) continue;
    if constexpr (MEAN) {
      if constexpr (VEC == 4) a = f4scale(a, inv);
      else if constexpr (VEC == 2) a = make_float2(a.x * inv, a.y * inv);
      else a *= inv;
    }
    reinterpret_cast<T*>(out + (int64_t)r * (ldo > 0 ? ldo : F))[v] = a;
  }
}

// out[e, :] = x[idx[e], :]
template <int VEC>
__global__ void __launch_bounds__(256) gather_rows_kernel(const float* __restrict__ x,
                                                          const int* __restrict__ idx,
                                                          float* __restrict__ out, int E, int F,
                                                          int tpr, int rpb) {
  using T = typename VecT<VEC>::T;
  const int r = blockIdx.x * rpb + threadIdx.x / tpr;
  const int c = threadIdx.x % tpr;
  if (r >= E) return;
  const int64_t s = idx[r];
  const int nv = F / VEC;
  for (int v = c; v < nv; v += tpr)
    reinterpret_cast<T*>(out + (int64_t)r * F)[v] = reinterpret_cast<const T*>(x + s * F)[v];
}

// Segment min/max with argument (edge position, -1 for an empty segment -> value 0,
// matching PyG's scatter(reduce="min"/"max") fill for isolated nodes).
template <bool IS_MAX>
__global__ void __launch_bounds__(256) seg_minmax_kernel(const float* __restrict__ x,
                                                         const int* __restrict__ rowptr,
                                                         const int* __restrict__ perm,
                                                         float* __restrict__ out,
                                                         int* __restrict__ arg, int N, int F) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)N * F) return;
  const int n = (int)(t / F), f = (int)(t % F);
  const int beg = rowptr[n], end = rowptr[n + 1];
  float best = IS_MAX ? -INFINITY : INFINITY;
  int besti = -1;
  for (int e = beg; e < end; ++e) {
    // permuted CSR (e.g. the source view): rows arrive out of order, so ties go to the
    // smallest row id explicitly (the composite's first-row rule)
    const int row = perm ? perm[e] : e;
    const float v = x[(int64_t)row * F + f];
    if ((IS_MAX ? (v > best) : (v < best)) || (v == best && besti >= 0 && row < besti)) {
      best = v;
      besti = row;
    }
  }
  out[t] = besti < 0 ? 0.f : best;
  arg[t] = besti;
}

// PNA degree-scaler aggregation of a per-row message table in one pass (the PNAEq message,
// reference PNAEqStack.py:59-66 / :310-387 over PyG DegreeScalerAggregation with aggregators
// [mean, min, max, std] and any of the 5 scalers incl. inverse_linear): one thread per
// (segment, column) walks the segment's rows once for sum, sum of squares and the two
// extrema, then writes out[n, s*4F + k*F + f] = scaler_s(deg_n) * agg_k for every scaler.
// The composite it replaces (ops.pna.pna_aggregate_composite) takes 4 reductions, a
// sqrt/clamp/mask chain, two cats and S multiplies.  Scaler codes are packed 3 bits each
// (0 identity, 1 amplification, 2 attenuation, 3 linear, 4 inverse_linear).
__device__ __forceinline__ float pna_scaler(int code, float d, float avg_log, float avg_lin) {
  switch (code) {
    case 0: return 1.f;
    case 1: return logf(d + 1.f) / avg_log;
    case 2: return avg_log / logf(d + 1.f);
    case 3: return d / avg_lin;
    default: return avg_lin / d;
  }
}

struct PnaAggArgs {
  const float* x;
  const int* rowptr;
  const int* perm;
  float* out;    // [N, S*4F]
  float* stat;   // [N, 2F]: mean, std (0 where masked)
  int* arg;      // [N, 2F]: row of the min / max (-1 for an empty segment)
  const float* g;  // backward: dL/dout
  float* dx;       // backward: [E, F]
  int N, F, S, codes;
  float avg_log, avg_lin, eps, sqrt_eps;
};

__global__ void __launch_bounds__(256) seg_pna_agg_kernel(PnaAggArgs a) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)a.N * a.F) return;
  const int F = a.F, n = (int)(t / F), f = (int)(t % F);
  const int beg = a.rowptr[n], end = a.rowptr[n + 1];
  float s = 0.f, s2 = 0.f, mn = INFINITY, mx = -INFINITY;
  int imn = -1, imx = -1;
  for (int e = beg; e < end; ++e) {
    const int row = a.perm ? a.perm[e] : e;
    const float v = a.x[(int64_t)row * F + f];
    s += v;
    s2 += v * v;
    if (v < mn) { mn = v; imn = row; }
    if (v > mx) { mx = v; imx = row; }
  }
  const float d = (float)max(end - beg, 1);
  const float mean = s / d;
  float sd = sqrtf(fmaxf(s2 / d - mean * mean, a.eps));
  if (sd <= a.sqrt_eps) sd = 0.f;
  if (imn < 0) { mn = 0.f; mx = 0.f; }
  const float agg[4] = {mean, mn, mx, sd};
  float* o = a.out + (int64_t)n * a.S * 4 * F + f;
  for (int si = 0; si < a.S; ++si) {
    const float sc = pna_scaler((a.codes >> (3 * si)) & 7, d, a.avg_log, a.avg_lin);
#pragma unroll
    for (int k = 0; k < 4; ++k) o[(si * 4 + k) * F] = agg[k] * sc;
  }
  a.stat[(int64_t)n * 2 * F + f] = mean;
  a.stat[(int64_t)n * 2 * F + F + f] = sd;
  a.arg[(int64_t)n * 2 * F + f] = imn;
  a.arg[(int64_t)n * 2 * F + F + f] = imx;
}

// dx[row, f] = Gmean/d + Gstd (x - mean)/(d std) + [row == argmin] Gmin + [row == argmax] Gmax
// with G_k = sum_s scaler_s(d) g[n, s*4F + k*F + f]: the same (segment, column) threads
// fold the scalers once and write every row of the segment (rows partition the segments,
// so each dx element is written exactly once, without atomics).
__global__ void __launch_bounds__(256) seg_pna_agg_bwd_kernel(PnaAggArgs a) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)a.N * a.F) return;
  const int F = a.F, n = (int)(t / F), f = (int)(t % F);
  const int beg = a.rowptr[n], end = a.rowptr[n + 1];
  if (end <= beg) return;
  const float d = (float)(end - beg);
  float G[4] = {0.f, 0.f, 0.f, 0.f};
  const float* gp = a.g + (int64_t)n * a.S * 4 * F + f;
  for (int si = 0; si < a.S; ++si) {
    const float sc = pna_scaler((a.codes >> (3 * si)) & 7, d, a.avg_log, a.avg_lin);
#pragma unroll
    for (int k = 0; k < 4; ++k) G[k] += sc * gp[(si * 4 + k) * F];
  }
  const float mean = a.stat[(int64_t)n * 2 * F + f], sd = a.stat[(int64_t)n * 2 * F + F + f];
  const int imn = a.arg[(int64_t)n * 2 * F + f], imx = a.arg[(int64_t)n * 2 * F + F + f];
  const float gm = G[0] / d, gs = sd > 0.f ? G[3] / (d * sd) : 0.f;
  for (int e = beg; e < end; ++e) {
    const int row = a.perm ? a.perm[e] : e;
    const float v = a.x[(int64_t)row * F + f];
    float r = gm;
    if (gs != 0.f) r += gs * (v - mean);  // no 0 * inf from a non-finite padding row
    if (row == imn) r += G[1];
    if (row == imx) r += G[2];
    a.dx[(int64_t)row * F + f] = r;
  }
}

// out[E, F] = 0; out[arg[n,f], f] = g[n,f]   (segments are disjoint -> no conflicts)
__global__ void __launch_bounds__(256) scatter_arg_kernel(const float* __restrict__ g,
                                                          const int* __restrict__ arg,
                                                          float* __restrict__ out, int N, int F) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)N * F) return;
  const int a = arg[t];
  if (a >= 0) out[(int64_t)a * F + (t % F)] = g[t];
}

// out[n,f] = x[arg[n,f], f] (0 when arg < 0)
__global__ void __launch_bounds__(256) gather_arg_kernel(const float* __restrict__ x,
                                                         const int* __restrict__ arg,
                                                         float* __restrict__ out, int N, int F) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)N * F) return;
  const int a = arg[t];
  out[t] = a >= 0 ? x[(int64_t)a * F + (t % F)] : 0.f;
}

// out[e, :] = x[ia[e], :] * y[ib[e], :]   (the filter gradient of gather-multiply-sum)
template <int VEC>
__global__ void __launch_bounds__(256) gather_mul2_kernel(const float* __restrict__ x, const int* __restrict__ ia,
                                                          const float* __restrict__ y, const int* __restrict__ ib,
                                                          float* __restrict__ out, int E, int F, int tpr, int rpb) {
  using T = typename VecT<VEC>::T;
  const int r = blockIdx.x * rpb + threadIdx.x / tpr;
  const int c = threadIdx.x % tpr;
  if (r >= E) return;
  const int64_t a = ia[r], b = ib[r];
  const int nv = F / VEC;
  for (int v = c; v < nv; v += tpr)
    reinterpret_cast<T*>(out + (int64_t)r * F)[v] =
        vmul(reinterpret_cast<const T*>(x + a * F)[v], reinterpret_cast<const T*>(y + b * F)[v]);
}

// ---------------------------------------------------------------- host side

static at::Tensor as2d(const at::Tensor& x) { return x.dim() == 1 ? x.unsqueeze(1) : x; }

at::Tensor seg_sum(const at::Tensor& x_, const at::Tensor& rowptr, const c10::optional<at::Tensor>& perm,
                   int64_t N, bool mean, const c10::optional<at::Tensor>& limit) {
  HY_CHECK_CUDA(x_);
  auto x = as2d(x_).contiguous();
  HY_CHECK_F32(x);
  HY_CHECK_I32(rowptr);
  HY_CHECK(rowptr.numel() == N + 1, "rowptr must have N+1 entries");
  const int F = (int)x.size(1);
  auto out = at::empty({N, F}, x.options());
  if (N == 0 || F == 0) return out;
  const int* pp = nullptr;
  if (perm.has_value() && perm->defined()) {
    HY_CHECK_I32(*perm);
    pp = perm->data_ptr<int>();
  }
  const int* lim = nullptr;
  if (limit.has_value() && limit->defined()) {
    HY_CHECK(limit->is_cuda() && limit->scalar_type() == at::kInt && limit->numel() == 1,
             "seg_sum: limit must be a device int32 scalar");
    // with a perm the limit bounds positions in the permuted order (the caller's padding
    // rows must sit at the tail of that order, e.g. the static radius graph's source view)
    lim = limit->data_ptr<int>();
  }
  const bool v4 = (F % 4 == 0);
  // wide odd-multiple-of-2 rows (the SC25 EGNN's 866 channels): float2 loads halve the
  // per-column dependent load chains of the scalar path
  const bool v2 = !v4 && (F % 2 == 0) && F >= 128;
  auto g = row_geom(N, v4 ? F : (v2 ? F * 2 : F * 4));
  // KS row streams per segment, as long as one segment's threads stay inside a wave
  const int ks = g.tpr <= 16 ? 4 : (g.tpr <= 32 ? 2 : 1);
  const int rpb = 256 / (g.tpr * ks);
  const int blocks = (int)std::max<int64_t>(1, (N + rpb - 1) / rpb);
#define HY_SEG_SUM(VEC, MEAN, KS)                                                                              \
  seg_sum_kernel<VEC, MEAN, KS><<<blocks, 256, 0, stream()>>>(x.data_ptr<float>(), rowptr.data_ptr<int>(), pp, \
                                                              out.data_ptr<float>(), N, F, g.tpr, rpb, nullptr,  \
                                                              nullptr, 0, lim)
#define HY_SEG_SUM_KS(VEC, MEAN) \
  if (ks == 4) HY_SEG_SUM(VEC, MEAN, 4); else if (ks == 2) HY_SEG_SUM(VEC, MEAN, 2); else HY_SEG_SUM(VEC, MEAN, 1)
  if (v4) {
    if (mean) { HY_SEG_SUM_KS(4, true); } else { HY_SEG_SUM_KS(4, false); }
  } else if (v2) {
    if (mean) { HY_SEG_SUM_KS(2, true); } else { HY_SEG_SUM_KS(2, false); }
  } else {
    if (mean) { HY_SEG_SUM_KS(1, true); } else { HY_SEG_SUM_KS(1, false); }
  }
#undef HY_SEG_SUM_KS
#undef HY_SEG_SUM
  return x_.dim() == 1 ? out.squeeze(1) : out;
}

// seg_sum into a caller-provided [N, F] view with row stride out.stride(0) (e.g. the right
// half of a concatenated gradient buffer: no separate torch.cat launch)
void seg_sum_out(const at::Tensor& x_, const at::Tensor& rowptr, const c10::optional<at::Tensor>& perm,
                 at::Tensor out) {
  HY_CHECK_CUDA(x_);
  auto x = as2d(x_).contiguous();
  HY_CHECK_F32(x);
  HY_CHECK_F32(out);
  HY_CHECK_I32(rowptr);
  const int64_t N = out.size(0);
  const int F = (int)x.size(1);
  HY_CHECK(out.dim() == 2 && out.size(1) == F && out.stride(1) == 1 && rowptr.numel() == N + 1,
           "seg_sum_out: shapes");
  const int ldo = (int)out.stride(0);
  if (N == 0 || F == 0) return;
  const int* pp = nullptr;
  if (perm.has_value() && perm->defined()) {
    HY_CHECK_I32(*perm);
    pp = perm->data_ptr<int>();
  }
  const bool v4 = (F % 4 == 0) && (ldo % 4 == 0) && (reinterpret_cast<uintptr_t>(out.data_ptr<float>()) % 16 == 0);
  auto g = row_geom(N, v4 ? F : F * 4);
  const int ks = g.tpr <= 16 ? 4 : (g.tpr <= 32 ? 2 : 1);
  const int rpb = 256 / (g.tpr * ks);
  const int blocks = (int)std::max<int64_t>(1, (N + rpb - 1) / rpb);
#define HY_SSO(VEC, KS)                                                                                          \
  seg_sum_kernel<VEC, false, KS><<<blocks, 256, 0, stream()>>>(x.data_ptr<float>(), rowptr.data_ptr<int>(), pp,  \
                                                               out.data_ptr<float>(), (int)N, F, g.tpr, rpb,     \
                                                               nullptr, nullptr, ldo)
  if (v4) {
    if (ks == 4) HY_SSO(4, 4); else if (ks == 2) HY_SSO(4, 2); else HY_SSO(4, 1);
  } else {
    if (ks == 4) HY_SSO(1, 4); else if (ks == 2) HY_SSO(1, 2); else HY_SSO(1, 1);
  }
#undef HY_SSO
}

// out[n] = sum over the rowptr segment n (rows through perm) of w[row] * x[gidx[row]]
at::Tensor gather_mul_sum(const at::Tensor& x_, const at::Tensor& w_, const at::Tensor& gidx,
                          const at::Tensor& rowptr, const c10::optional<at::Tensor>& perm, int64_t N,
                          const c10::optional<at::Tensor>& limit) {
  HY_CHECK_CUDA(x_);
  auto x = as2d(x_).contiguous(), w = as2d(w_).contiguous();
  HY_CHECK_F32(x);
  HY_CHECK_F32(w);
  HY_CHECK_I32(gidx);
  HY_CHECK_I32(rowptr);
  HY_CHECK(rowptr.numel() == N + 1, "rowptr must have N+1 entries");
  HY_CHECK(w.size(1) == x.size(1) && gidx.numel() == w.size(0), "gather_mul_sum: shapes");
  const int F = (int)x.size(1);
  auto out = at::empty({N, F}, x.options());
  if (N == 0 || F == 0) return out;
  const int* pp = nullptr;
  if (perm.has_value() && perm->defined()) {
    HY_CHECK_I32(*perm);
    pp = perm->data_ptr<int>();
  }
  const int* lim = nullptr;
  if (limit.has_value() && limit->defined()) {
    HY_CHECK(limit->is_cuda() && limit->scalar_type() == at::kInt && limit->numel() == 1,
             "gather_mul_sum: limit must be a device int32 scalar");
    lim = limit->data_ptr<int>();  // CSR positions at or past it are padding: skipped
  }
  const bool v4 = (F % 4 == 0);
  auto g = row_geom(N, v4 ? F : F * 4);
  const int ks = g.tpr <= 16 ? 4 : (g.tpr <= 32 ? 2 : 1);
  const int rpb = 256 / (g.tpr * ks);
  const int blocks = (int)std::max<int64_t>(1, (N + rpb - 1) / rpb);
#define HY_GMS(VEC, KS)                                                                                  \
  seg_sum_kernel<VEC, false, KS, true><<<blocks, 256, 0, stream()>>>(                                    \
      x.data_ptr<float>(), rowptr.data_ptr<int>(), pp, out.data_ptr<float>(), (int)N, F, g.tpr, rpb,     \
      w.data_ptr<float>(), gidx.data_ptr<int>(), 0, lim)
  if (v4) {
    if (ks == 4) HY_GMS(4, 4); else if (ks == 2) HY_GMS(4, 2); else HY_GMS(4, 1);
  } else {
    if (ks == 4) HY_GMS(1, 4); else if (ks == 2) HY_GMS(1, 2); else HY_GMS(1, 1);
  }
#undef HY_GMS
  return x_.dim() == 1 ? out.squeeze(1) : out;
}

at::Tensor gather_mul2(const at::Tensor& x_, const at::Tensor& ia, const at::Tensor& y_, const at::Tensor& ib) {
  HY_CHECK_CUDA(x_);
  auto x = as2d(x_).contiguous(), y = as2d(y_).contiguous();
  HY_CHECK_F32(x);
  HY_CHECK_F32(y);
  HY_CHECK_I32(ia);
  HY_CHECK_I32(ib);
  HY_CHECK(x.size(1) == y.size(1) && ia.numel() == ib.numel(), "gather_mul2: shapes");
  const int64_t E = ia.numel();
  const int F = (int)x.size(1);
  auto out = at::empty({E, F}, x.options());
  if (E == 0 || F == 0) return out;
  const bool v4 = (F % 4 == 0);
  auto g = row_geom(E, v4 ? F : F * 4);
  const int rpb = 256 / g.tpr;
  const int blocks = (int)std::max<int64_t>(1, (E + rpb - 1) / rpb);
  if (v4)
    gather_mul2_kernel<4><<<blocks, 256, 0, stream()>>>(x.data_ptr<float>(), ia.data_ptr<int>(), y.data_ptr<float>(),
                                                        ib.data_ptr<int>(), out.data_ptr<float>(), (int)E, F, g.tpr,
                                                        rpb);
  else
    gather_mul2_kernel<1><<<blocks, 256, 0, stream()>>>(x.data_ptr<float>(), ia.data_ptr<int>(), y.data_ptr<float>(),
                                                        ib.data_ptr<int>(), out.data_ptr<float>(), (int)E, F, g.tpr,
                                                        rpb);
  return x_.dim() == 1 ? out.squeeze(1) : out;
}

at::Tensor gather_rows(const at::Tensor& x_, const at::Tensor& idx) {
  HY_CHECK_CUDA(x_);
  auto x = as2d(x_).contiguous();
  HY_CHECK_F32(x);
  HY_CHECK_I32(idx);
  const int64_t E = idx.numel();
  const int F = (int)x.size(1);
  auto out = at::empty({E, F}, x.options());
  if (E == 0 || F == 0) return x_.dim() == 1 ? out.squeeze(1) : out;
  const bool v4 = (F % 4 == 0);
  auto g = row_geom(E, v4 ? F : F * 4);
  if (v4)
    gather_rows_kernel<4><<<g.blocks, 256, 0, stream()>>>(x.data_ptr<float>(), idx.data_ptr<int>(),
                                                         out.data_ptr<float>(), E, F, g.tpr, g.rows_per_block);
  else
    gather_rows_kernel<1><<<g.blocks, 256, 0, stream()>>>(x.data_ptr<float>(), idx.data_ptr<int>(),
                                                         out.data_ptr<float>(), E, F, g.tpr, g.rows_per_block);
  return x_.dim() == 1 ? out.squeeze(1) : out;
}

std::tuple<at::Tensor, at::Tensor> seg_minmax(const at::Tensor& x_, const at::Tensor& rowptr, int64_t N,
                                              bool is_max, const c10::optional<at::Tensor>& perm) {
  HY_CHECK_CUDA(x_);
  auto x = as2d(x_).contiguous();
  HY_CHECK_F32(x);
  HY_CHECK_I32(rowptr);
  const int F = (int)x.size(1);
  auto out = at::empty({N, F}, x.options());
  auto arg = at::empty({N, F}, x.options().dtype(at::kInt));
  const int64_t tot = N * F;
  const int* pp = nullptr;
  if (perm.has_value() && perm->defined()) {
    HY_CHECK_I32(*perm);
    pp = perm->data_ptr<int>();
  }
  if (tot > 0) {
    if (is_max)
      seg_minmax_kernel<true><<<ceil_div(tot, 256), 256, 0, stream()>>>(
          x.data_ptr<float>(), rowptr.data_ptr<int>(), pp, out.data_ptr<float>(), arg.data_ptr<int>(), N, F);
    else
      seg_minmax_kernel<false><<<ceil_div(tot, 256), 256, 0, stream()>>>(
          x.data_ptr<float>(), rowptr.data_ptr<int>(), pp, out.data_ptr<float>(), arg.data_ptr<int>(), N, F);
  }
  return {out, arg};
}

at::Tensor scatter_arg(const at::Tensor& g_, const at::Tensor& arg, int64_t E) {
  HY_CHECK_CUDA(g_);
  auto g = g_.contiguous();
  HY_CHECK_F32(g);
  HY_CHECK_I32(arg);
  const int64_t N = g.size(0);
  const int F = (int)g.size(1);
  auto out = at::zeros({E, F}, g.options());
  if (N * F > 0)
    scatter_arg_kernel<<<ceil_div(N * F, 256), 256, 0, stream()>>>(g.data_ptr<float>(), arg.data_ptr<int>(),
                                                                  out.data_ptr<float>(), N, F);
  return out;
}

at::Tensor gather_arg(const at::Tensor& x_, const at::Tensor& arg) {
  HY_CHECK_CUDA(x_);
  auto x = x_.contiguous();
  HY_CHECK_F32(x);
  HY_CHECK_I32(arg);
  const int64_t N = arg.size(0);
  const int F = (int)arg.size(1);
  auto out = at::empty({N, F}, x.options());
  if (N * F > 0)
    gather_arg_kernel<<<ceil_div(N * F, 256), 256, 0, stream()>>>(x.data_ptr<float>(), arg.data_ptr<int>(),
                                                                 out.data_ptr<float>(), N, F);
  return out;
}

static PnaAggArgs pna_agg_args(const at::Tensor& x, const at::Tensor& rowptr, const c10::optional<at::Tensor>& perm,
                               int64_t S, int64_t codes, double avg_log, double avg_lin) {
  HY_CHECK_CUDA(x);
  HY_CHECK_F32(x);
  HY_CHECK(x.dim() == 2 && x.is_contiguous(), "seg_pna_agg: x must be a contiguous [E, F] table");
  HY_CHECK_I32(rowptr);
  HY_CHECK(S >= 1 && S <= 8, "seg_pna_agg: 1..8 scalers");
  PnaAggArgs a{};
  a.x = x.data_ptr<float>();
  a.rowptr = rowptr.data_ptr<int>();
  if (perm.has_value() && perm->defined()) {
    HY_CHECK_I32(*perm);
    HY_CHECK(perm->numel() == x.size(0), "seg_pna_agg: perm must list every row");
    a.perm = perm->data_ptr<int>();
  }
  a.N = (int)(rowptr.numel() - 1);
  a.F = (int)x.size(1);
  a.S = (int)S;
  a.codes = (int)codes;
  a.avg_log = (float)avg_log;
  a.avg_lin = (float)avg_lin;
  return a;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> seg_pna_agg(const at::Tensor& x, const at::Tensor& rowptr,
                                                           const c10::optional<at::Tensor>& perm, int64_t S,
                                                           int64_t codes, double avg_log, double avg_lin, double eps,
                                                           double sqrt_eps) {
  auto a = pna_agg_args(x, rowptr, perm, S, codes, avg_log, avg_lin);
  a.eps = (float)eps;
  a.sqrt_eps = (float)sqrt_eps;
  auto out = at::empty({a.N, 4 * S * a.F}, x.options());
  auto stat = at::empty({a.N, 2 * a.F}, x.options());
  auto arg = at::empty({a.N, 2 * a.F}, x.options().dtype(at::kInt));
  a.out = out.data_ptr<float>();
  a.stat = stat.data_ptr<float>();
  a.arg = arg.data_ptr<int>();
  const int64_t tot = (int64_t)a.N * a.F;
  if (tot > 0) seg_pna_agg_kernel<<<ceil_div(tot, 256), 256, 0, stream()>>>(a);
  return {out, stat, arg};
}

at::Tensor seg_pna_agg_bwd(const at::Tensor& g_, const at::Tensor& x, const at::Tensor& rowptr,
                           const c10::optional<at::Tensor>& perm, const at::Tensor& stat, const at::Tensor& arg,
                           int64_t S, int64_t codes, double avg_log, double avg_lin) {
  auto a = pna_agg_args(x, rowptr, perm, S, codes, avg_log, avg_lin);
  auto g = g_.contiguous();
  HY_CHECK_F32(g);
  HY_CHECK(g.size(0) == a.N && g.size(1) == 4 * S * a.F, "seg_pna_agg_bwd: gradient shape");
  HY_CHECK(stat.size(0) == a.N && stat.size(1) == 2 * a.F && arg.size(1) == 2 * a.F, "seg_pna_agg_bwd: saved shapes");
  // zero-filled: a padded batch's permutation need not list every padding row (rows no
  // segment owns get zero gradient, as in the composite's gather / arg-scatter)
  auto dx = at::zeros_like(x);
  a.g = g.data_ptr<float>();
  a.stat = const_cast<float*>(stat.data_ptr<float>());
  a.arg = const_cast<int*>(arg.data_ptr<int>());
  a.dx = dx.data_ptr<float>();
  const int64_t tot = (int64_t)a.N * a.F;
  if (tot > 0) seg_pna_agg_bwd_kernel<<<ceil_div(tot, 256), 256, 0, stream()>>>(a);
  return dx;
}


// ------------------------------------------------------------------ element CSR (one wave)
// Owner index over a FEW segments (MACE's per-element weight tables: ~10-100 elements over a
// batch's nodes) -> (rowptr [S+1], stable permutation [N]) in ONE launch of one wave, instead
// of the count/scan/radix-sort chain (~9 launches per step).  Counts by LDS atomics, a scan
// of the S counts, then the nodes in order, 64 at a time: each lane's rank among the earlier
// lanes of the same segment comes from ballots over the chunk's distinct values (a
// stable counting sort), and each segment's leader lane advances its cursor.
constexpr int kElemMaxS = 1024;

__global__ void __launch_bounds__(64) elem_csr_kernel(const int64_t* __restrict__ idx, int N, int S,
                                                      int* __restrict__ rowptr, int* __restrict__ perm,
                                                      int* __restrict__ idx32, int* __restrict__ err) {
  __shared__ int cnt[kElemMaxS + 1];
  __shared__ int cur[kElemMaxS];
  const int lane = threadIdx.x;
  for (int s = lane; s < S; s += 64) {
    cnt[s] = 0;
    cur[s] = 0;
  }
  __syncthreads();
  int bad = 0;
  for (int n = lane; n < N; n += 64) {
    const int64_t r = idx[n];
    const bool ok = r >= 0 && r < S;
    bad += ok ? 0 : 1;
    const int v = ok ? (int)r : S - 1;  // out of range: clamped for memory safety, flagged
    idx32[n] = v;
    atomicAdd(&cnt[v], 1);
  }
  if (__ballot(bad != 0) && err != nullptr && lane == 0) atomicMax(err, 1);
  __syncthreads();
  if (lane == 0) {  // S is small: one lane's serial scan
    int run = 0;
    for (int s = 0; s < S; ++s) {
      const int c = cnt[s];
      cnt[s] = run;
      run += c;
    }
    cnt[S] = run;
  }
  __syncthreads();
  for (int s = lane; s <= S; s += 64) rowptr[s] = cnt[s];
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (int n0 = 0; n0 < N; n0 += 64) {
    const int n = n0 + lane;
    const bool act = n < N;
    int v = act ? (int)idx[n] : -1;
    if (act && (v < 0 || v >= S)) v = S - 1;
    unsigned long long todo = __ballot(act);
    int rank = 0, count = 0;
    while (todo) {  // one round per distinct value of the chunk
      const int src = __ffsll((long long)todo) - 1;
      const int u = __shfl(v, src, 64);
      const unsigned long long same = __ballot(act && v == u);
      if (v == u) {
        rank = __popcll(same & lt);
        count = __popcll(same);
      }
      todo &= ~same;
    }
    if (act) perm[cnt[v] + cur[v] + rank] = n;
    __syncthreads();
    if (act && rank == count - 1) cur[v] += count;  // the segment's last lane in the chunk
    __syncthreads();
  }
}

// idx int64 [N] in [0, S) -> (index int32 [N], rowptr int32 [S+1], perm int32 [N])
std::vector<at::Tensor> elem_csr(const at::Tensor& idx_, int64_t S, const c10::optional<at::Tensor>& err) {
  HY_CHECK_CUDA(idx_);
  auto idx = idx_.to(at::kLong).contiguous().view({-1});
  const int64_t N = idx.numel();
  HY_CHECK(S > 0 && S <= kElemMaxS && N < (1LL << 31), "elem_csr: 0 < segments <= ", kElemMaxS);
  HY_CHECK(!err.has_value() || (err->is_cuda() && err->scalar_type() == at::kInt && err->numel() >= 1),
           "elem_csr: err must be a device int32 flag");
  auto io = idx.options().dtype(at::kInt);
  auto rowptr = at::empty({S + 1}, io), perm = at::empty({N}, io), idx32 = at::empty({N}, io);
  elem_csr_kernel<<<1, 64, 0, stream()>>>(idx.data_ptr<int64_t>(), (int)N, (int)S, rowptr.data_ptr<int>(),
                                          perm.data_ptr<int>(), idx32.data_ptr<int>(),
                                          err.has_value() ? err->data_ptr<int>() : nullptr);
  return {idx32, rowptr, perm};
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("elem_csr(Tensor idx, int S, Tensor(a!)? err=None) -> Tensor[]");
  m.def("seg_pna_agg(Tensor x, Tensor rowptr, Tensor? perm, int S, int codes, float avg_log, float avg_lin, "
        "float eps, float sqrt_eps) -> (Tensor, Tensor, Tensor)");
  m.def("seg_pna_agg_bwd(Tensor g, Tensor x, Tensor rowptr, Tensor? perm, Tensor stat, Tensor arg, int S, "
        "int codes, float avg_log, float avg_lin) -> Tensor");
  m.def("seg_sum(Tensor x, Tensor rowptr, Tensor? perm, int N, bool mean, Tensor? limit=None) -> Tensor");
  m.def("gather_rows(Tensor x, Tensor idx) -> Tensor");
  m.def("seg_minmax(Tensor x, Tensor rowptr, int N, bool is_max, Tensor? perm=None) -> (Tensor, Tensor)");
  m.def("scatter_arg(Tensor g, Tensor arg, int E) -> Tensor");
  m.def("gather_arg(Tensor x, Tensor arg) -> Tensor");
  m.def("gather_mul_sum(Tensor x, Tensor w, Tensor gidx, Tensor rowptr, Tensor? perm, int N, Tensor? limit=None) -> Tensor");
  m.def("gather_mul2(Tensor x, Tensor ia, Tensor y, Tensor ib) -> Tensor");
  m.def("seg_sum_out(Tensor x, Tensor rowptr, Tensor? perm, Tensor(a!) out) -> ()");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("elem_csr", hy::elem_csr);
  m.impl("seg_sum", hy::seg_sum);
  m.impl("gather_rows", hy::gather_rows);
  m.impl("seg_minmax", hy::seg_minmax);
  m.impl("scatter_arg", hy::scatter_arg);
  m.impl("gather_arg", hy::gather_arg);
  m.impl("gather_mul_sum", hy::gather_mul_sum);
  m.impl("gather_mul2", hy::gather_mul2);
  m.impl("seg_sum_out", hy::seg_sum_out);
  m.impl("seg_pna_agg", hy::seg_pna_agg);
  m.impl("seg_pna_agg_bwd", hy::seg_pna_agg_bwd);
}
