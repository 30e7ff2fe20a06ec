// e3nn o3.Linear (per-(l, p) channel mixing of a flat irreps row) on gfx950 — reference
// e3nn ``o3.Linear`` used throughout hydragnn/utils/mace_utils/modules/blocks.py
// (linear_up / linear_down / skip_tp / linear / product-basis linear).
//
// Flat layout: a block (m channels, degree l) of a row occupies m * (2l+1) consecutive
// columns, channel-major (column = off + u * (2l+1) + c).  A path p maps input block ii
// to output block io of the same (l, p) with the weight W_p[mi, mo] (flat weight vector
// at w_off, row-major) times the path normalisation a_p:
//
//     out[n, io(o, c)] = sum_{p -> io} a_p sum_i x[n, ii(i, c)] W_p[i, o]  (+ res[n, io(o, c)])
//
// The optional residual ``res`` is added in the epilogue: the MACE product block's skip
// connection (``linear(.) + sc``) forward, and, in the transposed orientation, the sum of
// the input gradients of several linears reading the same rows (skip / up / down of one
// interaction) without a separate add pass each.
//
// The torch composite is a transposing copy + GEMM + transposing copy per path plus a
// concat (and a zero-fill + copy per slice in backward); for MACE widths (64 channels,
// l <= 3, a few hundred nodes) every one of those is a launch-bound few-microsecond
// kernel.  Here:
//   * il_fwd_kernel: one launch computes every output column of a row tile: the tile's
//     input rows sit in LDS, each thread owns one output column for the tile's rows (a
//     column table gives its path range, o and c; weights are read once per (path, i)
//     and broadcast over the rows).  The SAME kernel in "transposed orientation"
//     (reduction over o, weight stride swapped) is the input gradient.
//   * il_wgrad_kernel: dW_p[i, o] = a_p sum_{n, c} x[n, ii(i, c)] g[n, io(o, c)]: 64x64
//     weight tiles x node splits, (node, c) rows staged in LDS, 4x4 register outer
//     products per thread, per-split partial slabs; il_wreduce_kernel sums the splits in
//     order (deterministic) and applies a_p.
#include "common.h"

#include <cstdio>
#include <cstdlib>

namespace hy {
namespace il {

constexpr int TR = 4;          // rows (nodes) per forward tile (N / 4 workgroups: fills the chip)
constexpr int MAXCOLS = 4096;  // input columns held in LDS (TR * 4096 * 4 B = 64 KB; a MACE
                               // message row after the uvu product is ~1.6 k columns)

// orientation-specific path entry: source column offset, reduction length, weight
// offset / strides (index = w_off + r * w_rs + o * w_os), degree width d, scale a
struct Path {
  int src_off, rlen, w_off, w_rs, w_os, d;
  float a;
};
// output column: paths [p0, p1), output channel o, component c
struct Col {
  int p0, p1, o, c;
};

// U: reduction steps unrolled (weight loads in flight per thread; the kernel is bound by
// their latency at MACE sizes)
// RT: rows (nodes) per workgroup (the LDS tile the host sizes: RT x Din floats)
template <int U, int RT>
__global__ __launch_bounds__(256) void il_fwd_kernel(const float* __restrict__ x, int N, int Din,
                                                     const float* __restrict__ W, const Path* __restrict__ paths,
                                                     const Col* __restrict__ cols, int Dout,
                                                     const float* __restrict__ res, float* __restrict__ out) {
  extern __shared__ float xs[];  // [RT][Din]
  const int n0 = blockIdx.x * RT;
  const int rows = min(RT, N - n0);
  for (int t = threadIdx.x; t < rows * Din; t += 256) xs[t] = x[(int64_t)n0 * Din + t];
  __syncthreads();
  const int j = blockIdx.y * 256 + threadIdx.x;  // one output column per thread
  if (j < Dout) {
    const Col cl = cols[j];
    float acc[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r) acc[r] = 0.f;
    for (int q = cl.p0; q < cl.p1; ++q) {
      const Path P = paths[q];
      const float* Wp = W + P.w_off + (int64_t)cl.o * P.w_os;
      const float* xc = xs + P.src_off + cl.c;
#pragma unroll U
      for (int i = 0; i < P.rlen; ++i) {
        const float w = Wp[(int64_t)i * P.w_rs] * P.a;
        const float* xr = xc + i * P.d;
#pragma unroll
        for (int r = 0; r < RT; ++r) acc[r] = fmaf(xr[r * Din], w, acc[r]);
      }
    }
    if (res != nullptr)
      for (int r = 0; r < rows; ++r) acc[r] += res[(int64_t)(n0 + r) * Dout + j];
    for (int r = 0; r < rows; ++r) out[(int64_t)(n0 + r) * Dout + j] = acc[r];
  }
}

// weight-gradient tile job: path columns (in_off / out_off), sizes, degree width, weight
// offset, and this job's 64x64 tile origin (i0, o0) inside the path's [mi, mo] matrix
struct WJob {
  int in_off, out_off, mi, mo, d, w_off, i0, o0;
};

constexpr int WT = 64, NCH = 8;  // weight tile edge, nodes staged per LDS round

// slab[s][w_off + i * mo + o] = sum_{n in split s, c} x[n, in_off + i*d + c] g[n, out_off + o*d + c]
__global__ __launch_bounds__(256) void il_wgrad_kernel(const float* __restrict__ x, int Din,
                                                       const float* __restrict__ g, int Dout, int N,
                                                       const WJob* __restrict__ jobs, int nodes_per_split,
                                                       float* __restrict__ slab, int64_t numel) {
  __shared__ float xs[NCH * 9][WT];  // (node, c) rows x i  (d <= 9: l <= 4)
  __shared__ float gs[NCH * 9][WT];
  const WJob J = jobs[blockIdx.x];
  const int s = blockIdx.y;
  const int nbeg = s * nodes_per_split, nend = min(N, nbeg + nodes_per_split);
  const int ti = threadIdx.x >> 4, to = threadIdx.x & 15;  // 4 i rows x 4 o cols each
  float acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = 0.f;
  const int d = J.d;
  for (int nb = nbeg; nb < nend; nb += NCH) {
    const int nn = min(NCH, nend - nb);
    const int R = nn * d;
    __syncthreads();
    for (int t = threadIdx.x; t < R * WT; t += 256) {
      const int r = t / WT, k = t % WT;  // row r = (node, c), column k
      const int n = nb + r / d, c = r % d;
      const int i = J.i0 + k, o = J.o0 + k;
      xs[r][k] = i < J.mi ? x[(int64_t)n * Din + J.in_off + i * d + c] : 0.f;
      gs[r][k] = o < J.mo ? g[(int64_t)n * Dout + J.out_off + o * d + c] : 0.f;
    }
    __syncthreads();
    for (int r = 0; r < R; ++r) {
      float xv[4], gv[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) xv[a] = xs[r][4 * ti + a];
#pragma unroll
      for (int b = 0; b < 4; ++b) gv[b] = gs[r][4 * to + b];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = fmaf(xv[a], gv[b], acc[a][b]);
    }
  }
  float* sl = slab + (int64_t)s * numel + J.w_off;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int i = J.i0 + 4 * ti + a;
    if (i >= J.mi) continue;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int o = J.o0 + 4 * to + b;
      if (o < J.mo) sl[(int64_t)i * J.mo + o] = acc[a][b];
    }
  }
}

// dW[k] = scale[k] * sum_s slab[s][k]  (splits summed in order: deterministic)
__global__ void il_wreduce_kernel(const float* __restrict__ slab, int S, int64_t numel,
                                  const float* __restrict__ scale, float* __restrict__ dW) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= numel) return;
  // 8 independent partial chains keep 8 slab loads in flight (the order of the final
  // combine is fixed: deterministic)
  float part[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int s = 0;
  for (; s + 8 <= S; s += 8)
#pragma unroll
    for (int u = 0; u < 8; ++u) part[u] += slab[(int64_t)(s + u) * numel + k];
  for (; s < S; ++s) part[0] += slab[(int64_t)s * numel + k];
  const float acc = ((part[0] + part[1]) + (part[2] + part[3])) + ((part[4] + part[5]) + (part[6] + part[7]));
  dW[k] = acc * scale[k];
}

}  // namespace il

using namespace il;

// x [N, Din] fp32; W flat fp32; paths int32 [P, 7] (last column: float bits of a);
// cols int32 [Dout, 4]; res (optional) fp32 [N, Dout] added to the output
at::Tensor irreps_linear(const at::Tensor& x_, const at::Tensor& W, const at::Tensor& paths, const at::Tensor& cols,
                         const c10::optional<at::Tensor>& res_) {
  at::Tensor x = x_.contiguous();
  HY_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.dim() == 2, "irreps_linear: x [N, Din] fp32");
  HY_CHECK(W.is_cuda() && W.scalar_type() == at::kFloat && W.is_contiguous(), "irreps_linear: W fp32 contiguous");
  HY_CHECK(paths.scalar_type() == at::kInt && paths.dim() == 2 && paths.size(1) == 7 && paths.is_contiguous(),
           "irreps_linear: path table int32 [P, 7]");
  HY_CHECK(cols.scalar_type() == at::kInt && cols.dim() == 2 && cols.size(1) == 4 && cols.is_contiguous(),
           "irreps_linear: column table int32 [Dout, 4]");
  const int64_t N = x.size(0), Din = x.size(1), Dout = cols.size(0);
  HY_CHECK(Din <= MAXCOLS, "irreps_linear: at most 4096 input columns");
  at::Tensor res;
  if (res_.has_value() && res_->defined()) {
    res = res_->contiguous();
    HY_CHECK(res.is_cuda() && res.scalar_type() == at::kFloat && res.dim() == 2 && res.size(0) == N &&
                 res.size(1) == Dout,
             "irreps_linear: res fp32 [N, Dout]");
  }
  auto out = at::empty({N, Dout}, x.options());
  if (N == 0 || Dout == 0) return out;
  static const int unroll = std::getenv("HYDRA_IL_UNROLL") ? std::atoi(std::getenv("HYDRA_IL_UNROLL")) : 8;  // MI355X MACE: 8 > 4 (+0.8%) >> 16 (-14%)
  // HYDRA_IL_ROWS = 8 / 4 / 2 / 1: nodes per workgroup (fewer: more workgroups, weights re-read)
  static const int rows_env = std::getenv("HYDRA_IL_ROWS") ? std::atoi(std::getenv("HYDRA_IL_ROWS")) : 4;
  // 8 rows while the tile fits the 64 KB default LDS allocation
  const int rt = (rows_env >= 8 && 8 * Din * (int64_t)sizeof(float) <= 65536) ? 8
               : (rows_env >= 4 ? 4 : (rows_env >= 2 ? 2 : 1));
  const size_t lds = (size_t)rt * Din * sizeof(float);
  auto* kern = rt == 8 ? (unroll >= 8 ? il_fwd_kernel<8, 8> : il_fwd_kernel<4, 8>)
             : rt == 4 ? (unroll >= 16 ? il_fwd_kernel<16, 4> : (unroll >= 8 ? il_fwd_kernel<8, 4> : il_fwd_kernel<4, 4>))
             : rt == 2 ? (unroll >= 8 ? il_fwd_kernel<8, 2> : il_fwd_kernel<4, 2>)
                       : (unroll >= 8 ? il_fwd_kernel<8, 1> : il_fwd_kernel<4, 1>);
  kern<<<dim3((unsigned)ceil_div(N, rt), (unsigned)ceil_div(Dout, 256)), 256, lds, stream()>>>(x.data_ptr<float>(), (int)N, (int)Din, W.data_ptr<float>(),
                                                         reinterpret_cast<const Path*>(paths.data_ptr()),
                                                         reinterpret_cast<const Col*>(cols.data_ptr()), (int)Dout,
                                                         res.defined() ? res.data_ptr<float>() : nullptr,
                                                         out.data_ptr<float>());
  return out;
}

// dW (flat, like W) of the linear: jobs int32 [J, 8]; scale fp32 [numel] (a_p per element)
at::Tensor irreps_linear_wgrad(const at::Tensor& x_, const at::Tensor& g_, const at::Tensor& jobs,
                               const at::Tensor& scale, int64_t max_d, const c10::optional<at::Tensor>& out) {
  at::Tensor x = x_.contiguous(), g = g_.contiguous();
  HY_CHECK(x.is_cuda() && g.is_cuda() && x.scalar_type() == at::kFloat && g.scalar_type() == at::kFloat &&
               x.dim() == 2 && g.dim() == 2 && x.size(0) == g.size(0),
           "irreps_linear_wgrad: x [N, Din], g [N, Dout] fp32");
  HY_CHECK(jobs.scalar_type() == at::kInt && jobs.dim() == 2 && jobs.size(1) == 8 && jobs.is_contiguous(),
           "irreps_linear_wgrad: job table int32 [J, 8]");
  HY_CHECK(scale.is_cuda() && scale.scalar_type() == at::kFloat && scale.is_contiguous(),
           "irreps_linear_wgrad: scale fp32 [numel]");
  HY_CHECK(max_d >= 1 && max_d <= 9, "irreps_linear_wgrad: l <= 4");
  const int64_t N = x.size(0), numel = scale.numel(), J = jobs.size(0);
  // out: the weight's gradient slot in the step's flat buffer (parallel/gradslots.py)
  at::Tensor dW;
  if (out.has_value() && out->defined()) {
    HY_CHECK(out->is_cuda() && out->scalar_type() == at::kFloat && out->is_contiguous() && out->numel() == numel,
             "irreps_linear_wgrad: out fp32 contiguous [numel]");
    dW = *out;
  } else {
    dW = at::empty({numel}, x.options());
  }
  if (numel == 0) return dW;
  if (N == 0 || J == 0) return dW.zero_();
  // splits: ~512 workgroups over the chip, at least NCH nodes each, at most 128 (the reduce
  // reads every split's slab)
  // HYDRA_IL_WG="target,cap": workgroups aimed for and the split cap (A/B knob)
  static int wg_target = 512, wg_cap = 128;  // MACE on MI355X: 256,64 14.69 k; 512,128 14.84 k; 1024,256 14.86 k
  static bool wg_init = false;
  if (!wg_init) {
    wg_init = true;
    if (const char* e = std::getenv("HYDRA_IL_WG")) {
      int a = 0, c = 0;
      if (std::sscanf(e, "%d,%d", &a, &c) == 2 && a >= 1 && c >= 1 && c <= 256) {
        wg_target = a;
        wg_cap = c;
      }
    }
  }
  int64_t S = std::max<int64_t>(1, std::min<int64_t>({ceil_div(wg_target, J), ceil_div(N, NCH), (int64_t)wg_cap}));
  const int64_t per = ceil_div(N, S);
  S = ceil_div(N, per);
  // every split writes every weight element of every path (partial tiles mask their pad)
  auto slab = at::empty({S, numel}, x.options());
  il_wgrad_kernel<<<dim3((unsigned)J, (unsigned)S), 256, 0, stream()>>>(
      x.data_ptr<float>(), (int)x.size(1), g.data_ptr<float>(), (int)g.size(1), (int)N,
      reinterpret_cast<const WJob*>(jobs.data_ptr()), (int)per, slab.data_ptr<float>(), numel);
  il_wreduce_kernel<<<ceil_div(numel, 256), 256, 0, stream()>>>(slab.data_ptr<float>(), (int)S, numel,
                                                                 scale.data_ptr<float>(), dW.data_ptr<float>());
  return dW;
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("irreps_linear(Tensor x, Tensor W, Tensor paths, Tensor cols, Tensor? res=None) -> Tensor");
  m.def("irreps_linear_wgrad(Tensor x, Tensor g, Tensor jobs, Tensor scale, int max_d, Tensor? out=None) -> Tensor");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("irreps_linear", hy::irreps_linear);
  m.impl("irreps_linear_wgrad", hy::irreps_linear_wgrad);
}
