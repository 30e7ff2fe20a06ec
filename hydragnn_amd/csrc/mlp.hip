// Fused small-batch MLP chain (graph-level heads) for gfx950.
//
// The graph heads of every HydraGNN model (Base.py:_multihead, shared layers ->
// head layers -> output Linear, ReLU between) run on G = batch-size rows (32-ish)
// after pooling.  As torch ops that is ~6 launches per Linear+ReLU forward and
// backward (addmm, relu, mm x2, bias sum, threshold_backward, accumulation), i.e.
// ~30 launches of a few microseconds each for a few hundred kFLOP of work.  Here
// the chain is ONE forward launch and TWO backward launches.
//
// Rows are independent in the forward and in the input-gradient chain, so
// workgroups own blocks of kMlpRows rows.  Each workgroup first stages everything
// it reads (all layers' weights + its rows) into LDS with all loads in flight
// (one round of L2 latency), then runs the layer chain out of LDS -- a single
// workgroup doing all rows was bound by one CU's LDS bandwidth (~30 us).
//   forward : weights transposed [i][o] in LDS, activations ping-pong through LDS,
//             every layer's post-activation output is saved for backward;
//   backward: the workgroup walks the layers in reverse for its rows: partial
//             dW = dy^T a_in and db = sum_r dy over its rows, da = dy W (masked by
//             the previous layer's ReLU); partials are then summed over the row
//             blocks in a fixed order by a second launch -> deterministic.
// Limits (host checks, Python falls back to torch beyond them): <= 8 layers,
// widths <= 128, G <= 1024 rows, weights <= ~150 KB of LDS.
#include "common.h"

namespace hy {

constexpr int kMlpMaxLayers = 8;
constexpr int kMlpMaxDim = 128;  // layer widths
constexpr int kMlpMaxG = 1024;   // rows
constexpr int kMlpRows = 4;      // rows per workgroup
constexpr int kMlpThreads = 256;
constexpr int kMlpBatch = 16;    // staged loads in flight per thread
constexpr size_t kMlpMaxLds = 159 * 1024;  // + the small static table block

struct MlpArgs {
  int n;                                // layers
  int dims[kMlpMaxLayers + 1];          // dims[0] = input width
  int relu[kMlpMaxLayers];              // ReLU after layer l
  int aoff[kMlpMaxLayers + 1];          // column offset of layer l's output in acts (aoff[n] = S)
  int woff[kMlpMaxLayers + 1];          // offset of layer l's weights (woff[n] = total weights)
  int goff[kMlpMaxLayers + 1];          // offset of layer l's (dW, db) in the gradient image
  const float* W[kMlpMaxLayers];        // [dims[l+1], dims[l]]
  const float* b[kMlpMaxLayers];        // [dims[l+1]]
};

// Stage cnt floats src -> LDS with kMlpBatch loads in flight per thread.  The loads
// are unconditional (index clamped into range) and only the LDS stores are guarded:
// a guarded (branchy) load makes the compiler drain the memory counter at every
// branch join, which serialised the first version into one L2/MALL latency per
// element (~30 us for a 10k-float staging pass).
template <typename Dst>
__device__ __forceinline__ void stage_seg(const float* __restrict__ src, int cnt, Dst dst) {
  for (int base = threadIdx.x; base < cnt; base += kMlpBatch * kMlpThreads) {
    float v[kMlpBatch];
#pragma unroll
    for (int k = 0; k < kMlpBatch; ++k) v[k] = src[min(base + k * kMlpThreads, cnt - 1)];
#pragma unroll
    for (int k = 0; k < kMlpBatch; ++k) {
      const int idx = base + k * kMlpThreads;
      if (idx < cnt) dst(idx, v[k]);
    }
  }
}

__device__ __forceinline__ int max_width(const MlpArgs& a) {
  int m = 1;
  for (int l = 0; l <= a.n; ++l) m = max(m, a.dims[l]);
  return m;
}

// LDS: weights^T per layer [i][o] (woff) | buf[2][kMlpRows][md + 1]
__global__ void __launch_bounds__(kMlpThreads) mlp_fwd_kernel(const float* __restrict__ x, int G, MlpArgs a,
                                                              float* __restrict__ acts) {
  extern __shared__ float sm[];
  const int md = max_width(a) + 1;
  const int n = a.n, nw = a.woff[n], S = a.aoff[n], D0 = a.dims[0];
  float* WS = sm;
  float* buf = sm + nw;
  const int r0 = blockIdx.x * kMlpRows;
  const int nr = min(kMlpRows, G - r0);
  for (int l = 0; l < n; ++l) {  // weights, transposed to [i][o]
    const int I = a.dims[l], O = a.dims[l + 1];
    float* dst = WS + a.woff[l];
    stage_seg(a.W[l], O * I, [&](int idx, float v) { dst[(idx % I) * O + idx / I] = v; });
  }
  stage_seg(x + (int64_t)r0 * D0, nr * D0, [&](int idx, float v) { buf[(idx / D0) * md + idx % D0] = v; });
  int cur = 0;
  for (int l = 0; l < n; ++l) {
    __syncthreads();
    const int I = a.dims[l], O = a.dims[l + 1];
    const float* __restrict__ bb = a.b[l];
    const float* Wl = WS + a.woff[l];
    const float* in = buf + cur * kMlpRows * md;
    float* out = buf + (cur ^ 1) * kMlpRows * md;
    for (int idx = threadIdx.x; idx < nr * O; idx += kMlpThreads) {
      const int r = idx / O, o = idx % O;
      float acc = bb[o];
      const float* xr = in + r * md;
#pragma unroll 8
      for (int i = 0; i < I; ++i) acc = fmaf(xr[i], Wl[i * O + o], acc);
      if (a.relu[l]) acc = fmaxf(acc, 0.f);
      out[r * md + o] = acc;
      acts[(int64_t)(r0 + r) * S + a.aoff[l] + o] = acc;
    }
    cur ^= 1;
  }
}

// LDS: weights per layer [o][i] (woff) | acts rows [kMlpRows][S] | x rows [kMlpRows][D0] | dy [kMlpRows][md]
// part: [blocks][goff[n]] with layer l's dW at goff[l] and db at goff[l] + O*I
__global__ void __launch_bounds__(kMlpThreads) mlp_bwd_kernel(const float* __restrict__ dout,
                                                              const float* __restrict__ x,
                                                              const float* __restrict__ acts, int G, MlpArgs a,
                                                              float* __restrict__ part, float* __restrict__ dx) {
  extern __shared__ float sm[];
  const int md = max_width(a) + 1;
  const int n = a.n, nw = a.woff[n], S = a.aoff[n], D0 = a.dims[0];
  const int r0 = blockIdx.x * kMlpRows;
  const int nr = min(kMlpRows, G - r0);
  float* WS = sm;
  float* AS = WS + nw;
  float* XS = AS + kMlpRows * S;
  float* DY = XS + kMlpRows * D0;
  float* P = part + (int64_t)blockIdx.x * a.goff[n];
  const int t = threadIdx.x;
  for (int l = 0; l < n; ++l) {  // weights, natural [o][i]
    float* dst = WS + a.woff[l];
    stage_seg(a.W[l], a.dims[l] * a.dims[l + 1], [&](int idx, float v) { dst[idx] = v; });
  }
  stage_seg(acts + (int64_t)r0 * S, nr * S, [&](int idx, float v) { AS[idx] = v; });
  stage_seg(x + (int64_t)r0 * D0, nr * D0, [&](int idx, float v) { XS[idx] = v; });
  __syncthreads();
  {
    const int O = a.dims[n];
    const int off = a.aoff[n - 1];
    const bool rl = a.relu[n - 1];
    for (int idx = t; idx < nr * O; idx += kMlpThreads) {
      const int r = idx / O, o = idx % O;
      const float v = dout[(int64_t)r0 * O + idx];
      DY[r * md + o] = rl && AS[r * S + off + o] <= 0.f ? 0.f : v;
    }
  }
  __syncthreads();
  for (int l = n - 1; l >= 0; --l) {
    const int I = a.dims[l], O = a.dims[l + 1];
    const float* ain = l == 0 ? XS : AS + a.aoff[l - 1];
    const int lda = l == 0 ? D0 : S;
    const float* Wl = WS + a.woff[l];
    float* Pl = P + a.goff[l];
    // partial dW[o, i] = sum_{r in block} dy[r, o] ain[r, i];  db[o] = sum_r dy[r, o]
    for (int idx = t; idx < O * I + O; idx += kMlpThreads) {
      float acc = 0.f;
      if (idx < O * I) {
        const int o = idx / I, i = idx % I;
        for (int r = 0; r < nr; ++r) acc = fmaf(DY[r * md + o], ain[r * lda + i], acc);
      } else {
        const int o = idx - O * I;
        for (int r = 0; r < nr; ++r) acc += DY[r * md + o];
      }
      Pl[idx] = acc;
    }
    // da[r, i] = sum_o dy[r, o] W[o, i]  (x ReLU'(ain) for the previous layer)
    const bool mask = l > 0 && a.relu[l - 1];
    constexpr int kRegs = kMlpRows * kMlpMaxDim / kMlpThreads;
    float da[kRegs];
#pragma unroll
    for (int k = 0; k < kRegs; ++k) {
      const int idx = t + k * kMlpThreads;
      float acc = 0.f;
      if (idx < nr * I) {
        const int r = idx / I, i = idx % I;
        if (!mask || ain[r * lda + i] > 0.f) {
#pragma unroll 8
          for (int o = 0; o < O; ++o) acc = fmaf(DY[r * md + o], Wl[o * I + i], acc);
        }
      }
      da[k] = acc;
    }
    __syncthreads();  // everyone done reading DY
#pragma unroll
    for (int k = 0; k < kRegs; ++k) {
      const int idx = t + k * kMlpThreads;
      if (idx < nr * I) {
        if (l == 0)
          dx[(int64_t)r0 * I + idx] = da[k];
        else
          DY[(idx / I) * md + idx % I] = da[k];
      }
    }
    __syncthreads();
  }
}

// out[j] = sum_b part[b * n + j] over the row blocks, fixed order
__global__ void __launch_bounds__(256) mlp_sum_kernel(const float* __restrict__ part, int nb, int n,
                                                      float* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  float a0 = 0.f, a1 = 0.f;
  int b = 0;
  for (; b + 1 < nb; b += 2) {
    a0 += part[(int64_t)b * n + j];
    a1 += part[(int64_t)(b + 1) * n + j];
  }
  if (b < nb) a0 += part[(int64_t)b * n + j];
  out[j] = a0 + a1;
}

static MlpArgs make_args(const at::Tensor& x, const std::vector<at::Tensor>& Ws, const std::vector<at::Tensor>& bs,
                         const std::vector<int64_t>& relu) {
  const int n = (int)Ws.size();
  HY_CHECK(n >= 1 && n <= kMlpMaxLayers && (int)bs.size() == n && (int)relu.size() == n,
           "mlp: 1..8 layers, one bias and one relu flag per layer");
  MlpArgs a{};
  a.n = n;
  a.dims[0] = (int)x.size(1);
  HY_CHECK(a.dims[0] <= kMlpMaxDim, "mlp: widths up to 128");
  int off = 0, woff = 0, goff = 0;
  for (int l = 0; l < n; ++l) {
    const auto& W = Ws[l];
    HY_CHECK(W.is_cuda() && W.scalar_type() == at::kFloat && W.is_contiguous() && W.dim() == 2 &&
                 W.size(1) == a.dims[l],
             "mlp: layer weights must be contiguous fp32 [out, in] chaining from the input width");
    HY_CHECK(bs[l].is_contiguous() && bs[l].numel() == W.size(0) && bs[l].scalar_type() == at::kFloat,
             "mlp: bias must be contiguous fp32 [out]");
    a.dims[l + 1] = (int)W.size(0);
    HY_CHECK(a.dims[l + 1] <= kMlpMaxDim, "mlp: widths up to 128");
    a.relu[l] = relu[l] ? 1 : 0;
    a.aoff[l] = off;
    a.woff[l] = woff;
    a.goff[l] = goff;
    off += a.dims[l + 1];
    woff += a.dims[l + 1] * a.dims[l];
    goff += a.dims[l + 1] * (a.dims[l] + 1);
    a.W[l] = W.data_ptr<float>();
    a.b[l] = bs[l].data_ptr<float>();
  }
  a.aoff[n] = off;
  a.woff[n] = woff;
  a.goff[n] = goff;
  return a;
}

static int host_max_width(const MlpArgs& a) {
  int m = 1;
  for (int l = 0; l <= a.n; ++l) m = std::max(m, a.dims[l]);
  return m;
}

// keep in sync with ops/mlp.py:_lds_ok
static size_t fwd_lds(const MlpArgs& a) {
  return sizeof(float) * ((size_t)a.woff[a.n] + 2 * (size_t)kMlpRows * (host_max_width(a) + 1));
}

// keep in sync with ops/mlp.py:_lds_ok
static size_t bwd_lds(const MlpArgs& a) {
  return sizeof(float) *
         ((size_t)a.woff[a.n] + (size_t)kMlpRows * (a.aoff[a.n] + a.dims[0] + host_max_width(a) + 1));
}

static void set_lds_limits() {
  static bool once = [] {
    hipFuncSetAttribute((const void*)mlp_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMlpMaxLds);
    hipFuncSetAttribute((const void*)mlp_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMlpMaxLds);
    return true;
  }();
  (void)once;
}

std::tuple<at::Tensor, at::Tensor> mlp_fwd(const at::Tensor& x_, at::TensorList Ws_, at::TensorList bs_,
                                           at::IntArrayRef relu) {
  HY_CHECK_CUDA(x_);
  auto x = x_.contiguous();
  HY_CHECK_F32(x);
  HY_CHECK(x.dim() == 2, "mlp: x must be [G, D]");
  std::vector<at::Tensor> Ws(Ws_.begin(), Ws_.end()), bs(bs_.begin(), bs_.end());
  auto a = make_args(x, Ws, bs, relu.vec());
  const int64_t G = x.size(0);
  HY_CHECK(G <= kMlpMaxG, "mlp_fwd: at most 1024 rows");
  const size_t lds = fwd_lds(a);
  HY_CHECK(lds <= kMlpMaxLds, "mlp_fwd: weights exceed the LDS budget");
  set_lds_limits();
  auto acts = at::empty({G, a.aoff[a.n]}, x.options());
  if (G > 0)
    mlp_fwd_kernel<<<ceil_div(G, kMlpRows), kMlpThreads, lds, stream()>>>(x.data_ptr<float>(), (int)G, a,
                                                                          acts.data_ptr<float>());
  auto out = acts.narrow(1, a.aoff[a.n - 1], a.dims[a.n]);
  return {out, acts};
}

std::tuple<at::Tensor, std::vector<at::Tensor>, std::vector<at::Tensor>> mlp_bwd(const at::Tensor& dout_,
                                                                                 const at::Tensor& x_,
                                                                                 const at::Tensor& acts,
                                                                                 at::TensorList Ws_,
                                                                                 at::TensorList bs_,
                                                                                 at::IntArrayRef relu) {
  auto x = x_.contiguous(), dout = dout_.contiguous();
  std::vector<at::Tensor> Ws(Ws_.begin(), Ws_.end()), bs(bs_.begin(), bs_.end());
  auto a = make_args(x, Ws, bs, relu.vec());
  const int64_t G = x.size(0);
  HY_CHECK(dout.dim() == 2 && dout.size(0) == G && dout.size(1) == a.dims[a.n], "mlp_bwd: dout shape");
  HY_CHECK(acts.is_contiguous() && acts.size(0) == G && acts.size(1) == a.aoff[a.n], "mlp_bwd: acts shape");
  HY_CHECK(G <= kMlpMaxG, "mlp_bwd: at most 1024 rows");
  const size_t lds = bwd_lds(a);
  HY_CHECK(lds <= kMlpMaxLds, "mlp_bwd: chain exceeds the LDS budget");
  set_lds_limits();
  const int ng = a.goff[a.n];
  auto flat = at::empty({ng}, x.options());  // [dW_0 | db_0 | dW_1 | db_1 | ...]
  std::vector<at::Tensor> dWs, dbs;
  for (int l = 0; l < a.n; ++l) {
    const int O = a.dims[l + 1], I = a.dims[l];
    dWs.push_back(flat.narrow(0, a.goff[l], O * I).view({O, I}));
    dbs.push_back(flat.narrow(0, a.goff[l] + O * I, O));
  }
  auto dx = at::empty_like(x);
  if (G == 0) {
    flat.zero_();
    return {dx, dWs, dbs};
  }
  const int nb = ceil_div(G, kMlpRows);
  auto part = at::empty({nb, ng}, x.options());
  mlp_bwd_kernel<<<nb, kMlpThreads, lds, stream()>>>(dout.data_ptr<float>(), x.data_ptr<float>(),
                                                      acts.data_ptr<float>(), (int)G, a, part.data_ptr<float>(),
                                                      dx.data_ptr<float>());
  mlp_sum_kernel<<<ceil_div(ng, 256), 256, 0, stream()>>>(part.data_ptr<float>(), nb, ng, flat.data_ptr<float>());
  return {dx, dWs, dbs};
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("mlp_fwd(Tensor x, Tensor[] Ws, Tensor[] bs, int[] relu) -> (Tensor, Tensor)");
  m.def(
      "mlp_bwd(Tensor dout, Tensor x, Tensor acts, Tensor[] Ws, Tensor[] bs, int[] relu) -> "
      "(Tensor, Tensor[], Tensor[])");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("mlp_fwd", hy::mlp_fwd);
  m.impl("mlp_bwd", hy::mlp_bwd);
}
