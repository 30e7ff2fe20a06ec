// Fused small-batch MLP chain (graph-level heads) for gfx950.
//
// The graph heads of every HydraGNN model (Base.py:_multihead, shared layers ->
// head layers -> output Linear, ReLU between) run on G = batch-size rows (32-ish)
// after pooling.  As torch ops that is ~6 launches per Linear+ReLU forward and
// backward (addmm, relu, mm x2, bias sum, threshold_backward, accumulation), i.e.
// ~30 launches of a few microseconds each for a few hundred kFLOP of work.  Here
// the whole chain is ONE forward and ONE backward launch.
//
// The work is tiny; what costs time is memory latency between dependent layers.
// So each kernel first stages EVERYTHING it will read (all layers' weights, and in
// the backward also the saved activations and the input) into LDS with all loads
// in flight at once (one round of L2/HBM latency), then runs the layer chain out
// of LDS (the first version staged per layer: 5 serial latency rounds, ~40 us).
//   forward : one workgroup (1024 threads); weights transposed [i][o] in LDS,
//             activations ping-pong through LDS, each layer's post-activation
//             output is saved for backward;
//   backward: ONE workgroup (1024 threads) walks the layers in reverse: dW =
//             dy^T a_in, db = sum_r dy, da = dy W (masked by the previous layer's
//             ReLU); fixed-order loops over rows -> deterministic, no atomics.
// Limits (host checks, Python falls back to torch beyond them): <= 8 layers,
// widths <= 128, G <= 64 rows, LDS footprint <= 160 KB.
#include "common.h"

namespace hy {

constexpr int kMlpMaxLayers = 8;
constexpr int kMlpMaxDim = 128;  // layer widths
constexpr int kMlpMaxG = 64;     // rows (graphs) for the one-workgroup backward
constexpr int kMlpThreads = 1024;  // one workgroup runs the whole chain
constexpr int kMlpBatch = 16;      // staged loads in flight per thread
constexpr int kMlpRegs = kMlpMaxG * kMlpMaxDim / kMlpThreads;  // da entries per thread
constexpr size_t kMlpMaxLds = 159 * 1024;  // + the small static table block

struct MlpArgs {
  int n;                                // layers
  int dims[kMlpMaxLayers + 1];          // dims[0] = input width
  int relu[kMlpMaxLayers];              // ReLU after layer l
  int aoff[kMlpMaxLayers + 1];          // column offset of layer l's output in acts (aoff[n] = S)
  int woff[kMlpMaxLayers + 1];          // offset of layer l's weights in the LDS image (woff[n] = total)
  const float* W[kMlpMaxLayers];        // [dims[l+1], dims[l]]
  const float* b[kMlpMaxLayers];        // [dims[l+1]]
};

struct MlpGrads {
  float* dW[kMlpMaxLayers];
  float* db[kMlpMaxLayers];
};

// Per-lane lookups into the argument tables (which layer owns staged element idx)
// go through a small LDS copy: indexing the by-value kernel-argument struct with a
// lane-varying index makes the compiler copy it to scratch.
struct MlpTables {
  const float* W[kMlpMaxLayers];
  int woff[kMlpMaxLayers + 1];
  int dims[kMlpMaxLayers + 1];
};

__device__ __forceinline__ void load_tables(const MlpArgs& a, MlpTables& t) {
  if (threadIdx.x == 0) {
    for (int l = 0; l < kMlpMaxLayers; ++l) t.W[l] = a.W[l];
    for (int l = 0; l <= kMlpMaxLayers; ++l) {
      t.woff[l] = a.woff[l];
      t.dims[l] = a.dims[l];
    }
  }
  __syncthreads();
}

__device__ __forceinline__ int layer_of(const MlpTables& t, int n, int idx) {
  int l = 0;
  while (l + 1 < n && idx >= t.woff[l + 1]) ++l;
  return l;
}

__device__ __forceinline__ int max_width(const MlpArgs& a) {
  int m = 1;
  for (int l = 0; l <= a.n; ++l) m = max(m, a.dims[l]);
  return m;
}

// LDS: weights^T per layer [i][o] (woff) | buf[2][G][md + 1]
__global__ void __launch_bounds__(kMlpThreads) mlp_fwd_kernel(const float* __restrict__ x, int G, MlpArgs a,
                                                      float* __restrict__ acts) {
  extern __shared__ float sm[];
  const int md = max_width(a) + 1;
  float* WS = sm;
  float* buf = sm + a.woff[a.n];
  const int r0 = 0, nr = G;
  const int S = a.aoff[a.n];
  const int D0 = a.dims[0];
  const int nw = a.woff[a.n];
  // one combined staging pass: all weights (transposed), then this block's input rows
  __shared__ MlpTables tb;
  load_tables(a, tb);
  const int n = a.n;
  for (int base = threadIdx.x; base < nw + nr * D0; base += kMlpBatch * kMlpThreads) {
    float v[kMlpBatch];
#pragma unroll
    for (int k = 0; k < kMlpBatch; ++k) {
      const int idx = base + k * kMlpThreads;
      v[k] = 0.f;
      if (idx < nw) {
        const int l = layer_of(tb, n, idx);
        v[k] = tb.W[l][idx - tb.woff[l]];
      } else if (idx < nw + nr * D0) {
        v[k] = x[(int64_t)r0 * D0 + (idx - nw)];
      }
    }
#pragma unroll
    for (int k = 0; k < kMlpBatch; ++k) {
      const int idx = base + k * kMlpThreads;
      if (idx < nw) {
        const int l = layer_of(tb, n, idx);
        const int q = idx - tb.woff[l], I = tb.dims[l], O = tb.dims[l + 1];
        WS[tb.woff[l] + (q % I) * O + q / I] = v[k];
      } else if (idx < nw + nr * D0) {
        const int q = idx - nw;
        buf[(q / D0) * md + q % D0] = v[k];
      }
    }
  }
  int cur = 0;
  for (int l = 0; l < a.n; ++l) {
    __syncthreads();
    const int I = a.dims[l], O = a.dims[l + 1];
    const float* __restrict__ bb = a.b[l];
    const float* Wl = WS + a.woff[l];
    const float* in = buf + cur * G * md;
    float* out = buf + (cur ^ 1) * G * md;
    for (int idx = threadIdx.x; idx < nr * O; idx += blockDim.x) {
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

// LDS: weights per layer [o][i] (woff) | acts [G][S] | x [G][D0] | dy [G][md + 1]
__global__ void __launch_bounds__(kMlpThreads) mlp_bwd_kernel(const float* __restrict__ dout,
                                                                 const float* __restrict__ x,
                                                                 const float* __restrict__ acts, int G, MlpArgs a,
                                                                 MlpGrads g, float* __restrict__ dx) {
  extern __shared__ float sm[];
  const int md = max_width(a) + 1;
  const int S = a.aoff[a.n];
  const int D0 = a.dims[0];
  const int nw = a.woff[a.n];
  float* WS = sm;
  float* AS = WS + nw;
  float* XS = AS + G * S;
  float* DY = XS + G * D0;
  const int t = threadIdx.x;
  const int na = G * S, nx = G * D0;
  __shared__ MlpTables tb;
  load_tables(a, tb);
  const int n = a.n;
  for (int base = t; base < nw + na + nx; base += kMlpBatch * kMlpThreads) {
    float v[kMlpBatch];
#pragma unroll
    for (int k = 0; k < kMlpBatch; ++k) {
      const int idx = base + k * kMlpThreads;
      v[k] = 0.f;
      if (idx < nw) {
        const int l = layer_of(tb, n, idx);
        v[k] = tb.W[l][idx - tb.woff[l]];
      } else if (idx < nw + na) {
        v[k] = acts[idx - nw];
      } else if (idx < nw + na + nx) {
        v[k] = x[idx - nw - na];
      }
    }
#pragma unroll
    for (int k = 0; k < kMlpBatch; ++k) {
      const int idx = base + k * kMlpThreads;
      if (idx < nw + na + nx) sm[idx] = v[k];
    }
  }
  __syncthreads();
  {
    const int O = a.dims[a.n];
    const int off = a.aoff[a.n - 1];
    const bool rl = a.relu[a.n - 1];
    for (int idx = t; idx < G * O; idx += kMlpThreads) {
      const int r = idx / O, o = idx % O;
      const float v = dout[idx];
      DY[r * md + o] = rl && AS[r * S + off + o] <= 0.f ? 0.f : v;
    }
  }
  __syncthreads();
  for (int l = a.n - 1; l >= 0; --l) {
    const int I = a.dims[l], O = a.dims[l + 1];
    const float* ain = l == 0 ? XS : AS + a.aoff[l - 1];
    const int lda = l == 0 ? D0 : S;
    const float* Wl = WS + a.woff[l];
    // dW[o, i] = sum_r dy[r, o] ain[r, i];  db[o] = sum_r dy[r, o]
    for (int idx = t; idx < O * I + O; idx += kMlpThreads) {
      float acc = 0.f;
      if (idx < O * I) {
        const int o = idx / I, i = idx % I;
#pragma unroll 8
        for (int r = 0; r < G; ++r) acc = fmaf(DY[r * md + o], ain[r * lda + i], acc);
        g.dW[l][idx] = acc;
      } else {
        const int o = idx - O * I;
#pragma unroll 8
        for (int r = 0; r < G; ++r) acc += DY[r * md + o];
        g.db[l][o] = acc;
      }
    }
    // da[r, i] = sum_o dy[r, o] W[o, i]  (x ReLU'(ain) for the previous layer), held in registers
    const bool mask = l > 0 && a.relu[l - 1];
    float da[kMlpRegs];
#pragma unroll
    for (int k = 0; k < kMlpRegs; ++k) {
      const int idx = t + k * kMlpThreads;
      float acc = 0.f;
      if (idx < G * I) {
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
    for (int k = 0; k < kMlpRegs; ++k) {
      const int idx = t + k * kMlpThreads;
      if (idx < G * I) {
        if (l == 0)
          dx[idx] = da[k];
        else
          DY[(idx / I) * md + idx % I] = da[k];
      }
    }
    __syncthreads();
  }
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
  int off = 0, woff = 0;
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
    off += a.dims[l + 1];
    woff += a.dims[l + 1] * a.dims[l];
    a.W[l] = W.data_ptr<float>();
    a.b[l] = bs[l].data_ptr<float>();
  }
  a.aoff[n] = off;
  a.woff[n] = woff;
  return a;
}

static int host_max_width(const MlpArgs& a) {
  int m = 1;
  for (int l = 0; l <= a.n; ++l) m = std::max(m, a.dims[l]);
  return m;
}

// keep in sync with ops/mlp.py:_lds_ok
static size_t fwd_lds(const MlpArgs& a, int64_t G) {
  return sizeof(float) * ((size_t)a.woff[a.n] + 2 * (size_t)G * (host_max_width(a) + 1));
}

// keep in sync with ops/mlp.py:_lds_ok
static size_t bwd_lds(const MlpArgs& a, int64_t G) {
  return sizeof(float) * ((size_t)a.woff[a.n] + (size_t)G * (a.aoff[a.n] + a.dims[0] + host_max_width(a) + 1));
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
  HY_CHECK(G <= kMlpMaxG, "mlp_fwd: at most 64 rows");
  const size_t lds = fwd_lds(a, G);
  HY_CHECK(lds <= kMlpMaxLds, "mlp_fwd: weights exceed the LDS budget");
  set_lds_limits();
  auto acts = at::empty({G, a.aoff[a.n]}, x.options());
  if (G > 0)
    mlp_fwd_kernel<<<1, kMlpThreads, lds, stream()>>>(x.data_ptr<float>(), (int)G, a,
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
  HY_CHECK(G <= kMlpMaxG, "mlp_bwd: at most 64 rows");
  const size_t lds = bwd_lds(a, G);
  HY_CHECK(lds <= kMlpMaxLds, "mlp_bwd: chain exceeds the LDS budget");
  set_lds_limits();
  MlpGrads g{};
  std::vector<at::Tensor> dWs, dbs;
  for (int l = 0; l < a.n; ++l) {
    dWs.push_back(at::empty_like(Ws[l]));
    dbs.push_back(at::empty_like(bs[l]));
    g.dW[l] = dWs.back().data_ptr<float>();
    g.db[l] = dbs.back().data_ptr<float>();
  }
  auto dx = at::empty_like(x);
  if (G == 0) {
    for (auto& t : dWs) t.zero_();
    for (auto& t : dbs) t.zero_();
    return {dx, dWs, dbs};
  }
  mlp_bwd_kernel<<<1, kMlpThreads, lds, stream()>>>(dout.data_ptr<float>(), x.data_ptr<float>(),
                                                        acts.data_ptr<float>(), (int)G, a, g, dx.data_ptr<float>());
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
