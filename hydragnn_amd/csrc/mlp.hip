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

#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <utility>

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

// csrc/loss.hip loss_term (0 mse, 1 mae, 2 rmse, 3 smooth_l1)
__device__ __forceinline__ float loss_term_hl(int kind, float d) {
  const float a = fabsf(d);
  return kind == 1 ? a : (kind == 3 ? (a < 1.f ? 0.5f * d * d : a - 0.5f) : d * d);
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

// ------------------------------------------------------------------------------------
// Head + loss in one workgroup (the training step's graph-level decoder, Base.py:_multihead
// followed by Base.loss_hpweighted's masked loss, csrc/loss.hip):
//   forward : pred = MLP(x), loss = masked mean of loss_term(pred - target)
//   backward: dpred = g dloss/dpred, then the chain backward with COMPLETE weight
//             gradients (all rows are in the workgroup: no partials, no sum pass).
// For the ~32 pooled rows of a training batch the old path was 7 launches (MLP fwd,
// loss fwd, grad seed fill, loss bwd, MLP bwd, partial sum, copy), ~70 us of serial
// dependent launches between the encoder's forward and backward; this is 2.
// One 1024-thread workgroup; everything lives in LDS: W per layer natural [o][i],
// X [G][D0], every layer's activation A [G][S] and two dY buffers [G][md].
// The backward launch recomputes the (tiny) forward chain instead of reading it back.
typedef float f4v_hl __attribute__((ext_vector_type(4)));
constexpr int kHlThreads = 1024;
constexpr int kHlWaves = kHlThreads / 64;
constexpr int kHlBatch = 16;  // staged loads in flight per thread
constexpr size_t kHlMaxLds = 150 * 1024;

// Every layer product runs on v_mfma_f32_16x16x4f32 (exact fp32): a 16x16 output tile per
// wave, operands read straight from LDS.  (A VALU form, one output per lane, needed two LDS
// reads per FMA and was LDS-issue bound: ~6 us per 33 x 50 x 64 layer.)  Every LDS matrix
// is [rows padded to 16][cols padded to 16, + 1] with zeroed padding, so tiles never need
// bounds checks and reads along either dimension are bank-conflict free (odd row stride).
__device__ __host__ __forceinline__ int hl_r16(int v) { return (v + 15) / 16 * 16; }
__device__ __host__ __forceinline__ int hl_ld(int cols) { return hl_r16(cols) + 1; }

struct HlLayout {  // float offsets into the dynamic LDS block
  int w[kMlpMaxLayers];      // W_l   [r16(O)][ld(I)]
  int b[kMlpMaxLayers];      // b_l   [r16(O)]
  int act[kMlpMaxLayers];    // A_l   [Gp][ld(O)]   (layer l's output)
  int x, dy, dy2, tg, mk, total, Gp, ldy;  // tg: target [G][Do]; mk: row mask [Gp] (1 / 0)
};

// Every head kernel is instantiated per layer count NL (1..kMlpMaxLayers): the layer loops
// unroll, each layer's widths / offsets are compile-time-indexed (registers and hoisted
// kernel-argument loads instead of a dependent load chain at every layer), and the layout is
// computed by every thread (a runtime-indexed struct would live in scratch memory).
template <int NL>
__device__ __host__ inline void hl_layout_into(HlLayout& L, const MlpArgs& a, int G) {
  L.Gp = hl_r16(G);
  int o = 0, mw = a.dims[0];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    L.w[l] = o;
    o += hl_r16(a.dims[l + 1]) * hl_ld(a.dims[l]);
    mw = a.dims[l + 1] > mw ? a.dims[l + 1] : mw;
  }
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    L.b[l] = o;
    o += hl_r16(a.dims[l + 1]);
  }
  L.x = o;
  o += L.Gp * hl_ld(a.dims[0]);
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    L.act[l] = o;
    o += L.Gp * hl_ld(a.dims[l + 1]);
  }
  L.ldy = hl_ld(mw);
  L.dy = o;
  o += L.Gp * L.ldy;
  L.dy2 = o;
  o += L.Gp * L.ldy;
  L.tg = o;
  o += G * a.dims[NL];
  L.mk = o;
  o += L.Gp;
  L.total = o;
}

template <int NL>
__device__ __host__ inline HlLayout hl_layout(const MlpArgs& a, int G) {
  HlLayout L{};
  hl_layout_into<NL>(L, a, G);
  return L;
}

__device__ __forceinline__ f4v_hl hl_mfma(float a, float b, f4v_hl c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// sum over k-steps 0..K4-1 of mfma(ap[k sa], bp[k sb]): the LDS reads of 8 steps are
// issued together (one latency per group instead of one per step) and two accumulators
// alternate (dependent-accumulator latency); steps past K4 read nothing and add zero
__device__ __forceinline__ f4v_hl hl_dot(const float* ap, int sa, const float* bp, int sb, int K4) {
  f4v_hl a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
  for (int k = 0; k < K4; k += 8) {
    float x[8], y[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = k + j < K4;
      x[j] = ok ? ap[(k + j) * sa] : 0.f;
      y[j] = ok ? bp[(k + j) * sb] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      a0 = hl_mfma(x[j], y[j], a0);
      a1 = hl_mfma(x[j + 1], y[j + 1], a1);
    }
  }
  return a0 + a1;
}

// workgroup barrier that waits for this wave's LDS traffic only: the global stores of
// activations / gradients stay in flight (nothing in these kernels reads them back), where
// __syncthreads' release fence would drain them at every layer
// optional cycle stamps (tools/bench_head_loss.py --stamps): thread 0 records the shader
// clock at phase boundaries into dbg[i]
__device__ __forceinline__ void hl_stamp(long long* dbg, int i) {
  if (dbg != nullptr && threadIdx.x == 0) dbg[i] = (long long)__builtin_amdgcn_s_memtime();
}

__device__ __forceinline__ void hl_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Zero the whole block, then copy every weight and bias, the input rows, the targets and
// (backward) the saved activations straight into it with LDS-DMA (global_load_lds_dword: no
// staging registers, no ds_write pass): one wave instruction per (matrix row, 64-column
// chunk), rows dealt round-robin to the waves (continuing across matrices), every copy in
// flight together, so staging costs ~one memory latency and nothing later in the kernel
// reads global memory.  The matrix loop is unrolled over the layers (NL): its parameters
// are compile-time kernel-argument offsets, loaded once, not searched per row.
template <int NL>
__device__ void hl_stage(const MlpArgs& a, const HlLayout& L, const float* __restrict__ x,
                         const float* __restrict__ acts, const float* __restrict__ target,
                         const bool* __restrict__ mask, int G, float* sm) {
  for (int e = threadIdx.x; e < L.total; e += kHlThreads) sm[e] = 0.f;
  hl_sync();  // zero fill done before any copy lands
  // the row mask (bool -> 1 / 0; padding rows stay 0)
  for (int r = threadIdx.x; r < G; r += kHlThreads) sm[L.mk + r] = (mask == nullptr || mask[r]) ? 1.f : 0.f;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  int base = 0;  // rows dealt so far (wave-uniform)
  auto rows = [&](const float* src, int n, int width, int sld, int dst, int dld) {
    // this wave's rows r = (wv - base) mod kHlWaves, + kHlWaves, ...
    for (int r = (wv - base % kHlWaves + kHlWaves) % kHlWaves; r < n; r += kHlWaves)
      for (int c0 = 0; c0 < width; c0 += 64)
        if (c0 + lane < width)
          __builtin_amdgcn_global_load_lds(
              (__attribute__((address_space(1))) void*)(src + (int64_t)r * sld + c0 + lane),
              (__attribute__((address_space(3))) void*)(sm + dst + r * dld + c0), 4, 0, 0);
    base += n;
  };
#pragma unroll
  for (int l = 0; l < NL; ++l) rows(a.W[l], a.dims[l + 1], a.dims[l], a.dims[l], L.w[l], hl_ld(a.dims[l]));
#pragma unroll
  for (int l = 0; l < NL; ++l) rows(a.b[l], 1, a.dims[l + 1], 0, L.b[l], 0);
  rows(x, G, a.dims[0], a.dims[0], L.x, hl_ld(a.dims[0]));
  rows(target, G, a.dims[NL], a.dims[NL], L.tg, a.dims[NL]);
  if (acts) {  // acts [G, S]: layer l's block of columns -> A_l
#pragma unroll
    for (int l = 0; l < NL; ++l) rows(acts + a.aoff[l], G, a.dims[l + 1], a.aoff[NL], L.act[l], hl_ld(a.dims[l + 1]));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  hl_sync();
}

// forward chain: A_l = act(A_{l-1} W_l^T + b_l), tiles of 16 rows x 16 outputs per wave;
// padding rows/columns stay exactly zero; rows < G, columns < O also go to the global acts
template <int NL>
__device__ void hl_chain(const MlpArgs& a, const HlLayout& L, int G, float* sm, float* __restrict__ acts,
                         long long* dbg = nullptr) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, lg = lane >> 4;
  const int S = a.aoff[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    const int I = a.dims[l], O = a.dims[l + 1];
    const float* in = sm + (l == 0 ? L.x : L.act[l - 1]);
    const int ldi = hl_ld(I), ldo = hl_ld(O);
    const float* W = sm + L.w[l];
    float* out = sm + L.act[l];
    const int ct = hl_r16(O) / 16, tiles = (L.Gp / 16) * ct, K4 = (I + 3) / 4;
    const float* bb = sm + L.b[l];
    for (int t = wv; t < tiles; t += kHlWaves) {
      const int r0 = (t / ct) * 16, c0 = (t % ct) * 16;
      const f4v_hl acc = hl_dot(in + (r0 + li) * ldi + lg, 4, W + (c0 + li) * ldi + lg, 4, K4);
      const int col = c0 + li;
      const float bias = col < O ? bb[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + 4 * lg + r;
        float v = acc[r] + bias;
        if (a.relu[l]) v = fmaxf(v, 0.f);
        const bool live = row < G && col < O;
        out[row * ldo + col] = live ? v : 0.f;
        if (live && acts) acts[(int64_t)row * S + a.aoff[l] + col] = v;
      }
    }
    hl_sync();
    hl_stamp(dbg, 3 + l);
  }
}

// pred [G, Do] and the masked loss of the staged chain's output; thread 0 writes out =
// [loss, count] and every thread returns them (for the fused backward)
// fixed-order workgroup sum of two doubles: wave shuffle tree, then one thread over the
// per-wave sums; every thread returns the totals
__device__ __forceinline__ double2 hl_block_sum2(double s, double c) {
  __shared__ double red[kHlWaves][2];
  __shared__ double res[2];
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off);
    c += __shfl_xor(c, off);
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    red[w][0] = s;
    red[w][1] = c;
  }
  hl_sync();
  if (threadIdx.x == 0) {
    double ts = 0.0, tc = 0.0;
    for (int k = 0; k < kHlWaves; ++k) {
      ts += red[k][0];
      tc += red[k][1];
    }
    res[0] = ts;
    res[1] = tc;
  }
  hl_sync();
  return make_double2(res[0], res[1]);
}

template <int NL>
__device__ float2 hl_loss(const MlpArgs& a, const HlLayout& L, int G, const float* sm,
                          const float* __restrict__ target, const bool* __restrict__ mask, int kind,
                          float* __restrict__ out, float* __restrict__ pred) {
  const int Do = a.dims[NL], ldo = hl_ld(Do);
  const float* P = sm + L.act[NL - 1];
  __shared__ double red[kHlWaves][2];
  __shared__ float res[2];
  double s = 0.0, c = 0.0;
  for (int idx = threadIdx.x; idx < G * Do; idx += kHlThreads) {
    const int r = idx / Do, o = idx % Do;
    const float p = P[r * ldo + o];
    pred[idx] = p;
    if (sm[L.mk + r] != 0.f) {
      s += (double)loss_term_hl(kind, p - sm[L.tg + idx]);
      c += 1.0;
    }
  }
  // fixed-order reduction: wave shuffle tree, then thread 0 over the per-wave sums
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off);
    c += __shfl_xor(c, off);
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    red[w][0] = s;
    red[w][1] = c;
  }
  hl_sync();
  if (threadIdx.x == 0) {
    double ts = 0.0, tc = 0.0;
    for (int k = 0; k < kHlWaves; ++k) {
      ts += red[k][0];
      tc += red[k][1];
    }
    double l = ts / (tc > 0.0 ? tc : 1.0);
    if (kind == 2) l = sqrt(l);
    out[0] = res[0] = (float)l;
    out[1] = res[1] = (float)tc;
  }
  hl_sync();
  return make_float2(res[0], res[1]);
}

// out: [loss, count]; pred [G, Do]; acts [G, S] (every layer's output, for the backward)
template <int NL>
__global__ void __launch_bounds__(kHlThreads) head_loss_fwd_kernel(const float* __restrict__ x, int G, MlpArgs a,
                                                                   const float* __restrict__ target,
                                                                   const bool* __restrict__ mask, int kind,
                                                                   float* __restrict__ out, float* __restrict__ pred,
                                                                   float* __restrict__ acts) {
  extern __shared__ float sm[];
  const HlLayout L = hl_layout<NL>(a, G);
  hl_stage<NL>(a, L, x, nullptr, target, mask, G, sm);
  hl_chain<NL>(a, L, G, sm, acts);
  hl_loss<NL>(a, L, G, sm, target, mask, kind, out, pred);
}

// backward of the staged chain (every activation in LDS) and the loss with upstream gradient
// g, loss value lv and kept count cnt.  grads: [dW_0 | db_0 | dW_1 | db_1 | ...] (goff),
// dx [G, D0]
template <int NL>
__device__ void hl_backward(const MlpArgs& a, const HlLayout& L, int G, float* sm, const float* __restrict__ target,
                            const bool* __restrict__ mask, int kind, float g, float lv, float cnt,
                            float* __restrict__ grads, float* __restrict__ dx, long long* dbg = nullptr) {
  const int n = NL, Do = a.dims[n];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, lg = lane >> 4;
  float* DY = sm + L.dy;
  float* DY2 = sm + L.dy2;
  const int ldy = L.ldy;
  {
    const float den = cnt > 0.f ? cnt : 1.f;
    const bool rl = a.relu[n - 1];
    const float* P = sm + L.act[n - 1];
    const int ldo = hl_ld(Do);
    for (int idx = threadIdx.x; idx < G * Do; idx += kHlThreads) {
      const int r = idx / Do, o = idx % Do;
      const float p = P[r * ldo + o];
      float v = 0.f;
      if (sm[L.mk + r] != 0.f) {
        const float d = p - sm[L.tg + idx];
        const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
        switch (kind) {
          case 1: v = sgn / den; break;
          case 3: v = (fabsf(d) < 1.f ? d : sgn) / den; break;
          case 2: v = lv > 0.f ? d / (den * lv) : 0.f; break;
          default: v = 2.f * d / den; break;
        }
        v *= g;
      }
      DY[r * ldy + o] = (rl && p <= 0.f) ? 0.f : v;
    }
  }
  hl_sync();
#pragma unroll
  for (int l = n - 1; l >= 0; --l) {
    const int I = a.dims[l], O = a.dims[l + 1];
    const float* ain = sm + (l == 0 ? L.x : L.act[l - 1]);
    const int lda = hl_ld(I);
    const float* W = sm + L.w[l];
    float* gl = grads + a.goff[l];
    // dW = DY^T A_in: 16 x 16 (o, i) tiles, K = the rows (DY rows >= G are zero)
    const int ti = hl_r16(I) / 16, to = hl_r16(O) / 16;
    for (int t = wv; t < to * ti; t += kHlWaves) {
      const int o0 = (t / ti) * 16, i0 = (t % ti) * 16;
      const f4v_hl acc = hl_dot(DY + lg * ldy + o0 + li, 4 * ldy, ain + lg * lda + i0 + li, 4 * lda, L.Gp / 4);
      const int i = i0 + li;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = o0 + 4 * lg + r;
        if (o < O && i < I) gl[o * I + i] = acc[r];
      }
    }
    // db[o] = sum_r dy[r, o]: 16 lanes per column (rows part, part + 16, ...), folded by a
    // fixed xor tree
    for (int c0 = 0; c0 < O; c0 += kHlThreads / 16) {
      const int o = c0 + (threadIdx.x >> 4), part = threadIdx.x & 15;
      float v = 0.f;
      if (o < O)
        for (int r = part; r < G; r += 16) v += DY[r * ldy + o];
      v += __shfl_xor(v, 8);
      v += __shfl_xor(v, 4);
      v += __shfl_xor(v, 2);
      v += __shfl_xor(v, 1);
      if (part == 0 && o < O) gl[O * I + o] = v;
    }
    // da = DY W (K = O; DY columns >= O and W rows >= O are zero), masked by ReLU'(A_in)
    const bool msk = l > 0 && a.relu[l - 1];
    const int K4 = (O + 3) / 4;
    for (int t = wv; t < (L.Gp / 16) * ti; t += kHlWaves) {
      const int r0 = (t / ti) * 16, i0 = (t % ti) * 16;
      const f4v_hl acc = hl_dot(DY + (r0 + li) * ldy + lg, 4, W + lg * lda + i0 + li, 4 * lda, K4);
      const int col = i0 + li;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + 4 * lg + r;
        float v = acc[r];
        if (msk && !(ain[row * lda + col] > 0.f)) v = 0.f;
        const bool live = row < G && col < I;
        if (l == 0) {
          if (live) dx[row * I + col] = v;
        } else {
          DY2[row * ldy + col] = live ? v : 0.f;
        }
      }
    }
    hl_sync();
    hl_stamp(dbg, 20 + l);
    float* t = DY;
    DY = DY2;
    DY2 = t;
  }
}

template <int NL>
__global__ void __launch_bounds__(kHlThreads) head_loss_bwd_kernel(const float* __restrict__ gout,
                                                                   const float* __restrict__ x,
                                                                   const float* __restrict__ acts, int G, MlpArgs a,
                                                                   const float* __restrict__ target,
                                                                   const bool* __restrict__ mask, int kind,
                                                                   const float* __restrict__ fwd,
                                                                   float* __restrict__ grads, float* __restrict__ dx) {
  extern __shared__ float sm[];
  const HlLayout L = hl_layout<NL>(a, G);
  hl_stage<NL>(a, L, x, acts, target, mask, G, sm);
  hl_backward<NL>(a, L, G, sm, target, mask, kind, gout[0], fwd[0], fwd[1], grads, dx);
}

// forward, loss and the backward for a unit upstream gradient in ONE launch: the chain's
// activations never leave LDS and the backward launch (a second staging of every weight and
// activation) disappears from the step; _HeadLoss.backward scales by g unless g is the
// training step's unit seed
template <int NL>
__global__ void __launch_bounds__(kHlThreads) head_loss_fused_kernel(const float* __restrict__ x, int G, MlpArgs a,
                                                                     const float* __restrict__ target,
                                                                     const bool* __restrict__ mask, int kind,
                                                                     float* __restrict__ out,
                                                                     float* __restrict__ pred,
                                                                     float* __restrict__ grads,
                                                                     float* __restrict__ dx, long long* dbg) {
  hl_stamp(dbg, 0);
  extern __shared__ float sm[];
  const HlLayout L = hl_layout<NL>(a, G);
  hl_stamp(dbg, 1);
  hl_stage<NL>(a, L, x, nullptr, target, mask, G, sm);
  hl_stamp(dbg, 2);
  hl_chain<NL>(a, L, G, sm, nullptr, dbg);
  const float2 lc = hl_loss<NL>(a, L, G, sm, target, mask, kind, out, pred);
  hl_stamp(dbg, 19);
  hl_backward<NL>(a, L, G, sm, target, mask, kind, 1.f, lc.x, lc.y, grads, dx, dbg);
  hl_stamp(dbg, 31);
}

// ------------------------------------------------------------------------------------
// Row-split head + loss + backward (the training path, ops/mlp.py _HeadLoss fused): one
// workgroup per kHlRows rows.  A single workgroup runs every layer on ONE CU's matrix cores
// (a 33-row x 64-wide layer is ~1.5k MFMA cycles there, and the backward twice that), so the
// one-workgroup kernels above spend most of their time MFMA-bound on a nearly idle chip.
// Rows are independent through the forward chain, the loss terms and the backward's dgrad
// chain; only the weight gradients (sums over rows) and the loss (a mean) couple the
// workgroups: each writes its dW/db partial slab and loss partial, draws an agent-scope
// ticket, and the last arriver sums the slabs in workgroup order (deterministic) and writes
// the loss.  Every workgroup counts the kept elements of the whole batch itself (the loss
// normalisation), so no other cross-workgroup step exists.  RMSE's dpred = d / (n lv) needs
// the global loss lv: the workgroups seed d / n and the reducer rescales dW, db and dx by 1/lv.
constexpr int kHlRows = 16;

// The row-split kernel is ONE compact instantiation for every layer count: its layer loops
// are rolled and read their widths / LDS offsets from a table built in LDS at entry.  The
// per-NL unrolled form was ~36 KB of straight-line code executed once per launch by 3
// workgroups: every layer paid its instruction-cache misses (~1.8k cycles per layer even at
// K = 8, tools/bench_head_loss.py --stamps), which was most of the kernel's 32 us.
// LDS layout: every matrix is [rows][r32(cols) + 4] with rows of W / b padded to r32(O) and
// zero padding, so the 8-deep operand groups of hl_dotp read unconditionally (no per-step
// bounds branches) and the +4 row stride spreads a 16 x 4-lane tile read over distinct banks.
__device__ __host__ __forceinline__ int hl_r32(int v) { return (v + 31) / 32 * 32; }
__device__ __host__ __forceinline__ int hl_ldp(int cols) { return hl_r32(cols) + 4; }

struct HlTab {
  int n, Gp, ldy, x, dy, dy2, tg, mk, total;
  int dims[kMlpMaxLayers + 1];
  int relu[kMlpMaxLayers];
  int goff[kMlpMaxLayers + 1];
  int w[kMlpMaxLayers], b[kMlpMaxLayers], act[kMlpMaxLayers];
  const float* W[kMlpMaxLayers];
  const float* bias[kMlpMaxLayers];
  // LDS copy jobs (hl_jobs): W_0..W_{n-1}, b_0..b_{n-1}, the x rows, the target rows.  Rows
  // of a job past its source rows, and columns past its width, are zero padding.  Row jobs
  // (x, target) start at the workgroup's first row and hold its Gl rows (pr < 0: pr = Gl).
  int njobs;
  const float* jsrc[2 * kMlpMaxLayers + 2];
  int jnr[2 * kMlpMaxLayers + 2], jpr[2 * kMlpMaxLayers + 2], jw[2 * kMlpMaxLayers + 2];
  int jsld[2 * kMlpMaxLayers + 2], jdst[2 * kMlpMaxLayers + 2], jdld[2 * kMlpMaxLayers + 2];
  int jzw[2 * kMlpMaxLayers + 2], jrow[2 * kMlpMaxLayers + 2];
  // destinations of the reduced gradients: dW_l at gout[2l], db_l at gout[2l + 1]
  float* gout[2 * kMlpMaxLayers];
};

// host: the copy-job table of a launch over x [G, D0] / target [G, Do]
inline void hl_jobs(HlTab& T, const float* x, const float* target) {
  const int n = T.n;
  int j = 0;
  auto job = [&](const float* src, int nr, int pr, int w, int sld, int dst, int dld, int zw, int row) {
    T.jsrc[j] = src;
    T.jnr[j] = nr;
    T.jpr[j] = pr;
    T.jw[j] = w;
    T.jsld[j] = sld;
    T.jdst[j] = dst;
    T.jdld[j] = dld;
    T.jzw[j] = zw;
    T.jrow[j] = row;
    ++j;
  };
  for (int l = 0; l < n; ++l)
    job(T.W[l], T.dims[l + 1], hl_r32(T.dims[l + 1]), T.dims[l], T.dims[l], T.w[l], hl_ldp(T.dims[l]),
        hl_ldp(T.dims[l]), 0);
  for (int l = 0; l < n; ++l) job(T.bias[l], 1, 1, T.dims[l + 1], 0, T.b[l], 0, hl_r32(T.dims[l + 1]), 0);
  job(x, 0, T.Gp, T.dims[0], T.dims[0], T.x, hl_ldp(T.dims[0]), hl_ldp(T.dims[0]), 1);
  job(target, 0, -1, T.dims[n], T.dims[n], T.tg, T.dims[n], T.dims[n], 1);
  T.njobs = j;
  while (j < 2 * kMlpMaxLayers + 2) job(nullptr, 0, 0, 0, 0, 0, 0, 0, 0);
}

__device__ __host__ inline void hl_tab_fill(HlTab& T, const MlpArgs& a, int G) {
  const int n = a.n;
  T.n = n;
  T.Gp = hl_r16(G);
  int o = 0, mw = a.dims[0];
  for (int l = 0; l <= n; ++l) {
    T.dims[l] = a.dims[l];
    T.goff[l] = a.goff[l];
  }
  for (int l = 0; l < n; ++l) {
    T.relu[l] = a.relu[l];
    T.W[l] = a.W[l];
    T.bias[l] = a.b[l];
    T.w[l] = o;
    o += hl_r32(a.dims[l + 1]) * hl_ldp(a.dims[l]);
    mw = a.dims[l + 1] > mw ? a.dims[l + 1] : mw;
  }
  for (int l = 0; l < n; ++l) {
    T.b[l] = o;
    o += hl_r32(a.dims[l + 1]);
  }
  T.x = o;
  o += T.Gp * hl_ldp(a.dims[0]);
  for (int l = 0; l < n; ++l) {
    T.act[l] = o;
    o += T.Gp * hl_ldp(a.dims[l + 1]);
  }
  T.ldy = hl_ldp(mw);
  T.dy = o;
  o += T.Gp * T.ldy;
  T.dy2 = o;
  o += T.Gp * T.ldy;
  T.tg = o;
  o += G * a.dims[n];
  T.mk = o;
  o += T.Gp;
  T.total = (o + 3) & ~3;  // whole float4s (the zero fill)
}

__device__ __forceinline__ int hl_u(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int hl_rl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float* hl_rlp(const float* p, int l) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l), hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return (float*)(((uint64_t)hi << 32) | lo);
}

// 16 x 16 tile product over K4 k-steps (K4 a multiple of 8, <= 32, operands zero-padded):
// the operands of 16 steps are read from LDS before their MFMAs (one LDS latency per 64-deep
// slice, not one per 8 steps)
__device__ __forceinline__ f4v_hl hl_tile(const float* ap, int sa, const float* bp, int sb, int K4) {
  f4v_hl a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
  for (int k = 0; k < K4; k += 16) {
    const bool two = k + 8 < K4;
    float x[16], y[16];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      x[j] = ap[(k + j) * sa];
      y[j] = bp[(k + j) * sb];
    }
    if (two) {
#pragma unroll
      for (int j = 8; j < 16; ++j) {
        x[j] = ap[(k + j) * sa];
        y[j] = bp[(k + j) * sb];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      a0 = hl_mfma(x[j], y[j], a0);
      a1 = hl_mfma(x[j + 1], y[j + 1], a1);
    }
    if (two) {
#pragma unroll
      for (int j = 8; j < 16; j += 2) {
        a0 = hl_mfma(x[j], y[j], a0);
        a1 = hl_mfma(x[j + 1], y[j + 1], a1);
      }
    }
  }
  return a0 + a1;
}

// 16 x 16 tile over exactly 4 k-steps (the weight gradients: K = the 16 rows of a block)
__device__ __forceinline__ f4v_hl hl_tile4(const float* ap, int sa, const float* bp, int sb) {
  float x[4], y[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    x[j] = ap[j * sa];
    y[j] = bp[j * sb];
  }
  f4v_hl a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
  a0 = hl_mfma(x[0], y[0], a0);
  a1 = hl_mfma(x[1], y[1], a1);
  a0 = hl_mfma(x[2], y[2], a0);
  a1 = hl_mfma(x[3], y[3], a1);
  return a0 + a1;
}

__device__ __forceinline__ bool hl_arrive(int* counter, int expected) {
  __shared__ int flag;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int tk = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag = (tk == expected - 1);
  }
  __syncthreads();
  if (!flag) return false;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    *counter = 0;  // reset for the next launch (every ticket of this launch is drawn)
  }
  __syncthreads();
  return true;
}

__global__ void __launch_bounds__(kHlThreads) head_loss_rows_kernel(
    const float* __restrict__ x, int G, const HlTab tab, const float* __restrict__ target,
    const bool* __restrict__ mask, int kind, float* __restrict__ out, float* __restrict__ pred,
    float* __restrict__ grads, float* __restrict__ dx, float* __restrict__ part, double* __restrict__ lpart,
    int* __restrict__ cnt, long long* dbg, int full) {
  // full = 0: the input-gradient chain only (dx; the training step's critical path, see
  // ops/mlp.py): no predictions, loss, weight gradients or cross-workgroup reduction.
  // full = 1 with dx == null: everything but dx (the side-stream twin of a full = 0 launch)
  hl_stamp(dbg, 0);
  extern __shared__ float sm[];
  __shared__ double redl[kHlWaves];
  __shared__ int redk[kHlWaves];
  const int R = gridDim.x, b = blockIdx.x, row0 = b * kHlRows, Gl = min(kHlRows, G - row0);
  const int tid = threadIdx.x, wv = hl_u(tid >> 6), lane = tid & 63, li = lane & 15, lg = lane >> 4;
  const int n = tab.n, Gp = tab.Gp, D0 = tab.dims[0], nw = tab.goff[n];
  // per-layer parameters held lane-indexed (lane l: layer l), broadcast with v_readlane
  const int ll = min(lane, kMlpMaxLayers - 1);
  const int v_dims = tab.dims[min(lane, kMlpMaxLayers)], v_goff = tab.goff[min(lane, kMlpMaxLayers)];
  const int v_relu = tab.relu[ll], v_w = tab.w[ll], v_b = tab.b[ll], v_act = tab.act[ll];
  float* const v_gout = tab.gout[min(lane, 2 * kMlpMaxLayers - 1)];
  const int Do = hl_rl(v_dims, n);
  // lane j: copy job j's parameters; with the row mask these are the only loads ahead of the
  // copies (all issued together: one memory round trip), consumed before any copy is issued
  // (a wait on them after the copies would also wait for every copy)
  const int jl = min(lane, 2 * kMlpMaxLayers + 1);
  const float* j_src = tab.jsrc[jl];
  const int j_nr = tab.jnr[jl], j_pr = tab.jpr[jl], j_w = tab.jw[jl], j_sld = tab.jsld[jl], j_dst = tab.jdst[jl];
  const int j_dld = tab.jdld[jl], j_zw = tab.jzw[jl], j_row = tab.jrow[jl];
  // the row-mask reads go out with the table loads (clamped, unconditional: a guarded load
  // would be waited for on its own, one more memory round trip before the copies)
  const bool mk_all = mask == nullptr || mask[min(tid, G - 1)];
  const bool mk_own = mask == nullptr || mask[row0 + min(tid, Gl - 1)];
  // kept rows per wave: ballot + popcount (no shuffle rounds)
  int kr = __popcll(__ballot(tid < G && mk_all));
  for (int r0 = kHlThreads; r0 < G; r0 += kHlThreads) {
    const int r = r0 + tid;
    kr += __popcll(__ballot(r < G && (mask == nullptr || mask[min(r, G - 1)])));
  }
  if (tid < Gp) sm[tab.mk + tid] = (tid < Gl && mk_own) ? 1.f : 0.f;
  if (lane == 0) redk[wv] = kr;
  hl_stamp(dbg, 28);
  const int nj = tab.njobs;
  // LDS-DMA copy jobs: one wave instruction per (matrix row, 64-column chunk), rows dealt
  // round-robin to the waves (continuing across jobs), every copy in flight together; each
  // row's zero padding is written by the wave that copies it (disjoint addresses).
  // (Measured alternatives, tools/bench_head_loss.py: zero stores in a separate pass before
  // the copies, and register staging of 16 rows per wave with one wait, were both slower.)
  int base = 0;
  for (int j = 0; j < nj; ++j) {
    const float* src = hl_rlp(j_src, j);
    int nr = hl_rl(j_nr, j), pr = hl_rl(j_pr, j);
    const int width = hl_rl(j_w, j), sld = hl_rl(j_sld, j);
    const int dst = hl_rl(j_dst, j), dld = hl_rl(j_dld, j), zw = hl_rl(j_zw, j);
    if (hl_rl(j_row, j)) {
      src += (int64_t)row0 * sld;
      nr = Gl;
      if (pr < 0) pr = Gl;
    }
    for (int r = (wv - base % kHlWaves + kHlWaves) % kHlWaves; r < pr; r += kHlWaves) {
      if (r < nr) {
        for (int c0 = 0; c0 < width; c0 += 64)
          if (c0 + lane < width)
            __builtin_amdgcn_global_load_lds(
                (__attribute__((address_space(1))) void*)(src + (int64_t)r * sld + c0 + lane),
                (__attribute__((address_space(3))) void*)(sm + dst + r * dld + c0), 4, 0, 0);
      }
      for (int c = (r < nr ? width : 0) + lane; c < zw; c += 64) sm[dst + r * dld + c] = 0.f;
    }
    base += pr;
  }
  // activations, dY buffers: plain zero fill (disjoint from every copy)
  for (int e = tab.act[0] + 4 * tid; e < tab.tg; e += 4 * kHlThreads)
    *reinterpret_cast<float4*>(sm + e) = make_float4(0.f, 0.f, 0.f, 0.f);
  hl_stamp(dbg, 29);
  hl_stamp(dbg, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  hl_sync();
  hl_stamp(dbg, 2);
  int keptr = 0;
#pragma unroll
  for (int k = 0; k < kHlWaves; ++k) keptr += redk[k];
  const double kept = (double)keptr * (double)Do;
  // forward chain: A_l = act(A_{l-1} W_l^T + b_l), 16 x 16 output tiles per wave
  for (int l = 0; l < n; ++l) {
    const int I = hl_rl(v_dims, l), O = hl_rl(v_dims, l + 1);
    const float* in = sm + (l == 0 ? tab.x : hl_rl(v_act, l > 0 ? l - 1 : 0));
    const float* W = sm + hl_rl(v_w, l);
    const float* bb = sm + hl_rl(v_b, l);
    float* outp = sm + hl_rl(v_act, l);
    const bool rl = hl_rl(v_relu, l) != 0;
    const int ldi = hl_ldp(I), ldo = hl_ldp(O), ct = hl_r16(O) / 16, tiles = (Gp / 16) * ct, K4 = hl_r32(I) / 4;
    for (int t = wv; t < tiles; t += kHlWaves) {
      const int r0 = (t / ct) * 16, c0 = (t % ct) * 16;
      const f4v_hl acc = hl_tile(in + (r0 + li) * ldi + lg, 4, W + (c0 + li) * ldi + lg, 4, K4);
      const int col = c0 + li;
      const float bias = bb[col];  // zero past O
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + 4 * lg + r;
        float v = acc[r] + bias;
        if (rl) v = fmaxf(v, 0.f);
        outp[row * ldo + col] = (row < Gl && col < O) ? v : 0.f;
      }
    }
    hl_sync();
    hl_stamp(dbg, 3 + l);
  }
  // predictions, the loss partial and the loss gradient in one pass (the normalisation is the
  // batch's kept count, known to every workgroup; RMSE's 1 / lv is applied by the reducer)
  const int ldy = tab.ldy;
  float* DY = sm + tab.dy;
  float* DY2 = sm + tab.dy2;
  {
    const float* P = sm + hl_rl(v_act, n - 1);
    const float* TG = sm + tab.tg;
    const float* MKp = sm + tab.mk;
    const int ldP = hl_ldp(Do);
    const bool rl = hl_rl(v_relu, n - 1) != 0;
    const float den = kept > 0.0 ? (float)kept : 1.f;
    double ls = 0.0;
    for (int idx = tid; idx < Gl * Do; idx += kHlThreads) {
      const int r = idx / Do, o = idx % Do;
      const float p = P[r * ldP + o];
      if (full) pred[(int64_t)row0 * Do + idx] = p;
      float v = 0.f;
      if (MKp[r] != 0.f) {
        const float d = p - TG[idx];
        ls += (double)loss_term_hl(kind, d);
        const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
        switch (kind) {
          case 1: v = sgn / den; break;
          case 3: v = (fabsf(d) < 1.f ? d : sgn) / den; break;
          case 2: v = d / den; break;
          default: v = 2.f * d / den; break;
        }
      }
      DY[r * ldy + o] = (rl && p <= 0.f) ? 0.f : v;
    }
    for (int off = 32; off > 0; off >>= 1) ls += __shfl_xor(ls, off);
    if (lane == 0) redl[wv] = ls;
  }
  hl_sync();
  hl_stamp(dbg, 19);
  // backward, per layer in reverse: DY' = (DY W) * relu'(A_in) on waves 0..nx-1 (the chain),
  // while the other waves form dW = DY^T A_in (K = the block's rows) and db = sum_r DY
  float* pb = part + (int64_t)b * nw;
  float* dxb = dx + (int64_t)row0 * D0;
  for (int l = n - 1; l >= 0; --l) {
    const int I = hl_rl(v_dims, l), O = hl_rl(v_dims, l + 1);
    const float* ain = sm + (l == 0 ? tab.x : hl_rl(v_act, l > 0 ? l - 1 : 0));
    const float* W = sm + hl_rl(v_w, l);
    float* gl = pb + hl_rl(v_goff, l);
    const int lda = hl_ldp(I), ti = hl_r16(I) / 16, to = hl_r16(O) / 16, nx = (Gp / 16) * ti;
    const int w0 = nx < kHlWaves - 2 ? nx : 0, nd = kHlWaves - w0;
    if (full && wv >= w0) {
      for (int t = wv - w0; t < to * ti; t += nd) {
        const int o0 = (t / ti) * 16, i0 = (t % ti) * 16;
        f4v_hl acc = {0.f, 0.f, 0.f, 0.f};
        for (int k0 = 0; k0 < Gp; k0 += 16) {
          const f4v_hl p4 = hl_tile4(DY + (k0 + lg) * ldy + o0 + li, 4 * ldy, ain + (k0 + lg) * lda + i0 + li, 4 * lda);
          acc += p4;
        }
        const int i = i0 + li;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int o = o0 + 4 * lg + r;
          if (o < O && i < I) gl[o * I + i] = acc[r];
        }
      }
    }
    {
      const int c = tid - (kHlThreads - 128);  // the last two waves
      for (int o = c; full && o >= 0 && o < O; o += 128) {
        float v = 0.f;
        for (int r = 0; r < Gl; ++r) v += DY[r * ldy + o];
        gl[O * I + o] = v;
      }
    }
    const bool msk = l > 0 && hl_rl(v_relu, l > 0 ? l - 1 : 0) != 0;
    const int K4 = hl_r32(O) / 4, i32 = hl_r32(I);
    for (int t = wv; t < nx; t += kHlWaves) {
      const int r0 = (t / ti) * 16, i0 = (t % ti) * 16;
      const f4v_hl acc = hl_tile(DY + (r0 + li) * ldy + lg, 4, W + lg * lda + i0 + li, 4 * lda, K4);
      const int col = i0 + li;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + 4 * lg + r;
        float v = acc[r];
        if (msk && !(ain[row * lda + col] > 0.f)) v = 0.f;
        const bool live = row < Gl && col < I;
        if (l == 0) {
          if (live && dx != nullptr) dxb[row * I + col] = v;
        } else {
          DY2[row * ldy + col] = live ? v : 0.f;
          // columns [r16(I), r32(I)) of DY' are read (as zeros) by the next layer's tiles
          if (col + 16 >= ti * 16 && col + 16 < i32) DY2[row * ldy + col + 16] = 0.f;
        }
      }
    }
    hl_sync();
    hl_stamp(dbg, 20 + l);
    float* sw = DY;
    DY = DY2;
    DY2 = sw;
  }
  if (!full) return;
  double2 tot;
  {
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < kHlWaves; ++k) t += redl[k];
    tot = make_double2(t, kept);
  }
  if (tid == 0) lpart[b] = tot.x;
  if (!hl_arrive(cnt, R)) return;
  __shared__ float scale_s;
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int k = 0; k < R; ++k) t += lpart[k];
    const double tc = tot.y;
    double l = t / (tc > 0.0 ? tc : 1.0);
    float sc = 1.f;
    if (kind == 2) {
      l = sqrt(l);
      sc = l > 0.0 ? (float)(1.0 / l) : 0.f;
    }
    out[0] = (float)l;
    out[1] = (float)tc;
    scale_s = sc;
  }
  __syncthreads();
  const float sc = scale_s;
  // 4 elements per thread per pass with all their slab loads in flight (a load -> add chain
  // per element paid one memory latency each)
  for (int e0 = threadIdx.x; e0 < nw; e0 += 4 * kHlThreads) {
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < R; ++k) {
      float t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + u * kHlThreads;
        t[u] = e < nw ? part[(int64_t)k * nw + e] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] += t[u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * kHlThreads;
      float* dst = nullptr;
      for (int l = 0; l < n; ++l) {  // element e of the gradient image -> its tensor
        const int g0 = hl_rl(v_goff, l), oi = hl_rl(v_dims, l) * hl_rl(v_dims, l + 1);
        if (e >= g0 && e < hl_rl(v_goff, l + 1))
          dst = e < g0 + oi ? hl_rlp(v_gout, 2 * l) + (e - g0) : hl_rlp(v_gout, 2 * l + 1) + (e - g0 - oi);
      }
      if (dst != nullptr) *(__attribute__((address_space(1))) float*)dst = v[u] * sc;
    }
  }
  if (kind == 2 && dx != nullptr)
    for (int e = threadIdx.x; e < G * D0; e += kHlThreads) dx[e] *= sc;
  hl_stamp(dbg, 31);
}

#define HL_NL_SWITCH(n, F)                                        \
  switch (n) {                                                    \
    case 1: F(1); break;                                          \
    case 2: F(2); break;                                          \
    case 3: F(3); break;                                          \
    case 4: F(4); break;                                          \
    case 5: F(5); break;                                          \
    case 6: F(6); break;                                          \
    case 7: F(7); break;                                          \
    case 8: F(8); break;                                          \
    default: HY_CHECK(false, "head_loss: 1..8 layers");           \
  }
static_assert(kMlpMaxLayers == 8, "HL_NL_SWITCH covers 1..8 layers");

static size_t hl_lds(const MlpArgs& a, int G) {
  size_t r = 0;
#define HL_LDS(N) r = sizeof(float) * (size_t)hl_layout<N>(a, G).total
  HL_NL_SWITCH(a.n, HL_LDS)
#undef HL_LDS
  return r;
}

template <int N>
static void hl_attrs() {
  hipFuncSetAttribute((const void*)head_loss_fwd_kernel<N>, hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)kHlMaxLds);
  hipFuncSetAttribute((const void*)head_loss_bwd_kernel<N>, hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)kHlMaxLds);
  hipFuncSetAttribute((const void*)head_loss_fused_kernel<N>, hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)kHlMaxLds);
}

static void hl_checks(const at::Tensor& x, const at::Tensor& target, const c10::optional<at::Tensor>& mask,
                      const MlpArgs& a, int64_t kind, bool one_wg = true) {
  const int64_t G = x.size(0);
  HY_CHECK(kind >= 0 && kind <= 3, "head_loss: unknown loss kind");
  HY_CHECK(target.is_contiguous() && target.scalar_type() == at::kFloat && target.numel() == G * a.dims[a.n],
           "head_loss: target must be contiguous fp32 [G, out]");
  if (mask.has_value() && mask->defined())
    HY_CHECK(mask->scalar_type() == at::kBool && mask->is_contiguous() && mask->numel() == G,
             "head_loss: bool mask [G]");
  HY_CHECK(G >= 1 && (!one_wg || hl_lds(a, (int)G) <= kHlMaxLds),
           "head_loss: rows x widths exceed one workgroup's LDS");
  static bool once = [] {
    hl_attrs<1>();
    hl_attrs<2>();
    hl_attrs<3>();
    hl_attrs<4>();
    hl_attrs<5>();
    hl_attrs<6>();
    hl_attrs<7>();
    hl_attrs<8>();
    hipFuncSetAttribute((const void*)head_loss_rows_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)kHlMaxLds);
    return true;
  }();
  (void)once;
}

// returns [stats [2] = (loss, kept count), pred [G, out], acts [G, sum of widths]]
std::vector<at::Tensor> head_loss_fwd(const at::Tensor& x_, at::TensorList Ws_, at::TensorList bs_,
                                      at::IntArrayRef relu, const at::Tensor& target,
                                      const c10::optional<at::Tensor>& mask, int64_t kind) {
  HY_CHECK_CUDA(x_);
  auto x = x_.contiguous();
  HY_CHECK_F32(x);
  HY_CHECK(x.dim() == 2, "head_loss: x must be [G, D]");
  std::vector<at::Tensor> Ws(Ws_.begin(), Ws_.end()), bs(bs_.begin(), bs_.end());
  auto a = make_args(x, Ws, bs, relu.vec());
  hl_checks(x, target, mask, a, kind);
  const int64_t G = x.size(0);
  auto stats = at::empty({2}, x.options());
  auto pred = at::empty({G, a.dims[a.n]}, x.options());
  auto acts = at::empty({G, a.aoff[a.n]}, x.options());
  const bool* mp = mask.has_value() && mask->defined() ? mask->data_ptr<bool>() : nullptr;
  const size_t lds = hl_lds(a, (int)G);
#define HL_FWD(N)                                                                                                \
  head_loss_fwd_kernel<N><<<1, kHlThreads, lds, stream()>>>(x.data_ptr<float>(), (int)G, a, target.data_ptr<float>(), \
                                                            mp, (int)kind, stats.data_ptr<float>(),                 \
                                                            pred.data_ptr<float>(), acts.data_ptr<float>())
  HL_NL_SWITCH(a.n, HL_FWD)
#undef HL_FWD
  return {stats, pred, acts};
}

// returns [dx, dW_0, db_0, dW_1, db_1, ...]
std::vector<at::Tensor> head_loss_bwd(const at::Tensor& gout, const at::Tensor& x_, const at::Tensor& acts,
                                      at::TensorList Ws_, at::TensorList bs_, at::IntArrayRef relu,
                                      const at::Tensor& target, const c10::optional<at::Tensor>& mask,
                                      const at::Tensor& stats, int64_t kind) {
  auto x = x_.contiguous();
  std::vector<at::Tensor> Ws(Ws_.begin(), Ws_.end()), bs(bs_.begin(), bs_.end());
  auto a = make_args(x, Ws, bs, relu.vec());
  hl_checks(x, target, mask, a, kind);
  HY_CHECK(gout.numel() == 1 && gout.scalar_type() == at::kFloat && gout.is_contiguous() && stats.numel() == 2,
           "head_loss_bwd: scalar upstream gradient and the forward's stats");
  const int64_t G = x.size(0);
  HY_CHECK(acts.is_contiguous() && acts.size(0) == G && acts.size(1) == a.aoff[a.n], "head_loss_bwd: acts shape");
  auto flat = at::empty({a.goff[a.n]}, x.options());
  auto dx = at::empty_like(x);
  const bool* mp = mask.has_value() && mask->defined() ? mask->data_ptr<bool>() : nullptr;
  const size_t lds = hl_lds(a, (int)G);
#define HL_BWD(N)                                                                                               \
  head_loss_bwd_kernel<N><<<1, kHlThreads, lds, stream()>>>(                                                    \
      gout.data_ptr<float>(), x.data_ptr<float>(), acts.data_ptr<float>(), (int)G, a, target.data_ptr<float>(), \
      mp, (int)kind, stats.data_ptr<float>(), flat.data_ptr<float>(), dx.data_ptr<float>())
  HL_NL_SWITCH(a.n, HL_BWD)
#undef HL_BWD
  std::vector<at::Tensor> out{dx};
  for (int l = 0; l < a.n; ++l) {
    const int O = a.dims[l + 1], I = a.dims[l];
    out.push_back(flat.narrow(0, a.goff[l], O * I).view({O, I}));
    out.push_back(flat.narrow(0, a.goff[l] + O * I, O));
  }
  return out;
}

// the ticket counter of head_loss_rows_kernel: persistent per (device, stream) — launches on
// one stream never overlap, and the reducer resets it to zero (an at::zeros per call was a
// fill launch on the step's critical path)
static at::Tensor hl_counter(const at::Tensor& like) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, at::Tensor> counters;
  std::lock_guard<std::mutex> lk(mu);
  auto key = std::make_pair((int)like.get_device(), stream());
  auto it = counters.find(key);
  if (it == counters.end()) it = counters.emplace(key, at::zeros({1}, like.options().dtype(at::kInt))).first;
  return it->second;
}

static bool hl_rows_split() {
  // row-split launch (head_loss_rows_kernel); HYDRA_HEADLOSS_ROWS=0: the one-workgroup kernel
  static const bool on = [] {
    const char* e = std::getenv("HYDRA_HEADLOSS_ROWS");
    return e == nullptr || std::string(e) != "0";
  }();
  return on;
}

// returns [stats [2], pred [G, out], dx, dW_0, db_0, dW_1, db_1, ...] (gradients of the loss
// itself, upstream gradient 1).  grads_out: optional fp32 buffer of the gradient image
// (goff[n] elements, e.g. a slice of the step's flat gradient buffer) written in place;
// want_dx = false: dx is not written (returned empty) — the twin of a head_loss_dx launch.
std::vector<at::Tensor> head_loss_fused(const at::Tensor& x_, at::TensorList Ws_, at::TensorList bs_,
                                        at::IntArrayRef relu, const at::Tensor& target,
                                        const c10::optional<at::Tensor>& mask, int64_t kind,
                                        const c10::optional<at::Tensor>& dbg,
                                        c10::optional<at::TensorList> grads_out, bool want_dx) {
  HY_CHECK_CUDA(x_);
  auto x = x_.contiguous();
  HY_CHECK_F32(x);
  HY_CHECK(x.dim() == 2, "head_loss: x must be [G, D]");
  std::vector<at::Tensor> Ws(Ws_.begin(), Ws_.end()), bs(bs_.begin(), bs_.end());
  auto a = make_args(x, Ws, bs, relu.vec());
  hl_checks(x, target, mask, a, kind);
  long long* dp = nullptr;
  if (dbg.has_value() && dbg->defined()) {
    HY_CHECK(dbg->is_cuda() && dbg->scalar_type() == at::kLong && dbg->is_contiguous() && dbg->numel() >= 32,
             "head_loss_fused: dbg must be int64 [>= 32]");
    dp = (long long*)dbg->data_ptr<int64_t>();
  }
  const int64_t G = x.size(0);
  auto stats = at::empty({2}, x.options());
  auto pred = at::empty({G, a.dims[a.n]}, x.options());
  // gradient tensors: dW_0, db_0, dW_1, ... (caller-provided, e.g. the step's gradient slots, or
  // views of one fresh buffer)
  std::vector<at::Tensor> gts;
  if (grads_out.has_value()) {
    HY_CHECK((int)grads_out->size() == 2 * a.n, "head_loss_fused: grads_out holds dW_l, db_l for every layer");
    for (int l = 0; l < a.n; ++l)
      for (int k = 0; k < 2; ++k) {
        const at::Tensor& t = (*grads_out)[2 * l + k];
        const int64_t want = k == 0 ? (int64_t)a.dims[l + 1] * a.dims[l] : a.dims[l + 1];
        HY_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == want &&
                     t.get_device() == x.get_device(),
                 "head_loss_fused: grads_out tensors must be contiguous fp32 shaped like the weights and biases");
        gts.push_back(t);
      }
  } else {
    auto flat = at::empty({a.goff[a.n]}, x.options());
    for (int l = 0; l < a.n; ++l) {
      const int O = a.dims[l + 1], I = a.dims[l];
      gts.push_back(flat.narrow(0, a.goff[l], O * I).view({O, I}));
      gts.push_back(flat.narrow(0, a.goff[l] + O * I, O));
    }
  }
  auto dx = want_dx ? at::empty_like(x) : at::empty({0}, x.options());
  const bool* mp = mask.has_value() && mask->defined() ? mask->data_ptr<bool>() : nullptr;
  HlTab tab;
  hl_tab_fill(tab, a, (int)std::min<int64_t>(G, kHlRows));
  hl_jobs(tab, x.data_ptr<float>(), target.data_ptr<float>());
  for (int k = 0; k < 2 * a.n; ++k) tab.gout[k] = gts[k].data_ptr<float>();
  if (hl_rows_split() && sizeof(float) * (size_t)tab.total <= kHlMaxLds) {
    const int R = (int)ceil_div(G, (int64_t)kHlRows);
    const size_t lds = sizeof(float) * (size_t)tab.total;
    auto part = at::empty({(int64_t)R * a.goff[a.n]}, x.options());
    auto lpart = at::empty({R}, x.options().dtype(at::kDouble));
    auto cnt = hl_counter(x);
    head_loss_rows_kernel<<<R, kHlThreads, lds, stream()>>>(
        x.data_ptr<float>(), (int)G, tab, target.data_ptr<float>(), mp, (int)kind, stats.data_ptr<float>(),
        pred.data_ptr<float>(), nullptr, want_dx ? dx.data_ptr<float>() : nullptr,
        part.data_ptr<float>(), lpart.data_ptr<double>(), cnt.data_ptr<int>(), dp, 1);
  } else {
    HY_CHECK(want_dx, "head_loss_fused: want_dx = false needs the row-split kernel");
    const size_t lds = hl_lds(a, (int)G);
    auto flat = at::empty({a.goff[a.n]}, x.options());
#define HL_FUSED(N)                                                                                            \
  head_loss_fused_kernel<N><<<1, kHlThreads, lds, stream()>>>(                                                 \
      x.data_ptr<float>(), (int)G, a, target.data_ptr<float>(), mp, (int)kind, stats.data_ptr<float>(),        \
      pred.data_ptr<float>(), flat.data_ptr<float>(), dx.data_ptr<float>(), dp)
    HL_NL_SWITCH(a.n, HL_FUSED)
#undef HL_FUSED
    for (int l = 0; l < a.n; ++l) {
      const int O = a.dims[l + 1], I = a.dims[l];
      gts[2 * l].view(-1).copy_(flat.narrow(0, a.goff[l], O * I));
      gts[2 * l + 1].view(-1).copy_(flat.narrow(0, a.goff[l] + O * I, O));
    }
  }
  std::vector<at::Tensor> out{stats, pred, dx};
  for (int l = 0; l < a.n; ++l) {
    const int O = a.dims[l + 1], I = a.dims[l];
    out.push_back(gts[2 * l].view({O, I}));
    out.push_back(gts[2 * l + 1].view({O}));
  }
  return out;
}

// ------------------------------------------------------------ dx chain: one workgroup per row
// The dx-only launch sits on the training step's critical path.  The row-split kernel above
// runs it on ceil(G / 16) workgroups (3 at the OC20 batch) walking 16-row MFMA tiles.  Rows
// are independent through the forward, the loss gradient (MAE / MSE / smooth-L1: the batch's
// kept count is the only coupling, and every workgroup counts it itself) and the dgrad chain,
// so here ONE workgroup (4 waves) owns ONE row:
//   * every weight matrix and bias is DMA'd into LDS at entry (global_load_lds, all copies
//     in flight together: one memory round trip);
//   * forward, per layer: lane i of wave w forms x[i] W[16 w + jj][i] for its 16 outputs jj
//     (conflict-free LDS rows); the wave's [16][64] product tile goes through LDS once and
//     lane t sums a quarter row (out[16 w + t / 4] after two xor shuffles) — a register
//     butterfly with per-lane half selects was compiled into 16-way select chains;
//   * backward, per layer: dh[i] = sum_j W[j][i] dy[j] from the same LDS rows against
//     broadcast dy reads; the 4 waves' partials meet in LDS.
// The layer loops are ROLLED: the chain executes once per launch, and a first version with
// the layers unrolled (weights held in registers) was 8.5k instructions of straight-line code
// whose instruction-cache misses alone took ~30 us.  Widths: input <= 64 CI, every later
// width <= 64, layers <= 8.  Not RMSE (its dx needs the batch loss).
template <int CI>
__global__ void __launch_bounds__(256) head_dx_row_kernel(const float* __restrict__ x, int G, const MlpArgs a,
                                                          const float* __restrict__ target,
                                                          const bool* __restrict__ mask, int kind,
                                                          float* __restrict__ dx) {
  constexpr int IW = 64 * CI;
  extern __shared__ float sm[];  // W_0, b_0, W_1, b_1, ... (dense, a.woff / biases after each W)
  __shared__ float act[kMlpMaxLayers + 1][IW];
  __shared__ float part[4][IW];
  __shared__ float dyb[IW];
  __shared__ float red[4 * 16 * 65];
  __shared__ int kc[4];
  const int g = blockIdx.x, tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  // per-layer parameters held lane-indexed (lane l: layer l) and broadcast with v_readlane:
  // dynamic indexing of the by-value argument struct inside the layer loops expands into
  // select chains (code size: this kernel runs once per launch, instruction fetch bound)
  const int ll = lane < kMlpMaxLayers ? lane : kMlpMaxLayers - 1;
  const int v_dims = a.dims[lane <= kMlpMaxLayers ? lane : kMlpMaxLayers], v_relu = a.relu[ll];
  const float* v_W = a.W[ll];
  const float* v_b = a.b[ll];
  const int n = a.n, D0 = a.dims[0], Do = hl_rl(v_dims, n);
  // 1) LDS-DMA of every layer's W [O, I] then b [O], 64 floats per wave instruction
  {
    int off = 0, chunk = 0;
    for (int l = 0; l < n; ++l) {
      const int O = hl_rl(v_dims, l + 1), I = hl_rl(v_dims, l);
      for (int part2 = 0; part2 < 2; ++part2) {
        const float* src = part2 == 0 ? hl_rlp(v_W, l) : hl_rlp(v_b, l);
        const int cnt = part2 == 0 ? O * I : O;
        for (int c0 = 0; c0 < cnt; c0 += 64, ++chunk)
          if ((chunk & 3) == w && c0 + lane < cnt)
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src + c0 + lane),
                                             (__attribute__((address_space(3))) void*)(sm + off + c0), 4, 0, 0);
        off += cnt;
      }
    }
  }
  // 2) the row, the kept count, zeroed buffers
  const bool keep = mask == nullptr || mask[g];
  int k = 0;
  for (int t = tid; t < G; t += 256) k += (mask == nullptr || mask[t]) ? 1 : 0;
  for (int off = 32; off > 0; off >>= 1) k += __shfl_xor(k, off, 64);
  if (lane == 0) kc[w] = k;
  for (int e = tid; e < (kMlpMaxLayers + 1) * IW; e += 256) (&act[0][0])[e] = 0.f;
  for (int e = tid; e < IW; e += 256) dyb[e] = 0.f;
  __syncthreads();
  for (int i = tid; i < D0; i += 256) act[0][i] = x[(int64_t)g * D0 + i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // 3) forward chain (rolled over layers)
  int off = 0;
  for (int l = 0; l < n; ++l) {
    const int O = hl_rl(v_dims, l + 1), I = hl_rl(v_dims, l);
    const float* Wl = sm + off;
    float v[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) v[jj] = 0.f;
#pragma unroll
    for (int c = 0; c < CI; ++c) {
      const int i = lane + 64 * c;
      const float xi = act[l][i];
      const bool iok = i < I;
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) {
        const int j = 16 * w + jj;
        const bool ok = iok && j < O;
        const float wv = Wl[ok ? j * I + i : 0];
        v[jj] = fmaf(ok ? wv : 0.f, xi, v[jj]);
      }
    }
    // cross-lane sum over i through LDS: the wave's [16][64] product tile, then lane t sums
    // a quarter (16 columns) of row t / 4 and the 4 quarters meet by two xor shuffles
    float* rw = red + w * 16 * 65;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) rw[jj * 65 + lane] = v[jj];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave reads its own tile back
    __builtin_amdgcn_wave_barrier();
    float o = 0.f;
    {
      const float* rr = rw + (lane >> 2) * 65 + 16 * (lane & 3);
#pragma unroll
      for (int r = 0; r < 16; ++r) o += rr[r];
    }
    o += __shfl_xor(o, 1, 64);
    o += __shfl_xor(o, 2, 64);
    const int j = 16 * w + (lane >> 2);
    const float bj = sm[off + O * I + (j < O ? j : 0)];
    o += bj;
    if (hl_rl(v_relu, l)) o = fmaxf(o, 0.f);
    if ((lane & 3) == 0) act[l + 1][j] = j < O ? o : 0.f;
    off += O * I + O;
    __syncthreads();
  }
  // 4) loss gradient of the row (upstream gradient 1): MSE 2d / n, MAE sgn(d) / n, smooth-L1
  // clamp(d) / n over the batch's n = kept rows x outputs
  if (w == 0 && lane < Do) {
    const float den0 = (float)(kc[0] + kc[1] + kc[2] + kc[3]) * (float)Do;
    const float den = den0 > 0.f ? den0 : 1.f;
    const float p = act[n][lane];
    float v = 0.f;
    if (keep) {
      const float d = p - target[(int64_t)g * Do + lane];
      const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
      v = kind == 1 ? sgn / den : (kind == 3 ? (fabsf(d) < 1.f ? d : sgn) / den : 2.f * d / den);
    }
    dyb[lane] = (hl_rl(v_relu, n - 1) && p <= 0.f) ? 0.f : v;
  }
  __syncthreads();
  // 5) dgrad chain (rolled, layers in reverse)
  for (int l = n - 1; l >= 0; --l) {
    const int O = hl_rl(v_dims, l + 1), I = hl_rl(v_dims, l);
    off -= O * I + O;
    const float* Wl = sm + off;
    float dj[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) dj[jj] = dyb[16 * w + jj];
#pragma unroll
    for (int c = 0; c < CI; ++c) {
      const int i = lane + 64 * c;
      const bool iok = i < I;
      float s2 = 0.f;
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) {
        const int j = 16 * w + jj;
        const bool ok = iok && j < O;
        const float wv = Wl[ok ? j * I + i : 0];
        s2 = fmaf(ok ? wv : 0.f, dj[jj], s2);
      }
      part[w][i] = s2;
    }
    __syncthreads();
    for (int t = tid; t < IW; t += 256) {
      float s2 = (part[0][t] + part[1][t]) + (part[2][t] + part[3][t]);
      if (l == 0) {
        if (t < I) dx[(int64_t)g * I + t] = s2;
      } else {
        if (hl_rl(v_relu, l > 0 ? l - 1 : 0) && !(act[l][t] > 0.f)) s2 = 0.f;
        dyb[t] = t < I ? s2 : 0.f;
      }
    }
    __syncthreads();
  }
}

static size_t hdx_lds(const MlpArgs& a) {
  size_t f = 0;
  for (int l = 0; l < a.n; ++l) f += (size_t)a.dims[l + 1] * a.dims[l] + a.dims[l + 1];
  return f * sizeof(float);
}

static bool hdx_row_eligible(const MlpArgs& a, int64_t kind) {
  static const bool on = [] {
    const char* e = std::getenv("HYDRA_HEADDX_ROW");
    return e == nullptr || std::string(e) != "0";
  }();
  if (!on || kind == 2 || a.n < 1 || a.n > kMlpMaxLayers || a.dims[0] > 128) return false;
  for (int l = 1; l <= a.n; ++l)
    if (a.dims[l] > 64) return false;
  return hdx_lds(a) <= 96 * 1024;
}

// dx of the masked loss (upstream gradient 1) alone: the forward chain and the input-gradient
// chain, nothing else (no predictions, loss value, weight gradients or cross-workgroup step).
// Not for RMSE (its dx needs the batch loss).  Pairs with head_loss_fused(want_dx=false) on a
// side stream.
at::Tensor head_loss_dx(const at::Tensor& x_, at::TensorList Ws_, at::TensorList bs_, at::IntArrayRef relu,
                        const at::Tensor& target, const c10::optional<at::Tensor>& mask, int64_t kind,
                        const c10::optional<at::Tensor>& dbg) {
  HY_CHECK_CUDA(x_);
  auto x = x_.contiguous();
  HY_CHECK_F32(x);
  HY_CHECK(x.dim() == 2, "head_loss: x must be [G, D]");
  HY_CHECK(kind != 2, "head_loss_dx: RMSE's input gradient needs the batch loss (use head_loss_fused)");
  std::vector<at::Tensor> Ws(Ws_.begin(), Ws_.end()), bs(bs_.begin(), bs_.end());
  auto a = make_args(x, Ws, bs, relu.vec());
  hl_checks(x, target, mask, a, kind, !hdx_row_eligible(a, kind));
  long long* dp = nullptr;
  if (dbg.has_value() && dbg->defined()) {
    HY_CHECK(dbg->is_cuda() && dbg->scalar_type() == at::kLong && dbg->is_contiguous() && dbg->numel() >= 32,
             "head_loss_dx: dbg must be int64 [>= 32]");
    dp = (long long*)dbg->data_ptr<int64_t>();
  }
  const int64_t G = x.size(0);
  auto dx = at::empty_like(x);
  const bool* mp = mask.has_value() && mask->defined() ? mask->data_ptr<bool>() : nullptr;
  if (dp == nullptr && hdx_row_eligible(a, kind)) {
    const size_t lds = hdx_lds(a);
    static bool attrs = [] {
      hipFuncSetAttribute((const void*)head_dx_row_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
      hipFuncSetAttribute((const void*)head_dx_row_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
      return true;
    }();
    (void)attrs;
    if (a.dims[0] <= 64)
      head_dx_row_kernel<1><<<(int)G, 256, lds, stream()>>>(x.data_ptr<float>(), (int)G, a, target.data_ptr<float>(),
                                                            mp, (int)kind, dx.data_ptr<float>());
    else
      head_dx_row_kernel<2><<<(int)G, 256, lds, stream()>>>(x.data_ptr<float>(), (int)G, a, target.data_ptr<float>(),
                                                            mp, (int)kind, dx.data_ptr<float>());
    return dx;
  }
  HlTab tab;
  hl_tab_fill(tab, a, (int)std::min<int64_t>(G, kHlRows));
  hl_jobs(tab, x.data_ptr<float>(), target.data_ptr<float>());
  HY_CHECK(sizeof(float) * (size_t)tab.total <= kHlMaxLds, "head_loss_dx: chain exceeds the LDS budget");
  const int R = (int)ceil_div(G, (int64_t)kHlRows);
  head_loss_rows_kernel<<<R, kHlThreads, sizeof(float) * (size_t)tab.total, stream()>>>(
      x.data_ptr<float>(), (int)G, tab, target.data_ptr<float>(), mp, (int)kind, nullptr, nullptr, nullptr,
      dx.data_ptr<float>(), nullptr, nullptr, nullptr, dp, 0);
  return dx;
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("mlp_fwd(Tensor x, Tensor[] Ws, Tensor[] bs, int[] relu) -> (Tensor, Tensor)");
  m.def(
      "mlp_bwd(Tensor dout, Tensor x, Tensor acts, Tensor[] Ws, Tensor[] bs, int[] relu) -> "
      "(Tensor, Tensor[], Tensor[])");
  m.def(
      "head_loss_fwd(Tensor x, Tensor[] Ws, Tensor[] bs, int[] relu, Tensor target, Tensor? mask, int kind) -> "
      "Tensor[]");
  m.def(
      "head_loss_bwd(Tensor gout, Tensor x, Tensor acts, Tensor[] Ws, Tensor[] bs, int[] relu, Tensor target, "
      "Tensor? mask, Tensor stats, int kind) -> Tensor[]");
  m.def(
      "head_loss_fused(Tensor x, Tensor[] Ws, Tensor[] bs, int[] relu, Tensor target, Tensor? mask, int kind, "
      "Tensor? dbg=None, Tensor[]? grads_out=None, bool want_dx=True) -> "
      "Tensor[]");
  m.def(
      "head_loss_dx(Tensor x, Tensor[] Ws, Tensor[] bs, int[] relu, Tensor target, Tensor? mask, int kind, "
      "Tensor? dbg=None) -> Tensor");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("mlp_fwd", hy::mlp_fwd);
  m.impl("mlp_bwd", hy::mlp_bwd);
  m.impl("head_loss_fwd", hy::head_loss_fwd);
  m.impl("head_loss_bwd", hy::head_loss_bwd);
  m.impl("head_loss_fused", hy::head_loss_fused);
  m.impl("head_loss_dx", hy::head_loss_dx);
}
