// SchNet continuous-filter network in one launch each way (reference
// hydragnn/models/SCFStack.py:214-293, CFConv: W_e = nn(rbf_e) * C_e with
// nn = Linear(K, F) -> ShiftedSoftplus -> Linear(F, F)):
//
//   forward   h1 = rbf W1^T + b1,  a1 = softplus(h1) - log 2,  W = (a1 W2^T + b2) * C
//             -> W [E, F] and h1 [E, F] (the backward's only saved activation)
//   backward  dh2 = dW * C,  a1 = ssp(h1),  dh1 = (dh2 W2) * sigmoid(h1)
//             -> dh2, a1, dh1: the row factors of the four weight/bias gradients, which
//                the caller hands to the grouped split-K weight-gradient launch
//                (linear.hip linear_wgrad_grouped) with the step's other deferred maps.
//
// Replaces GEMM + softplus + shift + GEMM + cutoff multiply (and the mirrored backward
// chain): QM9-sized batches (~6k edges) are launch-bound, so one launch per direction
// matters more than MFMA throughput (~10^8 FMAs per layer).  Layout: a workgroup owns 16
// edges; wave q handles edges q, q+4, ..., lane c owns output column c, its weight row
// (column for the dgrad) lives in registers (staged through LDS with coalesced loads: a
// lane-strided row read touches 64 cache lines per instruction), and the edge's input row
// is read from LDS as a broadcast (one address per wave: no bank conflicts).
#include "common.h"

namespace hy {
namespace sch {

constexpr int kEB = 16;    // edges per workgroup (~6k-edge QM9 batches: ~400 workgroups)
constexpr int kMaxW = 64;  // K, F <= 64
constexpr int kLd = kMaxW + 4;

__device__ __forceinline__ float softplus(float x) { return x > 20.f ? x : log1pf(__expf(x)); }
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// one output of a row: sum_k xs[r][k] w[k] (k < kMaxW; w zero past the width)
__device__ __forceinline__ float rowdot(const float* xr, const float* w) {
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxW; k += 4) {
    const float4 v = *reinterpret_cast<const float4*>(xr + k);
    a0 = fmaf(v.x, w[k], a0);
    a1 = fmaf(v.y, w[k + 1], a1);
    a2 = fmaf(v.z, w[k + 2], a2);
    a3 = fmaf(v.w, w[k + 3], a3);
  }
  return (a0 + a1) + (a2 + a3);
}

__global__ void __launch_bounds__(256) cf_filter_fwd_kernel(const float* __restrict__ rbf, int ldr, int K,
                                                            const float* __restrict__ W1, const float* __restrict__ b1,
                                                            const float* __restrict__ W2, const float* __restrict__ b2,
                                                            const float* __restrict__ C, int E, int F,
                                                            float* __restrict__ Wout, float* __restrict__ H1) {
  __shared__ __attribute__((aligned(16))) float xs[kEB][kLd];
  __shared__ __attribute__((aligned(16))) float as[kEB][kLd];
  __shared__ float ws[2][kMaxW][kMaxW + 1];  // W1, W2 rows (odd stride: row-per-lane reads conflict-free)
  const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int e0 = blockIdx.x * kEB;
  // every global load of the staging is issued before the first LDS store (a loop that
  // stores each load to LDS waits one memory latency per iteration)
  float tx[kEB / 4], t1[kMaxW / 4], t2[kMaxW / 4];
#pragma unroll
  for (int u = 0; u < kEB / 4; ++u) {
    const int r = q + 4 * u;
    tx[u] = (e0 + r < E && c < K) ? rbf[(int64_t)(e0 + r) * ldr + c] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < kMaxW / 4; ++u) {  // row r of W1 / W2: lanes over its columns (coalesced)
    const int r = q + 4 * u;
    t1[u] = (r < F && c < K) ? W1[r * K + c] : 0.f;
    t2[u] = (r < F && c < F) ? W2[r * F + c] : 0.f;
  }
  const float bias1 = c < F ? b1[c] : 0.f, bias2 = c < F ? b2[c] : 0.f;
#pragma unroll
  for (int u = 0; u < kEB / 4; ++u) xs[q + 4 * u][c] = tx[u];
#pragma unroll
  for (int u = 0; u < kMaxW / 4; ++u) {
    ws[0][q + 4 * u][c] = t1[u];
    ws[1][q + 4 * u][c] = t2[u];
  }
  __syncthreads();
  float w[kMaxW];
#pragma unroll
  for (int k = 0; k < kMaxW; ++k) w[k] = (c < F && k < K) ? ws[0][c][k] : 0.f;
  constexpr float kLog2 = 0.69314718055994531f;
#pragma unroll 2
  for (int u = 0; u < kEB / 4; ++u) {
    const int r = q + 4 * u, e = e0 + r;
    const float h = bias1 + rowdot(xs[r], w);
    if (e < E && c < F) H1[(int64_t)e * F + c] = h;
    as[r][c] = c < F ? softplus(h) - kLog2 : 0.f;
  }
#pragma unroll
  for (int k = 0; k < kMaxW; ++k) w[k] = (c < F && k < F) ? ws[1][c][k] : 0.f;
#pragma unroll 2
  for (int u = 0; u < kEB / 4; ++u) {
    const int r = q + 4 * u, e = e0 + r;
    const float v = bias2 + rowdot(as[r], w);
    if (e < E && c < F) Wout[(int64_t)e * F + c] = v * C[e];
  }
}

__global__ void __launch_bounds__(256) cf_filter_bwd_kernel(const float* __restrict__ dW, const float* __restrict__ C,
                                                            const float* __restrict__ H1,
                                                            const float* __restrict__ W2, int E, int F,
                                                            float* __restrict__ dH2, float* __restrict__ A1,
                                                            float* __restrict__ dH1) {
  __shared__ __attribute__((aligned(16))) float gs[kEB][kLd];
  const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int e0 = blockIdx.x * kEB;
  float tg[kEB / 4], tc[kEB / 4];
#pragma unroll
  for (int u = 0; u < kEB / 4; ++u) {  // all loads in flight before any use
    const int e = e0 + q + 4 * u;
    tg[u] = (e < E && c < F) ? dW[(int64_t)e * F + c] : 0.f;
    tc[u] = e < E ? C[e] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < kEB / 4; ++u) {
    const int r = q + 4 * u, e = e0 + r;
    const float g = tg[u] * tc[u];
    if (e < E && c < F) dH2[(int64_t)e * F + c] = g;
    gs[r][c] = g;
  }
  // dgrad operand: column c of W2 (da1[e, c] = sum_j dh2[e, j] W2[j, c])
  float w[kMaxW];
#pragma unroll
  for (int k = 0; k < kMaxW; ++k) w[k] = (c < F && k < F) ? W2[k * F + c] : 0.f;
  __syncthreads();
  constexpr float kLog2 = 0.69314718055994531f;
#pragma unroll 2
  for (int u = 0; u < kEB / 4; ++u) {
    const int r = q + 4 * u, e = e0 + r;
    const float da = rowdot(gs[r], w);
    if (e < E && c < F) {
      const int64_t o = (int64_t)e * F + c;
      const float h = H1[o];
      A1[o] = softplus(h) - kLog2;
      dH1[o] = da * (h > 20.f ? 1.f : sigm(h));
    }
  }
}

}  // namespace sch

static void cf_check(const at::Tensor& t, const char* name) {
  HY_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), name, " must be a contiguous fp32 GPU tensor");
}

// rbf [E, K] (row stride ldr, unit column stride), W1 [F, K], b1 [F], W2 [F, F], b2 [F], C [E]
std::vector<at::Tensor> cf_filter_fwd(const at::Tensor& rbf, const at::Tensor& W1, const at::Tensor& b1,
                                      const at::Tensor& W2, const at::Tensor& b2, const at::Tensor& C) {
  HY_CHECK(rbf.is_cuda() && rbf.scalar_type() == at::kFloat && rbf.dim() == 2 && rbf.stride(1) == 1,
           "cf_filter_fwd: rbf [E, K] fp32 with unit column stride");
  cf_check(W1, "W1");
  cf_check(b1, "b1");
  cf_check(W2, "W2");
  cf_check(b2, "b2");
  cf_check(C, "C");
  const int64_t E = rbf.size(0);
  const int K = (int)rbf.size(1), F = (int)W1.size(0);
  HY_CHECK(K <= sch::kMaxW && F <= sch::kMaxW && W1.size(1) == K && b1.numel() == F && W2.size(0) == F &&
               W2.size(1) == F && b2.numel() == F && C.numel() == E && E < (1LL << 31),
           "cf_filter_fwd: shapes (K, F <= 64)");
  auto Wout = at::empty({E, F}, rbf.options()), H1 = at::empty({E, F}, rbf.options());
  if (E)
    sch::cf_filter_fwd_kernel<<<ceil_div(E, sch::kEB), 256, 0, stream()>>>(
        rbf.data_ptr<float>(), (int)rbf.stride(0), K, W1.data_ptr<float>(), b1.data_ptr<float>(), W2.data_ptr<float>(),
        b2.data_ptr<float>(), C.data_ptr<float>(), (int)E, F, Wout.data_ptr<float>(), H1.data_ptr<float>());
  return {Wout, H1};
}

// -> (dh2, a1, dh1), each [E, F]
std::vector<at::Tensor> cf_filter_bwd(const at::Tensor& dW_, const at::Tensor& C, const at::Tensor& H1,
                                      const at::Tensor& W2) {
  auto dW = dW_.contiguous();
  cf_check(dW, "dW");
  cf_check(C, "C");
  cf_check(H1, "H1");
  cf_check(W2, "W2");
  const int64_t E = H1.size(0);
  const int F = (int)H1.size(1);
  HY_CHECK(F <= sch::kMaxW && dW.sizes() == H1.sizes() && C.numel() == E && W2.size(0) == F && W2.size(1) == F,
           "cf_filter_bwd: shapes");
  auto dH2 = at::empty_like(H1), A1 = at::empty_like(H1), dH1 = at::empty_like(H1);
  if (E)
    sch::cf_filter_bwd_kernel<<<ceil_div(E, sch::kEB), 256, 0, stream()>>>(
        dW.data_ptr<float>(), C.data_ptr<float>(), H1.data_ptr<float>(), W2.data_ptr<float>(), (int)E, F,
        dH2.data_ptr<float>(), A1.data_ptr<float>(), dH1.data_ptr<float>());
  return {dH2, A1, dH1};
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("cf_filter_fwd(Tensor rbf, Tensor W1, Tensor b1, Tensor W2, Tensor b2, Tensor C) -> Tensor[]");
  m.def("cf_filter_bwd(Tensor dW, Tensor C, Tensor H1, Tensor W2) -> Tensor[]");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("cf_filter_fwd", hy::cf_filter_fwd);
  m.impl("cf_filter_bwd", hy::cf_filter_bwd);
}
