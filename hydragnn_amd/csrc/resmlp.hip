// Residual SiLU block in one launch each way (DimeNet++ ResidualLayer, reference
// hydragnn/models/DIMEStack.py -> PyG ResidualLayer: y = x + act(lin2(act(lin1(x)))), act = SiLU):
//
//   forward   h1 = x W1^T + b1,  a1 = silu(h1),  h2 = a1 W2^T + b2,  y = x + silu(h2)
//             -> y, h1, h2 (the backward's saved pre-activations)
//   backward  dh2 = dy * silu'(h2),  a1 = silu(h1),  dh1 = (dh2 W2) * silu'(h1),
//             dx = dy + dh1 W1
//             -> dx and the row factors (dh2, a1) / (dh1, x) of the four weight/bias
//                gradients, which join the step's grouped weight-gradient launch.
//
// Five launches forward (two GEMMs, two activations, the residual add) and seven backward
// become one each: edge-sized (~2x10^4 rows) maps of width 64 are launch/latency-bound on
// MI355X (each library GEMM ~10 us on 40 workgroups).  Layout as csrc/schnet.hip: a
// workgroup owns 16 rows, wave q rows q, q+4, ..., lane c column c; weights staged through
// LDS with every global load issued before the first LDS store; row inputs read from LDS as
// wave-wide broadcasts.
#include "common.h"

namespace hy {
namespace rm {

constexpr int kRB = 16;    // rows per workgroup
constexpr int kMaxW = 64;  // F <= 64
constexpr int kLd = kMaxW + 4;

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float silu(float x) { return x * sigm(x); }
__device__ __forceinline__ float dsilu(float x) {
  const float s = sigm(x);
  return s * (1.f + x * (1.f - s));
}

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

// rows of two F x F weights into LDS (row r, lanes over its columns; loads first)
__device__ __forceinline__ void stage_weights(float (*ws)[kMaxW][kMaxW + 1], const float* __restrict__ W1,
                                              const float* __restrict__ W2, int F, int c, int q) {
  float t1[kMaxW / 4], t2[kMaxW / 4];
#pragma unroll
  for (int u = 0; u < kMaxW / 4; ++u) {
    const int r = q + 4 * u;
    t1[u] = (r < F && c < F) ? W1[r * F + c] : 0.f;
    t2[u] = (r < F && c < F) ? W2[r * F + c] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < kMaxW / 4; ++u) {
    ws[0][q + 4 * u][c] = t1[u];
    ws[1][q + 4 * u][c] = t2[u];
  }
}

__global__ void __launch_bounds__(256) res_mlp_fwd_kernel(const float* __restrict__ x, const float* __restrict__ W1,
                                                          const float* __restrict__ b1, const float* __restrict__ W2,
                                                          const float* __restrict__ b2, int M, int F,
                                                          float* __restrict__ y, float* __restrict__ H1,
                                                          float* __restrict__ H2) {
  __shared__ __attribute__((aligned(16))) float xs[kRB][kLd];
  __shared__ __attribute__((aligned(16))) float as[kRB][kLd];
  __shared__ float ws[2][kMaxW][kMaxW + 1];
  const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int m0 = blockIdx.x * kRB;
  float tx[kRB / 4];
#pragma unroll
  for (int u = 0; u < kRB / 4; ++u) {
    const int m = m0 + q + 4 * u;
    tx[u] = (m < M && c < F) ? x[(int64_t)m * F + c] : 0.f;
  }
  stage_weights(ws, W1, W2, F, c, q);
  const float bias1 = c < F ? b1[c] : 0.f, bias2 = c < F ? b2[c] : 0.f;
#pragma unroll
  for (int u = 0; u < kRB / 4; ++u) xs[q + 4 * u][c] = tx[u];
  __syncthreads();
  float w[kMaxW];
#pragma unroll
  for (int k = 0; k < kMaxW; ++k) w[k] = (c < F && k < F) ? ws[0][c][k] : 0.f;
#pragma unroll
  for (int u = 0; u < kRB / 4; ++u) {  // rows of wave q only: no barrier before their reads
    const int r = q + 4 * u, m = m0 + r;
    const float h = bias1 + rowdot(xs[r], w);
    if (m < M && c < F) H1[(int64_t)m * F + c] = h;
    as[r][c] = c < F ? silu(h) : 0.f;
  }
#pragma unroll
  for (int k = 0; k < kMaxW; ++k) w[k] = (c < F && k < F) ? ws[1][c][k] : 0.f;
#pragma unroll
  for (int u = 0; u < kRB / 4; ++u) {
    const int r = q + 4 * u, m = m0 + r;
    const float h = bias2 + rowdot(as[r], w);
    if (m < M && c < F) {
      H2[(int64_t)m * F + c] = h;
      y[(int64_t)m * F + c] = xs[r][c] + silu(h);
    }
  }
}

__global__ void __launch_bounds__(256) res_mlp_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ H1,
                                                          const float* __restrict__ H2, const float* __restrict__ W1,
                                                          const float* __restrict__ W2, int M, int F,
                                                          float* __restrict__ dx, float* __restrict__ dH2,
                                                          float* __restrict__ A1, float* __restrict__ dH1) {
  __shared__ __attribute__((aligned(16))) float gs[kRB][kLd];  // dh2 rows
  __shared__ __attribute__((aligned(16))) float hs[kRB][kLd];  // dh1 rows
  __shared__ float ws[2][kMaxW][kMaxW + 1];
  const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int m0 = blockIdx.x * kRB;
  float tg[kRB / 4], th2[kRB / 4], th1[kRB / 4];
#pragma unroll
  for (int u = 0; u < kRB / 4; ++u) {
    const int m = m0 + q + 4 * u;
    const bool ok = m < M && c < F;
    tg[u] = ok ? dy[(int64_t)m * F + c] : 0.f;
    th2[u] = ok ? H2[(int64_t)m * F + c] : 0.f;
    th1[u] = ok ? H1[(int64_t)m * F + c] : 0.f;
  }
  stage_weights(ws, W1, W2, F, c, q);
#pragma unroll
  for (int u = 0; u < kRB / 4; ++u) {
    const int r = q + 4 * u, m = m0 + r;
    const float g = tg[u] * dsilu(th2[u]);
    if (m < M && c < F) dH2[(int64_t)m * F + c] = g;
    gs[r][c] = c < F ? g : 0.f;
  }
  __syncthreads();  // weights
  // da1[m, c] = sum_j dh2[m, j] W2[j, c]: column c of W2
  float w[kMaxW];
#pragma unroll
  for (int k = 0; k < kMaxW; ++k) w[k] = (c < F && k < F) ? ws[1][k][c] : 0.f;
#pragma unroll
  for (int u = 0; u < kRB / 4; ++u) {
    const int r = q + 4 * u, m = m0 + r;
    const float da = rowdot(gs[r], w);
    const float h = th1[u];
    const float d1 = da * dsilu(h);
    if (m < M && c < F) {
      A1[(int64_t)m * F + c] = silu(h);
      dH1[(int64_t)m * F + c] = d1;
    }
    hs[r][c] = c < F ? d1 : 0.f;
  }
#pragma unroll
  for (int k = 0; k < kMaxW; ++k) w[k] = (c < F && k < F) ? ws[0][k][c] : 0.f;
#pragma unroll
  for (int u = 0; u < kRB / 4; ++u) {
    const int r = q + 4 * u, m = m0 + r;
    const float v = tg[u] + rowdot(hs[r], w);
    if (m < M && c < F) dx[(int64_t)m * F + c] = v;
  }
}

// One SiLU linear in one launch each way (the DimeNet++ interaction / embedding blocks'
// act(lin(x)) * m + a chains, reference DIMEStack.py -> PyG InteractionPPBlock):
//   forward   z = x W^T + b,  y = silu(z) * mul + add      (mul / add optional, [M, O])
//   backward  g = dy * mul,  dz = g * silu'(z),  dx = dz W,  dmul = dy * silu(z)
// (z saved by the forward; the weight gradient's row factors (dz, x) join the step's grouped
// weight-gradient launch).  I, O <= 64; layout as the residual block above.
__global__ void __launch_bounds__(256) lin_act_fwd_kernel(const float* __restrict__ x, const float* __restrict__ W,
                                                          const float* __restrict__ b, const float* __restrict__ mul,
                                                          const float* __restrict__ add, int M, int I, int O,
                                                          float scale, int trans, float* __restrict__ y,
                                                          float* __restrict__ Z) {
  __shared__ __attribute__((aligned(16))) float xs[kRB][kLd];
  __shared__ float ws[kMaxW][kMaxW + 1];
  const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int m0 = blockIdx.x * kRB;
  float tx[kRB / 4], tw[kMaxW / 4];
#pragma unroll
  for (int u = 0; u < kRB / 4; ++u) {
    const int m = m0 + q + 4 * u;
    tx[u] = (m < M && c < I) ? x[(int64_t)m * I + c] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < kMaxW / 4; ++u) {
    const int r = q + 4 * u;
    tw[u] = (r < O && c < I) ? W[trans ? c * O + r : r * I + c] : 0.f;
  }
  const float bias = (b != nullptr && c < O) ? b[c] : 0.f;
#pragma unroll
  for (int u = 0; u < kRB / 4; ++u) xs[q + 4 * u][c] = tx[u];
#pragma unroll
  for (int u = 0; u < kMaxW / 4; ++u) ws[q + 4 * u][c] = tw[u];
  __syncthreads();
  float w[kMaxW];
#pragma unroll
  for (int k = 0; k < kMaxW; ++k) w[k] = (c < O && k < I) ? ws[c][k] : 0.f;
#pragma unroll
  for (int u = 0; u < kRB / 4; ++u) {
    const int r = q + 4 * u, m = m0 + r;
    if (m < M && c < O) {
      const float z = scale * (bias + rowdot(xs[r], w));
      const int64_t o = (int64_t)m * O + c;
      Z[o] = z;
      float v = silu(z);
      if (mul != nullptr) v *= mul[o];
      if (add != nullptr) v += add[o];
      y[o] = v;
    }
  }
}

__global__ void __launch_bounds__(256) lin_act_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ Z,
                                                          const float* __restrict__ W, const float* __restrict__ mul,
                                                          int M, int I, int O, float scale, int trans,
                                                          float* __restrict__ dx, float* __restrict__ dZ,
                                                          float* __restrict__ dmul) {
  __shared__ __attribute__((aligned(16))) float gs[kRB][kLd];
  __shared__ float ws[kMaxW][kMaxW + 1];
  const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int m0 = blockIdx.x * kRB;
  float tg[kRB / 4], tz[kRB / 4], tm[kRB / 4], tw[kMaxW / 4];
#pragma unroll
  for (int u = 0; u < kRB / 4; ++u) {
    const int m = m0 + q + 4 * u;
    const bool ok = m < M && c < O;
    tg[u] = ok ? dy[(int64_t)m * O + c] : 0.f;
    tz[u] = ok ? Z[(int64_t)m * O + c] : 0.f;
    tm[u] = (ok && mul != nullptr) ? mul[(int64_t)m * O + c] : 1.f;
  }
#pragma unroll
  for (int u = 0; u < kMaxW / 4; ++u) {
    const int r = q + 4 * u;
    tw[u] = (r < O && c < I) ? W[trans ? c * O + r : r * I + c] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < kMaxW / 4; ++u) ws[q + 4 * u][c] = tw[u];
#pragma unroll
  for (int u = 0; u < kRB / 4; ++u) {
    const int r = q + 4 * u, m = m0 + r;
    const float g = tg[u] * tm[u] * dsilu(tz[u]) * scale;
    if (m < M && c < O) {
      const int64_t o = (int64_t)m * O + c;
      dZ[o] = g;
      if (dmul != nullptr) dmul[o] = tg[u] * silu(tz[u]);
    }
    gs[r][c] = c < O ? g : 0.f;
  }
  __syncthreads();
  // dx[m, i] = sum_o dz[m, o] W[o, i]: column i of W
  float w[kMaxW];
#pragma unroll
  for (int k = 0; k < kMaxW; ++k) w[k] = (k < O && c < I) ? ws[k][c] : 0.f;
#pragma unroll
  for (int u = 0; u < kRB / 4; ++u) {
    const int r = q + 4 * u, m = m0 + r;
    if (m < M && c < I) dx[(int64_t)m * I + c] = rowdot(gs[r], w);
  }
}

}  // namespace rm

static void rm_check(const at::Tensor& t, const char* name) {
  HY_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), name, " must be a contiguous fp32 GPU tensor");
}

// x [M, F], W1/W2 [F, F], b1/b2 [F] -> (y, h1, h2)
std::vector<at::Tensor> res_mlp_fwd(const at::Tensor& x, const at::Tensor& W1, const at::Tensor& b1,
                                    const at::Tensor& W2, const at::Tensor& b2) {
  rm_check(x, "x");
  rm_check(W1, "W1");
  rm_check(b1, "b1");
  rm_check(W2, "W2");
  rm_check(b2, "b2");
  HY_CHECK(x.dim() == 2, "res_mlp_fwd: x [M, F]");
  const int64_t M = x.size(0);
  const int F = (int)x.size(1);
  HY_CHECK(F <= rm::kMaxW && W1.size(0) == F && W1.size(1) == F && W2.size(0) == F && W2.size(1) == F &&
               b1.numel() == F && b2.numel() == F && M < (1LL << 31),
           "res_mlp_fwd: shapes (F <= 64, square weights)");
  auto y = at::empty_like(x), H1 = at::empty_like(x), H2 = at::empty_like(x);
  if (M)
    rm::res_mlp_fwd_kernel<<<ceil_div(M, rm::kRB), 256, 0, stream()>>>(
        x.data_ptr<float>(), W1.data_ptr<float>(), b1.data_ptr<float>(), W2.data_ptr<float>(), b2.data_ptr<float>(),
        (int)M, F, y.data_ptr<float>(), H1.data_ptr<float>(), H2.data_ptr<float>());
  return {y, H1, H2};
}

// -> (dx, dh2, a1, dh1)
std::vector<at::Tensor> res_mlp_bwd(const at::Tensor& dy_, const at::Tensor& H1, const at::Tensor& H2,
                                    const at::Tensor& W1, const at::Tensor& W2) {
  auto dy = dy_.contiguous();
  rm_check(dy, "dy");
  rm_check(H1, "H1");
  rm_check(H2, "H2");
  rm_check(W1, "W1");
  rm_check(W2, "W2");
  const int64_t M = H1.size(0);
  const int F = (int)H1.size(1);
  HY_CHECK(F <= rm::kMaxW && dy.sizes() == H1.sizes() && H2.sizes() == H1.sizes() && W1.size(0) == F &&
               W1.size(1) == F && W2.size(0) == F && W2.size(1) == F,
           "res_mlp_bwd: shapes");
  auto dx = at::empty_like(H1), dH2 = at::empty_like(H1), A1 = at::empty_like(H1), dH1 = at::empty_like(H1);
  if (M)
    rm::res_mlp_bwd_kernel<<<ceil_div(M, rm::kRB), 256, 0, stream()>>>(
        dy.data_ptr<float>(), H1.data_ptr<float>(), H2.data_ptr<float>(), W1.data_ptr<float>(), W2.data_ptr<float>(),
        (int)M, F, dx.data_ptr<float>(), dH2.data_ptr<float>(), A1.data_ptr<float>(), dH1.data_ptr<float>());
  return {dx, dH2, A1, dH1};
}

// x [M, I], W [O, I], b [O] | None, mul / add [M, O] | None -> (y, z)
// scale s: z = s (x W^T + b) (the activation's pre-scale; dZ carries it back); trans: W is
// [I, O] (the e3nn ``x @ W`` layout) instead of [O, I]
std::vector<at::Tensor> lin_act_fwd(const at::Tensor& x, const at::Tensor& W, const c10::optional<at::Tensor>& b,
                                    const c10::optional<at::Tensor>& mul, const c10::optional<at::Tensor>& add,
                                    double scale, bool trans) {
  rm_check(x, "x");
  rm_check(W, "W");
  const int64_t Wi = trans ? W.size(0) : W.size(1), Wo = trans ? W.size(1) : W.size(0);
  HY_CHECK(x.dim() == 2 && W.dim() == 2 && Wi == x.size(1) && x.size(1) <= rm::kMaxW && Wo <= rm::kMaxW,
           "lin_act_fwd: x [M, I], W [O, I] ([I, O] with trans), I, O <= 64");
  const int64_t M = x.size(0);
  const int I = (int)x.size(1), O = (int)Wo;
  const float *bp = nullptr, *mp = nullptr, *ap = nullptr;
  if (b.has_value() && b->defined()) {
    rm_check(*b, "b");
    HY_CHECK(b->numel() == O, "lin_act_fwd: b [O]");
    bp = b->data_ptr<float>();
  }
  if (mul.has_value() && mul->defined()) {
    rm_check(*mul, "mul");
    HY_CHECK(mul->numel() == M * O, "lin_act_fwd: mul [M, O]");
    mp = mul->data_ptr<float>();
  }
  if (add.has_value() && add->defined()) {
    rm_check(*add, "add");
    HY_CHECK(add->numel() == M * O, "lin_act_fwd: add [M, O]");
    ap = add->data_ptr<float>();
  }
  auto y = at::empty({M, O}, x.options()), Z = at::empty({M, O}, x.options());
  if (M)
    rm::lin_act_fwd_kernel<<<ceil_div(M, rm::kRB), 256, 0, stream()>>>(x.data_ptr<float>(), W.data_ptr<float>(), bp, mp,
                                                                         ap, (int)M, I, O, (float)scale, trans ? 1 : 0,
                                                                         y.data_ptr<float>(), Z.data_ptr<float>());
  return {y, Z};
}

// -> (dx, dz, dmul | empty)
std::vector<at::Tensor> lin_act_bwd(const at::Tensor& dy_, const at::Tensor& Z, const at::Tensor& W,
                                    const c10::optional<at::Tensor>& mul, bool want_dmul, double scale, bool trans) {
  auto dy = dy_.contiguous();
  rm_check(dy, "dy");
  rm_check(Z, "Z");
  rm_check(W, "W");
  const int64_t M = Z.size(0);
  const int O = (int)Z.size(1), I = (int)(trans ? W.size(0) : W.size(1));
  HY_CHECK(dy.sizes() == Z.sizes() && (trans ? W.size(1) : W.size(0)) == O && I <= rm::kMaxW && O <= rm::kMaxW,
           "lin_act_bwd: shapes");
  const float* mp = nullptr;
  if (mul.has_value() && mul->defined()) {
    rm_check(*mul, "mul");
    HY_CHECK(mul->sizes() == Z.sizes(), "lin_act_bwd: mul [M, O]");
    mp = mul->data_ptr<float>();
  }
  auto dx = at::empty({M, (int64_t)I}, Z.options()), dZ = at::empty_like(Z);
  auto dmul = want_dmul ? at::empty_like(Z) : at::empty({0}, Z.options());
  if (M)
    rm::lin_act_bwd_kernel<<<ceil_div(M, rm::kRB), 256, 0, stream()>>>(
        dy.data_ptr<float>(), Z.data_ptr<float>(), W.data_ptr<float>(), mp, (int)M, I, O, (float)scale, trans ? 1 : 0,
        dx.data_ptr<float>(), dZ.data_ptr<float>(), want_dmul ? dmul.data_ptr<float>() : nullptr);
  return {dx, dZ, dmul};
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("res_mlp_fwd(Tensor x, Tensor W1, Tensor b1, Tensor W2, Tensor b2) -> Tensor[]");
  m.def("res_mlp_bwd(Tensor dy, Tensor H1, Tensor H2, Tensor W1, Tensor W2) -> Tensor[]");
  m.def("lin_act_fwd(Tensor x, Tensor W, Tensor? b, Tensor? mul, Tensor? add, float scale=1.0, bool trans=False) "
        "-> Tensor[]");
  m.def("lin_act_bwd(Tensor dy, Tensor Z, Tensor W, Tensor? mul, bool want_dmul, float scale=1.0, bool trans=False) "
        "-> Tensor[]");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("res_mlp_fwd", hy::res_mlp_fwd);
  m.impl("res_mlp_bwd", hy::res_mlp_bwd);
  m.impl("lin_act_fwd", hy::lin_act_fwd);
  m.impl("lin_act_bwd", hy::lin_act_bwd);
}
