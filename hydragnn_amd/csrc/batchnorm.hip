// Training-mode BatchNorm over node rows [N, F] with an optional valid-row count (gfx950).
//
// Reference: PyG BatchNorm -> torch BatchNorm1d (Base.py:206,215,466; gps.py:80-83),
// 4 per GPS layer.  torch's channels-last BN issues 4 kernels forward + 3 backward
// for an [N, 64] tensor.  Here: forward = partial (sum, sumsq) per row slab +
// one apply kernel in which every workgroup re-reduces the (tiny) partials, block 0
// also writing the saved statistics and the running-stat update; backward = the
// same two-pass shape.  Rows >= num_valid (static padding for hipGraph capture)
// are excluded from the statistics but still normalised, exactly matching the
// masked reference path in ops/norm.py.  Per-slab partials are combined with
// Chan's parallel-variance formula in a fixed order (deterministic).
#include "common.h"

namespace hy {

constexpr int kBnRows = 128;  // rows per slab

__device__ __forceinline__ int nvalid_of(const int* nv, int N) { return nv ? min(*nv, N) : N; }

// part: [S][3][F] = (count, mean, std) per slab, per column.  Two passes over the
// (L2-hot) slab: mean first, then M2 = sum (x - mean)^2 — no E[x^2] - E[x]^2
// cancellation, and no overflow of sum x^2 for large activations (|x| ~ 1e19
// appears when a deep multiplicative stack such as DimeNet drifts in training;
// the one-pass form turned that into inf - inf = NaN statistics).
__global__ void __launch_bounds__(256) bn_fwd_partial_kernel(const float* __restrict__ x, const int* __restrict__ nv,
                                                             float* __restrict__ part, int N, int F, int tpr) {
  const int s = blockIdx.x;
  const int Nv = nvalid_of(nv, N);
  const int r0 = s * kBnRows, r1 = min(Nv, r0 + kBnRows);
  const int rl = threadIdx.x / tpr, c = threadIdx.x % tpr;
  const int rpb = 256 / tpr;
  const float n = (float)max(r1 - r0, 0);
  __shared__ float red[256];
  __shared__ double redd[256];
  __shared__ float smu[64];
  // every thread runs the same number of column passes (barriers stay uniform)
  for (int f0 = 0; f0 < F; f0 += tpr) {
    const int f = f0 + c;
    const bool act = f < F;
    float sm = 0.f;
    if (act)
      for (int r = r0 + rl; r < r1; r += rpb) sm += x[(int64_t)r * F + f];
    red[threadIdx.x] = sm;
    __syncthreads();
    if (rl == 0) {
      float a = 0.f;
      for (int k = 0; k < rpb; ++k) a += red[k * tpr + c];
      smu[c] = n > 0.f ? a / n : 0.f;
    }
    __syncthreads();
    const float mu = smu[c];
    double sq = 0.0;  // fp64: (x - mu)^2 overflows fp32 for |x| > 1.8e19
    if (act)
      for (int r = r0 + rl; r < r1; r += rpb) {
        const double t = (double)x[(int64_t)r * F + f] - (double)mu;
        sq = fma(t, t, sq);
      }
    redd[threadIdx.x] = sq;
    __syncthreads();
    if (rl == 0 && act) {
      double b = 0.0;
      for (int k = 0; k < rpb; ++k) b += redd[k * tpr + c];
      part[((int64_t)s * 3 + 0) * F + f] = n;
      part[((int64_t)s * 3 + 1) * F + f] = mu;
      part[((int64_t)s * 3 + 2) * F + f] = n > 0.f ? (float)sqrt(b / (double)n) : 0.f;  // slab std
    }
    __syncthreads();
  }
}

// combine slabs in a fixed order (fp64): mean, biased var
__device__ __forceinline__ void bn_combine(const float* part, int S, int F, int f, float& mean, double& var) {
  double n = 0.0, sm = 0.0;
  for (int s = 0; s < S; ++s) {
    const double nb = part[((int64_t)s * 3 + 0) * F + f];
    n += nb;
    sm += nb * (double)part[((int64_t)s * 3 + 1) * F + f];
  }
  const double m = n > 0.0 ? sm / n : 0.0;
  double M2 = 0.0;
  for (int s = 0; s < S; ++s) {
    const double nb = part[((int64_t)s * 3 + 0) * F + f];
    if (nb <= 0.0) continue;
    const double d = (double)part[((int64_t)s * 3 + 1) * F + f] - m;
    const double sd = part[((int64_t)s * 3 + 2) * F + f];
    M2 += nb * (sd * sd + d * d);
  }
  mean = (float)m;
  var = n > 0.0 ? M2 / n : 0.0;
}

__global__ void __launch_bounds__(256) bn_fwd_apply_kernel(
    const float* __restrict__ x, const int* __restrict__ nv, const float* __restrict__ part, int S,
    const float* __restrict__ w, const float* __restrict__ b, float* __restrict__ y, float* __restrict__ save_mean,
    float* __restrict__ save_invstd, float* __restrict__ rmean, float* __restrict__ rvar, float momentum, float eps,
    int N, int F, int relu, int rows_per_block) {
  extern __shared__ float sh[];  // [2][F]
  float* smean = sh;
  float* sinv = sh + F;
  for (int f = threadIdx.x; f < F; f += 256) {
    float mean;
    double var;
    bn_combine(part, S, F, f, mean, var);
    const float inv = (float)(1.0 / sqrt(var + (double)eps));
    smean[f] = mean;
    sinv[f] = inv;
    if (blockIdx.x == 0) {
      save_mean[f] = mean;
      save_invstd[f] = inv;
      if (rmean) {
        const int Nv = nvalid_of(nv, N);
        const float unb = (float)(Nv > 1 ? var * (double)Nv / (double)(Nv - 1) : var);
        rmean[f] = (1.f - momentum) * rmean[f] + momentum * mean;
        rvar[f] = (1.f - momentum) * rvar[f] + momentum * unb;
      }
    }
  }
  __syncthreads();
  const int64_t e0 = (int64_t)blockIdx.x * rows_per_block * F;
  const int64_t e1 = min((int64_t)N * F, e0 + (int64_t)rows_per_block * F);
  for (int64_t e = e0 + threadIdx.x; e < e1; e += 256) {
    const int f = (int)(e % F);
    float v = (x[e] - smean[f]) * sinv[f];
    if (w) v = fmaf(v, w[f], b[f]);
    if (relu) v = fmaxf(v, 0.f);
    y[e] = v;
  }
}

// backward partials over ALL rows: [S][2][F] = (sum dy, sum dy*xhat)
__global__ void __launch_bounds__(256) bn_bwd_partial_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ invstd,
                                                             float* __restrict__ part, int N, int F, int tpr) {
  const int s = blockIdx.x;
  const int r0 = s * kBnRows, r1 = min(N, r0 + kBnRows);
  const int rl = threadIdx.x / tpr, c = threadIdx.x % tpr;
  const int rpb = 256 / tpr;
  __shared__ float red[256 * 2];
  for (int f0 = 0; f0 < F; f0 += tpr) {
    const int f = f0 + c;
    const bool act = f < F;
    float a = 0.f, b = 0.f;
    if (act) {
      const float mu = mean[f], is = invstd[f];
      for (int r = r0 + rl; r < r1; r += rpb) {
        const float g = dy[(int64_t)r * F + f];
        a += g;
        b = fmaf(g, (x[(int64_t)r * F + f] - mu) * is, b);
      }
    }
    red[threadIdx.x] = a;
    red[256 + threadIdx.x] = b;
    __syncthreads();
    if (rl == 0 && act) {
      float sa = 0.f, sb = 0.f;
      for (int k = 0; k < rpb; ++k) {
        sa += red[k * tpr + c];
        sb += red[256 + k * tpr + c];
      }
      part[((int64_t)s * 2 + 0) * F + f] = sa;
      part[((int64_t)s * 2 + 1) * F + f] = sb;
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, const int* __restrict__ nv,
    const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ w,
    const float* __restrict__ part, int S, float* __restrict__ dx, float* __restrict__ dw, float* __restrict__ db,
    int N, int F, int rows_per_block) {
  extern __shared__ float sh[];  // [2][F]
  float* sdy = sh;
  float* sdyx = sh + F;
  for (int f = threadIdx.x; f < F; f += 256) {
    float a = 0.f, b = 0.f;
    for (int s = 0; s < S; ++s) {
      a += part[((int64_t)s * 2 + 0) * F + f];
      b += part[((int64_t)s * 2 + 1) * F + f];
    }
    sdy[f] = a;
    sdyx[f] = b;
    if (blockIdx.x == 0 && dw) {
      dw[f] = b;
      db[f] = a;
    }
  }
  __syncthreads();
  const int Nv = nvalid_of(nv, N);
  const float invn = 1.f / (float)max(Nv, 1);
  const int64_t e0 = (int64_t)blockIdx.x * rows_per_block * F;
  const int64_t e1 = min((int64_t)N * F, e0 + (int64_t)rows_per_block * F);
  for (int64_t e = e0 + threadIdx.x; e < e1; e += 256) {
    const int f = (int)(e % F);
    const int r = (int)(e / F);
    const float is = invstd[f];
    const float g = dy[e] * (w ? w[f] : 1.f) * is;
    if (r < Nv) {
      const float xh = (x[e] - mean[f]) * is;
      dx[e] = g - (w ? w[f] : 1.f) * is * invn * (sdy[f] + xh * sdyx[f]);
    } else {
      dx[e] = g;
    }
  }
}

static int bn_tpr(int F) {
  int t = 1;
  while (t < F && t < 64) t <<= 1;
  return t;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> bn_forward(const at::Tensor& x_, const c10::optional<at::Tensor>& nv,
                                                          const c10::optional<at::Tensor>& w,
                                                          const c10::optional<at::Tensor>& b,
                                                          const c10::optional<at::Tensor>& rmean,
                                                          const c10::optional<at::Tensor>& rvar, double momentum,
                                                          double eps, bool relu) {
  HY_CHECK_CUDA(x_);
  auto x = x_.contiguous();
  HY_CHECK_F32(x);
  const int N = (int)x.size(0), F = (int)x.size(1);
  auto y = at::empty_like(x);
  auto smean = at::empty({F}, x.options());
  auto sinv = at::empty({F}, x.options());
  if (N == 0) return {y, smean, sinv};
  const int S = ceil_div(N, kBnRows);
  auto part = at::empty({S, 3, F}, x.options());
  const int* nvp = nullptr;
  if (nv.has_value() && nv->defined()) {
    HY_CHECK(nv->scalar_type() == at::kInt && nv->numel() == 1, "num_valid must be an int32 scalar");
    nvp = nv->data_ptr<int>();
  }
  bn_fwd_partial_kernel<<<S, 256, 0, stream()>>>(x.data_ptr<float>(), nvp, part.data_ptr<float>(), N, F, bn_tpr(F));
  const int rpb = std::max(1, 2048 / std::max(F, 1));
  const int blocks = ceil_div(N, rpb);
  const bool track = rmean.has_value() && rmean->defined();
  bn_fwd_apply_kernel<<<blocks, 256, 2 * F * sizeof(float), stream()>>>(
      x.data_ptr<float>(), nvp, part.data_ptr<float>(), S, w.has_value() && w->defined() ? w->data_ptr<float>() : nullptr,
      b.has_value() && b->defined() ? b->data_ptr<float>() : nullptr, y.data_ptr<float>(), smean.data_ptr<float>(),
      sinv.data_ptr<float>(), track ? rmean->data_ptr<float>() : nullptr, track ? rvar->data_ptr<float>() : nullptr,
      (float)momentum, (float)eps, N, F, relu ? 1 : 0, rpb);
  return {y, smean, sinv};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> bn_backward(const at::Tensor& dy_, const at::Tensor& x_,
                                                           const c10::optional<at::Tensor>& nv,
                                                           const at::Tensor& smean, const at::Tensor& sinv,
                                                           const c10::optional<at::Tensor>& w) {
  auto dy = dy_.contiguous();
  auto x = x_.contiguous();
  const int N = (int)x.size(0), F = (int)x.size(1);
  auto dx = at::empty_like(x);
  const bool hw = w.has_value() && w->defined();
  auto dw = hw ? at::empty({F}, x.options()) : at::empty({0}, x.options());
  auto db = hw ? at::empty({F}, x.options()) : at::empty({0}, x.options());
  if (N == 0) {
    if (hw) { dw.zero_(); db.zero_(); }
    return {dx, dw, db};
  }
  const int S = ceil_div(N, kBnRows);
  auto part = at::empty({S, 2, F}, x.options());
  const int* nvp = (nv.has_value() && nv->defined()) ? nv->data_ptr<int>() : nullptr;
  bn_bwd_partial_kernel<<<S, 256, 0, stream()>>>(dy.data_ptr<float>(), x.data_ptr<float>(), smean.data_ptr<float>(),
                                                 sinv.data_ptr<float>(), part.data_ptr<float>(), N, F, bn_tpr(F));
  const int rpb = std::max(1, 2048 / std::max(F, 1));
  bn_bwd_apply_kernel<<<ceil_div(N, rpb), 256, 2 * F * sizeof(float), stream()>>>(
      dy.data_ptr<float>(), x.data_ptr<float>(), nvp, smean.data_ptr<float>(), sinv.data_ptr<float>(),
      hw ? w->data_ptr<float>() : nullptr, part.data_ptr<float>(), S, dx.data_ptr<float>(),
      hw ? dw.data_ptr<float>() : nullptr, hw ? db.data_ptr<float>() : nullptr, N, F, rpb);
  return {dx, dw, db};
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def(
      "bn_forward(Tensor x, Tensor? num_valid, Tensor? weight, Tensor? bias, Tensor? running_mean, "
      "Tensor? running_var, float momentum, float eps, bool relu) -> (Tensor, Tensor, Tensor)");
  m.def(
      "bn_backward(Tensor dy, Tensor x, Tensor? num_valid, Tensor mean, Tensor invstd, Tensor? weight) "
      "-> (Tensor, Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("bn_forward", hy::bn_forward);
  m.impl("bn_backward", hy::bn_backward);
}
