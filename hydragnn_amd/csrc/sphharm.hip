// Real spherical harmonics of edge vectors, l <= 4 (gfx950).  SURVEY K9; reference:
// e3nn o3.SphericalHarmonics(normalize=True, normalization="component") in MACE
// (mace_utils/modules/blocks.py, models/MACEStack.py edge attributes).
//
// The torch composite (ops/o3.py spherical_harmonics) lowers to ~60 elementwise launches
// over the edges for lmax = 3 — in a captured MACE step those are ~60 graph nodes of a
// few microseconds each.  Here one thread owns one edge and evaluates the same
// recurrences in registers:
//   u = v / (|v| + eps)
//   A_m + i B_m = (u_x + i u_y)^m
//   Q_l^m: reduced associated Legendre functions (no Condon-Shortley phase)
//   Y_l^m = c_lm Q_l^|m| {1 | sqrt2 A_m | sqrt2 B_|m|}
// Backward: the same evaluation in forward-mode dual numbers (value + 3 tangents), so
// dY/dv is exact and one pass gives dL/dv = sum_k g_k dY_k/dv (no stored Jacobian).
#include "common.h"

namespace hy {

constexpr int kShMaxL = 4;

struct ShCoef {
  float c[(kShMaxL + 1) * (kShMaxL + 1)];
};

template <typename T>
struct ShOps;

template <>
struct ShOps<float> {
  static __device__ __forceinline__ float cst(float v) { return v; }
};

struct Dual3 {
  float v, dx, dy, dz;
};
__device__ __forceinline__ Dual3 operator+(Dual3 a, Dual3 b) { return {a.v + b.v, a.dx + b.dx, a.dy + b.dy, a.dz + b.dz}; }
__device__ __forceinline__ Dual3 operator-(Dual3 a, Dual3 b) { return {a.v - b.v, a.dx - b.dx, a.dy - b.dy, a.dz - b.dz}; }
__device__ __forceinline__ Dual3 operator*(Dual3 a, Dual3 b) {
  return {a.v * b.v, a.dx * b.v + a.v * b.dx, a.dy * b.v + a.v * b.dy, a.dz * b.v + a.v * b.dz};
}
__device__ __forceinline__ Dual3 operator*(float s, Dual3 a) { return {s * a.v, s * a.dx, s * a.dy, s * a.dz}; }
template <>
struct ShOps<Dual3> {
  static __device__ __forceinline__ Dual3 cst(float v) { return {v, 0.f, 0.f, 0.f}; }
};
__device__ __forceinline__ float scale_by(float s, float a) { return s * a; }
__device__ __forceinline__ Dual3 scale_by(float s, Dual3 a) { return s * a; }

// Y[(l+1)^2] from the unit vector (x, y, z); T = float or Dual3
template <int LMAX, typename T>
__device__ __forceinline__ void sh_eval(T x, T y, T z, const float* __restrict__ coef, T* __restrict__ Y) {
  T A[LMAX + 1], B[LMAX + 1];
  A[0] = ShOps<T>::cst(1.f);
  B[0] = ShOps<T>::cst(0.f);
#pragma unroll
  for (int m = 0; m < LMAX; ++m) {
    A[m + 1] = x * A[m] - y * B[m];
    B[m + 1] = x * B[m] + y * A[m];
  }
  T Q[LMAX + 1][LMAX + 1];
#pragma unroll
  for (int m = 0; m <= LMAX; ++m) {
    float dfact = 1.f;  // (2m-1)!!
#pragma unroll
    for (int k = 2 * m - 1; k > 0; k -= 2) dfact *= (float)k;
    Q[m][m] = ShOps<T>::cst(dfact);
    if (m + 1 <= LMAX) Q[m + 1][m] = scale_by((float)(2 * m + 1), z * Q[m][m]);
#pragma unroll
    for (int l = m + 2; l <= LMAX; ++l)
      Q[l][m] = scale_by(1.f / (float)(l - m),
                         scale_by((float)(2 * l - 1), z * Q[l - 1][m]) - scale_by((float)(l + m - 1), Q[l - 2][m]));
  }
  int k = 0;
#pragma unroll
  for (int l = 0; l <= LMAX; ++l) {
#pragma unroll
    for (int m = -l; m <= l; ++m, ++k) {
      const int am = m < 0 ? -m : m;
      if (m == 0)
        Y[k] = scale_by(coef[k], Q[l][0]);
      else if (m > 0)
        Y[k] = scale_by(coef[k], Q[l][am] * A[am]);
      else
        Y[k] = scale_by(coef[k], Q[l][am] * B[am]);
    }
  }
}

template <int LMAX>
__global__ void __launch_bounds__(256) sh_fwd_kernel(const float* __restrict__ vec, float* __restrict__ out,
                                                     int64_t E, float eps, int normalize, ShCoef coef) {
  constexpr int D = (LMAX + 1) * (LMAX + 1);
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= E) return;
  float x = vec[3 * e], y = vec[3 * e + 1], z = vec[3 * e + 2];
  if (normalize) {
    const float inv = 1.f / (sqrtf(x * x + y * y + z * z) + eps);
    x *= inv;
    y *= inv;
    z *= inv;
  }
  float Y[D];
  sh_eval<LMAX, float>(x, y, z, coef.c, Y);
#pragma unroll
  for (int k = 0; k < D; ++k) out[e * D + k] = Y[k];
}

template <int LMAX>
__global__ void __launch_bounds__(256) sh_bwd_kernel(const float* __restrict__ vec, const float* __restrict__ g,
                                                     float* __restrict__ dvec, int64_t E, float eps, int normalize,
                                                     ShCoef coef) {
  constexpr int D = (LMAX + 1) * (LMAX + 1);
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= E) return;
  Dual3 x = {vec[3 * e], 1.f, 0.f, 0.f};
  Dual3 y = {vec[3 * e + 1], 0.f, 1.f, 0.f};
  Dual3 z = {vec[3 * e + 2], 0.f, 0.f, 1.f};
  if (normalize) {
    const float r = sqrtf(x.v * x.v + y.v * y.v + z.v * z.v);
    const float inv = 1.f / (r + eps);
    // d inv / d v_i = -v_i / (r (r + eps)^2)   (0 at r = 0)
    const float f = r > 0.f ? -inv * inv / r : 0.f;
    const Dual3 s = {inv, f * x.v, f * y.v, f * z.v};
    x = x * s;
    y = y * s;
    z = z * s;
  }
  Dual3 Y[D];
  sh_eval<LMAX, Dual3>(x, y, z, coef.c, Y);
  float ax = 0.f, ay = 0.f, az = 0.f;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    const float gk = g[e * D + k];
    ax = fmaf(gk, Y[k].dx, ax);
    ay = fmaf(gk, Y[k].dy, ay);
    az = fmaf(gk, Y[k].dz, az);
  }
  dvec[3 * e] = ax;
  dvec[3 * e + 1] = ay;
  dvec[3 * e + 2] = az;
}

static ShCoef sh_coef(int lmax) {
  ShCoef c{};
  int k = 0;
  auto fact = [](int n) {
    double f = 1.0;
    for (int i = 2; i <= n; ++i) f *= i;
    return f;
  };
  for (int l = 0; l <= lmax; ++l)
    for (int m = -l; m <= l; ++m, ++k) {
      const int am = m < 0 ? -m : m;
      double v = std::sqrt((2.0 * l + 1.0) * fact(l - am) / fact(l + am));
      if (m != 0) v *= std::sqrt(2.0);
      c.c[k] = (float)v;
    }
  return c;
}

#define HY_SH_DISPATCH(L, ...)                                                      \
  switch (L) {                                                                      \
    case 0: { constexpr int kL = 0; __VA_ARGS__; break; }                           \
    case 1: { constexpr int kL = 1; __VA_ARGS__; break; }                           \
    case 2: { constexpr int kL = 2; __VA_ARGS__; break; }                           \
    case 3: { constexpr int kL = 3; __VA_ARGS__; break; }                           \
    case 4: { constexpr int kL = 4; __VA_ARGS__; break; }                           \
    default: HY_CHECK(false, "spherical harmonics: lmax must be in [0, 4], got ", L); \
  }

at::Tensor sh_fwd(const at::Tensor& vec_, int64_t lmax, double eps, bool normalize) {
  HY_CHECK_CUDA(vec_);
  auto vec = vec_.contiguous();
  HY_CHECK_F32(vec);
  HY_CHECK(vec.dim() == 2 && vec.size(1) == 3, "sh_fwd: vec must be [E, 3]");
  const int64_t E = vec.size(0);
  auto out = at::empty({E, (lmax + 1) * (lmax + 1)}, vec.options());
  if (E == 0) return out;
  const ShCoef c = sh_coef((int)lmax);
  HY_SH_DISPATCH((int)lmax, sh_fwd_kernel<kL><<<ceil_div(E, 256), 256, 0, stream()>>>(
                                vec.data_ptr<float>(), out.data_ptr<float>(), E, (float)eps, normalize ? 1 : 0, c));
  return out;
}

at::Tensor sh_bwd(const at::Tensor& g_, const at::Tensor& vec_, int64_t lmax, double eps, bool normalize) {
  HY_CHECK_CUDA(vec_);
  auto vec = vec_.contiguous(), g = g_.contiguous();
  HY_CHECK_F32(vec);
  HY_CHECK_F32(g);
  const int64_t E = vec.size(0);
  HY_CHECK(g.dim() == 2 && g.size(0) == E && g.size(1) == (lmax + 1) * (lmax + 1), "sh_bwd: grad shape");
  auto dvec = at::empty({E, 3}, vec.options());
  if (E == 0) return dvec;
  const ShCoef c = sh_coef((int)lmax);
  HY_SH_DISPATCH((int)lmax, sh_bwd_kernel<kL><<<ceil_div(E, 256), 256, 0, stream()>>>(
                                vec.data_ptr<float>(), g.data_ptr<float>(), dvec.data_ptr<float>(), E, (float)eps,
                                normalize ? 1 : 0, c));
  return dvec;
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("sh_fwd(Tensor vec, int lmax, float eps, bool normalize) -> Tensor");
  m.def("sh_bwd(Tensor g, Tensor vec, int lmax, float eps, bool normalize) -> Tensor");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("sh_fwd", hy::sh_fwd);
  m.impl("sh_bwd", hy::sh_bwd);
}
