// DimeNet++ triplet angle + spherical basis in one pass (reference
// hydragnn/models/DIMEStack.py:170-190 -> PyG SphericalBasisLayer):
//
//   v1 = vec[e_ji], v2 = vec[e_kj] + vec[e_ji]          (vec = pos[dst] - pos[src])
//   t  = cos(angle(v1, v2)) = v1.v2 / (|v1| |v2|)         (PyG: atan2(|v1 x v2|, v1.v2))
//   d  = |vec[e_kj]| / cutoff
//   sbf[t, l*K + j] = u(d) * norm[l][j] * j_l(z[l][j] d) * sqrt((2l+1)/4pi) P_l(t)
//
// with u the DimeNet polynomial envelope, j_l spherical Bessel functions (upward
// recurrence in fp64, as the torch path) and P_l Legendre polynomials.  One thread per
// triplet computes all n*K outputs: the [T, n*K] tensor is written once, the per-edge
// radial part is never materialised and gathered.
//
// Backward (analytic): d/dd through u and j_l' (j_l' = j_{l-1} - (l+1)/x j_l,
// j_0' = -j_1), d/dt through P_l' (P'_{l+1} = P'_{l-1} + (2l+1) P_l), then the chain to
// vec[e_kj] and vec[e_ji]; the per-triplet vector gradients are added to dvec with fp32
// atomics (a triplet touches two edges; no CSR by e_kj exists).
#include "common.h"

namespace hy {
namespace dn {

constexpr int MAXL = 8, MAXK = 8;

struct SbfArgs {
  const float* vec;  // [E, 3]
  const int* kj;     // [T]
  const int* ji;     // [T]
  const double* z;   // [n, K] Bessel zeros
  const double* nrm; // [n, K]
  int T, n, K;
  float inv_cut, pa, pb, pc;
  int p;             // envelope exponent + 1
  const int* limit;  // optional device scalar: triplets at or past it are padding (zero basis)
};

__device__ __forceinline__ void envelope(double x, int p, double a, double b, double c, double& u, double& du) {
  if (x >= 1.0 || x <= 0.0) {
    u = 0.0;
    du = 0.0;
    return;
  }
  const double xp0 = pow(x, (double)(p - 1));
  u = 1.0 / x + a * xp0 + b * xp0 * x + c * xp0 * x * x;
  du = -1.0 / (x * x) + a * (p - 1) * xp0 / x + b * p * xp0 + c * (p + 1) * xp0 * x;
}

// j_0 .. j_{L}(x) by upward recurrence
__device__ __forceinline__ void sph_jn(int L, double x, double* j) {
  const double s = sin(x), c = cos(x);
  j[0] = s / x;
  if (L >= 1) j[1] = s / (x * x) - c / x;
  for (int l = 1; l < L; ++l) j[l + 1] = (2 * l + 1) / x * j[l] - j[l - 1];
}

__device__ __forceinline__ void geom(const SbfArgs& a, int t, float3& v1, float3& v2, double& d, double& ct, double& n1,
                                     double& n2) {
  const int e1 = a.ji[t], e2 = a.kj[t];
  v1 = make_float3(a.vec[e1 * 3], a.vec[e1 * 3 + 1], a.vec[e1 * 3 + 2]);
  const float3 w = make_float3(a.vec[e2 * 3], a.vec[e2 * 3 + 1], a.vec[e2 * 3 + 2]);
  v2 = make_float3(w.x + v1.x, w.y + v1.y, w.z + v1.z);
  d = sqrt((double)w.x * w.x + (double)w.y * w.y + (double)w.z * w.z) * a.inv_cut;
  n1 = sqrt((double)v1.x * v1.x + (double)v1.y * v1.y + (double)v1.z * v1.z);
  n2 = sqrt((double)v2.x * v2.x + (double)v2.y * v2.y + (double)v2.z * v2.z);
  const double dot = (double)v1.x * v2.x + (double)v1.y * v2.y + (double)v1.z * v2.z;
  ct = (n1 > 0.0 && n2 > 0.0) ? dot / (n1 * n2) : 1.0;
  ct = fmin(1.0, fmax(-1.0, ct));
}

__global__ void sbf_fwd_kernel(SbfArgs a, float* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.T) return;
  float* o = out + (int64_t)t * a.n * a.K;
  if (a.limit && t >= *a.limit) {
    for (int q = 0; q < a.n * a.K; ++q) o[q] = 0.f;
    return;
  }
  float3 v1, v2;
  double d, ct, n1, n2;
  geom(a, t, v1, v2, d, ct, n1, n2);
  double u, du;
  envelope(d, a.p, a.pa, a.pb, a.pc, u, du);
  double P[MAXL];
  P[0] = 1.0;
  if (a.n > 1) P[1] = ct;
  for (int l = 1; l + 1 < a.n; ++l) P[l + 1] = ((2 * l + 1) * ct * P[l] - l * P[l - 1]) / (l + 1);
  double j[MAXL + 1];
  for (int l = 0; l < a.n; ++l) {
    const double cb = sqrt((2 * l + 1) / (4.0 * M_PI)) * P[l];
    for (int k = 0; k < a.K; ++k) {
      const double x = a.z[l * a.K + k] * d;
      double r = 0.0;
      if (u != 0.0) {
        sph_jn(l, x, j);
        r = a.nrm[l * a.K + k] * j[l] * u;
      }
      o[l * a.K + k] = (float)(r * cb);
    }
  }
}

__global__ void sbf_bwd_kernel(SbfArgs a, const float* __restrict__ gout, float* __restrict__ dvec) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.T || (a.limit && t >= *a.limit)) return;
  float3 v1, v2;
  double d, ct, n1, n2;
  geom(a, t, v1, v2, d, ct, n1, n2);
  double u, du;
  envelope(d, a.p, a.pa, a.pb, a.pc, u, du);
  if (u == 0.0 && du == 0.0) return;
  double P[MAXL], dP[MAXL];
  P[0] = 1.0;
  dP[0] = 0.0;
  if (a.n > 1) {
    P[1] = ct;
    dP[1] = 1.0;
  }
  for (int l = 1; l + 1 < a.n; ++l) {
    P[l + 1] = ((2 * l + 1) * ct * P[l] - l * P[l - 1]) / (l + 1);
    dP[l + 1] = dP[l - 1] + (2 * l + 1) * P[l];
  }
  const float* g = gout + (int64_t)t * a.n * a.K;
  double gd = 0.0, gt = 0.0;  // d loss / d d (scaled distance), d loss / d t
  double j[MAXL + 2];
  for (int l = 0; l < a.n; ++l) {
    const double c0 = sqrt((2 * l + 1) / (4.0 * M_PI));
    for (int k = 0; k < a.K; ++k) {
      const double go = g[l * a.K + k];
      const double z = a.z[l * a.K + k], x = z * d;
      sph_jn(l + 1, x, j);
      const double jl = j[l];
      const double djl = l == 0 ? -j[1] : j[l - 1] - (l + 1) / x * jl;
      const double nr = a.nrm[l * a.K + k];
      const double r = nr * jl * u;
      const double dr = nr * (du * jl + u * z * djl);
      gd += go * c0 * P[l] * dr;
      gt += go * c0 * dP[l] * r;
    }
  }
  // chain: d = |w| / cutoff (w = vec[kj]); t = v1.v2 / (|v1||v2|), v2 = w + v1
  const int e1 = a.ji[t], e2 = a.kj[t];
  const double wx = (double)v2.x - v1.x, wy = (double)v2.y - v1.y, wz = (double)v2.z - v1.z;
  const double wn = d / a.inv_cut;
  double g1[3] = {0, 0, 0}, g2[3] = {0, 0, 0};  // d/dv1, d/dv2
  if (n1 > 0.0 && n2 > 0.0) {
    const double i12 = 1.0 / (n1 * n2);
    const double a1 = ct / (n1 * n1), a2 = ct / (n2 * n2);
    g1[0] = gt * (v2.x * i12 - a1 * v1.x);
    g1[1] = gt * (v2.y * i12 - a1 * v1.y);
    g1[2] = gt * (v2.z * i12 - a1 * v1.z);
    g2[0] = gt * (v1.x * i12 - a2 * v2.x);
    g2[1] = gt * (v1.y * i12 - a2 * v2.y);
    g2[2] = gt * (v1.z * i12 - a2 * v2.z);
  }
  double gw[3] = {g2[0], g2[1], g2[2]};
  if (wn > 0.0) {
    const double s = gd * a.inv_cut / wn;
    gw[0] += s * wx;
    gw[1] += s * wy;
    gw[2] += s * wz;
  }
  // v2 = w + v1: vec[ji] receives g1 + g2, vec[kj] receives g2 (+ the distance term)
  for (int c = 0; c < 3; ++c) {
    atomicAdd(dvec + e1 * 3 + c, (float)(g1[c] + g2[c]));
    atomicAdd(dvec + e2 * 3 + c, (float)gw[c]);
  }
}

}  // namespace dn

using namespace dn;

static SbfArgs sbf_args(const at::Tensor& vec, const at::Tensor& kj, const at::Tensor& ji, const at::Tensor& z,
                        const at::Tensor& nrm, double cutoff, int64_t exponent,
                        const c10::optional<at::Tensor>& limit) {
  HY_CHECK(vec.is_cuda() && vec.scalar_type() == at::kFloat && vec.is_contiguous() && vec.dim() == 2 &&
               vec.size(1) == 3,
           "sbf: vec [E, 3] fp32");
  HY_CHECK_I32(kj);
  HY_CHECK_I32(ji);
  HY_CHECK(kj.numel() == ji.numel(), "sbf: triplet index lengths");
  HY_CHECK(z.scalar_type() == at::kDouble && z.is_contiguous() && nrm.sizes() == z.sizes() && nrm.is_contiguous() &&
               z.dim() == 2 && z.size(0) <= MAXL && z.size(1) <= MAXK,
           "sbf: zeros / norm [n <= 8, K <= 8] fp64");
  SbfArgs a{};
  a.vec = vec.data_ptr<float>();
  a.kj = kj.data_ptr<int>();
  a.ji = ji.data_ptr<int>();
  a.z = z.data_ptr<double>();
  a.nrm = nrm.data_ptr<double>();
  a.T = (int)kj.numel();
  a.n = (int)z.size(0);
  a.K = (int)z.size(1);
  a.inv_cut = (float)(1.0 / cutoff);
  a.p = (int)exponent + 1;
  a.pa = (float)(-(a.p + 1) * (a.p + 2) / 2.0);
  a.pb = (float)(a.p * (a.p + 2));
  a.pc = (float)(-a.p * (a.p + 1) / 2.0);
  a.limit = nullptr;
  if (limit.has_value() && limit->defined()) {
    HY_CHECK(limit->is_cuda() && limit->scalar_type() == at::kInt && limit->numel() == 1,
             "sbf: limit must be a device int32 scalar");
    a.limit = limit->data_ptr<int>();
  }
  return a;
}

at::Tensor dimenet_sbf_fwd(const at::Tensor& vec, const at::Tensor& kj, const at::Tensor& ji, const at::Tensor& z,
                           const at::Tensor& nrm, double cutoff, int64_t exponent,
                           const c10::optional<at::Tensor>& limit) {
  SbfArgs a = sbf_args(vec, kj, ji, z, nrm, cutoff, exponent, limit);
  auto out = at::empty({(int64_t)a.T, (int64_t)a.n * a.K}, vec.options());
  if (a.T) sbf_fwd_kernel<<<ceil_div(a.T, 128), 128, 0, stream()>>>(a, out.data_ptr<float>());
  return out;
}

at::Tensor dimenet_sbf_bwd(const at::Tensor& gout, const at::Tensor& vec, const at::Tensor& kj, const at::Tensor& ji,
                           const at::Tensor& z, const at::Tensor& nrm, double cutoff, int64_t exponent,
                           const c10::optional<at::Tensor>& limit) {
  SbfArgs a = sbf_args(vec, kj, ji, z, nrm, cutoff, exponent, limit);
  HY_CHECK(gout.scalar_type() == at::kFloat && gout.is_contiguous() && gout.numel() == (int64_t)a.T * a.n * a.K,
           "sbf_bwd: gout [T, n*K]");
  auto dvec = at::zeros_like(vec);
  if (a.T) sbf_bwd_kernel<<<ceil_div(a.T, 128), 128, 0, stream()>>>(a, gout.data_ptr<float>(), dvec.data_ptr<float>());
  return dvec;
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("dimenet_sbf_fwd(Tensor vec, Tensor kj, Tensor ji, Tensor z, Tensor nrm, float cutoff, int exponent, Tensor? limit=None) -> Tensor");
  m.def(
      "dimenet_sbf_bwd(Tensor gout, Tensor vec, Tensor kj, Tensor ji, Tensor z, Tensor nrm, float cutoff, int exponent, "
      "Tensor? limit=None) -> Tensor");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("dimenet_sbf_fwd", hy::dimenet_sbf_fwd);
  m.impl("dimenet_sbf_bwd", hy::dimenet_sbf_bwd);
}
