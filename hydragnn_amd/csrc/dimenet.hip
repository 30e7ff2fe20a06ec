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


// ------------------------------------------------------------------ low-rank triplet filter
// DimeNet++ interaction (reference DIMEStack.py -> PyG InteractionPPBlock):
//     sbf = lin_sbf2(lin_sbf1(sbf_raw))     [T, I] = s8 [T, B] x W2^T  (B = basis_emb, 8)
//     out[e] = sum_{t in ji-row e} x_kj[kj(t)] * sbf[t]
// The [T, I] filter (T ~ 3e5 triplets: 87 MB written then read back, twice each way) is never
// formed: each output column c recomputes w[t, c] = s8[t] . W2[c] (B FMAs) from the 32-byte
// s8 row.  Backward: dx = the same kernel over the kj CSR with g gathered by ji; and
// u[t, c] = x[kj(t), c] g[ji(t), c] feeds ds8[t] = u[t] W2 (wave reductions) and
// dW2 = sum_t u[t]^T s8[t] (per-workgroup partials, one reduce launch).
constexpr int kLrB = 8;  // basis width

// out[r, :] = sum over CSR row r (positions through perm) of x[gidx[t], :] * (s8[t] W2^T)
__global__ void __launch_bounds__(256) lr_gms_kernel(const float* __restrict__ x, const float* __restrict__ s8,
                                                     const float* __restrict__ W2, const int* __restrict__ gidx,
                                                     const int* __restrict__ rowptr, const int* __restrict__ perm,
                                                     const int* __restrict__ row_limit, int N, int F, int tpr,
                                                     int rpb, float* __restrict__ out) {
  const int r = blockIdx.x * rpb + threadIdx.x / tpr;
  const int v = threadIdx.x % tpr;  // float4 column group
  if (r >= N || 4 * v >= F) return;
  const int end = row_limit ? min(rowptr[r + 1], *row_limit) : rowptr[r + 1];
  const int beg = min(rowptr[r], end);
  float wc[4][kLrB];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < kLrB; ++j) wc[q][j] = W2[(4 * v + q) * kLrB + j];
  // U rows per batch: every index load, then every row load, in flight together (one row
  // at a time paid the perm -> gidx -> row chain of dependent latencies per triplet)
  constexpr int U = 8;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int e = beg; e < end; e += U) {
    int tt[U], gi[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ee = min(e + u, end - 1);
      tt[u] = perm ? perm[ee] : ee;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) gi[u] = gidx[tt[u]];
    float4 xv[U], s0[U], s1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xv[u] = reinterpret_cast<const float4*>(x + (int64_t)gi[u] * F)[v];
      s0[u] = reinterpret_cast<const float4*>(s8 + (int64_t)tt[u] * kLrB)[0];
      s1[u] = reinterpret_cast<const float4*>(s8 + (int64_t)tt[u] * kLrB)[1];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (e + u >= end) break;
      const float sv[kLrB] = {s0[u].x, s0[u].y, s0[u].z, s0[u].w, s1[u].x, s1[u].y, s1[u].z, s1[u].w};
      float wq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float p = 0.f;
#pragma unroll
        for (int j = 0; j < kLrB; ++j) p = fmaf(sv[j], wc[q][j], p);
        wq[q] = p;
      }
      a.x = fmaf(xv[u].x, wq[0], a.x);
      a.y = fmaf(xv[u].y, wq[1], a.y);
      a.z = fmaf(xv[u].z, wq[2], a.z);
      a.w = fmaf(xv[u].w, wq[3], a.w);
    }
  }
  reinterpret_cast<float4*>(out + (int64_t)r * F)[v] = a;
}

// u[t, c] = x[ia[t], c] * g[ib[t], c] (t < Tlim): ds8[t, j] = sum_c u W2[c, j] and per-block
// partials dW2p[blk][c][j] = sum_{t of blk} u[t, c] s8[t, j].  One wave per triplet stripe,
// lane = column (F <= 64) for the loads and the dW2 sums; ds8 goes through LDS: a batch of 8
// triplets' u rows is staged, then lane (triplet u, basis j) forms its dot product over the
// columns (per-triplet wave reductions were 8 chains of 6 dependent lane permutes).
constexpr int kLrWaves = 4, kLrPerWave = 64;
__global__ void __launch_bounds__(64 * kLrWaves) lr_wgrad_kernel(const float* __restrict__ x,
                                                                 const int* __restrict__ ia,
                                                                 const float* __restrict__ g,
                                                                 const int* __restrict__ ib,
                                                                 const float* __restrict__ s8,
                                                                 const float* __restrict__ W2, int T, int F,
                                                                 const int* __restrict__ t_limit,
                                                                 float* __restrict__ ds8,
                                                                 float* __restrict__ dW2p) {
  __shared__ float red[kLrWaves][64][kLrB];
  __shared__ float w2s[64][kLrB + 1];
  __shared__ float su[kLrWaves][8][65];
  const int w = threadIdx.x >> 6, c = threadIdx.x & 63;
  const int Te = t_limit ? min(T, *t_limit) : T;
  const bool live = c < F;
  for (int k = threadIdx.x; k < 64 * kLrB; k += 64 * kLrWaves) {
    const int cc = k / kLrB, j = k % kLrB;
    w2s[cc][j] = cc < F ? W2[cc * kLrB + j] : 0.f;
  }
  __syncthreads();
  float acc[kLrB];
#pragma unroll
  for (int j = 0; j < kLrB; ++j) acc[j] = 0.f;
  const int t0 = (blockIdx.x * kLrWaves + w) * kLrPerWave;
  const int t1 = min(t0 + kLrPerWave, T);
  constexpr int U = 8;  // triplets per batch: all their loads in flight together
  const int myu = c >> 3, myj = c & 7;  // ds8 lane role: (triplet of the batch, basis index)
  for (int tb = t0; tb < t1; tb += U) {
    int ja[U], jb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = min(tb + u, t1 - 1);
      ja[u] = ia[t];
      jb[u] = ib[t];
    }
    float xu[U], gu[U];
    float4 s0[U], s1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = min(tb + u, t1 - 1);
      xu[u] = live ? x[(int64_t)ja[u] * F + c] : 0.f;
      gu[u] = live ? g[(int64_t)jb[u] * F + c] : 0.f;
      s0[u] = reinterpret_cast<const float4*>(s8 + (int64_t)t * kLrB)[0];
      s1[u] = reinterpret_cast<const float4*>(s8 + (int64_t)t * kLrB)[1];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = tb + u;
      // padding triplets (t >= Te) and the stripe's tail: no share of either gradient
      const float uu = (t < t1 && t < Te) ? xu[u] * gu[u] : 0.f;
      su[w][u][c] = uu;
      const float sv[kLrB] = {s0[u].x, s0[u].y, s0[u].z, s0[u].w, s1[u].x, s1[u].y, s1[u].z, s1[u].w};
#pragma unroll
      for (int j = 0; j < kLrB; ++j) acc[j] = fmaf(uu, sv[j], acc[j]);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float d = 0.f;
#pragma unroll 8
    for (int cc = 0; cc < 64; ++cc) d = fmaf(su[w][myu][cc], w2s[cc][myj], d);
    const int t = tb + myu;
    if (t < t1) ds8[(int64_t)t * kLrB + myj] = d;
    __builtin_amdgcn_wave_barrier();  // su is rewritten by the next batch
  }
#pragma unroll
  for (int j = 0; j < kLrB; ++j) red[w][c][j] = acc[j];
  __syncthreads();
  for (int k = threadIdx.x; k < 64 * kLrB; k += 64 * kLrWaves) {
    const int cc = k / kLrB;
    if (cc >= F) continue;
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < kLrWaves; ++q) v += red[q][cc][k % kLrB];
    dW2p[(int64_t)blockIdx.x * F * kLrB + k] = v;
  }
}

// out[k] = sum_b p[b][k]: 32 threads per element over the partials, then an LDS fold
__global__ void __launch_bounds__(256) lr_wreduce_kernel(const float* __restrict__ p, int nb, int n,
                                                         float* __restrict__ out) {
  __shared__ float part[8][33];
  const int e = threadIdx.x >> 5, l = threadIdx.x & 31;
  const int k = blockIdx.x * 8 + e;
  float a = 0.f;
  if (k < n)
    for (int b = l; b < nb; b += 32) a += p[(int64_t)b * n + k];
  part[e][l] = a;
  __syncthreads();
  if (l == 0 && k < n) {
    float v = 0.f;
    for (int q = 0; q < 32; ++q) v += part[e][q];
    out[k] = v;
  }
}

at::Tensor lr_gather_mul_sum(const at::Tensor& x_, const at::Tensor& s8_, const at::Tensor& W2_,
                             const at::Tensor& gidx, const at::Tensor& rowptr, const c10::optional<at::Tensor>& perm,
                             int64_t N, const c10::optional<at::Tensor>& limit) {
  auto x = x_.contiguous(), s8 = s8_.contiguous(), W2 = W2_.contiguous();
  HY_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && s8.scalar_type() == at::kFloat &&
               W2.scalar_type() == at::kFloat && gidx.scalar_type() == at::kInt && rowptr.scalar_type() == at::kInt,
           "lr_gather_mul_sum: fp32 operands, int32 indices");
  const int F = (int)x.size(1);
  HY_CHECK(x.dim() == 2 && F % 4 == 0 && s8.dim() == 2 && s8.size(1) == kLrB && W2.size(0) == F &&
               W2.size(1) == kLrB && gidx.numel() == s8.size(0) && rowptr.numel() == N + 1,
           "lr_gather_mul_sum: x [*, F % 4 == 0], s8 [T, 8], W2 [F, 8], gidx [T], rowptr [N + 1]");
  auto out = at::empty({N, F}, x.options());
  if (N == 0) return out;
  const int* pp = (perm.has_value() && perm->defined()) ? perm->data_ptr<int>() : nullptr;
  const int* lim = (limit.has_value() && limit->defined()) ? limit->data_ptr<int>() : nullptr;
  int tpr = 1;
  while (tpr < F / 4 && tpr < 64) tpr <<= 1;
  HY_CHECK(tpr * 4 >= F, "lr_gather_mul_sum: F <= 256");
  const int rpb = 256 / tpr;
  lr_gms_kernel<<<ceil_div(N, rpb), 256, 0, stream()>>>(x.data_ptr<float>(), s8.data_ptr<float>(),
                                                       W2.data_ptr<float>(), gidx.data_ptr<int>(),
                                                       rowptr.data_ptr<int>(), pp, lim, (int)N, F, tpr, rpb,
                                                       out.data_ptr<float>());
  return out;
}

// -> (ds8 [T, 8], dW2 [F, 8])
std::vector<at::Tensor> lr_filter_grad(const at::Tensor& x_, const at::Tensor& ia, const at::Tensor& g_,
                                       const at::Tensor& ib, const at::Tensor& s8_, const at::Tensor& W2_,
                                       const c10::optional<at::Tensor>& t_limit) {
  auto x = x_.contiguous(), g = g_.contiguous(), s8 = s8_.contiguous(), W2 = W2_.contiguous();
  const int64_t T = s8.size(0);
  const int F = (int)x.size(1);
  HY_CHECK(F <= 64 && g.size(1) == F && ia.numel() == T && ib.numel() == T && W2.size(0) == F &&
               W2.size(1) == kLrB && s8.size(1) == kLrB,
           "lr_filter_grad: F <= 64, ia / ib [T], s8 [T, 8], W2 [F, 8]");
  auto ds8 = at::empty({T, kLrB}, x.options()), dW2 = at::empty({F, kLrB}, x.options());
  const int per = kLrWaves * kLrPerWave;
  const int nb = (int)std::max<int64_t>(1, ceil_div(T, per));
  auto part = at::empty({nb, F * kLrB}, x.options());
  if (T > 0)
    lr_wgrad_kernel<<<nb, 64 * kLrWaves, 0, stream()>>>(
        x.data_ptr<float>(), ia.data_ptr<int>(), g.data_ptr<float>(), ib.data_ptr<int>(), s8.data_ptr<float>(),
        W2.data_ptr<float>(), (int)T, F, (t_limit.has_value() && t_limit->defined()) ? t_limit->data_ptr<int>() : nullptr,
        ds8.data_ptr<float>(), part.data_ptr<float>());
  else
    part.zero_();
  lr_wreduce_kernel<<<ceil_div(F * kLrB, 8), 256, 0, stream()>>>(part.data_ptr<float>(), nb, F * kLrB,
                                                                dW2.data_ptr<float>());
  return {ds8, dW2};
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("lr_gather_mul_sum(Tensor x, Tensor s8, Tensor W2, Tensor gidx, Tensor rowptr, Tensor? perm, int N, "
        "Tensor? limit=None) -> Tensor");
  m.def("lr_filter_grad(Tensor x, Tensor ia, Tensor g, Tensor ib, Tensor s8, Tensor W2, Tensor? t_limit=None) "
        "-> Tensor[]");
  m.def("dimenet_sbf_fwd(Tensor vec, Tensor kj, Tensor ji, Tensor z, Tensor nrm, float cutoff, int exponent, Tensor? limit=None) -> Tensor");
  m.def(
      "dimenet_sbf_bwd(Tensor gout, Tensor vec, Tensor kj, Tensor ji, Tensor z, Tensor nrm, float cutoff, int exponent, "
      "Tensor? limit=None) -> Tensor");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("lr_gather_mul_sum", hy::lr_gather_mul_sum);
  m.impl("lr_filter_grad", hy::lr_filter_grad);
  m.impl("dimenet_sbf_fwd", hy::dimenet_sbf_fwd);
  m.impl("dimenet_sbf_bwd", hy::dimenet_sbf_bwd);
}
