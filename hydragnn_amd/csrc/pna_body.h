// Fused PNA / PNAPlus message + DegreeScalerAggregation forward, per node (see pna.hip for
// the semantics).  A header so that other kernels can run it in the same launch
// (attention8.hip: the GPS layer's attention and PNA aggregation as one launch, no stream
// fork / join between them in the captured step).
#pragma once
#include "common.h"

namespace hy {

template <int VEC>
struct PVec {
  float v[VEC];
};

template <int VEC>
__device__ __forceinline__ PVec<VEC> pld(const float* p) {
  PVec<VEC> r;
  if constexpr (VEC == 4) {
    float4 t = *reinterpret_cast<const float4*>(p);
    r.v[0] = t.x; r.v[1] = t.y; r.v[2] = t.z; r.v[3] = t.w;
  } else {
#pragma unroll
    for (int i = 0; i < VEC; ++i) r.v[i] = p[i];
  }
  return r;
}

template <int VEC>
__device__ __forceinline__ void pst(float* p, const PVec<VEC>& r) {
  if constexpr (VEC == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(r.v[0], r.v[1], r.v[2], r.v[3]);
  } else {
#pragma unroll
    for (int i = 0; i < VEC; ++i) p[i] = r.v[i];
  }
}

constexpr float kStdEps = 1e-5f;

// PyG's StdAggregation evaluates var = E[m^2] - E[m]^2 with rounded products (separate
// torch kernels); these helpers keep the compiler from contracting them into FMAs
// (the build uses -ffp-contract=fast), see the note in pna_fwd_kernel.
__device__ __forceinline__ float add_sq_nofma(float acc, float m) {
#pragma clang fp contract(off)
  const float sq = m * m;
  return acc + sq;
}
__device__ __forceinline__ float var_nofma(float s, float s2, float d, float& mean) {
#pragma clang fp contract(off)
  mean = s / d;
  const float m2 = s2 / d;
  const float mm = mean * mean;
  return m2 - mm;
}

// Forward of node n by its tpr threads (c = this thread's index among them).
// AB: [N, ldab] with A at column offset 0 and B at column offset F.
template <int VEC>
__device__ __forceinline__ void pna_fwd_node(
    const float* __restrict__ x, const float* __restrict__ AB, int ldab, const float* __restrict__ C,
    const float* __restrict__ G, const int* __restrict__ src, const int* __restrict__ rowptr,
    float* __restrict__ Z, int* __restrict__ amin, int* __restrict__ amax, int n, int c, int N, int F, float avg_log,
    float avg_lin, int tpr) {
  if (n >= N) return;
  const int beg = rowptr[n], end = rowptr[n + 1];
  const int cnt = end - beg;
  const float d = (float)max(cnt, 1);
  const float lg = logf(d + 1.f);
  const float sc[4] = {1.f, lg / avg_log, avg_log / lg, d / avg_lin};
  const int ldz = 17 * F;
  const int nv = F / VEC;
  for (int v = c; v < nv; v += tpr) {
    const int f0 = v * VEC;
    const PVec<VEC> a = pld<VEC>(AB + (int64_t)n * ldab + f0);
    PVec<VEC> s, s2, mn, mx;
    int imn[VEC], imx[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      s.v[i] = 0.f; s2.v[i] = 0.f; mn.v[i] = INFINITY; mx.v[i] = -INFINITY; imn[i] = -1; imx[i] = -1;
    }
    // edges in batches of EB: every source index, then every gathered row of the batch, is in
    // flight together (one edge at a time paid two dependent memory latencies per edge:
    // src[e], then AB[src[e]]); the statistics still fold edge by edge in CSR order
    constexpr int EB = VEC == 1 ? 8 : 4;
    for (int e0 = beg; e0 < end; e0 += EB) {
      int js[EB];
#pragma unroll
      for (int k = 0; k < EB; ++k) js[k] = src[min(e0 + k, end - 1)];
      PVec<VEC> b[EB], cc[EB], g[EB];
#pragma unroll
      for (int k = 0; k < EB; ++k) {
        const int e = min(e0 + k, end - 1);
        b[k] = pld<VEC>(AB + (int64_t)js[k] * ldab + F + f0);
        if (C) cc[k] = pld<VEC>(C + (int64_t)e * F + f0); else { for (int i = 0; i < VEC; ++i) cc[k].v[i] = 0.f; }
        if (G) g[k] = pld<VEC>(G + (int64_t)e * F + f0); else { for (int i = 0; i < VEC; ++i) g[k].v[i] = 1.f; }
      }
#pragma unroll
      for (int k = 0; k < EB; ++k) {
        const int e = e0 + k;
        if (e >= end) break;
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const float m = (a.v[i] + b[k].v[i] + cc[k].v[i]) * g[k].v[i];
          s.v[i] += m;
          s2.v[i] = add_sq_nofma(s2.v[i], m);  // no FMA: see the variance note below
          if (m < mn.v[i]) { mn.v[i] = m; imn[i] = e; }
          if (m > mx.v[i]) { mx.v[i] = m; imx[i] = e; }
        }
      }
    }
    // var = E[m^2] - E[m]^2 exactly as PyG's StdAggregation evaluates it (rounded products,
    // true divisions, NO fused multiply-add).  The formula cancels catastrophically when the
    // messages of a node are (nearly) equal; with FMA contraction the rounding error of m^2
    // survives the cancellation (var = fl(m^2) - m^2 != 0 for a single neighbour), crosses
    // the 1e-5 clamp for |m| >~ 20 and switches std from 0 to >= 3e-3 — a systematic
    // forward difference that the trajectory bisection (tools/trajectory_bisect.py) traced
    // as the only source of GPU-vs-CPU training drift.
    PVec<VEC> mean, sd;
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      const float var = var_nofma(s.v[i], s2.v[i], d, mean.v[i]);
      float t = sqrtf(fmaxf(var, kStdEps));
      sd.v[i] = (t <= sqrtf(kStdEps)) ? 0.f : t;
      if (cnt == 0) { mn.v[i] = 0.f; mx.v[i] = 0.f; }
    }
    float* zr = Z + (int64_t)n * ldz;
    pst<VEC>(zr + f0, pld<VEC>(x + (int64_t)n * F + f0));
#pragma unroll
    for (int sidx = 0; sidx < 4; ++sidx) {
      float* zb = zr + F + sidx * 4 * F + f0;
      PVec<VEC> t0, t1, t2, t3;
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        t0.v[i] = mean.v[i] * sc[sidx];
        t1.v[i] = mn.v[i] * sc[sidx];
        t2.v[i] = mx.v[i] * sc[sidx];
        t3.v[i] = sd.v[i] * sc[sidx];
      }
      pst<VEC>(zb, t0);
      pst<VEC>(zb + F, t1);
      pst<VEC>(zb + 2 * F, t2);
      pst<VEC>(zb + 3 * F, t3);
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      amin[(int64_t)n * F + f0 + i] = imn[i];
      amax[(int64_t)n * F + f0 + i] = imx[i];
    }
  }
}


}  // namespace hy
