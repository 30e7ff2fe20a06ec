// Fused  y = [relu](BN(dropout_p(a) + b))  over node rows [N, C], one launch forward,
// one launch backward (gfx950).
//
// Reference sites: GPS layer (hydragnn/globalAtt/gps.py:120-150: dropout -> residual
// add -> BatchNorm, x3 per layer) and Base.encode (Base.py:466: BatchNorm -> ReLU per
// conv layer).  torch issues dropout + add + BN(4) + relu + mask = 7-8 launches per
// site forward and ~6 backward.  Here: 2 launches each way, both row-slab parallel
// with coalesced rows (tpr threads x V channels per row):
//
//   fwd 1: z = dropout(a) + b (kept for backward), per-slab (count, mean, M2)
//          (two-pass within the L2-hot slab)
//   fwd 2: every block folds the S slab stats (Chan, fixed order -> deterministic),
//          y = (z - mean) * invstd * w + beta, relu, rows >= num_valid -> 0
//          (zero_pad); block 0 writes the saved stats and running-stat update
//   bwd 1: per-slab (sum g, sum g*xhat), g = dy masked by relu / padding
//   bwd 2: fold partials, dw/db, dz and the dropout'd da for the slab.
// (A one-workgroup-per-column-group single-launch variant was measured at
// 11-13 us for [2816, 64]: column-strided float4 loads touch a cache line per
// row and only C/4 CUs work.)
//
// Dropout uses a counter-based hash (lowbias32 of seed, call-site salt, element
// index) with the seed read from a device int64 counter: capture-safe in hipGraphs
// (the counter is advanced by a captured kernel each step) and recomputed in the
// backward instead of storing a mask.
#include "common.h"
#include "dropout.h"

namespace hy {



template <int V>
struct VecT;
template <>
struct VecT<4> {
  using T = float4;
};
template <>
struct VecT<1> {
  using T = float;
};

template <int V>
__device__ __forceinline__ float el(const typename VecT<V>::T& v, int k);
template <>
__device__ __forceinline__ float el<4>(const float4& v, int k) {
  return k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w));
}
template <>
__device__ __forceinline__ float el<1>(const float& v, int) {
  return v;
}
template <int V>
__device__ __forceinline__ void set_el(typename VecT<V>::T& v, int k, float x);
template <>
__device__ __forceinline__ void set_el<4>(float4& v, int k, float x) {
  if (k == 0) v.x = x;
  else if (k == 1) v.y = x;
  else if (k == 2) v.z = x;
  else v.w = x;
}
template <>
__device__ __forceinline__ void set_el<1>(float& v, int, float x) {
  v = x;
}

// ---------------------------------------------------------------------------------
// Slab geometry: a 256-thread workgroup owns kSlab consecutive rows; `tpr` threads
// cover one row (V channels each, coalesced along the row) and the block covers
// 256/tpr rows per step.  Channel groups beyond tpr*V loop.
constexpr int kBlk = 256;
#ifndef HY_BN_ROWS
#define HY_BN_ROWS 4
#endif
constexpr int kRows = HY_BN_ROWS;  // rows per thread per slab, all loads issued before use

struct Geo {
  int tpr, rpb, ngrp, slab;  // threads per row, rows per block-step, channel groups (C / V), rows per block
};

// Row index clamped into [0, r1): loads are issued unconditionally at clamped
// addresses and masked where used.  A guarded (if/else) load makes the compiler
// drain the memory counter at the branch join, serialising the kRows loads a
// thread is meant to have in flight.
__device__ __forceinline__ int rowc(int r, int r1) { return max(min(r, r1 - 1), 0); }


// Sum over the S slab partials of channel c, T threads per channel (thread j takes
// s = j, j+T, ...), folded across the T threads in a fixed order.  red: [kBlk].
__device__ __forceinline__ float chan_sum(float v, float* red, int T) {
  red[threadIdx.x] = v;
  __syncthreads();
  float t = 0.f;
  const int base = (threadIdx.x / T) * T;
  for (int q = 0; q < T; ++q) t += red[base + q];
  __syncthreads();
  return t;
}

__device__ __forceinline__ double chan_sum_d(double v, double* red, int T) {
  red[threadIdx.x] = v;
  __syncthreads();
  double t = 0.0;
  const int base = (threadIdx.x / T) * T;
  for (int q = 0; q < T; ++q) t += red[base + q];
  __syncthreads();
  return t;
}

template <int V>
__device__ __forceinline__ typename VecT<V>::T ldv(const float* p) {
  return *reinterpret_cast<const typename VecT<V>::T*>(p);
}
template <int V>
__device__ __forceinline__ void stv(float* p, const typename VecT<V>::T& v) {
  *reinterpret_cast<typename VecT<V>::T*>(p) = v;
}

// z = dropout(a) + b for one V-chunk
template <int V>
__device__ __forceinline__ typename VecT<V>::T make_z(const float* a, const float* b, const DropCfg& d, int64_t off) {
  typename VecT<V>::T v = ldv<V>(a + off);
  if (d.on) {
#pragma unroll
    for (int k = 0; k < V; ++k)
      set_el<V>(v, k, keep_elem(d.seed, (uint32_t)(off + k), d.thresh) ? el<V>(v, k) * d.scale : 0.f);
  }
  if (b) {
    const typename VecT<V>::T bb = ldv<V>(b + off);
#pragma unroll
    for (int k = 0; k < V; ++k) set_el<V>(v, k, el<V>(v, k) + el<V>(bb, k));
  }
  return v;
}

// Fold the per-thread column partials of one channel group across the rpb row lanes of
// the block (fixed order).  red: [kBlk * V].  Result valid in threads with rl == 0.
template <int V>
__device__ __forceinline__ void fold_rows(float (&v)[V], float* red, int rl, int cg_l, const Geo& g) {
#pragma unroll
  for (int k = 0; k < V; ++k) red[threadIdx.x * V + k] = v[k];
  __syncthreads();
  if (rl == 0) {
#pragma unroll
    for (int k = 0; k < V; ++k) {
      float s = 0.f;
      for (int q = 0; q < g.rpb; ++q) s += red[(q * g.tpr + cg_l) * V + k];
      v[k] = s;
    }
  }
  __syncthreads();
}

// fp64 variant of fold_rows for the squared deviations (red: [kBlk * V] doubles).
template <int V>
__device__ __forceinline__ void fold_rows_d(double (&v)[V], double* red, int rl, int cg_l, const Geo& g) {
#pragma unroll
  for (int k = 0; k < V; ++k) red[threadIdx.x * V + k] = v[k];
  __syncthreads();
  if (rl == 0) {
#pragma unroll
    for (int k = 0; k < V; ++k) {
      double s = 0.0;
      for (int q = 0; q < g.rpb; ++q) s += red[(q * g.tpr + cg_l) * V + k];
      v[k] = s;
    }
  }
  __syncthreads();
}

// forward pass 1: z (if fused) + per-slab (count, mean, std) -> part[S][3][C].
// Squared deviations accumulate in fp64 and the slab spread is stored as a standard
// deviation: activations of |x| > 1.8e19 (seen when deep multiplicative stacks drift)
// would overflow an fp32 sum of squares / variance, and the CPU reference (torch's
// fp64-accumulating CPU BatchNorm) trains through them.
template <int V>
__global__ void __launch_bounds__(kBlk)
    bnf_stats_kernel(const float* __restrict__ a, const float* __restrict__ b, const int* __restrict__ nvp,
                     const int64_t* __restrict__ rng, int64_t salt, float p, float* __restrict__ z,
                     float* __restrict__ part, int N, int C, Geo g) {
  using T = typename VecT<V>::T;
  __shared__ float red[kBlk * V];
  __shared__ double redd[kBlk * V];
  __shared__ float smean[kBlk];
  const int Nv = nvp ? min(*nvp, N) : N;
  const DropCfg d = drop_cfg(rng, salt, p);
  const int r0 = blockIdx.x * g.slab, r1 = min(N, r0 + g.slab), rv1 = min(Nv, r1);
  const int rl = threadIdx.x / g.tpr, cg_l = threadIdx.x % g.tpr;
  const bool fused = z != nullptr;
  for (int cg0 = 0; cg0 < g.ngrp; cg0 += g.tpr) {
    const int cg = cg0 + cg_l;
    const bool act = cg < g.ngrp;
    const int c0 = cg * V;
    // unconditional loads at clamped addresses (see rowc); validity is applied where
    // the values are used
    const int c0c = min(cg, g.ngrp - 1) * V;
    T v[kRows], bbv[kRows];
#pragma unroll
    for (int i = 0; i < kRows; ++i) v[i] = ldv<V>(a + (int64_t)rowc(r0 + rl + i * g.rpb, r1) * C + c0c);
    if (fused && b) {
#pragma unroll
      for (int i = 0; i < kRows; ++i) bbv[i] = ldv<V>(b + (int64_t)rowc(r0 + rl + i * g.rpb, r1) * C + c0c);
    }
    if (fused) {
#pragma unroll
      for (int i = 0; i < kRows; ++i) {
        const int r = r0 + rl + i * g.rpb;
        if (act && r < r1) {
          const int64_t off = (int64_t)r * C + c0;
          const T bb = bbv[i];
#pragma unroll
          for (int k = 0; k < V; ++k) {
            float x = el<V>(v[i], k);
            if (d.on) x = keep_elem(d.seed, (uint32_t)(off + k), d.thresh) ? x * d.scale : 0.f;
            if (b) x += el<V>(bb, k);
            set_el<V>(v[i], k, x);
          }
          stv<V>(z + off, v[i]);
        }
      }
    }
    float sm[V];
#pragma unroll
    for (int k = 0; k < V; ++k) sm[k] = 0.f;
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      const int r = r0 + rl + i * g.rpb;
      if (act && r < rv1) {
#pragma unroll
        for (int k = 0; k < V; ++k) sm[k] += el<V>(v[i], k);
      }
    }
    fold_rows<V>(sm, red, rl, cg_l, g);
    const float cnt = (float)max(rv1 - r0, 0);
    if (rl == 0 && act) {
#pragma unroll
      for (int k = 0; k < V; ++k) smean[cg_l * V + k] = cnt > 0.f ? sm[k] / cnt : 0.f;
    }
    __syncthreads();
    float mu[V];
    double m2[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      mu[k] = act ? smean[cg_l * V + k] : 0.f;
      m2[k] = 0.0;
    }
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      const int r = r0 + rl + i * g.rpb;
      if (act && r < rv1) {
#pragma unroll
        for (int k = 0; k < V; ++k) {
          const double t = (double)el<V>(v[i], k) - (double)mu[k];
          m2[k] = fma(t, t, m2[k]);
        }
      }
    }
    fold_rows_d<V>(m2, redd, rl, cg_l, g);
    if (rl == 0 && act) {
      float* P = part + (int64_t)blockIdx.x * 3 * C;
#pragma unroll
      for (int k = 0; k < V; ++k) {
        P[c0 + k] = cnt;
        P[C + c0 + k] = mu[k];
        P[2 * C + c0 + k] = cnt > 0.f ? (float)sqrt(m2[k] / (double)cnt) : 0.f;
      }
    }
    __syncthreads();
  }
}

// forward pass 2: every workgroup folds the S slab stats (exact two-pass combine,
// T threads per channel, fixed order), then y = z * scale + shift (+relu, padding
// rows -> 0) for its slab; workgroup 0 writes the saved stats and running stats.
template <int V>
__global__ void __launch_bounds__(kBlk)
    bnf_apply_kernel(const float* __restrict__ zr, const int* __restrict__ nvp, const float* __restrict__ part, int S,
                     const float* __restrict__ w, const float* __restrict__ beta, float* __restrict__ rmean,
                     float* __restrict__ rvar, int64_t* __restrict__ nbt, float momentum, float eps, int relu,
                     int zero_pad, float* __restrict__ y, float* __restrict__ smean, float* __restrict__ sinvstd,
                     int N, int C, Geo g) {
  extern __shared__ float sh[];  // scale[C], shift[C]
  __shared__ float red[kBlk];
  __shared__ double redd[kBlk];
  float* scl = sh;
  float* shf = sh + C;
  const int Nv = nvp ? min(*nvp, N) : N;
  const int r0 = blockIdx.x * g.slab, r1 = min(N, r0 + g.slab);
  const int rl = threadIdx.x / g.tpr, cg_l = threadIdx.x % g.tpr;
  // prefetch this slab's rows (first channel-group pass) before touching the partials
  typename VecT<V>::T v[kRows];
  {
    const int c0 = min(cg_l, g.ngrp - 1) * V;
#pragma unroll
    for (int i = 0; i < kRows; ++i) v[i] = ldv<V>(zr + (int64_t)rowc(r0 + rl + i * g.rpb, r1) * C + c0);
  }
  const int TT = max(1, kBlk / C);
  for (int cb = 0; cb < C; cb += kBlk / TT) {
    const int c = cb + threadIdx.x / TT, j = threadIdx.x % TT;
    const bool ok = c < C && threadIdx.x < (kBlk / TT) * TT;
    // all of this thread's partials in registers (one memory round trip)
    constexpr int kQ = 16;
    float qn[kQ], qm[kQ], q2[kQ];
    const int cc = min(c, C - 1);
#pragma unroll
    for (int t = 0; t < kQ; ++t) {
      const int64_t o = (int64_t)min(j + t * TT, S - 1) * 3 * C + cc;
      qn[t] = part[o];
      qm[t] = part[o + C];
      q2[t] = part[o + 2 * C];
    }
#pragma unroll
    for (int t = 0; t < kQ; ++t) {
      if (!(ok && j + t * TT < S)) qn[t] = qm[t] = q2[t] = 0.f;
    }
    float n = 0.f, sm = 0.f;
#pragma unroll
    for (int t = 0; t < kQ; ++t) {
      n += qn[t];
      sm = fmaf(qn[t], qm[t], sm);
    }
    for (int q = j + kQ * TT; ok && q < S; q += TT) {  // rare: more than 16 partials per thread
      const float nb = part[(int64_t)q * 3 * C + c];
      n += nb;
      sm = fmaf(nb, part[(int64_t)q * 3 * C + C + c], sm);
    }
    n = chan_sum(n, red, TT);
    sm = chan_sum(sm, red, TT);
    const float mean = n > 0.f ? sm / n : 0.f;
    double M2 = 0.0;  // sum_s n_s (std_s^2 + (mean_s - mean)^2), fp64 (see pass 1)
#pragma unroll
    for (int t = 0; t < kQ; ++t) {
      const double dl = (double)qm[t] - (double)mean, sd = q2[t];
      M2 += (double)qn[t] * (sd * sd + dl * dl);
    }
    for (int q = j + kQ * TT; ok && q < S; q += TT) {
      const float* P = part + (int64_t)q * 3 * C;
      const double dl = (double)P[C + c] - (double)mean, sd = P[2 * C + c];
      M2 += (double)P[c] * (sd * sd + dl * dl);
    }
    M2 = chan_sum_d(M2, redd, TT);
    if (ok && j == 0) {
      const double vard = n > 0.f ? M2 / (double)n : 0.0;
      const float var = (float)vard;
      const float is = (float)(1.0 / sqrt(vard + (double)eps));
      const float ww = w ? w[c] : 1.f, bb = beta ? beta[c] : 0.f;
      scl[c] = is * ww;
      shf[c] = bb - mean * is * ww;
      if (blockIdx.x == 0) {
        smean[c] = mean;
        sinvstd[c] = is;
        if (rmean) {
          const float unb = n > 1.f ? var * n / (n - 1.f) : var;
          rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
          rvar[c] = (1.f - momentum) * rvar[c] + momentum * unb;
        }
      }
    }
  }
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) nbt[0] += 1;
  __syncthreads();
  for (int cg = cg_l; cg < g.ngrp; cg += g.tpr) {
    const int c0 = cg * V;
    if (cg != cg_l) {  // further channel-group passes (C > 4 * tpr): load now
#pragma unroll
      for (int i = 0; i < kRows; ++i) {
        const int r = r0 + rl + i * g.rpb;
        if (r < r1) v[i] = ldv<V>(zr + (int64_t)r * C + c0);
      }
    }
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      const int r = r0 + rl + i * g.rpb;
      if (r < r1) {
        typename VecT<V>::T o;
        const bool pad = zero_pad && r >= Nv;
#pragma unroll
        for (int k = 0; k < V; ++k) {
          float t = fmaf(el<V>(v[i], k), scl[c0 + k], shf[c0 + k]);
          if (relu) t = fmaxf(t, 0.f);
          set_el<V>(o, k, pad ? 0.f : t);
        }
        stv<V>(y + (int64_t)r * C + c0, o);
      }
    }
  }
}

// backward pass 1: per-slab (sum g, sum g*xhat) -> part[S][2][C]; g = dy masked by relu / padding
template <int V>
__global__ void __launch_bounds__(kBlk)
    bnb_partial_kernel(const float* __restrict__ dy, const float* __restrict__ z, const int* __restrict__ nvp,
                       const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ w,
                       const float* __restrict__ beta, int relu, int zero_pad, float* __restrict__ part, int N, int C,
                       Geo g) {
  __shared__ float red[kBlk * V];
  const int Nv = nvp ? min(*nvp, N) : N;
  const int Ns = zero_pad ? Nv : N;
  const int r0 = blockIdx.x * g.slab, r1 = min(Ns, r0 + g.slab);
  const int rl = threadIdx.x / g.tpr, cg_l = threadIdx.x % g.tpr;
  for (int cg0 = 0; cg0 < g.ngrp; cg0 += g.tpr) {
    const int cg = cg0 + cg_l;
    const bool act = cg < g.ngrp;
    const int c0 = cg * V;
    float sg[V], sx[V], mu[V], is[V], ww[V], bb[V];
    const int c0c = min(cg, g.ngrp - 1) * V;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      sg[k] = sx[k] = 0.f;
      mu[k] = mean[c0c + k];
      is[k] = invstd[c0c + k];
      ww[k] = w ? w[c0c + k] : 1.f;
      bb[k] = beta ? beta[c0c + k] : 0.f;
    }
    typename VecT<V>::T gv[kRows], zv[kRows];
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      const int64_t off = (int64_t)rowc(r0 + rl + i * g.rpb, r1) * C + c0c;
      gv[i] = ldv<V>(dy + off);
      zv[i] = ldv<V>(z + off);
    }
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      const int r = r0 + rl + i * g.rpb;
      if (act && r < r1) {
#pragma unroll
        for (int k = 0; k < V; ++k) {
          const float xh = (el<V>(zv[i], k) - mu[k]) * is[k];
          float gg = el<V>(gv[i], k);
          if (relu && fmaf(xh, ww[k], bb[k]) <= 0.f) gg = 0.f;
          sg[k] += gg;
          sx[k] = fmaf(gg, xh, sx[k]);
        }
      }
    }
    fold_rows<V>(sg, red, rl, cg_l, g);
    fold_rows<V>(sx, red, rl, cg_l, g);
    if (rl == 0 && act) {
      float* P = part + (int64_t)blockIdx.x * 2 * C;
#pragma unroll
      for (int k = 0; k < V; ++k) {
        P[c0 + k] = sg[k];
        P[C + c0 + k] = sx[k];
      }
    }
  }
}

// backward pass 2: reduce partials (fixed order), dw/db (block 0), dz and dropout'd da for the slab
template <int V>
__global__ void __launch_bounds__(kBlk)
    bnb_apply_kernel(const float* __restrict__ dy, const float* __restrict__ z, const int* __restrict__ nvp,
                     const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ w,
                     const float* __restrict__ beta, const float* __restrict__ part, int S,
                     const int64_t* __restrict__ rng, int64_t salt, float p, int relu, int zero_pad,
                     float* __restrict__ dz, float* __restrict__ da, float* __restrict__ dw, float* __restrict__ db,
                     int N, int C, Geo g) {
  extern __shared__ float sh[];  // sum g [C], sum g*xhat [C]
  __shared__ float red[kBlk];
  float* Sg = sh;
  float* Sx = sh + C;
  const int Nv = nvp ? min(*nvp, N) : N;
  const int r0 = blockIdx.x * g.slab, r1 = min(N, r0 + g.slab);
  const int rl = threadIdx.x / g.tpr, cg_l = threadIdx.x % g.tpr;
  typename VecT<V>::T gvs[kRows], zvs[kRows];
  {
    const int c0 = min(cg_l, g.ngrp - 1) * V;
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      const int64_t off = (int64_t)rowc(r0 + rl + i * g.rpb, r1) * C + c0;
      gvs[i] = ldv<V>(dy + off);
      zvs[i] = ldv<V>(z + off);
    }
  }
  const int TT = max(1, kBlk / C);
  for (int cb = 0; cb < C; cb += kBlk / TT) {
    const int c = cb + threadIdx.x / TT, j = threadIdx.x % TT;
    const bool ok = c < C && threadIdx.x < (kBlk / TT) * TT;
    constexpr int kQ = 16;
    float qa[kQ], qb[kQ];
    const int cc = min(c, C - 1);
#pragma unroll
    for (int t = 0; t < kQ; ++t) {
      const int64_t o = (int64_t)min(j + t * TT, S - 1) * 2 * C + cc;
      qa[t] = part[o];
      qb[t] = part[o + C];
    }
#pragma unroll
    for (int t = 0; t < kQ; ++t) {
      if (!(ok && j + t * TT < S)) qa[t] = qb[t] = 0.f;
    }
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int t = 0; t < kQ; ++t) {
      a0 += qa[t];
      a1 += qb[t];
    }
    for (int q = j + kQ * TT; ok && q < S; q += TT) {
      a0 += part[(int64_t)q * 2 * C + c];
      a1 += part[(int64_t)q * 2 * C + C + c];
    }
    a0 = chan_sum(a0, red, TT);
    a1 = chan_sum(a1, red, TT);
    if (ok && j == 0) {
      Sg[c] = a0;
      Sx[c] = a1;
      if (blockIdx.x == 0) {
        if (dw) dw[c] = a1;
        if (db) db[c] = a0;
      }
    }
  }
  __syncthreads();
  const DropCfg d = drop_cfg(rng, salt, p);
  const float inv_n = Nv > 0 ? 1.f / (float)Nv : 0.f;
  for (int cg = cg_l; cg < g.ngrp; cg += g.tpr) {
    const int c0 = cg * V;
    float mu[V], is[V], ww[V], bb[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      mu[k] = mean[c0 + k];
      is[k] = invstd[c0 + k];
      ww[k] = w ? w[c0 + k] : 1.f;
      bb[k] = beta ? beta[c0 + k] : 0.f;
    }
    if (cg != cg_l) {
#pragma unroll
      for (int i = 0; i < kRows; ++i) {
        const int r = r0 + rl + i * g.rpb;
        if (r < r1) {
          gvs[i] = ldv<V>(dy + (int64_t)r * C + c0);
          zvs[i] = ldv<V>(z + (int64_t)r * C + c0);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < kRows; ++i) {
      const int r = r0 + rl + i * g.rpb;
      if (r >= r1) continue;
      const int64_t off = (int64_t)r * C + c0;
      const typename VecT<V>::T gv = gvs[i];
      const typename VecT<V>::T zv = zvs[i];
      typename VecT<V>::T o, od;
      const bool valid = r < Nv;
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const float xh = (el<V>(zv, k) - mu[k]) * is[k];
        float gg = el<V>(gv, k);
        if (relu && fmaf(xh, ww[k], bb[k]) <= 0.f) gg = 0.f;
        float t;
        if (valid) {
          t = ww[k] * is[k] * (gg - (Sg[c0 + k] + xh * Sx[c0 + k]) * inv_n);
        } else {
          t = zero_pad ? 0.f : gg * ww[k] * is[k];
        }
        set_el<V>(o, k, t);
        if (da) set_el<V>(od, k, keep_elem(d.seed, (uint32_t)(off + k), d.thresh) ? t * d.scale : 0.f);
      }
      stv<V>(dz + off, o);
      if (da) stv<V>(da + off, od);
    }
  }
}

static const float* optf(const c10::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr;
}

static Geo make_geo(int C, int V) {
  const int ngrp = C / V;
  int tpr = 1;
  while (tpr < ngrp && tpr < 64) tpr <<= 1;
  return Geo{tpr, kBlk / tpr, ngrp, (kBlk / tpr) * kRows};
}

// returns (y, z, mean, invstd); z is empty (use `a`) when neither dropout nor residual is fused
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> bn_fused_fwd(
    const at::Tensor& a, const c10::optional<at::Tensor>& b, const c10::optional<at::Tensor>& nv,
    const c10::optional<at::Tensor>& w, const c10::optional<at::Tensor>& beta,
    const c10::optional<at::Tensor>& rmean, const c10::optional<at::Tensor>& rvar,
    const c10::optional<at::Tensor>& nbt, const c10::optional<at::Tensor>& rng, int64_t salt, double p,
    double momentum, double eps, bool relu, bool zero_pad) {
  HY_CHECK_CUDA(a);
  HY_CHECK_F32(a);
  HY_CHECK_CONTIG(a);
  HY_CHECK(a.dim() == 2, "bn_fused_fwd expects [N, C]");
  const int N = (int)a.size(0), C = (int)a.size(1);
  const bool has_b = b.has_value() && b->defined();
  if (has_b) {
    HY_CHECK(b->sizes() == a.sizes() && b->is_contiguous() && b->scalar_type() == at::kFloat, "residual shape");
  }
  const bool drop = rng.has_value() && rng->defined() && p > 0.0;
  if (drop) HY_CHECK(rng->scalar_type() == at::kLong && rng->numel() >= 1, "rng must be an int64 counter");
  if (nv.has_value() && nv->defined()) HY_CHECK_I32(*nv);
  if (nbt.has_value() && nbt->defined()) HY_CHECK(nbt->scalar_type() == at::kLong, "num_batches_tracked int64");
  const bool fused_z = has_b || drop;
  at::Tensor z = fused_z ? at::empty_like(a) : at::empty({0}, a.options());
  at::Tensor y = at::empty_like(a);
  auto opt = a.options();
  at::Tensor mean = at::empty({C}, opt), invstd = at::empty({C}, opt);
  if (N == 0 || C == 0) return {y, z, mean.zero_(), invstd.fill_(0.f)};
  const int64_t* rp = drop ? rng->data_ptr<int64_t>() : nullptr;
  const int* nvp = nv.has_value() && nv->defined() ? nv->data_ptr<int>() : nullptr;
  int64_t* nb = nbt.has_value() && nbt->defined() ? nbt->data_ptr<int64_t>() : nullptr;
  float* rm = rmean.has_value() && rmean->defined() ? rmean->data_ptr<float>() : nullptr;
  float* rv = rvar.has_value() && rvar->defined() ? rvar->data_ptr<float>() : nullptr;
  const float* bp = has_b ? b->data_ptr<float>() : nullptr;
  float* zp = fused_z ? z.data_ptr<float>() : nullptr;
  const float* zr = fused_z ? z.data_ptr<float>() : a.data_ptr<float>();
  const Geo g0 = make_geo(C, C % 4 == 0 ? 4 : 1);
  const int S = ceil_div(N, g0.slab);
  at::Tensor part = at::empty({S, 3, C}, opt);
  const size_t lds = 2 * (size_t)C * sizeof(float);
#define HY_BNF(VV)                                                                                                 \
  {                                                                                                                \
    const Geo g = make_geo(C, VV);                                                                                 \
    bnf_stats_kernel<VV><<<S, kBlk, 0, stream()>>>(a.data_ptr<float>(), bp, nvp, rp, salt, (float)p, zp,          \
                                                   part.data_ptr<float>(), N, C, g);                              \
    bnf_apply_kernel<VV><<<S, kBlk, lds, stream()>>>(zr, nvp, part.data_ptr<float>(), S, optf(w), optf(beta), rm,  \
                                                     rv, nb, (float)momentum, (float)eps, relu, zero_pad,         \
                                                     y.data_ptr<float>(), mean.data_ptr<float>(),                 \
                                                     invstd.data_ptr<float>(), N, C, g);                          \
  }
  if (C % 4 == 0) HY_BNF(4) else HY_BNF(1)
#undef HY_BNF
  return {y, z, mean, invstd};
}

// returns (dz, da, dw, db); da undefined when no dropout (== dz)
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> bn_fused_bwd(
    const at::Tensor& dy_, const at::Tensor& z, const c10::optional<at::Tensor>& nv, const at::Tensor& mean,
    const at::Tensor& invstd, const c10::optional<at::Tensor>& w, const c10::optional<at::Tensor>& beta,
    const c10::optional<at::Tensor>& rng, int64_t salt, double p, bool relu, bool zero_pad) {
  at::Tensor dy = dy_.contiguous();
  HY_CHECK(dy.sizes() == z.sizes(), "dy/z shape mismatch");
  HY_CHECK_CONTIG(z);
  const int N = (int)z.size(0), C = (int)z.size(1);
  const bool drop = rng.has_value() && rng->defined() && p > 0.0;
  at::Tensor dz = at::empty_like(z);
  at::Tensor da = drop ? at::empty_like(z) : at::Tensor();
  at::Tensor dw = at::empty({C}, z.options()), db = at::empty({C}, z.options());
  if (N == 0 || C == 0) return {dz, da, dw.zero_(), db.zero_()};
  const int* nvp = nv.has_value() && nv->defined() ? nv->data_ptr<int>() : nullptr;
  const int64_t* rp = drop ? rng->data_ptr<int64_t>() : nullptr;
  float* dap = drop ? da.data_ptr<float>() : nullptr;
  const Geo g0 = make_geo(C, C % 4 == 0 ? 4 : 1);
  const int S = ceil_div(N, g0.slab);
  at::Tensor part = at::empty({S, 2, C}, z.options());  // every slab writes its (possibly zero) sums
  const size_t lds = 2 * (size_t)C * sizeof(float);
#define HY_BNB(VV)                                                                                                 \
  {                                                                                                                \
    const Geo g = make_geo(C, VV);                                                                                 \
    bnb_partial_kernel<VV><<<S, kBlk, 0, stream()>>>(dy.data_ptr<float>(), z.data_ptr<float>(), nvp,               \
                                                     mean.data_ptr<float>(), invstd.data_ptr<float>(), optf(w),   \
                                                     optf(beta), relu, zero_pad, part.data_ptr<float>(), N, C, g);\
    bnb_apply_kernel<VV><<<S, kBlk, lds, stream()>>>(dy.data_ptr<float>(), z.data_ptr<float>(), nvp,               \
                                                     mean.data_ptr<float>(), invstd.data_ptr<float>(), optf(w),   \
                                                     optf(beta), part.data_ptr<float>(), S, rp, salt, (float)p,   \
                                                     relu, zero_pad, dz.data_ptr<float>(), dap,                   \
                                                     dw.data_ptr<float>(), db.data_ptr<float>(), N, C, g);        \
  }
  if (C % 4 == 0) HY_BNB(4) else HY_BNB(1)
#undef HY_BNB
  return {dz, da, dw, db};
}

// standalone dropout with the same counter hash (for sites without a following BN)
__global__ void dropout_hash_kernel(const float* __restrict__ x, float* __restrict__ y, const int64_t* __restrict__ rng,
                                    int64_t salt, float p, int64_t n) {
  const DropCfg d = drop_cfg(rng, salt, p);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = keep_elem(d.seed, (uint32_t)i, d.thresh) ? x[i] * d.scale : 0.f;
}

at::Tensor dropout_hash(const at::Tensor& x_, const at::Tensor& rng, int64_t salt, double p) {
  at::Tensor x = x_.contiguous();
  HY_CHECK_F32(x);
  at::Tensor y = at::empty_like(x);
  const int64_t n = x.numel();
  if (n == 0) return y;
  const int blocks = (int)std::min<int64_t>(ceil_div(n, 256), 4096);
  dropout_hash_kernel<<<blocks, 256, 0, stream()>>>(x.data_ptr<float>(), y.data_ptr<float>(),
                                                    rng.data_ptr<int64_t>(), salt, (float)p, n);
  return y;
}

__global__ void counter_incr_kernel(int64_t* c) { c[0] += 1; }

void rng_advance(const at::Tensor& rng) {
  HY_CHECK(rng.scalar_type() == at::kLong && rng.is_cuda(), "rng must be a GPU int64 counter");
  counter_incr_kernel<<<1, 1, 0, stream()>>>(rng.data_ptr<int64_t>());
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def(
      "bn_fused_fwd(Tensor a, Tensor? b, Tensor? nv, Tensor? w, Tensor? beta, Tensor(a!)? rmean, Tensor(b!)? rvar, "
      "Tensor(c!)? nbt, Tensor? rng, int salt, float p, float momentum, float eps, bool relu, bool zero_pad) -> "
      "(Tensor, Tensor, Tensor, Tensor)");
  m.def(
      "bn_fused_bwd(Tensor dy, Tensor z, Tensor? nv, Tensor mean, Tensor invstd, Tensor? w, Tensor? beta, Tensor? rng, "
      "int salt, float p, bool relu, bool zero_pad) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("dropout_hash(Tensor x, Tensor rng, int salt, float p) -> Tensor");
  m.def("rng_advance(Tensor(a!) rng) -> ()");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("bn_fused_fwd", hy::bn_fused_fwd);
  m.impl("bn_fused_bwd", hy::bn_fused_bwd);
  m.impl("dropout_hash", hy::dropout_hash);
  m.impl("rng_advance", hy::rng_advance);
}
