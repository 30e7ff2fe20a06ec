// Segment-block-diagonal multi-head self-attention (flash style) for GPS (gfx950).
//
// Reference: hydragnn/globalAtt/gps.py:126-133 runs torch.nn.MultiheadAttention
// over `to_dense_batch(x, None)`, i.e. ALL nodes of the mini-batch form ONE
// sequence [1, N, F] ("batch" scope).  We generalise to a partition of the N
// tokens into segments (seg_ptr / seg_id): a query attends to the keys of its own
// segment.  batch scope = one segment (plus one segment holding padding rows),
// graph scope = one segment per graph (varlen, O(sum n_g^2)).
//
// GPS configs use small heads (hidden 64 / 8 heads -> D = 8), where the score
// work is exp/VALU-bound rather than matrix-bound, so this kernel keeps Q, the
// running max/sum and the output accumulator in registers (one query row per
// lane), stages K/V tiles through LDS (broadcast reads, conflict-free), and
// splits the key range over the 4 waves of a workgroup (merged through LDS at
// the end) and over S workgroups (merged by a combine pass), so that
// N/64 x H x S workgroups x 4 waves keep all 256 CUs busy.
// Never materialises the N x N score matrix; backward recomputes P from the
// saved log-sum-exp (two atomic-free passes: dQ by query rows, dK/dV by key
// rows).
#include "common.h"

namespace hy {

constexpr float kLog2e = 1.4426950408889634f;

// Raw v_exp_f32 (2^x).  exp2f() wraps it in a denormal-range fix-up (compare, select,
// offset, v_ldexp: 4 instructions per exponential); softmax arguments are <= 0 (or a
// few units above 0 with lazy rescaling) and results below 2^-126 only need to be ~0,
// so the bare instruction is exact enough and -inf still maps to 0.
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Packed fp32 (v_pk_fma_f32 on gfx950): two lanes of math per VALU op.  The
// D-wide dot products and rank-1 updates of the inner loops run on float2 pairs,
// halving the FMA instruction count (the kernels are VALU-issue bound at D = 8).
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 splat2(float v) { return f2{v, v}; }

template <int D>
__device__ __forceinline__ float pdot(const f2 (&a)[D / 2], const f2* __restrict__ b) {
  f2 t = a[0] * b[0];
#pragma unroll
  for (int d = 1; d < D / 2; ++d) t = pfma(a[d], b[d], t);
  return t.x + t.y;
}

template <int D>
struct AttnCfg {
  static constexpr int KT = D <= 8 ? 64 : (D <= 16 ? 32 : 16);  // keys per wave tile
};

__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

// Work decomposition (gfx950, 256 CUs): grid = (query blocks of 64, heads, key
// splits S).  Each workgroup's 4 waves share one 64-query block and stripe the
// keys of split s (KT-key tiles staged in LDS, broadcast reads); their online-
// softmax states are merged through LDS and written as a partial (m, l, acc)
// per (split, head, query).  A combine pass merges the S partials in a fixed
// order (deterministic).  S is chosen on the host so that the launch has
// >= ~6 workgroups per CU: the GPS batch-scope sequence (N ~ 2.3k tokens, 8
// heads) has only 40 x 8 = 320 query blocks, which left the chip at ~1.25
// waves per SIMD and latency-bound (rocprof: 84 us fwd) before the split.
//
// Q/K/V rows: element (n, h, d) at ptr[n * ld + h * D + d].  O: [N, H*D].  LSE: [H, N] (natural log).
// part: [S][H][N][D + 2]  (m in log2 units, l, acc[D])
__device__ __forceinline__ void split_range(int ub, int ue, int S, int s, int KT, int& cb, int& ce) {
  const int L = max(ue - ub, 0);
  const int C = ((L + S - 1) / S + KT - 1) / KT * KT;
  cb = ub + s * C;
  ce = min(ue, cb + C);
}

template <int D>
__global__ void __launch_bounds__(256) attn_fwd_kernel(const float* __restrict__ Q, const float* __restrict__ K,
                                                       const float* __restrict__ V, int ld,
                                                       float* __restrict__ part,
                                                       const int* __restrict__ seg_id,
                                                       const int* __restrict__ seg_ptr, int N, int H, int S,
                                                       float scale) {
  constexpr int KT = AttnCfg<D>::KT;
  __shared__ __attribute__((aligned(16))) float Ks[4][KT][D];
  __shared__ __attribute__((aligned(16))) float Vs[4][KT][D];
  __shared__ float Mrg[64][D + 2];
  const int h = blockIdx.y, sp = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int qi = blockIdx.x * 64 + lane;
  const bool qv = qi < N;
  int kb = INT_MAX, ke = 0;
  if (qv) {
    const int s = seg_id[qi];
    kb = seg_ptr[s];
    ke = seg_ptr[s + 1];
  }
  int cb, ce;
  split_range(wave_min_i(kb), wave_max_i(ke), S, sp, KT, cb, ce);
  f2 q[D / 2], acc[D / 2];
  const float qs = scale * kLog2e;  // scores in log2 domain
#pragma unroll
  for (int d = 0; d < D / 2; ++d) {
    q[d] = qv ? f2{Q[(int64_t)qi * ld + h * D + 2 * d], Q[(int64_t)qi * ld + h * D + 2 * d + 1]} * qs : splat2(0.f);
    acc[d] = splat2(0.f);
  }
  float m = -INFINITY, l = 0.f;
  for (int base = cb; base < ce; base += 4 * KT) {
    const int t = base + w * KT;
    for (int idx = lane; idx < KT * D; idx += 64) {
      const int j = t + idx / D, d = idx % D;
      const bool ok = j < ce;
      Ks[w][idx / D][d] = ok ? K[(int64_t)j * ld + h * D + d] : 0.f;
      Vs[w][idx / D][d] = ok ? V[(int64_t)j * ld + h * D + d] : 0.f;
    }
    __syncthreads();
    if (t < ce) {
      float s[KT];
      float mt = -INFINITY;
#pragma unroll
      for (int jj = 0; jj < KT; ++jj) {
        const float a = pdot<D>(q, reinterpret_cast<const f2*>(&Ks[w][jj][0]));
        const int j = t + jj;
        s[jj] = (j >= kb && j < ke && j < ce) ? a : -INFINITY;
        mt = fmaxf(mt, s[jj]);
      }
      if (mt > -INFINITY) {
        const float mn = fmaxf(m, mt);
        const float alpha = fexp2(m - mn);  // m=-inf -> 0
        l *= alpha;
#pragma unroll
        for (int d = 0; d < D / 2; ++d) acc[d] *= alpha;
#pragma unroll
        for (int jj = 0; jj < KT; ++jj) {
          const float p = fexp2(s[jj] - mn);
          l += p;
          const f2* vr = reinterpret_cast<const f2*>(&Vs[w][jj][0]);
          const f2 pp = splat2(p);
#pragma unroll
          for (int d = 0; d < D / 2; ++d) acc[d] = pfma(pp, vr[d], acc[d]);
        }
        m = mn;
      }
    }
    __syncthreads();
  }
  // merge the 4 key stripes: wave w folds its (m, l, acc) into the running LDS copy
  for (int step = 0; step < 4; ++step) {
    if (w == step) {
      if (step > 0) {
        const float mo = Mrg[lane][0], lo = Mrg[lane][1];
        const float M = fmaxf(m, mo);
        const float fo = (M > -INFINITY) ? fexp2(mo - M) : 0.f;
        const float fs = (M > -INFINITY) ? fexp2(m - M) : 0.f;
        l = lo * fo + l * fs;
#pragma unroll
        for (int d = 0; d < D / 2; ++d)
          acc[d] = f2{Mrg[lane][2 + 2 * d], Mrg[lane][3 + 2 * d]} * fo + acc[d] * fs;
        m = M;
      }
      if (step < 3) {
        Mrg[lane][0] = m;
        Mrg[lane][1] = l;
#pragma unroll
        for (int d = 0; d < D / 2; ++d) {
          Mrg[lane][2 + 2 * d] = acc[d].x;
          Mrg[lane][3 + 2 * d] = acc[d].y;
        }
      } else if (qv) {
        float* P = part + (((int64_t)sp * H + h) * N + qi) * (D + 2);
        P[0] = m;
        P[1] = l;
#pragma unroll
        for (int d = 0; d < D / 2; ++d) {
          P[2 + 2 * d] = acc[d].x;
          P[3 + 2 * d] = acc[d].y;
        }
      }
    }
    __syncthreads();
  }
}

// Scalar-operand variant of the forward kernel (D <= 16).  All 64 lanes of a wave
// need every key/value row of the stripe, so instead of staging K/V through LDS
// (64-lane broadcast ds_read_b128: 1 KB of LDS data path per 16 B used, which
// bounded the LDS version at ~54 us for the OC20 shape) the rows are fetched with
// wave-uniform addresses -> s_load into SGPRs, and the VALU math takes them as
// scalar operands.  Each wave owns a contiguous quarter of the split's keys;
// the 4 stripes are merged through LDS exactly as in attn_fwd_kernel.
__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

template <int D>
__global__ void __launch_bounds__(256) attn_fwd_sk_kernel(const float* __restrict__ Q, const float* __restrict__ K,
                                                          const float* __restrict__ V, int ld,
                                                          float* __restrict__ part,
                                                          const int* __restrict__ seg_id,
                                                          const int* __restrict__ seg_ptr, int N, int H, int S,
                                                          float scale) {
  constexpr int U = 8;  // keys per online-softmax chunk
  __shared__ float Mrg[64][D + 2];
  const int h = blockIdx.y, sp = blockIdx.z;
  const int lane = threadIdx.x & 63, w = uniform(threadIdx.x >> 6);
  const int qi = blockIdx.x * 64 + lane;
  const bool qv = qi < N;
  int kb = INT_MAX, ke = 0;
  if (qv) {
    const int s = seg_id[qi];
    kb = seg_ptr[s];
    ke = seg_ptr[s + 1];
  }
  int cb, ce;
  split_range(uniform(wave_min_i(kb)), uniform(wave_max_i(ke)), S, sp, 4 * U, cb, ce);
  const int L4 = ((max(ce - cb, 0) + 4 * U - 1) / (4 * U)) * U;  // stripe length, multiple of U
  const int wb = uniform(cb + w * L4), we = uniform(min(ce, wb + L4));
  f2 q[D / 2], acc[D / 2];
  const float qs = scale * kLog2e;  // scores in log2 domain
#pragma unroll
  for (int d = 0; d < D / 2; ++d) {
    q[d] = qv ? f2{Q[(int64_t)qi * ld + h * D + 2 * d], Q[(int64_t)qi * ld + h * D + 2 * d + 1]} * qs : splat2(0.f);
    acc[d] = splat2(0.f);
  }
  float m = -INFINITY, l = 0.f;
  const int klo = max(kb, wb), khi = min(ke, we);  // this lane's valid keys in the stripe
  for (int j0 = wb; j0 < we; j0 += U) {
    float s[U];
    float mt = -INFINITY;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = min(j0 + u, we - 1);  // uniform, in range
      const f2* kr = reinterpret_cast<const f2*>(K + (int64_t)j * ld + h * D);
      const float a = pdot<D>(q, kr);
      s[u] = (j0 + u >= klo && j0 + u < khi) ? a : -INFINITY;
      mt = fmaxf(mt, s[u]);
    }
    const float mn = fmaxf(m, mt);
    if (mn > -INFINITY) {
      const float alpha = fexp2(m - mn);
      l *= alpha;
#pragma unroll
      for (int d = 0; d < D / 2; ++d) acc[d] *= alpha;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = min(j0 + u, we - 1);
        const f2* vr = reinterpret_cast<const f2*>(V + (int64_t)j * ld + h * D);
        const float p = fexp2(s[u] - mn);  // -inf -> 0
        l += p;
        const f2 pp = splat2(p);
#pragma unroll
        for (int d = 0; d < D / 2; ++d) acc[d] = pfma(pp, vr[d], acc[d]);
      }
      m = mn;
    }
  }
  for (int step = 0; step < 4; ++step) {
    if (w == step) {
      if (step > 0) {
        const float mo = Mrg[lane][0], lo = Mrg[lane][1];
        const float M = fmaxf(m, mo);
        const float fo = (M > -INFINITY) ? fexp2(mo - M) : 0.f;
        const float fs = (M > -INFINITY) ? fexp2(m - M) : 0.f;
        l = lo * fo + l * fs;
#pragma unroll
        for (int d = 0; d < D / 2; ++d)
          acc[d] = f2{Mrg[lane][2 + 2 * d], Mrg[lane][3 + 2 * d]} * fo + acc[d] * fs;
        m = M;
      }
      if (step < 3) {
        Mrg[lane][0] = m;
        Mrg[lane][1] = l;
#pragma unroll
        for (int d = 0; d < D / 2; ++d) {
          Mrg[lane][2 + 2 * d] = acc[d].x;
          Mrg[lane][3 + 2 * d] = acc[d].y;
        }
      } else if (qv) {
        float* P = part + (((int64_t)sp * H + h) * N + qi) * (D + 2);
        P[0] = m;
        P[1] = l;
#pragma unroll
        for (int d = 0; d < D / 2; ++d) {
          P[2 + 2 * d] = acc[d].x;
          P[3 + 2 * d] = acc[d].y;
        }
      }
    }
    __syncthreads();
  }
}

// Merge the S split partials of every (head, query) in a fixed order -> O, LSE.
template <int D>
__global__ void __launch_bounds__(256) attn_fwd_combine_kernel(const float* __restrict__ part,
                                                               float* __restrict__ O, float* __restrict__ LSE,
                                                               int N, int H, int S) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)N * H) return;
  const int h = (int)(t / N), qi = (int)(t % N);
  const int64_t sstride = (int64_t)H * N * (D + 2);
  const float* P = part + ((int64_t)h * N + qi) * (D + 2);
  float M = -INFINITY;
  for (int s = 0; s < S; ++s) M = fmaxf(M, P[s * sstride]);
  float l = 0.f, acc[D];
#pragma unroll
  for (int d = 0; d < D; ++d) acc[d] = 0.f;
  if (M > -INFINITY) {
    for (int s = 0; s < S; ++s) {
      const float* p = P + s * sstride;
      const float f = fexp2(p[0] - M);  // p[0] = -inf -> 0
      l = fmaf(p[1], f, l);
#pragma unroll
      for (int d = 0; d < D; ++d) acc[d] = fmaf(p[2 + d], f, acc[d]);
    }
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d) O[(int64_t)qi * (H * D) + h * D + d] = acc[d] * inv;
  LSE[(int64_t)h * N + qi] = l > 0.f ? (M + log2f(l)) / kLog2e : -INFINITY;
}

// delta[h, i] = sum_d dO[i,h,d] * O[i,h,d]
__global__ void attn_delta_kernel(const float* __restrict__ dO, const float* __restrict__ O,
                                  float* __restrict__ delta, int N, int H, int D) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)N * H) return;
  const int i = (int)(t / H), h = (int)(t % H);
  float a = 0.f;
  for (int d = 0; d < D; ++d) a += dO[(int64_t)i * H * D + h * D + d] * O[(int64_t)i * H * D + h * D + d];
  delta[(int64_t)h * N + i] = a;
}

// dQ: one query row per lane, key stripes over 4 waves, key splits over blockIdx.z.
// Output rows (already scaled) at dQ + z * split_stride + i * lddq + h * D.
template <int D>
__global__ void __launch_bounds__(256) attn_bwd_dq_kernel(
    const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V, int ld,
    const float* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ delta,
    float* __restrict__ dQ, int lddq, int64_t split_stride, const int* __restrict__ seg_id,
    const int* __restrict__ seg_ptr, int N, int H, int S, float scale) {
  constexpr int KT = AttnCfg<D>::KT;
  __shared__ __attribute__((aligned(16))) float Ks[4][KT][D];
  __shared__ __attribute__((aligned(16))) float Vs[4][KT][D];
  __shared__ float Mrg[64][D];
  const int h = blockIdx.y, sp = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int qi = blockIdx.x * 64 + lane;
  const bool qv = qi < N;
  int kb = INT_MAX, ke = 0;
  if (qv) {
    const int s = seg_id[qi];
    kb = seg_ptr[s];
    ke = seg_ptr[s + 1];
  }
  int cb, ce;
  split_range(wave_min_i(kb), wave_max_i(ke), S, sp, KT, cb, ce);
  f2 q[D / 2], go[D / 2], dq[D / 2];
#pragma unroll
  for (int d = 0; d < D / 2; ++d) {
    const int64_t o = (int64_t)qi * ld + h * D + 2 * d;
    const int64_t og = (int64_t)qi * H * D + h * D + 2 * d;
    q[d] = qv ? f2{Q[o], Q[o + 1]} * scale : splat2(0.f);
    go[d] = qv ? f2{dO[og], dO[og + 1]} : splat2(0.f);
    dq[d] = splat2(0.f);
  }
  const float lse = qv ? LSE[(int64_t)h * N + qi] : 0.f;
  const float dl = qv ? delta[(int64_t)h * N + qi] : 0.f;
  for (int base = cb; base < ce; base += 4 * KT) {
    const int t = base + w * KT;
    for (int idx = lane; idx < KT * D; idx += 64) {
      const int j = t + idx / D, d = idx % D;
      const bool ok = j < ce;
      Ks[w][idx / D][d] = ok ? K[(int64_t)j * ld + h * D + d] : 0.f;
      Vs[w][idx / D][d] = ok ? V[(int64_t)j * ld + h * D + d] : 0.f;
    }
    __syncthreads();
    if (t < ce) {
#pragma unroll 4
      for (int jj = 0; jj < KT; ++jj) {
        const int j = t + jj;
        if (j >= kb && j < ke && j < ce) {
          const f2* kr = reinterpret_cast<const f2*>(&Ks[w][jj][0]);
          const float sc = pdot<D>(q, kr);
          const float dp = pdot<D>(go, reinterpret_cast<const f2*>(&Vs[w][jj][0]));
          const float p = fexp2((sc - lse) * kLog2e);
          const f2 ds = splat2(p * (dp - dl));
#pragma unroll
          for (int d = 0; d < D / 2; ++d) dq[d] = pfma(ds, kr[d], dq[d]);
        }
      }
    }
    __syncthreads();
  }
  for (int step = 0; step < 4; ++step) {
    if (w == step) {
#pragma unroll
      for (int d = 0; d < D / 2; ++d) {
        const float t0 = (step > 0 ? Mrg[lane][2 * d] : 0.f) + dq[d].x;
        const float t1 = (step > 0 ? Mrg[lane][2 * d + 1] : 0.f) + dq[d].y;
        if (step < 3) {
          Mrg[lane][2 * d] = t0;
          Mrg[lane][2 * d + 1] = t1;
        } else if (qv) {
          float* o = dQ + sp * split_stride + (int64_t)qi * lddq + h * D + 2 * d;
          o[0] = t0 * scale;
          o[1] = t1 * scale;
        }
      }
    }
    __syncthreads();
  }
}

// dK, dV: one key row per lane, query stripes over 4 waves, query splits over blockIdx.z.
template <int D>
__global__ void __launch_bounds__(256) attn_bwd_dkv_kernel(
    const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V, int ld,
    const float* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ delta,
    float* __restrict__ dK, float* __restrict__ dV, int lddkv, int64_t split_stride,
    const int* __restrict__ seg_id, const int* __restrict__ seg_ptr, int N, int H, int S, float scale) {
  constexpr int QT = AttnCfg<D>::KT;
  __shared__ __attribute__((aligned(16))) float Qs[4][QT][D];
  __shared__ __attribute__((aligned(16))) float Gs[4][QT][D];
  __shared__ float Ls[4][QT][2];
  __shared__ float Mrg[64][2 * D];
  const int h = blockIdx.y, sp = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int kj = blockIdx.x * 64 + lane;
  const bool kv = kj < N;
  int qb = INT_MAX, qe = 0;
  if (kv) {
    const int s = seg_id[kj];
    qb = seg_ptr[s];
    qe = seg_ptr[s + 1];
  }
  int cb, ce;
  split_range(wave_min_i(qb), wave_max_i(qe), S, sp, QT, cb, ce);
  f2 k[D / 2], v[D / 2], dk[D / 2], dv[D / 2];
#pragma unroll
  for (int d = 0; d < D / 2; ++d) {
    const int64_t o = (int64_t)kj * ld + h * D + 2 * d;
    k[d] = kv ? f2{K[o], K[o + 1]} * scale : splat2(0.f);
    v[d] = kv ? f2{V[o], V[o + 1]} : splat2(0.f);
    dk[d] = splat2(0.f);
    dv[d] = splat2(0.f);
  }
  for (int base = cb; base < ce; base += 4 * QT) {
    const int t = base + w * QT;
    for (int idx = lane; idx < QT * D; idx += 64) {
      const int i = t + idx / D, d = idx % D;
      const bool ok = i < ce;
      Qs[w][idx / D][d] = ok ? Q[(int64_t)i * ld + h * D + d] : 0.f;
      Gs[w][idx / D][d] = ok ? dO[(int64_t)i * H * D + h * D + d] : 0.f;
    }
    for (int idx = lane; idx < QT; idx += 64) {
      const int i = t + idx;
      const bool ok = i < ce;
      Ls[w][idx][0] = ok ? LSE[(int64_t)h * N + i] : 0.f;
      Ls[w][idx][1] = ok ? delta[(int64_t)h * N + i] : 0.f;
    }
    __syncthreads();
    if (t < ce) {
#pragma unroll 4
      for (int ii = 0; ii < QT; ++ii) {
        const int i = t + ii;
        if (i >= qb && i < qe && i < ce) {
          const f2* qr = reinterpret_cast<const f2*>(&Qs[w][ii][0]);
          const f2* gr = reinterpret_cast<const f2*>(&Gs[w][ii][0]);
          const float sc = pdot<D>(k, qr);
          const float dp = pdot<D>(v, gr);
          const float p = fexp2((sc - Ls[w][ii][0]) * kLog2e);
          const f2 pp = splat2(p);
          const f2 ds = splat2(p * (dp - Ls[w][ii][1]));
#pragma unroll
          for (int d = 0; d < D / 2; ++d) {
            dv[d] = pfma(pp, gr[d], dv[d]);
            dk[d] = pfma(ds, qr[d], dk[d]);
          }
        }
      }
    }
    __syncthreads();
  }
  for (int step = 0; step < 4; ++step) {
    if (w == step) {
#pragma unroll
      for (int d = 0; d < D / 2; ++d) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int c = 2 * d + e;
          const float tk = (step > 0 ? Mrg[lane][c] : 0.f) + (e ? dk[d].y : dk[d].x);
          const float tv = (step > 0 ? Mrg[lane][D + c] : 0.f) + (e ? dv[d].y : dv[d].x);
          if (step < 3) {
            Mrg[lane][c] = tk;
            Mrg[lane][D + c] = tv;
          } else if (kv) {
            dK[sp * split_stride + (int64_t)kj * lddkv + h * D + c] = tk * scale;
            dV[sp * split_stride + (int64_t)kj * lddkv + h * D + c] = tv;
          }
        }
      }
    }
    __syncthreads();
  }
}

// Scalar-operand backward kernels (D <= 16), same stripe structure as attn_fwd_sk_kernel.
template <int D>
__global__ void __launch_bounds__(256) attn_bwd_dq_sk_kernel(
    const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V, int ld,
    const float* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ delta,
    float* __restrict__ dQ, int lddq, int64_t split_stride, const int* __restrict__ seg_id,
    const int* __restrict__ seg_ptr, int N, int H, int S, float scale) {
  constexpr int U = 8;
  __shared__ float Mrg[64][D];
  const int h = blockIdx.y, sp = blockIdx.z;
  const int lane = threadIdx.x & 63, w = uniform(threadIdx.x >> 6);
  const int qi = blockIdx.x * 64 + lane;
  const bool qv = qi < N;
  int kb = INT_MAX, ke = 0;
  if (qv) {
    const int s = seg_id[qi];
    kb = seg_ptr[s];
    ke = seg_ptr[s + 1];
  }
  int cb, ce;
  split_range(uniform(wave_min_i(kb)), uniform(wave_max_i(ke)), S, sp, 4 * U, cb, ce);
  const int L4 = ((max(ce - cb, 0) + 4 * U - 1) / (4 * U)) * U;
  const int wb = uniform(cb + w * L4), we = uniform(min(ce, wb + L4));
  f2 q[D / 2], go[D / 2], dq[D / 2];
#pragma unroll
  for (int d = 0; d < D / 2; ++d) {
    const int64_t o = (int64_t)qi * ld + h * D + 2 * d;
    const int64_t og = (int64_t)qi * H * D + h * D + 2 * d;
    q[d] = qv ? f2{Q[o], Q[o + 1]} * scale : splat2(0.f);
    go[d] = qv ? f2{dO[og], dO[og + 1]} : splat2(0.f);
    dq[d] = splat2(0.f);
  }
  const float lse = qv ? LSE[(int64_t)h * N + qi] : 0.f;
  const float dl = qv ? delta[(int64_t)h * N + qi] : 0.f;
  const int klo = max(kb, wb), khi = min(ke, we);
  for (int j0 = wb; j0 < we; j0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = min(j0 + u, we - 1);
      const f2* kr = reinterpret_cast<const f2*>(K + (int64_t)j * ld + h * D);
      const f2* vr = reinterpret_cast<const f2*>(V + (int64_t)j * ld + h * D);
      const float sc = pdot<D>(q, kr);
      const float dp = pdot<D>(go, vr);
      const bool ok = j0 + u >= klo && j0 + u < khi;
      const float p = ok ? fexp2((sc - lse) * kLog2e) : 0.f;
      const f2 ds = splat2(p * (dp - dl));
#pragma unroll
      for (int d = 0; d < D / 2; ++d) dq[d] = pfma(ds, kr[d], dq[d]);
    }
  }
  for (int step = 0; step < 4; ++step) {
    if (w == step) {
#pragma unroll
      for (int d = 0; d < D / 2; ++d) {
        const float t0 = (step > 0 ? Mrg[lane][2 * d] : 0.f) + dq[d].x;
        const float t1 = (step > 0 ? Mrg[lane][2 * d + 1] : 0.f) + dq[d].y;
        if (step < 3) {
          Mrg[lane][2 * d] = t0;
          Mrg[lane][2 * d + 1] = t1;
        } else if (qv) {
          float* o = dQ + sp * split_stride + (int64_t)qi * lddq + h * D + 2 * d;
          o[0] = t0 * scale;
          o[1] = t1 * scale;
        }
      }
    }
    __syncthreads();
  }
}

template <int D>
__global__ void __launch_bounds__(256) attn_bwd_dkv_sk_kernel(
    const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V, int ld,
    const float* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ delta,
    float* __restrict__ dK, float* __restrict__ dV, int lddkv, int64_t split_stride,
    const int* __restrict__ seg_id, const int* __restrict__ seg_ptr, int N, int H, int S, float scale) {
  constexpr int U = 8;
  __shared__ float Mrg[64][2 * D];
  const int h = blockIdx.y, sp = blockIdx.z;
  const int lane = threadIdx.x & 63, w = uniform(threadIdx.x >> 6);
  const int kj = blockIdx.x * 64 + lane;
  const bool kv = kj < N;
  int qb = INT_MAX, qe = 0;
  if (kv) {
    const int s = seg_id[kj];
    qb = seg_ptr[s];
    qe = seg_ptr[s + 1];
  }
  int cb, ce;
  split_range(uniform(wave_min_i(qb)), uniform(wave_max_i(qe)), S, sp, 4 * U, cb, ce);
  const int L4 = ((max(ce - cb, 0) + 4 * U - 1) / (4 * U)) * U;
  const int wb = uniform(cb + w * L4), we = uniform(min(ce, wb + L4));
  f2 k[D / 2], v[D / 2], dk[D / 2], dv[D / 2];
#pragma unroll
  for (int d = 0; d < D / 2; ++d) {
    const int64_t o = (int64_t)kj * ld + h * D + 2 * d;
    k[d] = kv ? f2{K[o], K[o + 1]} * scale : splat2(0.f);
    v[d] = kv ? f2{V[o], V[o + 1]} : splat2(0.f);
    dk[d] = splat2(0.f);
    dv[d] = splat2(0.f);
  }
  const int ilo = max(qb, wb), ihi = min(qe, we);
  const float* Lh = LSE + (int64_t)h * N;
  const float* Dh = delta + (int64_t)h * N;
  for (int i0 = wb; i0 < we; i0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(i0 + u, we - 1);
      const f2* qr = reinterpret_cast<const f2*>(Q + (int64_t)i * ld + h * D);
      const f2* gr = reinterpret_cast<const f2*>(dO + (int64_t)i * H * D + h * D);
      const float sc = pdot<D>(k, qr);
      const float dp = pdot<D>(v, gr);
      const bool ok = i0 + u >= ilo && i0 + u < ihi;
      const float p = ok ? fexp2((sc - Lh[i]) * kLog2e) : 0.f;
      const f2 pp = splat2(p);
      const f2 ds = splat2(p * (dp - Dh[i]));
#pragma unroll
      for (int d = 0; d < D / 2; ++d) {
        dv[d] = pfma(pp, gr[d], dv[d]);
        dk[d] = pfma(ds, qr[d], dk[d]);
      }
    }
  }
  for (int step = 0; step < 4; ++step) {
    if (w == step) {
#pragma unroll
      for (int d = 0; d < D / 2; ++d) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int c = 2 * d + e;
          const float tk = (step > 0 ? Mrg[lane][c] : 0.f) + (e ? dk[d].y : dk[d].x);
          const float tv = (step > 0 ? Mrg[lane][D + c] : 0.f) + (e ? dv[d].y : dv[d].x);
          if (step < 3) {
            Mrg[lane][c] = tk;
            Mrg[lane][D + c] = tv;
          } else if (kv) {
            dK[sp * split_stride + (int64_t)kj * lddkv + h * D + c] = tk * scale;
            dV[sp * split_stride + (int64_t)kj * lddkv + h * D + c] = tv;
          }
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// v3 kernels (D <= 16): scalar-operand K/V (or Q/dO) rows like the *_sk kernels, with the
// per-score VALU work cut to the arithmetic itself.  rocprofv3 PMC on the OC20 shape
// (N = 2311, H = 8, D = 8) put the sk forward at ~20 VALU instructions per 64 scores
// against a floor of ~12; the difference was masking, max/subtract bookkeeping and
// per-key address clamps.  Here:
//  * every lane owns QPL rows (queries for fwd / dQ, keys for dK/dV), so each scalar row
//    load and its address arithmetic feeds QPL x the math;
//  * chunks of U keys that lie inside every valid lane's range ("interior" chunks, the
//    bulk of a batch-scope sequence) run without per-score masks or clamps;
//  * the subtraction of the running max / LSE / delta is folded into the initial value of
//    the packed dot product (no separate subtract);
//  * forward: lazy rescaling — the running max m only moves when a chunk exceeds it by
//    more than 8 (log2 units), so p = exp2(s - m) stays <= 256 and the rescale (exp +
//    D+1 multiplies) runs on a handful of chunks per row instead of every chunk.
// Masked boundary chunks take the exact per-key path.  Same partial layouts as the v1/sk
// kernels, so the combine / sum passes are shared.
template <int D>
__device__ __forceinline__ float pdot_init(const f2 (&a)[D / 2], const f2* __restrict__ b, float init) {
  f2 t = pfma(a[0], b[0], f2{init, 0.f});
#pragma unroll
  for (int d = 1; d < D / 2; ++d) t = pfma(a[d], b[d], t);
  return t.x + t.y;
}

__device__ __forceinline__ bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }

template <int D, int QPL>
__global__ void __launch_bounds__(256) attn_fwd_v3_kernel(const float* __restrict__ Q, const float* __restrict__ K,
                                                          const float* __restrict__ V, int ld,
                                                          float* __restrict__ part,
                                                          const int* __restrict__ seg_id,
                                                          const int* __restrict__ seg_ptr, int N, int H, int S,
                                                          float scale) {
  constexpr int U = 8;
  constexpr float kTau = 8.f;  // lazy-rescale threshold (log2 units)
  __shared__ float Mrg[64 * QPL][D + 2];
  const int h = blockIdx.y, sp = blockIdx.z;
  const int lane = threadIdx.x & 63, w = uniform(threadIdx.x >> 6);
  int qi[QPL], kb[QPL], ke[QPL];
  int bmin = INT_MAX, bmax = 0;
#pragma unroll
  for (int r = 0; r < QPL; ++r) {
    qi[r] = (blockIdx.x * QPL + r) * 64 + lane;
    kb[r] = INT_MAX;
    ke[r] = 0;
    if (qi[r] < N) {
      const int s = seg_id[qi[r]];
      kb[r] = seg_ptr[s];
      ke[r] = seg_ptr[s + 1];
    }
    bmin = min(bmin, kb[r]);
    bmax = max(bmax, ke[r]);
  }
  int cb, ce;
  split_range(uniform(wave_min_i(bmin)), uniform(wave_max_i(bmax)), S, sp, 4 * U, cb, ce);
  const int L4 = ((max(ce - cb, 0) + 4 * U - 1) / (4 * U)) * U;
  const int wb = uniform(cb + w * L4), we = uniform(min(ce, wb + L4));
  // interior range: keys valid for every valid row of the wave
  int lo_all = wb, hi_all = we;
  int klo[QPL], khi[QPL];
#pragma unroll
  for (int r = 0; r < QPL; ++r) {
    klo[r] = max(kb[r], wb);
    khi[r] = min(ke[r], we);
    if (qi[r] < N) {
      lo_all = max(lo_all, klo[r]);
      hi_all = min(hi_all, khi[r]);
    }
  }
  lo_all = uniform(wave_max_i(lo_all));
  hi_all = uniform(wave_min_i(hi_all));
  const float qs = scale * kLog2e;
  f2 q[QPL][D / 2], acc[QPL][D / 2];
  float m[QPL], l[QPL];
#pragma unroll
  for (int r = 0; r < QPL; ++r) {
    const bool v = qi[r] < N;
#pragma unroll
    for (int d = 0; d < D / 2; ++d) {
      q[r][d] = v ? f2{Q[(int64_t)qi[r] * ld + h * D + 2 * d], Q[(int64_t)qi[r] * ld + h * D + 2 * d + 1]} * qs
                  : splat2(0.f);
      acc[r][d] = splat2(0.f);
    }
    m[r] = v ? -INFINITY : 0.f;  // rows past N: finite m, q = 0 -> harmless p = 1
    l[r] = 0.f;
  }
  bool started = false;  // every valid row has a finite running max
  for (int j0 = wb; j0 < we; j0 += U) {
    if (started && j0 >= lo_all && j0 + U <= hi_all) {
      // interior chunk: no masks, scores relative to the running max, lazy rescale
      float s[QPL][U];
      float mt[QPL];
#pragma unroll
      for (int r = 0; r < QPL; ++r) mt[r] = -INFINITY;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const f2* kr = reinterpret_cast<const f2*>(K + (int64_t)(j0 + u) * ld + h * D);
#pragma unroll
        for (int r = 0; r < QPL; ++r) {
          s[r][u] = pdot_init<D>(q[r], kr, -m[r]);
          mt[r] = fmaxf(mt[r], s[r][u]);
        }
      }
      bool need = false;
#pragma unroll
      for (int r = 0; r < QPL; ++r) need |= mt[r] > kTau;
      if (wave_any(need)) {
#pragma unroll
        for (int r = 0; r < QPL; ++r) {
          const float c = mt[r] > kTau ? mt[r] : 0.f;
          const float alpha = fexp2(-c);
          l[r] *= alpha;
#pragma unroll
          for (int d = 0; d < D / 2; ++d) acc[r][d] *= alpha;
#pragma unroll
          for (int u = 0; u < U; ++u) s[r][u] -= c;
          m[r] += c;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const f2* vr = reinterpret_cast<const f2*>(V + (int64_t)(j0 + u) * ld + h * D);
#pragma unroll
        for (int r = 0; r < QPL; ++r) {
          const float p = fexp2(s[r][u]);
          l[r] += p;
          const f2 pp = splat2(p);
#pragma unroll
          for (int d = 0; d < D / 2; ++d) acc[r][d] = pfma(pp, vr[d], acc[r][d]);
        }
      }
    } else {
      // boundary chunk: exact masked online softmax
#pragma unroll
      for (int r = 0; r < QPL; ++r) {
        float s[U];
        float mt = -INFINITY;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int j = min(j0 + u, we - 1);
          const float a = pdot<D>(q[r], reinterpret_cast<const f2*>(K + (int64_t)j * ld + h * D));
          s[u] = (j0 + u >= klo[r] && j0 + u < khi[r]) ? a : -INFINITY;
          mt = fmaxf(mt, s[u]);
        }
        const float mn = fmaxf(m[r], mt);
        if (mn > -INFINITY) {
          const float alpha = fexp2(m[r] - mn);
          l[r] *= alpha;
#pragma unroll
          for (int d = 0; d < D / 2; ++d) acc[r][d] *= alpha;
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int j = min(j0 + u, we - 1);
            const f2* vr = reinterpret_cast<const f2*>(V + (int64_t)j * ld + h * D);
            const float p = fexp2(s[u] - mn);
            l[r] += p;
            const f2 pp = splat2(p);
#pragma unroll
            for (int d = 0; d < D / 2; ++d) acc[r][d] = pfma(pp, vr[d], acc[r][d]);
          }
          m[r] = mn;
        }
      }
      bool miss = false;
#pragma unroll
      for (int r = 0; r < QPL; ++r) miss |= !(m[r] > -INFINITY);
      started = !wave_any(miss);
    }
  }
  // merge the 4 key stripes through LDS (fixed order), write the split partial
  for (int step = 0; step < 4; ++step) {
    if (w == step) {
#pragma unroll
      for (int r = 0; r < QPL; ++r) {
        const int row = r * 64 + lane;
        if (step > 0) {
          const float mo = Mrg[row][0], lo = Mrg[row][1];
          const float M = fmaxf(m[r], mo);
          const float fo = (M > -INFINITY) ? fexp2(mo - M) : 0.f;
          const float fs = (M > -INFINITY) ? fexp2(m[r] - M) : 0.f;
          l[r] = lo * fo + l[r] * fs;
#pragma unroll
          for (int d = 0; d < D / 2; ++d)
            acc[r][d] = f2{Mrg[row][2 + 2 * d], Mrg[row][3 + 2 * d]} * fo + acc[r][d] * fs;
          m[r] = M;
        }
        if (step < 3) {
          Mrg[row][0] = m[r];
          Mrg[row][1] = l[r];
#pragma unroll
          for (int d = 0; d < D / 2; ++d) {
            Mrg[row][2 + 2 * d] = acc[r][d].x;
            Mrg[row][3 + 2 * d] = acc[r][d].y;
          }
        } else if (qi[r] < N) {
          // rows with no valid key keep l = 0 (m may be finite from the lazy path: harmless)
          float* P = part + (((int64_t)sp * H + h) * N + qi[r]) * (D + 2);
          P[0] = l[r] > 0.f ? m[r] : -INFINITY;
          P[1] = l[r];
#pragma unroll
          for (int d = 0; d < D / 2; ++d) {
            P[2 + 2 * d] = acc[r][d].x;
            P[3 + 2 * d] = acc[r][d].y;
          }
        }
      }
    }
    __syncthreads();
  }
}

// dQ, v3: QPL query rows per lane; K/V rows as scalar operands.
template <int D, int QPL>
__global__ void __launch_bounds__(256) attn_bwd_dq_v3_kernel(
    const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V, int ld,
    const float* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ delta,
    float* __restrict__ dQ, int lddq, int64_t split_stride, const int* __restrict__ seg_id,
    const int* __restrict__ seg_ptr, int N, int H, int S, float scale) {
  constexpr int U = 4;  // K+V (dQ) or Q+dO+LSE+delta (dK/dV) rows per chunk fit the SGPR file
  __shared__ float Mrg[64 * QPL][D];
  const int h = blockIdx.y, sp = blockIdx.z;
  const int lane = threadIdx.x & 63, w = uniform(threadIdx.x >> 6);
  int qi[QPL], kb[QPL], ke[QPL];
  int bmin = INT_MAX, bmax = 0;
#pragma unroll
  for (int r = 0; r < QPL; ++r) {
    qi[r] = (blockIdx.x * QPL + r) * 64 + lane;
    kb[r] = INT_MAX;
    ke[r] = 0;
    if (qi[r] < N) {
      const int s = seg_id[qi[r]];
      kb[r] = seg_ptr[s];
      ke[r] = seg_ptr[s + 1];
    }
    bmin = min(bmin, kb[r]);
    bmax = max(bmax, ke[r]);
  }
  int cb, ce;
  split_range(uniform(wave_min_i(bmin)), uniform(wave_max_i(bmax)), S, sp, 4 * U, cb, ce);
  const int L4 = ((max(ce - cb, 0) + 4 * U - 1) / (4 * U)) * U;
  const int wb = uniform(cb + w * L4), we = uniform(min(ce, wb + L4));
  int lo_all = wb, hi_all = we;
  int klo[QPL], khi[QPL];
#pragma unroll
  for (int r = 0; r < QPL; ++r) {
    klo[r] = max(kb[r], wb);
    khi[r] = min(ke[r], we);
    if (qi[r] < N) {
      lo_all = max(lo_all, klo[r]);
      hi_all = min(hi_all, khi[r]);
    }
  }
  lo_all = uniform(wave_max_i(lo_all));
  hi_all = uniform(wave_min_i(hi_all));
  const float qs = scale * kLog2e;
  f2 q[QPL][D / 2], go[QPL][D / 2], dq[QPL][D / 2];
  float nl[QPL], nd[QPL];  // -LSE (log2 units), -delta
#pragma unroll
  for (int r = 0; r < QPL; ++r) {
    const bool v = qi[r] < N;
#pragma unroll
    for (int d = 0; d < D / 2; ++d) {
      const int64_t o = (int64_t)qi[r] * ld + h * D + 2 * d;
      const int64_t og = (int64_t)qi[r] * H * D + h * D + 2 * d;
      q[r][d] = v ? f2{Q[o], Q[o + 1]} * qs : splat2(0.f);
      go[r][d] = v ? f2{dO[og], dO[og + 1]} : splat2(0.f);
      dq[r][d] = splat2(0.f);
    }
    nl[r] = v ? -LSE[(int64_t)h * N + qi[r]] * kLog2e : 0.f;
    nd[r] = v ? -delta[(int64_t)h * N + qi[r]] : 0.f;
  }
  for (int j0 = wb; j0 < we; j0 += U) {
    if (j0 >= lo_all && j0 + U <= hi_all) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const f2* kr = reinterpret_cast<const f2*>(K + (int64_t)(j0 + u) * ld + h * D);
        const f2* vr = reinterpret_cast<const f2*>(V + (int64_t)(j0 + u) * ld + h * D);
#pragma unroll
        for (int r = 0; r < QPL; ++r) {
          const float p = fexp2(pdot_init<D>(q[r], kr, nl[r]));
          const f2 ds = splat2(p * pdot_init<D>(go[r], vr, nd[r]));
#pragma unroll
          for (int d = 0; d < D / 2; ++d) dq[r][d] = pfma(ds, kr[d], dq[r][d]);
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = min(j0 + u, we - 1);
        const f2* kr = reinterpret_cast<const f2*>(K + (int64_t)j * ld + h * D);
        const f2* vr = reinterpret_cast<const f2*>(V + (int64_t)j * ld + h * D);
#pragma unroll
        for (int r = 0; r < QPL; ++r) {
          const bool ok = j0 + u >= klo[r] && j0 + u < khi[r];
          const float p = ok ? fexp2(pdot_init<D>(q[r], kr, nl[r])) : 0.f;
          const f2 ds = splat2(p * pdot_init<D>(go[r], vr, nd[r]));
#pragma unroll
          for (int d = 0; d < D / 2; ++d) dq[r][d] = pfma(ds, kr[d], dq[r][d]);
        }
      }
    }
  }
  for (int step = 0; step < 4; ++step) {
    if (w == step) {
#pragma unroll
      for (int r = 0; r < QPL; ++r) {
        const int row = r * 64 + lane;
#pragma unroll
        for (int d = 0; d < D / 2; ++d) {
          const float t0 = (step > 0 ? Mrg[row][2 * d] : 0.f) + dq[r][d].x;
          const float t1 = (step > 0 ? Mrg[row][2 * d + 1] : 0.f) + dq[r][d].y;
          if (step < 3) {
            Mrg[row][2 * d] = t0;
            Mrg[row][2 * d + 1] = t1;
          } else if (qi[r] < N) {
            float* o = dQ + sp * split_stride + (int64_t)qi[r] * lddq + h * D + 2 * d;
            o[0] = t0 * scale;
            o[1] = t1 * scale;
          }
        }
      }
    }
    __syncthreads();
  }
}

// dK, dV, v3: QPL key rows per lane; Q / dO rows and LSE / delta as scalar operands.
template <int D, int QPL>
__global__ void __launch_bounds__(256) attn_bwd_dkv_v3_kernel(
    const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V, int ld,
    const float* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ delta,
    float* __restrict__ dK, float* __restrict__ dV, int lddkv, int64_t split_stride,
    const int* __restrict__ seg_id, const int* __restrict__ seg_ptr, int N, int H, int S, float scale) {
  constexpr int U = 4;  // K+V (dQ) or Q+dO+LSE+delta (dK/dV) rows per chunk fit the SGPR file
  __shared__ float Mrg[64 * QPL][2 * D];
  const int h = blockIdx.y, sp = blockIdx.z;
  const int lane = threadIdx.x & 63, w = uniform(threadIdx.x >> 6);
  int kj[QPL], qb[QPL], qe[QPL];
  int bmin = INT_MAX, bmax = 0;
#pragma unroll
  for (int r = 0; r < QPL; ++r) {
    kj[r] = (blockIdx.x * QPL + r) * 64 + lane;
    qb[r] = INT_MAX;
    qe[r] = 0;
    if (kj[r] < N) {
      const int s = seg_id[kj[r]];
      qb[r] = seg_ptr[s];
      qe[r] = seg_ptr[s + 1];
    }
    bmin = min(bmin, qb[r]);
    bmax = max(bmax, qe[r]);
  }
  int cb, ce;
  split_range(uniform(wave_min_i(bmin)), uniform(wave_max_i(bmax)), S, sp, 4 * U, cb, ce);
  const int L4 = ((max(ce - cb, 0) + 4 * U - 1) / (4 * U)) * U;
  const int wb = uniform(cb + w * L4), we = uniform(min(ce, wb + L4));
  int lo_all = wb, hi_all = we;
  int ilo[QPL], ihi[QPL];
#pragma unroll
  for (int r = 0; r < QPL; ++r) {
    ilo[r] = max(qb[r], wb);
    ihi[r] = min(qe[r], we);
    if (kj[r] < N) {
      lo_all = max(lo_all, ilo[r]);
      hi_all = min(hi_all, ihi[r]);
    }
  }
  lo_all = uniform(wave_max_i(lo_all));
  hi_all = uniform(wave_min_i(hi_all));
  const float ks = scale * kLog2e;
  f2 k[QPL][D / 2], v[QPL][D / 2], dk[QPL][D / 2], dv[QPL][D / 2];
#pragma unroll
  for (int r = 0; r < QPL; ++r) {
    const bool ok = kj[r] < N;
#pragma unroll
    for (int d = 0; d < D / 2; ++d) {
      const int64_t o = (int64_t)kj[r] * ld + h * D + 2 * d;
      k[r][d] = ok ? f2{K[o], K[o + 1]} * ks : splat2(0.f);
      v[r][d] = ok ? f2{V[o], V[o + 1]} : splat2(0.f);
      dk[r][d] = splat2(0.f);
      dv[r][d] = splat2(0.f);
    }
  }
  const float* Lh = LSE + (int64_t)h * N;
  const float* Dh = delta + (int64_t)h * N;
  for (int i0 = wb; i0 < we; i0 += U) {
    if (i0 >= lo_all && i0 + U <= hi_all) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u;
        const f2* qr = reinterpret_cast<const f2*>(Q + (int64_t)i * ld + h * D);
        const f2* gr = reinterpret_cast<const f2*>(dO + (int64_t)i * H * D + h * D);
        const float nl = -Lh[i] * kLog2e, nd = -Dh[i];  // uniform: one op per query per wave
#pragma unroll
        for (int r = 0; r < QPL; ++r) {
          const float p = fexp2(pdot_init<D>(k[r], qr, nl));
          const f2 pp = splat2(p);
          const f2 ds = splat2(p * pdot_init<D>(v[r], gr, nd));
#pragma unroll
          for (int d = 0; d < D / 2; ++d) {
            dv[r][d] = pfma(pp, gr[d], dv[r][d]);
            dk[r][d] = pfma(ds, qr[d], dk[r][d]);
          }
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = min(i0 + u, we - 1);
        const f2* qr = reinterpret_cast<const f2*>(Q + (int64_t)i * ld + h * D);
        const f2* gr = reinterpret_cast<const f2*>(dO + (int64_t)i * H * D + h * D);
        const float nl = -Lh[i] * kLog2e, nd = -Dh[i];
#pragma unroll
        for (int r = 0; r < QPL; ++r) {
          const bool ok = i0 + u >= ilo[r] && i0 + u < ihi[r];
          const float p = ok ? fexp2(pdot_init<D>(k[r], qr, nl)) : 0.f;
          const f2 pp = splat2(p);
          const f2 ds = splat2(p * pdot_init<D>(v[r], gr, nd));
#pragma unroll
          for (int d = 0; d < D / 2; ++d) {
            dv[r][d] = pfma(pp, gr[d], dv[r][d]);
            dk[r][d] = pfma(ds, qr[d], dk[r][d]);
          }
        }
      }
    }
  }
  for (int step = 0; step < 4; ++step) {
    if (w == step) {
#pragma unroll
      for (int r = 0; r < QPL; ++r) {
        const int row = r * 64 + lane;
#pragma unroll
        for (int d = 0; d < D / 2; ++d) {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int c = 2 * d + e;
            const float tk = (step > 0 ? Mrg[row][c] : 0.f) + (e ? dk[r][d].y : dk[r][d].x);
            const float tv = (step > 0 ? Mrg[row][D + c] : 0.f) + (e ? dv[r][d].y : dv[r][d].x);
            if (step < 3) {
              Mrg[row][c] = tk;
              Mrg[row][D + c] = tv;
            } else if (kj[r] < N) {
              dK[sp * split_stride + (int64_t)kj[r] * lddkv + h * D + c] = tk * scale;
              dV[sp * split_stride + (int64_t)kj[r] * lddkv + h * D + c] = tv;
            }
          }
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// MFMA forward (D = 8): QK^T and PV on v_mfma_f32_16x16x32_f16 with two-term fp16 splits.
//
// Every fp32 operand x is carried as hi = f16(x), lo = f16(x - hi) (22 significant bits);
// a product is hi*hi + hi*lo + lo*hi, so scores and outputs keep fp32-level accuracy
// (relative error ~2^-21, vs 2^-24 for fp32 FMA chains) while the dot products run on
// the matrix cores and the VALU only does the softmax bookkeeping (max, exp, sum,
// splitting P).  The VALU-bound sk/v3 kernels spend ~20 VALU instructions per 64 scores
// and are limited by delivering K/V rows; here K/V fragments stream through plain
// coalesced 16 B / 8 B vector loads from pre-split copies (attn_split_kv_kernel, once
// per key instead of once per query tile).
//
// Per wave: 16 queries (the MFMA N dimension) x one key split, 32 keys per step.
//   S^T[key, query] = K' Q'^T: A = K' rows [k_hi | k_lo | k_hi | 0] (K = 32), B = the
//     wave's queries [q_hi; q_hi; q_lo; 0], loop-invariant in registers.  Two MFMAs give
//     lane l the 8 scores of query l&15 for keys 4(l>>4)+i and 16+4(l>>4)+i.
//   O^T[row, query] += V'' P^T: A = V'' (rows 0-7 v_hi dims, 8-15 v_lo dims; the lane's K
//     slots are those same 8 keys, so P^T needs no data movement), B = P_hi, then
//     A = [v_hi; 0] with B = P_lo.  O = rows 0-7 + rows 8-15.
//   P is formed as exp2(s - m + 8) (x256) so its fp16 low part stays normal down to
//   2^-22 of the row max; the partial stores m - 8 (same (m, l, acc) convention as the
//   other kernels, so attn_fwd_combine_kernel merges the splits unchanged).
// The 4 lanes that share a query (lane, lane^16, lane^32, lane^48) agree on the running
// max; it moves lazily (only when a score exceeds it by > 6, then through two xor
// shuffles), so steady-state steps need no cross-lane traffic.  K/V fragments of step
// j+1 are loaded while step j computes.
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef _Float16 h4v __attribute__((ext_vector_type(4)));
typedef float f4m __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split_f16(float x, _Float16& hi, _Float16& lo) {
  x = fminf(fmaxf(x, -65504.f), 65504.f);  // fp16 range (|x| beyond it saturates)
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}

// K' [H][Npad][32] = [k_hi(8) | k_lo(8) | k_hi(8) | 0(8)];  V'' [H][16][Npad] = v_hi rows, v_lo rows.
// Rows j >= N are zero.
// One thread per (key, head): the head's K and V rows are two float4 loads each.
__global__ void __launch_bounds__(256) attn_split_kv_kernel(const float* __restrict__ K, const float* __restrict__ V,
                                                            int ld, int N, int Npad, int H,
                                                            _Float16* __restrict__ Kp, _Float16* __restrict__ Vt) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)H * Npad) return;
  const int j = (int)(t / H), h = (int)(t % H);  // consecutive threads: the heads of one key row
  const bool ok = j < N;
  float kr[8], vr[8];
  if (ok) {
    const float4* k4 = reinterpret_cast<const float4*>(K + (int64_t)j * ld + h * 8);
    const float4* v4 = reinterpret_cast<const float4*>(V + (int64_t)j * ld + h * 8);
    const float4 ka = k4[0], kb = k4[1], va = v4[0], vb = v4[1];
    kr[0] = ka.x; kr[1] = ka.y; kr[2] = ka.z; kr[3] = ka.w; kr[4] = kb.x; kr[5] = kb.y; kr[6] = kb.z; kr[7] = kb.w;
    vr[0] = va.x; vr[1] = va.y; vr[2] = va.z; vr[3] = va.w; vr[4] = vb.x; vr[5] = vb.y; vr[6] = vb.z; vr[7] = vb.w;
  } else {
#pragma unroll
    for (int d = 0; d < 8; ++d) kr[d] = vr[d] = 0.f;
  }
  h8v hi, lo, z;
#pragma unroll
  for (int d = 0; d < 8; ++d) {
    _Float16 a, b;
    split_f16(kr[d], a, b);
    hi[d] = a;
    lo[d] = b;
    z[d] = (_Float16)0.f;
  }
  h8v* kp = reinterpret_cast<h8v*>(Kp + ((int64_t)h * Npad + j) * 32);
  kp[0] = hi;
  kp[1] = lo;
  kp[2] = hi;
  kp[3] = z;
#pragma unroll
  for (int d = 0; d < 8; ++d) {
    _Float16 a, b;
    split_f16(vr[d], a, b);
    Vt[((int64_t)h * 16 + d) * Npad + j] = a;
    Vt[((int64_t)h * 16 + 8 + d) * Npad + j] = b;
  }
}

__global__ void __launch_bounds__(256) attn_fwd_mfma_kernel(const float* __restrict__ Q, int ld,
                                                            const _Float16* __restrict__ Kp,
                                                            const _Float16* __restrict__ Vt, int Npad,
                                                            float* __restrict__ part, const int* __restrict__ seg_id,
                                                            const int* __restrict__ seg_ptr, int N, int H, int S,
                                                            float scale) {
  constexpr int D = 8;
  const int h = blockIdx.y, sp = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int qi = (blockIdx.x * 4 + w) * 16 + c;
  const bool qv = qi < N;
  int kb = INT_MAX, ke = 0;
  if (qv) {
    const int s = seg_id[qi];
    kb = seg_ptr[s];
    ke = seg_ptr[s + 1];
  }
  int cb, ce;
  split_range(uniform(wave_min_i(kb)), uniform(wave_max_i(ke)), S, sp, 32, cb, ce);
  const int lo_all = uniform(wave_max_i(qv ? max(cb, kb) : cb));
  const int hi_all = uniform(wave_min_i(qv ? min(ce, ke) : ce));
  // B operand of S^T: this lane's query, k-slots [q_hi | q_hi | q_lo | 0]
  h8v qb;
  {
    const float qs = scale * kLog2e;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      _Float16 a, b;
      split_f16(qv ? Q[(int64_t)qi * ld + h * D + d] * qs : 0.f, a, b);
      qb[d] = g == 3 ? (_Float16)0.f : (g == 2 ? b : a);
    }
  }
  const _Float16* kh = Kp + (int64_t)h * Npad * 32;
  const _Float16* vh = Vt + ((int64_t)h * 16 + c) * Npad;
  f4m acc = {0.f, 0.f, 0.f, 0.f};
  const f4m zero4 = {0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  constexpr float kOff = 8.f;  // P scaled by 2^8: its fp16 low part stays normal to 2^-22 of the row max
  constexpr float kTau = 6.f;  // lazy max: rescale only when a score exceeds m by > 6 (P' <= 2^14 < fp16 max)
  int j0 = uniform(cb & ~31);
  // software pipeline: the next step's K / V fragments are in flight while this step computes
  h8v a0n, a1n;
  h4v v0n, v1n;
  auto fetch = [&](int j) {
    a0n = *reinterpret_cast<const h8v*>(kh + (int64_t)(j + c) * 32 + 8 * g);
    a1n = *reinterpret_cast<const h8v*>(kh + (int64_t)(j + 16 + c) * 32 + 8 * g);
    v0n = *reinterpret_cast<const h4v*>(vh + j + 4 * g);
    v1n = *reinterpret_cast<const h4v*>(vh + j + 16 + 4 * g);
  };
  if (j0 < ce) fetch(j0);
  for (; j0 < ce; j0 += 32) {
    const h8v a0 = a0n, a1 = a1n;
    const h4v v0 = v0n, v1 = v1n;
    if (j0 + 32 < ce) fetch(j0 + 32);  // rows < Npad: j0 + 63 < roundup(N, 32) + 32
    const f4m s0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, qb, zero4, 0, 0, 0);
    const f4m s1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, qb, zero4, 0, 0, 0);
    float s[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
    if (!(j0 >= lo_all && j0 + 32 <= hi_all)) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int key = j0 + (k < 4 ? 4 * g + k : 16 + 4 * g + k - 4);
        s[k] = (key >= kb && key < ke && key >= cb && key < ce) ? s[k] : -INFINITY;
      }
    }
    float mt = fmaxf(fmaxf(fmaxf(s[0], s[1]), fmaxf(s[2], s[3])), fmaxf(fmaxf(s[4], s[5]), fmaxf(s[6], s[7])));
    // the 4 lanes of a query must agree on m: the max is exchanged (two xor shuffles) only in
    // steps where some lane's local max exceeds its m by more than kTau (wave-uniform branch)
    if (wave_any(mt > m + kTau)) {
      mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float mn = fmaxf(m, mt);
      const float mref = mn > -INFINITY ? mn : 0.f;
      const float alpha = fexp2(m - mref);  // m = -inf -> 0
      l *= alpha;
      acc *= alpha;
      m = mn;
    }
    const float mref = m > -INFINITY ? m : 0.f;
    h8v ph, pl;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float p = fexp2(s[k] - mref + kOff);  // -inf -> 0
      l += p;
      const _Float16 hi = (_Float16)p;
      ph[k] = hi;
      pl[k] = (_Float16)(p - (float)hi);
    }
    const h8v va = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(va, ph, acc, 0, 0, 0);
    const h8v va2 = c < 8 ? va : h8v{};
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(va2, pl, acc, 0, 0, 0);
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] += __shfl_xor(acc[i], 32, 64);  // v_hi rows + v_lo rows
  if (qv && g < 2) {
    float* P = part + (((int64_t)sp * H + h) * N + qi) * (D + 2);
    if (g == 0) {
      P[0] = l > 0.f ? m - kOff : -INFINITY;
      P[1] = l;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) P[2 + 4 * g + i] = acc[i];
  }
}

// dqkv[i, c] = sum_s part[s, i, c]  over the query-split partials (c < F, Sq of them)
// and the key-split partials (c >= F, Sk of them); fixed order, float4 columns.
__global__ void __launch_bounds__(256) attn_bwd_sum_kernel(const float4* __restrict__ pq, int Sq,
                                                           const float4* __restrict__ pkv, int Sk,
                                                           float4* __restrict__ dqkv, int64_t N, int F4) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t tot = N * 3 * F4;
  if (t >= tot) return;
  const int64_t i = t / (3 * F4);
  const int c = (int)(t % (3 * F4));
  float4 a = f4zero();
  if (c < F4) {
    const int64_t st = N * F4;
    for (int s = 0; s < Sq; ++s) a = f4add(a, pq[s * st + i * F4 + c]);
  } else {
    const int64_t st = N * 2 * F4;
    for (int s = 0; s < Sk; ++s) a = f4add(a, pkv[s * st + i * 2 * F4 + (c - F4)]);
  }
  dqkv[t] = a;
}

#define HY_ATTN_DISPATCH(D, ...)                       \
  switch (D) {                                          \
    case 4: { constexpr int kD = 4; __VA_ARGS__; break; }   \
    case 8: { constexpr int kD = 8; __VA_ARGS__; break; }   \
    case 16: { constexpr int kD = 16; __VA_ARGS__; break; } \
    case 32: { constexpr int kD = 32; __VA_ARGS__; break; } \
    case 64: { constexpr int kD = 64; __VA_ARGS__; break; } \
    default: HY_CHECK(false, "attention head_dim must be one of 4,8,16,32,64, got ", D); \
  }

// HYDRA_ATTN_LDS=1 selects the LDS-staged kernels for every head size (A/B testing).
static bool attn_scalar_path() {
  static const bool v = [] {
    const char* e = std::getenv("HYDRA_ATTN_LDS");
    return !(e && e[0] == '1');
  }();
  return v;
}

static bool attn_scalar_bwd() {
  static const bool v = [] {
    const char* e = std::getenv("HYDRA_ATTN_SCALAR_BWD");
    return e && e[0] == '1';
  }();
  return v;
}

static int attn_keytile(int D) { return D <= 8 ? 64 : (D <= 16 ? 32 : 16); }

// v3 kernels (D <= 16) are opt-in (HYDRA_ATTN_V3=1).  Measured on MI355X at the OC20
// shape (N 2311, H 8, D 8, standalone, auto splits): fwd 46.7 us (QPL 1) / 45.2 (QPL 2) vs
// 48.3 for the sk forward; bwd 154 / 142 vs 115 for the LDS backward; headline step 2.33 /
// 2.07 vs 1.95 ms.  Cutting VALU instructions ~40% barely moved the forward: these kernels
// are bound by delivering K/V rows (scalar loads), not by VALU issue.
// HYDRA_ATTN_QPL = rows per lane of the v3 kernels (1 or 2, default 2).
static bool attn_v3(int D) {
  static const bool v = [] {
    const char* e = std::getenv("HYDRA_ATTN_V3");
    return e && e[0] == '1';
  }();
  return v && D <= 16;
}
// MFMA forward (D = 8) is opt-in (HYDRA_ATTN_MFMA=1).  Measured on MI355X at the OC20
// shape (N 2311, H 8, standalone, rocprofv3): the MFMA kernel itself takes 35 us at 3-6
// key splits (50 us at 1) plus 5 us for the K/V split pass and 5 us for the combine,
// against 34-42 us for the whole VALU sk forward; headline step 2.02 vs 2.01 ms.  At
// D = 8 the matrix work per score is tiny and the VALU still carries the softmax and
// the fp16 splitting of P, so the matrix cores do not pay for the extra passes.
static bool attn_mfma() {
  static const bool v = [] {
    const char* e = std::getenv("HYDRA_ATTN_MFMA");
    return e && e[0] == '1';
  }();
  return v;
}
static int attn_qpl(int D) {
  static const int v = [] {
    const char* e = std::getenv("HYDRA_ATTN_QPL");
    return (e && e[0] == '1') ? 1 : 2;
  }();
  return attn_v3(D) ? v : 1;
}

// Number of key (or query) splits: ~3 workgroups per CU, but never less than two 4-wave
// tiles per split.
// max_span: host bound on the longest attention segment (N for batch scope).
static int attn_splits(int64_t N, int64_t H, int D, int64_t max_span, int64_t split_override) {
  if (split_override > 0) return (int)split_override;
  const int64_t blocks = (int64_t)ceil_div(N, 64 * attn_qpl(D)) * H;
  // ~3 workgroups per CU: the GPS layer runs attention concurrently with the local MPNN on
  // a second stream, and a grid that fills the chip alone (the round-1 target of 1536
  // workgroups, S = 5 for the OC20 shape) starves that branch; measured on MI355X the
  // headline step is 4% faster at S = 3 than at S = 5 (and slower at S = 2, 8, 12, 16)
  const int64_t want = std::max<int64_t>(1, (768 + blocks - 1) / blocks);
  const int64_t per = 2 * 4 * attn_keytile(D);
  const int64_t cap = std::max<int64_t>(1, (max_span + 64 + per - 1) / per);
  return (int)std::min<int64_t>(std::min(want, cap), 32);
}

// qkv: [N, 3*H*D] packed rows (q | k | v), as produced by the in-projection.
std::tuple<at::Tensor, at::Tensor> attn_fwd(const at::Tensor& qkv, const at::Tensor& seg_id,
                                            const at::Tensor& seg_ptr, int64_t H, double scale, int64_t max_span,
                                            int64_t splits) {
  HY_CHECK_CUDA(qkv);
  HY_CHECK_F32(qkv);
  HY_CHECK(qkv.stride(1) == 1, "qkv rows must be contiguous");
  HY_CHECK_I32(seg_id);
  HY_CHECK_I32(seg_ptr);
  const int64_t N = qkv.size(0);
  const int64_t F = qkv.size(1) / 3;
  const int D = (int)(F / H);
  HY_CHECK(D * H == F, "hidden must be divisible by heads");
  HY_CHECK(seg_id.numel() == N, "seg_id must have one entry per row");
  auto O = at::empty({N, F}, qkv.options());
  auto LSE = at::empty({H, N}, qkv.options());
  if (N == 0) return {O, LSE};
  const int ld = (int)qkv.stride(0);
  const float* base = qkv.data_ptr<float>();
  const int S = attn_splits(N, H, D, max_span > 0 ? max_span : N, splits);
  auto part = at::empty({(int64_t)S * H * N * (D + 2)}, qkv.options());
  dim3 grid(ceil_div(N, 64 * attn_qpl(D)), H, S);
  HY_ATTN_DISPATCH(D, {
    bool done = false;
    if constexpr (kD == 8) {
      if (attn_mfma() && ld % 4 == 0 && reinterpret_cast<uintptr_t>(base) % 16 == 0) {
        const int64_t Npad = (N + 31) / 32 * 32 + 32;
        auto hopt = qkv.options().dtype(at::kHalf);
        auto Kp = at::empty({H * Npad * 32}, hopt);
        auto Vt = at::empty({H * 16 * Npad}, hopt);
        auto* kp = reinterpret_cast<_Float16*>(Kp.data_ptr<at::Half>());
        auto* vt = reinterpret_cast<_Float16*>(Vt.data_ptr<at::Half>());
        attn_split_kv_kernel<<<ceil_div(H * Npad, 256), 256, 0, stream()>>>(base + F, base + 2 * F, ld, (int)N,
                                                                            (int)Npad, (int)H, kp, vt);
        attn_fwd_mfma_kernel<<<dim3(ceil_div(N, 64), H, S), 256, 0, stream()>>>(
            base, ld, kp, vt, (int)Npad, part.data_ptr<float>(), seg_id.data_ptr<int>(), seg_ptr.data_ptr<int>(),
            (int)N, (int)H, S, (float)scale);
        done = true;
      }
    }
    if constexpr (kD <= 16) {
      if (!done && attn_v3(kD)) {
        auto kern = attn_qpl(kD) == 2 ? attn_fwd_v3_kernel<kD, 2> : attn_fwd_v3_kernel<kD, 1>;
        kern<<<grid, 256, 0, stream()>>>(base, base + F, base + 2 * F, ld, part.data_ptr<float>(),
                                         seg_id.data_ptr<int>(), seg_ptr.data_ptr<int>(), (int)N, (int)H, S,
                                         (float)scale);
        done = true;
      }
    }
    if (done) {
    } else if (kD <= 16 && attn_scalar_path())
      attn_fwd_sk_kernel<kD><<<grid, 256, 0, stream()>>>(base, base + F, base + 2 * F, ld, part.data_ptr<float>(),
                                                         seg_id.data_ptr<int>(), seg_ptr.data_ptr<int>(), (int)N,
                                                         (int)H, S, (float)scale);
    else
      attn_fwd_kernel<kD><<<grid, 256, 0, stream()>>>(base, base + F, base + 2 * F, ld, part.data_ptr<float>(),
                                                      seg_id.data_ptr<int>(), seg_ptr.data_ptr<int>(), (int)N, (int)H,
                                                      S, (float)scale);
    attn_fwd_combine_kernel<kD><<<ceil_div(N * H, 256), 256, 0, stream()>>>(
        part.data_ptr<float>(), O.data_ptr<float>(), LSE.data_ptr<float>(), (int)N, (int)H, S);
  });
  return {O, LSE};
}

// kernel selection for the backward: scalar-operand kernels for D <= 16
// (measured on MI355X, N=2560, H=8, D=8: the scalar-operand backward is slower —
// 184 vs 130 us — so it is opt-in via HYDRA_ATTN_SCALAR_BWD=1; the forward gains ~10%)
template <int D>
static decltype(&attn_bwd_dq_kernel<D>) pick_dq() {
  if constexpr (D <= 16) {
    if (attn_v3(D)) return attn_qpl(D) == 2 ? attn_bwd_dq_v3_kernel<D, 2> : attn_bwd_dq_v3_kernel<D, 1>;
  }
  return D <= 16 && attn_scalar_bwd() ? attn_bwd_dq_sk_kernel<D> : attn_bwd_dq_kernel<D>;
}
template <int D>
static decltype(&attn_bwd_dkv_kernel<D>) pick_dkv() {
  if constexpr (D <= 16) {
    if (attn_v3(D)) return attn_qpl(D) == 2 ? attn_bwd_dkv_v3_kernel<D, 2> : attn_bwd_dkv_v3_kernel<D, 1>;
  }
  return D <= 16 && attn_scalar_bwd() ? attn_bwd_dkv_sk_kernel<D> : attn_bwd_dkv_kernel<D>;
}
#define HY_DQ(kD) pick_dq<kD>()<<<grid, 256, 0, stream()>>>
#define HY_DKV(kD) pick_dkv<kD>()<<<grid, 256, 0, stream()>>>

at::Tensor attn_bwd(const at::Tensor& dO_, const at::Tensor& qkv, const at::Tensor& O, const at::Tensor& LSE,
                    const at::Tensor& seg_id, const at::Tensor& seg_ptr, int64_t H, double scale, int64_t max_span,
                    int64_t splits) {
  auto dO = dO_.contiguous();
  HY_CHECK_CUDA(dO);
  const int64_t N = qkv.size(0);
  const int64_t F = qkv.size(1) / 3;
  const int D = (int)(F / H);
  auto dqkv = at::empty({N, 3 * F}, qkv.options());
  if (N == 0) return dqkv;
  auto delta = at::empty({H, N}, qkv.options());
  attn_delta_kernel<<<ceil_div(N * H, 256), 256, 0, stream()>>>(dO.data_ptr<float>(), O.data_ptr<float>(),
                                                                 delta.data_ptr<float>(), (int)N, (int)H, D);
  const int ld = (int)qkv.stride(0);
  const float* base = qkv.data_ptr<float>();
  float* dbase = dqkv.data_ptr<float>();
  const int S = attn_splits(N, H, D, max_span > 0 ? max_span : N, splits);
  dim3 grid(ceil_div(N, 64 * attn_qpl(D)), H, S);
  if (S == 1) {
    HY_ATTN_DISPATCH(D, {
      HY_DQ(kD)(
          base, base + F, base + 2 * F, ld, dO.data_ptr<float>(), LSE.data_ptr<float>(), delta.data_ptr<float>(),
          dbase, (int)(3 * F), 0, seg_id.data_ptr<int>(), seg_ptr.data_ptr<int>(), (int)N, (int)H, 1, (float)scale);
      HY_DKV(kD)(
          base, base + F, base + 2 * F, ld, dO.data_ptr<float>(), LSE.data_ptr<float>(), delta.data_ptr<float>(),
          dbase + F, dbase + 2 * F, (int)(3 * F), 0, seg_id.data_ptr<int>(), seg_ptr.data_ptr<int>(), (int)N,
          (int)H, 1, (float)scale);
    });
    return dqkv;
  }
  auto pq = at::empty({(int64_t)S * N * F}, qkv.options());
  auto pkv = at::empty({(int64_t)S * N * 2 * F}, qkv.options());
  HY_ATTN_DISPATCH(D, {
    HY_DQ(kD)(
        base, base + F, base + 2 * F, ld, dO.data_ptr<float>(), LSE.data_ptr<float>(), delta.data_ptr<float>(),
        pq.data_ptr<float>(), (int)F, N * F, seg_id.data_ptr<int>(), seg_ptr.data_ptr<int>(), (int)N, (int)H, S,
        (float)scale);
    HY_DKV(kD)(
        base, base + F, base + 2 * F, ld, dO.data_ptr<float>(), LSE.data_ptr<float>(), delta.data_ptr<float>(),
        pkv.data_ptr<float>(), pkv.data_ptr<float>() + F, (int)(2 * F), N * 2 * F, seg_id.data_ptr<int>(),
        seg_ptr.data_ptr<int>(), (int)N, (int)H, S, (float)scale);
  });
  const int F4 = (int)(F / 4);
  HY_CHECK(F % 4 == 0, "attention hidden must be a multiple of 4");
  attn_bwd_sum_kernel<<<ceil_div(N * 3 * F4, 256), 256, 0, stream()>>>(
      reinterpret_cast<const float4*>(pq.data_ptr<float>()), S, reinterpret_cast<const float4*>(pkv.data_ptr<float>()),
      S, reinterpret_cast<float4*>(dbase), N, F4);
  return dqkv;
}

// ---- split backward: the dQ pass and the dK/dV pass as separate ops, so the caller can
// run them on two streams (they only share read-only inputs); attn_bwd_combine sums the
// split partials (or concatenates the S == 1 outputs) into dqkv.
at::Tensor attn_bwd_delta(const at::Tensor& dO_, const at::Tensor& O, int64_t H) {
  auto dO = dO_.contiguous();
  HY_CHECK_CUDA(dO);
  const int64_t N = O.size(0);
  const int D = (int)(O.size(1) / H);
  auto delta = at::empty({H, N}, O.options());
  if (N > 0)
    attn_delta_kernel<<<ceil_div(N * H, 256), 256, 0, stream()>>>(dO.data_ptr<float>(), O.data_ptr<float>(),
                                                                   delta.data_ptr<float>(), (int)N, (int)H, D);
  return delta;
}

// which = 0: dQ partials [S, N, F]; which = 1: dK|dV partials [S, N, 2F]
at::Tensor attn_bwd_part(const at::Tensor& dO_, const at::Tensor& qkv, const at::Tensor& LSE, const at::Tensor& delta,
                         const at::Tensor& seg_id, const at::Tensor& seg_ptr, int64_t H, double scale,
                         int64_t max_span, int64_t splits, int64_t which) {
  auto dO = dO_.contiguous();
  HY_CHECK_CUDA(dO);
  const int64_t N = qkv.size(0);
  const int64_t F = qkv.size(1) / 3;
  const int D = (int)(F / H);
  const int ld = (int)qkv.stride(0);
  const float* base = qkv.data_ptr<float>();
  const int S = attn_splits(N, H, D, max_span > 0 ? max_span : N, splits);
  dim3 grid(ceil_div(N, 64 * attn_qpl(D)), H, S);
  if (which == 0) {
    auto pq = at::empty({(int64_t)S, N, F}, qkv.options());
    if (N > 0)
      HY_ATTN_DISPATCH(D, {
        HY_DQ(kD)(base, base + F, base + 2 * F, ld, dO.data_ptr<float>(), LSE.data_ptr<float>(),
                  delta.data_ptr<float>(), pq.data_ptr<float>(), (int)F, N * F, seg_id.data_ptr<int>(),
                  seg_ptr.data_ptr<int>(), (int)N, (int)H, S, (float)scale);
      });
    return pq;
  }
  auto pkv = at::empty({(int64_t)S, N, 2 * F}, qkv.options());
  if (N > 0)
    HY_ATTN_DISPATCH(D, {
      HY_DKV(kD)(base, base + F, base + 2 * F, ld, dO.data_ptr<float>(), LSE.data_ptr<float>(),
                 delta.data_ptr<float>(), pkv.data_ptr<float>(), pkv.data_ptr<float>() + F, (int)(2 * F), N * 2 * F,
                 seg_id.data_ptr<int>(), seg_ptr.data_ptr<int>(), (int)N, (int)H, S, (float)scale);
    });
  return pkv;
}

at::Tensor attn_bwd_combine(const at::Tensor& pq, const at::Tensor& pkv) {
  HY_CHECK(pq.dim() == 3 && pkv.dim() == 3 && pq.size(1) == pkv.size(1) && pkv.size(2) == 2 * pq.size(2),
           "attn_bwd_combine: partial shapes");
  const int64_t N = pq.size(1), F = pq.size(2);
  HY_CHECK(F % 4 == 0, "attention hidden must be a multiple of 4");
  auto dqkv = at::empty({N, 3 * F}, pq.options());
  const int F4 = (int)(F / 4);
  if (N > 0)
    attn_bwd_sum_kernel<<<ceil_div(N * 3 * F4, 256), 256, 0, stream()>>>(
        reinterpret_cast<const float4*>(pq.data_ptr<float>()), (int)pq.size(0),
        reinterpret_cast<const float4*>(pkv.data_ptr<float>()), (int)pkv.size(0),
        reinterpret_cast<float4*>(dqkv.data_ptr<float>()), N, F4);
  return dqkv;
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("attn_bwd_delta(Tensor dO, Tensor O, int H) -> Tensor");
  m.def(
      "attn_bwd_part(Tensor dO, Tensor qkv, Tensor LSE, Tensor delta, Tensor seg_id, Tensor seg_ptr, int H, "
      "float scale, int max_span, int splits, int which) -> Tensor");
  m.def("attn_bwd_combine(Tensor pq, Tensor pkv) -> Tensor");
  m.def(
      "attn_fwd(Tensor qkv, Tensor seg_id, Tensor seg_ptr, int H, float scale, int max_span, int splits) "
      "-> (Tensor, Tensor)");
  m.def(
      "attn_bwd(Tensor dO, Tensor qkv, Tensor O, Tensor LSE, Tensor seg_id, Tensor seg_ptr, int H, float scale, "
      "int max_span, int splits) -> Tensor");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("attn_bwd_delta", hy::attn_bwd_delta);
  m.impl("attn_bwd_part", hy::attn_bwd_part);
  m.impl("attn_bwd_combine", hy::attn_bwd_combine);
  m.impl("attn_fwd", hy::attn_fwd);
  m.impl("attn_bwd", hy::attn_bwd);
}
