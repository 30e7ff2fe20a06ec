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

// The forward uses the scalar-operand (sk) kernel for D <= 16 and the LDS-staged kernel for
// wider heads; the backward uses the LDS-staged dQ / dK,dV kernels for every D.  (Measured
// on MI355X at the OC20 shape, N 2311, H 8, D 8: the sk forward beat the LDS forward by
// ~10%, while an sk backward was slower, 184 vs 130 us; a later "v3" VALU-trimmed variant
// and an fp16-split MFMA forward lost their A/B against these and were removed -- the
// 8-wide-head MFMA path that won is csrc/attention8.hip.)
static int attn_keytile(int D) { return D <= 8 ? 64 : (D <= 16 ? 32 : 16); }

// Number of key (or query) splits: ~3 workgroups per CU, but never less than two 4-wave
// tiles per split.
// max_span: host bound on the longest attention segment (N for batch scope).
static int attn_splits(int64_t N, int64_t H, int D, int64_t max_span, int64_t split_override) {
  if (split_override > 0) return (int)split_override;
  const int64_t blocks = (int64_t)ceil_div(N, 64) * H;
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
  dim3 grid(ceil_div(N, 64), H, S);
  HY_ATTN_DISPATCH(D, {
    if (kD <= 16)
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

#define HY_DQ(kD) attn_bwd_dq_kernel<kD><<<grid, 256, 0, stream()>>>
#define HY_DKV(kD) attn_bwd_dkv_kernel<kD><<<grid, 256, 0, stream()>>>

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
  dim3 grid(ceil_div(N, 64), H, S);
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
  dim3 grid(ceil_div(N, 64), H, S);
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
