// GPS multi-head attention for 8-wide heads (hidden 64 / 8 heads, the OC20 headline
// config) on the fp32 matrix cores of gfx950 (v_mfma_f32_16x16x4_f32: exact fp32, the
// reference's precision).
//
// Reference: hydragnn/globalAtt/gps.py:126-133 (torch.nn.MultiheadAttention over all
// nodes of the batch, key-padding mask) — generalised to a partition of the tokens into
// segments (seg_ptr / seg_id), as csrc/attention.hip.
//
// Design (one wave = 16 query (or key) rows of one head, all in MFMA tiles):
//   forward   S^T = K Q^T        (2 MFMAs per 16x16 tile, D = 8 = 2 k-steps)
//             online softmax over the key index (4 registers x 4 lane groups)
//             O^T += Vx^T P^T    (4 MFMAs; Vx = [V | 1 | 0]: row 8 of O^T is the row sum l)
//   dQ pass   S^T, dP^T = V dO^T (2 + 2), dS^T = P^T (dP^T - delta), dQ^T += K^T dS^T (4)
//   dK/dV     S = Q K^T, dP = dO V^T (2 + 2), dV^T += dO^T P, dK^T += Q^T dS (4 + 4)
// so the softmax and masking are the only VALU work; the score/probability tiles never
// leave registers (each MFMA's accumulator layout is the next MFMA's B operand).
// Scores carry scale * log2(e) folded into Q (forward, dQ) or K (dK/dV) so exp2 is one
// v_exp_f32; LSE2 = m + log2(l) is stored in the same units.
//
// Operand layouts (written by the producer of Q/K/V, csrc/gps_fused.hip node_fwd, or by
// attn8_pack): for head h and row n (rows padded to Nq = 16k, padding zero)
//   "pair" [H][Nq][8], element d at 2 (d % 4) + d / 4: lane group g reads (d=g, d=g+4)
//          as one float2 — the A/B fragments of the two k-steps of a D = 8 product;
//   "quad" [H][Nq/4][8][4], element (n, d) at ((n/4) 8 + d) 4 + n % 4: lane (i, g) reads
//          rows 4g..4g+3 of column d = i as one float4 — the A fragment of a product
//          summed over 16 rows.
#include "common.h"
#include "pna_body.h"

#include <cstdio>
#include <cstdlib>
#include <type_traits>

namespace hy {
namespace a8 {

typedef float f4v __attribute__((ext_vector_type(4)));
constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ f4v mfma(float a, float b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f4v f4z() { return f4v{0.f, 0.f, 0.f, 0.f}; }
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ int pair_pos(int d) { return 2 * (d & 3) + (d >> 2); }
__device__ __forceinline__ int64_t pair_idx(int h, int Nq, int n, int d) {
  return ((int64_t)h * Nq + n) * 8 + pair_pos(d);
}
__device__ __forceinline__ int64_t quad_idx(int h, int Nq, int n, int d) {
  return (((int64_t)h * (Nq >> 2) + (n >> 2)) * 8 + d) * 4 + (n & 3);
}

__device__ __forceinline__ float2 ld2(const float* p) { return *reinterpret_cast<const float2*>(p); }
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

__device__ __forceinline__ float wmin16(float v) {
  v = fminf(v, __shfl_xor(v, 16, 64));
  return fminf(v, __shfl_xor(v, 32, 64));
}
__device__ __forceinline__ float wmax16(float v) {
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  return fmaxf(v, __shfl_xor(v, 32, 64));
}
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
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// ------------------------------------------------------------------------------------ fwd
// grid (ceil(N/64), H, S); wave w: queries 64 bx + 16 w + i.
// part: [S][H][N][10] = (m, l, o[8]) in log2 units (S > 1); else O [N, 8H] and LSE2 [H][Nq]
// (rows N..Nq of LSE2 are written 0 so the key-major backward reads whole float4 groups).
//
// Two passes over the split's keys inside the kernel: (1) S^T tiles only -> the exact
// per-query max m (lane-local running max, ONE cross-lane fold at the end), (2) S^T with
// the accumulator initialised to -m (the MFMA emits s - m directly), p = exp2, O^T += Vx^T P^T.
// No online rescaling and no cross-lane traffic in the loops: the VALU work per 16x16 tile
// is 4 v_exp_f32.  Operands of tile t+2 are loaded while tile t computes (register ring),
// since each tile's MFMAs depend on its loads (L1/L2 latency >> one tile of MFMA work).
struct KV8 {
  float2 k;   // K pair fragment of row k0 + i
  float4 v;   // Vx quad fragment (V rows k0 + 4g .. +3, column i; 1 at i = 8)
};

__device__ __forceinline__ KV8 ld_kv(const float* __restrict__ Kp, const float* __restrict__ Vq, int h, int Nq, int k0,
                                     int i, int g, float vone) {
  KV8 t;
  const int kc = min(k0, Nq - 16);  // prefetches past the split stay in bounds
  t.k = ld2(Kp + ((int64_t)h * Nq + kc + i) * 8 + 2 * g);
  // branch-free (a load under an exec branch makes the compiler drain vmcnt there)
  const float4 v = ld4(Vq + (((int64_t)h * (Nq >> 2) + (kc >> 2) + g) * 8 + (i & 7)) * 4);
  t.v = i < 8 ? v : make_float4(vone, vone, vone, vone);
  return t;
}

template <int RT>
__global__ void __launch_bounds__(256) attn8_fwd_kernel(const float* __restrict__ Qp, const float* __restrict__ Kp,
                                                        const float* __restrict__ Vq, int N, int Nq, int H,
                                                        const int* __restrict__ seg_id,
                                                        const int* __restrict__ seg_ptr, int S, float qscale,
                                                        float* __restrict__ part, float* __restrict__ O,
                                                        float* __restrict__ LSE2) {
  // RT row tiles (16 queries each) per wave: every K/V fragment feeds RT independent chains
  const int h = blockIdx.y, sp_ = blockIdx.z;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int qbase = blockIdx.x * 64 * RT + 16 * RT * w;
  int q[RT], sb[RT], se[RT];
  float bq0[RT], bq1[RT];
  int lo = N, hi = 0, ilo = 0, ihi = N;
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    q[t] = qbase + 16 * t + i;
    sb[t] = N;
    se[t] = 0;
    if (q[t] < N) {
      const int sg = seg_id[q[t]];
      sb[t] = seg_ptr[sg];
      se[t] = seg_ptr[sg + 1];
    }
    lo = min(lo, sb[t]);
    hi = max(hi, se[t]);
    ilo = max(ilo, q[t] < N ? sb[t] : 0);
    ihi = min(ihi, q[t] < N ? se[t] : N);
    const float2 bq = ld2(Qp + ((int64_t)h * Nq + min(q[t], Nq - 1)) * 8 + 2 * g);
    bq0[t] = bq.x * qscale;
    bq1[t] = bq.y * qscale;
  }
  lo = uni(wave_min_i(lo)) & ~15;
  hi = uni(wave_max_i(hi));
  ilo = uni(wave_max_i(ilo));
  ihi = uni(wave_min_i(ihi));
  const int L = max(hi - lo, 0);
  const int C = (((L + S - 1) / S) + 15) / 16 * 16;
  const int cb = uni(min(lo + sp_ * C, max(hi, lo))), ce = uni(min(hi, cb + C));
  const float vone = (i == 8) ? 1.f : 0.f;
  auto full_tile = [&](int k0) { return k0 >= ilo && k0 + 16 <= ihi && k0 + 16 <= ce; };
  // pass 1: row max
  float m[RT];
  {
    float mx[RT][4];
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) mx[t][r] = -INFINITY;
    float2 k0r = ld2(Kp + ((int64_t)h * Nq + min(cb, Nq - 16) + i) * 8 + 2 * g);
    float2 k1r = ld2(Kp + ((int64_t)h * Nq + min(cb + 16, Nq - 16) + i) * 8 + 2 * g);
    for (int k0 = cb; k0 < ce; k0 += 16) {
      const float2 kn = ld2(Kp + ((int64_t)h * Nq + min(k0 + 32, Nq - 16) + i) * 8 + 2 * g);
      const bool full = full_tile(k0);
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        f4v s = mfma(k0r.x, bq0[t], f4z());
        s = mfma(k0r.y, bq1[t], s);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + 4 * g + r;
          const bool ok = full || (key >= sb[t] && key < se[t] && key < ce);
          mx[t][r] = fmaxf(mx[t][r], ok ? s[r] : -INFINITY);
        }
      }
      k0r = k1r;
      k1r = kn;
    }
#pragma unroll
    for (int t = 0; t < RT; ++t) m[t] = wmax16(fmaxf(fmaxf(mx[t][0], mx[t][1]), fmaxf(mx[t][2], mx[t][3])));
  }
  // pass 2: p = exp2(s - m), O^T += Vx^T P^T (row 8 of O^T = l); control flow stays
  // wave-uniform (every lane supplies A-operand rows of V; dead queries are fully masked)
  f4v o[RT];
  float negm[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    o[t] = f4z();
    negm[t] = m[t] > -INFINITY ? -m[t] : 0.f;
  }
  {
    KV8 t0 = ld_kv(Kp, Vq, h, Nq, cb, i, g, vone);
    KV8 t1 = ld_kv(Kp, Vq, h, Nq, cb + 16, i, g, vone);
    for (int k0 = cb; k0 < ce; k0 += 16) {
      const KV8 tn = ld_kv(Kp, Vq, h, Nq, k0 + 32, i, g, vone);
      const bool full = full_tile(k0);
      f4v s[RT];
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        s[t] = mfma(t0.k.x, bq0[t], f4v{negm[t], negm[t], negm[t], negm[t]});
        s[t] = mfma(t0.k.y, bq1[t], s[t]);
      }
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        float p[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + 4 * g + r;
          const bool ok = full || (key >= sb[t] && key < se[t] && key < ce);
          p[r] = ok ? fexp2(s[t][r]) : 0.f;
        }
        o[t] = mfma(t0.v.x, p[0], o[t]);
        o[t] = mfma(t0.v.y, p[1], o[t]);
        o[t] = mfma(t0.v.z, p[2], o[t]);
        o[t] = mfma(t0.v.w, p[3], o[t]);
      }
      t0 = t1;
      t1 = tn;
    }
  }
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    // o: lane (i, g) rows 4g + r of O^T for query i: g = 0, 1 -> d 0..7, g = 2, r = 0 -> l
    const float l = __shfl(o[t][0], 32 + i, 64);
    const int qq = q[t];
    if (qq >= N) {
      if (S == 1 && g == 2 && qq < Nq) LSE2[(int64_t)h * Nq + qq] = 0.f;
      continue;
    }
    if (S == 1) {
      if (g < 2) {
        const float inv = l > 0.f ? 1.f / l : 0.f;
        float4 v = make_float4(o[t][0] * inv, o[t][1] * inv, o[t][2] * inv, o[t][3] * inv);
        *reinterpret_cast<float4*>(O + (int64_t)qq * 8 * H + h * 8 + 4 * g) = v;
      } else if (g == 2) {
        LSE2[(int64_t)h * Nq + qq] = l > 0.f ? m[t] + __log2f(l) : -INFINITY;
      }
      continue;
    }
    float* P = part + (((int64_t)sp_ * H + h) * N + qq) * 10;
    if (g < 2) {
      *reinterpret_cast<float4*>(P + 2 + 4 * g) = make_float4(o[t][0], o[t][1], o[t][2], o[t][3]);
    } else if (g == 2) {
      P[0] = m[t] > -INFINITY ? m[t] : -INFINITY;
      P[1] = l;
    }
  }
}

// merge the S split partials of every (head, query) in a fixed order
__global__ void __launch_bounds__(256) attn8_combine_kernel(const float* __restrict__ part, float* __restrict__ O,
                                                            float* __restrict__ LSE2, int N, int Nq, int H, int S) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)Nq * H) return;
  const int q = (int)(t / H), h = (int)(t % H);
  if (q >= N) {
    LSE2[(int64_t)h * Nq + q] = 0.f;
    return;
  }
  const int64_t ss = (int64_t)H * N * 10;
  const float* P = part + ((int64_t)h * N + q) * 10;
  float M = -INFINITY;
  for (int s = 0; s < S; ++s) M = fmaxf(M, P[s * ss]);
  float l = 0.f, acc[8];
#pragma unroll
  for (int d = 0; d < 8; ++d) acc[d] = 0.f;
  if (M > -INFINITY) {
    for (int s = 0; s < S; ++s) {
      const float* p = P + s * ss;
      const float f = fexp2(p[0] - M);
      l = fmaf(p[1], f, l);
#pragma unroll
      for (int d = 0; d < 8; ++d) acc[d] = fmaf(p[2 + d], f, acc[d]);
    }
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
  float* o = O + (int64_t)q * 8 * H + h * 8;
  *reinterpret_cast<float4*>(o) = make_float4(acc[0] * inv, acc[1] * inv, acc[2] * inv, acc[3] * inv);
  *reinterpret_cast<float4*>(o + 4) = make_float4(acc[4] * inv, acc[5] * inv, acc[6] * inv, acc[7] * inv);
  LSE2[(int64_t)h * Nq + q] = l > 0.f ? M + __log2f(l) : -INFINITY;
}

// ------------------------------------------------------------------------------------ bwd
// dQ pass: grid (ceil(N/64), H, S over keys).  Output dQ (x scale) rows at
// out + s * sstride + q * ldo + h * 8.  The S^T accumulator starts at -LSE2 (p = exp2(acc)),
// the dP^T accumulator at -delta (dS = p * acc); operands two tiles ahead are in flight.
struct DQ8 {
  float2 k, v;
  float4 kt;
};

__device__ __forceinline__ DQ8 ld_dq(const float* __restrict__ Kp, const float* __restrict__ Kq,
                                     const float* __restrict__ Vp, int h, int Nq, int k0, int i, int g) {
  DQ8 t;
  const int kc = min(k0, Nq - 16);
  t.k = ld2(Kp + ((int64_t)h * Nq + kc + i) * 8 + 2 * g);
  t.v = ld2(Vp + ((int64_t)h * Nq + kc + i) * 8 + 2 * g);
  // lanes i >= 8 load a duplicate column: rows 8..15 of dQ^T are junk and never stored
  // (branch- and select-free: either makes the compiler wait for the load right away)
  t.kt = ld4(Kq + (((int64_t)h * (Nq >> 2) + (kc >> 2) + g) * 8 + (i & 7)) * 4);
  return t;
}

// Span of RT row tiles of a wave (rows base + 16 t + i): per-row segments, wave union /
// intersection, split range (as span_of)
template <int RT>
struct SpanR {
  int b[RT], e[RT], row[RT];
  int ilo, ihi, cb, ce;
};

template <int RT>
__device__ __forceinline__ SpanR<RT> span_rt(int base, int i, int N, const int* seg_id, const int* seg_ptr, int S,
                                              int s) {
  SpanR<RT> sp;
  int lo = N, hi = 0, ilo = 0, ihi = N;
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const int r = base + 16 * t + i;
    sp.row[t] = r;
    sp.b[t] = N;
    sp.e[t] = 0;
    if (r < N) {
      const int sg = seg_id[r];
      sp.b[t] = seg_ptr[sg];
      sp.e[t] = seg_ptr[sg + 1];
    }
    lo = min(lo, sp.b[t]);
    hi = max(hi, sp.e[t]);
    ilo = max(ilo, r < N ? sp.b[t] : 0);
    ihi = min(ihi, r < N ? sp.e[t] : N);
  }
  lo = uni(wave_min_i(lo)) & ~15;
  hi = uni(wave_max_i(hi));
  sp.ilo = uni(wave_max_i(ilo));
  sp.ihi = uni(wave_min_i(ihi));
  const int L = max(hi - lo, 0);
  const int C = (((L + S - 1) / S) + 15) / 16 * 16;
  sp.cb = uni(min(lo + s * C, max(hi, lo)));
  sp.ce = uni(min(hi, sp.cb + C));
  return sp;
}

template <int RT>
__device__ __forceinline__ void attn8_bwd_dq_body(int bx, 
    const float* __restrict__ Qp, const float* __restrict__ Kp, const float* __restrict__ Kq,
    const float* __restrict__ Vp, const float* __restrict__ dOp, const float* __restrict__ LSE2,
    const float* __restrict__ delta, int N, int Nq, int H, const int* __restrict__ seg_id,
    const int* __restrict__ seg_ptr, int S, float scale, float qscale, float* __restrict__ out, int ldo,
    int64_t sstride) {
  const int h = blockIdx.y, sp_ = blockIdx.z;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const SpanR<RT> sp = span_rt<RT>(bx * 64 * RT + 16 * RT * w, i, N, seg_id, seg_ptr, S, sp_);
  float bq0[RT], bq1[RT], bo0[RT], bo1[RT], nlse[RT], ndl[RT];
  f4v dq[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const int q = sp.row[t], qc = min(q, Nq - 1);
    const float2 bq = ld2(Qp + ((int64_t)h * Nq + qc) * 8 + 2 * g);
    const float2 bo = ld2(dOp + ((int64_t)h * Nq + qc) * 8 + 2 * g);
    bq0[t] = bq.x * qscale;
    bq1[t] = bq.y * qscale;
    bo0[t] = bo.x;
    bo1[t] = bo.y;
    nlse[t] = q < N ? -LSE2[(int64_t)h * Nq + q] : 0.f;
    ndl[t] = q < N ? delta[(int64_t)h * Nq + q] : 0.f;  // delta buffer holds -delta
    dq[t] = f4z();
  }
  DQ8 t0 = ld_dq(Kp, Kq, Vp, h, Nq, sp.cb, i, g), t1 = ld_dq(Kp, Kq, Vp, h, Nq, sp.cb + 16, i, g);
  for (int k0 = sp.cb; k0 < sp.ce; k0 += 16) {
    const DQ8 tn = ld_dq(Kp, Kq, Vp, h, Nq, k0 + 32, i, g);
    const bool full = k0 >= sp.ilo && k0 + 16 <= sp.ihi && k0 + 16 <= sp.ce;
    f4v s[RT], dp[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      s[t] = mfma(t0.k.x, bq0[t], f4v{nlse[t], nlse[t], nlse[t], nlse[t]});
      dp[t] = mfma(t0.v.x, bo0[t], f4v{ndl[t], ndl[t], ndl[t], ndl[t]});
    }
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      s[t] = mfma(t0.k.y, bq1[t], s[t]);
      dp[t] = mfma(t0.v.y, bo1[t], dp[t]);
    }
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      float ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + 4 * g + r;
        const bool ok = full || (key >= sp.b[t] && key < sp.e[t] && key < sp.ce);
        ds[r] = ok ? fexp2(s[t][r]) * dp[t][r] : 0.f;
      }
      dq[t] = mfma(t0.kt.x, ds[0], dq[t]);
      dq[t] = mfma(t0.kt.y, ds[1], dq[t]);
      dq[t] = mfma(t0.kt.z, ds[2], dq[t]);
      dq[t] = mfma(t0.kt.w, ds[3], dq[t]);
    }
    t0 = t1;
    t1 = tn;
  }
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const int q = sp.row[t];
    if (q < N && g < 2) {
      *reinterpret_cast<float4*>(out + sp_ * sstride + (int64_t)q * ldo + h * 8 + 4 * g) =
          make_float4(dq[t][0] * scale, dq[t][1] * scale, dq[t][2] * scale, dq[t][3] * scale);
    }
  }
}

template <int RT>
__global__ void __launch_bounds__(256) attn8_bwd_dq_kernel(
    const float* __restrict__ Qp, const float* __restrict__ Kp, const float* __restrict__ Kq,
    const float* __restrict__ Vp, const float* __restrict__ dOp, const float* __restrict__ LSE2,
    const float* __restrict__ delta, int N, int Nq, int H, const int* __restrict__ seg_id,
    const int* __restrict__ seg_ptr, int S, float scale, float qscale, float* __restrict__ out, int ldo,
    int64_t sstride) {
  attn8_bwd_dq_body<RT>(blockIdx.x, Qp, Kp, Kq, Vp, dOp, LSE2, delta, N, Nq, H, seg_id, seg_ptr, S, scale, qscale, out, ldo, sstride);
}


// dK/dV pass: grid (ceil(N/64) key blocks, H, S over queries).  Outputs dK (x scale) at
// out + s * sstride + k * ldo + h * 8 and dV at the same + 8H.  Operands two tiles ahead in
// flight, as in the dQ pass.
struct KV8b {
  float2 q, o;     // Q, dO pair fragments of row q0 + i
  float4 qt, ot;   // Q, dO quad fragments (rows q0 + 4g .. +3, column i)
  float4 lse, dl;  // LSE2 / delta of rows q0 + 4g .. +3
};

__device__ __forceinline__ KV8b ld_kvb(const float* __restrict__ Qp, const float* __restrict__ Qq,
                                       const float* __restrict__ dOp, const float* __restrict__ dOq,
                                       const float* __restrict__ LSE2, const float* __restrict__ delta, int h, int Nq,
                                       int q0, int i, int g) {
  KV8b t;
  const int qc = min(q0, Nq - 16);
  t.q = ld2(Qp + ((int64_t)h * Nq + qc + i) * 8 + 2 * g);
  t.o = ld2(dOp + ((int64_t)h * Nq + qc + i) * 8 + 2 * g);
  const int64_t qo = (((int64_t)h * (Nq >> 2) + (qc >> 2) + g) * 8 + (i & 7)) * 4;
  t.qt = ld4(Qq + qo);  // lanes i >= 8: duplicate columns (rows 8..15 of dK^T / dV^T unused)
  t.ot = ld4(dOq + qo);
  t.lse = ld4(LSE2 + (int64_t)h * Nq + qc + 4 * g);
  t.dl = ld4(delta + (int64_t)h * Nq + qc + 4 * g);
  return t;
}

template <int RT>
__device__ __forceinline__ void attn8_bwd_dkv_body(int bx, 
    const float* __restrict__ Qp, const float* __restrict__ Qq, const float* __restrict__ Kp,
    const float* __restrict__ Vp, const float* __restrict__ dOp, const float* __restrict__ dOq,
    const float* __restrict__ LSE2, const float* __restrict__ delta, int N, int Nq, int H,
    const int* __restrict__ seg_id, const int* __restrict__ seg_ptr, int S, float scale, float qscale,
    float* __restrict__ out, int ldo, int64_t sstride) {
  const int h = blockIdx.y, sp_ = blockIdx.z;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  // keys and queries share segments: the key rows' spans are the query ranges to visit
  const SpanR<RT> sp = span_rt<RT>(bx * 64 * RT + 16 * RT * w, i, N, seg_id, seg_ptr, S, sp_);
  float bk0[RT], bk1[RT], bv0[RT], bv1[RT];
  f4v dk[RT], dv[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const int kc = min(sp.row[t], Nq - 1);
    const float2 bk = ld2(Kp + ((int64_t)h * Nq + kc) * 8 + 2 * g);
    const float2 bv = ld2(Vp + ((int64_t)h * Nq + kc) * 8 + 2 * g);
    bk0[t] = bk.x * qscale;
    bk1[t] = bk.y * qscale;
    bv0[t] = bv.x;
    bv1[t] = bv.y;
    dk[t] = f4z();
    dv[t] = f4z();
  }
  KV8b t0 = ld_kvb(Qp, Qq, dOp, dOq, LSE2, delta, h, Nq, sp.cb, i, g);
  KV8b t1 = ld_kvb(Qp, Qq, dOp, dOq, LSE2, delta, h, Nq, sp.cb + 16, i, g);
  for (int q0 = sp.cb; q0 < sp.ce; q0 += 16) {
    const KV8b tn = ld_kvb(Qp, Qq, dOp, dOq, LSE2, delta, h, Nq, q0 + 32, i, g);
    const bool full = q0 >= sp.ilo && q0 + 16 <= sp.ihi && q0 + 16 <= sp.ce;
    const f4v nl = f4v{-t0.lse.x, -t0.lse.y, -t0.lse.z, -t0.lse.w};
    const f4v nd = f4v{t0.dl.x, t0.dl.y, t0.dl.z, t0.dl.w};  // delta buffer holds -delta
    f4v s[RT], dp[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      s[t] = mfma(t0.q.x, bk0[t], nl);
      dp[t] = mfma(t0.o.x, bv0[t], nd);
    }
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      s[t] = mfma(t0.q.y, bk1[t], s[t]);
      dp[t] = mfma(t0.o.y, bv1[t], dp[t]);
    }
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      float p[4], ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = q0 + 4 * g + r;
        const bool ok = full || (qq >= sp.b[t] && qq < sp.e[t] && qq < sp.ce);
        p[r] = ok ? fexp2(s[t][r]) : 0.f;
        ds[r] = p[r] * dp[t][r];
      }
      dv[t] = mfma(t0.ot.x, p[0], dv[t]);
      dk[t] = mfma(t0.qt.x, ds[0], dk[t]);
      dv[t] = mfma(t0.ot.y, p[1], dv[t]);
      dk[t] = mfma(t0.qt.y, ds[1], dk[t]);
      dv[t] = mfma(t0.ot.z, p[2], dv[t]);
      dk[t] = mfma(t0.qt.z, ds[2], dk[t]);
      dv[t] = mfma(t0.ot.w, p[3], dv[t]);
      dk[t] = mfma(t0.qt.w, ds[3], dk[t]);
    }
    t0 = t1;
    t1 = tn;
  }
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const int k = sp.row[t];
    if (k < N && g < 2) {
      float* o = out + sp_ * sstride + (int64_t)k * ldo + h * 8 + 4 * g;
      *reinterpret_cast<float4*>(o) =
          make_float4(dk[t][0] * scale, dk[t][1] * scale, dk[t][2] * scale, dk[t][3] * scale);
      *reinterpret_cast<float4*>(o + 8 * H) = make_float4(dv[t][0], dv[t][1], dv[t][2], dv[t][3]);
    }
  }
}

template <int RT>
__global__ void __launch_bounds__(256) attn8_bwd_dkv_kernel(
    const float* __restrict__ Qp, const float* __restrict__ Qq, const float* __restrict__ Kp,
    const float* __restrict__ Vp, const float* __restrict__ dOp, const float* __restrict__ dOq,
    const float* __restrict__ LSE2, const float* __restrict__ delta, int N, int Nq, int H,
    const int* __restrict__ seg_id, const int* __restrict__ seg_ptr, int S, float scale, float qscale,
    float* __restrict__ out, int ldo, int64_t sstride) {
  attn8_bwd_dkv_body<RT>(blockIdx.x, Qp, Qq, Kp, Vp, dOp, dOq, LSE2, delta, N, Nq, H, seg_id, seg_ptr, S, scale, qscale, out, ldo, sstride);
}


// dqkv [N, 3F] = [sum_s dQ_s | sum_s dKV_s] over split partials (fixed order)
// dQ and dK/dV passes in ONE launch: blocks [0, nbq) run the dQ body, the rest the dK/dV
// body (they only share read-only inputs).  Each pass alone leaves most of the chip idle
// in its tail; one grid lets the two overlap without a second stream.
struct A8Bwd {
  const float *Qp, *Qq, *Kp, *Kq, *Vp, *dOp, *dOq, *LSE2, *delta;
  int N, Nq, H;
  const int *seg_id, *seg_ptr;
  int S;
  float scale, qscale;
  float *out_q, *out_kv;
  int ldq, ldkv;
  int64_t sq, skv;
  int nbq;
};

template <int RT>
__global__ void __launch_bounds__(256) attn8_bwd_fused_kernel(A8Bwd a) {
  if ((int)blockIdx.x < a.nbq) {
    attn8_bwd_dq_body<RT>(blockIdx.x, a.Qp, a.Kp, a.Kq, a.Vp, a.dOp, a.LSE2, a.delta, a.N, a.Nq, a.H, a.seg_id,
                          a.seg_ptr, a.S, a.scale, a.qscale, a.out_q, a.ldq, a.sq);
  } else {
    attn8_bwd_dkv_body<RT>(blockIdx.x - a.nbq, a.Qp, a.Qq, a.Kp, a.Vp, a.dOp, a.dOq, a.LSE2, a.delta, a.N, a.Nq,
                           a.H, a.seg_id, a.seg_ptr, a.S, a.scale, a.qscale, a.out_kv, a.ldkv, a.skv);
  }
}

__global__ void __launch_bounds__(256) attn8_bwd_sum_kernel(const float4* __restrict__ pq, int Sq,
                                                            const float4* __restrict__ pkv, int Skv,
                                                            float4* __restrict__ dqkv, int N, int F) {
  const int F4 = F / 4;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)N * 3 * F4) return;
  const int n = (int)(t / (3 * F4)), c = (int)(t % (3 * F4));
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < F4) {
    for (int s = 0; s < Sq; ++s) a = f4add(a, pq[((int64_t)s * N + n) * F4 + c]);
  } else {
    for (int s = 0; s < Skv; ++s) a = f4add(a, pkv[((int64_t)s * N + n) * 2 * F4 + (c - F4)]);
  }
  dqkv[t] = a;
}

// pack one [N, F] block (columns of head h at h*8) of a row-major matrix into the pair and
// quad layouts (rows >= N zero)
__global__ void __launch_bounds__(256) attn8_pack_kernel(const float* __restrict__ X, int ldx, int N, int Nq, int H,
                                                         float* __restrict__ pair, float* __restrict__ quad) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)Nq * H * 8) return;
  const int n = (int)(t / (H * 8)), c = (int)(t % (H * 8)), h = c >> 3, d = c & 7;
  const float v = n < N ? X[(int64_t)n * ldx + c] : 0.f;
  if (pair) pair[pair_idx(h, Nq, n, d)] = v;
  if (quad) quad[quad_idx(h, Nq, n, d)] = v;
}

// delta[h][q] = sum_d dO[q, h, d] O[q, h, d] (+ dO in pair / quad layouts)
__global__ void __launch_bounds__(256) attn8_delta_pack_kernel(const float* __restrict__ dO,
                                                               const float* __restrict__ O, int N, int Nq, int H,
                                                               float* __restrict__ delta, float* __restrict__ pair,
                                                               float* __restrict__ quad) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)Nq * H) return;
  const int n = (int)(t / H), h = (int)(t % H);
  float a = 0.f;
#pragma unroll
  for (int d = 0; d < 8; ++d) {
    const float v = n < N ? dO[(int64_t)n * 8 * H + h * 8 + d] : 0.f;
    if (n < N) a = fmaf(v, O[(int64_t)n * 8 * H + h * 8 + d], a);
    pair[pair_idx(h, Nq, n, d)] = v;
    quad[quad_idx(h, Nq, n, d)] = v;
  }
  delta[(int64_t)h * Nq + n] = -a;  // stored negated: the MFMA accumulator seed of dP - delta
}

// ------------------------------------------------------------------- v2: one launch each way
// The grid-split kernels above leave a combine (fwd) / partial-sum (bwd) launch behind and
// run the forward in two passes over the keys (exact row max first).  v2:
//   * a workgroup = W waves on the SAME RT query (or key) row tiles, each wave a 1/W slice
//     of the other index; the W partial results meet in LDS and are merged in a fixed
//     order at the end of the launch (deterministic, no partial buffers, no extra launch);
//   * forward in ONE pass with a deferred-rescale softmax: scores are shifted by a running
//     per-row reference m (exact max of the keys seen when it was last moved) that only
//     moves when a score exceeds it by more than kTau (p <= 2^kTau, l stays far from fp32
//     overflow); the check is 3 VALU ops per tile, the rescale (cross-lane max, o *= 2^dm)
//     runs on the few tiles that raise a row's max by > kTau, so the score MFMAs run once
//     per tile instead of twice.  Results equal the two-pass kernel to fp32 rounding;
//   * lean tile bodies (the loops are issue-bound, not MFMA-bound, when written plainly):
//     operands come through buffer loads whose lane offset is a loop-invariant VGPR and
//     whose tile offset is a scalar (no per-tile 64-bit address VALU), two operand buffers
//     are reloaded in place right after use (a register copy of an in-flight load would
//     force a vmcnt drain), MFMA accumulator seeds (-m, -LSE, -delta) stay in persistent
//     registers, the forward stores -LSE2 and the backward prep -delta so no tile negates;
//     lanes i >= 8 load duplicate columns (rows 8..15 of the d-major products are junk and
//     never stored) instead of selecting zeros, and the forward's row sum l is VALU adds.
// Contract: the v2 forward returns NL = -LSE2 (rows Nq > q >= N: 0), which the v2 backward
// consumes; the grid kernels keep LSE2.
constexpr float kTau = 8.f;

typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc mk_rsrc(const float* p, int nfloats) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, nfloats * 4, 0x00020000);
}
__device__ __forceinline__ float2 bl2(Rsrc r, int vo, int so) {
  return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 0));
}
__device__ __forceinline__ float4 bl4(Rsrc r, int vo, int so) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0));
}
__device__ __forceinline__ float max4(f4v s) { return fmaxf(fmaxf(s[0], s[1]), fmaxf(s[2], s[3])); }


// bf16 mode (precision "bf16"): every product on v_mfma_f32_16x16x16_bf16 (fp32 accumulate).
// Lane (i, g) supplies A[i][4g .. 4g+3] / B[4g .. 4g+3][i].  D = 8 contractions (S = Q K^T,
// dP = dO V^T) use lane groups 0, 1 only — each reads one float4 of the pair layout, d in the
// order {0, 4, 1, 5} / {2, 6, 3, 7}, the same for both operands — and zeros in groups 2, 3; the
// 16-key / 16-query contractions (O, dQ, dK, dV) take a quad-layout float4 and the four
// probabilities / dS values of the score accumulator, exactly as the fp32 path's four k-steps.
typedef short s4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ s4v pk4(float a, float b, float c, float d) {
  typedef __bf16 b4v __attribute__((ext_vector_type(4)));
  const b4v v = {(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)d};
  return __builtin_bit_cast(s4v, v);
}
__device__ __forceinline__ s4v pk4(float4 v) { return pk4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ s4v pk4z(float4 v, bool live) {  // zero in lane groups 2, 3
  return live ? pk4(v) : s4v{0, 0, 0, 0};
}
__device__ __forceinline__ f4v mfma_bf(s4v a, s4v b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
// pair-layout float4 of row k0 + i for the D = 8 bf16 contractions (lane groups 0, 1)
__device__ __forceinline__ int off_pair4(int i, int g) { return (8 * i + 4 * (g & 1)) * 4; }

// Byte offsets inside one head's [Nq][8] pair / [Nq/4][8][4] quad block: a 16-row tile at
// row k0 starts at k0 * 32 bytes in both layouts; lane (i, g) reads
//   pair: row k0 + i, float2 at 2g        -> (8 i + 2 g) * 4
//   quad: rows k0 + 4g .. +3, column i&7   -> (32 g + 4 (i & 7)) * 4
__device__ __forceinline__ int off_pair(int i, int g) { return (8 * i + 2 * g) * 4; }
__device__ __forceinline__ int off_quad(int i, int g) { return (32 * g + 4 * (i & 7)) * 4; }

template <int RT, int W, bool BF = false>
__global__ void __launch_bounds__(64 * W) attn8_fwd2_kernel(const float* __restrict__ Qp,
                                                            const float* __restrict__ Kp,
                                                            const float* __restrict__ Vq, int N, int Nq, int H,
                                                            const int* __restrict__ seg_id,
                                                            const int* __restrict__ seg_ptr, float qscale,
                                                            float* __restrict__ O, float* __restrict__ NL) {
  __shared__ float red[W][RT][16][10];  // per wave and query: (m, l, o[8])
  const int h = blockIdx.y;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int qbase = blockIdx.x * 16 * RT;
  const SpanR<RT> sp = span_rt<RT>(qbase, i, N, seg_id, seg_ptr, W, w);
  const Rsrc rk = mk_rsrc(Kp + (int64_t)h * Nq * 8, Nq * 8), rv = mk_rsrc(Vq + (int64_t)h * Nq * 8, Nq * 8);
  const int ok_ = BF ? off_pair4(i, g) : off_pair(i, g), ov_ = off_quad(i, g);
  const bool lo2 = g < 2;
  float bq0[RT], bq1[RT], m[RT], l[RT], thr[RT];
  s4v qb[RT];
  f4v o[RT], cin[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    if constexpr (BF) {
      float4 q4 = ld4(Qp + ((int64_t)h * Nq + min(sp.row[t], Nq - 1)) * 8 + 4 * (g & 1));
      qb[t] = pk4z(make_float4(q4.x * qscale, q4.y * qscale, q4.z * qscale, q4.w * qscale), lo2);
    } else {
      const float2 bq = ld2(Qp + ((int64_t)h * Nq + min(sp.row[t], Nq - 1)) * 8 + 2 * g);
      bq0[t] = bq.x * qscale;
      bq1[t] = bq.y * qscale;
    }
    m[t] = -INFINITY;
    thr[t] = -INFINITY;  // unset reference: any valid score moves it
    l[t] = 0.f;
    o[t] = f4z();
    cin[t] = f4z();
  }
  // one key tile: S^T (shifted by the row references), mask, deferred rescale, O^T += V^T P^T.
  // Tiles past the slice end (k0 >= ce, the odd tail of the 2-tile loop) are fully masked.
  auto tile = [&](auto kk, float4 vv, int k0) {
    const bool full = k0 >= sp.ilo && k0 + 16 <= sp.ihi && k0 + 16 <= sp.ce;
    f4v s[RT];
    if constexpr (BF) {
      const s4v ka = pk4z(kk, lo2);
#pragma unroll
      for (int t = 0; t < RT; ++t) s[t] = mfma_bf(ka, qb[t], cin[t]);
    } else {
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        s[t] = mfma(kk.x, bq0[t], cin[t]);
        s[t] = mfma(kk.y, bq1[t], s[t]);
      }
    }
    if (!full) {
#pragma unroll
      for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + 4 * g + r;
          if (!(key >= sp.b[t] && key < sp.e[t] && key < sp.ce)) s[t][r] = -INFINITY;
        }
    }
    bool trig = false;
#pragma unroll
    for (int t = 0; t < RT; ++t) trig |= max4(s[t]) > thr[t];
    if (__any(trig)) {  // wave-uniform: move the row references, rescale o and l
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        const float base = -cin[t][0];
        const float mn = fmaxf(m[t], wmax16(max4(s[t])) + base);
        if (mn > -INFINITY) {
          const float f = fexp2(m[t] - mn), sh = mn - base;
          o[t] = o[t] * f;
          l[t] *= f;
          s[t] = s[t] - f4v{sh, sh, sh, sh};
          m[t] = mn;
          thr[t] = kTau;
          cin[t] = f4v{-mn, -mn, -mn, -mn};
        }
      }
    }
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const float p0 = fexp2(s[t][0]), p1 = fexp2(s[t][1]), p2 = fexp2(s[t][2]), p3 = fexp2(s[t][3]);
      if constexpr (BF) {
        o[t] = mfma_bf(pk4(vv), pk4(p0, p1, p2, p3), o[t]);
      } else {
        o[t] = mfma(vv.x, p0, o[t]);
        o[t] = mfma(vv.y, p1, o[t]);
        o[t] = mfma(vv.z, p2, o[t]);
        o[t] = mfma(vv.w, p3, o[t]);
      }
      l[t] += (p0 + p1) + (p2 + p3);
    }
  };
  // load order pinned by scheduling barriers: the loop header is entered with the same
  // in-flight sequence (ka va kb vb) from the preheader and from the latch, so the compiler's
  // wait before the first tile is vmcnt(2), not a drain
  const int cmax = (Nq - 16) * 32;
  auto ldk = [&](int off) {
    if constexpr (BF) return bl4(rk, ok_, off); else return bl2(rk, ok_, off);
  };
  auto ka = ldk(min(sp.cb * 32, cmax));
  float4 va = bl4(rv, ov_, min(sp.cb * 32, cmax));
  __builtin_amdgcn_sched_barrier(0);
  auto kb = ldk(min(sp.cb * 32 + 512, cmax));
  float4 vb = bl4(rv, ov_, min(sp.cb * 32 + 512, cmax));
  __builtin_amdgcn_sched_barrier(0);
  for (int k0 = sp.cb; k0 < sp.ce; k0 += 32) {
    tile(ka, va, k0);
    ka = ldk(min(k0 * 32 + 1024, cmax));
    va = bl4(rv, ov_, min(k0 * 32 + 1024, cmax));
    __builtin_amdgcn_sched_barrier(0);
    tile(kb, vb, k0 + 16);
    kb = ldk(min(k0 * 32 + 1536, cmax));
    vb = bl4(rv, ov_, min(k0 * 32 + 1536, cmax));
    __builtin_amdgcn_sched_barrier(0);
  }
  // o: lane (i, g) rows 4g + r of O^T for query i (g = 0, 1 -> d 0..7); l: this lane's
  // 4-key share of the row sum -> total over the 4 lane groups
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    float lt = l[t] + __shfl_xor(l[t], 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    if (g < 2) {
#pragma unroll
      for (int r = 0; r < 4; ++r) red[w][t][i][2 + 4 * g + r] = o[t][r];
    } else if (g == 2) {
      red[w][t][i][0] = m[t];
      red[w][t][i][1] = lt;
    }
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < RT * 128; idx += 64 * W) {
    const int t = idx >> 7, qi = (idx >> 3) & 15, d = idx & 7;
    const int qq = qbase + 16 * t + qi;
    float M = -INFINITY;
#pragma unroll
    for (int v = 0; v < W; ++v) M = fmaxf(M, red[v][t][qi][0]);
    float lsum = 0.f, a = 0.f;
    if (M > -INFINITY) {
#pragma unroll
      for (int v = 0; v < W; ++v) {
        const float f = fexp2(red[v][t][qi][0] - M);
        lsum = fmaf(red[v][t][qi][1], f, lsum);
        a = fmaf(red[v][t][qi][2 + d], f, a);
      }
    }
    if (qq < N) {
      O[(int64_t)qq * 8 * H + h * 8 + d] = lsum > 0.f ? a * (1.f / lsum) : 0.f;
      if (d == 0) NL[(int64_t)h * Nq + qq] = lsum > 0.f ? -(M + __log2f(lsum)) : INFINITY;
    } else if (qq < Nq && d == 0) {
      NL[(int64_t)h * Nq + qq] = 0.f;
    }
  }
}

// v2 forward on quad-block MFMAs (fp32).  Measured on MI355X (tools/mfma_rate.hip): an f32
// MFMA and f32 VALU work of the same SIMD do NOT overlap (4 x 16x16x4 + 16 v_fma take the SUM
// of their times), and v_mfma_f32_4x4x1_16b_f32 retires 512 FLOP in ~10 cycles against the
// 16x16x4's 2,048 in 32.  The P.V product of an 8-wide head wastes half of every 16x16x4
// (only 8 of its 16 output rows are real), so here it runs as 4x4x1_16b blocks instead:
// block b = 4g + i/4 of lane (i, g) owns queries 4(i/4)..+3 x dims 4dh..+3 and sums over its
// lane group's keys 4g + r (r = the instruction), so the A operand is the lane's OWN
// probability p[r] (no shuffles) and the B operand comes straight from the quad layout
// (keys 4g..4g+3 of dim 4dh + i%4: one float4 per d half).  2 x 4 independent 10-cycle MFMAs
// replace 4 dependent 32-cycle ones; the 4 lane groups' partial O are summed once per slice.
// VALU per tile is kept minimal (it adds to the MFMA time): the -m seed is rebuilt from one
// register.  (A raw inline-asm v_max3_f32 on the score accumulator, skipping the compiler's
// canonicalising v_max x, x, read the MFMA result without the hazard wait states the compiler
// inserts for its own instructions: the rescale decisions, and so the rounding, varied between
// launches.)
__device__ __forceinline__ f4v mfma4(float a, float b, f4v c) {
  return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
}
template <int W>
__device__ __forceinline__ void attn8_fwd2q_body(const float* __restrict__ Qp, const float* __restrict__ Kp,
                                                 const float* __restrict__ Vq, int N, int Nq, int H,
                                                 const int* __restrict__ seg_id, const int* __restrict__ seg_ptr,
                                                 float qscale, float* __restrict__ O, float* __restrict__ NL,
                                                 int qtile, int h) {
  __shared__ float red[W][16][10];
  const int w = uni(threadIdx.x >> 6), lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int qbase = qtile * 16;
  const SpanR<1> sp = span_rt<1>(qbase, i, N, seg_id, seg_ptr, W, w);
  const Rsrc rk = mk_rsrc(Kp + (int64_t)h * Nq * 8, Nq * 8), rv = mk_rsrc(Vq + (int64_t)h * Nq * 8, Nq * 8);
  // K pair fragment of row k0 + i; V quad float4s of keys k0 + 4g..+3, dims i%4 and 4 + i%4
  const int ok_ = off_pair(i, g), ov0 = (32 * g + 4 * (i & 3)) * 4, ov1 = ov0 + 64;
  const float2 bq = ld2(Qp + ((int64_t)h * Nq + min(sp.row[0], Nq - 1)) * 8 + 2 * g);
  const float bq0 = bq.x * qscale, bq1 = bq.y * qscale;
  float m = -INFINITY, thr = -INFINITY, l = 0.f, negm = 0.f;
  f4v o0 = f4z(), o1 = f4z();  // O[query i][dim 4dh + r], partial over the lane group's keys
  auto tile = [&](float2 kk, float4 va, float4 vb, int k0) {
    const f4v cin = f4v{negm, negm, negm, negm};
    f4v s = mfma(kk.x, bq0, cin);
    s = mfma(kk.y, bq1, s);
    const bool full = k0 >= sp.ilo && k0 + 16 <= sp.ihi && k0 + 16 <= sp.ce;
    if (!full) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + 4 * g + r;
        if (!(key >= sp.b[0] && key < sp.e[0] && key < sp.ce)) s[r] = -INFINITY;
      }
    }
    const float mx = max4(s);
    if (__any(mx > thr)) {  // move the row reference (rare), rescale o and l
      const float mn = fmaxf(m, wmax16(mx) - negm);
      if (mn > -INFINITY) {
        const float f = fexp2(m - mn), sh = mn + negm;
        o0 = o0 * f;
        o1 = o1 * f;
        l *= f;
        s = s - f4v{sh, sh, sh, sh};
        m = mn;
        thr = kTau;
        negm = -mn;
      }
    }
    const float p0 = fexp2(s[0]), p1 = fexp2(s[1]), p2 = fexp2(s[2]), p3 = fexp2(s[3]);
    o0 = mfma4(va.x, p0, o0);
    o1 = mfma4(vb.x, p0, o1);
    o0 = mfma4(va.y, p1, o0);
    o1 = mfma4(vb.y, p1, o1);
    o0 = mfma4(va.z, p2, o0);
    o1 = mfma4(vb.z, p2, o1);
    o0 = mfma4(va.w, p3, o0);
    o1 = mfma4(vb.w, p3, o1);
    l += (p0 + p1) + (p2 + p3);
  };
  const int cmax = (Nq - 16) * 32;
  float2 ka = bl2(rk, ok_, min(sp.cb * 32, cmax));
  float4 va0 = bl4(rv, ov0, min(sp.cb * 32, cmax)), va1 = bl4(rv, ov1, min(sp.cb * 32, cmax));
  __builtin_amdgcn_sched_barrier(0);
  float2 kb = bl2(rk, ok_, min(sp.cb * 32 + 512, cmax));
  float4 vb0 = bl4(rv, ov0, min(sp.cb * 32 + 512, cmax)), vb1 = bl4(rv, ov1, min(sp.cb * 32 + 512, cmax));
  __builtin_amdgcn_sched_barrier(0);
  for (int k0 = sp.cb; k0 < sp.ce; k0 += 32) {
    tile(ka, va0, va1, k0);
    ka = bl2(rk, ok_, min(k0 * 32 + 1024, cmax));
    va0 = bl4(rv, ov0, min(k0 * 32 + 1024, cmax));
    va1 = bl4(rv, ov1, min(k0 * 32 + 1024, cmax));
    __builtin_amdgcn_sched_barrier(0);
    tile(kb, vb0, vb1, k0 + 16);
    kb = bl2(rk, ok_, min(k0 * 32 + 1536, cmax));
    vb0 = bl4(rv, ov0, min(k0 * 32 + 1536, cmax));
    vb1 = bl4(rv, ov1, min(k0 * 32 + 1536, cmax));
    __builtin_amdgcn_sched_barrier(0);
  }
  // sum the 4 lane groups' partial blocks and row sums; lanes of group 0 hold the slice's O
  float lt = l + __shfl_xor(l, 16, 64);
  lt += __shfl_xor(lt, 32, 64);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    o0[r] += __shfl_xor(o0[r], 16, 64);
    o0[r] += __shfl_xor(o0[r], 32, 64);
    o1[r] += __shfl_xor(o1[r], 16, 64);
    o1[r] += __shfl_xor(o1[r], 32, 64);
  }
  if (g == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      red[w][i][2 + r] = o0[r];
      red[w][i][6 + r] = o1[r];
    }
  } else if (g == 1) {
    red[w][i][0] = m;
    red[w][i][1] = lt;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < 128; idx += 64 * W) {
    const int qi = idx >> 3, d = idx & 7;
    const int qq = qbase + qi;
    float M = -INFINITY;
#pragma unroll
    for (int v = 0; v < W; ++v) M = fmaxf(M, red[v][qi][0]);
    float lsum = 0.f, a = 0.f;
    if (M > -INFINITY) {
#pragma unroll
      for (int v = 0; v < W; ++v) {
        const float f = fexp2(red[v][qi][0] - M);
        lsum = fmaf(red[v][qi][1], f, lsum);
        a = fmaf(red[v][qi][2 + d], f, a);
      }
    }
    if (qq < N) {
      O[(int64_t)qq * 8 * H + h * 8 + d] = lsum > 0.f ? a * (1.f / lsum) : 0.f;
      if (d == 0) NL[(int64_t)h * Nq + qq] = lsum > 0.f ? -(M + __log2f(lsum)) : INFINITY;
    } else if (qq < Nq && d == 0) {
      NL[(int64_t)h * Nq + qq] = 0.f;
    }
  }
}

template <int W>
__global__ void __launch_bounds__(64 * W) attn8_fwd2q_kernel(const float* __restrict__ Qp,
                                                             const float* __restrict__ Kp,
                                                             const float* __restrict__ Vq, int N, int Nq, int H,
                                                             const int* __restrict__ seg_id,
                                                             const int* __restrict__ seg_ptr, float qscale,
                                                             float* __restrict__ O, float* __restrict__ NL) {
  attn8_fwd2q_body<W>(Qp, Kp, Vq, N, Nq, H, seg_id, seg_ptr, qscale, O, NL, blockIdx.x, blockIdx.y);
}

// The GPS layer's two independent branches in ONE launch: workgroups [0, nA) run the
// attention forward (query tile, head), the rest the PNA message + aggregation forward
// (pna_body.h, one wave per node).  In the captured step the two were a stream fork / join
// (attention on a side stream): every fork or join edge of a hipGraph costs ~7 us on MI355X
// (tools/graph_fork_cost.py) and each layer paid two on its critical path.  Attention
// workgroups come first in the grid (the long ones dispatch first); the PNA workgroups fill
// the remaining slots exactly as the second stream's did.
struct PnaFwdArgs {
  const float *x, *AB, *C, *G;
  const int *src, *rowptr;
  float* Z;
  int *amin, *amax;
  int ldab, N, F, tpr;
  float avg_log, avg_lin;
};

template <int W>
__global__ void __launch_bounds__(64 * W) attn8_pna_fwd_kernel(const float* __restrict__ Qp,
                                                               const float* __restrict__ Kp,
                                                               const float* __restrict__ Vq, int N, int Nq, int H,
                                                               const int* __restrict__ seg_id,
                                                               const int* __restrict__ seg_ptr, float qscale,
                                                               float* __restrict__ O, float* __restrict__ NL, int nqt,
                                                               PnaFwdArgs p) {
  const int b = blockIdx.x, nA = nqt * H;
  if (b < nA) {
    attn8_fwd2q_body<W>(Qp, Kp, Vq, N, Nq, H, seg_id, seg_ptr, qscale, O, NL, b % nqt, b / nqt);
    return;
  }
  const int rpb = 64 * W / p.tpr;
  pna_fwd_node<1>(p.x, p.AB, p.ldab, p.C, p.G, p.src, p.rowptr, p.Z, p.amin, p.amax,
                  (b - nA) * rpb + (int)threadIdx.x / p.tpr, (int)threadIdx.x % p.tpr, p.N, p.F, p.avg_log,
                  p.avg_lin, p.tpr);
}

// Backward v2: blocks [0, nbq) produce dQ for RT query tiles (W waves split the keys),
// the rest dK | dV for RT key tiles (W waves split the queries); per-wave partials are
// summed in LDS in wave order and written straight into dqkv [N, 3F].
struct A8Bwd2 {
  const float *Qp, *Qq, *Kp, *Kq, *Vp, *dOp, *dOq, *NL, *ndelta;
  int N, Nq, H;
  const int *seg_id, *seg_ptr;
  float scale, qscale;
  float* dqkv;
  int nbq;
};

template <int RT, int W, bool BF>
__device__ __forceinline__ void attn8_bwd2_dq(const A8Bwd2& a, int bx, float* red) {
  const int h = blockIdx.y;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int N = a.N, Nq = a.Nq;
  const int base = bx * 16 * RT;
  const SpanR<RT> sp = span_rt<RT>(base, i, N, a.seg_id, a.seg_ptr, W, w);
  const int64_t hb = (int64_t)h * Nq * 8;
  const Rsrc rk = mk_rsrc(a.Kp + hb, Nq * 8), rv = mk_rsrc(a.Vp + hb, Nq * 8), rkt = mk_rsrc(a.Kq + hb, Nq * 8);
  const int op = BF ? off_pair4(i, g) : off_pair(i, g), oq = off_quad(i, g);
  const bool lo2 = g < 2;
  float bq0[RT], bq1[RT], bo0[RT], bo1[RT];
  s4v qb[RT], ob[RT];
  f4v dq[RT], cs[RT], cd[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const int q = sp.row[t], qc = min(q, Nq - 1);
    if constexpr (BF) {
      const float4 q4 = ld4(a.Qp + hb + (int64_t)qc * 8 + 4 * (g & 1));
      qb[t] = pk4z(make_float4(q4.x * a.qscale, q4.y * a.qscale, q4.z * a.qscale, q4.w * a.qscale), lo2);
      ob[t] = pk4z(ld4(a.dOp + hb + (int64_t)qc * 8 + 4 * (g & 1)), lo2);
    } else {
      const float2 bq = ld2(a.Qp + hb + (int64_t)qc * 8 + 2 * g);
      const float2 bo = ld2(a.dOp + hb + (int64_t)qc * 8 + 2 * g);
      bq0[t] = bq.x * a.qscale;
      bq1[t] = bq.y * a.qscale;
      bo0[t] = bo.x;
      bo1[t] = bo.y;
    }
    const float nl = q < N ? a.NL[(int64_t)h * Nq + q] : 0.f;
    const float nd = q < N ? a.ndelta[(int64_t)h * Nq + q] : 0.f;
    cs[t] = f4v{nl, nl, nl, nl};
    cd[t] = f4v{nd, nd, nd, nd};
    dq[t] = f4z();
  }
  auto tile = [&](auto kk, auto vv, float4 kt, int k0) {
    const bool full = k0 >= sp.ilo && k0 + 16 <= sp.ihi && k0 + 16 <= sp.ce;
    f4v s[RT], dp[RT];
    if constexpr (BF) {
      const s4v ka = pk4z(kk, lo2), va = pk4z(vv, lo2);
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        s[t] = mfma_bf(ka, qb[t], cs[t]);
        dp[t] = mfma_bf(va, ob[t], cd[t]);
      }
    } else {
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        s[t] = mfma(kk.x, bq0[t], cs[t]);
        dp[t] = mfma(vv.x, bo0[t], cd[t]);
      }
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        s[t] = mfma(kk.y, bq1[t], s[t]);
        dp[t] = mfma(vv.y, bo1[t], dp[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      float ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) ds[r] = fexp2(s[t][r]) * dp[t][r];
      if (!full) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + 4 * g + r;
          if (!(key >= sp.b[t] && key < sp.e[t] && key < sp.ce)) ds[r] = 0.f;
        }
      }
      if constexpr (BF) {
        dq[t] = mfma_bf(pk4(kt), pk4(ds[0], ds[1], ds[2], ds[3]), dq[t]);
      } else {
        dq[t] = mfma(kt.x, ds[0], dq[t]);
        dq[t] = mfma(kt.y, ds[1], dq[t]);
        dq[t] = mfma(kt.z, ds[2], dq[t]);
        dq[t] = mfma(kt.w, ds[3], dq[t]);
      }
    }
  };
  const int cmax = (Nq - 16) * 32;
  auto ldp = [&](Rsrc r, int off) {
    if constexpr (BF) return bl4(r, op, off); else return bl2(r, op, off);
  };
  int o0 = min(sp.cb * 32, cmax), o1 = min(sp.cb * 32 + 512, cmax);
  auto ka = ldp(rk, o0);
  auto va = ldp(rv, o0);
  float4 ta = bl4(rkt, oq, o0);
  __builtin_amdgcn_sched_barrier(0);
  auto kb = ldp(rk, o1);
  auto vb = ldp(rv, o1);
  float4 tb = bl4(rkt, oq, o1);
  __builtin_amdgcn_sched_barrier(0);
  for (int k0 = sp.cb; k0 < sp.ce; k0 += 32) {
    tile(ka, va, ta, k0);
    o0 = min(k0 * 32 + 1024, cmax);
    ka = ldp(rk, o0);
    va = ldp(rv, o0);
    ta = bl4(rkt, oq, o0);
    __builtin_amdgcn_sched_barrier(0);
    tile(kb, vb, tb, k0 + 16);
    o1 = min(k0 * 32 + 1536, cmax);
    kb = ldp(rk, o1);
    vb = ldp(rv, o1);
    tb = bl4(rkt, oq, o1);
    __builtin_amdgcn_sched_barrier(0);
  }
  // red [W][RT][16 rows][8]: dQ^T rows 4g + r (g < 2) of column i
  if (g < 2) {
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[((w * RT + t) * 16 + i) * 8 + 4 * g + r] = dq[t][r];
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < RT * 128; idx += 64 * W) {
    const int t = idx >> 7, qi = (idx >> 3) & 15, d = idx & 7;
    float v = 0.f;
#pragma unroll
    for (int u = 0; u < W; ++u) v += red[((u * RT + t) * 16 + qi) * 8 + d];
    const int q = base + 16 * t + qi;
    if (q < N) a.dqkv[(int64_t)q * 24 * a.H + h * 8 + d] = v * a.scale;
  }
}

template <int RT, int W, bool BF>
__device__ __forceinline__ void attn8_bwd2_dkv(const A8Bwd2& a, int bx, float* red) {
  const int h = blockIdx.y;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int N = a.N, Nq = a.Nq;
  const int base = bx * 16 * RT;
  // keys and queries share segments: the key rows' spans are the query ranges to visit
  const SpanR<RT> sp = span_rt<RT>(base, i, N, a.seg_id, a.seg_ptr, W, w);
  const int64_t hb = (int64_t)h * Nq * 8;
  const Rsrc rq = mk_rsrc(a.Qp + hb, Nq * 8), ro = mk_rsrc(a.dOp + hb, Nq * 8);
  const Rsrc rqt = mk_rsrc(a.Qq + hb, Nq * 8), rot = mk_rsrc(a.dOq + hb, Nq * 8);
  const Rsrc rl = mk_rsrc(a.NL + (int64_t)h * Nq, Nq), rd = mk_rsrc(a.ndelta + (int64_t)h * Nq, Nq);
  const int op = BF ? off_pair4(i, g) : off_pair(i, g), oq = off_quad(i, g), os = 16 * g;
  const bool lo2 = g < 2;
  float bk0[RT], bk1[RT], bv0[RT], bv1[RT];
  s4v kb4[RT], vb4[RT];
  f4v dk[RT], dv[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const int kc = min(sp.row[t], Nq - 1);
    if constexpr (BF) {
      const float4 k4 = ld4(a.Kp + hb + (int64_t)kc * 8 + 4 * (g & 1));
      kb4[t] = pk4z(make_float4(k4.x * a.qscale, k4.y * a.qscale, k4.z * a.qscale, k4.w * a.qscale), lo2);
      vb4[t] = pk4z(ld4(a.Vp + hb + (int64_t)kc * 8 + 4 * (g & 1)), lo2);
    } else {
      const float2 bk = ld2(a.Kp + hb + (int64_t)kc * 8 + 2 * g);
      const float2 bv = ld2(a.Vp + hb + (int64_t)kc * 8 + 2 * g);
      bk0[t] = bk.x * a.qscale;
      bk1[t] = bk.y * a.qscale;
      bv0[t] = bv.x;
      bv1[t] = bv.y;
    }
    dk[t] = f4z();
    dv[t] = f4z();
  }
  typedef typename std::conditional<BF, float4, float2>::type PT;
  struct T6 {
    PT q, o;
    float4 qt, ot, nl, nd;
  };
  auto ldp = [&](Rsrc r, int off) {
    if constexpr (BF) return bl4(r, op, off); else return bl2(r, op, off);
  };
  auto load = [&](int q0) {
    const int ob = min(q0 * 32, (Nq - 16) * 32), os_ = min(q0 * 4, (Nq - 16) * 4);
    T6 x;
    x.q = ldp(rq, ob);
    x.o = ldp(ro, ob);
    x.qt = bl4(rqt, oq, ob);
    x.ot = bl4(rot, oq, ob);
    x.nl = bl4(rl, os, os_);
    x.nd = bl4(rd, os, os_);
    return x;
  };
  auto tile = [&](const T6& x, int q0) {
    const bool full = q0 >= sp.ilo && q0 + 16 <= sp.ihi && q0 + 16 <= sp.ce;
    const f4v nl = f4v{x.nl.x, x.nl.y, x.nl.z, x.nl.w}, nd = f4v{x.nd.x, x.nd.y, x.nd.z, x.nd.w};
    f4v s[RT], dp[RT];
    if constexpr (BF) {
      const s4v qa = pk4z(x.q, lo2), oa = pk4z(x.o, lo2);
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        s[t] = mfma_bf(qa, kb4[t], nl);
        dp[t] = mfma_bf(oa, vb4[t], nd);
      }
    } else {
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        s[t] = mfma(x.q.x, bk0[t], nl);
        dp[t] = mfma(x.o.x, bv0[t], nd);
      }
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        s[t] = mfma(x.q.y, bk1[t], s[t]);
        dp[t] = mfma(x.o.y, bv1[t], dp[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      float p[4], ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) p[r] = fexp2(s[t][r]);
      if (!full) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qq = q0 + 4 * g + r;
          if (!(qq >= sp.b[t] && qq < sp.e[t] && qq < sp.ce)) p[r] = 0.f;
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) ds[r] = p[r] * dp[t][r];
      if constexpr (BF) {
        dv[t] = mfma_bf(pk4(x.ot), pk4(p[0], p[1], p[2], p[3]), dv[t]);
        dk[t] = mfma_bf(pk4(x.qt), pk4(ds[0], ds[1], ds[2], ds[3]), dk[t]);
      } else {
        dv[t] = mfma(x.ot.x, p[0], dv[t]);
        dk[t] = mfma(x.qt.x, ds[0], dk[t]);
        dv[t] = mfma(x.ot.y, p[1], dv[t]);
        dk[t] = mfma(x.qt.y, ds[1], dk[t]);
        dv[t] = mfma(x.ot.z, p[2], dv[t]);
        dk[t] = mfma(x.qt.z, ds[2], dk[t]);
        dv[t] = mfma(x.ot.w, p[3], dv[t]);
        dk[t] = mfma(x.qt.w, ds[3], dk[t]);
      }
    }
  };
  T6 xa = load(sp.cb);
  __builtin_amdgcn_sched_barrier(0);
  T6 xb = load(sp.cb + 16);
  __builtin_amdgcn_sched_barrier(0);
  for (int q0 = sp.cb; q0 < sp.ce; q0 += 32) {
    tile(xa, q0);
    xa = load(q0 + 32);
    __builtin_amdgcn_sched_barrier(0);
    tile(xb, q0 + 16);
    xb = load(q0 + 48);
    __builtin_amdgcn_sched_barrier(0);
  }
  // red [W][RT][16 rows][16]: (dK^T | dV^T) rows 4g + r (g < 2) of column i
  if (g < 2) {
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        red[((w * RT + t) * 16 + i) * 16 + 4 * g + r] = dk[t][r];
        red[((w * RT + t) * 16 + i) * 16 + 8 + 4 * g + r] = dv[t][r];
      }
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < RT * 256; idx += 64 * W) {
    const int t = idx >> 8, ki = (idx >> 4) & 15, c = idx & 15;
    float v = 0.f;
#pragma unroll
    for (int u = 0; u < W; ++u) v += red[((u * RT + t) * 16 + ki) * 16 + c];
    const int k = base + 16 * t + ki;
    if (k < N) {
      const int F = 8 * a.H;
      // dK at column F + 8h + d (x scale), dV at 2F + 8h + d
      a.dqkv[(int64_t)k * 3 * F + (c < 8 ? F : 2 * F) + h * 8 + (c & 7)] = c < 8 ? v * a.scale : v;
    }
  }
}

template <int RT, int W, bool BF = false>
__global__ void __launch_bounds__(64 * W) attn8_bwd2_kernel(A8Bwd2 a) {
  __shared__ float red[W * RT * 16 * 16];
  if ((int)blockIdx.x < a.nbq)
    attn8_bwd2_dq<RT, W, BF>(a, blockIdx.x, red);
  else
    attn8_bwd2_dkv<RT, W, BF>(a, blockIdx.x - a.nbq, red);
}

// ----------------------------------------------------- v3: persistent, cost-balanced (batch scope)
// The v2 grids are (row tiles x heads) workgroups of W waves: at the OC20 shape that is
// 1,160-1,264 workgroups for 1,024 resident slots, so the chip runs a full round and then a
// second round on a fraction of its CUs (profiled: 4-5 of 8 waves per SIMD resident on
// average over the launch).  v3 launches ONE 16-wave workgroup per CU and deals the work
// out by cost:
//   * a UNIT is one (head, 16-row tile) of the outer index (queries for the forward and the
//     dQ pass, keys for the dK/dV pass); its cost is the number of 16-wide tiles of the other
//     index in its segment span.  Units are ordered head-major, tile-minor, and their costs
//     have a closed form for the batch-scope layouts (one segment [0, N), or the valid
//     segment [0, nv) + the padding segment [nv, N), nv read on the device);
//   * workgroup b owns the whole units whose flattened start is nearest to b * T / G
//     (T = total cost): no unit is split across workgroups (no inter-workgroup hand-off), and
//     the makespan is within half a unit of T / G;
//   * the workgroup takes its units in GROUPS of up to R consecutive units of one head and
//     one span type (R = 5 forward, 3 dQ and dK/dV: register budget of 4 waves per SIMD).  Every wave of the workgroup owns a
//     1/16 slice of the group's span and runs it for ALL units of the group: each K/V (or
//     Q/dO) fragment it loads feeds R independent MFMA chains (R x less operand traffic than
//     one tile per wave, and R chains of instruction-level parallelism).  The 16 per-wave
//     partial results of a unit meet in LDS and are merged in wave order (deterministic).
// (A first v3 split each workgroup's tile range contiguously over its waves, one unit per
// wave at a time: 4 waves per SIMD streaming private key ranges spent 42 % of their cycles
// waiting on loads and ran the forward in 35 us against v2's 31 us.)
// The backward flattens [dQ units | dK/dV units] with tile weights 2 : 3 (8 vs 12 MFMAs).
// Tile bodies as v2 (fp32 16x16x4 MFMA, deferred-rescale softmax, accumulator-seeded LSE).
constexpr int kNW3 = 16;   // waves per v3 workgroup
// group-size caps (register budget of 4 waves per SIMD): RF forward, RQ dQ, RK dK/dV

// closed-form unit costs of a batch-scope layout (segments [0, nv) and [nv, N))
struct BPlan {
  int N, nv, nqt, nvt, bnd, cv, ca, cp, plo, Tq;
  __device__ __forceinline__ void init(int N_, int nv_) {
    N = N_;
    nv = min(max(nv_, 0), N_);
    nqt = (N + 15) >> 4;
    bnd = (nv < N && (nv & 15)) ? 1 : 0;        // one tile holds rows of both segments
    nvt = nv == N ? nqt : (nv >> 4);            // tiles whose rows are all valid
    cv = (nv + 15) >> 4;                        // span [0, nv)
    ca = nqt;                                   // span [0, N)
    plo = nv >> 4;                              // padding span starts at tile nv / 16
    cp = nqt - plo;                             // span [16 plo, N)
    Tq = pre(nqt);
  }
  // arithmetic selects: a select of two fields lets the compiler select their ADDRESSES,
  // which pins the whole plan in (LDS-promoted) private memory
  __device__ __forceinline__ int cost(int t) const {
    const int v = t < nvt ? 1 : 0, a = (bnd && t == nvt) ? 1 : 0;
    return cp + v * (cv - cp) + a * (ca - cp);
  }
  // 0 valid, 1 boundary, 2 padding (units of one type share span and masks)
  __device__ __forceinline__ int type(int t) const { return t < nvt ? 0 : ((bnd && t == nvt) ? 1 : 2); }
  __device__ __forceinline__ int lo(int t) const { return (t < nvt + bnd ? 0 : 16) * plo; }
  __device__ __forceinline__ int pre(int t) const {
    if (t <= nvt) return t * cv;
    int p = nvt * cv, r = t - nvt;
    if (bnd) {
      p += ca;
      r -= 1;
    }
    return p + r * cp;
  }
  // y in [0, Tq) -> (tile t, tile k of its span)
  __device__ __forceinline__ void decode(int y, int& t, int& k) const {
    const int a = nvt * cv;
    if (y < a) {
      t = y / cv;
      k = y - t * cv;
      return;
    }
    y -= a;
    if (bnd) {
      if (y < ca) {
        t = nvt;
        k = y;
        return;
      }
      y -= ca;
    }
    t = nvt + bnd + y / cp;
    k = y - (t - nvt - bnd) * cp;
  }
  // segment span of row r (empty for r >= N) and the intersection [ilo, ihi) over the
  // valid rows of tile t (empty when the tile holds rows of both segments)
  __device__ __forceinline__ void row_span(int r, int& b, int& e) const {
    b = r < nv ? 0 : (r < N ? nv : N);
    e = r < nv ? nv : (r < N ? N : 0);
  }
  __device__ __forceinline__ void tile_isect(int t, int& ilo, int& ihi) const {
    const int ty = type(t);
    ilo = ty == 0 ? 0 : nv;
    ihi = ty == 0 ? nv : (ty == 1 ? nv : N);
  }
};

// the unit boundary nearest to tile j of the flattened tile space of one or two unit kinds
// (tiles [0, D) of kind 0, [D, 2D) of kind 1; D = H * Tq): returns a unit index
__device__ __forceinline__ int nearest_unit(BPlan P, int D, int H, int j, int ntiles) {
  if (j >= ntiles) return (ntiles / D) * H * P.nqt;
  const int kind = j < D ? 0 : 1, jj = j - kind * D;
  const int h = jj / P.Tq;
  int t, k;
  P.decode(jj - h * P.Tq, t, k);
  return kind * H * P.nqt + h * P.nqt + t + (2 * k > P.cost(t) ? 1 : 0);
}

__device__ __forceinline__ float4 f4scale(f4v v, float s) { return make_float4(v[0] * s, v[1] * s, v[2] * s, v[3] * s); }

// one wave, R query tiles [t0, t0 + R) of head h against key tiles [kb0, kb1) of their span:
// per-unit partial (m, l, o[8]) into LDS pr[R][16][10]
template <int R>
__device__ __forceinline__ void fwd3_group(const float* __restrict__ Qp, Rsrc rk, Rsrc rv, int64_t hb, int Nq,
                                           const BPlan& P, int t0, int klo, int kb0, int kb1, float qscale,
                                           int i, int g, float* __restrict__ pr) {
  const int ok_ = off_pair(i, g), ov_ = off_quad(i, g);
  const int cmax = (Nq - 16) * 32;
  int ilo, ihi;
  P.tile_isect(t0, ilo, ihi);
  const int cb = klo + 16 * kb0, ce = klo + 16 * kb1;
  float bq0[R], bq1[R], m[R], thr[R], l[R];
  f4v o[R], cin[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int row = 16 * (t0 + j) + i;
    const float2 bq = ld2(Qp + hb + (int64_t)min(row, Nq - 1) * 8 + 2 * g);
    bq0[j] = bq.x * qscale;
    bq1[j] = bq.y * qscale;
    m[j] = -INFINITY;
    thr[j] = -INFINITY;
    l[j] = 0.f;
    o[j] = f4z();
    cin[j] = f4z();
  }
  auto tile = [&](float2 kk, float4 vv, int k0) {
    const bool full = k0 >= ilo && k0 + 16 <= ihi && k0 + 16 <= ce;
    f4v s[R];
    auto scores = [&]() {
#pragma unroll
      for (int j = 0; j < R; ++j) s[j] = mfma(kk.x, bq0[j], cin[j]);
#pragma unroll
      for (int j = 0; j < R; ++j) s[j] = mfma(kk.y, bq1[j], s[j]);
      if (!full) {
#pragma unroll
        for (int j = 0; j < R; ++j) {
          int rb, re;
          P.row_span(16 * (t0 + j) + i, rb, re);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = k0 + 4 * g + r;
            if (!(key >= rb && key < re && key < ce)) s[j][r] = -INFINITY;
          }
        }
      }
    };
    scores();
    bool trig = false;
#pragma unroll
    for (int j = 0; j < R; ++j) trig |= max4(s[j]) > thr[j];
    if (__any(trig)) {
      // move the row references (rare: a score beyond the reference by > kTau), rescale
      // o and l, and re-issue the score MFMAs against the new reference (keeps s in place)
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const float base = -cin[j][0];
        const float mn = fmaxf(m[j], wmax16(max4(s[j])) + base);
        if (mn > -INFINITY) {
          const float f = fexp2(m[j] - mn);
          o[j] = o[j] * f;
          l[j] *= f;
          m[j] = mn;
          thr[j] = kTau;
          cin[j] = f4v{-mn, -mn, -mn, -mn};
        }
      }
      scores();
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const float p0 = fexp2(s[j][0]), p1 = fexp2(s[j][1]), p2 = fexp2(s[j][2]), p3 = fexp2(s[j][3]);
      o[j] = mfma(vv.x, p0, o[j]);
      o[j] = mfma(vv.y, p1, o[j]);
      o[j] = mfma(vv.z, p2, o[j]);
      o[j] = mfma(vv.w, p3, o[j]);
      l[j] += (p0 + p1) + (p2 + p3);
    }
  };
  if (cb < ce) {
    float2 ka = bl2(rk, ok_, min(cb * 32, cmax));
    float4 va = bl4(rv, ov_, min(cb * 32, cmax));
    __builtin_amdgcn_sched_barrier(0);
    float2 kb = bl2(rk, ok_, min(cb * 32 + 512, cmax));
    float4 vb = bl4(rv, ov_, min(cb * 32 + 512, cmax));
    __builtin_amdgcn_sched_barrier(0);
    for (int k0 = cb; k0 < ce; k0 += 32) {
      tile(ka, va, k0);
      ka = bl2(rk, ok_, min(k0 * 32 + 1024, cmax));
      va = bl4(rv, ov_, min(k0 * 32 + 1024, cmax));
      __builtin_amdgcn_sched_barrier(0);
      if (k0 + 16 < ce) tile(kb, vb, k0 + 16);
      kb = bl2(rk, ok_, min(k0 * 32 + 1536, cmax));
      vb = bl4(rv, ov_, min(k0 * 32 + 1536, cmax));
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int j = 0; j < R; ++j) {
    float lt = l[j] + __shfl_xor(l[j], 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    float* q = pr + (j * 16 + i) * 10;
    if (g < 2) {
#pragma unroll
      for (int r = 0; r < 4; ++r) q[2 + 4 * g + r] = o[j][r];
    } else if (g == 2) {
      q[0] = m[j];
      q[1] = lt;
    }
  }
}

// forward: O [N, 8H], NL [H][Nq] (-LSE2; rows N..Nq: 0)
template <int kRF>
__global__ void __launch_bounds__(64 * kNW3) attn8_fwd3_kernel(const float* __restrict__ Qp,
                                                               const float* __restrict__ Kp,
                                                               const float* __restrict__ Vq, int N, int Nq, int H,
                                                               const int* __restrict__ seg_ptr, int nseg,
                                                               float qscale, float* __restrict__ O,
                                                               float* __restrict__ NL) {
  __shared__ float red[kNW3][kRF][16][10];
  // the wave index is uniform: readfirstlane keeps the group loop scalar (no exec branches)
  const int w = uni(threadIdx.x >> 6), lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  BPlan P;
  P.init(N, nseg >= 2 ? seg_ptr[1] : N);
  const int nqt = P.nqt, ntiles = H * P.Tq, G = gridDim.x, b = blockIdx.x;
  const int uA = uni(b == 0 ? 0 : nearest_unit(P, ntiles, H, (int)((int64_t)b * ntiles / G), ntiles));
  const int uB = uni(b + 1 >= G ? H * nqt : nearest_unit(P, ntiles, H, (int)((int64_t)(b + 1) * ntiles / G), ntiles));
  for (int u = uA; u < uB;) {
    const int h = uni(u / nqt), t0 = uni(u - h * nqt), ty = P.type(t0);
    int R = 1;
    while (R < kRF && u + R < uB && t0 + R < nqt && P.type(t0 + R) == ty) ++R;
    R = uni(R);
    const int cost = P.cost(t0), klo = P.lo(t0);
    const int kb0 = uni(w * cost / kNW3), kb1 = uni((w + 1) * cost / kNW3);
    const int64_t hb = (int64_t)h * Nq * 8;
    const Rsrc rk = mk_rsrc(Kp + hb, Nq * 8), rv = mk_rsrc(Vq + hb, Nq * 8);
    float* pr = &red[w][0][0][0];
    switch (R) {
      case 1: if constexpr (kRF >= 1) fwd3_group<1>(Qp, rk, rv, hb, Nq, P, t0, klo, kb0, kb1, qscale, i, g, pr); break;
      case 2: if constexpr (kRF >= 2) fwd3_group<2>(Qp, rk, rv, hb, Nq, P, t0, klo, kb0, kb1, qscale, i, g, pr); break;
      case 3: if constexpr (kRF >= 3) fwd3_group<3>(Qp, rk, rv, hb, Nq, P, t0, klo, kb0, kb1, qscale, i, g, pr); break;
      case 4: if constexpr (kRF >= 4) fwd3_group<4>(Qp, rk, rv, hb, Nq, P, t0, klo, kb0, kb1, qscale, i, g, pr); break;
      case 5: if constexpr (kRF >= 5) fwd3_group<5>(Qp, rk, rv, hb, Nq, P, t0, klo, kb0, kb1, qscale, i, g, pr); break;
      default: break;
    }
    __syncthreads();
    // merge the 16 wave partials of each unit in wave order: thread -> (unit, query, d)
    for (int idx = threadIdx.x; idx < R * 128; idx += 64 * kNW3) {
      const int j = idx >> 7, qi = (idx >> 3) & 15, d = idx & 7;
      float M = -INFINITY;
#pragma unroll 4
      for (int v = 0; v < kNW3; ++v) M = fmaxf(M, red[v][j][qi][0]);
      float lsum = 0.f, a = 0.f;
      if (M > -INFINITY) {
#pragma unroll 4
        for (int v = 0; v < kNW3; ++v) {
          const float f = fexp2(red[v][j][qi][0] - M);
          lsum = fmaf(red[v][j][qi][1], f, lsum);
          a = fmaf(red[v][j][qi][2 + d], f, a);
        }
      }
      const int q = 16 * (t0 + j) + qi;
      if (q < N) {
        O[(int64_t)q * 8 * H + h * 8 + d] = lsum > 0.f ? a * (1.f / lsum) : 0.f;
        if (d == 0) NL[(int64_t)h * Nq + q] = lsum > 0.f ? -(M + __log2f(lsum)) : INFINITY;
      } else if (q < Nq && d == 0) {
        NL[(int64_t)h * Nq + q] = 0.f;
      }
    }
    __syncthreads();
    u += R;
  }
}

// one wave, R query tiles of head h (dQ) against key tiles [kb0, kb1) of their span
template <int R>
__device__ __forceinline__ void dq3_group(const A8Bwd2& a, int64_t hb, int h, const BPlan& P, int t0, int klo,
                                          int kb0, int kb1, int i, int g, float* __restrict__ pr) {
  const int Nq = a.Nq, N = a.N;
  const int op = off_pair(i, g), oq = off_quad(i, g);
  const int cmax = (Nq - 16) * 32;
  int ilo, ihi;
  P.tile_isect(t0, ilo, ihi);
  const int cb = klo + 16 * kb0, ce = klo + 16 * kb1;
  const Rsrc rk = mk_rsrc(a.Kp + hb, Nq * 8), rv = mk_rsrc(a.Vp + hb, Nq * 8), rkt = mk_rsrc(a.Kq + hb, Nq * 8);
  float bq0[R], bq1[R], bo0[R], bo1[R];
  f4v cs[R], cd[R], dq[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int row = 16 * (t0 + j) + i, rc = min(row, Nq - 1);
    const float2 bq = ld2(a.Qp + hb + (int64_t)rc * 8 + 2 * g);
    const float2 bo = ld2(a.dOp + hb + (int64_t)rc * 8 + 2 * g);
    bq0[j] = bq.x * a.qscale;
    bq1[j] = bq.y * a.qscale;
    bo0[j] = bo.x;
    bo1[j] = bo.y;
    const float nl = row < N ? a.NL[(int64_t)h * Nq + row] : 0.f;
    const float nd = row < N ? a.ndelta[(int64_t)h * Nq + row] : 0.f;
    cs[j] = f4v{nl, nl, nl, nl};
    cd[j] = f4v{nd, nd, nd, nd};
    dq[j] = f4z();
  }
  auto tile = [&](float2 kk, float2 vv, float4 kt, int k0) {
    const bool full = k0 >= ilo && k0 + 16 <= ihi && k0 + 16 <= ce;
    f4v s[R], dp[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      s[j] = mfma(kk.x, bq0[j], cs[j]);
      dp[j] = mfma(vv.x, bo0[j], cd[j]);
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      s[j] = mfma(kk.y, bq1[j], s[j]);
      dp[j] = mfma(vv.y, bo1[j], dp[j]);
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      float ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) ds[r] = fexp2(s[j][r]) * dp[j][r];
      if (!full) {
        int rb, re;
        P.row_span(16 * (t0 + j) + i, rb, re);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + 4 * g + r;
          if (!(key >= rb && key < re && key < ce)) ds[r] = 0.f;
        }
      }
      dq[j] = mfma(kt.x, ds[0], dq[j]);
      dq[j] = mfma(kt.y, ds[1], dq[j]);
      dq[j] = mfma(kt.z, ds[2], dq[j]);
      dq[j] = mfma(kt.w, ds[3], dq[j]);
    }
  };
  if (cb < ce) {
    int o0 = min(cb * 32, cmax), o1 = min(cb * 32 + 512, cmax);
    float2 ka = bl2(rk, op, o0), va = bl2(rv, op, o0);
    float4 ta = bl4(rkt, oq, o0);
    __builtin_amdgcn_sched_barrier(0);
    float2 kb = bl2(rk, op, o1), vb = bl2(rv, op, o1);
    float4 tb = bl4(rkt, oq, o1);
    __builtin_amdgcn_sched_barrier(0);
    for (int k0 = cb; k0 < ce; k0 += 32) {
      tile(ka, va, ta, k0);
      o0 = min(k0 * 32 + 1024, cmax);
      ka = bl2(rk, op, o0);
      va = bl2(rv, op, o0);
      ta = bl4(rkt, oq, o0);
      __builtin_amdgcn_sched_barrier(0);
      if (k0 + 16 < ce) tile(kb, vb, tb, k0 + 16);
      o1 = min(k0 * 32 + 1536, cmax);
      kb = bl2(rk, op, o1);
      vb = bl2(rv, op, o1);
      tb = bl4(rkt, oq, o1);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (g < 2) {
#pragma unroll
    for (int j = 0; j < R; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) pr[(j * 16 + i) * 16 + 4 * g + r] = dq[j][r];
  }
}

// one wave, R key tiles of head h (dK, dV) against query tiles [kb0, kb1) of their span
template <int R>
__device__ __forceinline__ void dkv3_group(const A8Bwd2& a, int64_t hb, int h, const BPlan& P, int t0, int klo,
                                           int kb0, int kb1, int i, int g, float* __restrict__ pr) {
  const int Nq = a.Nq;
  const int op = off_pair(i, g), oq = off_quad(i, g), os = 16 * g;
  const int cmax = (Nq - 16) * 32;
  int ilo, ihi;
  P.tile_isect(t0, ilo, ihi);
  const int cb = klo + 16 * kb0, ce = klo + 16 * kb1;
  const Rsrc rq = mk_rsrc(a.Qp + hb, Nq * 8), ro = mk_rsrc(a.dOp + hb, Nq * 8);
  const Rsrc rqt = mk_rsrc(a.Qq + hb, Nq * 8), rot = mk_rsrc(a.dOq + hb, Nq * 8);
  const Rsrc rl = mk_rsrc(a.NL + (int64_t)h * Nq, Nq), rd = mk_rsrc(a.ndelta + (int64_t)h * Nq, Nq);
  float bk0[R], bk1[R], bv0[R], bv1[R];
  f4v dk[R], dv[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int row = 16 * (t0 + j) + i, rc = min(row, Nq - 1);
    const float2 bk = ld2(a.Kp + hb + (int64_t)rc * 8 + 2 * g);
    const float2 bv = ld2(a.Vp + hb + (int64_t)rc * 8 + 2 * g);
    bk0[j] = bk.x * a.qscale;
    bk1[j] = bk.y * a.qscale;
    bv0[j] = bv.x;
    bv1[j] = bv.y;
    dk[j] = f4z();
    dv[j] = f4z();
  }
  struct T6 {
    float2 q, o;
    float4 qt, ot, nl, nd;
  };
  auto load = [&](int q0) {
    const int ob = min(q0 * 32, cmax), os_ = min(q0 * 4, (Nq - 16) * 4);
    T6 x;
    x.q = bl2(rq, op, ob);
    x.o = bl2(ro, op, ob);
    x.qt = bl4(rqt, oq, ob);
    x.ot = bl4(rot, oq, ob);
    x.nl = bl4(rl, os, os_);
    x.nd = bl4(rd, os, os_);
    return x;
  };
  auto tile = [&](const T6& x, int q0) {
    const bool full = q0 >= ilo && q0 + 16 <= ihi && q0 + 16 <= ce;
    const f4v nl = f4v{x.nl.x, x.nl.y, x.nl.z, x.nl.w}, nd = f4v{x.nd.x, x.nd.y, x.nd.z, x.nd.w};
    f4v s[R], dp[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      s[j] = mfma(x.q.x, bk0[j], nl);
      dp[j] = mfma(x.o.x, bv0[j], nd);
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      s[j] = mfma(x.q.y, bk1[j], s[j]);
      dp[j] = mfma(x.o.y, bv1[j], dp[j]);
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      float p[4], ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) p[r] = fexp2(s[j][r]);
      if (!full) {
        int rb, re;
        P.row_span(16 * (t0 + j) + i, rb, re);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qq = q0 + 4 * g + r;
          if (!(qq >= rb && qq < re && qq < ce)) p[r] = 0.f;
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) ds[r] = p[r] * dp[j][r];
      dv[j] = mfma(x.ot.x, p[0], dv[j]);
      dk[j] = mfma(x.qt.x, ds[0], dk[j]);
      dv[j] = mfma(x.ot.y, p[1], dv[j]);
      dk[j] = mfma(x.qt.y, ds[1], dk[j]);
      dv[j] = mfma(x.ot.z, p[2], dv[j]);
      dk[j] = mfma(x.qt.z, ds[2], dk[j]);
      dv[j] = mfma(x.ot.w, p[3], dv[j]);
      dk[j] = mfma(x.qt.w, ds[3], dk[j]);
    }
  };
  if (cb < ce) {
    T6 xa = load(cb);
    __builtin_amdgcn_sched_barrier(0);
    T6 xb = load(cb + 16);
    __builtin_amdgcn_sched_barrier(0);
    for (int q0 = cb; q0 < ce; q0 += 32) {
      tile(xa, q0);
      xa = load(q0 + 32);
      __builtin_amdgcn_sched_barrier(0);
      if (q0 + 16 < ce) tile(xb, q0 + 16);
      xb = load(q0 + 48);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (g < 2) {
#pragma unroll
    for (int j = 0; j < R; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pr[(j * 16 + i) * 16 + 4 * g + r] = dk[j][r];
        pr[(j * 16 + i) * 16 + 8 + 4 * g + r] = dv[j][r];
      }
  }
}

// backward: dqkv [N, 24H] = [dQ | dK | dV] (dQ, dK scaled by `scale`).  Units: dQ units
// [0, H nqt), dK/dV units [H nqt, 2 H nqt); flattened tile weights 2 and 3.
template <int kRQ, int kRK>
__global__ void __launch_bounds__(64 * kNW3) attn8_bwd3_kernel(A8Bwd2 a, int nseg) {
  __shared__ float red[kNW3][kRK > kRQ ? kRK : kRQ][16][16];
  const int w = uni(threadIdx.x >> 6), lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int N = a.N, Nq = a.Nq, H = a.H, F = 8 * H;
  BPlan P;
  P.init(N, nseg >= 2 ? a.seg_ptr[1] : N);
  const int nqt = P.nqt, D = H * P.Tq, G = gridDim.x, b = blockIdx.x, U = H * nqt;
  const int64_t wtot = 5LL * D;
  auto tile_at = [D](int64_t z) -> int {
    return z <= 2LL * D ? (int)((z + 1) / 2) : D + (int)((z - 2LL * D + 2) / 3);
  };
  const int uA = uni(b == 0 ? 0 : nearest_unit(P, D, H, tile_at((int64_t)b * wtot / G), 2 * D));
  const int uB = uni(b + 1 >= G ? 2 * U : nearest_unit(P, D, H, tile_at((int64_t)(b + 1) * wtot / G), 2 * D));
  for (int u = uA; u < uB;) {
    const int kind = u < U ? 0 : 1, uu = u - kind * U;
    const int h = uni(uu / nqt), t0 = uni(uu - h * nqt), ty = P.type(t0);
    const int rmax = kind == 0 ? kRQ : kRK;
    int R = 1;
    while (R < rmax && u + R < uB && t0 + R < nqt && (u + R < U) == (kind == 0) && P.type(t0 + R) == ty) ++R;
    R = uni(R);
    const int cost = P.cost(t0), klo = P.lo(t0);
    const int kb0 = uni(w * cost / kNW3), kb1 = uni((w + 1) * cost / kNW3);
    const int64_t hb = (int64_t)h * Nq * 8;
    float* pr = &red[w][0][0][0];
    if (kind == 0) {
      switch (R) {
        case 1: if constexpr (kRQ >= 1) dq3_group<1>(a, hb, h, P, t0, klo, kb0, kb1, i, g, pr); break;
        case 2: if constexpr (kRQ >= 2) dq3_group<2>(a, hb, h, P, t0, klo, kb0, kb1, i, g, pr); break;
        case 3: if constexpr (kRQ >= 3) dq3_group<3>(a, hb, h, P, t0, klo, kb0, kb1, i, g, pr); break;
        case 4: if constexpr (kRQ >= 4) dq3_group<4>(a, hb, h, P, t0, klo, kb0, kb1, i, g, pr); break;
        case 5: if constexpr (kRQ >= 5) dq3_group<5>(a, hb, h, P, t0, klo, kb0, kb1, i, g, pr); break;
        default: break;
      }
    } else {
      switch (R) {
        case 1: if constexpr (kRK >= 1) dkv3_group<1>(a, hb, h, P, t0, klo, kb0, kb1, i, g, pr); break;
        case 2: if constexpr (kRK >= 2) dkv3_group<2>(a, hb, h, P, t0, klo, kb0, kb1, i, g, pr); break;
        case 3: if constexpr (kRK >= 3) dkv3_group<3>(a, hb, h, P, t0, klo, kb0, kb1, i, g, pr); break;
        case 4: if constexpr (kRK >= 4) dkv3_group<4>(a, hb, h, P, t0, klo, kb0, kb1, i, g, pr); break;
        case 5: if constexpr (kRK >= 5) dkv3_group<5>(a, hb, h, P, t0, klo, kb0, kb1, i, g, pr); break;
        default: break;
      }
    }
    __syncthreads();
    // sum the 16 wave partials in wave order: thread -> (unit, row, column)
    const int ncol = kind == 0 ? 8 : 16;
    for (int idx = threadIdx.x; idx < R * 16 * ncol; idx += 64 * kNW3) {
      const int j = idx / (16 * ncol), rr = idx - j * 16 * ncol, ri = rr / ncol, c = rr - ri * ncol;
      float v = 0.f;
#pragma unroll 4
      for (int x = 0; x < kNW3; ++x) v += red[x][j][ri][c];
      const int row = 16 * (t0 + j) + ri;
      if (row < N) {
        float* dst = a.dqkv + (int64_t)row * 3 * F + h * 8 + (c & 7);
        if (kind == 0)
          dst[0] = v * a.scale;
        else if (c < 8)
          dst[F] = v * a.scale;
        else
          dst[2 * F] = v;
      }
    }
    __syncthreads();
    u += R;
  }
}

// Backward v2 on quad-block MFMAs (fp32): the three 8-wide products (dQ, dK, dV), which
// waste half of every 16x16x4, run as v_mfma_f32_4x4x1_16b_f32 blocks with the lane's own
// dS / P value as the A operand and quad-layout float4s as B (as attn8_fwd2q_kernel).
template <int W>
__device__ __forceinline__ void attn8_bwd2q_dq(const A8Bwd2& a, int bx, float* red) {
  const int h = blockIdx.y;
  const int w = uni(threadIdx.x >> 6), lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int N = a.N, Nq = a.Nq;
  const int base = bx * 16;
  const SpanR<1> sp = span_rt<1>(base, i, N, a.seg_id, a.seg_ptr, W, w);
  const int64_t hb = (int64_t)h * Nq * 8;
  const Rsrc rk = mk_rsrc(a.Kp + hb, Nq * 8), rv = mk_rsrc(a.Vp + hb, Nq * 8), rkt = mk_rsrc(a.Kq + hb, Nq * 8);
  const int op = off_pair(i, g), oq0 = (32 * g + 4 * (i & 3)) * 4, oq1 = oq0 + 64;
  const int q = sp.row[0], qc = min(q, Nq - 1);
  const float2 bq = ld2(a.Qp + hb + (int64_t)qc * 8 + 2 * g);
  const float2 bo = ld2(a.dOp + hb + (int64_t)qc * 8 + 2 * g);
  const float bq0 = bq.x * a.qscale, bq1 = bq.y * a.qscale, bo0 = bo.x, bo1 = bo.y;
  const float nl = q < N ? a.NL[(int64_t)h * Nq + q] : 0.f;
  const float nd = q < N ? a.ndelta[(int64_t)h * Nq + q] : 0.f;
  const f4v cs = f4v{nl, nl, nl, nl}, cd = f4v{nd, nd, nd, nd};
  f4v dq0 = f4z(), dq1 = f4z();
  struct T {
    float2 k, v;
    float4 t0, t1;
  };
  auto load = [&](int k0) {
    const int o = min(k0 * 32, (Nq - 16) * 32);
    T x;
    x.k = bl2(rk, op, o);
    x.v = bl2(rv, op, o);
    x.t0 = bl4(rkt, oq0, o);
    x.t1 = bl4(rkt, oq1, o);
    return x;
  };
  auto tile = [&](const T& x, int k0) {
    f4v s = mfma(x.k.x, bq0, cs), dp = mfma(x.v.x, bo0, cd);
    s = mfma(x.k.y, bq1, s);
    dp = mfma(x.v.y, bo1, dp);
    float ds[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) ds[r] = fexp2(s[r]) * dp[r];
    const bool full = k0 >= sp.ilo && k0 + 16 <= sp.ihi && k0 + 16 <= sp.ce;
    if (!full) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + 4 * g + r;
        if (!(key >= sp.b[0] && key < sp.e[0] && key < sp.ce)) ds[r] = 0.f;
      }
    }
    dq0 = mfma4(x.t0.x, ds[0], dq0);
    dq1 = mfma4(x.t1.x, ds[0], dq1);
    dq0 = mfma4(x.t0.y, ds[1], dq0);
    dq1 = mfma4(x.t1.y, ds[1], dq1);
    dq0 = mfma4(x.t0.z, ds[2], dq0);
    dq1 = mfma4(x.t1.z, ds[2], dq1);
    dq0 = mfma4(x.t0.w, ds[3], dq0);
    dq1 = mfma4(x.t1.w, ds[3], dq1);
  };
  T xa = load(sp.cb);
  __builtin_amdgcn_sched_barrier(0);
  T xb = load(sp.cb + 16);
  __builtin_amdgcn_sched_barrier(0);
  for (int k0 = sp.cb; k0 < sp.ce; k0 += 32) {
    tile(xa, k0);
    xa = load(k0 + 32);
    __builtin_amdgcn_sched_barrier(0);
    tile(xb, k0 + 16);
    xb = load(k0 + 48);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    dq0[r] += __shfl_xor(dq0[r], 16, 64);
    dq0[r] += __shfl_xor(dq0[r], 32, 64);
    dq1[r] += __shfl_xor(dq1[r], 16, 64);
    dq1[r] += __shfl_xor(dq1[r], 32, 64);
  }
  // red [W][16 rows][8]: lane i of group 0 holds query i, dims r and 4 + r
  if (g == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      red[(w * 16 + i) * 8 + r] = dq0[r];
      red[(w * 16 + i) * 8 + 4 + r] = dq1[r];
    }
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < 128; idx += 64 * W) {
    const int qi = idx >> 3, d = idx & 7;
    float v = 0.f;
#pragma unroll
    for (int u = 0; u < W; ++u) v += red[(u * 16 + qi) * 8 + d];
    const int qq = base + qi;
    if (qq < N) a.dqkv[(int64_t)qq * 24 * a.H + h * 8 + d] = v * a.scale;
  }
}

template <int W>
__device__ __forceinline__ void attn8_bwd2q_dkv(const A8Bwd2& a, int bx, float* red) {
  const int h = blockIdx.y;
  const int w = uni(threadIdx.x >> 6), lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int N = a.N, Nq = a.Nq;
  const int base = bx * 16;
  const SpanR<1> sp = span_rt<1>(base, i, N, a.seg_id, a.seg_ptr, W, w);
  const int64_t hb = (int64_t)h * Nq * 8;
  const Rsrc rq = mk_rsrc(a.Qp + hb, Nq * 8), ro = mk_rsrc(a.dOp + hb, Nq * 8);
  const Rsrc rqt = mk_rsrc(a.Qq + hb, Nq * 8), rot = mk_rsrc(a.dOq + hb, Nq * 8);
  const Rsrc rl = mk_rsrc(a.NL + (int64_t)h * Nq, Nq), rd = mk_rsrc(a.ndelta + (int64_t)h * Nq, Nq);
  const int op = off_pair(i, g), oq0 = (32 * g + 4 * (i & 3)) * 4, oq1 = oq0 + 64, os = 16 * g;
  const int kc = min(sp.row[0], Nq - 1);
  const float2 bk = ld2(a.Kp + hb + (int64_t)kc * 8 + 2 * g);
  const float2 bv = ld2(a.Vp + hb + (int64_t)kc * 8 + 2 * g);
  const float bk0 = bk.x * a.qscale, bk1 = bk.y * a.qscale, bv0 = bv.x, bv1 = bv.y;
  f4v dk0 = f4z(), dk1 = f4z(), dv0 = f4z(), dv1 = f4z();
  struct T {
    float2 q, o;
    float4 qt0, qt1, ot0, ot1, nl, nd;
  };
  auto load = [&](int q0) {
    const int ob = min(q0 * 32, (Nq - 16) * 32), os_ = min(q0 * 4, (Nq - 16) * 4);
    T x;
    x.q = bl2(rq, op, ob);
    x.o = bl2(ro, op, ob);
    x.nl = bl4(rl, os, os_);
    x.nd = bl4(rd, os, os_);
    x.qt0 = bl4(rqt, oq0, ob);
    x.qt1 = bl4(rqt, oq1, ob);
    x.ot0 = bl4(rot, oq0, ob);
    x.ot1 = bl4(rot, oq1, ob);
    return x;
  };
  auto tile = [&](const T& x, int q0) {
    const f4v nl = f4v{x.nl.x, x.nl.y, x.nl.z, x.nl.w}, nd = f4v{x.nd.x, x.nd.y, x.nd.z, x.nd.w};
    f4v s = mfma(x.q.x, bk0, nl), dp = mfma(x.o.x, bv0, nd);
    s = mfma(x.q.y, bk1, s);
    dp = mfma(x.o.y, bv1, dp);
    float p[4], ds[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) p[r] = fexp2(s[r]);
    const bool full = q0 >= sp.ilo && q0 + 16 <= sp.ihi && q0 + 16 <= sp.ce;
    if (!full) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = q0 + 4 * g + r;
        if (!(qq >= sp.b[0] && qq < sp.e[0] && qq < sp.ce)) p[r] = 0.f;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) ds[r] = p[r] * dp[r];
    dv0 = mfma4(x.ot0.x, p[0], dv0);
    dv1 = mfma4(x.ot1.x, p[0], dv1);
    dk0 = mfma4(x.qt0.x, ds[0], dk0);
    dk1 = mfma4(x.qt1.x, ds[0], dk1);
    dv0 = mfma4(x.ot0.y, p[1], dv0);
    dv1 = mfma4(x.ot1.y, p[1], dv1);
    dk0 = mfma4(x.qt0.y, ds[1], dk0);
    dk1 = mfma4(x.qt1.y, ds[1], dk1);
    dv0 = mfma4(x.ot0.z, p[2], dv0);
    dv1 = mfma4(x.ot1.z, p[2], dv1);
    dk0 = mfma4(x.qt0.z, ds[2], dk0);
    dk1 = mfma4(x.qt1.z, ds[2], dk1);
    dv0 = mfma4(x.ot0.w, p[3], dv0);
    dv1 = mfma4(x.ot1.w, p[3], dv1);
    dk0 = mfma4(x.qt0.w, ds[3], dk0);
    dk1 = mfma4(x.qt1.w, ds[3], dk1);
  };
  T xa = load(sp.cb);
  __builtin_amdgcn_sched_barrier(0);
  T xb = load(sp.cb + 16);
  __builtin_amdgcn_sched_barrier(0);
  for (int q0 = sp.cb; q0 < sp.ce; q0 += 32) {
    tile(xa, q0);
    xa = load(q0 + 32);
    __builtin_amdgcn_sched_barrier(0);
    tile(xb, q0 + 16);
    xb = load(q0 + 48);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    dk0[r] += __shfl_xor(dk0[r], 16, 64);
    dk0[r] += __shfl_xor(dk0[r], 32, 64);
    dk1[r] += __shfl_xor(dk1[r], 16, 64);
    dk1[r] += __shfl_xor(dk1[r], 32, 64);
    dv0[r] += __shfl_xor(dv0[r], 16, 64);
    dv0[r] += __shfl_xor(dv0[r], 32, 64);
    dv1[r] += __shfl_xor(dv1[r], 16, 64);
    dv1[r] += __shfl_xor(dv1[r], 32, 64);
  }
  // red [W][16 rows][16]: (dK | dV) of key i, dims r and 4 + r
  if (g == 0) {
    float* row = red + (w * 16 + i) * 16;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      row[r] = dk0[r];
      row[4 + r] = dk1[r];
      row[8 + r] = dv0[r];
      row[12 + r] = dv1[r];
    }
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < 256; idx += 64 * W) {
    const int ki = idx >> 4, c = idx & 15;
    float v = 0.f;
#pragma unroll
    for (int u = 0; u < W; ++u) v += red[(u * 16 + ki) * 16 + c];
    const int k = base + ki;
    if (k < N) {
      const int F = 8 * a.H;
      a.dqkv[(int64_t)k * 3 * F + (c < 8 ? F : 2 * F) + h * 8 + (c & 7)] = c < 8 ? v * a.scale : v;
    }
  }
}

// QM bit 0: dQ pass on quad blocks, bit 1: dK/dV pass on quad blocks (else the v2 bodies).
// Default (HYDRA_ATTN8_QUADB) 1: the quad dK/dV body needs 28 operand registers per tile slot
// (two float4 per quad operand) against 20, which drops the kernel to 5 waves per SIMD; at the
// OC20 shape (MI355X) dQ-only measured 83.2 us against 85.6 (v2) and 90.1 (both passes).
template <int W, int QM>
__global__ void __launch_bounds__(64 * W) attn8_bwd2q_kernel(A8Bwd2 a) {
  __shared__ float red[W * 16 * 16];
  if ((int)blockIdx.x < a.nbq) {
    if constexpr (QM & 1)
      attn8_bwd2q_dq<W>(a, blockIdx.x, red);
    else
      attn8_bwd2_dq<1, W, false>(a, blockIdx.x, red);
  } else {
    if constexpr (QM & 2)
      attn8_bwd2q_dkv<W>(a, blockIdx.x - a.nbq, red);
    else
      attn8_bwd2_dkv<1, W, false>(a, blockIdx.x - a.nbq, red);
  }
}

// ------------------------------------------------------------------------------------ host
constexpr int kRT = 2;  // row tiles per wave (grid-split kernels)

static int pick_splits(int N, int H, int64_t splits) {
  if (splits > 0) return (int)splits;
  // >= ~5 waves per SIMD over 256 CUs x 4 SIMDs: blocks x H x S x 4 waves >= 5120
  const int blocks = ceil_div(N, 64 * kRT) * H;
  int S = 1;
  while (S < 16 && (int64_t)blocks * S * 4 < 5120 && N / (S * 2) >= 128) S *= 2;
  return S;
}

// v2 launch shape.  One row tile per wave (RT = 1: more rows per wave raised the register
// count and lowered occupancy, measured slower); W waves split one (row tile, head) unit's
// key (query) range.  Measured at the OC20 shape (Nq 2560, 8 heads, MI355X): W = 8 is the
// fastest both ways (fwd 31.3 us vs 31.4-41.9 for W = 2..6; bwd 85.3 vs 87.4-109), an
// occupancy-driven choice (fill exactly one round of resident workgroups) was slower; short
// key ranges (graph scope, small batches) use fewer waves so no wave runs empty.
// splits < 0 forces W = -splits (sweeps and tests).
static int pick_w(int ntiles) { return ntiles >= 32 ? 8 : (ntiles >= 12 ? 4 : 2); }

// HYDRA_ATTN8_QUAD=0 keeps the 16x16x4 P.V product (A/B)
static bool quad_enabled() {
  static int flag = -1;
  if (flag < 0) {
    const char* e = std::getenv("HYDRA_ATTN8_QUAD");
    flag = (e != nullptr && e[0] == '0') ? 0 : 1;
  }
  return flag == 1;
}

template <int W, bool BF>
static void fwd2_go(const float* Qp, const float* Kp, const float* Vq, int N, int Nq, int H, const int* sid,
                    const int* sptr, float qs, float* O, float* L) {
  dim3 grid(ceil_div(Nq, 16), H);
  if (!BF && quad_enabled()) {
    attn8_fwd2q_kernel<W><<<grid, 64 * W, 0, stream()>>>(Qp, Kp, Vq, N, Nq, H, sid, sptr, qs, O, L);
    return;
  }
  attn8_fwd2_kernel<1, W, BF><<<grid, 64 * W, 0, stream()>>>(Qp, Kp, Vq, N, Nq, H, sid, sptr, qs, O, L);
}

template <bool BF>
static void launch_fwd2_p(int var, const float* Qp, const float* Kp, const float* Vq, int N, int Nq, int H,
                          const int* sid, const int* sptr, float qs, float* O, float* L) {
  const int W = var > 0 ? var : pick_w(ceil_div(N, 16));
  switch (W) {
    case 2: fwd2_go<2, BF>(Qp, Kp, Vq, N, Nq, H, sid, sptr, qs, O, L); break;
    case 3: fwd2_go<3, BF>(Qp, Kp, Vq, N, Nq, H, sid, sptr, qs, O, L); break;
    case 4: fwd2_go<4, BF>(Qp, Kp, Vq, N, Nq, H, sid, sptr, qs, O, L); break;
    case 5: fwd2_go<5, BF>(Qp, Kp, Vq, N, Nq, H, sid, sptr, qs, O, L); break;
    case 6: fwd2_go<6, BF>(Qp, Kp, Vq, N, Nq, H, sid, sptr, qs, O, L); break;
    default: fwd2_go<8, BF>(Qp, Kp, Vq, N, Nq, H, sid, sptr, qs, O, L); break;
  }
}

// v3 (persistent, cost-balanced) eligibility: fp32, batch-scope segment layouts (<= 2
// contiguous segments ending at N), Nq the 16-row padding of N.  HYDRA_ATTN8_V3=0 keeps v2.
static bool v3_enabled() {
  static int flag = -1;
  if (flag < 0) {
    const char* e = std::getenv("HYDRA_ATTN8_V3");
    flag = (e != nullptr && e[0] == '1') ? 1 : 0;
  }
  return flag == 1;
}
static bool v3_ok(int var, int N, int Nq, int nseg, bool bf16) {
  return v3_enabled() && var == 0 && !bf16 && nseg >= 1 && nseg <= 2 && Nq == 16 * ceil_div(N, 16) && N > 0;
}
static int v3_grid(int64_t units) {
  static int per_cu = -1;
  if (per_cu < 0) {
    const char* e = std::getenv("HYDRA_ATTN8_V3_PERCU");
    per_cu = e ? std::max(1, std::min(4, std::atoi(e))) : 1;
  }
  return (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)num_cus() * per_cu, units));
}
// group-size caps (forward, dQ, dK/dV); HYDRA_ATTN8_V3_R="rf,rq,rk" for sweeps
static void v3_caps(int& rf, int& rq, int& rk) {
  static int c[3] = {2, 1, 1};
  static bool init = false;
  if (!init) {
    init = true;
    if (const char* e = std::getenv("HYDRA_ATTN8_V3_R")) {
      int a = 0, b = 0, d = 0;
      if (std::sscanf(e, "%d,%d,%d", &a, &b, &d) == 3 && a >= 1 && a <= 4 && b >= 1 && b <= 3 && d >= 1 && d <= 3) {
        c[0] = a;
        c[1] = b;
        c[2] = d;
      }
    }
  }
  rf = c[0];
  rq = c[1];
  rk = c[2];
}

static void launch_fwd2(int var, const float* Qp, const float* Kp, const float* Vq, int N, int Nq, int H,
                        const int* sid, const int* sptr, float qs, float* O, float* L, bool bf16 = false,
                        int nseg = 0) {
  if (v3_ok(var, N, Nq, nseg, bf16)) {
    int rf, rq, rk;
    v3_caps(rf, rq, rk);
    const int G = v3_grid((int64_t)H * (Nq / 16));
    switch (rf) {
      case 1: attn8_fwd3_kernel<1><<<G, 64 * kNW3, 0, stream()>>>(Qp, Kp, Vq, N, Nq, H, sptr, nseg, qs, O, L); break;
      case 2: attn8_fwd3_kernel<2><<<G, 64 * kNW3, 0, stream()>>>(Qp, Kp, Vq, N, Nq, H, sptr, nseg, qs, O, L); break;
      case 3: attn8_fwd3_kernel<3><<<G, 64 * kNW3, 0, stream()>>>(Qp, Kp, Vq, N, Nq, H, sptr, nseg, qs, O, L); break;
      default: attn8_fwd3_kernel<4><<<G, 64 * kNW3, 0, stream()>>>(Qp, Kp, Vq, N, Nq, H, sptr, nseg, qs, O, L); break;
    }
    return;
  }
  if (bf16)
    launch_fwd2_p<true>(var, Qp, Kp, Vq, N, Nq, H, sid, sptr, qs, O, L);
  else
    launch_fwd2_p<false>(var, Qp, Kp, Vq, N, Nq, H, sid, sptr, qs, O, L);
}

template <int W, bool BF>
static void bwd2_go(A8Bwd2 b) {
  b.nbq = ceil_div(b.Nq, 16);
  dim3 grid(2 * b.nbq, b.H);
  if (!BF && quad_enabled()) {
    static const int qm = std::getenv("HYDRA_ATTN8_QUADB") ? std::atoi(std::getenv("HYDRA_ATTN8_QUADB")) : 1;
    switch (qm) {
      case 1: attn8_bwd2q_kernel<W, 1><<<grid, 64 * W, 0, stream()>>>(b); return;
      case 2: attn8_bwd2q_kernel<W, 2><<<grid, 64 * W, 0, stream()>>>(b); return;
      case 3: attn8_bwd2q_kernel<W, 3><<<grid, 64 * W, 0, stream()>>>(b); return;
      default: break;
    }
  }
  attn8_bwd2_kernel<1, W, BF><<<grid, 64 * W, 0, stream()>>>(b);
}

template <bool BF>
static void launch_bwd2_p(int var, const A8Bwd2& b) {
  const int W = var > 0 ? var : pick_w(ceil_div(b.N, 16));
  switch (W) {
    case 2: bwd2_go<2, BF>(b); break;
    case 3: bwd2_go<3, BF>(b); break;
    case 4: bwd2_go<4, BF>(b); break;
    case 5: bwd2_go<5, BF>(b); break;
    case 6: bwd2_go<6, BF>(b); break;
    default: bwd2_go<8, BF>(b); break;
  }
}

static void launch_bwd2(int var, const A8Bwd2& b, bool bf16 = false, int nseg = 0) {
  if (v3_ok(var, b.N, b.Nq, nseg, bf16)) {
    int rf, rq, rk;
    v3_caps(rf, rq, rk);
    const int G = v3_grid(2LL * b.H * (b.Nq / 16));
    if (rq == 1 && rk == 1)
      attn8_bwd3_kernel<1, 1><<<G, 64 * kNW3, 0, stream()>>>(b, nseg);
    else if (rq == 2 && rk == 1)
      attn8_bwd3_kernel<2, 1><<<G, 64 * kNW3, 0, stream()>>>(b, nseg);
    else if (rq == 2 && rk == 2)
      attn8_bwd3_kernel<2, 2><<<G, 64 * kNW3, 0, stream()>>>(b, nseg);
    else if (rq == 3 && rk == 2)
      attn8_bwd3_kernel<3, 2><<<G, 64 * kNW3, 0, stream()>>>(b, nseg);
    else
      attn8_bwd3_kernel<3, 3><<<G, 64 * kNW3, 0, stream()>>>(b, nseg);
    return;
  }
  if (bf16)
    launch_bwd2_p<true>(var, b);
  else
    launch_bwd2_p<false>(var, b);
}

// chosen W of the v2 kernels for a shape (tools / tests)
std::vector<int64_t> attn8_v2_shape(int64_t N, int64_t H) {
  (void)H;
  const int W = pick_w(ceil_div(N, 16));
  return {W, W};
}

static void chk_seg(const at::Tensor& seg_id, const at::Tensor& seg_ptr, int64_t N) {
  HY_CHECK(seg_id.is_cuda() && seg_id.scalar_type() == at::kInt && seg_id.numel() == N, "attn8: seg_id [N] int32");
  HY_CHECK(seg_ptr.is_cuda() && seg_ptr.scalar_type() == at::kInt && seg_ptr.numel() >= 2, "attn8: seg_ptr int32");
}

// packed Q/K/V in pair + quad layouts from qkv [N, 3F] (module path; the fused encoder's
// node kernel writes them directly)
std::vector<at::Tensor> attn8_pack(const at::Tensor& qkv_, int64_t H) {
  at::Tensor qkv = qkv_.contiguous();
  HY_CHECK(qkv.is_cuda() && qkv.scalar_type() == at::kFloat && qkv.dim() == 2 && qkv.size(1) == 24 * H,
           "attn8_pack: qkv [N, 3 * 8H] fp32");
  const int64_t N = qkv.size(0), Nq = (N + 15) / 16 * 16;
  auto o = qkv.options();
  std::vector<at::Tensor> out;
  for (int j = 0; j < 3; ++j) {
    auto pr = at::empty({H, Nq, 8}, o), qd = at::empty({H, Nq / 4, 8, 4}, o);
    if (Nq > 0)
      attn8_pack_kernel<<<ceil_div(Nq * H * 8, 256), 256, 0, stream()>>>(
          qkv.data_ptr<float>() + j * 8 * H, (int)(24 * H), (int)N, (int)Nq, (int)H, pr.data_ptr<float>(),
          qd.data_ptr<float>());
    out.push_back(pr);
    out.push_back(qd);
  }
  return out;  // Qp, Qq, Kp, Kq, Vp, Vq
}

std::vector<at::Tensor> attn8_fwd(const at::Tensor& Qp, const at::Tensor& Kp, const at::Tensor& Vq,
                                  const at::Tensor& seg_id, const at::Tensor& seg_ptr, int64_t N, double scale,
                                  int64_t splits, bool bf16) {
  HY_CHECK(!bf16 || splits <= 0, "attn8_fwd: bf16 MFMA mode is the v2 (one-launch) kernel only");
  const int64_t H = Qp.size(0), Nq = Qp.size(1);
  HY_CHECK(Qp.is_contiguous() && Kp.is_contiguous() && Vq.is_contiguous() && Qp.size(2) == 8 && Nq % 16 == 0 &&
               Nq >= N && Kp.sizes() == Qp.sizes() && Vq.numel() == Qp.numel(),
           "attn8_fwd: packed operands [H, Nq, 8] (Nq % 16 == 0)");
  chk_seg(seg_id, seg_ptr, N);
  auto opt = Qp.options();
  auto O = at::empty({N, 8 * H}, opt), L = at::empty({H, Nq}, opt);
  if (N == 0) return {O, L};
  const float qs = (float)scale * kLog2e;
  if (splits <= 0) {  // v2: one launch, in-workgroup key split (variant -splits, 0 = default)
    launch_fwd2((int)(-splits), Qp.data_ptr<float>(), Kp.data_ptr<float>(), Vq.data_ptr<float>(), (int)N, (int)Nq,
                (int)H, seg_id.data_ptr<int>(), seg_ptr.data_ptr<int>(), qs, O.data_ptr<float>(), L.data_ptr<float>(),
                bf16, (int)seg_ptr.numel() - 1);
    return {O, L};
  }
  const int S = pick_splits((int)N, (int)H, splits);
  dim3 grid(ceil_div(N, 64 * kRT), H, S);
  if (S == 1) {
    attn8_fwd_kernel<kRT><<<grid, 256, 0, stream()>>>(Qp.data_ptr<float>(), Kp.data_ptr<float>(), Vq.data_ptr<float>(),
                                                 (int)N, (int)Nq, (int)H, seg_id.data_ptr<int>(),
                                                 seg_ptr.data_ptr<int>(), 1, qs, nullptr, O.data_ptr<float>(),
                                                 L.data_ptr<float>());
  } else {
    auto part = at::empty({S, H, N, 10}, opt);
    attn8_fwd_kernel<kRT><<<grid, 256, 0, stream()>>>(Qp.data_ptr<float>(), Kp.data_ptr<float>(), Vq.data_ptr<float>(),
                                                 (int)N, (int)Nq, (int)H, seg_id.data_ptr<int>(),
                                                 seg_ptr.data_ptr<int>(), S, qs, part.data_ptr<float>(), nullptr,
                                                 nullptr);
    attn8_combine_kernel<<<ceil_div(Nq * H, 256), 256, 0, stream()>>>(part.data_ptr<float>(), O.data_ptr<float>(),
                                                                       L.data_ptr<float>(), (int)N, (int)Nq, (int)H, S);
  }
  return {O, L};
}

// attention forward + PNA forward as one launch (see attn8_pna_fwd_kernel); fp32, v2 quad
// path only.  Returns [O, LSE2, Z, amin, amax].
std::vector<at::Tensor> attn8_pna_fwd(const at::Tensor& Qp, const at::Tensor& Kp, const at::Tensor& Vq,
                                      const at::Tensor& seg_id, const at::Tensor& seg_ptr, int64_t N, double scale,
                                      const at::Tensor& x, const at::Tensor& AB, const c10::optional<at::Tensor>& C_,
                                      const c10::optional<at::Tensor>& G_, const at::Tensor& src,
                                      const at::Tensor& rowptr, double avg_log, double avg_lin) {
  const int64_t H = Qp.size(0), Nq = Qp.size(1);
  HY_CHECK(Qp.is_contiguous() && Kp.is_contiguous() && Vq.is_contiguous() && Qp.size(2) == 8 && Nq % 16 == 0 &&
               Nq >= N && Kp.sizes() == Qp.sizes() && Vq.numel() == Qp.numel(),
           "attn8_pna_fwd: packed operands [H, Nq, 8] (Nq % 16 == 0)");
  chk_seg(seg_id, seg_ptr, N);
  HY_CHECK(quad_enabled(), "attn8_pna_fwd: the quad-block forward path only");
  HY_CHECK_F32(x);
  HY_CHECK_F32(AB);
  HY_CHECK_I32(src);
  HY_CHECK_I32(rowptr);
  HY_CHECK(x.is_contiguous() && x.dim() == 2 && x.size(0) == N, "attn8_pna_fwd: x [N, F]");
  const int F = (int)x.size(1);
  HY_CHECK(F == 64, "attn8_pna_fwd: the one-wave-per-node PNA layout (F = 64)");
  HY_CHECK(AB.size(0) == N && AB.size(1) == 2 * F && AB.stride(1) == 1, "attn8_pna_fwd: AB [N, 2F]");
  HY_CHECK(rowptr.numel() == N + 1, "attn8_pna_fwd: rowptr [N + 1]");
  const int64_t E = src.numel();
  auto edge = [&](const c10::optional<at::Tensor>& t) -> const float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    HY_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->dim() == 2 && t->size(0) == E &&
                 t->size(1) == F,
             "attn8_pna_fwd: edge terms [E, F]");
    return t->data_ptr<float>();
  };
  auto opt = Qp.options();
  auto O = at::empty({N, 8 * H}, opt), L = at::empty({H, Nq}, opt);
  auto Z = at::empty({N, 17 * F}, opt);
  auto amin = at::empty({N, F}, opt.dtype(at::kInt)), amax = at::empty({N, F}, opt.dtype(at::kInt));
  if (N == 0) return {O, L, Z, amin, amax};
  PnaFwdArgs p{x.data_ptr<float>(), AB.data_ptr<float>(), edge(C_), edge(G_), src.data_ptr<int>(),
               rowptr.data_ptr<int>(), Z.data_ptr<float>(), amin.data_ptr<int>(), amax.data_ptr<int>(),
               (int)AB.stride(0), (int)N, F, 64, (float)avg_log, (float)avg_lin};
  const float qs = (float)scale * kLog2e;
  const int nqt = ceil_div(Nq, 16);
  const int W = pick_w(ceil_div(N, 16));
#define HY_APF(WW)                                                                                              \
  attn8_pna_fwd_kernel<WW><<<nqt * (int)H + ceil_div(N, 64 * (WW) / 64), 64 * (WW), 0, stream()>>>(           \
      Qp.data_ptr<float>(), Kp.data_ptr<float>(), Vq.data_ptr<float>(), (int)N, (int)Nq, (int)H,               \
      seg_id.data_ptr<int>(), seg_ptr.data_ptr<int>(), qs, O.data_ptr<float>(), L.data_ptr<float>(), nqt, p)
  switch (W) {
    case 2: HY_APF(2); break;
    case 3: HY_APF(3); break;
    case 4: HY_APF(4); break;
    case 5: HY_APF(5); break;
    case 6: HY_APF(6); break;
    default: HY_APF(8); break;
  }
#undef HY_APF
  return {O, L, Z, amin, amax};
}

// dqkv [N, 24H] from dO [N, 8H] (and O, LSE2 of the forward)
// Backward in parts (the dQ and dK/dV passes are independent given delta; running them
// on two streams measured slower in the GPS step, see ops/gps_encoder.py):
//   prep: delta = rowsum(dO * O) + packed dO   ->  [delta, dOp, dOq]
//   dq:   per-split dQ partials [S, N, F]       (S == 1: written straight into dqkv[:, :F])
//   dkv:  per-split dK|dV partials [S, N, 2F]   (S == 1: straight into dqkv[:, F:])
//   sum:  dqkv = [sum_s dQ | sum_s dKV]         (skipped when S == 1)
std::vector<at::Tensor> attn8_bwd_prep(const at::Tensor& dO_, const at::Tensor& O, int64_t Nq, int64_t H) {
  at::Tensor dO = dO_.contiguous();
  const int64_t N = dO.size(0);
  HY_CHECK(dO.dim() == 2 && dO.size(1) == 8 * H && O.is_contiguous() && O.sizes() == dO.sizes() && Nq >= N &&
               Nq % 16 == 0,
           "attn8_bwd_prep: shapes");
  auto opt = dO.options();
  auto delta = at::empty({H, Nq}, opt), dOp = at::empty({H, Nq, 8}, opt), dOq = at::empty({H, Nq / 4, 8, 4}, opt);
  if (Nq * H > 0)
    attn8_delta_pack_kernel<<<ceil_div(Nq * H, 256), 256, 0, stream()>>>(
        dO.data_ptr<float>(), O.data_ptr<float>(), (int)N, (int)Nq, (int)H, delta.data_ptr<float>(),
        dOp.data_ptr<float>(), dOq.data_ptr<float>());
  return {delta, dOp, dOq};
}

static void chk_bwd(const at::Tensor& Qp, const at::Tensor& LSE2, const at::Tensor& delta, const at::Tensor& dOp,
                    int64_t N) {
  const int64_t H = Qp.size(0), Nq = Qp.size(1);
  HY_CHECK(Qp.dim() == 3 && Qp.size(2) == 8 && Nq >= N && Nq % 16 == 0 && LSE2.numel() == H * Nq &&
               delta.numel() == H * Nq && dOp.sizes() == Qp.sizes(),
           "attn8_bwd: operand shapes");
}

// out: [S, N, F] partials (S > 1) or the dqkv buffer [N, 3F] (S == 1)
at::Tensor attn8_bwd_dq(const at::Tensor& Qp, const at::Tensor& Kp, const at::Tensor& Kq, const at::Tensor& Vp,
                        const at::Tensor& dOp, const at::Tensor& LSE2, const at::Tensor& delta,
                        const at::Tensor& seg_id, const at::Tensor& seg_ptr, int64_t N, double scale, int64_t splits,
                        const c10::optional<at::Tensor>& dqkv) {
  chk_bwd(Qp, LSE2, delta, dOp, N);
  chk_seg(seg_id, seg_ptr, N);
  const int64_t H = Qp.size(0), Nq = Qp.size(1), F = 8 * H;
  const int S = pick_splits((int)N, (int)H, splits);
  at::Tensor out;
  if (S == 1) {
    HY_CHECK(dqkv.has_value() && dqkv->is_contiguous() && dqkv->size(0) == N && dqkv->size(1) == 3 * F,
             "attn8_bwd_dq: S == 1 writes into dqkv [N, 3F]");
    out = *dqkv;
  } else {
    out = at::empty({S, N, F}, Qp.options());
  }
  if (N == 0) return out;
  dim3 grid(ceil_div(N, 64 * kRT), H, S);
  attn8_bwd_dq_kernel<kRT><<<grid, 256, 0, stream()>>>(
      Qp.data_ptr<float>(), Kp.data_ptr<float>(), Kq.data_ptr<float>(), Vp.data_ptr<float>(), dOp.data_ptr<float>(),
      LSE2.data_ptr<float>(), delta.data_ptr<float>(), (int)N, (int)Nq, (int)H, seg_id.data_ptr<int>(),
      seg_ptr.data_ptr<int>(), S, (float)scale, (float)scale * kLog2e, out.data_ptr<float>(),
      S == 1 ? (int)(3 * F) : (int)F, S == 1 ? 0 : N * F);
  return out;
}

at::Tensor attn8_bwd_dkv(const at::Tensor& Qp, const at::Tensor& Qq, const at::Tensor& Kp, const at::Tensor& Vp,
                         const at::Tensor& dOp, const at::Tensor& dOq, const at::Tensor& LSE2, const at::Tensor& delta,
                         const at::Tensor& seg_id, const at::Tensor& seg_ptr, int64_t N, double scale, int64_t splits,
                         const c10::optional<at::Tensor>& dqkv) {
  chk_bwd(Qp, LSE2, delta, dOp, N);
  chk_seg(seg_id, seg_ptr, N);
  const int64_t H = Qp.size(0), Nq = Qp.size(1), F = 8 * H;
  HY_CHECK(Qq.numel() == Qp.numel() && dOq.numel() == dOp.numel(), "attn8_bwd_dkv: quad operand shapes");
  const int S = pick_splits((int)N, (int)H, splits);
  at::Tensor out;
  if (S == 1) {
    HY_CHECK(dqkv.has_value() && dqkv->is_contiguous() && dqkv->size(0) == N && dqkv->size(1) == 3 * F,
             "attn8_bwd_dkv: S == 1 writes into dqkv [N, 3F]");
    out = *dqkv;
  } else {
    out = at::empty({S, N, 2 * F}, Qp.options());
  }
  if (N == 0) return out;
  dim3 grid(ceil_div(N, 64 * kRT), H, S);
  attn8_bwd_dkv_kernel<kRT><<<grid, 256, 0, stream()>>>(
      Qp.data_ptr<float>(), Qq.data_ptr<float>(), Kp.data_ptr<float>(), Vp.data_ptr<float>(), dOp.data_ptr<float>(),
      dOq.data_ptr<float>(), LSE2.data_ptr<float>(), delta.data_ptr<float>(), (int)N, (int)Nq, (int)H,
      seg_id.data_ptr<int>(), seg_ptr.data_ptr<int>(), S, (float)scale, (float)scale * kLog2e,
      out.data_ptr<float>() + (S == 1 ? F : 0), S == 1 ? (int)(3 * F) : (int)(2 * F), S == 1 ? 0 : N * 2 * F);
  return out;
}

at::Tensor attn8_bwd_sum(const at::Tensor& pq, const at::Tensor& pkv) {
  HY_CHECK(pq.dim() == 3 && pkv.dim() == 3 && pq.is_contiguous() && pkv.is_contiguous() && pq.size(1) == pkv.size(1) &&
               pkv.size(2) == 2 * pq.size(2) && pq.size(2) % 4 == 0,
           "attn8_bwd_sum: partials [Sq, N, F] and [Skv, N, 2F]");
  const int64_t N = pq.size(1), F = pq.size(2);
  auto dqkv = at::empty({N, 3 * F}, pq.options());
  if (N > 0)
    attn8_bwd_sum_kernel<<<ceil_div(N * 3 * (F / 4), 256), 256, 0, stream()>>>(
        reinterpret_cast<const float4*>(pq.data_ptr<float>()), (int)pq.size(0),
        reinterpret_cast<const float4*>(pkv.data_ptr<float>()), (int)pkv.size(0),
        reinterpret_cast<float4*>(dqkv.data_ptr<float>()), (int)N, (int)F);
  return dqkv;
}

// single-stream composition: prep, ONE fused dQ + dK/dV launch, partial sum
// v2 backward from operands packed by the producer of dO (csrc/gps_fused.hip att_bwd with O):
// -delta [H, Nq], dO in the pair / quad layouts [H, Nq, 8]
at::Tensor attn8_bwd_packed(const at::Tensor& ndelta, const at::Tensor& dOp, const at::Tensor& dOq,
                            const at::Tensor& LSE2, const at::Tensor& Qp, const at::Tensor& Qq, const at::Tensor& Kp,
                            const at::Tensor& Kq, const at::Tensor& Vp, const at::Tensor& seg_id,
                            const at::Tensor& seg_ptr, int64_t N, double scale, bool bf16) {
  const int64_t H = Qp.size(0), Nq = Qp.size(1), F = 8 * H;
  chk_bwd(Qp, LSE2, ndelta, dOp, N);
  chk_seg(seg_id, seg_ptr, N);
  HY_CHECK(Qq.numel() == Qp.numel() && dOq.numel() == dOp.numel() && dOp.is_contiguous() && dOq.is_contiguous() &&
               ndelta.is_contiguous(),
           "attn8_bwd_packed: operand shapes");
  auto dqkv = at::empty({N, 3 * F}, Qp.options());
  if (N == 0) return dqkv;
  A8Bwd2 b{};
  b.Qp = Qp.data_ptr<float>();
  b.Qq = Qq.data_ptr<float>();
  b.Kp = Kp.data_ptr<float>();
  b.Kq = Kq.data_ptr<float>();
  b.Vp = Vp.data_ptr<float>();
  b.dOp = dOp.data_ptr<float>();
  b.dOq = dOq.data_ptr<float>();
  b.NL = LSE2.data_ptr<float>();  // v2 forward: -LSE2
  b.ndelta = ndelta.data_ptr<float>();
  b.N = (int)N;
  b.Nq = (int)Nq;
  b.H = (int)H;
  b.seg_id = seg_id.data_ptr<int>();
  b.seg_ptr = seg_ptr.data_ptr<int>();
  b.scale = (float)scale;
  b.qscale = (float)scale * kLog2e;
  b.dqkv = dqkv.data_ptr<float>();
  launch_bwd2(0, b, bf16, (int)seg_ptr.numel() - 1);
  return dqkv;
}

at::Tensor attn8_bwd(const at::Tensor& dO, const at::Tensor& O, const at::Tensor& LSE2, const at::Tensor& Qp,
                     const at::Tensor& Qq, const at::Tensor& Kp, const at::Tensor& Kq, const at::Tensor& Vp,
                     const at::Tensor& seg_id, const at::Tensor& seg_ptr, double scale, int64_t splits) {
  const int64_t H = Qp.size(0), Nq = Qp.size(1), N = dO.size(0), F = 8 * H;
  auto pre = attn8_bwd_prep(dO, O, Nq, H);
  chk_bwd(Qp, LSE2, pre[0], pre[1], N);
  chk_seg(seg_id, seg_ptr, N);
  HY_CHECK(Qq.numel() == Qp.numel() && pre[2].numel() == pre[1].numel(), "attn8_bwd: quad operand shapes");
  if (splits <= 0) {
    auto dqkv = at::empty({N, 3 * F}, dO.options());
    if (N == 0) return dqkv;
    A8Bwd2 b{};
    b.Qp = Qp.data_ptr<float>();
    b.Qq = Qq.data_ptr<float>();
    b.Kp = Kp.data_ptr<float>();
    b.Kq = Kq.data_ptr<float>();
    b.Vp = Vp.data_ptr<float>();
    b.dOp = pre[1].data_ptr<float>();
    b.dOq = pre[2].data_ptr<float>();
    b.NL = LSE2.data_ptr<float>();  // v2 forward: -LSE2
    b.ndelta = pre[0].data_ptr<float>();
    b.N = (int)N;
    b.Nq = (int)Nq;
    b.H = (int)H;
    b.seg_id = seg_id.data_ptr<int>();
    b.seg_ptr = seg_ptr.data_ptr<int>();
    b.scale = (float)scale;
    b.qscale = (float)scale * kLog2e;
    b.dqkv = dqkv.data_ptr<float>();
    launch_bwd2((int)(-splits), b, false, (int)seg_ptr.numel() - 1);
    return dqkv;
  }
  const int S = pick_splits((int)N, (int)H, splits);
  at::Tensor dqkv, pq, pkv;
  A8Bwd a{};
  if (S == 1) {
    dqkv = at::empty({N, 3 * F}, dO.options());
    a.out_q = dqkv.data_ptr<float>();
    a.out_kv = dqkv.data_ptr<float>() + F;
    a.ldq = a.ldkv = (int)(3 * F);
  } else {
    pq = at::empty({S, N, F}, dO.options());
    pkv = at::empty({S, N, 2 * F}, dO.options());
    a.out_q = pq.data_ptr<float>();
    a.out_kv = pkv.data_ptr<float>();
    a.ldq = (int)F;
    a.ldkv = (int)(2 * F);
    a.sq = N * F;
    a.skv = N * 2 * F;
  }
  if (N == 0) return S == 1 ? dqkv : at::zeros({N, 3 * F}, dO.options());
  a.Qp = Qp.data_ptr<float>();
  a.Qq = Qq.data_ptr<float>();
  a.Kp = Kp.data_ptr<float>();
  a.Kq = Kq.data_ptr<float>();
  a.Vp = Vp.data_ptr<float>();
  a.dOp = pre[1].data_ptr<float>();
  a.dOq = pre[2].data_ptr<float>();
  a.LSE2 = LSE2.data_ptr<float>();
  a.delta = pre[0].data_ptr<float>();
  a.N = (int)N;
  a.Nq = (int)Nq;
  a.H = (int)H;
  a.seg_id = seg_id.data_ptr<int>();
  a.seg_ptr = seg_ptr.data_ptr<int>();
  a.S = S;
  a.scale = (float)scale;
  a.qscale = (float)scale * kLog2e;
  a.nbq = ceil_div(N, 64 * kRT);
  dim3 grid(2 * a.nbq, H, S);
  attn8_bwd_fused_kernel<kRT><<<grid, 256, 0, stream()>>>(a);
  return S == 1 ? dqkv : attn8_bwd_sum(pq, pkv);
}

}  // namespace a8
}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("attn8_pack(Tensor qkv, int H) -> Tensor[]");
  m.def("attn8_v2_shape(int N, int H) -> int[]", hy::a8::attn8_v2_shape);
  m.def(
      "attn8_pna_fwd(Tensor Qp, Tensor Kp, Tensor Vq, Tensor seg_id, Tensor seg_ptr, int N, float scale, Tensor x, "
      "Tensor AB, Tensor? C, Tensor? G, Tensor src, Tensor rowptr, float avg_log, float avg_lin) -> Tensor[]");
  m.def(
      "attn8_fwd(Tensor Qp, Tensor Kp, Tensor Vq, Tensor seg_id, Tensor seg_ptr, int N, float scale, int splits, "
      "bool bf16=False) -> Tensor[]");
  m.def(
      "attn8_bwd(Tensor dO, Tensor O, Tensor LSE2, Tensor Qp, Tensor Qq, Tensor Kp, Tensor Kq, Tensor Vp, "
      "Tensor seg_id, Tensor seg_ptr, float scale, int splits) -> Tensor");
  m.def(
      "attn8_bwd_packed(Tensor ndelta, Tensor dOp, Tensor dOq, Tensor LSE2, Tensor Qp, Tensor Qq, Tensor Kp, "
      "Tensor Kq, Tensor Vp, Tensor seg_id, Tensor seg_ptr, int N, float scale, bool bf16=False) -> Tensor");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("attn8_pack", hy::a8::attn8_pack);
  m.impl("attn8_fwd", hy::a8::attn8_fwd);
  m.impl("attn8_pna_fwd", hy::a8::attn8_pna_fwd);
  m.impl("attn8_bwd", hy::a8::attn8_bwd);
  m.impl("attn8_bwd_packed", hy::a8::attn8_bwd_packed);
}
