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
  t.v = make_float4(vone, vone, vone, vone);
  if (i < 8) t.v = ld4(Vq + (((int64_t)h * (Nq >> 2) + (kc >> 2) + g) * 8 + i) * 4);
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
  t.kt = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < 8) t.kt = ld4(Kq + (((int64_t)h * (Nq >> 2) + (kc >> 2) + g) * 8 + i) * 4);
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
    ndl[t] = q < N ? -delta[(int64_t)h * Nq + q] : 0.f;
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
  t.qt = make_float4(0.f, 0.f, 0.f, 0.f);
  t.ot = t.qt;
  if (i < 8) {
    const int64_t qo = (((int64_t)h * (Nq >> 2) + (qc >> 2) + g) * 8 + i) * 4;
    t.qt = ld4(Qq + qo);
    t.ot = ld4(dOq + qo);
  }
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
    const f4v nd = f4v{-t0.dl.x, -t0.dl.y, -t0.dl.z, -t0.dl.w};
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
  delta[(int64_t)h * Nq + n] = a;
}

// ------------------------------------------------------------------------------------ host
constexpr int kRT = 2;  // row tiles per wave

static int pick_splits(int N, int H, int64_t splits) {
  if (splits > 0) return (int)splits;
  // >= ~5 waves per SIMD over 256 CUs x 4 SIMDs: blocks x H x S x 4 waves >= 5120
  const int blocks = ceil_div(N, 64 * kRT) * H;
  int S = 1;
  while (S < 16 && (int64_t)blocks * S * 4 < 5120 && N / (S * 2) >= 128) S *= 2;
  return S;
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
                                  int64_t splits) {
  const int64_t H = Qp.size(0), Nq = Qp.size(1);
  HY_CHECK(Qp.is_contiguous() && Kp.is_contiguous() && Vq.is_contiguous() && Qp.size(2) == 8 && Nq % 16 == 0 &&
               Nq >= N && Kp.sizes() == Qp.sizes() && Vq.numel() == Qp.numel(),
           "attn8_fwd: packed operands [H, Nq, 8] (Nq % 16 == 0)");
  chk_seg(seg_id, seg_ptr, N);
  auto opt = Qp.options();
  auto O = at::empty({N, 8 * H}, opt), L = at::empty({H, Nq}, opt);
  if (N == 0) return {O, L};
  const int S = pick_splits((int)N, (int)H, splits);
  const float qs = (float)scale * kLog2e;
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
at::Tensor attn8_bwd(const at::Tensor& dO, const at::Tensor& O, const at::Tensor& LSE2, const at::Tensor& Qp,
                     const at::Tensor& Qq, const at::Tensor& Kp, const at::Tensor& Kq, const at::Tensor& Vp,
                     const at::Tensor& seg_id, const at::Tensor& seg_ptr, double scale, int64_t splits) {
  const int64_t H = Qp.size(0), Nq = Qp.size(1), N = dO.size(0), F = 8 * H;
  auto pre = attn8_bwd_prep(dO, O, Nq, H);
  chk_bwd(Qp, LSE2, pre[0], pre[1], N);
  chk_seg(seg_id, seg_ptr, N);
  HY_CHECK(Qq.numel() == Qp.numel() && pre[2].numel() == pre[1].numel(), "attn8_bwd: quad operand shapes");
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
  m.def(
      "attn8_fwd(Tensor Qp, Tensor Kp, Tensor Vq, Tensor seg_id, Tensor seg_ptr, int N, float scale, int splits) -> "
      "Tensor[]");
  m.def(
      "attn8_bwd(Tensor dO, Tensor O, Tensor LSE2, Tensor Qp, Tensor Qq, Tensor Kp, Tensor Kq, Tensor Vp, "
      "Tensor seg_id, Tensor seg_ptr, float scale, int splits) -> Tensor");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("attn8_pack", hy::a8::attn8_pack);
  m.impl("attn8_fwd", hy::a8::attn8_fwd);
  m.impl("attn8_bwd", hy::a8::attn8_bwd);
}
