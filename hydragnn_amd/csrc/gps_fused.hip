// Fused GPS(PNAPlus) encoder layer for gfx950: row-block MFMA GEMM chains with
// BatchNorm folded into producer epilogues / consumer prologues.
//
// Reference layer (hydragnn/globalAtt/gps.py:103-152 wrapping PNAPlusStack.py:228-279,
// then Base.py:466 BatchNorm + ReLU):
//   qkv = x Win^T + bin ; o = MHA(qkv) ; z2 = drop(o Wo^T + bo) + x        h_att = BN2(z2)
//   AB = x Wab^T ; Z = PNA(x, AB, C, G) ; z1 = drop((Z Wpost^T + bp) Wlin^T + bl) + x   h_loc = BN1(z1)
//   out = h_loc + h_att ; md = drop(relu(out W1^T + b1)) ; z3 = drop(md W2^T + b2) + out
//   x' = relu(BN4(BN3(z3)))  (rows >= num_valid zeroed)
//
// MI355X design:
// * every node-level linear of the layer runs on v_mfma_f32_16x16x4_f32 (exact fp32,
//   the reference precision) inside a 16-row workgroup tile; chained GEMMs (post -> lin,
//   W1 -> W2, and their backward duals) hand the intermediate tile over through LDS, so
//   a layer's node-level work is 4 launches forward (node, o-proj, post, mlp) instead of
//   ~17 (GEMMs + bias/act/dropout/residual/BN stats/BN apply kernels);
// * BatchNorm statistics are accumulated in the PRODUCER's epilogue (fp64 column sums
//   of z and z^2 over valid rows, atomically added to one of 8 replicas per site to keep
//   contention low) and finalised in the CONSUMER's prologue (every workgroup folds the 8
//   replicas of its 64 columns: 1 KB), which also applies the affine normalisation while
//   staging its input tile;
// * BN4(BN3(z)) is one per-column affine map: BN4's batch statistics are those of an
//   affine image of z (mean = beta3, var = gamma3^2 var3 / (var3 + eps)), so the pair costs
//   one reduction, not two; its backward is derived in closed form (gps_encoder.py);
// * dropout masks are the counter hash of dropout.h with the same (salt, row*C + col)
//   indices as the unfused kernels, recomputed in the backward.
//
// Tile mapping of v_mfma_f32_16x16x4_f32: lane l, i = l & 15, g = l >> 4.  A operand
// A[i][k], B operand B[k][i] with k = kb + 4g + s for the s-th MFMA of a 16-deep chunk
// (each lane loads one float4 of A and of B per chunk); C/D: row 4g + r, column i.
#include "common.h"
#include "dropout.h"

namespace hy {
namespace gf {

typedef float f4v __attribute__((ext_vector_type(4)));
constexpr int BM = 16;   // rows per workgroup
constexpr int NREP = 8;  // atomic replicas per statistics site

__device__ __forceinline__ f4v mfma(float a, float b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f4v f4z() { return f4v{0.f, 0.f, 0.f, 0.f}; }

// B fragment for output column j and k = k..k+3:
//   WT:  y = x W^T, W [N][K] row-major -> contiguous float4 of row j
//   !WT: y = x W,   W [K][N] row-major -> four strided loads of column j
template <bool WT>
__device__ __forceinline__ float4 ldB(const float* __restrict__ W, int ldw, int k, int j) {
  if (WT) return *reinterpret_cast<const float4*>(W + (int64_t)j * ldw + k);
  return make_float4(W[(int64_t)k * ldw + j], W[(int64_t)(k + 1) * ldw + j], W[(int64_t)(k + 2) * ldw + j],
                     W[(int64_t)(k + 3) * ldw + j]);
}

// acc += As[16 x (kb .. kb + 16*KC)] * B[. x 16] at output columns n0..n0+15.
// Two accumulators alternate over 16-deep chunks (the dependent-accumulator latency of
// 16x16x4 is 40 cycles against a 32-cycle issue interval).
template <bool WT, int KC>
__device__ __forceinline__ void mma_chunks(f4v& a0, f4v& a1, const float* As, int lda, const float* __restrict__ W,
                                           int ldw, int kb, int n0) {
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  float4 xa[KC], wb[KC];
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    wb[c] = ldB<WT>(W, ldw, kb + 16 * c + 4 * g, n0 + i);
    xa[c] = *reinterpret_cast<const float4*>(As + i * lda + kb + 16 * c + 4 * g);
  }
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    f4v& a = (c & 1) ? a1 : a0;
    a = mfma(xa[c].x, wb[c].x, a);
    a = mfma(xa[c].y, wb[c].y, a);
    a = mfma(xa[c].z, wb[c].z, a);
    a = mfma(xa[c].w, wb[c].w, a);
  }
}

// Full tile product over k in [k0, k1) (multiple of 64 when k1 - k0 >= 64, else 16/32/48).
template <bool WT>
__device__ __forceinline__ f4v tile_mma(const float* As, int lda, const float* __restrict__ W, int ldw, int k0,
                                        int k1, int n0) {
  f4v a0 = f4z(), a1 = f4z();
  int kb = k0;
  for (; kb + 64 <= k1; kb += 64) mma_chunks<WT, 4>(a0, a1, As, lda, W, ldw, kb, n0);
  for (; kb + 16 <= k1; kb += 16) mma_chunks<WT, 1>(a0, a1, As, lda, W, ldw, kb, n0);
  return a0 + a1;
}

struct Drop {
  const int64_t* rng;
  int64_t salt;
  float p;
};

__device__ __forceinline__ float dropv(const DropCfg& d, uint32_t idx, float v) {
  return d.on ? (keep_elem(d.seed, idx, d.thresh) ? v * d.scale : 0.f) : v;
}

// Column statistics of a 16x16 tile (this lane: rows row0 + 4g + r, column c) over
// rows < nv, folded over the 4 lane groups and added to replica (blockIdx.x % NREP).
// site: [NREP][NS][F] entries of 3 x 64-bit words; s = stat index (NS stats per site).
//
// Deterministic accumulation: a block's partial v is split into exact fixed-point words
// (integer part, fraction bits 2^-1..2^-32, 2^-33..2^-64) and each word is added with an
// INTEGER atomic.  Integer sums do not depend on the order the workgroups arrive in, so the
// statistics are bitwise reproducible run to run; fp64 atomics were not.
// Range |v| < 2^62, resolution 2^-64 (backward sums of small gradients keep full relative
// precision down to ~1e-19).
typedef unsigned long long u64;
constexpr double kTwo32 = 4294967296.0;

__device__ __forceinline__ void fx_add(u64* q, double v) {
  const double fl = floor(v);
  const double f = (v - fl) * kTwo32;  // [0, 2^32), exact
  const double fh = floor(f);
  atomicAdd(q, (u64)(long long)fl);
  atomicAdd(q + 1, (u64)fh);
  atomicAdd(q + 2, (u64)((f - fh) * kTwo32));
}

__device__ __forceinline__ void col_sum_add(double v, double* site, int NS, int s, int F, int c) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  if ((threadIdx.x & 63) < 16)
    fx_add(reinterpret_cast<u64*>(site) + 3 * (((blockIdx.x & (NREP - 1)) * NS + s) * F + c), v);
}

__device__ __forceinline__ void stats2(const f4v& v, int row0, int nv, double* site, int F, int c) {
  const int g = (threadIdx.x & 63) >> 4;
  double s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (row0 + 4 * g + r < nv) {
      const double x = v[r];
      s1 += x;
      s2 += x * x;
    }
  }
  col_sum_add(s1, site, 2, 0, F, c);
  col_sum_add(s2, site, 2, 1, F, c);
}

__device__ __forceinline__ double site_sum(const double* site, int NS, int s, int F, int c) {
  const u64* q = reinterpret_cast<const u64*>(site);
  u64 I = 0, H = 0, L = 0;  // exact integer sums over the replicas (wrap-around = two's complement)
#pragma unroll
  for (int r = 0; r < NREP; ++r) {
    const u64* e = q + 3 * ((r * NS + s) * F + c);
    I += e[0];
    H += e[1];
    L += e[2];
  }
  return (double)(long long)I + (double)H * (1.0 / kTwo32) + (double)L * (1.0 / (kTwo32 * kTwo32));
}

// BN parameters of one site (affine weight/bias, running stats, batches counter)
struct BNP {
  const float* w;
  const float* b;
  float* rm;
  float* rv;
  int64_t* nbt;
  float mom;
  float eps;
};

// forward statistics of a site: biased mean / var over n valid rows
__device__ __forceinline__ void site_moments(const double* site, int F, int c, int n, double& mean, double& var) {
  const double s1 = site_sum(site, 2, 0, F, c), s2 = site_sum(site, 2, 1, F, c);
  const double nn = (double)max(n, 1);
  mean = s1 / nn;
  var = fmax(s2 / nn - mean * mean, 0.0);
}

__device__ __forceinline__ void running_update(const BNP& p, int c, int n, double mean, double var) {
  if (p.rm) {
    const double unb = n > 1 ? var * (double)n / (double)(n - 1) : var;
    p.rm[c] = (float)((1.0 - p.mom) * p.rm[c] + p.mom * mean);
    p.rv[c] = (float)((1.0 - p.mom) * p.rv[c] + p.mom * unb);
  }
}

// Per-layer saved statistics (fp32, [7][F]): mean1 inv1 mean2 inv2 mean3 inv3 inv4
enum { S_M1 = 0, S_I1, S_M2, S_I2, S_M3, S_I3, S_I4, S_N };

// Finalise the BN3 -> BN4 pair of a layer into the per-column affine map x = relu(A z + B).
// Workgroup 0 also saves mean3/inv3/inv4 and updates both running statistics.
struct PairFin {
  const double* site;  // fwd BN3 site [NREP][2][F]
  BNP bn3, bn4;
  float* saved;        // [S_N][F] of that layer
};

__device__ __forceinline__ void pair_coef(const PairFin& pf, int F, int c, int n, float& A, float& B) {
  double mean, var;
  site_moments(pf.site, F, c, n, mean, var);
  const float inv3 = (float)(1.0 / sqrt(var + (double)pf.bn3.eps));
  const float g3 = pf.bn3.w[c], b3 = pf.bn3.b[c], g4 = pf.bn4.w[c], b4 = pf.bn4.b[c];
  const double var4 = (double)g3 * g3 * (double)inv3 * inv3 * var;
  const float inv4 = (float)(1.0 / sqrt(var4 + (double)pf.bn4.eps));
  A = g4 * g3 * inv3 * inv4;
  B = b4 - A * (float)mean;
  if (blockIdx.x == 0) {
    pf.saved[S_M3 * F + c] = (float)mean;
    pf.saved[S_I3 * F + c] = inv3;
    pf.saved[S_I4 * F + c] = inv4;
    running_update(pf.bn3, c, n, mean, var);
    running_update(pf.bn4, c, n, (double)b3, var4);
  }
}

__device__ __forceinline__ void bump(int64_t* nbt) {
  if (nbt) nbt[0] += 1;
}

// ------------------------------------------------------------------------------------
// Forward 1 (main): x = layer input (layer 0: x0; else relu(A z3_prev + B), rows >= nv -> 0),
// [AB | qkv] = x [Wab; Win]^T + [0; bin].  Layer 0 also zeroes the step's statistics
// accumulators (consumed only by later kernels of this step).
struct NodeFwd {
  const float* src;     // [N, F]: x0 (layer 0) or z3 of the previous layer
  PairFin prev;         // valid when has_prev
  int has_prev;
  const float* Wab;     // [2F, F]
  const float* Win;     // [3F, F]
  const float* bin;     // [3F]
  float* x;             // [N, F] out
  float* AB;            // [N, 2F] out
  float* qkv;           // [N, 3F] out (or null: packed attention operands instead)
  float* pk[6];         // Q, K, V in the pair / quad layouts of csrc/attention8.hip (8-wide heads)
  int Nq;               // packed row count (N rounded up to 16)
  const int* nvp;
  int N;
  double* zero_buf;     // accumulators to clear (layer 0) or null
  int64_t zero_n;
};

template <int F>
__global__ void __launch_bounds__(256) node_fwd_kernel(NodeFwd a) {
  constexpr int LD = F + 4;
  __shared__ __attribute__((aligned(16))) float xs[BM * LD];
  __shared__ float cA[F], cB[F];
  const int nv = a.nvp ? min(*a.nvp, a.N) : a.N;
  const int row0 = blockIdx.x * BM;
  if (a.zero_buf) {
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < a.zero_n; t += (int64_t)gridDim.x * 256)
      a.zero_buf[t] = 0.0;
  }
  if (a.has_prev && threadIdx.x < F) {
    float A, B;
    pair_coef(a.prev, F, threadIdx.x, nv, A, B);
    cA[threadIdx.x] = A;
    cB[threadIdx.x] = B;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      bump(a.prev.bn3.nbt);
      bump(a.prev.bn4.nbt);
    }
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < BM * F / 4; idx += 256) {
    const int r = idx / (F / 4), c = (idx % (F / 4)) * 4, row = row0 + r;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < nv) {
      v = *reinterpret_cast<const float4*>(a.src + (int64_t)row * F + c);
      if (a.has_prev) {
        v.x = fmaxf(cA[c] * v.x + cB[c], 0.f);
        v.y = fmaxf(cA[c + 1] * v.y + cB[c + 1], 0.f);
        v.z = fmaxf(cA[c + 2] * v.z + cB[c + 2], 0.f);
        v.w = fmaxf(cA[c + 3] * v.w + cB[c + 3], 0.f);
      }
    }
    *reinterpret_cast<float4*>(xs + r * LD + c) = v;
    if (row < a.N) *reinterpret_cast<float4*>(a.x + (int64_t)row * F + c) = v;
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  constexpr int T = 5 * F / 16;
  for (int t = w; t < T; t += 4) {
    const int n0 = 16 * t;
    const bool ab = n0 < 2 * F;
    const float* W = ab ? a.Wab + (int64_t)n0 * F : a.Win + (int64_t)(n0 - 2 * F) * F;
    f4v acc = tile_mma<true>(xs, LD, W, F, 0, F, 0);
    const int col = ab ? n0 + i : n0 - 2 * F + i;
    const float bias = ab ? 0.f : a.bin[col];
    if (!ab && a.qkv == nullptr) {
      // packed attention operands: which = Q/K/V, head h, lane d (rows up to Nq: padding rows
      // hold the bias, finite)
      const int which = col / F, hd = col % F, h = hd >> 3, d = hd & 7;
      float* pr = a.pk[2 * which];
      float* qd = a.pk[2 * which + 1];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + 4 * g + r;
        if (row < a.Nq) {
          const float v = acc[r] + bias;
          pr[((int64_t)h * a.Nq + row) * 8 + 2 * (d & 3) + (d >> 2)] = v;
          qd[(((int64_t)h * (a.Nq >> 2) + (row >> 2)) * 8 + d) * 4 + (row & 3)] = v;
        }
      }
      continue;
    }
    float* out = ab ? a.AB : a.qkv;
    const int ldo = ab ? 2 * F : 3 * F;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + 4 * g + r;
      if (row < a.N) out[(int64_t)row * ldo + col] = acc[r] + bias;
    }
  }
}

// ------------------------------------------------------------------------------------
// Forward 2 (side): z2 = drop(o Wo^T + bo) + x, BN2 statistics.
struct OprojFwd {
  const float* o;   // [N, F]
  const float* Wo;  // [F, F]
  const float* bo;
  const float* x;
  float* z2;
  double* site;     // fwd BN2
  Drop drop;
  const int* nvp;
  int N;
};

template <int F, int NT = 256>
__device__ __forceinline__ void oproj_fwd_body(const OprojFwd& a, int bid) {
  constexpr int LD = F + 4;
  __shared__ __attribute__((aligned(16))) float os[BM * LD];
  const int nv = a.nvp ? min(*a.nvp, a.N) : a.N;
  const int row0 = bid * BM;
  for (int idx = threadIdx.x; idx < BM * F / 4; idx += NT) {
    const int r = idx / (F / 4), c = (idx % (F / 4)) * 4, row = row0 + r;
    *reinterpret_cast<float4*>(os + r * LD + c) =
        row < a.N ? *reinterpret_cast<const float4*>(a.o + (int64_t)row * F + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  const DropCfg d = drop_cfg(a.drop.rng, a.drop.salt, a.drop.p);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  for (int t = w; t < F / 16; t += 4) {
    const int n0 = 16 * t, col = n0 + i;
    f4v acc = tile_mma<true>(os, LD, a.Wo + (int64_t)n0 * F, F, 0, F, 0);
    const float bias = a.bo[col];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + 4 * g + r;
      const int rc = min(row, a.N - 1);
      float v = dropv(d, (uint32_t)(row * F + col), acc[r] + bias) + a.x[(int64_t)rc * F + col];
      acc[r] = v;
      if (row < a.N) a.z2[(int64_t)row * F + col] = v;
    }
    stats2(acc, row0, nv, a.site, F, col);
  }
}

template <int F>
__global__ void __launch_bounds__(256) oproj_fwd_kernel(OprojFwd a) {
  oproj_fwd_body<F>(a, blockIdx.x);
}

// ------------------------------------------------------------------------------------
// Forward 3 (main): p = Z Wpost^T + bpost ; z1 = drop(p Wlin^T + blin) + x ; BN1 statistics.
// 512 threads: waves w and w + 4 split the 17F-deep product in halves (folded through LDS).
struct PostFwd {
  const float* Z;     // [N, 17F]
  const float* Wp;    // [F, 17F]
  const float* bp;
  const float* Wl;    // [F, F]
  const float* bl;
  const float* x;
  float* p;           // [N, F] out
  float* z1;          // [N, F] out
  double* site;       // fwd BN1
  Drop drop;
  const int* nvp;
  int N;
};

template <int F>
__device__ __forceinline__ void post_fwd_body(const PostFwd& a, int bid) {
  constexpr int K = 17 * F, LDZ = K + 4, LD = F + 4;
  __shared__ __attribute__((aligned(16))) float zs[BM * LDZ];
  __shared__ __attribute__((aligned(16))) float ps[BM * LD];
  __shared__ f4v red[4][64];
  const int nv = a.nvp ? min(*a.nvp, a.N) : a.N;
  const int row0 = bid * BM;
  for (int idx = threadIdx.x; idx < BM * K / 4; idx += 512) {
    const int r = idx / (K / 4), c = (idx % (K / 4)) * 4, row = row0 + r;
    *reinterpret_cast<float4*>(zs + r * LDZ + c) =
        row < a.N ? *reinterpret_cast<const float4*>(a.Z + (int64_t)row * K + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int wt = w & 3, half = w >> 2;
  // K = 17F: split at a 64-multiple boundary (F = 64: 1088 -> [0, 576) + [576, 1088))
  constexpr int KH = ((K / 2 + 63) / 64) * 64;
  static_assert(F / 16 <= 4, "post_fwd: one 16-column tile per wave");
  f4v acc = f4z();
  if (wt < F / 16) {
    acc = half == 0 ? tile_mma<true>(zs, LDZ, a.Wp + (int64_t)(16 * wt) * K, K, 0, KH, 0)
                    : tile_mma<true>(zs, LDZ, a.Wp + (int64_t)(16 * wt) * K, K, KH, K, 0);
    if (half == 1) red[wt][lane] = acc;
  }
  __syncthreads();
  if (half == 0 && wt < F / 16) {
    acc += red[wt][lane];
    const int col = 16 * wt + i;
    const float bias = a.bp[col];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + 4 * g + r;
      const float v = acc[r] + bias;
      ps[(4 * g + r) * LD + col] = v;
      if (row < a.N) a.p[(int64_t)row * F + col] = v;
    }
  }
  __syncthreads();
  if (half == 0 && wt < F / 16) {
    const DropCfg d = drop_cfg(a.drop.rng, a.drop.salt, a.drop.p);
    const int col = 16 * wt + i;
    f4v q = tile_mma<true>(ps, LD, a.Wl + (int64_t)(16 * wt) * F, F, 0, F, 0);
    const float bias = a.bl[col];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + 4 * g + r;
      const int rc = min(row, a.N - 1);
      const float v = dropv(d, (uint32_t)(row * F + col), q[r] + bias) + a.x[(int64_t)rc * F + col];
      q[r] = v;
      if (row < a.N) a.z1[(int64_t)row * F + col] = v;
    }
    stats2(q, row0, nv, a.site, F, col);
  }
}

template <int F>
__global__ void __launch_bounds__(512) post_fwd_kernel(PostFwd a) {
  post_fwd_body<F>(a, blockIdx.x);
}

// The output projection and the local post-NN of a layer in one launch (both read only the
// outputs of the attention + PNA launch; one dispatch and one tail instead of two in a row):
// workgroups [0, nP) run post_fwd, the rest oproj_fwd (its loops stride 512 threads).
template <int F>
__global__ void __launch_bounds__(512) oproj_post_fwd_kernel(PostFwd pa, OprojFwd oa, int nP) {
  if ((int)blockIdx.x < nP)
    post_fwd_body<F>(pa, blockIdx.x);
  else
    oproj_fwd_body<F, 512>(oa, blockIdx.x - nP);
}

// ------------------------------------------------------------------------------------
// Forward 4 (join): out = BN1(z1) + BN2(z2) ; md = drop(relu(out W1^T + b1)) ;
// z3 = drop(md W2^T + b2) + out ; BN3 statistics.  Workgroup 0 saves BN1/BN2 statistics
// and updates their running statistics.
struct MlpFwd {
  const float* z1;
  const float* z2;
  const double* site1;
  const double* site2;
  BNP bn1, bn2;
  float* saved;       // this layer's [S_N][F]
  const float* W1;    // [2F, F]
  const float* b1;
  const float* W2;    // [F, 2F]
  const float* b2;
  float* out;         // [N, F]
  float* md;          // [N, 2F]
  float* z3;          // [N, F]
  double* site3;      // fwd BN3
  Drop drop2, drop3;
  const int* nvp;
  int N;
};

template <int F>
__global__ void __launch_bounds__(256) mlp_fwd_kernel(MlpFwd a) {
  constexpr int LD = F + 4, LD2 = 2 * F + 4;
  __shared__ __attribute__((aligned(16))) float os[BM * LD];
  __shared__ __attribute__((aligned(16))) float ms[BM * LD2];
  __shared__ float s1a[F], s1b[F], s2a[F], s2b[F];
  const int nv = a.nvp ? min(*a.nvp, a.N) : a.N;
  const int row0 = blockIdx.x * BM;
  if (threadIdx.x < F) {
    const int c = threadIdx.x;
    double m1, v1, m2, v2;
    site_moments(a.site1, F, c, nv, m1, v1);
    site_moments(a.site2, F, c, nv, m2, v2);
    const float i1 = (float)(1.0 / sqrt(v1 + (double)a.bn1.eps)), i2 = (float)(1.0 / sqrt(v2 + (double)a.bn2.eps));
    const float sc1 = a.bn1.w[c] * i1, sc2 = a.bn2.w[c] * i2;
    s1a[c] = sc1;
    s1b[c] = a.bn1.b[c] - sc1 * (float)m1;
    s2a[c] = sc2;
    s2b[c] = a.bn2.b[c] - sc2 * (float)m2;
    if (blockIdx.x == 0) {
      a.saved[S_M1 * F + c] = (float)m1;
      a.saved[S_I1 * F + c] = i1;
      a.saved[S_M2 * F + c] = (float)m2;
      a.saved[S_I2 * F + c] = i2;
      running_update(a.bn1, c, nv, m1, v1);
      running_update(a.bn2, c, nv, m2, v2);
      if (c == 0) {
        bump(a.bn1.nbt);
        bump(a.bn2.nbt);
      }
    }
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < BM * F / 4; idx += 256) {
    const int r = idx / (F / 4), c = (idx % (F / 4)) * 4, row = row0 + r;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < a.N) {
      const float4 u1 = *reinterpret_cast<const float4*>(a.z1 + (int64_t)row * F + c);
      const float4 u2 = *reinterpret_cast<const float4*>(a.z2 + (int64_t)row * F + c);
      // torch BN: (z - mean) * invstd * w + b, summed branch by branch
      v.x = (s1a[c] * u1.x + s1b[c]) + (s2a[c] * u2.x + s2b[c]);
      v.y = (s1a[c + 1] * u1.y + s1b[c + 1]) + (s2a[c + 1] * u2.y + s2b[c + 1]);
      v.z = (s1a[c + 2] * u1.z + s1b[c + 2]) + (s2a[c + 2] * u2.z + s2b[c + 2]);
      v.w = (s1a[c + 3] * u1.w + s1b[c + 3]) + (s2a[c + 3] * u2.w + s2b[c + 3]);
      *reinterpret_cast<float4*>(a.out + (int64_t)row * F + c) = v;
    }
    *reinterpret_cast<float4*>(os + r * LD + c) = v;
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  {
    const DropCfg d = drop_cfg(a.drop2.rng, a.drop2.salt, a.drop2.p);
    for (int t = w; t < 2 * F / 16; t += 4) {
      const int n0 = 16 * t, col = n0 + i;
      f4v acc = tile_mma<true>(os, LD, a.W1 + (int64_t)n0 * F, F, 0, F, 0);
      const float bias = a.b1[col];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + 4 * g + r;
        const float v = dropv(d, (uint32_t)(row * 2 * F + col), fmaxf(acc[r] + bias, 0.f));
        ms[(4 * g + r) * LD2 + col] = v;
        if (row < a.N) a.md[(int64_t)row * 2 * F + col] = v;
      }
    }
  }
  __syncthreads();
  {
    const DropCfg d = drop_cfg(a.drop3.rng, a.drop3.salt, a.drop3.p);
    for (int t = w; t < F / 16; t += 4) {
      const int n0 = 16 * t, col = n0 + i;
      f4v acc = tile_mma<true>(ms, LD2, a.W2 + (int64_t)n0 * 2 * F, 2 * F, 0, 2 * F, 0);
      const float bias = a.b2[col];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + 4 * g + r;
        const float v = dropv(d, (uint32_t)(row * F + col), acc[r] + bias) + os[(4 * g + r) * LD + col];
        acc[r] = v;
        if (row < a.N) a.z3[(int64_t)row * F + col] = v;
      }
      stats2(acc, row0, nv, a.site3, F, col);
    }
  }
}

// ------------------------------------------------------------------------------------
// Forward 5 (after the last layer): x_L = relu(A z3 + B), rows >= nv -> 0.
// With a graph CSR (gptr [G+1]) the same launch also mean-pools x_L per graph
// (reference Base.py:478 global_mean_pool): workgroups [0, G) pool one graph each
// (recomputing its rows' x on the fly), the rest write x_L row-parallel.
struct FinalFwd {
  const float* z3;
  PairFin pf;
  float* x;
  const int* nvp;
  int N;
  const int* gptr;  // [G + 1] or null
  int G;
  float* pooled;    // [G, F]
};

template <int F>
__global__ void __launch_bounds__(256) final_fwd_kernel(FinalFwd a) {
  __shared__ float cA[F], cB[F];
  __shared__ float red[256 / F][F];
  const int nv = a.nvp ? min(*a.nvp, a.N) : a.N;
  if (threadIdx.x < F) {
    float A, B;
    pair_coef(a.pf, F, threadIdx.x, nv, A, B);
    cA[threadIdx.x] = A;
    cB[threadIdx.x] = B;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      bump(a.pf.bn3.nbt);
      bump(a.pf.bn4.nbt);
    }
  }
  __syncthreads();
  if ((int)blockIdx.x < a.G) {
    constexpr int RPP = 256 / F;  // rows per pass
    const int gb = a.gptr[blockIdx.x], ge = a.gptr[blockIdx.x + 1];
    const int c = threadIdx.x % F, rl = threadIdx.x / F;
    float acc = 0.f;
    for (int row = gb + rl; row < ge; row += RPP)
      if (row < nv) acc += fmaxf(cA[c] * a.z3[(int64_t)row * F + c] + cB[c], 0.f);
    red[rl][c] = acc;
    __syncthreads();
    if (threadIdx.x < F) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < RPP; ++q) t += red[q][threadIdx.x];
      a.pooled[(int64_t)blockIdx.x * F + threadIdx.x] = t / (float)max(ge - gb, 1);
    }
    return;
  }
  const int64_t total = (int64_t)a.N * F / 4;
  const int64_t nb = (int64_t)gridDim.x - a.G;
  for (int64_t t = ((int64_t)blockIdx.x - a.G) * 256 + threadIdx.x; t < total; t += nb * 256) {
    const int row = (int)(t / (F / 4)), c = (int)(t % (F / 4)) * 4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < nv) {
      v = *reinterpret_cast<const float4*>(a.z3 + t * 4);
      v.x = fmaxf(cA[c] * v.x + cB[c], 0.f);
      v.y = fmaxf(cA[c + 1] * v.y + cB[c + 1], 0.f);
      v.z = fmaxf(cA[c + 2] * v.z + cB[c + 2], 0.f);
      v.w = fmaxf(cA[c + 3] * v.w + cB[c + 3], 0.f);
    }
    *reinterpret_cast<float4*>(a.x + t * 4) = v;
  }
}

// ====================================================================================
// Backward.
//
// BN3 -> BN4 pair (valid rows, n of them; g = dL/dx' masked by relu and padding,
// zhat = (z - mean3) inv3, S1 = sum g, S2 = sum g zhat, c = gamma3 inv4, rho = var3 inv3^2):
//   dz = K (g - S1/n - zhat S2 kappa / n),  K = gamma3 gamma4 inv3 inv4,  kappa = 1 + c^2 (1 - rho)
//   dgamma4 = c S2, dbeta4 = S1, dgamma3 = gamma4 inv4 S2 (1 - c^2 rho), dbeta3 = 0
// (padding rows: g = 0 and the direct term only -> dz = 0).

// Pair statistics of the last layer: g = dxL * [xL > 0] -> S1, S2 (site [NREP][2][F]).
struct PairStatsBwd {
  const float* dx;     // [N, F] or null
  const float* x;      // relu output (mask)
  const float* z3;
  const float* saved;  // layer's [S_N][F]
  float* g;            // [N, F] out
  double* site;
  const int* nvp;
  int N;
  const float* dpool;  // [G, F] gradient of the per-graph mean pool, or null
  const int* gidx;     // [N] graph of each row
  const int* gptr;     // [G + 1]
};

template <int F>
__global__ void __launch_bounds__(256) pair_stats_bwd_kernel(PairStatsBwd a) {
  const int nv = a.nvp ? min(*a.nvp, a.N) : a.N;
  const int row0 = blockIdx.x * BM;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, gq = lane >> 4;
  for (int t = w; t < F / 16; t += 4) {
    const int col = 16 * t + i;
    const float m3 = a.saved[S_M3 * F + col], i3 = a.saved[S_I3 * F + col];
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + 4 * gq + r;
      if (row < a.N) {
        const int64_t o = (int64_t)row * F + col;
        float up = a.dx ? a.dx[o] : 0.f;
        if (a.dpool) {
          const int gi = a.gidx[row];
          up += a.dpool[(int64_t)gi * F + col] / (float)max(a.gptr[gi + 1] - a.gptr[gi], 1);
        }
        const float gv = (row < nv && a.x[o] > 0.f) ? up : 0.f;
        a.g[o] = gv;
        if (row < nv) {
          s1 += gv;
          s2 += (double)gv * (double)((a.z3[o] - m3) * i3);
        }
      }
    }
    col_sum_add(s1, a.site, 2, 0, F, col);
    col_sum_add(s2, a.site, 2, 1, F, col);
  }
}

// parameter-gradient outputs of one BN
struct BNG {
  float* dw;
  float* db;
};

// Backward 1: dz3 from the pair; dg = dz3 * drop3 ; dpre = (dg W2) * [md > 0] * scale2 ;
// dout = dz3 + dpre W1 ; statistics for BN1/BN2 backward (S1' = sum dout,
// S2_1 = sum dout zhat1, S2_2 = sum dout zhat2 over valid rows; site [NREP][3][F]).
struct MlpBwd {
  const float* g;        // [N, F] masked dL/dx'
  const float* z3;
  const double* psite;   // bwd pair site [NREP][2][F]
  const float* saved;    // this layer's saved stats
  const float* g3;       // gamma3
  const float* g4;       // gamma4
  float eps3, eps4;
  BNG d3, d4;
  const float* md;       // [N, 2F]
  const float* W2;       // [F, 2F]
  const float* W1;       // [2F, F]
  const float* z1;
  const float* z2;
  float* dg;             // [N, F]
  float* dpre;           // [N, 2F]
  float* dout;           // [N, F]
  double* site12;        // bwd BN1/BN2 site [NREP][3][F]
  Drop drop2, drop3;
  const int* nvp;
  int N;
};

template <int F>
__global__ void __launch_bounds__(256) mlp_bwd_kernel(MlpBwd a) {
  constexpr int LD = F + 4, LD2 = 2 * F + 4;
  __shared__ __attribute__((aligned(16))) float dzs[BM * LD];
  __shared__ __attribute__((aligned(16))) float dgs[BM * LD];
  __shared__ __attribute__((aligned(16))) float dps[BM * LD2];
  __shared__ float cK[F], cS1[F], cS2[F], cM[F], cI[F];
  const int nv = a.nvp ? min(*a.nvp, a.N) : a.N;
  const int row0 = blockIdx.x * BM;
  if (threadIdx.x < F) {
    const int c = threadIdx.x;
    const double S1 = site_sum(a.psite, 2, 0, F, c), S2 = site_sum(a.psite, 2, 1, F, c);
    const float m3 = a.saved[S_M3 * F + c], i3 = a.saved[S_I3 * F + c], i4 = a.saved[S_I4 * F + c];
    const float ga3 = a.g3[c], ga4 = a.g4[c];
    const double n = (double)max(nv, 1);
    // rho = var3 inv3^2 = 1 - eps3 inv3^2
    const double rho = 1.0 - (double)a.eps3 * i3 * i3;
    const double cc = (double)ga3 * i4;
    const double kappa = 1.0 + cc * cc * (1.0 - rho);
    cK[c] = ga3 * ga4 * i3 * i4;
    cS1[c] = (float)(S1 / n);
    cS2[c] = (float)(S2 * kappa / n);
    cM[c] = m3;
    cI[c] = i3;
    if (blockIdx.x == 0) {
      a.d4.dw[c] = (float)(cc * S2);
      a.d4.db[c] = (float)S1;
      a.d3.dw[c] = (float)((double)ga4 * i4 * S2 * (1.0 - cc * cc * rho));
      a.d3.db[c] = 0.f;
    }
  }
  __syncthreads();
  const DropCfg d3 = drop_cfg(a.drop3.rng, a.drop3.salt, a.drop3.p);
  for (int idx = threadIdx.x; idx < BM * F; idx += 256) {
    const int r = idx / F, c = idx % F, row = row0 + r;
    float dz = 0.f;
    if (row < nv) {
      const int64_t o = (int64_t)row * F + c;
      dz = cK[c] * (a.g[o] - cS1[c] - (a.z3[o] - cM[c]) * cI[c] * cS2[c]);
    }
    const float dgv = dropv(d3, (uint32_t)(row * F + c), dz);
    dzs[r * LD + c] = dz;
    dgs[r * LD + c] = dgv;
    if (row < a.N) a.dg[(int64_t)row * F + c] = dgv;
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  {
    const float sc = (a.drop2.rng && a.drop2.p > 0.f) ? 1.f / (1.f - a.drop2.p) : 1.f;
    for (int t = w; t < 2 * F / 16; t += 4) {
      const int n0 = 16 * t, col = n0 + i;
      f4v acc = tile_mma<false>(dgs, LD, a.W2, 2 * F, 0, F, n0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + 4 * g + r;
        const int rc = min(row, a.N - 1);
        const float v = a.md[(int64_t)rc * 2 * F + col] > 0.f ? acc[r] * sc : 0.f;
        dps[(4 * g + r) * LD2 + col] = v;
        if (row < a.N) a.dpre[(int64_t)row * 2 * F + col] = v;
      }
    }
  }
  __syncthreads();
  for (int t = w; t < F / 16; t += 4) {
    const int n0 = 16 * t, col = n0 + i;
    f4v acc = tile_mma<false>(dps, LD2, a.W1, F, 0, 2 * F, n0);
    const float m1 = a.saved[S_M1 * F + col], i1 = a.saved[S_I1 * F + col];
    const float m2 = a.saved[S_M2 * F + col], i2 = a.saved[S_I2 * F + col];
    double s1 = 0.0, s21 = 0.0, s22 = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + 4 * g + r;
      const float v = dzs[(4 * g + r) * LD + col] + acc[r];
      if (row < a.N) {
        const int64_t o = (int64_t)row * F + col;
        a.dout[o] = v;
        if (row < nv) {
          s1 += v;
          s21 += (double)v * (double)((a.z1[o] - m1) * i1);
          s22 += (double)v * (double)((a.z2[o] - m2) * i2);
        }
      }
    }
    col_sum_add(s1, a.site12, 3, 0, F, col);
    col_sum_add(s21, a.site12, 3, 1, F, col);
    col_sum_add(s22, a.site12, 3, 2, F, col);
  }
}

// BN backward coefficients of BN k (k = 1: local branch, 2: attention branch) from the
// shared site: dz = gamma inv (dout - S1'/n - zhat S2_k / n) on valid rows, gamma inv dout on
// padding rows.  Workgroup 0 writes dgamma_k = S2_k, dbeta_k = S1'.
__device__ __forceinline__ void bn_bwd_coef(const double* site12, int k, const float* saved, const float* gam, BNG dgr,
                                            int F, int c, int nv, float& cg, float& cs1, float& cs2, float& cm,
                                            float& ci) {
  const double S1 = site_sum(site12, 3, 0, F, c), S2 = site_sum(site12, 3, k, F, c);
  const double n = (double)max(nv, 1);
  cm = saved[(k == 1 ? S_M1 : S_M2) * F + c];
  ci = saved[(k == 1 ? S_I1 : S_I2) * F + c];
  cg = gam[c] * ci;
  cs1 = (float)(S1 / n);
  cs2 = (float)(S2 / n);
  if (blockIdx.x == 0) {
    dgr.dw[c] = (float)S2;
    dgr.db[c] = (float)S1;
  }
}

// Backward 2 (main): dz1 (BN1) ; dq = dz1 * drop0 ; dp = dq Wlin ; dZ = dp Wpost.
// 512 threads: 8 waves over the 17F output columns of dZ.
struct LocBwd {
  const float* dout;
  const float* z1;
  const double* site12;
  const float* saved;
  const float* gamma1;
  BNG d1;
  const float* Wl;     // [F, F]
  const float* Wp;     // [F, 17F]
  float* dz1;          // [N, F]
  float* dq;           // [N, F]
  float* dp;           // [N, F]
  float* dZ;           // [N, 17F]
  Drop drop0;
  const int* nvp;
  int N;
};

template <int F>
__global__ void __launch_bounds__(512) loc_bwd_kernel(LocBwd a) {
  constexpr int LD = F + 4;
  __shared__ __attribute__((aligned(16))) float dqs[BM * LD];
  __shared__ __attribute__((aligned(16))) float dps[BM * LD];
  __shared__ float cG[F], cS1[F], cS2[F], cM[F], cI[F];
  const int nv = a.nvp ? min(*a.nvp, a.N) : a.N;
  const int row0 = blockIdx.x * BM;
  if (threadIdx.x < F) {
    const int c = threadIdx.x;
    bn_bwd_coef(a.site12, 1, a.saved, a.gamma1, a.d1, F, c, nv, cG[c], cS1[c], cS2[c], cM[c], cI[c]);
  }
  __syncthreads();
  const DropCfg d0 = drop_cfg(a.drop0.rng, a.drop0.salt, a.drop0.p);
  for (int idx = threadIdx.x; idx < BM * F; idx += 512) {
    const int r = idx / F, c = idx % F, row = row0 + r;
    float dz = 0.f;
    if (row < a.N) {
      const int64_t o = (int64_t)row * F + c;
      const float dv = a.dout[o];
      dz = row < nv ? cG[c] * (dv - cS1[c] - (a.z1[o] - cM[c]) * cI[c] * cS2[c]) : cG[c] * dv;
      a.dz1[o] = dz;
    }
    const float dqv = dropv(d0, (uint32_t)(row * F + c), dz);
    dqs[r * LD + c] = dqv;
    if (row < a.N) a.dq[(int64_t)row * F + c] = dqv;
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  if (w < F / 16) {
    const int n0 = 16 * w, col = n0 + i;
    f4v acc = tile_mma<false>(dqs, LD, a.Wl, F, 0, F, n0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + 4 * g + r;
      dps[(4 * g + r) * LD + col] = acc[r];
      if (row < a.N) a.dp[(int64_t)row * F + col] = acc[r];
    }
  }
  __syncthreads();
  constexpr int K17 = 17 * F;
  for (int t = w; t < K17 / 16; t += 8) {
    const int n0 = 16 * t, col = n0 + i;
    f4v acc = tile_mma<false>(dps, LD, a.Wp, K17, 0, F, n0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + 4 * g + r;
      if (row < a.N) a.dZ[(int64_t)row * K17 + col] = acc[r];
    }
  }
}

// Backward 3 (side): dz2 (BN2) ; da = dz2 * drop1 ; do = da Wo.
struct AttBwd {
  const float* dout;
  const float* z2;
  const double* site12;
  const float* saved;
  const float* gamma2;
  BNG d2;
  const float* Wo;    // [F, F]
  float* dz2;
  float* da;
  float* dO;
  Drop drop1;
  const int* nvp;
  int N;
  // 8-wide-head attention backward operands written here instead of dO (csrc/attention8.hip
  // attn8_delta_pack, folded into this epilogue): -delta[h][q] = -sum_d dO O, dO in the
  // "pair" and "quad" layouts; rows N..Nq zero
  const float* O;
  float *ndelta, *dOp, *dOq;
  int Nq;
};

// attention8.hip operand layouts of one head (element d of row n)
__device__ __forceinline__ int64_t a8_pair_idx(int h, int Nq, int n, int d) {
  return ((int64_t)h * Nq + n) * 8 + 2 * (d & 3) + (d >> 2);
}
__device__ __forceinline__ int64_t a8_quad_idx(int h, int Nq, int n, int d) {
  return (((int64_t)h * (Nq >> 2) + (n >> 2)) * 8 + d) * 4 + (n & 3);
}

template <int F>
__global__ void __launch_bounds__(256) att_bwd_kernel(AttBwd a) {
  constexpr int LD = F + 4;
  __shared__ __attribute__((aligned(16))) float das[BM * LD];
  __shared__ float cG[F], cS1[F], cS2[F], cM[F], cI[F];
  const int nv = a.nvp ? min(*a.nvp, a.N) : a.N;
  const int row0 = blockIdx.x * BM;
  if (threadIdx.x < F) {
    const int c = threadIdx.x;
    bn_bwd_coef(a.site12, 2, a.saved, a.gamma2, a.d2, F, c, nv, cG[c], cS1[c], cS2[c], cM[c], cI[c]);
  }
  __syncthreads();
  const DropCfg d1 = drop_cfg(a.drop1.rng, a.drop1.salt, a.drop1.p);
  for (int idx = threadIdx.x; idx < BM * F; idx += 256) {
    const int r = idx / F, c = idx % F, row = row0 + r;
    float dz = 0.f;
    if (row < a.N) {
      const int64_t o = (int64_t)row * F + c;
      const float dv = a.dout[o];
      dz = row < nv ? cG[c] * (dv - cS1[c] - (a.z2[o] - cM[c]) * cI[c] * cS2[c]) : cG[c] * dv;
      a.dz2[o] = dz;
    }
    const float dav = dropv(d1, (uint32_t)(row * F + c), dz);
    das[r * LD + c] = dav;
    if (row < a.N) a.da[(int64_t)row * F + c] = dav;
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  for (int t = w; t < F / 16; t += 4) {
    const int n0 = 16 * t, col = n0 + i;
    f4v acc = tile_mma<false>(das, LD, a.Wo, F, 0, F, n0);
    if (a.dOp == nullptr) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + 4 * g + r;
        if (row < a.N) a.dO[(int64_t)row * F + col] = acc[r];
      }
    } else {
      // a 16-column tile holds two heads (lanes i < 8, i >= 8): delta by an xor tree over
      // the 8 lanes of a head
      const int h = col >> 3, d = col & 7;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + 4 * g + r;
        const float v = row < a.N ? acc[r] : 0.f;
        float pd = row < a.N ? v * a.O[(int64_t)row * F + col] : 0.f;
        pd += __shfl_xor(pd, 1);
        pd += __shfl_xor(pd, 2);
        pd += __shfl_xor(pd, 4);
        if (row < a.Nq) {
          a.dOp[a8_pair_idx(h, a.Nq, row, d)] = v;
          a.dOq[a8_quad_idx(h, a.Nq, row, d)] = v;
          if (d == 0) a.ndelta[(int64_t)h * a.Nq + row] = -pd;
        }
      }
    }
  }
}

// Backward 4 (join): dx = [dAB | dqkv] [Wab; Win] + dZ[:, :F] + dz1 + dz2 ;
// layer > 0: g_prev = dx * [x > 0] and the previous layer's pair statistics;
// layer 0: dx0 = dx on valid rows.
struct NodeBwd {
  const float* dAB;    // [N, 2F]
  const float* dqkv;   // [N, 3F]
  const float* Wab;    // [2F, F]
  const float* Win;    // [3F, F]
  const float* dZ;     // [N, 17F] (first F columns)
  const float* dz1;
  const float* dz2;
  const float* x;      // this layer's input (relu output of the previous layer)
  float* out;          // g_prev or dx0 [N, F]
  int has_prev;
  const float* z3p;    // previous layer's z3
  const float* savedp; // previous layer's saved stats
  double* psite;       // previous layer's bwd pair site
  const int* nvp;
  int N;
};

template <int F>
__global__ void __launch_bounds__(256) node_bwd_kernel(NodeBwd a) {
  constexpr int K = 5 * F, LD = K + 4;
  __shared__ __attribute__((aligned(16))) float gs[BM * LD];
  const int nv = a.nvp ? min(*a.nvp, a.N) : a.N;
  const int row0 = blockIdx.x * BM;
  for (int idx = threadIdx.x; idx < BM * K / 4; idx += 256) {
    const int r = idx / (K / 4), c = (idx % (K / 4)) * 4, row = row0 + r;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < a.N)
      v = c < 2 * F ? *reinterpret_cast<const float4*>(a.dAB + (int64_t)row * 2 * F + c)
                    : *reinterpret_cast<const float4*>(a.dqkv + (int64_t)row * 3 * F + (c - 2 * F));
    *reinterpret_cast<float4*>(gs + r * LD + c) = v;
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  for (int t = w; t < F / 16; t += 4) {
    const int n0 = 16 * t, col = n0 + i;
    f4v acc = tile_mma<false>(gs, LD, a.Wab, F, 0, 2 * F, n0);
    acc += tile_mma<false>(gs + 2 * F, LD, a.Win, F, 0, 3 * F, n0);
    const float m3 = a.has_prev ? a.savedp[S_M3 * F + col] : 0.f;
    const float i3 = a.has_prev ? a.savedp[S_I3 * F + col] : 0.f;
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + 4 * g + r;
      if (row < a.N) {
        const int64_t o = (int64_t)row * F + col;
        float v = acc[r] + a.dZ[(int64_t)row * 17 * F + col] + a.dz1[o] + a.dz2[o];
        if (a.has_prev) {
          v = (row < nv && a.x[o] > 0.f) ? v : 0.f;
          if (row < nv) {
            s1 += v;
            s2 += (double)v * (double)((a.z3p[o] - m3) * i3);
          }
        } else if (row >= nv) {
          v = 0.f;
        }
        a.out[o] = v;
      }
    }
    if (a.has_prev) {
      col_sum_add(s1, a.psite, 2, 0, F, col);
      col_sum_add(s2, a.psite, 2, 1, F, col);
    }
  }
}

// ------------------------------------------------------------------------------------
// Edge rows (E ~ 10 x N): the PNAPlus edge term C = r Wr^T + e Wd^T + bc and its dgrad
// dr = dC Wr (optionally masked by r > 0, the ReLU of the radial embedding) and
// de (+)= dC Wd, accumulated in place over the layers (one launch each way per layer,
// replacing GEMM + addmm + copy library calls).
struct EdgeFwd {
  const float* r;   // [E, F]
  const float* e;   // [E, D]
  const float* Wr;  // [F, F]
  const float* Wd;  // [F, D]
  const float* bc;  // [F]
  float* C;         // [E, F]
  int E;
};

template <int F, int D>
__device__ __forceinline__ void edge_fwd_body(const EdgeFwd& a);

template <int F, int D>
__global__ void __launch_bounds__(256) edge_fwd_kernel(EdgeFwd a) {
  edge_fwd_body<F, D>(a);
}

template <int F, int D>
__device__ __forceinline__ void edge_fwd_body(const EdgeFwd& a) {
  constexpr int K = F + D, LD = K + 4;
  __shared__ __attribute__((aligned(16))) float xs[BM * LD];
  const int row0 = blockIdx.x * BM;
  for (int idx = threadIdx.x; idx < BM * K / 4; idx += 256) {
    const int rr = idx / (K / 4), c = (idx % (K / 4)) * 4, row = row0 + rr;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < a.E)
      v = c < F ? *reinterpret_cast<const float4*>(a.r + (int64_t)row * F + c)
                : *reinterpret_cast<const float4*>(a.e + (int64_t)row * D + (c - F));
    *reinterpret_cast<float4*>(xs + rr * LD + c) = v;
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  for (int t = w; t < F / 16; t += 4) {
    const int n0 = 16 * t, col = n0 + i;
    f4v acc = tile_mma<true>(xs, LD, a.Wr + (int64_t)n0 * F, F, 0, F, 0);
    acc += tile_mma<true>(xs + F, LD, a.Wd + (int64_t)n0 * D, D, 0, D, 0);
    const float bias = a.bc[col];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + 4 * g + r;
      if (row < a.E) a.C[(int64_t)row * F + col] = acc[r] + bias;
    }
  }
}

// Every layer's edge term in ONE launch (blockIdx.y = layer), the 16-row body above per
// workgroup.  (A 64-row form with the layer's [Wr | Wd] staged in LDS ran slower, 35.6 vs
// 3 x 10.3 us on MI355X: 67 KB of LDS left 2 workgroups per CU and nothing overlapped the
// staging loads.)
constexpr int kEdgeMaxL = 8;
struct EdgeFwdMulti {
  const float* r[kEdgeMaxL];   // [E, F] per layer
  const float* e;              // [E, D]
  const float* Wr[kEdgeMaxL];  // [F, F]
  const float* Wd[kEdgeMaxL];  // [F, D]
  const float* bc[kEdgeMaxL];  // [F]
  float* C[kEdgeMaxL];         // [E, F]
  int E;
};

template <int F, int D>
__global__ void __launch_bounds__(256) edge_fwd_multi_kernel(EdgeFwdMulti m) {
  const int l = blockIdx.y;
  edge_fwd_body<F, D>(EdgeFwd{m.r[l], m.e, m.Wr[l], m.Wd[l], m.bc[l], m.C[l], m.E});
}

struct EdgeBwd {
  const float* dC;   // [E, F]
  const float* Wr;   // [F, F]
  const float* Wd;   // [F, D]
  const float* rmask;  // [E, F] or null: dr *= (rmask > 0)
  float* dr;         // [E, F]
  float* de;         // [E, D]
  int accumulate;    // de += (else =)
  int E;
  // optional radial-basis gradient: drbf (+)= dr Wemb + dG Wlin  ([E, K], K <= 16)
  const float* dG;   // [E, F]
  const float* Wemb; // [F, K]
  const float* Wlin; // [F, K]
  float* drbf;
  int K;
  int rbf_acc;
};

template <int F, int D>
__global__ void __launch_bounds__(256) edge_bwd_kernel(EdgeBwd a) {
  constexpr int LD = F + 4, LD2 = 2 * F + 4;
  __shared__ __attribute__((aligned(16))) float gs[BM * LD];
  __shared__ __attribute__((aligned(16))) float rs[BM * LD2];  // [dr masked | dG] for drbf
  const int row0 = blockIdx.x * BM;
  for (int idx = threadIdx.x; idx < BM * F / 4; idx += 256) {
    const int rr = idx / (F / 4), c = (idx % (F / 4)) * 4, row = row0 + rr;
    *reinterpret_cast<float4*>(gs + rr * LD + c) =
        row < a.E ? *reinterpret_cast<const float4*>(a.dC + (int64_t)row * F + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  constexpr int T = (F + D) / 16;
  for (int t = w; t < T; t += 4) {
    const int n0 = 16 * t;
    const bool isr = n0 < F;
    const int col = (isr ? n0 : n0 - F) + i;
    f4v acc = isr ? tile_mma<false>(gs, LD, a.Wr, F, 0, F, n0) : tile_mma<false>(gs, LD, a.Wd, D, 0, F, n0 - F);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + 4 * g + r;
      if (row >= a.E) continue;
      if (isr) {
        const int64_t o = (int64_t)row * F + col;
        const float v = (a.rmask == nullptr || a.rmask[o] > 0.f) ? acc[r] : 0.f;
        a.dr[o] = v;
        rs[(4 * g + r) * LD2 + col] = v;
      } else {
        const int64_t o = (int64_t)row * D + col;
        a.de[o] = a.accumulate ? a.de[o] + acc[r] : acc[r];
      }
    }
  }
  if (a.drbf == nullptr) return;
  // rows past E were skipped above: keep their LDS rows zero
  for (int idx = threadIdx.x; idx < BM * F; idx += 256) {
    const int rr = idx / F, c = idx % F, row = row0 + rr;
    rs[rr * LD2 + F + c] = row < a.E ? a.dG[(int64_t)row * F + c] : 0.f;
    if (row >= a.E) rs[rr * LD2 + c] = 0.f;
  }
  __syncthreads();
  if (w == 0) {
    f4v acc = f4z();
    for (int kb = 0; kb < 2 * F; kb += 16) {
      const float4 xa = *reinterpret_cast<const float4*>(rs + i * LD2 + kb + 4 * g);
      const int k = kb + 4 * g;
      const float* Wsrc = k < F ? a.Wemb + (int64_t)k * a.K : a.Wlin + (int64_t)(k - F) * a.K;
      const bool ok = i < a.K;
      const float b0 = ok ? Wsrc[i] : 0.f, b1 = ok ? Wsrc[a.K + i] : 0.f;
      const float b2 = ok ? Wsrc[2 * a.K + i] : 0.f, b3 = ok ? Wsrc[3 * a.K + i] : 0.f;
      acc = mfma(xa.x, b0, acc);
      acc = mfma(xa.y, b1, acc);
      acc = mfma(xa.z, b2, acc);
      acc = mfma(xa.w, b3, acc);
    }
    if (i < a.K) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + 4 * g + r;
        if (row < a.E) {
          float* o = a.drbf + (int64_t)row * a.K + i;
          *o = a.rbf_acc ? *o + acc[r] : acc[r];
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// GPS input embeddings (reference Base.py:229-243, _embedding):
//   node: x0 = node_lin(cat[node_emb(x), pos_emb(pe)]),  rows >= nv -> 0
//   edge: e  = edge_lin(cat[edge_emb(edge_attr), rel_pos_emb(rel_pe)])
// all bias-free: y = [A Wa^T | B Wb^T] Wl^T with narrow A, B (1-16 columns).  One launch
// per embedding: the [M, 2F] concat tile is built in LDS and multiplied on the spot.
// Backward needs no per-row pass at all: with the narrow products Ta = dy^T A [F, ka] and
// Tb = dy^T B [F, kb] (two rows of the encoder's grouped weight-gradient launch),
//   dWl = [Ta Wa^T | Tb Wb^T],  dWa = Wl[:, :F]^T Ta,  dWb = Wl[:, F:]^T Tb
// (gf_finish below), so neither the [M, 2F] concat nor d[concat] is ever written.
struct EmbFwd {
  const float* A;   // [M, ka]
  const float* B;   // [M, kb]
  const float* Wa;  // [F, ka]
  const float* Wb;  // [F, kb]
  const float* Wl;  // [F, 2F]
  float* y;         // [M, F]
  int ka, kb, M;
  const int* nvp;   // rows >= *nvp -> 0 (node embedding of a padded batch) or null
};

template <int F>
__global__ void __launch_bounds__(256) emb_fwd_kernel(EmbFwd a) {
  constexpr int LD = 2 * F + 4;
  __shared__ __attribute__((aligned(16))) float abs_[BM * LD];
  __shared__ float in[BM][33];       // [A | B] of the tile, <= 16 + 16 columns
  __shared__ float wab[2 * F][17];   // [Wa ; Wb] rows (<= 16 columns each), staged with the tile
  const int row0 = blockIdx.x * BM;
  const int kt = a.ka + a.kb;
  for (int idx = threadIdx.x; idx < BM * kt; idx += 256) {
    const int r = idx / kt, c = idx % kt, row = row0 + r;
    float v = 0.f;
    if (row < a.M) v = c < a.ka ? a.A[(int64_t)row * a.ka + c] : a.B[(int64_t)row * a.kb + (c - a.ka)];
    in[r][c] = v;
  }
  // (the first-stage weights were read from global memory inside the dot loops below: a
  // dependent L2 round trip per k, ~10 us of the edge embedding's 14)
  for (int idx = threadIdx.x; idx < F * kt; idx += 256) {
    const int c = idx / kt, k = idx % kt;
    if (k < a.ka)
      wab[c][k] = a.Wa[c * a.ka + k];
    else
      wab[F + c][k - a.ka] = a.Wb[c * a.kb + (k - a.ka)];
  }
  __syncthreads();
  // first stage (K <= 16): plain fp32 dot products, one output per thread-iteration
  for (int idx = threadIdx.x; idx < BM * 2 * F; idx += 256) {
    const int r = idx / (2 * F), c = idx % (2 * F);
    float acc = 0.f;
    if (c < F) {
      for (int k = 0; k < a.ka; ++k) acc = fmaf(in[r][k], wab[c][k], acc);
    } else {
      for (int k = 0; k < a.kb; ++k) acc = fmaf(in[r][a.ka + k], wab[c][k], acc);
    }
    abs_[r * LD + c] = acc;
  }
  __syncthreads();
  const int nv = a.nvp ? min(*a.nvp, a.M) : a.M;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  for (int t = w; t < F / 16; t += 4) {
    const int n0 = 16 * t, col = n0 + i;
    f4v acc = tile_mma<true>(abs_, LD, a.Wl + (int64_t)n0 * 2 * F, 2 * F, 0, 2 * F, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + 4 * g + r;
      if (row < a.M) a.y[(int64_t)row * F + col] = row < nv ? acc[r] : 0.f;
    }
  }
}

// ------------------------------------------------------------------------------------
// Weight-gradient epilogue of the encoder (one launch after the grouped wgrad reduction):
//   * per layer, the backward of pna_wprep_fwd (csrc/pna.hip): dW [F, 3F], db, dencW, dencb
//     from dWab, dWr, dWd, dbc;
//   * per embedding, dWl / dWa / dWb from the narrow products Ta, Tb (see EmbFwd);
//   * dfreq = diag(drbf^T drbf/dfreq).
// One thread per output element, dot products of length <= 3F with 4 partial sums.
constexpr int kFinMaxL = 8;
struct FinWprep {
  const float *dWab, *dWr, *dWd, *dbc, *W, *encW, *encb;
  float *dW, *db, *dencW, *dencb;
};
struct FinEmb {
  const float *Ta, *Tb, *Wa, *Wb, *Wl;
  float *dWa, *dWb, *dWl;
  int ka, kb;
};
// workgroups are assigned to jobs on the host (a job's parameters are then uniform across
// the workgroup: scalar loads, not per-lane loads from the kernarg segment)
struct Finish {
  FinWprep wp[kFinMaxL];
  FinEmb em[2];
  const float* dfw;  // [K, K] or null
  float* dfreq;      // [K]
  int L, ne, F, d, K;
  int per_l, per_e[2];
  int blk_l, blk_e[2], blk_f;  // workgroups per layer job / per embedding job / dfreq
};

__device__ __forceinline__ float fin_dot(const float* __restrict__ a, int sa, const float* __restrict__ b, int sb,
                                         int n) {
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int k = 0;
  for (; k + 8 <= n; k += 8) {
    float x[8], y[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      x[u] = a[(int64_t)(k + u) * sa];
      y[u] = b[(int64_t)(k + u) * sb];
    }
#pragma unroll
    for (int u = 0; u < 8; u += 4) {
      a0 = fmaf(x[u], y[u], a0);
      a1 = fmaf(x[u + 1], y[u + 1], a1);
      a2 = fmaf(x[u + 2], y[u + 2], a2);
      a3 = fmaf(x[u + 3], y[u + 3], a3);
    }
  }
  for (; k < n; ++k) a0 = fmaf(a[(int64_t)k * sa], b[(int64_t)k * sb], a0);
  return (a0 + a1) + (a2 + a3);
}

__global__ void __launch_bounds__(256) finish_kernel(Finish a) {
  int b = blockIdx.x;
  const int F = a.F, d = a.d, ld = 3 * F, le = d + F;
  if (b < a.L * a.blk_l) {
    const FinWprep& w = a.wp[b / a.blk_l];
    int q = (b % a.blk_l) * 256 + threadIdx.x;
    if (q >= a.per_l) return;
    if (q < 2 * F * F) {  // dW[:, :2F] <- dWab (row blocks [W_i; W_j])
      const int o = q / (2 * F), c = q % (2 * F);
      w.dW[o * ld + c] = w.dWab[((c / F) * F + o) * F + (c % F)];
      return;
    }
    q -= 2 * F * F;
    if (q < F) {
      w.db[q] = w.dbc[q];
      return;
    }
    q -= F;
    if (q < F * F) {  // dW_e[o, j] = dWr[o,:] . encW[j, d:] + dWd[o,:] . encW[j, :d] + dbc[o] encb[j]
      const int o = q / F, j = q % F;
      float v = fin_dot(w.dWr + o * F, 1, w.encW + j * le + d, 1, F) + w.dbc[o] * w.encb[j];
      if (d > 0) v += fin_dot(w.dWd + o * d, 1, w.encW + j * le, 1, d);
      w.dW[o * ld + 2 * F + j] = v;
      return;
    }
    q -= F * F;
    if (q < F * le) {  // dencW[j, c] = sum_o W_e[o, j] [dWd | dWr][o, c]
      const int j = q / le, c = q % le;
      w.dencW[q] = c < d ? fin_dot(w.W + 2 * F + j, ld, w.dWd + c, d, F)
                         : fin_dot(w.W + 2 * F + j, ld, w.dWr + (c - d), F, F);
      return;
    }
    q -= F * le;
    w.dencb[q] = fin_dot(w.W + 2 * F + q, ld, w.dbc, 1, F);
    return;
  }
  b -= a.L * a.blk_l;
  for (int m = 0; m < a.ne; ++m) {
    if (b >= a.blk_e[m]) {
      b -= a.blk_e[m];
      continue;
    }
    const FinEmb& e = a.em[m];
    int t = b * 256 + threadIdx.x;
    if (t >= a.per_e[m]) return;
    if (t < 2 * F * F) {  // dWl[o, c]
      const int o = t / (2 * F), c = t % (2 * F);
      e.dWl[t] = c < F ? fin_dot(e.Ta + o * e.ka, 1, e.Wa + c * e.ka, 1, e.ka)
                       : fin_dot(e.Tb + o * e.kb, 1, e.Wb + (c - F) * e.kb, 1, e.kb);
      return;
    }
    t -= 2 * F * F;
    if (t < F * e.ka) {  // dWa[c, k] = sum_o Wl[o, c] Ta[o, k]
      const int c = t / e.ka, k = t % e.ka;
      e.dWa[t] = fin_dot(e.Wl + c, 2 * F, e.Ta + k, e.ka, F);
      return;
    }
    t -= F * e.ka;
    const int c = t / e.kb, k = t % e.kb;  // dWb[c, k] = sum_o Wl[o, F + c] Tb[o, k]
    e.dWb[t] = fin_dot(e.Wl + F + c, 2 * F, e.Tb + k, e.kb, F);
    return;
  }
  if (threadIdx.x < a.K) a.dfreq[threadIdx.x] = a.dfw[threadIdx.x * a.K + threadIdx.x];
}

// ====================================================================================
// host side
static Drop mk_drop(const c10::optional<at::Tensor>& rng, int64_t salt, double p) {
  Drop d;
  d.rng = (rng.has_value() && rng->defined() && p > 0.0) ? rng->data_ptr<int64_t>() : nullptr;
  d.salt = salt;
  d.p = d.rng ? (float)p : 0.f;
  return d;
}

static const int* nvptr(const c10::optional<at::Tensor>& nv) {
  return (nv.has_value() && nv->defined()) ? nv->data_ptr<int>() : nullptr;
}

template <typename T>
static T* optp(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<T>() : nullptr;
}

static BNP mk_bnp(const at::Tensor& w, const at::Tensor& b, const c10::optional<at::Tensor>& rm,
                  const c10::optional<at::Tensor>& rv, const c10::optional<at::Tensor>& nbt, double mom, double eps) {
  BNP p;
  p.w = w.data_ptr<float>();
  p.b = b.data_ptr<float>();
  p.rm = optp<float>(rm);
  p.rv = optp<float>(rv);
  p.nbt = optp<int64_t>(nbt);
  p.mom = (float)mom;
  p.eps = (float)eps;
  return p;
}

#define HY_GF_DISPATCH(F, KERN, GRID, BLOCK, ARGS)                                   \
  do {                                                                               \
    if ((F) == 64)                                                                   \
      KERN<64><<<(GRID), (BLOCK), 0, stream()>>>(ARGS);                              \
    else if ((F) == 32)                                                              \
      KERN<32><<<(GRID), (BLOCK), 0, stream()>>>(ARGS);                              \
    else                                                                             \
      HY_CHECK(false, "gps_fused: hidden dim must be 32 or 64, got ", (F));          \
  } while (0)

static void chk(const at::Tensor& t, int64_t r, int64_t c, const char* n) {
  HY_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.dim() == 2 && t.size(0) == r &&
               t.size(1) == c,
           "gps_fused: ", n, " must be a contiguous fp32 GPU tensor [", r, ", ", c, "]");
}

// pair site / stats helpers: `acc` is one layer's accumulator block
// [fwd1 | fwd2 | fwd3 | bwd pair | bwd12] = NREP x (2 + 2 + 2 + 2 + 3) x F statistics of
// three 64-bit fixed-point words each (col_sum_add), held in a float64 tensor.
constexpr int kSiteStride = NREP * 11;
static double* site_ptr(const at::Tensor& acc, int which, int F) {
  // which: 0 fwd BN1, 1 fwd BN2, 2 fwd BN3, 3 bwd pair, 4 bwd BN1/BN2
  static const int off[5] = {0, 2, 4, 6, 8};
  return acc.data_ptr<double>() + 3 * (int64_t)NREP * off[which] * F;  // 3 words per statistic
}

// ---- forward ops --------------------------------------------------------------------
std::vector<at::Tensor> gf_node_fwd(const at::Tensor& src, const at::Tensor& Wab, const at::Tensor& Win,
                                    const at::Tensor& bin, const c10::optional<at::Tensor>& nv,
                                    const c10::optional<at::Tensor>& prev_acc, const c10::optional<at::Tensor>& prev_saved,
                                    const std::vector<at::Tensor>& prev_bn, const c10::optional<at::Tensor>& rm3,
                                    const c10::optional<at::Tensor>& rv3, const c10::optional<at::Tensor>& nbt3,
                                    const c10::optional<at::Tensor>& rm4, const c10::optional<at::Tensor>& rv4,
                                    const c10::optional<at::Tensor>& nbt4, double mom3, double eps3, double mom4,
                                    double eps4, const c10::optional<at::Tensor>& zero_buf, bool packed) {
  const int64_t N = src.size(0), F = src.size(1);
  chk(src, N, F, "src");
  chk(Wab, 2 * F, F, "Wab");
  chk(Win, 3 * F, F, "Win");
  auto x = at::empty({N, F}, src.options()), AB = at::empty({N, 2 * F}, src.options());
  const int64_t H8 = F / 8, Nq = (N + 15) / 16 * 16;
  std::vector<at::Tensor> pk;
  at::Tensor qkv;
  if (packed) {
    HY_CHECK(F % 8 == 0, "gf_node_fwd: packed attention operands need 8-wide heads");
    for (int j = 0; j < 3; ++j) {
      pk.push_back(at::empty({H8, Nq, 8}, src.options()));
      pk.push_back(at::empty({H8, Nq / 4, 8, 4}, src.options()));
    }
  } else {
    qkv = at::empty({N, 3 * F}, src.options());
  }
  std::vector<at::Tensor> ret = {x, AB};
  if (packed)
    ret.insert(ret.end(), pk.begin(), pk.end());
  else
    ret.push_back(qkv);
  if (N == 0) return ret;
  NodeFwd a{};
  a.Nq = (int)Nq;
  for (int j = 0; j < 6; ++j) a.pk[j] = packed ? pk[j].data_ptr<float>() : nullptr;
  a.src = src.data_ptr<float>();
  a.has_prev = prev_acc.has_value() && prev_acc->defined();
  if (a.has_prev) {
    HY_CHECK(prev_bn.size() == 4, "gf_node_fwd: prev_bn = [w3, b3, w4, b4]");
    a.prev.site = site_ptr(*prev_acc, 2, (int)F);
    a.prev.bn3 = mk_bnp(prev_bn[0], prev_bn[1], rm3, rv3, nbt3, mom3, eps3);
    a.prev.bn4 = mk_bnp(prev_bn[2], prev_bn[3], rm4, rv4, nbt4, mom4, eps4);
    a.prev.saved = prev_saved->data_ptr<float>();
  }
  a.Wab = Wab.data_ptr<float>();
  a.Win = Win.data_ptr<float>();
  a.bin = bin.data_ptr<float>();
  a.x = x.data_ptr<float>();
  a.AB = AB.data_ptr<float>();
  a.qkv = packed ? nullptr : qkv.data_ptr<float>();
  a.nvp = nvptr(nv);
  a.N = (int)N;
  a.zero_buf = optp<double>(zero_buf);
  a.zero_n = a.zero_buf ? zero_buf->numel() : 0;
  HY_GF_DISPATCH(F, node_fwd_kernel, ceil_div(Nq, BM), 256, a);
  return ret;
}

at::Tensor gf_oproj_fwd(const at::Tensor& o, const at::Tensor& Wo, const at::Tensor& bo, const at::Tensor& x,
                        const at::Tensor& acc, const c10::optional<at::Tensor>& rng, int64_t salt, double p,
                        const c10::optional<at::Tensor>& nv) {
  const int64_t N = o.size(0), F = o.size(1);
  chk(o, N, F, "o");
  chk(x, N, F, "x");
  chk(Wo, F, F, "Wo");
  auto z2 = at::empty({N, F}, o.options());
  if (N == 0) return z2;
  OprojFwd a{o.data_ptr<float>(), Wo.data_ptr<float>(), bo.data_ptr<float>(), x.data_ptr<float>(),
             z2.data_ptr<float>(), site_ptr(acc, 1, (int)F), mk_drop(rng, salt, p), nvptr(nv), (int)N};
  HY_GF_DISPATCH(F, oproj_fwd_kernel, ceil_div(N, BM), 256, a);
  return z2;
}

// oproj + post in one launch (oproj_post_fwd_kernel): returns [z2, p, z1]
std::vector<at::Tensor> gf_oproj_post_fwd(const at::Tensor& o, const at::Tensor& Wo, const at::Tensor& bo,
                                          const at::Tensor& Z, const at::Tensor& Wp, const at::Tensor& bp,
                                          const at::Tensor& Wl, const at::Tensor& bl, const at::Tensor& x,
                                          const at::Tensor& acc, const c10::optional<at::Tensor>& rng, int64_t salt1,
                                          int64_t salt0, double p, const c10::optional<at::Tensor>& nv) {
  const int64_t N = x.size(0), F = x.size(1);
  chk(o, N, F, "o");
  chk(x, N, F, "x");
  chk(Wo, F, F, "Wo");
  chk(Z, N, 17 * F, "Z");
  chk(Wp, F, 17 * F, "Wpost");
  chk(Wl, F, F, "Wlin");
  auto z2 = at::empty({N, F}, x.options()), pp = at::empty({N, F}, x.options()), z1 = at::empty({N, F}, x.options());
  if (N == 0) return {z2, pp, z1};
  OprojFwd oa{o.data_ptr<float>(), Wo.data_ptr<float>(), bo.data_ptr<float>(), x.data_ptr<float>(),
              z2.data_ptr<float>(), site_ptr(acc, 1, (int)F), mk_drop(rng, salt1, p), nvptr(nv), (int)N};
  PostFwd pa{Z.data_ptr<float>(), Wp.data_ptr<float>(), bp.data_ptr<float>(), Wl.data_ptr<float>(),
             bl.data_ptr<float>(), x.data_ptr<float>(), pp.data_ptr<float>(), z1.data_ptr<float>(),
             site_ptr(acc, 0, (int)F), mk_drop(rng, salt0, p), nvptr(nv), (int)N};
  const int nb = ceil_div(N, BM);
  if (F == 64)
    oproj_post_fwd_kernel<64><<<2 * nb, 512, 0, stream()>>>(pa, oa, nb);
  else if (F == 32)
    oproj_post_fwd_kernel<32><<<2 * nb, 512, 0, stream()>>>(pa, oa, nb);
  else
    HY_CHECK(false, "gps_fused: hidden dim must be 32 or 64, got ", F);
  return {z2, pp, z1};
}

std::vector<at::Tensor> gf_post_fwd(const at::Tensor& Z, const at::Tensor& Wp, const at::Tensor& bp,
                                    const at::Tensor& Wl, const at::Tensor& bl, const at::Tensor& x,
                                    const at::Tensor& acc, const c10::optional<at::Tensor>& rng, int64_t salt, double p,
                                    const c10::optional<at::Tensor>& nv) {
  const int64_t N = x.size(0), F = x.size(1);
  chk(Z, N, 17 * F, "Z");
  chk(Wp, F, 17 * F, "Wpost");
  chk(Wl, F, F, "Wlin");
  auto pp = at::empty({N, F}, x.options()), z1 = at::empty({N, F}, x.options());
  if (N == 0) return {pp, z1};
  PostFwd a{Z.data_ptr<float>(), Wp.data_ptr<float>(), bp.data_ptr<float>(), Wl.data_ptr<float>(),
            bl.data_ptr<float>(), x.data_ptr<float>(), pp.data_ptr<float>(), z1.data_ptr<float>(),
            site_ptr(acc, 0, (int)F), mk_drop(rng, salt, p), nvptr(nv), (int)N};
  HY_GF_DISPATCH(F, post_fwd_kernel, ceil_div(N, BM), 512, a);
  return {pp, z1};
}

std::vector<at::Tensor> gf_mlp_fwd(const at::Tensor& z1, const at::Tensor& z2, const at::Tensor& acc,
                                   const at::Tensor& saved, const std::vector<at::Tensor>& bn,
                                   const c10::optional<at::Tensor>& rm1, const c10::optional<at::Tensor>& rv1,
                                   const c10::optional<at::Tensor>& nbt1, const c10::optional<at::Tensor>& rm2,
                                   const c10::optional<at::Tensor>& rv2, const c10::optional<at::Tensor>& nbt2,
                                   double mom1, double eps1, double mom2, double eps2, const at::Tensor& W1,
                                   const at::Tensor& b1, const at::Tensor& W2, const at::Tensor& b2,
                                   const c10::optional<at::Tensor>& rng, int64_t salt2, int64_t salt3, double p,
                                   const c10::optional<at::Tensor>& nv) {
  const int64_t N = z1.size(0), F = z1.size(1);
  chk(z1, N, F, "z1");
  chk(z2, N, F, "z2");
  chk(W1, 2 * F, F, "W1");
  chk(W2, F, 2 * F, "W2");
  HY_CHECK(bn.size() == 4, "gf_mlp_fwd: bn = [w1, b1, w2, b2]");
  auto out = at::empty({N, F}, z1.options()), md = at::empty({N, 2 * F}, z1.options()),
       z3 = at::empty({N, F}, z1.options());
  if (N == 0) return {out, md, z3};
  MlpFwd a{};
  a.z1 = z1.data_ptr<float>();
  a.z2 = z2.data_ptr<float>();
  a.site1 = site_ptr(acc, 0, (int)F);
  a.site2 = site_ptr(acc, 1, (int)F);
  a.bn1 = mk_bnp(bn[0], bn[1], rm1, rv1, nbt1, mom1, eps1);
  a.bn2 = mk_bnp(bn[2], bn[3], rm2, rv2, nbt2, mom2, eps2);
  a.saved = saved.data_ptr<float>();
  a.W1 = W1.data_ptr<float>();
  a.b1 = b1.data_ptr<float>();
  a.W2 = W2.data_ptr<float>();
  a.b2 = b2.data_ptr<float>();
  a.out = out.data_ptr<float>();
  a.md = md.data_ptr<float>();
  a.z3 = z3.data_ptr<float>();
  a.site3 = site_ptr(acc, 2, (int)F);
  a.drop2 = mk_drop(rng, salt2, p);
  a.drop3 = mk_drop(rng, salt3, p);
  a.nvp = nvptr(nv);
  a.N = (int)N;
  HY_GF_DISPATCH(F, mlp_fwd_kernel, ceil_div(N, BM), 256, a);
  return {out, md, z3};
}

std::vector<at::Tensor> gf_final_fwd(const at::Tensor& z3, const at::Tensor& acc, const at::Tensor& saved,
                                     const std::vector<at::Tensor>& bn, const c10::optional<at::Tensor>& rm3,
                                     const c10::optional<at::Tensor>& rv3, const c10::optional<at::Tensor>& nbt3,
                                     const c10::optional<at::Tensor>& rm4, const c10::optional<at::Tensor>& rv4,
                                     const c10::optional<at::Tensor>& nbt4, double mom3, double eps3, double mom4,
                                     double eps4, const c10::optional<at::Tensor>& nv,
                                     const c10::optional<at::Tensor>& gptr) {
  const int64_t N = z3.size(0), F = z3.size(1);
  chk(z3, N, F, "z3");
  HY_CHECK(bn.size() == 4, "gf_final_fwd: bn = [w3, b3, w4, b4]");
  auto x = at::empty({N, F}, z3.options());
  const bool pool = gptr.has_value() && gptr->defined();
  const int64_t G = pool ? gptr->numel() - 1 : 0;
  if (pool) HY_CHECK(gptr->scalar_type() == at::kInt && gptr->is_contiguous(), "gf_final_fwd: gptr int32");
  auto pooled = at::empty({G, F}, z3.options());
  FinalFwd a{};
  a.z3 = z3.data_ptr<float>();
  a.pf.site = site_ptr(acc, 2, (int)F);
  a.pf.bn3 = mk_bnp(bn[0], bn[1], rm3, rv3, nbt3, mom3, eps3);
  a.pf.bn4 = mk_bnp(bn[2], bn[3], rm4, rv4, nbt4, mom4, eps4);
  a.pf.saved = saved.data_ptr<float>();
  a.x = x.data_ptr<float>();
  a.nvp = nvptr(nv);
  a.N = (int)N;
  a.gptr = pool ? gptr->data_ptr<int>() : nullptr;
  a.G = (int)G;
  a.pooled = pool ? pooled.data_ptr<float>() : nullptr;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(N * F / 4, 256), 1024));
  HY_GF_DISPATCH(F, final_fwd_kernel, blocks + (int)G, 256, a);
  return {x, pooled};
}

#define HY_GF_EDGE(F, D, KERN, GRID, ARGS)                                          \
  do {                                                                              \
    if ((F) == 64 && (D) == 64)                                                     \
      KERN<64, 64><<<(GRID), 256, 0, stream()>>>(ARGS);                             \
    else if ((F) == 32 && (D) == 32)                                                \
      KERN<32, 32><<<(GRID), 256, 0, stream()>>>(ARGS);                             \
    else                                                                            \
      HY_CHECK(false, "gps_fused edge kernels: (F, D) = (64, 64) or (32, 32)");     \
  } while (0)

// [C_0, C_1, ...] = r_l Wr_l^T + e Wd_l^T + bc_l for every layer, one launch
std::vector<at::Tensor> gf_edge_fwd_multi(at::TensorList rs, const at::Tensor& e, at::TensorList Wrs,
                                          at::TensorList Wds, at::TensorList bcs) {
  const int L = (int)rs.size();
  HY_CHECK(L >= 1 && L <= kEdgeMaxL && (int)Wrs.size() == L && (int)Wds.size() == L && (int)bcs.size() == L,
           "gf_edge_fwd_multi: 1..8 layers");
  const int64_t E = rs[0].size(0), F = rs[0].size(1), D = e.size(1);
  chk(e, E, D, "e");
  EdgeFwdMulti a{};
  a.e = e.data_ptr<float>();
  a.E = (int)E;
  std::vector<at::Tensor> out;
  for (int l = 0; l < L; ++l) {
    chk(rs[l], E, F, "r");
    chk(Wrs[l], F, F, "Wr");
    chk(Wds[l], F, D, "Wd");
    HY_CHECK(bcs[l].is_contiguous() && bcs[l].numel() == F, "gf_edge_fwd_multi: bc [F]");
    auto C = at::empty({E, F}, e.options());
    a.r[l] = rs[l].data_ptr<float>();
    a.Wr[l] = Wrs[l].data_ptr<float>();
    a.Wd[l] = Wds[l].data_ptr<float>();
    a.bc[l] = bcs[l].data_ptr<float>();
    a.C[l] = C.data_ptr<float>();
    out.push_back(C);
  }
  if (E == 0) return out;
  const dim3 grid((unsigned)ceil_div(E, (int64_t)BM), (unsigned)L);
  HY_GF_EDGE(F, D, edge_fwd_multi_kernel, grid, a);
  return out;
}

at::Tensor gf_edge_fwd(const at::Tensor& r, const at::Tensor& e, const at::Tensor& Wr, const at::Tensor& Wd,
                       const at::Tensor& bc) {
  const int64_t E = r.size(0), F = r.size(1), D = e.size(1);
  chk(r, E, F, "r");
  chk(e, E, D, "e");
  chk(Wr, F, F, "Wr");
  chk(Wd, F, D, "Wd");
  auto C = at::empty({E, F}, r.options());
  if (E == 0) return C;
  EdgeFwd a{r.data_ptr<float>(), e.data_ptr<float>(), Wr.data_ptr<float>(), Wd.data_ptr<float>(),
            bc.data_ptr<float>(), C.data_ptr<float>(), (int)E};
  HY_GF_EDGE(F, D, edge_fwd_kernel, ceil_div(E, BM), a);
  return C;
}

// dr = dC Wr (* [rmask > 0]); de = dC Wd, or de += dC Wd in place when de_acc is given
std::vector<at::Tensor> gf_edge_bwd(const at::Tensor& dC_, const at::Tensor& Wr, const at::Tensor& Wd,
                                    const c10::optional<at::Tensor>& rmask, const c10::optional<at::Tensor>& de_acc,
                                    const c10::optional<at::Tensor>& dG, const c10::optional<at::Tensor>& Wemb,
                                    const c10::optional<at::Tensor>& Wlin, const c10::optional<at::Tensor>& drbf_acc,
                                    int64_t K) {
  at::Tensor dC = dC_.contiguous();
  const int64_t E = dC.size(0), F = dC.size(1), D = Wd.size(1);
  chk(Wr, F, F, "Wr");
  chk(Wd, F, D, "Wd");
  auto dr = at::empty({E, F}, dC.options());
  const bool acc = de_acc.has_value() && de_acc->defined();
  at::Tensor de = acc ? *de_acc : at::empty({E, D}, dC.options());
  if (acc) chk(de, E, D, "de");
  const bool want_rbf = K > 0;
  const bool racc = drbf_acc.has_value() && drbf_acc->defined();
  at::Tensor drbf = racc ? *drbf_acc : (want_rbf ? at::empty({E, K}, dC.options()) : at::empty({0}, dC.options()));
  if (want_rbf) {
    HY_CHECK(K <= 16 && dG.has_value() && Wemb.has_value() && Wlin.has_value(), "gf_edge_bwd: radial operands");
    chk(*dG, E, F, "dG");
    chk(*Wemb, F, K, "Wemb");
    chk(*Wlin, F, K, "Wlin");
    chk(drbf, E, K, "drbf");
  }
  if (E == 0) return {dr, de, drbf};
  EdgeBwd a{};
  a.dC = dC.data_ptr<float>();
  a.Wr = Wr.data_ptr<float>();
  a.Wd = Wd.data_ptr<float>();
  a.rmask = optp<float>(rmask);
  a.dr = dr.data_ptr<float>();
  a.de = de.data_ptr<float>();
  a.accumulate = acc ? 1 : 0;
  a.E = (int)E;
  if (want_rbf) {
    a.dG = dG->data_ptr<float>();
    a.Wemb = Wemb->data_ptr<float>();
    a.Wlin = Wlin->data_ptr<float>();
    a.drbf = drbf.data_ptr<float>();
    a.K = (int)K;
    a.rbf_acc = racc ? 1 : 0;
  }
  HY_GF_EDGE(F, D, edge_bwd_kernel, ceil_div(E, BM), a);
  return {dr, de, drbf};
}

at::Tensor gf_embed_fwd(const at::Tensor& A_, const at::Tensor& B_, const at::Tensor& Wa, const at::Tensor& Wb,
                        const at::Tensor& Wl, const c10::optional<at::Tensor>& nv) {
  at::Tensor A = A_.contiguous(), B = B_.contiguous();
  const int64_t M = A.size(0), F = Wl.size(0), ka = A.size(1), kb = B.size(1);
  HY_CHECK(B.size(0) == M && ka >= 1 && kb >= 1 && ka <= 16 && kb <= 16 && A.scalar_type() == at::kFloat &&
               B.scalar_type() == at::kFloat,
           "gf_embed_fwd: inputs [M, 1..16] fp32");
  chk(Wa, F, ka, "Wa");
  chk(Wb, F, kb, "Wb");
  chk(Wl, F, 2 * F, "Wl");
  auto y = at::empty({M, F}, A.options());
  if (M == 0) return y;
  EmbFwd a{A.data_ptr<float>(), B.data_ptr<float>(), Wa.data_ptr<float>(), Wb.data_ptr<float>(), Wl.data_ptr<float>(),
           y.data_ptr<float>(), (int)ka, (int)kb, (int)M, nvptr(nv)};
  HY_GF_DISPATCH(F, emb_fwd_kernel, ceil_div(M, BM), 256, a);
  return y;
}

// wp: 7 tensors per layer (dWab, dWr, dWd, dbc, W_pre, encW, encb); em: 5 per embedding
// (Ta, Tb, Wa, Wb, Wl).  Returns per layer [dW_pre, db_pre, dencW, dencb], then per embedding
// [dWa, dWb, dWl], then dfreq (when dfw is given).
// Parameter-gradient outputs: the caller's tensors (e.g. the training step's flat gradient
// slots, parallel/gradslots.py) when given, else fresh ones.  outs, when present, holds one
// contiguous fp32 tensor per gradient output of the op, in output order.
static at::Tensor gout_or(const c10::optional<at::TensorList>& outs, size_t i, size_t n_expected,
                          at::IntArrayRef shape, const at::TensorOptions& opt) {
  if (!outs.has_value()) return at::empty(shape, opt);
  HY_CHECK(outs->size() == n_expected, "gradient outputs: one tensor per parameter gradient");
  const at::Tensor& t = (*outs)[i];
  int64_t n = 1;
  for (auto d : shape) n *= d;
  HY_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == n,
           "gradient outputs: contiguous fp32 tensors of the parameters' sizes");
  return t.view(shape);
}

std::vector<at::Tensor> gf_finish(const std::vector<at::Tensor>& wp, const std::vector<at::Tensor>& em,
                                  const c10::optional<at::Tensor>& dfw,
                                  c10::optional<at::TensorList> gouts) {
  HY_CHECK(wp.size() % 7 == 0 && wp.size() / 7 <= (size_t)kFinMaxL && em.size() % 5 == 0 && em.size() <= 10,
           "gf_finish: 7 tensors per layer (<= 8 layers), 5 per embedding (<= 2)");
  Finish a{};
  a.L = (int)(wp.size() / 7);
  a.ne = (int)(em.size() / 5);
  const at::Tensor& ref = a.L ? wp[4] : em[4];
  const int64_t F = a.L ? wp[4].size(0) : em[4].size(0);
  a.F = (int)F;
  a.d = a.L ? (int)(wp[5].size(1) - F) : 0;
  std::vector<at::Tensor> out;
  auto opt = ref.options();
  for (int l = 0; l < a.L; ++l) {
    const at::Tensor* t = &wp[7 * l];
    for (int u = 0; u < 7; ++u) HY_CHECK(t[u].is_contiguous() && t[u].scalar_type() == at::kFloat, "gf_finish: wp");
    HY_CHECK(t[0].numel() == 2 * F * F && t[1].numel() == F * F && t[2].numel() == F * a.d && t[3].numel() == F &&
                 t[4].size(0) == F && t[4].size(1) == 3 * F && t[5].size(0) == F && t[5].size(1) == F + a.d &&
                 t[6].numel() == F,
             "gf_finish: weight-prep shapes");
    const size_t ng = 4 * (wp.size() / 7) + 3 * (em.size() / 5) + ((dfw.has_value() && dfw->defined()) ? 1 : 0);
    auto dW = gout_or(gouts, 4 * l, ng, t[4].sizes(), opt), db = gout_or(gouts, 4 * l + 1, ng, {F}, opt);
    auto dencW = gout_or(gouts, 4 * l + 2, ng, t[5].sizes(), opt), dencb = gout_or(gouts, 4 * l + 3, ng, {F}, opt);
    a.wp[l] = FinWprep{t[0].data_ptr<float>(), t[1].data_ptr<float>(), t[2].data_ptr<float>(), t[3].data_ptr<float>(),
                       t[4].data_ptr<float>(), t[5].data_ptr<float>(), t[6].data_ptr<float>(), dW.data_ptr<float>(),
                       db.data_ptr<float>(), dencW.data_ptr<float>(), dencb.data_ptr<float>()};
    out.insert(out.end(), {dW, db, dencW, dencb});
  }
  a.per_l = (int)(3 * F * F + 2 * F + F * (F + a.d));
  a.blk_l = ceil_div(a.per_l, 256);
  int blocks = a.L * a.blk_l;
  for (int m = 0; m < a.ne; ++m) {
    const at::Tensor* t = &em[5 * m];
    for (int u = 0; u < 5; ++u) HY_CHECK(t[u].is_contiguous() && t[u].scalar_type() == at::kFloat, "gf_finish: em");
    const int64_t ka = t[2].size(1), kb = t[3].size(1);
    HY_CHECK(t[0].numel() == F * ka && t[1].numel() == F * kb && t[2].size(0) == F && t[3].size(0) == F &&
                 t[4].size(0) == F && t[4].size(1) == 2 * F,
             "gf_finish: embedding shapes");
    const size_t ng = 4 * (wp.size() / 7) + 3 * (em.size() / 5) + ((dfw.has_value() && dfw->defined()) ? 1 : 0);
    const size_t g0 = 4 * a.L + 3 * m;
    auto dWa = gout_or(gouts, g0, ng, t[2].sizes(), opt), dWb = gout_or(gouts, g0 + 1, ng, t[3].sizes(), opt);
    auto dWl = gout_or(gouts, g0 + 2, ng, t[4].sizes(), opt);
    a.em[m] = FinEmb{t[0].data_ptr<float>(), t[1].data_ptr<float>(), t[2].data_ptr<float>(), t[3].data_ptr<float>(),
                     t[4].data_ptr<float>(), dWa.data_ptr<float>(), dWb.data_ptr<float>(), dWl.data_ptr<float>(),
                     (int)ka, (int)kb};
    a.per_e[m] = (int)(2 * F * F + F * ka + F * kb);
    a.blk_e[m] = ceil_div(a.per_e[m], 256);
    blocks += a.blk_e[m];
    out.insert(out.end(), {dWa, dWb, dWl});
  }
  if (dfw.has_value() && dfw->defined()) {
    HY_CHECK(dfw->dim() == 2 && dfw->size(0) == dfw->size(1) && dfw->is_contiguous(), "gf_finish: dfw [K, K]");
    a.K = (int)dfw->size(0);
    const size_t ng = 4 * (size_t)a.L + 3 * (size_t)a.ne + 1;
    auto dfreq = gout_or(gouts, ng - 1, ng, {a.K}, opt);
    a.dfw = dfw->data_ptr<float>();
    a.dfreq = dfreq.data_ptr<float>();
    HY_CHECK(a.K <= 256, "gf_finish: dfw [K, K] with K <= 256");
    blocks += 1;
    out.push_back(dfreq);
  }
  if (blocks > 0) finish_kernel<<<blocks, 256, 0, stream()>>>(a);
  return out;
}

// ---- backward ops -------------------------------------------------------------------
at::Tensor gf_pair_stats_bwd(const c10::optional<at::Tensor>& dx, const at::Tensor& x, const at::Tensor& z3,
                             const at::Tensor& saved, const at::Tensor& acc, const c10::optional<at::Tensor>& nv,
                             const c10::optional<at::Tensor>& dpool, const c10::optional<at::Tensor>& gidx,
                             const c10::optional<at::Tensor>& gptr) {
  const int64_t N = z3.size(0), F = z3.size(1);
  chk(z3, N, F, "z3");
  chk(x, N, F, "x");
  at::Tensor d;
  if (dx.has_value() && dx->defined()) {
    d = dx->contiguous();
    chk(d, N, F, "dx");
  }
  at::Tensor dp;
  if (dpool.has_value() && dpool->defined()) {
    dp = dpool->contiguous();
    HY_CHECK(gidx.has_value() && gptr.has_value() && gidx->scalar_type() == at::kInt && gidx->numel() == N &&
                 gptr->scalar_type() == at::kInt && dp.size(0) == gptr->numel() - 1 && dp.size(1) == F,
             "gf_pair_stats_bwd: pooled gradient needs graph index / pointers");
  }
  auto g = at::empty({N, F}, z3.options());
  if (N == 0) return g;
  PairStatsBwd a{d.defined() ? d.data_ptr<float>() : nullptr, x.data_ptr<float>(), z3.data_ptr<float>(),
                 saved.data_ptr<float>(), g.data_ptr<float>(), site_ptr(acc, 3, (int)F), nvptr(nv), (int)N,
                 dp.defined() ? dp.data_ptr<float>() : nullptr, dp.defined() ? gidx->data_ptr<int>() : nullptr,
                 dp.defined() ? gptr->data_ptr<int>() : nullptr};
  HY_GF_DISPATCH(F, pair_stats_bwd_kernel, ceil_div(N, BM), 256, a);
  return g;
}

std::vector<at::Tensor> gf_mlp_bwd(const at::Tensor& g, const at::Tensor& z3, const at::Tensor& acc,
                                   const at::Tensor& saved, const at::Tensor& g3, const at::Tensor& g4, double eps3,
                                   double eps4, const at::Tensor& md, const at::Tensor& W2, const at::Tensor& W1,
                                   const at::Tensor& z1, const at::Tensor& z2, const c10::optional<at::Tensor>& rng,
                                   int64_t salt2, int64_t salt3, double p, const c10::optional<at::Tensor>& nv,
                                   c10::optional<at::TensorList> gouts) {
  const int64_t N = z3.size(0), F = z3.size(1);
  chk(g, N, F, "g");
  chk(md, N, 2 * F, "md");
  auto o = z3.options();
  auto dg = at::empty({N, F}, o), dpre = at::empty({N, 2 * F}, o), dout = at::empty({N, F}, o);
  auto dw3 = gout_or(gouts, 0, 4, {F}, o), db3 = gout_or(gouts, 1, 4, {F}, o), dw4 = gout_or(gouts, 2, 4, {F}, o),
       db4 = gout_or(gouts, 3, 4, {F}, o);
  MlpBwd a{};
  a.g = g.data_ptr<float>();
  a.z3 = z3.data_ptr<float>();
  a.psite = site_ptr(acc, 3, (int)F);
  a.saved = saved.data_ptr<float>();
  a.g3 = g3.data_ptr<float>();
  a.g4 = g4.data_ptr<float>();
  a.eps3 = (float)eps3;
  a.eps4 = (float)eps4;
  a.d3 = BNG{dw3.data_ptr<float>(), db3.data_ptr<float>()};
  a.d4 = BNG{dw4.data_ptr<float>(), db4.data_ptr<float>()};
  a.md = md.data_ptr<float>();
  a.W2 = W2.data_ptr<float>();
  a.W1 = W1.data_ptr<float>();
  a.z1 = z1.data_ptr<float>();
  a.z2 = z2.data_ptr<float>();
  a.dg = dg.data_ptr<float>();
  a.dpre = dpre.data_ptr<float>();
  a.dout = dout.data_ptr<float>();
  a.site12 = site_ptr(acc, 4, (int)F);
  a.drop2 = mk_drop(rng, salt2, p);
  a.drop3 = mk_drop(rng, salt3, p);
  a.nvp = nvptr(nv);
  a.N = (int)N;
  HY_GF_DISPATCH(F, mlp_bwd_kernel, std::max(1, ceil_div(N, BM)), 256, a);
  return {dg, dpre, dout, dw3, db3, dw4, db4};
}

std::vector<at::Tensor> gf_loc_bwd(const at::Tensor& dout, const at::Tensor& z1, const at::Tensor& acc,
                                   const at::Tensor& saved, const at::Tensor& gamma1, const at::Tensor& Wl,
                                   const at::Tensor& Wp, const c10::optional<at::Tensor>& rng, int64_t salt0, double p,
                                   const c10::optional<at::Tensor>& nv, c10::optional<at::TensorList> gouts) {
  const int64_t N = z1.size(0), F = z1.size(1);
  chk(dout, N, F, "dout");
  chk(Wp, F, 17 * F, "Wpost");
  auto o = z1.options();
  auto dz1 = at::empty({N, F}, o), dq = at::empty({N, F}, o), dp = at::empty({N, F}, o),
       dZ = at::empty({N, 17 * F}, o), dw1 = gout_or(gouts, 0, 2, {F}, o), db1 = gout_or(gouts, 1, 2, {F}, o);
  LocBwd a{dout.data_ptr<float>(), z1.data_ptr<float>(), site_ptr(acc, 4, (int)F), saved.data_ptr<float>(),
           gamma1.data_ptr<float>(), BNG{dw1.data_ptr<float>(), db1.data_ptr<float>()}, Wl.data_ptr<float>(),
           Wp.data_ptr<float>(), dz1.data_ptr<float>(), dq.data_ptr<float>(), dp.data_ptr<float>(),
           dZ.data_ptr<float>(), mk_drop(rng, salt0, p), nvptr(nv), (int)N};
  HY_GF_DISPATCH(F, loc_bwd_kernel, std::max(1, ceil_div(N, BM)), 512, a);
  return {dz1, dq, dp, dZ, dw1, db1};
}

std::vector<at::Tensor> gf_att_bwd(const at::Tensor& dout, const at::Tensor& z2, const at::Tensor& acc,
                                   const at::Tensor& saved, const at::Tensor& gamma2, const at::Tensor& Wo,
                                   const c10::optional<at::Tensor>& rng, int64_t salt1, double p,
                                   const c10::optional<at::Tensor>& nv, const c10::optional<at::Tensor>& O,
                                   c10::optional<at::TensorList> gouts) {
  const int64_t N = z2.size(0), F = z2.size(1);
  chk(dout, N, F, "dout");
  auto o = z2.options();
  const bool packed = O.has_value() && O->defined();
  auto dz2 = at::empty({N, F}, o), da = at::empty({N, F}, o), dw2 = gout_or(gouts, 0, 2, {F}, o),
       db2 = gout_or(gouts, 1, 2, {F}, o);
  auto dO = packed ? at::empty({0}, o) : at::empty({N, F}, o);
  AttBwd a{dout.data_ptr<float>(), z2.data_ptr<float>(), site_ptr(acc, 4, (int)F), saved.data_ptr<float>(),
           gamma2.data_ptr<float>(), BNG{dw2.data_ptr<float>(), db2.data_ptr<float>()}, Wo.data_ptr<float>(),
           dz2.data_ptr<float>(), da.data_ptr<float>(), packed ? nullptr : dO.data_ptr<float>(),
           mk_drop(rng, salt1, p), nvptr(nv), (int)N};
  at::Tensor ndelta, dOp, dOq;
  if (packed) {
    // with O: the 8-wide-head attention backward operands (heads H = F / 8, rows Nq = 16k)
    HY_CHECK(F % 8 == 0, "gf_att_bwd: packed attention operands need 8-wide heads");
    chk(*O, N, F, "O");
    const int64_t H = F / 8, Nq = ceil_div(N, (int64_t)BM) * BM;
    ndelta = at::empty({H, Nq}, o);
    dOp = at::empty({H, Nq, 8}, o);
    dOq = at::empty({H, Nq, 8}, o);
    a.O = O->data_ptr<float>();
    a.ndelta = ndelta.data_ptr<float>();
    a.dOp = dOp.data_ptr<float>();
    a.dOq = dOq.data_ptr<float>();
    a.Nq = (int)Nq;
  }
  HY_GF_DISPATCH(F, att_bwd_kernel, std::max(1, ceil_div(N, BM)), 256, a);
  if (packed) return {dz2, da, dO, dw2, db2, ndelta, dOp, dOq};
  return {dz2, da, dO, dw2, db2};
}

at::Tensor gf_node_bwd(const at::Tensor& dAB, const at::Tensor& dqkv, const at::Tensor& Wab, const at::Tensor& Win,
                       const at::Tensor& dZ, const at::Tensor& dz1, const at::Tensor& dz2, const at::Tensor& x,
                       const c10::optional<at::Tensor>& z3p, const c10::optional<at::Tensor>& savedp,
                       const c10::optional<at::Tensor>& accp, const c10::optional<at::Tensor>& nv) {
  const int64_t N = x.size(0), F = x.size(1);
  chk(dAB, N, 2 * F, "dAB");
  chk(dqkv, N, 3 * F, "dqkv");
  chk(dZ, N, 17 * F, "dZ");
  auto out = at::empty({N, F}, x.options());
  if (N == 0) return out;
  NodeBwd a{};
  a.dAB = dAB.data_ptr<float>();
  a.dqkv = dqkv.data_ptr<float>();
  a.Wab = Wab.data_ptr<float>();
  a.Win = Win.data_ptr<float>();
  a.dZ = dZ.data_ptr<float>();
  a.dz1 = dz1.data_ptr<float>();
  a.dz2 = dz2.data_ptr<float>();
  a.x = x.data_ptr<float>();
  a.out = out.data_ptr<float>();
  a.has_prev = accp.has_value() && accp->defined();
  if (a.has_prev) {
    a.z3p = z3p->data_ptr<float>();
    a.savedp = savedp->data_ptr<float>();
    a.psite = site_ptr(*accp, 3, (int)F);
  }
  a.nvp = nvptr(nv);
  a.N = (int)N;
  HY_GF_DISPATCH(F, node_bwd_kernel, ceil_div(N, BM), 256, a);
  return out;
}

}  // namespace gf
}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def(
      "gf_node_fwd(Tensor src, Tensor Wab, Tensor Win, Tensor bin, Tensor? nv, Tensor? prev_acc, Tensor(h!)? prev_saved, "
      "Tensor[] prev_bn, Tensor(a!)? rm3, Tensor(b!)? rv3, Tensor(c!)? nbt3, Tensor(d!)? rm4, Tensor(e!)? rv4, "
      "Tensor(f!)? nbt4, float mom3, float eps3, float mom4, float eps4, Tensor(g!)? zero_buf, bool packed) -> Tensor[]");
  m.def(
      "gf_oproj_fwd(Tensor o, Tensor Wo, Tensor bo, Tensor x, Tensor(a!) acc, Tensor? rng, int salt, float p, "
      "Tensor? nv) -> Tensor");
  m.def(
      "gf_post_fwd(Tensor Z, Tensor Wp, Tensor bp, Tensor Wl, Tensor bl, Tensor x, Tensor(a!) acc, Tensor? rng, "
      "int salt, float p, Tensor? nv) -> Tensor[]");
  m.def(
      "gf_mlp_fwd(Tensor z1, Tensor z2, Tensor(x!) acc, Tensor(a!) saved, Tensor[] bn, Tensor(b!)? rm1, Tensor(c!)? rv1, "
      "Tensor(d!)? nbt1, Tensor(e!)? rm2, Tensor(f!)? rv2, Tensor(g!)? nbt2, float mom1, float eps1, float mom2, "
      "float eps2, Tensor W1, Tensor b1, Tensor W2, Tensor b2, Tensor? rng, int salt2, int salt3, float p, "
      "Tensor? nv) -> Tensor[]");
  m.def(
      "gf_final_fwd(Tensor z3, Tensor acc, Tensor(a!) saved, Tensor[] bn, Tensor(b!)? rm3, Tensor(c!)? rv3, "
      "Tensor(d!)? nbt3, Tensor(e!)? rm4, Tensor(f!)? rv4, Tensor(g!)? nbt4, float mom3, float eps3, float mom4, "
      "float eps4, Tensor? nv, Tensor? gptr) -> Tensor[]");
  m.def("gf_embed_fwd(Tensor A, Tensor B, Tensor Wa, Tensor Wb, Tensor Wl, Tensor? nv) -> Tensor");
  m.def("gf_finish(Tensor[] wp, Tensor[] em, Tensor? dfw, Tensor[]? gouts=None) -> Tensor[]");
  m.def(
      "gf_oproj_post_fwd(Tensor o, Tensor Wo, Tensor bo, Tensor Z, Tensor Wp, Tensor bp, Tensor Wl, Tensor bl, "
      "Tensor x, Tensor(a!) acc, Tensor? rng, int salt1, int salt0, float p, Tensor? nv) -> Tensor[]");
  m.def("gf_edge_fwd(Tensor r, Tensor e, Tensor Wr, Tensor Wd, Tensor bc) -> Tensor");
  m.def("gf_edge_fwd_multi(Tensor[] r, Tensor e, Tensor[] Wr, Tensor[] Wd, Tensor[] bc) -> Tensor[]");
  m.def(
      "gf_edge_bwd(Tensor dC, Tensor Wr, Tensor Wd, Tensor? rmask, Tensor(a!)? de_acc, Tensor? dG, Tensor? Wemb, "
      "Tensor? Wlin, Tensor(b!)? drbf_acc, int K) -> Tensor[]");
  m.def(
      "gf_pair_stats_bwd(Tensor? dx, Tensor x, Tensor z3, Tensor saved, Tensor(a!) acc, Tensor? nv, Tensor? dpool, "
      "Tensor? gidx, Tensor? gptr) -> Tensor");
  m.def(
      "gf_mlp_bwd(Tensor g, Tensor z3, Tensor(a!) acc, Tensor saved, Tensor g3, Tensor g4, float eps3, float eps4, "
      "Tensor md, Tensor W2, Tensor W1, Tensor z1, Tensor z2, Tensor? rng, int salt2, int salt3, float p, Tensor? nv, "
      "Tensor[]? gouts=None) -> Tensor[]");
  m.def(
      "gf_loc_bwd(Tensor dout, Tensor z1, Tensor acc, Tensor saved, Tensor gamma1, Tensor Wl, Tensor Wp, Tensor? rng, "
      "int salt0, float p, Tensor? nv, Tensor[]? gouts=None) -> Tensor[]");
  m.def(
      "gf_att_bwd(Tensor dout, Tensor z2, Tensor acc, Tensor saved, Tensor gamma2, Tensor Wo, Tensor? rng, int salt1, "
      "float p, Tensor? nv, Tensor? O=None, Tensor[]? gouts=None) -> Tensor[]");
  m.def(
      "gf_node_bwd(Tensor dAB, Tensor dqkv, Tensor Wab, Tensor Win, Tensor dZ, Tensor dz1, Tensor dz2, Tensor x, "
      "Tensor? z3p, Tensor? savedp, Tensor(a!)? accp, Tensor? nv) -> Tensor");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("gf_node_fwd", hy::gf::gf_node_fwd);
  m.impl("gf_oproj_fwd", hy::gf::gf_oproj_fwd);
  m.impl("gf_post_fwd", hy::gf::gf_post_fwd);
  m.impl("gf_mlp_fwd", hy::gf::gf_mlp_fwd);
  m.impl("gf_final_fwd", hy::gf::gf_final_fwd);
  m.impl("gf_embed_fwd", hy::gf::gf_embed_fwd);
  m.impl("gf_finish", hy::gf::gf_finish);
  m.impl("gf_oproj_post_fwd", hy::gf::gf_oproj_post_fwd);
  m.impl("gf_edge_fwd", hy::gf::gf_edge_fwd);
  m.impl("gf_edge_fwd_multi", hy::gf::gf_edge_fwd_multi);
  m.impl("gf_edge_bwd", hy::gf::gf_edge_bwd);
  m.impl("gf_pair_stats_bwd", hy::gf::gf_pair_stats_bwd);
  m.impl("gf_mlp_bwd", hy::gf::gf_mlp_bwd);
  m.impl("gf_loc_bwd", hy::gf::gf_loc_bwd);
  m.impl("gf_att_bwd", hy::gf::gf_att_bwd);
  m.impl("gf_node_bwd", hy::gf::gf_node_bwd);
}
