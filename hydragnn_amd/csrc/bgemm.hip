// bf16 MFMA GEMM engine for gfx950 (v_mfma_f32_16x16x32_bf16, fp32 accumulate) with
// fused prologue / epilogue, built for the wide (866-channel) edge and node MLPs of the
// SC25 EGNN (reference hydragnn/models/EGCLStack.py:240-289) and the wide multi-branch
// decoder heads (Base.py:486-566).
//
// Storage convention ("padded bf16 activations"): an activation with K valid columns is
// a bf16 [rows, Kp] matrix, Kp = K rounded up to 64 (128 where it feeds a weight
// gradient), columns >= K zero except the ONES LANE at column K, which holds 1.0.  Padded
// weights are bf16 [Np, Kp] with zero pad rows/columns, so the ones lane never reaches a
// forward output, while a weight-gradient product dY^T X yields the bias gradient in its
// column K for free (sum_m dY[m, n] * 1).
//
// Kernels:
//  * nt_kernel<BM>:  C[M, Np] = epi(A[M, K] B[Np, K]^T), A optionally the K-concatenation
//    of two matrices (concat-linear inputs never materialised).  Tile BM x 128 x 64,
//    BM/64 x 2 waves of 64x64 (4x4 MFMA 16x16x32 tiles); A and B staged through LDS by
//    register double buffering with one barrier per K step; 16-byte XOR swizzle
//    (chunk ^ (row >> 1) & 7) makes the ds_read_b128 fragment reads conflict-free.  The
//    MFMA is issued as B.A^T so every lane owns 4 CONSECUTIVE output columns of one row:
//    8-byte bf16 / 16-byte fp32 epilogue stores, float4 bias / gate / gather loads.
//    Epilogue: + bias, + gathered fp32 rows addg[idx[m]], * relu'(gate), activation, fp32
//    and/or bf16 stores (pad columns forced to 0, ones lane to 1), row dot with a vector
//    (atomically accumulated; the EGNN coord_mlp's 866 -> 1 GEMV), fp32 accumulate (beta).
//  * tn_kernel:  slab[s][n][k] = sum_{m in split s} G[m, n] X[m, k] — weight gradients.
//    Both operands are [M, *] row-major: the reduction index is the row, so fragments
//    are read with ds_read_b64_tr_b16 (hardware 4x16 transpose) from a 256-byte-row LDS
//    image with a 32-byte XOR swizzle (slot ^ (m & 3 | (m >> 3 & 1) << 2)), conflict-free
//    for the transposed reads.  Split over M (rows) to fill the chip; the last split block
//    of each tile to finish (device-scope arrival counter) sums the tile's slabs in split
//    order — deterministic — into the fp32 parameter gradients (masked, strided, optional
//    accumulate) and extracts the bias gradient from the ones lane: no reduce launch.
//  * cast kernels: fp32 activation -> padded bf16 (+ ones lane, optional relu' gate), and
//    a batched weight caster writing W and W^T padded bf16 images in one launch.
//
// Block -> tile mapping is XCD-aware (bijective remap): the tiles of one A row block
// (all 128-column tiles) run on one XCD, so the row block is read into one L2.
#include "common.h"

namespace hy {
namespace bg {

typedef short s8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) s4v lds_s4v;

__device__ __forceinline__ float bf2f(uint16_t b) { return __uint_as_float((uint32_t)b << 16); }
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  bf2v v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ float lo_bf(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_bf(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

__device__ __forceinline__ f4v mfma(const s8v& a, const s8v& b, const f4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------------------ NT GEMM
struct NTArgs {
  const uint16_t* A;   // [M, lda] bf16 (k-tiles 0 .. kt1-1)
  const uint16_t* A2;  // [M, lda2] bf16 (k-tiles kt1 ..), may be null
  const uint16_t* B;   // [Np, ldb] bf16
  int lda, lda2, ldb, kt1;
  int M, N, Np, K;     // K multiple of 64; Np multiple of 128; N valid output columns
  const float* bias;   // [N] or null
  int act;             // 0 none, 1 relu, 2 silu
  const uint16_t* gate;  // multiply by (gate > 0): relu derivative from the saved output
  int ldgate;
  const float* addg;   // add addg[idx ? idx[m] : m][n] before the gate
  const int* addg_idx;
  int ldaddg;
  float* outf;         // fp32 output (columns < N), may be null
  int ldf;
  float beta;          // outf = beta * outf + v
  uint16_t* outb;      // bf16 output [M, ldo] (all Np columns: pad 0, ones lane)
  int ldo;
  int ones_col;        // column index of the ones lane in outb (-1: none)
  const float* rowvec; // rowdot[m] += sum_n act(v)[m, n] * rowvec[n]
  float* rowdot;
  int tiles_n;
  // branch-grouped mode (multi-branch heads): row m uses weight image B + bid[m] * bsB and
  // bias + bid[m] * bsbias; bid is non-decreasing (rows sorted by branch)
  const int* bid;
  int64_t bsB;
  int bsbias;
};

constexpr int BN = 128, BK = 64;

__device__ __forceinline__ int a_off(int row, int c) { return row * 128 + ((c ^ ((row >> 1) & 7)) << 4); }

// acc[i][j][r] = C[m = mb + i*16 + fr][n = nb + j*16 + 4*fg + r]
template <int NJ>
__device__ __forceinline__ void nt_epilogue(const NTArgs& p, f4v (&acc)[4][NJ], int mb, int nb, int fr, int fg,
                                            const float* bias, int br) {
  const bool fvec = (p.ldf & 3) == 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mb + i * 16 + fr;
    const bool mv = m < p.M && (br < 0 || p.bid[m] == br);
    float rd = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = nb + j * 16 + 4 * fg;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += (n + r < p.N) ? bias[n + r] : 0.f;
      }
      if (p.addg && mv) {
        const int src = p.addg_idx ? p.addg_idx[m] : m;
        const float* g = p.addg + (int64_t)src * p.ldaddg + n;
        if ((p.ldaddg & 3) == 0 && n + 3 < p.N) {
          const float4 t = *reinterpret_cast<const float4*>(g);
          v[0] += t.x; v[1] += t.y; v[2] += t.z; v[3] += t.w;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += (n + r < p.N) ? g[r] : 0.f;
        }
      }
      if (p.gate && mv) {
        const uint2 gg = *reinterpret_cast<const uint2*>(p.gate + (int64_t)m * p.ldgate + n);
        v[0] = lo_bf(gg.x) > 0.f ? v[0] : 0.f;
        v[1] = hi_bf(gg.x) > 0.f ? v[1] : 0.f;
        v[2] = lo_bf(gg.y) > 0.f ? v[2] : 0.f;
        v[3] = hi_bf(gg.y) > 0.f ? v[3] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (p.act == 1) v[r] = fmaxf(v[r], 0.f);
        else if (p.act == 2) v[r] = v[r] / (1.f + __expf(-v[r]));
        if (n + r >= p.N) v[r] = 0.f;
      }
      if (p.rowdot) {
#pragma unroll
        for (int r = 0; r < 4; ++r) rd += (n + r < p.N) ? v[r] * p.rowvec[n + r] : 0.f;
      }
      if (!mv) continue;
      if (p.outb) {
        float w[4] = {v[0], v[1], v[2], v[3]};
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n + r == p.ones_col) w[r] = 1.f;
        *reinterpret_cast<uint2*>(p.outb + (int64_t)m * p.ldo + n) = make_uint2(pack2(w[0], w[1]), pack2(w[2], w[3]));
      }
      if (p.outf && n < p.N) {
        float* o = p.outf + (int64_t)m * p.ldf + n;
        if (fvec && n + 3 < p.N) {
          float4 t = make_float4(v[0], v[1], v[2], v[3]);
          if (p.beta != 0.f) {
            const float4 q = *reinterpret_cast<const float4*>(o);
            t.x += p.beta * q.x; t.y += p.beta * q.y; t.z += p.beta * q.z; t.w += p.beta * q.w;
          }
          *reinterpret_cast<float4*>(o) = t;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) o[r] = v[r] + (p.beta != 0.f ? p.beta * o[r] : 0.f);
        }
      }
    }
    if (p.rowdot) {
      rd += __shfl_xor(rd, 16, 64);
      rd += __shfl_xor(rd, 32, 64);
      if (fg == 0 && mv) atomicAdd(p.rowdot + m, rd);
    }
  }
}

// BM x 128 tile; waves (BM/64) x WN, each wave 64 rows x (128/WN) columns
template <int BM, int WN>
__global__ __launch_bounds__(BM / 64 * WN * 64) void nt_kernel(NTArgs p) {
  constexpr int WM = BM / 64;            // waves along M
  constexpr int NTH = WM * WN * 64;
  constexpr int NJ = 128 / WN / 16;      // MFMA column tiles per wave
  constexpr int ACH = BM * 8 / NTH;      // A 16-byte chunks per thread per K step
  constexpr int BCH = BN * 8 / NTH;      // B chunks per thread
  constexpr int ABYTES = BM * 128, BBYTES = BN * 128, STAGE = ABYTES + BBYTES;
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid % WM, wn = wid / WM;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (wg / p.tiles_n) * BM, n0 = (wg % p.tiles_n) * BN;
  const int KT = p.K / BK;
  // branch range of this row tile (rows sorted by branch): one pass per branch present
  int br0 = -1, br1 = -1;
  if (p.bid) {
    br0 = p.bid[m0];
    br1 = p.bid[min(m0 + BM, p.M) - 1];
  }
  const uint16_t* Bw = p.B;

  uint4 ra[ACH], rb[BCH];
  auto load = [&](int kt) {
    const uint16_t* As;
    int ld, kk;
    if (kt < p.kt1) { As = p.A; ld = p.lda; kk = kt * BK; }
    else { As = p.A2; ld = p.lda2; kk = (kt - p.kt1) * BK; }
#pragma unroll
    for (int j = 0; j < ACH; ++j) {
      const int i = tid + j * NTH, row = i >> 3, c = i & 7;
      const int m = m0 + row;
      ra[j] = m < p.M ? *reinterpret_cast<const uint4*>(As + (int64_t)m * ld + kk + c * 8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < BCH; ++j) {
      const int i = tid + j * NTH, row = i >> 3, c = i & 7;
      rb[j] = *reinterpret_cast<const uint4*>(Bw + (int64_t)(n0 + row) * p.ldb + kt * BK + c * 8);
    }
  };
  auto store = [&](int buf) {
    uint8_t* s = lds + buf * STAGE;
#pragma unroll
    for (int j = 0; j < ACH; ++j) {
      const int i = tid + j * NTH;
      *reinterpret_cast<uint4*>(s + a_off(i >> 3, i & 7)) = ra[j];
    }
#pragma unroll
    for (int j = 0; j < BCH; ++j) {
      const int i = tid + j * NTH;
      *reinterpret_cast<uint4*>(s + ABYTES + a_off(i >> 3, i & 7)) = rb[j];
    }
  };

  const int fr = lane & 15, fg = lane >> 4;
  for (int br = br0; br <= br1; ++br) {
  Bw = p.bid ? p.B + (int64_t)br * p.bsB : p.B;
  f4v acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) load(kt + 1);
    const uint8_t* s = lds + cur * STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      s8v af[4], bfv[NJ];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = *reinterpret_cast<const s8v*>(s + a_off(wm * 64 + i * 16 + fr, ks * 4 + fg));
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        bfv[j] = *reinterpret_cast<const s8v*>(s + ABYTES + a_off(wn * NJ * 16 + j * 16 + fr, ks * 4 + fg));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma(bfv[j], af[i], acc[i][j]);
    }
    if (kt + 1 < KT) store(cur ^ 1);
    __syncthreads();
  }

  nt_epilogue<NJ>(p, acc, m0 + wm * 64, n0 + wn * NJ * 16, fr, fg,
                  p.bias ? p.bias + (p.bid ? (int64_t)br * p.bsbias : 0) : nullptr, br);
  }
}

// glds variant: A and B tiles copied global -> LDS by global_load_lds (16 bytes per lane,
// no staging registers, no ds_write pass).  The LDS image stays lane-linear (one wave
// instruction fills 8 rows x 128 bytes); the bank swizzle is applied to the per-lane
// SOURCE address (chunk ^ (row >> 1) & 7) and the identical XOR on the fragment reads.
// The next tile's copies stay in flight across the barrier: counted vmcnt + raw s_barrier
// (a __syncthreads would drain them).  Rows past M read a clamped valid row (masked in
// the epilogue).
template <int BM, int WN, bool GR>
__global__ __launch_bounds__(BM / 64 * WN * 64) void ntg_kernel(NTArgs p) {
  constexpr int WM = BM / 64;
  constexpr int NW = WM * WN;
  constexpr int NJ = 128 / WN / 16;
  constexpr int AI = BM / 8 / NW;  // glds instructions per wave for A (8 rows each)
  constexpr int BI = BN / 8 / NW;  // ... for B
  constexpr int ABYTES = BM * 128, BBYTES = BN * 128, STAGE = ABYTES + BBYTES;
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid % WM, wn = wid / WM;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (wg / p.tiles_n) * BM, n0 = (wg % p.tiles_n) * BN;
  const int KT = p.K / BK;
  const int lr = lane >> 3, ls = lane & 7;  // row within the 8-row group, LDS slot
  int br0 = -1, br1 = -1;  // branch-grouped mode: one pass per branch present in the tile
  if constexpr (GR) {
    br0 = p.bid[m0];
    br1 = p.bid[min(m0 + BM, p.M) - 1];
  }
  const uint16_t* Bw = p.B;

  auto issue = [&](int kt, int buf) {
    const uint16_t* As;
    int ld, kk;
    if (kt < p.kt1) { As = p.A; ld = p.lda; kk = kt * BK; }
    else { As = p.A2; ld = p.lda2; kk = (kt - p.kt1) * BK; }
    uint8_t* s = lds + buf * STAGE;
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int row = (wid * AI + j) * 8 + lr;
      const int m = min(m0 + row, p.M - 1);
      const int c = ls ^ ((row >> 1) & 7);
      __builtin_amdgcn_global_load_lds(As + (int64_t)m * ld + kk + c * 8,
                                       (__attribute__((address_space(3))) void*)(s + (wid * AI + j) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const int row = (wid * BI + j) * 8 + lr;
      const int c = ls ^ ((row >> 1) & 7);
      __builtin_amdgcn_global_load_lds(Bw + (int64_t)(n0 + row) * p.ldb + kt * BK + c * 8,
                                       (__attribute__((address_space(3))) void*)(s + ABYTES + (wid * BI + j) * 1024),
                                       16, 0, 0);
    }
  };

  const int fr = lane & 15, fg = lane >> 4;
  for (int br = br0; br <= br1; ++br) {
  if constexpr (GR) Bw = p.B + (int64_t)br * p.bsB;
  f4v acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  issue(0, 0);
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) {
      issue(kt + 1, cur ^ 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(AI + BI) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const uint8_t* s = lds + cur * STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      s8v af[4], bfv[NJ];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = *reinterpret_cast<const s8v*>(s + a_off(wm * 64 + i * 16 + fr, ks * 4 + fg));
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        bfv[j] = *reinterpret_cast<const s8v*>(s + ABYTES + a_off(wn * NJ * 16 + j * 16 + fr, ks * 4 + fg));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma(bfv[j], af[i], acc[i][j]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  }
  nt_epilogue<NJ>(p, acc, m0 + wm * 64, n0 + wn * NJ * 16, fr, fg,
                  p.bias ? p.bias + (GR ? (int64_t)br * p.bsbias : 0) : nullptr, GR ? br : -1);
  }
}

// ------------------------------------------------------------------------------ TN GEMM
// one destination of a fused weight-gradient reduce: out[n - n0][(k - k0) * ldk] for the
// slab rectangle [n0, n0 + N) x [k0, k0 + K), bias_out[n - n0] from slab column bias_col;
// group g (grouped products) writes at out + g * gout, bias_out + g * gbias
struct TNOut {
  float* out;
  float* bias_out;
  int ldo, ldk, n0, k0, N, K, bias_col;
  int64_t gout, gbias;
};

struct TNArgs {
  const uint16_t* G;   // [M, ldg]: output rows n
  const uint16_t* X;   // [M, ldx]: output cols k < kc1
  const uint16_t* X2;  // [M, ldx2]: output cols k >= kc1 (k - kc1), may be null
  int ldg, ldx, ldx2, kc1;
  int M, Np, Kp, rows_per_split, tiles_k, tiles_nk;
  float* slab;         // [S][Np][Kp]  ([nb][S][Np][Kp] when grouped)
  const int* boff;     // branch row offsets [nb + 1] (grouped: per-branch G^T X), or null
  int splits;
  // fused reduce: the last split block of each tile to finish (per-tile arrival counter)
  // sums the S slab tiles in split order (deterministic) into up to 3 output rectangles
  int* counters;       // [groups * tiles_nk] zero on entry, left zero on exit; null: slab only
  int nout;
  float beta;
  TNOut outs[3];
};

__device__ __forceinline__ int t_off(int m, int c16) {
  const int h = (m & 3) | (((m >> 3) & 1) << 2);
  return m * 256 + ((((c16 >> 1) ^ h)) << 5) + ((c16 & 1) << 4);
}
// byte offset of (row m, column col) for the transposed 4x(4 elements) reads
__device__ __forceinline__ int t_off_col(int m, int col) {
  const int h = (m & 3) | (((m >> 3) & 1) << 2);
  return m * 256 + ((((col >> 4) ^ h)) << 5) + ((col & 15) << 1);
}

__global__ __launch_bounds__(256) void tn_kernel(TNArgs p) {
  constexpr int TB = 64 * 256;  // one operand tile: 64 rows x 128 cols bf16
  constexpr int STAGE = 2 * TB;
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wk = wid & 1, wn = wid >> 1;  // wave tile: k rows wk*64.., n cols wn*64..
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wg / p.tiles_nk, t = wg % p.tiles_nk;
  const int n0 = (t / p.tiles_k) * 128, k0 = (t % p.tiles_k) * 128;
  int r0 = split * p.rows_per_split;
  int r1 = min(p.M, r0 + p.rows_per_split);
  if (p.boff) {  // split index = branch * splits + s over that branch's rows
    const int br = split / p.splits, sp = split % p.splits;
    const int b0 = p.boff[br], b1 = p.boff[br + 1];
    const int chunk = ((b1 - b0 + p.splits - 1) / p.splits + 63) / 64 * 64;
    r0 = b0 + sp * chunk;
    r1 = min(b1, r0 + chunk);
  }
  const int KT = (r1 - r0 + 63) / 64;
  const uint16_t* Xs;
  int ldx, kk;
  if (k0 < p.kc1) { Xs = p.X; ldx = p.ldx; kk = k0; }
  else { Xs = p.X2; ldx = p.ldx2; kk = k0 - p.kc1; }

  uint4 rg[4], rx[4];
  auto load = [&](int kt) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = tid + j * 256, row = i >> 4, c = i & 15;
      const int m = r0 + kt * 64 + row;
      const bool ok = m < r1;
      rg[j] = ok ? *reinterpret_cast<const uint4*>(p.G + (int64_t)m * p.ldg + n0 + c * 8) : make_uint4(0, 0, 0, 0);
      rx[j] = ok ? *reinterpret_cast<const uint4*>(Xs + (int64_t)m * ldx + kk + c * 8) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store = [&](int buf) {
    uint8_t* s = lds + buf * STAGE;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = tid + j * 256, row = i >> 4, c = i & 15;
      *reinterpret_cast<uint4*>(s + t_off(row, c)) = rg[j];
      *reinterpret_cast<uint4*>(s + TB + t_off(row, c)) = rx[j];
    }
  };
  f4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  if (KT > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) load(kt + 1);
    uint8_t* s = lds + cur * STAGE;
#pragma unroll
    for (int ms = 0; ms < 2; ++ms) {
      s8v xf[4], gf[4];
      const int mrow = ms * 32 + 8 * g + q;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = wk * 64 + i * 16 + 4 * pp;
        const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(s + TB + t_off_col(mrow, col)));
        const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(s + TB + t_off_col(mrow + 4, col)));
        xf[i] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wn * 64 + j * 16 + 4 * pp;
        const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(s + t_off_col(mrow, col)));
        const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(s + t_off_col(mrow + 4, col)));
        gf[j] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma(xf[i], gf[j], acc[i][j]);
    }
    if (kt + 1 < KT) store(cur ^ 1);
    __syncthreads();
  }
  // acc[i][j][r] = W[n = n0 + wn*64 + j*16 + li][k = k0 + wk*64 + i*16 + 4g + r]
  float* out = p.slab + (int64_t)split * p.Np * p.Kp;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + li, k = k0 + wk * 64 + i * 16 + 4 * g;
      *reinterpret_cast<float4*>(out + (int64_t)n * p.Kp + k) =
          make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
  if (!p.counters) return;
  // last-arriver fixup: release the slab tile (device scope: the L2 of another XCD), count
  // the arrival; the block that completes the tile reduces it
  __shared__ int last;
  const int S = p.splits, grp = p.boff ? split / p.splits : 0;
  const int cid = grp * p.tiles_nk + t;
  __threadfence();
  __syncthreads();
  if (tid == 0) last = atomicAdd(p.counters + cid, 1) == S - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
  const float* base = p.slab + (int64_t)grp * S * p.Np * p.Kp;
  const int64_t stride = (int64_t)p.Np * p.Kp;
  for (int idx = tid; idx < 128 * 32; idx += 256) {
    const int n = n0 + (idx >> 5), k = k0 + (idx & 31) * 4;
    const float* sp = base + (int64_t)n * p.Kp + k;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s2 = 0; s2 < S; ++s2) {
      const float4 v = *reinterpret_cast<const float4*>(sp + s2 * stride);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    const float av[4] = {a.x, a.y, a.z, a.w};
    for (int d = 0; d < p.nout; ++d) {
      const TNOut& o = p.outs[d];
      if (n < o.n0 || n >= o.n0 + o.N) continue;
      const int64_t row = n - o.n0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kk = k + r;
        if (kk >= o.k0 && kk < o.k0 + o.K) {
          float* q = o.out + grp * o.gout + row * o.ldo + (int64_t)(kk - o.k0) * o.ldk;
          *q = av[r] + (p.beta != 0.f ? p.beta * *q : 0.f);
        }
        if (kk == o.bias_col && o.bias_out) {
          float* q = o.bias_out + grp * o.gbias + row;
          *q = av[r] + (p.beta != 0.f ? p.beta * *q : 0.f);
        }
      }
    }
  }
  if (tid == 0) p.counters[cid] = 0;  // ready for the next product on this stream
}

// out[n][k] (n < N, k < K) = beta * out + sum_s slab[s][n0 + n][k];  bias_out[n] likewise
// from slab column bias_col.
// blockIdx.y = group (the per-branch problems of a grouped weight gradient): slab, out and
// bias_out advance by gslab / gout / gbias elements per group
__global__ void slab_reduce_kernel(const float* __restrict__ slab, int S, int Np, int Kp, int n0, int k0, int N, int K,
                                   float* __restrict__ out, int ldo, int ldk, float beta, int bias_col,
                                   float* __restrict__ bias_out, int64_t gslab, int64_t gout, int64_t gbias) {
  slab += blockIdx.y * gslab;
  out += blockIdx.y * gout;
  if (bias_out) bias_out += blockIdx.y * gbias;
  // threads [0, N * KQ): 4 consecutive columns each (16-byte slab loads, 4 slabs in flight);
  // threads [N * KQ, N * KQ + N): the bias column
  const int KQ = (K + 3) / 4;
  const int64_t total = (int64_t)N * KQ + (bias_out && bias_col >= 0 ? N : 0);
  const int64_t stride = (int64_t)Np * Kp;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    if (e >= (int64_t)N * KQ) {
      const int n = (int)(e - (int64_t)N * KQ);
      const float* sp = slab + (int64_t)(n0 + n) * Kp + bias_col;
      float v = 0.f;
      for (int i = 0; i < S; ++i) v += sp[i * stride];
      bias_out[n] = v + (beta != 0.f ? beta * bias_out[n] : 0.f);
      continue;
    }
    const int n = (int)(e / KQ), k = (int)(e % KQ) * 4;
    const float* sp = slab + (int64_t)(n0 + n) * Kp + k0 + k;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int i = 0;
    for (; i + 3 < S; i += 4) {
      const float4 a0 = *reinterpret_cast<const float4*>(sp + i * stride);
      const float4 a1 = *reinterpret_cast<const float4*>(sp + (i + 1) * stride);
      const float4 a2 = *reinterpret_cast<const float4*>(sp + (i + 2) * stride);
      const float4 a3 = *reinterpret_cast<const float4*>(sp + (i + 3) * stride);
      acc = f4add(acc, f4add(f4add(a0, a1), f4add(a2, a3)));
    }
    for (; i < S; ++i) acc = f4add(acc, *reinterpret_cast<const float4*>(sp + i * stride));
    const float v[4] = {acc.x, acc.y, acc.z, acc.w};
    float* o = out + (int64_t)n * ldo + (int64_t)k * ldk;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (k + r < K) o[r * ldk] = v[r] + (beta != 0.f ? beta * o[r * ldk] : 0.f);
  }
}

// ------------------------------------------------------------------------------ casts
// x fp32 [M, K] (row stride ldx) -> bf16 [M, Kp]; optional relu' gate from bf16 [M, ldgate]
// (value zeroed where gate <= 0); ones lane at column ones_col.
__global__ void cast_pad_kernel(const float* __restrict__ x, int64_t M, int K, int ldx, uint16_t* __restrict__ out,
                                int Kp, const uint16_t* __restrict__ gate, int ldgate, int ones_col) {
  const int kq = Kp / 4;
  const int64_t total = M * kq;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = e / kq;
    const int k = (int)(e % kq) * 4;
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int kk = k + r;
      v[r] = kk < K ? x[m * ldx + kk] : (kk == ones_col ? 1.f : 0.f);
    }
    if (gate) {
      const uint2 gg = *reinterpret_cast<const uint2*>(gate + m * ldgate + k);
      if (!(lo_bf(gg.x) > 0.f) && k < K) v[0] = 0.f;
      if (!(hi_bf(gg.x) > 0.f) && k + 1 < K) v[1] = 0.f;
      if (!(lo_bf(gg.y) > 0.f) && k + 2 < K) v[2] = 0.f;
      if (!(hi_bf(gg.y) > 0.f) && k + 3 < K) v[3] = 0.f;
    }
    *reinterpret_cast<uint2*>(out + m * Kp + k) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
  }
}

struct WJob {
  const float* src;  // [N rows][K cols] with row stride ld (column offset already applied)
  uint16_t* dst;     // [Np][Kp] (null: skip)
  uint16_t* dstT;    // [Kp][Np] (null: skip)
  int ld, ldd, lddt, N, K, Np, Kp, tiles_k, tile0;
};
constexpr int MAX_WJOBS = 48;
struct WJobs {
  WJob j[MAX_WJOBS];
  int n;
};

// 64x64 tiles of every job; LDS transpose for the W^T image
__global__ __launch_bounds__(256) void cast_weights_kernel(WJobs jobs) {
  __shared__ float tile[64][65];
  int b = blockIdx.x, ji = 0;
  while (ji + 1 < jobs.n && jobs.j[ji + 1].tile0 <= b) ++ji;
  const WJob J = jobs.j[ji];
  const int t = b - J.tile0;
  const int r0 = (t / J.tiles_k) * 64, c0 = (t % J.tiles_k) * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int n = r0 + r, k = c0 + tx;
    const float v = (n < J.N && k < J.K) ? J.src[(int64_t)n * J.ld + k] : 0.f;
    tile[r][tx] = v;
    if (J.dst) {
      __bf16 h = (__bf16)v;
      J.dst[(int64_t)n * J.ldd + k] = __builtin_bit_cast(uint16_t, h);
    }
  }
  if (!J.dstT) return;
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int k = c0 + r, n = r0 + tx;
    __bf16 h = (__bf16)tile[tx][r];
    J.dstT[(int64_t)k * J.lddt + n] = __builtin_bit_cast(uint16_t, h);
  }
}

}  // namespace bg

using namespace bg;

static const uint16_t* bfp(const at::Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
static uint16_t* bfpw(const at::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

static void check_bf(const at::Tensor& t, const char* name) {
  HY_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 2 && t.stride(1) == 1, name,
           " must be a row-contiguous 2-d bf16 GPU tensor");
  HY_CHECK(t.stride(0) % 8 == 0, name, " row stride must be a multiple of 8 elements");
  HY_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

// C = epi(A B^T).  A [M, >= K] bf16 (or [A | A2] K-concatenated at k-tile kt1), B [Np, >= K] bf16.
void bg_nt(const at::Tensor& A, const c10::optional<at::Tensor>& A2, int64_t k1, const at::Tensor& B, int64_t K,
           int64_t N, const c10::optional<at::Tensor>& bias, int64_t act, const c10::optional<at::Tensor>& gate,
           const c10::optional<at::Tensor>& addg, const c10::optional<at::Tensor>& addg_idx,
           const c10::optional<at::Tensor>& outf, double beta, const c10::optional<at::Tensor>& outb,
           int64_t ones_col, const c10::optional<at::Tensor>& rowvec, const c10::optional<at::Tensor>& rowdot,
           int64_t bm_, const c10::optional<at::Tensor>& bid, int64_t bsB, int64_t bsbias) {
  // bm_ = tile rows (64 / 128 / 256) + 1000 for the glds-staged variant
  const bool glds = bm_ >= 1000;
  const int64_t bm = bm_ % 1000;
  check_bf(A, "A");
  check_bf(B, "B");
  const int64_t M = A.size(0), Np = B.size(0);
  HY_CHECK(K % 64 == 0 && Np % 128 == 0 && N <= Np, "bg_nt: K % 64, Np % 128, N <= Np required");
  HY_CHECK(k1 % 64 == 0 && k1 <= K, "bg_nt: bad k1");
  HY_CHECK(B.size(1) >= K, "bg_nt: B narrower than K");
  NTArgs p{};
  p.A = bfp(A);
  p.lda = (int)A.stride(0);
  p.kt1 = (int)(k1 / 64);
  if (A2.has_value()) {
    check_bf(*A2, "A2");
    HY_CHECK(A2->size(0) == M && A2->size(1) >= K - k1, "bg_nt: A2 shape");
    p.A2 = bfp(*A2);
    p.lda2 = (int)A2->stride(0);
  } else {
    HY_CHECK(k1 == K && A.size(1) >= K, "bg_nt: A narrower than K");
  }
  p.B = bfp(B);
  p.ldb = (int)B.stride(0);
  p.M = (int)M;
  p.N = (int)N;
  p.Np = (int)Np;
  p.K = (int)K;
  if (bias.has_value()) {
    HY_CHECK(bias->scalar_type() == at::kFloat && bias->numel() >= N && bias->is_contiguous(), "bg_nt: bias");
    p.bias = bias->data_ptr<float>();
  }
  p.act = (int)act;
  if (gate.has_value()) {
    check_bf(*gate, "gate");
    HY_CHECK(gate->size(0) == M && gate->size(1) >= Np, "bg_nt: gate shape");
    p.gate = bfp(*gate);
    p.ldgate = (int)gate->stride(0);
  }
  if (addg.has_value()) {
    HY_CHECK(addg->scalar_type() == at::kFloat && addg->stride(1) == 1 && addg->size(1) >= N, "bg_nt: addg");
    p.addg = addg->data_ptr<float>();
    p.ldaddg = (int)addg->stride(0);
    if (addg_idx.has_value()) {
      HY_CHECK_I32(*addg_idx);
      HY_CHECK(addg_idx->numel() >= M, "bg_nt: addg_idx length");
      p.addg_idx = addg_idx->data_ptr<int>();
    } else {
      HY_CHECK(addg->size(0) >= M, "bg_nt: addg rows");
    }
  }
  if (outf.has_value()) {
    HY_CHECK(outf->scalar_type() == at::kFloat && outf->stride(1) == 1 && outf->size(0) == M && outf->size(1) >= N,
             "bg_nt: outf");
    p.outf = outf->data_ptr<float>();
    p.ldf = (int)outf->stride(0);
  }
  p.beta = (float)beta;
  if (outb.has_value()) {
    check_bf(*outb, "outb");
    HY_CHECK(outb->size(0) == M && outb->size(1) >= Np, "bg_nt: outb shape");
    p.outb = bfpw(*outb);
    p.ldo = (int)outb->stride(0);
  }
  p.ones_col = (int)ones_col;
  if (rowdot.has_value()) {
    HY_CHECK(rowvec.has_value() && rowvec->numel() >= N && rowdot->numel() >= M, "bg_nt: rowdot");
    p.rowvec = rowvec->data_ptr<float>();
    p.rowdot = rowdot->data_ptr<float>();
  }
  if (bid.has_value()) {
    HY_CHECK_I32(*bid);
    HY_CHECK(bid->numel() >= M, "bg_nt: grouped mode needs bid [M]");
    p.bid = bid->data_ptr<int>();
    p.bsB = bsB;
    p.bsbias = (int)bsbias;
  }
  if (M == 0) return;
  p.tiles_n = (int)(Np / 128);
  if (glds) {
    if (p.bid) {
      HY_CHECK(bm == 64, "bg_nt: grouped glds mode uses the 64-row tile");
      ntg_kernel<64, 4, true><<<ceil_div(M, 64) * p.tiles_n, 256, 0, stream()>>>(p);
    } else if (bm == 256) {
      ntg_kernel<256, 2, false><<<ceil_div(M, 256) * p.tiles_n, 512, 0, stream()>>>(p);
    } else if (bm == 128) {
      ntg_kernel<128, 2, false><<<ceil_div(M, 128) * p.tiles_n, 256, 0, stream()>>>(p);
    } else {
      ntg_kernel<64, 4, false><<<ceil_div(M, 64) * p.tiles_n, 256, 0, stream()>>>(p);
    }
    return;
  }
  if (bm == 256) {
    nt_kernel<256, 2><<<ceil_div(M, 256) * p.tiles_n, 512, 0, stream()>>>(p);
  } else if (bm == 128) {
    nt_kernel<128, 2><<<ceil_div(M, 128) * p.tiles_n, 256, 0, stream()>>>(p);
  } else {
    HY_CHECK(bm == 64, "bg_nt: bm in {64, 128, 256}");
    nt_kernel<64, 4><<<ceil_div(M, 64) * p.tiles_n, 256, 0, stream()>>>(p);
  }
}

// slab[S][Np][Kp] = split-M partial sums of G^T [X | X2]
void bg_tn(const at::Tensor& G, const at::Tensor& X, const c10::optional<at::Tensor>& X2, int64_t kc1,
           int64_t Np, int64_t Kp, const at::Tensor& slab, int64_t splits, const c10::optional<at::Tensor>& boff,
           at::TensorList outs, const c10::List<c10::optional<at::Tensor>>& bias_outs, at::IntArrayRef meta,
           double beta, const c10::optional<at::Tensor>& counters) {
  check_bf(G, "G");
  check_bf(X, "X");
  const int64_t M = G.size(0);
  HY_CHECK(Np % 128 == 0 && Kp % 128 == 0 && kc1 % 128 == 0, "bg_tn: Np, Kp, kc1 must be multiples of 128");
  HY_CHECK(G.size(1) >= Np && X.size(0) == M, "bg_tn: shapes");
  TNArgs p{};
  p.G = bfp(G);
  p.ldg = (int)G.stride(0);
  p.X = bfp(X);
  p.ldx = (int)X.stride(0);
  p.kc1 = (int)kc1;
  if (X2.has_value()) {
    check_bf(*X2, "X2");
    HY_CHECK(X2->size(0) == M && X2->size(1) >= Kp - kc1 && X.size(1) >= kc1, "bg_tn: X2 shape");
    p.X2 = bfp(*X2);
    p.ldx2 = (int)X2->stride(0);
  } else {
    HY_CHECK(kc1 == Kp && X.size(1) >= Kp, "bg_tn: X narrower than Kp");
  }
  int64_t groups = 1;
  if (boff.has_value()) {
    HY_CHECK_I32(*boff);
    groups = boff->numel() - 1;
    p.boff = boff->data_ptr<int>();
  }
  p.splits = (int)splits;
  HY_CHECK(slab.scalar_type() == at::kFloat && slab.is_contiguous() && slab.numel() >= groups * splits * Np * Kp,
           "bg_tn: slab");
  p.M = (int)M;
  p.Np = (int)Np;
  p.Kp = (int)Kp;
  p.rows_per_split = (int)(((M + splits - 1) / splits + 63) / 64 * 64);
  p.tiles_k = (int)(Kp / 128);
  p.tiles_nk = (int)((Np / 128) * p.tiles_k);
  p.slab = slab.data_ptr<float>();
  // fused reduce destinations: meta = (n0, k0, N, K, bias_col) per output (per group when
  // grouped: the output view is [groups * N, K], the bias [groups * N])
  HY_CHECK(outs.size() <= 3 && (int64_t)bias_outs.size() == (int64_t)outs.size() &&
               (int64_t)meta.size() == 5 * (int64_t)outs.size(),
           "bg_tn: at most 3 outputs with (n0, k0, N, K, bias_col) each");
  if (!outs.empty()) {
    HY_CHECK(counters.has_value() && counters->scalar_type() == at::kInt && counters->is_cuda() &&
                 counters->numel() >= groups * p.tiles_nk,
             "bg_tn: fused reduce needs an int32 counter buffer (zeroed) of groups * tiles");
    p.counters = counters->data_ptr<int>();
    p.nout = (int)outs.size();
    p.beta = (float)beta;
    for (size_t d = 0; d < outs.size(); ++d) {
      const at::Tensor& o = outs[d];
      TNOut& t = p.outs[d];
      HY_CHECK(o.scalar_type() == at::kFloat && o.dim() == 2 && o.is_cuda(), "bg_tn: outputs fp32 2-D");
      t.out = o.data_ptr<float>();
      t.ldo = (int)o.stride(0);
      t.ldk = (int)o.stride(1);
      t.n0 = (int)meta[5 * d];
      t.k0 = (int)meta[5 * d + 1];
      t.N = (int)meta[5 * d + 2];
      t.K = (int)meta[5 * d + 3];
      t.bias_col = (int)meta[5 * d + 4];
      HY_CHECK(o.size(0) >= groups * t.N && o.size(1) >= t.K, "bg_tn: output view smaller than (groups * N, K)");
      HY_CHECK(t.n0 >= 0 && t.k0 >= 0 && t.n0 + t.N <= Np && t.k0 + t.K <= Kp && t.bias_col < Kp,
               "bg_tn: output rectangle outside the product");
      t.gout = groups > 1 ? (int64_t)t.N * t.ldo : 0;
      HY_CHECK(groups == 1 || o.is_contiguous(), "bg_tn: grouped outputs are contiguous [groups * N, K]");
      const c10::optional<at::Tensor> bo = bias_outs.get(d);
      if (bo.has_value()) {
        HY_CHECK(bo->scalar_type() == at::kFloat && bo->is_contiguous() && bo->numel() >= groups * t.N,
                 "bg_tn: bias_out");
        t.bias_out = bo->data_ptr<float>();
        t.gbias = groups > 1 ? t.N : 0;
      }
    }
  }
  const int grid = (int)(p.tiles_nk * splits * groups);
  tn_kernel<<<grid, 256, 0, stream()>>>(p);
}

void bg_slab_reduce(const at::Tensor& slab, int64_t S, int64_t Np, int64_t Kp, int64_t n0, int64_t k0, int64_t N, int64_t K,
                    const at::Tensor& out, double beta, int64_t bias_col, const c10::optional<at::Tensor>& bias_out,
                    int64_t groups) {
  HY_CHECK(out.scalar_type() == at::kFloat && out.dim() == 2 && out.size(0) >= N && out.size(1) >= K,
           "bg_slab_reduce: out");
  HY_CHECK(n0 + N <= Np && k0 + K <= Kp && bias_col < Kp && Kp % 4 == 0 && k0 % 4 == 0, "bg_slab_reduce: bounds");
  float* bo = nullptr;
  if (bias_out.has_value()) {
    HY_CHECK(bias_out->scalar_type() == at::kFloat && bias_out->is_contiguous() && bias_out->numel() >= N,
             "bg_slab_reduce: bias_out");
    bo = bias_out->data_ptr<float>();
  }
  // groups > 1: out is [groups, N, K] (contiguous per group), bias_out [groups, N]
  HY_CHECK(groups >= 1 && (groups == 1 || (out.numel() >= groups * N * K && slab.numel() >= groups * S * Np * Kp)),
           "bg_slab_reduce: groups");
  const int64_t total = N * ((K + 3) / 4) + N;
  const int blocks = (int)std::min<int64_t>(4096, (total + 255) / 256);
  slab_reduce_kernel<<<dim3(blocks, (unsigned)groups), 256, 0, stream()>>>(
      slab.data_ptr<float>(), (int)S, (int)Np, (int)Kp, (int)n0, (int)k0, (int)N, (int)K, out.data_ptr<float>(),
      (int)out.stride(0), (int)out.stride(1), (float)beta, (int)bias_col, bo, S * Np * Kp, N * K, N);
}

void bg_cast_pad(const at::Tensor& x, const at::Tensor& out, const c10::optional<at::Tensor>& gate, int64_t ones_col) {
  HY_CHECK(x.scalar_type() == at::kFloat && x.dim() == 2 && x.stride(1) == 1, "bg_cast_pad: x");
  check_bf(out, "out");
  const int64_t M = x.size(0), K = x.size(1), Kp = out.size(1);
  HY_CHECK(out.size(0) == M && Kp >= K && Kp % 4 == 0 && out.is_contiguous(), "bg_cast_pad: out shape");
  const uint16_t* g = nullptr;
  int ldg = 0;
  if (gate.has_value()) {
    check_bf(*gate, "gate");
    HY_CHECK(gate->size(0) == M && gate->size(1) >= Kp, "bg_cast_pad: gate");
    g = bfp(*gate);
    ldg = (int)gate->stride(0);
  }
  if (M == 0) return;
  const int64_t total = M * (Kp / 4);
  const int blocks = (int)std::min<int64_t>(8192, (total + 255) / 256);
  cast_pad_kernel<<<blocks, 256, 0, stream()>>>(x.data_ptr<float>(), M, (int)K, (int)x.stride(0), bfpw(out),
                                                (int)Kp, g, ldg, (int)ones_col);
}

// Batched weight casts: srcs[i] fp32 [N, K] (row-contiguous, any row stride), dst[i] bf16
// [Np, Kp] and/or dstT[i] bf16 [Kp, Np] (empty tensor: skip).
void bg_cast_weights(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts,
                     const std::vector<at::Tensor>& dstTs) {
  HY_CHECK(srcs.size() == dsts.size() && srcs.size() == dstTs.size(), "bg_cast_weights: list lengths");
  size_t i = 0;
  while (i < srcs.size()) {
    WJobs jobs{};
    int tiles = 0;
    for (; i < srcs.size() && jobs.n < MAX_WJOBS; ++i) {
      const at::Tensor& s = srcs[i];
      HY_CHECK(s.scalar_type() == at::kFloat && s.dim() == 2 && s.stride(1) == 1, "bg_cast_weights: src");
      WJob J{};
      J.src = s.data_ptr<float>();
      J.ld = (int)s.stride(0);
      J.N = (int)s.size(0);
      J.K = (int)s.size(1);
      const at::Tensor& d = dsts[i];
      const at::Tensor& dt = dstTs[i];
      if (d.numel()) {
        HY_CHECK(d.scalar_type() == at::kBFloat16 && d.dim() == 2 && d.stride(1) == 1 && d.size(0) >= J.N &&
                     d.size(1) >= J.K,
                 "bg_cast_weights: dst");
        J.dst = bfpw(d);
        J.ldd = (int)d.stride(0);
        J.Np = (int)d.size(0);
        J.Kp = (int)d.size(1);
      }
      if (dt.numel()) {
        HY_CHECK(dt.scalar_type() == at::kBFloat16 && dt.dim() == 2 && dt.stride(1) == 1 && dt.size(1) >= J.N &&
                     dt.size(0) >= J.K,
                 "bg_cast_weights: dstT");
        J.dstT = bfpw(dt);
        J.lddt = (int)dt.stride(0);
        if (d.numel()) HY_CHECK(dt.size(0) == J.Kp && dt.size(1) == J.Np, "bg_cast_weights: dst/dstT shapes differ");
        J.Np = (int)dt.size(1);
        J.Kp = (int)dt.size(0);
      }
      HY_CHECK(J.Np % 64 == 0 && J.Kp % 64 == 0, "bg_cast_weights: padded dims must be multiples of 64");
      J.tiles_k = J.Kp / 64;
      J.tile0 = tiles;
      tiles += (J.Np / 64) * J.tiles_k;
      jobs.j[jobs.n++] = J;
    }
    if (tiles) cast_weights_kernel<<<tiles, 256, 0, stream()>>>(jobs);
  }
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def(
      "bg_nt(Tensor A, Tensor? A2, int k1, Tensor B, int K, int N, Tensor? bias, int act, Tensor? gate, Tensor? addg, "
      "Tensor? addg_idx, Tensor? outf, float beta, Tensor? outb, int ones_col, Tensor? rowvec, Tensor? rowdot, "
      "int bm, Tensor? bid=None, int bsB=0, int bsbias=0) -> ()");
  m.def(
      "bg_tn(Tensor G, Tensor X, Tensor? X2, int kc1, int Np, int Kp, Tensor slab, int splits, Tensor? boff, "
      "Tensor[] outs, Tensor?[] bias_outs, int[] meta, float beta, Tensor? counters) -> ()");
  m.def(
      "bg_slab_reduce(Tensor slab, int S, int Np, int Kp, int n0, int k0, int N, int K, Tensor out, float beta, int bias_col, "
      "Tensor? bias_out, int groups=1) -> ()");
  m.def("bg_cast_pad(Tensor x, Tensor out, Tensor? gate, int ones_col) -> ()");
  m.def("bg_cast_weights(Tensor[] srcs, Tensor[] dsts, Tensor[] dstTs) -> ()");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("bg_nt", hy::bg_nt);
  m.impl("bg_tn", hy::bg_tn);
  m.impl("bg_slab_reduce", hy::bg_slab_reduce);
  m.impl("bg_cast_pad", hy::bg_cast_pad);
  m.impl("bg_cast_weights", hy::bg_cast_weights);
}
