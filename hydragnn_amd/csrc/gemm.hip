// MFMA GEMM engine for the dense maps of every GNN stack.
//
// One launch runs a small *batch of GEMM problems* ("grouped GEMM"), each
//     C[M,N] = epilogue( sum_seg  A_seg[M,K_seg] . B_seg[K_seg,N] )
// with per-operand strides, so the same kernel serves
//   * the forward of a linear layer over a column-split input (concat-linear
//     decomposition: Y = act(sum_p X_p W_p^T + b) (+ residual), no concat
//     ever materialised),
//   * its whole backward in ONE launch: dX_p = dZ W_p for every input block and
//     dW_p = dZ^T X_p (+ db via an implicit ones-column of X) for every weight,
//     with dZ = dY * relu'(Y) applied while staging A.
// Weight gradients reduce over the (long) row dimension, so those problems are
// split along K and the K-slices are combined INSIDE the launch: every slice
// writes its 4 KB fp32 slab, takes an agent-scope ticket, and the last arriver sums
// the slabs in slice order (deterministic, no float atomics) and runs the
// epilogue (guide §5 "in-launch split-K reduction": release fence before the
// ticket, acquire fence after it; the counter is reset by the reducer).
//
// CDNA4 mapping: the GNN GEMMs are small (N, K = 8..1088) over 10^3-10^5 rows, so
// the design maximises parallelism instead of per-tile reuse: a 256-thread
// workgroup (4 wave64s) owns one 32x32 output tile (2x2 MFMA 16x16 tiles per
// wave) and its 4 waves split the tile's k-chunks; fragments load straight from
// global/L2 into VGPRs (no LDS staging: a k-contiguous operand is 1-2 16-byte
// loads per lane per chunk because A and B only need to AGREE on the k order
// inside a chunk), the next chunk in flight while the current one runs on the
// matrix cores; the wave partials are folded through LDS in a fixed order.
//   PREC_F32 : v_mfma_f32_16x16x4_f32 — exact fp32 (the reference's numerics).
//   PREC_BF16: v_mfma_f32_16x16x32_bf16 — operands rounded to bf16 in registers,
//              fp32 accumulate, fp32 storage (16x the fp32 MFMA rate).
#include "common.h"

namespace hy {

typedef float f4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));

constexpr int kMMTile = 32;     // output tile edge per workgroup
constexpr int kMMWaves = 4;     // waves per workgroup; they split the tile's k-chunks
constexpr int kMMMaxSeg = 3;
constexpr int kMMMaxProb = 6;

template <bool BF16>
struct MMCfg {
  static constexpr int KCL = BF16 ? 8 : 4;  // k values per lane per row tile per chunk
  static constexpr int KC = 4 * KCL;        // chunk depth (4 lane groups)
};

struct MMSeg {
  const float* A;      // A(m,k) = A[m*sam + k*sak]
  const float* Amask;  // optional: A(m,k) *= (Amask(m,k) > 0)   (relu' of the forward output)
  const float* B;      // B(k,n) = B[k*sbk + n*sbn]
  int64_t sam, sak, sbk, sbn;
  int K;
  int a_kc, b_kc;      // operand contiguous along k (else along m / n)
  int a_vec, b_vec;    // 16-byte loads allowed along k (kc operands only)
  int kc0;             // first k-chunk index of this segment in the problem's chunk list
};

struct MMProb {
  MMSeg seg[kMMMaxSeg];
  int nseg, M, N, kchunks;
  float* C;
  int64_t ldc;
  const float* bias;      // [N]
  const float* residual;  // [M, ldr], added after the activation
  int64_t ldr;
  int act;                // 0 none, 1 relu
  int ones_col;           // B(k, ones_col) == 1 (bias gradient column), -1 off
  float* ones_out;        // destination of column ones_col ([M])
  int split;              // K slices over workgroups (in-launch reduction when > 1)
  float* ws;              // [tiles*split][32*32] partial slabs
  int* cnt;               // [tiles] tickets
  int tiles_n, tile0;     // output tiles along N; first workgroup of this problem
  int code;               // operand-mode instantiation (see mm_kernel)
};

struct MMArgs {
  MMProb p[kMMMaxProb];
  int nprob;
};

// problems are read in place from the kernel-argument segment (address space 4)
typedef __attribute__((address_space(4))) const MMProb KProb;

__device__ __forceinline__ float relu_mask(float v, float m) { return m > 0.f ? v : 0.f; }

// Operand access modes (per problem, chosen on the host; the K loop is instantiated per
// mode so it is branch-free and the compiler can count outstanding loads exactly):
//   KCV: contiguous along k, 16-byte aligned rows -> KCL/4 dwordx4 loads per row tile
//   KCS: contiguous along k, unaligned -> KCL scalar loads per row tile
//   RC : contiguous along the row (m or n) dimension -> KCL scalar loads, coalesced over lanes
enum { OP_KCV = 0, OP_KCS = 1, OP_RC = 2 };

// Register fragments of one operand for a 32-row (2 x 16) slice of a chunk: lane l holds
// rows r = l&15 (+16 i) and the KCL k-values  k0 + KCL*(l>>4) + s.  (Any k order works as
// long as A and B agree, so a k-contiguous operand is one or two 16-byte loads per row.)
// Branch-free: clamped addresses + selects; ``valid`` == false (a chunk past the end of
// this wave's range) yields zeros.  ``rows`` rows are backed by memory; the wgrad B operand
// carries a ones column at ``ones_col`` (bias gradient).
template <int KCL, int MODE, bool MASK, bool ONES>
__device__ __forceinline__ void load_frag(const float* __restrict__ P, const float* __restrict__ Pm, int64_t srow,
                                          int64_t sk, int rows, int K, int row0, int k0, bool valid, int ones_col,
                                          float (&v)[2][KCL]) {
  const int lane = threadIdx.x & 63;
  const int kb = k0 + KCL * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = row0 + 16 * i + (lane & 15);
    const bool rv = valid && r < rows;
    const int rc = min(r, rows - 1);
    if constexpr (MODE == OP_KCV) {
      const float* base = P + (int64_t)rc * srow + min(kb, K - KCL);
#pragma unroll
      for (int q = 0; q < KCL / 4; ++q) {
        const float4 a = *reinterpret_cast<const float4*>(base + 4 * q);
        v[i][4 * q] = a.x; v[i][4 * q + 1] = a.y; v[i][4 * q + 2] = a.z; v[i][4 * q + 3] = a.w;
      }
      if constexpr (MASK) {
        const float* mb = Pm + (int64_t)rc * srow + min(kb, K - KCL);
#pragma unroll
        for (int q = 0; q < KCL / 4; ++q) {
          const float4 m = *reinterpret_cast<const float4*>(mb + 4 * q);
          v[i][4 * q] = relu_mask(v[i][4 * q], m.x); v[i][4 * q + 1] = relu_mask(v[i][4 * q + 1], m.y);
          v[i][4 * q + 2] = relu_mask(v[i][4 * q + 2], m.z); v[i][4 * q + 3] = relu_mask(v[i][4 * q + 3], m.w);
        }
      }
#pragma unroll
      for (int s = 0; s < KCL; ++s) v[i][s] = (rv && kb + s < K) ? v[i][s] : 0.f;
    } else {
#pragma unroll
      for (int s = 0; s < KCL; ++s) {
        const int k = kb + s;
        const int64_t off = MODE == OP_KCS ? (int64_t)rc * srow + min(k, K - 1)
                                           : (int64_t)min(k, K - 1) * sk + (int64_t)rc * srow;
        float x = P[off];
        if constexpr (MASK) x = relu_mask(x, Pm[off]);
        v[i][s] = (rv && k < K) ? x : 0.f;
      }
    }
    if constexpr (ONES) {
#pragma unroll
      for (int s = 0; s < KCL; ++s) v[i][s] = (valid && r == ones_col) ? ((kb + s) < K ? 1.f : 0.f) : v[i][s];
    }
  }
}

template <bool BF16>
__device__ __forceinline__ void mma_chunk(const float (&a)[2][MMCfg<BF16>::KCL], const float (&b)[2][MMCfg<BF16>::KCL],
                                          f4v (&acc)[2][2]) {
  if constexpr (BF16) {
    bf8v ap[2], bp[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        ap[i][s] = (__bf16)a[i][s];
        bp[i][s] = (__bf16)b[i][s];
      }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ap[i], bp[j], acc[i][j], 0, 0, 0);
  } else {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
  }
}

// The wave's chunks c = c0, c0+4, ... (< c_end) in groups of four: all four chunks' loads are
// issued first (straight-line code, so the compiler counts them and waits only for the set
// the next MFMA group needs), then the four MFMA groups run.  Chunks past c_end load as
// zeros (clamped addresses), keeping every load unconditional.
template <bool BF16, int AM, int BM, bool MASK, bool ONES>
__device__ __forceinline__ void tile_loop(KProb& P, int m0, int n0, int c0, int c_end, f4v (&acc)[2][2]) {
  constexpr int KCL = MMCfg<BF16>::KCL;
  constexpr int KC = MMCfg<BF16>::KC;
  if (c0 >= c_end) return;
  const int kc1 = P.nseg > 1 ? P.seg[1].kc0 : 1 << 30;
  const int kc2 = P.nseg > 2 ? P.seg[2].kc0 : 1 << 30;
  const int brows = ONES ? P.ones_col : P.N;
  // segment fields picked with static indices (a dynamic index into the kernel-argument
  // struct makes the compiler copy the whole struct to scratch)
#define HY_SEG(f) (s == 0 ? P.seg[0].f : (s == 1 ? P.seg[1].f : P.seg[2].f))
  auto fetch = [&](int c, float (&a)[2][KCL], float (&b)[2][KCL]) {
    const bool valid = c < c_end;
    const int cc = __builtin_amdgcn_readfirstlane(min(c, c_end - 1));
    const int s = (cc >= kc1) + (cc >= kc2);
    const int k0 = (cc - HY_SEG(kc0)) * KC;
    const int K = HY_SEG(K);
    load_frag<KCL, AM, MASK, false>(HY_SEG(A), HY_SEG(Amask), HY_SEG(sam), HY_SEG(sak), P.M, K, m0, k0, valid, -1, a);
    load_frag<KCL, BM, false, ONES>(HY_SEG(B), nullptr, HY_SEG(sbn), HY_SEG(sbk), brows, K, n0, k0, valid,
                                    P.ones_col, b);
  };
#undef HY_SEG
  float a0[2][KCL], b0[2][KCL], a1[2][KCL], b1[2][KCL], a2[2][KCL], b2[2][KCL], a3[2][KCL], b3[2][KCL];
#pragma unroll 1
  for (int c = c0; c < c_end; c += 4 * kMMWaves) {
    fetch(c, a0, b0);
    fetch(c + kMMWaves, a1, b1);
    fetch(c + 2 * kMMWaves, a2, b2);
    fetch(c + 3 * kMMWaves, a3, b3);
    mma_chunk<BF16>(a0, b0, acc);
    mma_chunk<BF16>(a1, b1, acc);
    mma_chunk<BF16>(a2, b2, acc);
    mma_chunk<BF16>(a3, b3, acc);
  }
}

__device__ __forceinline__ void epilogue_store(KProb& P, int r, int c, float v) {
  if (r >= P.M || c >= P.N) return;
  if (c == P.ones_col) {
    P.ones_out[r] = v;
    return;
  }
  if (P.bias) v += P.bias[c];
  if (P.act == 1) v = fmaxf(v, 0.f);
  if (P.residual) v += P.residual[(int64_t)r * P.ldr + c];
  P.C[(int64_t)r * P.ldc + c] = v;
}

__device__ __forceinline__ void epilogue4(KProb& P, int r, int c, float4 v) {
  epilogue_store(P, r, c, v.x);
  epilogue_store(P, r, c + 1, v.y);
  epilogue_store(P, r, c + 2, v.z);
  epilogue_store(P, r, c + 3, v.w);
}

// Publish this workgroup's slab and draw a ticket on ``counter``; true in the last arriver,
// which may then read every slab of the group (agent-scope release before the ticket,
// acquire after it — guide §5 in-launch split-K reduction).
__device__ __forceinline__ bool arrive(int* counter, int expected, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int tk = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = (tk == expected - 1);
  }
  __syncthreads();
  if (!*flag) return false;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *counter = 0;  // reset for the next launch (every ticket of this launch is drawn)
  }
  __syncthreads();
  return true;
}

__device__ __forceinline__ float4 sum_slabs(const float* slabs, int n) {
  float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f);
  int sl = 0;
#pragma unroll 1
  for (; sl + 4 <= n; sl += 4) {
    float4 u[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) u[q] = reinterpret_cast<const float4*>(slabs + (int64_t)(sl + q) * 1024)[threadIdx.x];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      s4.x += u[q].x; s4.y += u[q].y; s4.z += u[q].z; s4.w += u[q].w;
    }
  }
#pragma unroll 1
  for (; sl < n; ++sl) {
    const float4 u = reinterpret_cast<const float4*>(slabs + (int64_t)sl * 1024)[threadIdx.x];
    s4.x += u.x; s4.y += u.y; s4.z += u.z; s4.w += u.w;
  }
  return s4;
}

constexpr int kMMGroup = 8;  // slices per first-level reduction group

// Workgroup = 4 waves on one 32x32 output tile; wave w takes the k-chunks w, w+4, ... of the
// workgroup's K slice; the 4 wave partials are folded through LDS in a fixed order.  Split
// problems then reduce their slices in-launch, two-level (groups of 8 slices, then groups).
template <bool BF16>
__global__ void __launch_bounds__(256) mm_kernel(MMArgs args_) {
  __shared__ __attribute__((aligned(16))) float red[kMMWaves * kMMTile * kMMTile];
  __shared__ int last_flag;

  // Read the problem table straight from the kernel-argument segment (constant memory,
  // scalar loads): indexing the by-value parameter with a runtime problem id makes clang
  // copy the whole 2 KB struct to scratch first.
  typedef __attribute__((address_space(4))) const MMArgs KArgs;
  KArgs* A = (KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  int pi = 0;
  const int bid = blockIdx.x;
#pragma unroll 1
  for (int q = 1; q < A->nprob; ++q)
    if (bid >= A->p[q].tile0) pi = q;
  KProb& P = A->p[pi];
  const int local = bid - P.tile0;
  const int slice = local % P.split;
  const int tile = local / P.split;
  const int m0 = (tile / P.tiles_n) * kMMTile, n0 = (tile % P.tiles_n) * kMMTile;
  const int c_begin = (int)(((int64_t)P.kchunks * slice) / P.split);
  const int c_end = (int)(((int64_t)P.kchunks * (slice + 1)) / P.split);
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  f4v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f4v){0.f, 0.f, 0.f, 0.f};

  const int c0 = c_begin + w;
  switch (P.code) {
#define HY_MM_CASE(AM, BM, MASK, ONES)                                                   \
  case (AM) + 3 * (BM) + 9 * (MASK) + 18 * (ONES):                                      \
    tile_loop<BF16, AM, BM, MASK, ONES>(P, m0, n0, c0, c_end, acc);                     \
    break;
    HY_MM_CASE(OP_KCV, OP_KCV, 0, 0)
    HY_MM_CASE(OP_KCV, OP_KCS, 0, 0)
    HY_MM_CASE(OP_KCS, OP_KCV, 0, 0)
    HY_MM_CASE(OP_KCS, OP_KCS, 0, 0)
    HY_MM_CASE(OP_KCV, OP_RC, 0, 0)
    HY_MM_CASE(OP_KCS, OP_RC, 0, 0)
    HY_MM_CASE(OP_KCV, OP_RC, 1, 0)
    HY_MM_CASE(OP_KCS, OP_RC, 1, 0)
    HY_MM_CASE(OP_RC, OP_RC, 0, 0)
    HY_MM_CASE(OP_RC, OP_RC, 1, 0)
    HY_MM_CASE(OP_RC, OP_RC, 0, 1)
    HY_MM_CASE(OP_RC, OP_RC, 1, 1)
#undef HY_MM_CASE
    default:
      break;
  }

#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        red[w * 1024 + (16 * i + (lane >> 4) * 4 + e) * kMMTile + 16 * j + (lane & 15)] = acc[i][j][e];
  __syncthreads();
  const int e0 = threadIdx.x * 4;
  float4 v = reinterpret_cast<const float4*>(red)[threadIdx.x];
#pragma unroll
  for (int q = 1; q < kMMWaves; ++q) {
    const float4 u = reinterpret_cast<const float4*>(red + q * 1024)[threadIdx.x];
    v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
  }
  const int r = m0 + e0 / kMMTile, cc = n0 + e0 % kMMTile;
  if (P.split == 1) {
    epilogue4(P, r, cc, v);
    return;
  }

  // ---- split-K over workgroups: per tile [split slabs][ngroups group slabs] of 32x32 fp32
  const int ngroups = (P.split + kMMGroup - 1) / kMMGroup;
  float* tws = P.ws + (int64_t)tile * (P.split + ngroups) * 1024;
  int* tcnt = P.cnt + (int64_t)tile * (1 + ngroups);
  reinterpret_cast<float4*>(tws + (int64_t)slice * 1024)[threadIdx.x] = v;
  const int grp = slice / kMMGroup;
  const int g0 = grp * kMMGroup, gn = min(kMMGroup, P.split - g0);
  if (!arrive(tcnt + 1 + grp, gn, &last_flag)) return;
  float4 gs = sum_slabs(tws + (int64_t)g0 * 1024, gn);
  if (ngroups == 1) {
    epilogue4(P, r, cc, gs);
    return;
  }
  float* gslabs = tws + (int64_t)P.split * 1024;
  reinterpret_cast<float4*>(gslabs + (int64_t)grp * 1024)[threadIdx.x] = gs;
  if (!arrive(tcnt, ngroups, &last_flag)) return;
  epilogue4(P, r, cc, sum_slabs(gslabs, ngroups));
}

// ----------------------------------------------------------------------------- host side

// Tickets of one launch: allocated from the caching allocator on the CURRENT stream and
// zeroed in-stream (a memset node when captured), so two launches on different streams
// (e.g. the GPS attention branch's backward beside the local MPNN's) never share counters.
static at::Tensor ticket_buffer(const at::Tensor& like, int64_t need) {
  return at::zeros({need}, like.options().dtype(at::kInt));
}

struct ProbBuilder {
  MMArgs args{};
  int blocks = 0;
  int64_t tickets = 0;
  int64_t ws_floats = 0;
  std::vector<int64_t> ws_off;  // per problem (float offset), -1 if none
};

static void set_seg(MMSeg& g, const float* A, const float* Am, int64_t sam, int64_t sak, const float* B, int64_t sbk,
                    int64_t sbn, int K, bool akc, bool bkc) {
  g.A = A;
  g.Amask = Am;
  g.B = B;
  g.sam = sam; g.sak = sak; g.sbk = sbk; g.sbn = sbn;
  g.K = K;
  g.a_kc = akc;  // layouts are fixed by the problem kind (a width-1 operand has
  g.b_kc = bkc;  // unit stride along both dims, so strides alone are ambiguous)
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  // 16-byte loads: aligned base, a row stride that keeps alignment and K % 8 == 0 (so the
  // clamped last vector of a row never straddles into the next row)
  g.a_vec = g.a_kc && al(A) && (Am == nullptr || al(Am)) && sam % 4 == 0 && K % 8 == 0;
  g.b_vec = g.b_kc && al(B) && sbn % 4 == 0 && K % 8 == 0;
}

static int pick_split(int64_t tiles, int kchunks) {
  // The in-launch reduction costs agent-scope release fences, which are cheap only while few
  // workgroups run (measured, tools/bench_mm.py: +17 us on a 292-workgroup grid): split only
  // deep-K problems with a narrow grid (weight gradients), one group of chunks per wave.
  if (tiles > 48 || kchunks <= 64) return 1;
  int s = ceil_div(kchunks, 16);
  s = std::min<int>(s, (int)std::max<int64_t>(1, 192 / std::max<int64_t>(tiles, 1)));
  return std::max(1, std::min(s, 64));
}

static int op_mode(bool kc, bool vec) { return kc ? (vec ? OP_KCV : OP_KCS) : OP_RC; }

static void add_prob(ProbBuilder& pb, MMProb p, bool allow_split, int kc_depth, bool mask) {
  HY_CHECK(pb.args.nprob < kMMMaxProb, "too many GEMM problems in one launch");
  int kt = 0;
  bool avec = true, bvec = true;
  for (int s = 0; s < p.nseg; ++s) {
    p.seg[s].kc0 = kt;
    kt += ceil_div(p.seg[s].K, kc_depth);
    avec = avec && p.seg[s].a_vec;
    bvec = bvec && p.seg[s].b_vec;
    HY_CHECK(p.seg[s].a_kc == p.seg[0].a_kc && p.seg[s].b_kc == p.seg[0].b_kc, "segments must share operand layouts");
  }
  const int am = op_mode(p.seg[0].a_kc, avec), bm = op_mode(p.seg[0].b_kc, bvec);
  const bool ones = p.ones_col >= 0;
  HY_CHECK(!ones || (am == OP_RC && bm == OP_RC), "ones column only on the wgrad layout");
  HY_CHECK(!mask || bm == OP_RC, "relu mask only on backward layouts");
  HY_CHECK(am != OP_RC || bm == OP_RC, "unsupported operand layout combination");
  p.code = am + 3 * bm + 9 * (mask ? 1 : 0) + 18 * (ones ? 1 : 0);
  p.kchunks = kt;
  p.tiles_n = ceil_div(p.N, kMMTile);
  const int64_t tiles = (int64_t)ceil_div(p.M, kMMTile) * p.tiles_n;
  p.split = allow_split ? pick_split(tiles, kt) : 1;
  p.tile0 = pb.blocks;
  if (p.split > 1) {
    const int ngroups = ceil_div(p.split, kMMGroup);
    pb.ws_off.push_back(pb.ws_floats);
    pb.ws_floats += tiles * (p.split + ngroups) * kMMTile * kMMTile;
    p.cnt = reinterpret_cast<int*>(pb.tickets);  // offset, patched at launch
    pb.tickets += tiles * (1 + ngroups);
  } else {
    pb.ws_off.push_back(-1);
  }
  pb.blocks += (int)(tiles * p.split);
  pb.args.p[pb.args.nprob++] = p;
}

static void launch(ProbBuilder& pb, const at::Tensor& like, bool bf16) {
  if (pb.blocks == 0) return;
  at::Tensor ws;
  if (pb.ws_floats > 0) ws = at::empty({pb.ws_floats}, like.options().dtype(at::kFloat));
  int* tk = nullptr;
  at::Tensor tkbuf;
  if (pb.tickets > 0) {
    tkbuf = ticket_buffer(like, pb.tickets);
    tk = tkbuf.data_ptr<int>();
  }
  for (int q = 0; q < pb.args.nprob; ++q) {
    MMProb& p = pb.args.p[q];
    if (p.split > 1) {
      p.ws = ws.data_ptr<float>() + pb.ws_off[q];
      p.cnt = tk + reinterpret_cast<intptr_t>(p.cnt);
    }
  }
  if (bf16)
    mm_kernel<true><<<pb.blocks, 256, 0, stream()>>>(pb.args);
  else
    mm_kernel<false><<<pb.blocks, 256, 0, stream()>>>(pb.args);
}

static void check_2d(const at::Tensor& t, const char* name) {
  HY_CHECK(t.is_cuda() && t.dim() == 2 && t.scalar_type() == at::kFloat, name, " must be a 2-D fp32 GPU tensor");
  HY_CHECK(t.stride(1) == 1 || t.size(1) == 1, name, " must be row-contiguous");
}

// Y = act(sum_p Xs[p] Ws[p]^T + b) (+ residual)
at::Tensor mm_fwd(at::TensorList Xs, at::TensorList Ws, const c10::optional<at::Tensor>& b,
                  const c10::optional<at::Tensor>& residual, int64_t act, int64_t prec) {
  HY_CHECK(Xs.size() == Ws.size() && Xs.size() >= 1 && (int)Xs.size() <= kMMMaxSeg, "mm_fwd: 1-3 (X, W) pairs");
  const int64_t M = Xs[0].size(0), N = Ws[0].size(0);
  auto Y = at::empty({M, N}, Xs[0].options());
  if (M == 0 || N == 0) return Y;
  ProbBuilder pb;
  MMProb p{};
  p.nseg = (int)Xs.size();
  for (int s = 0; s < p.nseg; ++s) {
    check_2d(Xs[s], "X");
    check_2d(Ws[s], "W");
    HY_CHECK(Xs[s].size(0) == M && Ws[s].size(0) == N && Xs[s].size(1) == Ws[s].size(1), "mm_fwd: shape mismatch");
    HY_CHECK(Ws[s].stride(1) == 1, "W must be row-contiguous");
    const int K = (int)Xs[s].size(1);
    // A(m,k) = X[m,k];  B(k,n) = W[n,k]
    set_seg(p.seg[s], Xs[s].data_ptr<float>(), nullptr, Xs[s].stride(0), 1, Ws[s].data_ptr<float>(), 1,
            Ws[s].stride(0), std::max(K, 1), true, true);
  }
  p.M = (int)M;
  p.N = (int)N;
  p.C = Y.data_ptr<float>();
  p.ldc = N;
  if (b.has_value() && b->defined()) {
    HY_CHECK(b->is_contiguous() && b->numel() == N, "mm_fwd: bias [N]");
    p.bias = b->data_ptr<float>();
  }
  if (residual.has_value() && residual->defined()) {
    check_2d(*residual, "residual");
    HY_CHECK(residual->size(0) == M && residual->size(1) == N, "mm_fwd: residual [M,N]");
    p.residual = residual->data_ptr<float>();
    p.ldr = residual->stride(0);
  }
  p.act = (int)act;
  p.ones_col = -1;
  add_prob(pb, p, true, prec == 1 ? MMCfg<true>::KC : MMCfg<false>::KC, false);
  launch(pb, Y, prec == 1);
  return Y;
}

// One launch: dX_p = dZ W_p (need_dx[p]), dW_p = dZ^T X_p, db = colsum(dZ); dZ = dY * relu'(Y) when Y given.
std::vector<at::Tensor> mm_bwd(const at::Tensor& dY_, const c10::optional<at::Tensor>& Y, at::TensorList Xs,
                               at::TensorList Ws, at::IntArrayRef need_dx, bool need_dw, bool with_bias,
                               int64_t prec) {
  auto dY = dY_.stride(1) == 1 ? dY_ : dY_.contiguous();
  check_2d(dY, "dY");
  const int np = (int)Xs.size();
  HY_CHECK(np == (int)Ws.size() && np >= 1 && np <= 3 && (int)need_dx.size() == np, "mm_bwd: 1-3 (X, W) pairs");
  const int64_t M = dY.size(0), N = dY.size(1);
  const float* mask = nullptr;
  if (Y.has_value() && Y->defined()) {
    HY_CHECK(Y->sizes() == dY.sizes() && Y->stride(0) == dY.stride(0) && Y->stride(1) == 1,
             "mm_bwd: Y must match dY's layout");
    mask = Y->data_ptr<float>();
  }
  std::vector<at::Tensor> dxs, dws;
  at::Tensor db = with_bias ? at::empty({N}, dY.options()) : at::Tensor();
  ProbBuilder pb;
  for (int q = 0; q < np; ++q) {
    check_2d(Xs[q], "X");
    HY_CHECK(Ws[q].stride(1) == 1 || Ws[q].size(1) == 1, "W must be row-contiguous");
    const int K = (int)Xs[q].size(1);
    HY_CHECK(Xs[q].size(0) == M && Ws[q].size(0) == N && Ws[q].size(1) == K, "mm_bwd: shape mismatch");
    if (need_dx[q]) {
      auto dX = at::empty({M, K}, dY.options());
      dxs.push_back(dX);
      if (M > 0 && K > 0) {
        MMProb p{};
        p.nseg = 1;
        // A(m,k') = dZ[m,k'] (k' over N);  B(k',n) = W[k',n]
        set_seg(p.seg[0], dY.data_ptr<float>(), mask, dY.stride(0), 1, Ws[q].data_ptr<float>(), Ws[q].stride(0), 1,
                (int)N, true, false);
        p.M = (int)M; p.N = K; p.C = dX.data_ptr<float>(); p.ldc = K; p.ones_col = -1;
        add_prob(pb, p, true, prec == 1 ? MMCfg<true>::KC : MMCfg<false>::KC, mask != nullptr);
      }
    } else {
      dxs.push_back(at::Tensor());
    }
  }
  for (int q = 0; q < np; ++q) {
    const int K = (int)Xs[q].size(1);
    const bool bias_here = with_bias && q == 0;
    if (!need_dw && !bias_here) {
      dws.push_back(at::Tensor());
      continue;
    }
    auto dW = at::empty({N, K}, dY.options());
    dws.push_back(dW);
    if (M == 0) {
      dW.zero_();
      if (bias_here) db.zero_();
      continue;
    }
    MMProb p{};
    p.nseg = 1;
    // rows i over N, cols j over K (+1 ones column for db), reduction over the M data rows:
    // A(i,r) = dZ[r,i] (contiguous along i);  B(r,j) = X[r,j] (contiguous along j)
    set_seg(p.seg[0], dY.data_ptr<float>(), mask, 1, dY.stride(0), Xs[q].data_ptr<float>(), Xs[q].stride(0), 1,
            (int)M, false, false);
    p.M = (int)N;
    p.N = K + (bias_here ? 1 : 0);
    p.C = dW.data_ptr<float>();
    p.ldc = K;
    p.ones_col = bias_here ? K : -1;
    p.ones_out = bias_here ? db.data_ptr<float>() : nullptr;
    add_prob(pb, p, true, prec == 1 ? MMCfg<true>::KC : MMCfg<false>::KC, mask != nullptr);
  }
  launch(pb, dY, prec == 1);
  std::vector<at::Tensor> out;
  for (auto& t : dxs) out.push_back(t.defined() ? t : at::empty({0}, dY.options()));
  for (auto& t : dws) out.push_back(t.defined() ? t : at::empty({0}, dY.options()));
  out.push_back(with_bias ? db : at::empty({0}, dY.options()));
  return out;
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("mm_fwd(Tensor[] Xs, Tensor[] Ws, Tensor? b, Tensor? residual, int act, int prec) -> Tensor");
  m.def(
      "mm_bwd(Tensor dY, Tensor? Y, Tensor[] Xs, Tensor[] Ws, int[] need_dx, bool need_dw, bool with_bias, "
      "int prec) -> Tensor[]");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("mm_fwd", hy::mm_fwd);
  m.impl("mm_bwd", hy::mm_bwd);
}
