// Row-program interpreter for gfx950: one launch executes a whole node-level chain
// (ops/rowprog.py) — forward, first-order VJP or second-order (dual + reverse) program —
// over 16-row blocks, instead of one launch per op and per derivative order.
//
// Programs are straight-line lists of two instruction kinds (see rowprog.py):
//   LIN  y[row, c, n] (+)= sum_blk sum_k x_blk[row, c, k] B_blk(k, n) (+ bias[n])
//        B(k, n) = W[n * ldw + k0 + k] (x W^T)  or  W[k * ldw + k0 + n] (x W)
//        on v_mfma_f32_16x16x4_f32 (exact fp32): 16x16 output tiles (component, column
//        block) spread over the workgroup's 4 waves;
//   EW   y (+)= coef * op(a, b, c) element-wise (scalar operands broadcast over the 3
//        Cartesian components; DOT3 / NORM3 reduce over them).
// A workgroup (16 waves) owns 16 rows for the whole program.  Values live in LDS for their
// live range (allocated at lowering time by liveness, odd row strides), mirrored to a
// global home when something outside the program reads them (outputs; the factors of the
// weight gradients); values that do not fit stay in a per-call global workspace.
// Instructions are separated by a workgroup barrier (its workgroup-scope fence also makes
// global stores visible across the block's waves: same CU, shared L1).
//
// Weight gradients are NOT formed here: the program writes the row-wise factors (adjoints
// and activations) and the host issues one grouped MFMA weight-gradient launch
// (linear.hip linear_wgrad_grouped) over all of them.
#include "common.h"

#include <cstdlib>

namespace hy {
namespace rpg {

typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int kMaxPtr = 48;
constexpr int kInsInts = 64;
constexpr int kOpdInts = 12;
constexpr int kBM = 16;         // rows per workgroup (one per wave for element-wise work)

enum { E_COPY = 0, E_MUL, E_MUL3, E_ACT, E_DOT3, E_NORM3, E_SINV, E_MASK, E_ZERO };

struct Args {
  const int* ins;  // [nins][kInsInts], operand descriptors embedded (see rowprog.py opnd)
  int nins;
  int N;
  int lds_w;       // LDS floats per row
  float* ws;
  const float* mask;  // [N] 0/1 or null
  long long* dbg;     // optional per-instruction cycle stamps of workgroup 0 (profiling)
  int nwp;            // pointers [0, nwp) are the program's weights (L2 prefetch)
  int rb;             // rows a workgroup owns (<= kBM; the 16-row MFMA tiles run half / quarter full)
  int wlen[kMaxPtr];  // their element counts
  float* p[kMaxPtr];
};

// explicit address spaces: pointers that come out of the kernel-argument table are generic
// to the compiler, and generic accesses become FLAT instructions (global-like latency even
// for LDS, and both wait counters)
typedef __attribute__((address_space(1))) float gfloat;
typedef __attribute__((address_space(3))) float lfloat;
__device__ __forceinline__ gfloat* G(const float* p) { return (gfloat*)(p); }

// operand: LDS part (int offsets into the block's LDS: ds_read / ds_write) and/or a global
// home (absolute rows)
struct Opd {
  float* gb;
  int loff, lld, gld, cs, c0, w, nc;
};

// An instruction lives in one VGPR: lane t holds field t.  Fields are broadcast to SGPRs
// (v_readlane) at their use, not all 64 up front (that spilled SGPRs into VGPR lanes).
struct Ins {
  int v;
  __device__ __forceinline__ int operator[](int t) const { return __builtin_amdgcn_readlane(v, t); }
};

__device__ __forceinline__ Opd opd(const Args& A, const Ins& I, int o) {
  Opd d;
  d.nc = I[o] ? I[o + 9] : 0;
  const int gk = I[o + 1];
  d.gb = gk == 1 ? A.ws + (int64_t)I[o + 2] * A.N : (gk == 2 ? A.p[I[o + 2]] : nullptr);
  d.gld = I[o + 3];
  d.loff = I[o + 4];
  d.lld = I[o + 5];
  d.cs = I[o + 6];
  d.c0 = I[o + 7];
  d.w = I[o + 8];
  return d;
}

// The two homes are read by DIFFERENT instructions: a plain ternary lets the compiler select
// the address and issue one FLAT load, which waits like a global load even when it hits LDS
// (measured ~2 us per element-wise instruction); the global path is a non-temporal load,
// which cannot be merged with the ds_read.
__device__ __forceinline__ float rd(lfloat* smem, const Opd& d, int i, int row, int c, int f) {
  const int o = (d.nc == 1 ? 0 : c) * d.cs + d.c0 + f;
  if (d.loff >= 0) return smem[kBM * d.loff + i * d.lld + o];
  return G(d.gb)[(int64_t)row * d.gld + o];
}

__device__ __forceinline__ void wr(lfloat* smem, const Opd& d, int i, int row, int c, int f, float v, int acc) {
  const int o = c * d.cs + d.c0 + f;
  if (d.loff >= 0) {
    lfloat& p = smem[kBM * d.loff + i * d.lld + o];
    v = acc ? p + v : v;
    p = v;
    if (d.gb) G(d.gb)[(int64_t)row * d.gld + o] = v;
  } else {
    gfloat* p = G(d.gb) + (int64_t)row * d.gld + o;
    *p = acc ? *p + v : v;
  }
}

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// activation kind (0 identity, 1 relu, 2 silu, 3 tanh, 4 sigmoid), derivative order 0..2
__device__ __forceinline__ float act(int kind, int order, float x) {
  switch (kind) {
    case 1:
      return order == 0 ? fmaxf(x, 0.f) : (order == 1 ? (x > 0.f ? 1.f : 0.f) : 0.f);
    case 2: {
      const float s = sigm(x);
      if (order == 0) return x * s;
      if (order == 1) return s * (1.f + x * (1.f - s));
      return s * (1.f - s) * (2.f + x * (1.f - 2.f * s));
    }
    case 3: {
      const float t = tanhf(x);
      if (order == 0) return t;
      if (order == 1) return 1.f - t * t;
      return -2.f * t * (1.f - t * t);
    }
    case 4: {
      const float s = sigm(x);
      if (order == 0) return s;
      if (order == 1) return s * (1.f - s);
      return s * (1.f - s) * (1.f - 2.f * s);
    }
    default:
      return order == 0 ? x : (order == 1 ? 1.f : 0.f);
  }
}

// element-wise instruction: the opcode (and activation kind/order) dispatch happens ONCE
// per instruction, outside the element loop; FAST = every operand is an LDS value (the
// lowering guarantees it whenever the values fit), so the element loop has no home checks.
struct LOpd {  // LDS-only operand view
  int base, lld, cs, c0, nc;
};
__device__ __forceinline__ LOpd lopd(const Opd& d) { return LOpd{kBM * d.loff + d.c0, d.lld, d.cs, d.c0, d.nc}; }
__device__ __forceinline__ float lrd(const lfloat* smem, const LOpd& d, int i, int c, int f) {
  return smem[d.base + i * d.lld + (d.nc == 1 ? 0 : c) * d.cs + f];
}

template <int OP, int KIND, int ORD>
__device__ __forceinline__ float ew_op(float a, float b, float c, bool hb, bool hc) {
  if constexpr (OP == E_COPY) return a;
  if constexpr (OP == E_MUL) return a * b;
  if constexpr (OP == E_MUL3) return a * b * c;
  if constexpr (OP == E_SINV) return a > 0.f ? 1.f / a : 0.f;
  if constexpr (OP == E_ACT) {
    float r = act(KIND, ORD, a);
    if (hb) r *= b;
    if (hc) r *= c;
    return r;
  }
  return 0.f;
}

template <int NT, int OP, int KIND, int ORD>
__device__ void ew_fast(const Args& A, const Opd& y, const Opd& a, const Opd& b, const Opd& c, float coef, int acc,
                        int r0, lfloat* smem) {
  const int lane = threadIdx.x & 63;
  const LOpd la = lopd(a), lb = lopd(b), lc = lopd(c);
  const bool hb = b.nc != 0, hc = c.nc != 0;
  const int ync = (OP == E_DOT3 || OP == E_NORM3) ? 1 : y.nc;
  const int ybase = kBM * y.loff + y.c0;
  const int nlim = min(A.N, r0 + A.rb);
  for (int i = threadIdx.x >> 6; i < kBM; i += NT / 64) {
    const int row = r0 + i;
    if (row >= nlim) break;
    const float m = (OP == E_MASK) ? (A.mask ? G(A.mask)[row] : 1.f) : 1.f;
    for (int cc = 0; cc < ync; ++cc)
      for (int f = lane; f < y.w; f += 64) {
        float r;
        if constexpr (OP == E_ZERO) {
          r = 0.f;
        } else if constexpr (OP == E_DOT3) {
          r = 0.f;
#pragma unroll
          for (int q = 0; q < 3; ++q) r += lrd(smem, la, i, q, f) * lrd(smem, lb, i, q, f);
          if (hc) r *= lrd(smem, lc, i, 0, f);
          r *= coef;
        } else if constexpr (OP == E_NORM3) {
          float s2 = 0.f;
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            const float v = lrd(smem, la, i, q, f);
            s2 += v * v;
          }
          r = sqrtf(s2) * coef;
        } else if constexpr (OP == E_MASK) {
          r = lrd(smem, la, i, cc, f) * m * coef;
        } else {
          const float va = lrd(smem, la, i, cc, f);
          const float vb = (OP == E_MUL || OP == E_MUL3 || hb) ? lrd(smem, lb, i, cc, f) : 0.f;
          const float vc = (OP == E_MUL3 || hc) ? lrd(smem, lc, i, cc, f) : 0.f;
          r = ew_op<OP, KIND, ORD>(va, vb, vc, hb, hc) * coef;
        }
        lfloat& p = smem[ybase + i * y.lld + cc * y.cs + f];
        const float v = acc ? p + r : r;
        p = v;
        if (y.gb) G(y.gb)[(int64_t)row * y.gld + cc * y.cs + y.c0 + f] = v;
      }
  }
}

// general path (some operand lives in global memory): per-element home checks
template <int NT>
__device__ void ew_slow(const Args& A, const Ins& I, int r0, lfloat* smem) {
  const int op = I[1], arg = I[2], acc = I[4];
  const float coef = __int_as_float(I[3]);
  const Opd y = opd(A, I, 8), a = opd(A, I, 8 + kOpdInts), b = opd(A, I, 8 + 2 * kOpdInts),
            c = opd(A, I, 8 + 3 * kOpdInts);
  const int ync = (op == E_DOT3 || op == E_NORM3) ? 1 : y.nc;
  const int lane = threadIdx.x & 63;
  const int nlim = min(A.N, r0 + A.rb);
  for (int i = threadIdx.x >> 6; i < kBM; i += NT / 64) {
    const int row = r0 + i;
    if (row >= nlim) break;
    for (int cc = 0; cc < ync; ++cc)
      for (int f = lane; f < y.w; f += 64) {
        float r;
        switch (op) {
          case E_ZERO: r = 0.f; break;
          case E_COPY: r = rd(smem, a, i, row, cc, f); break;
          case E_MUL: r = rd(smem, a, i, row, cc, f) * rd(smem, b, i, row, cc, f); break;
          case E_MUL3: r = rd(smem, a, i, row, cc, f) * rd(smem, b, i, row, cc, f) * rd(smem, c, i, row, cc, f); break;
          case E_ACT: {
            r = act(arg >> 2, arg & 3, rd(smem, a, i, row, cc, f));
            if (b.nc) r *= rd(smem, b, i, row, cc, f);
            if (c.nc) r *= rd(smem, c, i, row, cc, f);
            break;
          }
          case E_DOT3: {
            r = 0.f;
#pragma unroll
            for (int q = 0; q < 3; ++q) r += rd(smem, a, i, row, q, f) * rd(smem, b, i, row, q, f);
            if (c.nc) r *= rd(smem, c, i, row, 0, f);
            break;
          }
          case E_NORM3: {
            float s2 = 0.f;
#pragma unroll
            for (int q = 0; q < 3; ++q) {
              const float v = rd(smem, a, i, row, q, f);
              s2 += v * v;
            }
            r = sqrtf(s2);
            break;
          }
          case E_SINV: {
            const float v = rd(smem, a, i, row, cc, f);
            r = v > 0.f ? 1.f / v : 0.f;
            break;
          }
          case E_MASK: r = rd(smem, a, i, row, cc, f) * (A.mask ? G(A.mask)[row] : 1.f); break;
          default: r = 0.f;
        }
        if (op != E_ZERO) r *= coef;
        wr(smem, y, i, row, cc, f, r, acc);
      }
  }
}

template <int NT>
__device__ void run_ew(const Args& A, const Ins& I, int r0, lfloat* smem) {
  if (!I[5]) {  // lowering flag: not every operand is an LDS value
    ew_slow<NT>(A, I, r0, smem);
    return;
  }
  const int op = I[1], arg = I[2], acc = I[4];
  const float coef = __int_as_float(I[3]);
  const Opd y = opd(A, I, 8), a = opd(A, I, 8 + kOpdInts), b = opd(A, I, 8 + 2 * kOpdInts),
            c = opd(A, I, 8 + 3 * kOpdInts);
#define HY_EW(OPC, K, O) ew_fast<NT, OPC, K, O>(A, y, a, b, c, coef, acc, r0, smem)
  switch (op) {
    case E_ZERO: HY_EW(E_ZERO, 0, 0); break;
    case E_COPY: HY_EW(E_COPY, 0, 0); break;
    case E_MUL: HY_EW(E_MUL, 0, 0); break;
    case E_MUL3: HY_EW(E_MUL3, 0, 0); break;
    case E_DOT3: HY_EW(E_DOT3, 0, 0); break;
    case E_NORM3: HY_EW(E_NORM3, 0, 0); break;
    case E_SINV: HY_EW(E_SINV, 0, 0); break;
    case E_MASK: HY_EW(E_MASK, 0, 0); break;
    case E_ACT:
      switch (arg) {
        case 0: HY_EW(E_ACT, 0, 0); break;
        case 1: HY_EW(E_ACT, 0, 1); break;
        case 2: HY_EW(E_ACT, 0, 2); break;
        case 4: HY_EW(E_ACT, 1, 0); break;
        case 5: HY_EW(E_ACT, 1, 1); break;
        case 6: HY_EW(E_ACT, 1, 2); break;
        case 8: HY_EW(E_ACT, 2, 0); break;
        case 9: HY_EW(E_ACT, 2, 1); break;
        case 10: HY_EW(E_ACT, 2, 2); break;
        case 12: HY_EW(E_ACT, 3, 0); break;
        case 13: HY_EW(E_ACT, 3, 1); break;
        case 14: HY_EW(E_ACT, 3, 2); break;
        case 16: HY_EW(E_ACT, 4, 0); break;
        case 17: HY_EW(E_ACT, 4, 1); break;
        case 18: HY_EW(E_ACT, 4, 2); break;
        default: break;
      }
      break;
    default: break;
  }
#undef HY_EW
}

__device__ __forceinline__ float ldB(const gfloat* W, int ldw, int k0, int trans, int k, int n) {
  return trans ? W[(int64_t)n * ldw + k0 + k] : W[(int64_t)k * ldw + k0 + n];
}

// 16x16 output tile (component c, columns n0..n0+15) of one LIN.  FAST (every A operand
// is an LDS value, flagged at lowering): per 64-deep K round the 16 weight loads are issued
// back to back with clamped, always-valid indices (no branch between them: a home check or
// a select there made the compiler wait out one full memory latency per K-step), then the
// 16 A values come from LDS (zeroed past K), then 16 MFMAs.  Rows past N only feed output
// rows that are never stored.
template <int NT, bool FAST>
__device__ void run_lin(const Args& A, const Ins& I, int r0, lfloat* smem) {
  const int acc = I[4];
  const Opd y = opd(A, I, 8), x0 = opd(A, I, 8 + kOpdInts), x1 = opd(A, I, 8 + 2 * kOpdInts);
  const gfloat* W = G(A.p[I[56]]);
  const int ldw = I[57], k0a = I[58], k0b = I[59], trans = I[61];
  const float* bias = I[60] >= 0 ? A.p[I[60]] : nullptr;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = NT >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int ntn = (y.w + 15) >> 4, tiles = y.nc * ntn;
  const int arow = r0 + i;
  const int nlim = min(A.N, r0 + A.rb);
  const bool rok = arow < nlim;
  for (int tile = wv; tile < tiles; tile += nw) {
    const int c = tile / ntn, n0 = (tile % ntn) * 16, n = n0 + i;
    const bool nok = n < y.w;
    const int nc_ = min(n, y.w - 1);
    const float bb = bias ? G(bias)[nc_] : 0.f;  // issued with the weight loads
    f4v a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
    for (int blk = 0; blk < 2; ++blk) {
      const Opd& x = blk == 0 ? x0 : x1;
      if (!x.nc) continue;
      const int k0 = blk == 0 ? k0a : k0b;
      const int K = x.w;
      const int xb = kBM * x.loff + i * x.lld + (x.nc == 1 ? 0 : c) * x.cs + x.c0;
      // the K order inside a 64-deep round is permuted (reduction order is free): lane group
      // g owns k = kb + 16 g + s, so a transposed-weight lane reads 16 CONSECUTIVE floats
      // (4 x 16-byte loads instead of 16 scattered dwords)
      const bool v4 = trans && ((ldw | k0) & 3) == 0;
      for (int kb = 0; kb < K; kb += 64) {
        float av[16], bv[16];
        if (v4 && kb + 16 * g + 16 <= K) {
          const gfloat* wr_ = W + (int64_t)nc_ * ldw + k0 + kb + 16 * g;
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            const f4v q = *reinterpret_cast<const __attribute__((address_space(1))) f4v*>(wr_ + 4 * s4);
            bv[4 * s4] = q[0];
            bv[4 * s4 + 1] = q[1];
            bv[4 * s4 + 2] = q[2];
            bv[4 * s4 + 3] = q[3];
          }
        } else {
#pragma unroll
          for (int s = 0; s < 16; ++s) {
            const int kc = min(kb + 16 * g + s, K - 1);
            bv[s] = trans ? W[(int64_t)nc_ * ldw + k0 + kc] : W[(int64_t)kc * ldw + k0 + nc_];
          }
        }
        if constexpr (FAST) {
#pragma unroll
          for (int s = 0; s < 16; ++s) {
            const int k = kb + 16 * g + s;
            const float v = smem[xb + min(k, K - 1)];
            av[s] = k < K ? v : 0.f;
          }
        } else {
#pragma unroll
          for (int s = 0; s < 16; ++s) {
            const int k = kb + 16 * g + s;
            av[s] = (rok && k < K) ? rd(smem, x, i, arow, c, k) : 0.f;
          }
        }
#pragma unroll
        for (int s = 0; s < 16; s += 2) {
          a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bv[s], a0, 0, 0, 0);
          a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s + 1], bv[s + 1], a1, 0, 0, 0);
        }
      }
    }
    const f4v s = a0 + a1;
    if (nok) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int il = 4 * g + r, row = r0 + il;
        if (row < nlim) wr(smem, y, il, row, c, n, s[r] + bb, acc);
      }
    }
  }
}

// the program is staged into LDS first (after the activation area): every instruction was
// a scalar-cache miss to L2 on a CU that runs one workgroup.  Each lane then reads ONE field
// of the next instruction (one LDS read per instruction, prefetched a step ahead) and the
// fields are broadcast from their lanes (v_readlane -> SGPRs); reading the 64 fields one by
// one cost ~2 us per instruction (measured, tools/bench_rowprog.py)
template <int NT>
__global__ void __launch_bounds__(NT) rowprog_kernel(Args A) {
  extern __shared__ float smem_[];
  lfloat* smem = (lfloat*)smem_;
  const int r0 = blockIdx.x * A.rb;
  __attribute__((address_space(3))) int* prog = (__attribute__((address_space(3))) int*)(smem + kBM * A.lds_w);
  const __attribute__((address_space(1))) int* gins = (const __attribute__((address_space(1))) int*)A.ins;
  for (int t = threadIdx.x; t < A.nins * kInsInts; t += NT) prog[t] = gins[t];
  // L2 prefetch of every weight the program reads: workgroups on one XCD (blockIdx % 8)
  // share an L2 and run the program in lockstep, so without it each LIN's weight loads
  // missed together to memory (one ~2 us latency per LIN instruction).  One touch per
  // 128-byte line, the XCD's workgroups splitting the lines; the loaded values feed a
  // never-taken store, so the loads are issued but nothing waits on them until they are
  // retired in order behind the first real loads.
  {
    const int xr = blockIdx.x >> 3, nxr = (gridDim.x + 7) >> 3;
    float sink = 0.f;
    for (int k = 0; k < A.nwp; ++k) {
      const gfloat* w = G(A.p[k]);
      const int lines = (A.wlen[k] + 31) >> 5;
      for (int l = xr + nxr * threadIdx.x; l < lines; l += nxr * NT) sink += w[l << 5];
    }
    if (sink == 1.234567e-30f && A.dbg) A.dbg[0] = 0;  // keeps the loads alive
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  int nxt = prog[lane];  // lane t holds field t of the next instruction (one LDS read per lane)
  for (int q = 0; q < A.nins; ++q) {
    const Ins I{nxt};
    if (q + 1 < A.nins) nxt = prog[(q + 1) * kInsInts + lane];
    const bool stamp = A.dbg && blockIdx.x == 0 && threadIdx.x == 0;
    long long t0 = stamp ? (long long)__builtin_amdgcn_s_memtime() : 0;
    long long t1 = t0;
    if (I[0] == 1) {
      if (I[5])
        run_lin<NT, true>(A, I, r0, smem);
      else
        run_lin<NT, false>(A, I, r0, smem);
    } else
      run_ew<NT>(A, I, r0, smem);
    long long t2 = stamp ? (long long)__builtin_amdgcn_s_memtime() : 0;
    if (!I[6]) __syncthreads();  // the lowering elides barriers between same-thread element-wise steps
    if (stamp) {
      const long long t3 = (long long)__builtin_amdgcn_s_memtime();
      A.dbg[4 * q] = t0;
      A.dbg[4 * q + 1] = t1;
      A.dbg[4 * q + 2] = t2;
      A.dbg[4 * q + 3] = t3;
    }
  }
}

}  // namespace rpg

void rowprog_run(const at::Tensor& prog, const at::Tensor& ws, const c10::optional<at::Tensor>& mask,
                 at::TensorList ptrs, int64_t N, int64_t lds_w, const c10::optional<at::Tensor>& dbg, int64_t nw) {
  HY_CHECK(prog.is_cuda() && prog.scalar_type() == at::kInt && prog.is_contiguous(), "rowprog: program");
  HY_CHECK(prog.numel() % rpg::kInsInts == 0, "rowprog: program size");
  HY_CHECK((int64_t)ptrs.size() <= rpg::kMaxPtr, "rowprog: too many pointers");
  rpg::Args a{};
  a.ins = prog.data_ptr<int>();
  a.nins = (int)(prog.numel() / rpg::kInsInts);
  a.N = (int)N;
  a.lds_w = (int)lds_w;
  HY_CHECK(lds_w >= 0, "rowprog: LDS width");
  a.ws = ws.numel() ? ws.data_ptr<float>() : nullptr;
  a.mask = nullptr;
  a.dbg = nullptr;
  if (dbg.has_value() && dbg->defined()) {
    HY_CHECK(dbg->is_cuda() && dbg->scalar_type() == at::kLong && dbg->numel() >= 4 * (prog.numel() / rpg::kInsInts),
             "rowprog: dbg must be int64 [4 * nins]");
    a.dbg = reinterpret_cast<long long*>(dbg->data_ptr<int64_t>());
  }
  if (mask.has_value() && mask->defined()) {
    HY_CHECK(mask->is_cuda() && mask->scalar_type() == at::kFloat && mask->numel() == N, "rowprog: mask [N] fp32");
    a.mask = mask->data_ptr<float>();
  }
  a.nwp = (int)std::min<int64_t>(nw, (int64_t)ptrs.size());
  for (size_t k = 0; k < ptrs.size(); ++k) {
    const auto& t = ptrs[k];
    a.wlen[k] = (t.defined() && (int64_t)k < a.nwp) ? (int)t.numel() : 0;
    HY_CHECK(!t.defined() || t.numel() == 0 || (t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous()),
             "rowprog: pointer ", k, " must be a contiguous fp32 GPU tensor");
    a.p[k] = (t.defined() && t.numel()) ? t.data_ptr<float>() : nullptr;
  }
  if (N == 0 || a.nins == 0) return;
  const size_t lds = (size_t)lds_w * rpg::kBM * sizeof(float) + (size_t)prog.numel() * sizeof(int);
  HY_CHECK(lds <= 160 * 1024, "rowprog: activations + program exceed the 160 KiB LDS");
  // workgroup size (HYDRA_ROWPROG_THREADS: 256 / 512 / 1024).  md17 PAINN forces on MI355X:
  // 512 -> 11.36k, 1024 -> 11.27k, 256 -> 9.85k graphs/s (tools/gpu_ab_env.sh)
  static int nt = [] {
    const char* e = std::getenv("HYDRA_ROWPROG_THREADS");
    const int v = e ? std::atoi(e) : 512;
    return (v == 1024 || v == 256) ? v : 512;
  }();
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)rpg::rowprog_kernel<256>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)rpg::rowprog_kernel<512>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)rpg::rowprog_kernel<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  // rows per workgroup: a small batch would fill a quarter of the 256 CUs with 16-row
  // blocks (md17 PAINN: 64 workgroups); every instruction is latency-bound, so smaller
  // blocks (the 16-row MFMA tiles then partly empty) spread the same program over more CUs.
  // HYDRA_ROWPROG_ROWS = 16 / 8 / 4 / 2 / 1 forces the block height.
  static int rows_env = [] {
    const char* e = std::getenv("HYDRA_ROWPROG_ROWS");
    const int v = e ? std::atoi(e) : 0;
    return (v == 16 || v == 8 || v == 4 || v == 2 || v == 1) ? v : 0;
  }();
  int rb = rows_env;
  if (rb == 0) {
    rb = rpg::kBM;
    while (rb > 4 && ceil_div(N, rb) < 2 * num_cus()) rb >>= 1;
  }
  a.rb = rb;
  const int grid = ceil_div(N, rb);
  if (nt == 1024)
    rpg::rowprog_kernel<1024><<<grid, 1024, lds, stream()>>>(a);
  else if (nt == 512)
    rpg::rowprog_kernel<512><<<grid, 512, lds, stream()>>>(a);
  else
    rpg::rowprog_kernel<256><<<grid, 256, lds, stream()>>>(a);
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("rowprog_run(Tensor prog, Tensor(a!) ws, Tensor? mask, Tensor(b!)[] ptrs, int N, int lds_w, Tensor(c!)? dbg=None, int nw=0) -> ()");
}
TORCH_LIBRARY_IMPL(hydra, CUDA, m) { m.impl("rowprog_run", hy::rowprog_run); }
