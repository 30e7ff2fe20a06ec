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

namespace hy {
namespace rpg {

typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int kMaxPtr = 48;
constexpr int kInsInts = 64;
constexpr int kOpdInts = 12;
constexpr int kBM = 16;         // rows per workgroup (one per wave for element-wise work)
constexpr int kThreads = 1024;  // 16 waves: every 16x16 output tile of a LIN in flight at once

enum { E_COPY = 0, E_MUL, E_MUL3, E_ACT, E_DOT3, E_NORM3, E_SINV, E_MASK, E_ZERO };

struct Args {
  const int* ins;  // [nins][kInsInts], operand descriptors embedded (see rowprog.py opnd)
  int nins;
  int N;
  int lds_w;       // LDS floats per row
  float* ws;
  const float* mask;  // [N] 0/1 or null
  float* p[kMaxPtr];
};

// operand: LDS part (int offsets into the block's LDS: ds_read / ds_write) and/or a global
// home (absolute rows)
struct Opd {
  float* gb;
  int loff, lld, gld, cs, c0, w, nc;
};

__device__ __forceinline__ Opd opd(const Args& A, const int* o) {
  Opd d;
  d.nc = o[0] ? o[9] : 0;
  d.gb = o[1] == 1 ? A.ws + (int64_t)o[2] * A.N : (o[1] == 2 ? A.p[o[2]] : nullptr);
  d.gld = o[3];
  d.loff = o[4];
  d.lld = o[5];
  d.cs = o[6];
  d.c0 = o[7];
  d.w = o[8];
  return d;
}

__device__ __forceinline__ float rd(const float* smem, const Opd& d, int i, int row, int c, int f) {
  const int o = (d.nc == 1 ? 0 : c) * d.cs + d.c0 + f;
  return d.loff >= 0 ? smem[kBM * d.loff + i * d.lld + o] : d.gb[(int64_t)row * d.gld + o];
}

__device__ __forceinline__ void wr(float* smem, const Opd& d, int i, int row, int c, int f, float v, int acc) {
  const int o = c * d.cs + d.c0 + f;
  if (d.loff >= 0) {
    float& p = smem[kBM * d.loff + i * d.lld + o];
    v = acc ? p + v : v;
    p = v;
    if (d.gb) d.gb[(int64_t)row * d.gld + o] = v;
  } else {
    float* p = d.gb + (int64_t)row * d.gld + o;
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

__device__ void run_ew(const Args& A, const int* I, int r0, float* smem) {
  const int op = I[1], arg = I[2], acc = I[4];
  const float coef = __int_as_float(I[3]);
  const Opd y = opd(A, I + 8), a = opd(A, I + 8 + kOpdInts), b = opd(A, I + 8 + 2 * kOpdInts),
            c = opd(A, I + 8 + 3 * kOpdInts);
  const int ync = (op == E_DOT3 || op == E_NORM3) ? 1 : y.nc;
  const int i = threadIdx.x >> 6, lane = threadIdx.x & 63, row = r0 + i;  // one row per wave
  if (row >= A.N) return;
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
        case E_MASK: r = rd(smem, a, i, row, cc, f) * (A.mask ? A.mask[row] : 1.f); break;
        default: r = 0.f;
      }
      if (op != E_ZERO) r *= coef;
      wr(smem, y, i, row, cc, f, r, acc);
    }
}

__device__ __forceinline__ float ldB(const float* W, int ldw, int k0, int trans, int k, int n) {
  return trans ? W[(int64_t)n * ldw + k0 + k] : W[(int64_t)k * ldw + k0 + n];
}

// 16x16 output tile (component c, columns n0..n0+15) of one LIN: 16 K-steps of operand
// loads issued together per round (one global latency per 64 K for the weights; A from LDS)
__device__ void run_lin(const Args& A, const int* I, int r0, float* smem) {
  const int acc = I[4];
  const Opd y = opd(A, I + 8), x0 = opd(A, I + 8 + kOpdInts), x1 = opd(A, I + 8 + 2 * kOpdInts);
  const float* W = A.p[I[56]];
  const int ldw = I[57], k0a = I[58], k0b = I[59], trans = I[61];
  const float* bias = I[60] >= 0 ? A.p[I[60]] : nullptr;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = kThreads >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int ntn = (y.w + 15) >> 4, tiles = y.nc * ntn;
  const int arow = r0 + i;
  const bool rok = arow < A.N;
  for (int tile = wv; tile < tiles; tile += nw) {
    const int c = tile / ntn, n0 = (tile % ntn) * 16, n = n0 + i;
    const bool nok = n < y.w;
    f4v a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
    for (int blk = 0; blk < 2; ++blk) {
      const Opd& x = blk == 0 ? x0 : x1;
      if (!x.nc) continue;
      const int k0 = blk == 0 ? k0a : k0b;
      const int K = x.w;
      for (int kb = 0; kb < K; kb += 64) {
        float av[16], bv[16];
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const int k = kb + 4 * s + g;
          const bool kok = k < K;
          bv[s] = (nok && kok) ? ldB(W, ldw, k0, trans, k, n) : 0.f;
          av[s] = (rok && kok) ? rd(smem, x, i, arow, c, k) : 0.f;
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
      const float bb = bias ? bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int il = 4 * g + r, row = r0 + il;
        if (row < A.N) wr(smem, y, il, row, c, n, s[r] + bb, acc);
      }
    }
  }
}

// the program is staged into LDS first (after the activation area): every instruction was
// a scalar-cache miss to L2 on a CU that runs one workgroup; its fields are then read from
// LDS (broadcast) and made wave-uniform with readfirstlane
__global__ void __launch_bounds__(kThreads) rowprog_kernel(Args A) {
  extern __shared__ float smem[];
  const int r0 = blockIdx.x * kBM;
  int* prog = reinterpret_cast<int*>(smem + kBM * A.lds_w);
  for (int t = threadIdx.x; t < A.nins * kInsInts; t += kThreads) prog[t] = A.ins[t];
  __syncthreads();
  int I[kInsInts];
  for (int q = 0; q < A.nins; ++q) {
#pragma unroll
    for (int t = 0; t < kInsInts; ++t) I[t] = __builtin_amdgcn_readfirstlane(prog[q * kInsInts + t]);
    if (I[0] == 1)
      run_lin(A, I, r0, smem);
    else
      run_ew(A, I, r0, smem);
    __syncthreads();
  }
}

}  // namespace rpg

void rowprog_run(const at::Tensor& prog, const at::Tensor& ws, const c10::optional<at::Tensor>& mask,
                 at::TensorList ptrs, int64_t N, int64_t lds_w) {
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
  if (mask.has_value() && mask->defined()) {
    HY_CHECK(mask->is_cuda() && mask->scalar_type() == at::kFloat && mask->numel() == N, "rowprog: mask [N] fp32");
    a.mask = mask->data_ptr<float>();
  }
  for (size_t k = 0; k < ptrs.size(); ++k) {
    const auto& t = ptrs[k];
    HY_CHECK(!t.defined() || t.numel() == 0 || (t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous()),
             "rowprog: pointer ", k, " must be a contiguous fp32 GPU tensor");
    a.p[k] = (t.defined() && t.numel()) ? t.data_ptr<float>() : nullptr;
  }
  if (N == 0 || a.nins == 0) return;
  const size_t lds = (size_t)lds_w * rpg::kBM * sizeof(float) + (size_t)prog.numel() * sizeof(int);
  HY_CHECK(lds <= 160 * 1024, "rowprog: activations + program exceed the 160 KiB LDS");
  if (lds > 64 * 1024) {
    static bool attr = false;
    if (!attr) {
      hipFuncSetAttribute((const void*)rpg::rowprog_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
  }
  rpg::rowprog_kernel<<<ceil_div(N, rpg::kBM), rpg::kThreads, lds, stream()>>>(a);
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("rowprog_run(Tensor prog, Tensor(a!) ws, Tensor? mask, Tensor(b!)[] ptrs, int N, int lds_w) -> ()");
}
TORCH_LIBRARY_IMPL(hydra, CUDA, m) { m.impl("rowprog_run", hy::rowprog_run); }
