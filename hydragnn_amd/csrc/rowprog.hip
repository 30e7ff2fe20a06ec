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
// Values live in a per-call workspace (slot-major regions [N, nc * w]) or in external
// tensors (inputs, outputs, weights: the pointer table).  A workgroup owns 16 rows for the
// whole program; instructions are separated by a workgroup barrier (the workgroup-scope
// fence makes every wave's global stores visible to the others: same CU, shared L1).
//
// Weight gradients are NOT formed here: the program writes the row-wise factors (adjoints
// and activations) and the host issues one grouped MFMA weight-gradient launch
// (linear.hip linear_wgrad_grouped) over all of them.
#include "common.h"

namespace hy {
namespace rpg {

typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int kMaxPtr = 48;
constexpr int kInsInts = 32;
constexpr int kBM = 16;

enum { E_COPY = 0, E_MUL, E_MUL3, E_ACT, E_DOT3, E_NORM3, E_SINV, E_MASK, E_ZERO };

struct Args {
  const int* ins;   // [nins][kInsInts]
  const int* bufs;  // [nbuf][4]: type (0 workspace, 1 pointer), prefix | pointer index, w, nc
  int nins;
  int N;
  float* ws;
  const float* mask;  // [N] 0/1 or null
  float* p[kMaxPtr];
};

struct Opd {
  float* base;
  int ld, cs, c0, w, nc;
};

__device__ __forceinline__ Opd opd(const Args& A, const int* o) {
  Opd d;
  const int b = o[0];
  if (b < 0) {
    d.base = nullptr;
    d.ld = d.cs = d.c0 = d.w = d.nc = 0;
    return d;
  }
  const int* bt = A.bufs + 4 * b;
  d.base = bt[0] == 0 ? A.ws + (int64_t)bt[1] * A.N : A.p[bt[1]];
  d.cs = bt[2];
  d.ld = bt[2] * bt[3];
  d.c0 = o[1];
  d.w = o[2];
  d.nc = o[3];
  return d;
}

__device__ __forceinline__ float* at(const Opd& d, int row, int c, int f) {
  return d.base + (int64_t)row * d.ld + (d.nc == 1 ? 0 : c) * d.cs + d.c0 + f;
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

__device__ void run_ew(const Args& A, const int* I, int r0) {
  const int op = I[1], arg = I[2], acc = I[4];
  const float coef = __int_as_float(I[3]);
  const Opd y = opd(A, I + 5), a = opd(A, I + 9), b = opd(A, I + 13), c = opd(A, I + 17);
  const int ync = (op == E_DOT3 || op == E_NORM3) ? 1 : y.nc;
  const int tot = kBM * ync * y.w;
  for (int e = threadIdx.x; e < tot; e += blockDim.x) {
    const int f = e % y.w, t = e / y.w, cc = t % ync, i = t / ync, row = r0 + i;
    if (row >= A.N) continue;
    float r;
    switch (op) {
      case E_ZERO: r = 0.f; break;
      case E_COPY: r = *at(a, row, cc, f); break;
      case E_MUL: r = *at(a, row, cc, f) * *at(b, row, cc, f); break;
      case E_MUL3: r = *at(a, row, cc, f) * *at(b, row, cc, f) * *at(c, row, cc, f); break;
      case E_ACT: {
        r = act(arg >> 2, arg & 3, *at(a, row, cc, f));
        if (b.base) r *= *at(b, row, cc, f);
        if (c.base) r *= *at(c, row, cc, f);
        break;
      }
      case E_DOT3: {
        r = 0.f;
#pragma unroll
        for (int q = 0; q < 3; ++q) r += *at(a, row, q, f) * *at(b, row, q, f);
        if (c.base) r *= *at(c, row, 0, f);
        break;
      }
      case E_NORM3: {
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const float v = *at(a, row, q, f);
          s += v * v;
        }
        r = sqrtf(s);
        break;
      }
      case E_SINV: {
        const float v = *at(a, row, cc, f);
        r = v > 0.f ? 1.f / v : 0.f;
        break;
      }
      case E_MASK: r = *at(a, row, cc, f) * (A.mask ? A.mask[row] : 1.f); break;
      default: r = 0.f;
    }
    float* py = at(y, row, cc, f);
    if (op != E_ZERO) r *= coef;
    *py = acc ? *py + r : r;
  }
}

__device__ __forceinline__ float ldB(const float* W, int ldw, int k0, int trans, int k, int n) {
  return trans ? W[(int64_t)n * ldw + k0 + k] : W[(int64_t)k * ldw + k0 + n];
}

__device__ void run_lin(const Args& A, const int* I, int r0) {
  const int acc = I[4];
  const Opd y = opd(A, I + 5), x0 = opd(A, I + 9), x1 = opd(A, I + 13);
  const float* W = A.p[I[21]];
  const int ldw = I[22], k0a = I[23], k0b = I[24], trans = I[26];
  const float* bias = I[25] >= 0 ? A.p[I[25]] : nullptr;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
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
      if (!x.base) continue;
      const int k0 = blk == 0 ? k0a : k0b;
      const int K = x.w;
      const float* xr = rok ? at(x, arow, c, 0) : nullptr;
      int kb = 0;
      for (; kb + 8 <= K; kb += 8) {
        const float av0 = rok ? xr[kb + g] : 0.f, av1 = rok ? xr[kb + 4 + g] : 0.f;
        const float bv0 = nok ? ldB(W, ldw, k0, trans, kb + g, n) : 0.f;
        const float bv1 = nok ? ldB(W, ldw, k0, trans, kb + 4 + g, n) : 0.f;
        a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av0, bv0, a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av1, bv1, a1, 0, 0, 0);
      }
      for (; kb < K; kb += 4) {
        const int k = kb + g;
        const float av = (rok && k < K) ? xr[k] : 0.f;
        const float bv = (nok && k < K) ? ldB(W, ldw, k0, trans, k, n) : 0.f;
        a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, a0, 0, 0, 0);
      }
    }
    const f4v s = a0 + a1;
    if (nok) {
      const float bb = bias ? bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + 4 * g + r;
        if (row < A.N) {
          float* py = at(y, row, c, n);
          const float v = s[r] + bb;
          *py = acc ? *py + v : v;
        }
      }
    }
  }
}

__global__ void __launch_bounds__(256) rowprog_kernel(Args A) {
  const int r0 = blockIdx.x * kBM;
  for (int q = 0; q < A.nins; ++q) {
    const int* I = A.ins + q * kInsInts;
    if (I[0] == 1)
      run_lin(A, I, r0);
    else
      run_ew(A, I, r0);
    __syncthreads();
  }
}

}  // namespace rpg

void rowprog_run(const at::Tensor& prog, const at::Tensor& bufs, const at::Tensor& ws,
                 const c10::optional<at::Tensor>& mask, at::TensorList ptrs, int64_t N) {
  HY_CHECK(prog.is_cuda() && prog.scalar_type() == at::kInt && prog.is_contiguous(), "rowprog: program");
  HY_CHECK(bufs.is_cuda() && bufs.scalar_type() == at::kInt && bufs.is_contiguous(), "rowprog: buffer table");
  HY_CHECK(prog.numel() % rpg::kInsInts == 0, "rowprog: program size");
  HY_CHECK((int64_t)ptrs.size() <= rpg::kMaxPtr, "rowprog: too many pointers");
  rpg::Args a{};
  a.ins = prog.data_ptr<int>();
  a.bufs = bufs.data_ptr<int>();
  a.nins = (int)(prog.numel() / rpg::kInsInts);
  a.N = (int)N;
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
  rpg::rowprog_kernel<<<ceil_div(N, rpg::kBM), 256, 0, stream()>>>(a);
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("rowprog_run(Tensor prog, Tensor bufs, Tensor(a!) ws, Tensor? mask, Tensor(b!)[] ptrs, int N) -> ()");
}
TORCH_LIBRARY_IMPL(hydra, CUDA, m) { m.impl("rowprog_run", hy::rowprog_run); }
