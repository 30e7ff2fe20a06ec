// Branch-stacked MLP read-out: every row runs the MLP chain of ITS branch (multi-branch
// decoders of the captured step, reference hydragnn/models/MACEStack.py:365-400 and
// mace_utils/modules/blocks.py:417-767: one head MLP per dataset branch, each row decoded by
// the branch of its graph).  The captured step cannot slice rows by branch on the host, and
// the torch form (every branch on every row through stacked GEMMs, then a per-row gather)
// cost ~12 launches per read-out head forward and ~20 backward; here a read-out head is one
// launch forward and one backward (+ one grouped weight-gradient launch pair).
//
// Layout: row r of branch b = rid[r] (rid < 0: padding, zero output / gradients).  Layer l
// maps I_l -> O_l: h_{l+1} = act_l(z_l), z_l = W_l[b] (s_l h_l) + bias_l[b]; W stored [O, I]
// row-major (trans = 0) or [I, O] (trans = 1, the e3nn x @ W layout of an o3.Linear to
// scalars).  One workgroup (4 waves) per row:
//   forward, per layer and 64-wide output chunk: lane i of wave w forms s h[i] W[j][i] for
//     its 16 outputs j = 64 c + 16 w + jj (rows of W read coalesced from L2), the wave's
//     [16][64] product tile goes through LDS once and lane t sums a quarter row; the layer
//     inputs h_l (scaled) and pre-activations z_l are saved for the backward;
//   backward: dz_l = dy act'(z_l), dh_l[i] = s_l sum_j W_l[b][j][i] dz_l[j] (lane i, the 4
//     waves split j, partials meet in LDS); dz_l is also written into a per-branch slab
//     [nb, R, O_l] (zero in the other branches' slabs), so dW_l[b] = slab_l[b]^T h_l and
//     db_l[b] = colsum(slab_l[b]) are plain grouped weight-gradient problems.
// Layer loops are rolled (the chain runs once per launch: instruction fetch bound when
// unrolled, see csrc/mlp.hip head_dx_row_kernel).
#include "common.h"

namespace hy {
namespace bm {

constexpr int kMaxL = 8, kMaxB = 8, kMaxW = 128;  // layers, branches, widths

struct Args {
  int L, nb, R, hd;
  int ldx;  // row stride of x (a column slice of a wider row, e.g. the scalar block)
  int dims[kMaxL + 1];
  int act[kMaxL];      // after layer l: 0 none, 1 relu, 2 silu, 3 tanh, 4 sigmoid
  int trans[kMaxL];
  float scale[kMaxL];  // input scale of layer l
  const long long* ptab;  // [2][L][nb] device pointer table: W then bias (0: none)
  float* hs[kMaxL];  // saved scaled inputs [R, I_l]
  float* zs[kMaxL];  // saved pre-activations [R, O_l]
  float* slab[kMaxL];  // backward: [nb, R, O_l]
};

__device__ __forceinline__ float act_f(int a, float z) {
  switch (a) {
    case 1: return fmaxf(z, 0.f);
    case 2: return z / (1.f + __expf(-z));
    case 3: return tanhf(z);
    case 4: return 1.f / (1.f + __expf(-z));
    default: return z;
  }
}
__device__ __forceinline__ float act_d(int a, float z) {
  switch (a) {
    case 1: return z > 0.f ? 1.f : 0.f;
    case 2: {
      const float s = 1.f / (1.f + __expf(-z));
      return s * (1.f + z * (1.f - s));
    }
    case 3: {
      const float t = tanhf(z);
      return 1.f - t * t;
    }
    case 4: {
      const float s = 1.f / (1.f + __expf(-z));
      return s * (1.f - s);
    }
    default: return 1.f;
  }
}

__device__ __forceinline__ int rl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float rlf(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ const float* rlp(const float* p, int l) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l), hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return (const float*)(((uint64_t)hi << 32) | lo);
}

__global__ void __launch_bounds__(256) fwd_kernel(const float* __restrict__ x, const int* __restrict__ rid, Args a,
                                                  const float* __restrict__ acc, float* __restrict__ out) {
  __shared__ float hbuf[kMaxW];
  __shared__ float zbuf[kMaxW];
  __shared__ float red[4 * 16 * 65];
  const int r = blockIdx.x, tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int L = a.L, nb = a.nb, b = rid[r];
  // per-layer scalars lane-indexed (lane l: layer l), broadcast with v_readlane (dynamic
  // indexing of the argument struct inside the rolled loop expands into select chains)
  const int ll = lane < kMaxL ? lane : kMaxL - 1;
  const int v_dims = a.dims[lane <= kMaxL ? lane : kMaxL], v_act = a.act[ll], v_tr = a.trans[ll];
  const float v_sc = a.scale[ll];
  const int bb = b < 0 ? 0 : b;
  // lane l holds layer l's weight / bias pointers of this row's branch (one load each)
  const float* v_W = (const float*)a.ptab[(0 * L + (lane < L ? lane : 0)) * nb + bb];
  const float* v_B = (const float*)a.ptab[(1 * L + (lane < L ? lane : 0)) * nb + bb];
  float* v_hs = a.hs[ll];
  float* v_zs = a.zs[ll];
  if (b < 0) {  // padding row: zero output (its saved values are never read through a slab)
    for (int j = tid; j < a.hd; j += 256)
      out[(int64_t)r * a.hd + j] = acc != nullptr ? acc[(int64_t)r * a.hd + j] : 0.f;
    for (int l = 0; l < L; ++l) {
      const int I = rl(v_dims, l), O = rl(v_dims, l + 1);
      float* hs = (float*)rlp(v_hs, l);
      float* zs = (float*)rlp(v_zs, l);
      for (int i = tid; i < I; i += 256) hs[(int64_t)r * I + i] = 0.f;
      for (int j = tid; j < O; j += 256) zs[(int64_t)r * O + j] = 0.f;
    }
    return;
  }
  (void)nb;
  {
    const int I0 = a.dims[0];
    const float s0 = a.scale[0];
    for (int i = tid; i < kMaxW; i += 256) hbuf[i] = i < I0 ? s0 * x[(int64_t)r * a.ldx + i] : 0.f;
  }
  __syncthreads();
  for (int l = 0; l < L; ++l) {
    const int I = rl(v_dims, l), O = rl(v_dims, l + 1), tr = rl(v_tr, l);
    const float* W = rlp(v_W, l);
    const float* B = rlp(v_B, l);
    float* hs = (float*)rlp(v_hs, l);
    for (int i = tid; i < I; i += 256) hs[(int64_t)r * I + i] = hbuf[i];
    for (int c0 = 0; c0 < O; c0 += 64) {
      float v[16];
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) v[jj] = 0.f;
      for (int ib = 0; ib < I; ib += 64) {
        const int i = ib + lane;
        const bool iok = i < I;
        const float hi = hbuf[iok ? i : 0];
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
          const int j = c0 + 16 * w + jj;
          const bool ok = iok && j < O;
          const int64_t off = tr ? (int64_t)i * O + j : (int64_t)j * I + i;
          const float wv = W[ok ? off : 0];
          v[jj] = fmaf(ok ? wv : 0.f, hi, v[jj]);
        }
      }
      // cross-lane sum over i through LDS: lane t sums a quarter of row t / 4
      float* rw = red + w * 16 * 65;
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) rw[jj * 65 + lane] = v[jj];
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      float o = 0.f;
      {
        const float* rr = rw + (lane >> 2) * 65 + 16 * (lane & 3);
#pragma unroll
        for (int q = 0; q < 16; ++q) o += rr[q];
      }
      o += __shfl_xor(o, 1, 64);
      o += __shfl_xor(o, 2, 64);
      const int j = c0 + 16 * w + (lane >> 2);
      if ((lane & 3) == 0 && j < O) zbuf[j] = o + (B != nullptr ? B[j] : 0.f);
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    const int ac = rl(v_act, l);
    float* zs = (float*)rlp(v_zs, l);
    const float sn = l + 1 < L ? rlf(v_sc, l + 1) : 1.f;
    for (int j = tid; j < kMaxW; j += 256) {
      const float z = j < O ? zbuf[j] : 0.f;
      if (j < O) zs[(int64_t)r * O + j] = z;
      hbuf[j] = j < O ? sn * act_f(ac, z) : 0.f;
    }
    __syncthreads();
  }
  for (int j = tid; j < a.hd; j += 256)
    out[(int64_t)r * a.hd + j] = hbuf[j] + (acc != nullptr ? acc[(int64_t)r * a.hd + j] : 0.f);
}

__global__ void __launch_bounds__(256) bwd_kernel(const float* __restrict__ gout, const int* __restrict__ rid, Args a,
                                                  float* __restrict__ dx) {
  __shared__ float dyb[kMaxW];
  __shared__ float part[4][kMaxW];
  const int r = blockIdx.x, tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int L = a.L, nb = a.nb, R = a.R, b = rid[r];
  const int ll = lane < kMaxL ? lane : kMaxL - 1;
  const int v_dims = a.dims[lane <= kMaxL ? lane : kMaxL], v_act = a.act[ll], v_tr = a.trans[ll];
  const float v_sc = a.scale[ll];
  const int bb = b < 0 ? 0 : b;
  const float* v_W = (const float*)a.ptab[(lane < L ? lane : 0) * nb + bb];
  float* v_zs = a.zs[ll];
  float* v_sl = a.slab[ll];
  const int OL = rl(v_dims, L);
  for (int j = tid; j < kMaxW; j += 256) dyb[j] = (b >= 0 && j < a.hd && j < OL) ? gout[(int64_t)r * a.hd + j] : 0.f;
  __syncthreads();
  for (int l = L - 1; l >= 0; --l) {
    const int I = rl(v_dims, l), O = rl(v_dims, l + 1), tr = rl(v_tr, l), ac = rl(v_act, l);
    const float* W = rlp(v_W, l);
    const float* zs = rlp(v_zs, l);
    float* sl = (float*)rlp(v_sl, l);
    // dz = dy act'(z): into LDS and the branch slabs
    for (int j = tid; j < O; j += 256) {
      const float d = b >= 0 ? dyb[j] * act_d(ac, zs[(int64_t)r * O + j]) : 0.f;
      dyb[j] = d;
      for (int q = 0; q < nb; ++q) sl[((int64_t)q * R + r) * O + j] = q == b ? d : 0.f;
    }
    __syncthreads();
    // dh[i] = s_l sum_j W[j][i] dz[j]: lane i, wave w takes j = 16 w + 64 c + jj
    const float s = rlf(v_sc, l);
    for (int ib = 0; ib < I; ib += 64) {
      const int i = ib + lane;
      const bool iok = i < I;
      float acc = 0.f;
      for (int c0 = 16 * w; c0 < O; c0 += 64) {
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
          const int j = c0 + jj;
          const bool ok = iok && j < O && b >= 0;
          const int64_t off = tr ? (int64_t)i * O + j : (int64_t)j * I + i;
          const float wv = W[ok ? off : 0];
          acc = fmaf(ok ? wv : 0.f, dyb[j < O ? j : 0], acc);
        }
      }
      if (iok) part[w][i] = acc;
    }
    __syncthreads();
    const float sp = l > 0 ? 1.f : 0.f;
    (void)sp;
    for (int i = tid; i < kMaxW; i += 256) {
      const float dh = i < I ? s * ((part[0][i] + part[1][i]) + (part[2][i] + part[3][i])) : 0.f;
      if (l == 0) {
        if (i < I) dx[(int64_t)r * I + i] = dh;
      } else {
        dyb[i] = dh;
      }
    }
    __syncthreads();
  }
}

}  // namespace bm

// ptab: int64 [2, L, nb] device addresses of W_l[b] (I x O floats, [O, I] or [I, O] by trans)
// and bias_l[b] (0: none), built once per parameter set by the caller.  Returns
// [out [R, hd], hs_0 .. hs_{L-1}, zs_0 .. zs_{L-1}].
static bm::Args bm_args(const at::Tensor& x, const at::Tensor& rid, const at::Tensor& ptab, int64_t nb_,
                        at::IntArrayRef dims, at::IntArrayRef acts, at::IntArrayRef trans, at::ArrayRef<double> scales,
                        int64_t hd) {
  HY_CHECK_CUDA(x);
  HY_CHECK_F32(x);
  HY_CHECK_I32(rid);
  const int L = (int)acts.size();
  HY_CHECK(L >= 1 && L <= bm::kMaxL && (int)dims.size() == L + 1 && (int)trans.size() == L && (int)scales.size() == L,
           "branch_mlp: 1..8 layers");
  const int nb = (int)nb_;
  HY_CHECK(nb >= 1 && nb <= bm::kMaxB, "branch_mlp: 1..8 branches");
  HY_CHECK(ptab.is_cuda() && ptab.scalar_type() == at::kLong && ptab.is_contiguous() && ptab.numel() == 2 * L * nb,
           "branch_mlp: pointer table int64 [2, L, nb]");
  HY_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.size(1) == dims[0] && rid.numel() == x.size(0) && rid.is_cuda(),
           "branch_mlp: x [R, I0] with unit column stride, rid [R]");
  bm::Args a{};
  a.ldx = (int)x.stride(0);
  a.L = L;
  a.nb = nb;
  a.R = (int)x.size(0);
  a.hd = (int)hd;
  a.ptab = reinterpret_cast<const long long*>(ptab.data_ptr<int64_t>());
  HY_CHECK(hd >= 1 && hd <= dims[L], "branch_mlp: hd <= last width");
  for (int l = 0; l <= L; ++l) {
    HY_CHECK(dims[l] >= 1 && dims[l] <= bm::kMaxW, "branch_mlp: widths 1..128");
    a.dims[l] = (int)dims[l];
  }
  for (int l = 0; l < L; ++l) {
    a.act[l] = (int)acts[l];
    a.trans[l] = (int)trans[l];
    a.scale[l] = (float)scales[l];
  }
  return a;
}

// acc (optional, [R, hd]): added to the output (read-outs summed over the stack's layers)
std::vector<at::Tensor> branch_mlp_fwd(const at::Tensor& x, const at::Tensor& rid, const at::Tensor& ptab, int64_t nb,
                                       at::IntArrayRef dims, at::IntArrayRef acts, at::IntArrayRef trans,
                                       at::ArrayRef<double> scales, int64_t hd, const c10::optional<at::Tensor>& acc) {
  bm::Args a = bm_args(x, rid, ptab, nb, dims, acts, trans, scales, hd);
  const int64_t R = x.size(0);
  const float* ap = nullptr;
  if (acc.has_value() && acc->defined()) {
    HY_CHECK(acc->is_cuda() && acc->scalar_type() == at::kFloat && acc->is_contiguous() && acc->numel() == R * hd,
             "branch_mlp: acc [R, hd] contiguous fp32");
    ap = acc->data_ptr<float>();
  }
  auto out = at::empty({R, hd}, x.options());
  std::vector<at::Tensor> res{out};
  for (int l = 0; l < a.L; ++l) res.push_back(at::empty({R, (int64_t)a.dims[l]}, x.options()));
  for (int l = 0; l < a.L; ++l) res.push_back(at::empty({R, (int64_t)a.dims[l + 1]}, x.options()));
  for (int l = 0; l < a.L; ++l) {
    a.hs[l] = res[1 + l].data_ptr<float>();
    a.zs[l] = res[1 + a.L + l].data_ptr<float>();
  }
  if (R > 0)
    bm::fwd_kernel<<<(int)R, 256, 0, stream()>>>(x.data_ptr<float>(), rid.data_ptr<int>(), a, ap, out.data_ptr<float>());
  return res;
}

// returns [dx [R, I0], slab_0 [nb, R, O_0], ..., slab_{L-1}]
std::vector<at::Tensor> branch_mlp_bwd(const at::Tensor& gout_, const at::Tensor& x, const at::Tensor& rid,
                                       const at::Tensor& ptab, int64_t nb, at::IntArrayRef dims,
                                       at::IntArrayRef acts, at::IntArrayRef trans, at::ArrayRef<double> scales,
                                       int64_t hd, at::TensorList zs) {
  bm::Args a = bm_args(x, rid, ptab, nb, dims, acts, trans, scales, hd);
  auto gout = gout_.contiguous();
  const int64_t R = x.size(0);
  HY_CHECK(gout.scalar_type() == at::kFloat && gout.numel() == R * hd, "branch_mlp_bwd: grad [R, hd]");
  HY_CHECK((int)zs.size() == a.L, "branch_mlp_bwd: saved pre-activations per layer");
  auto dx = at::empty({x.size(0), x.size(1)}, x.options());  // dense, whatever x's row stride
  std::vector<at::Tensor> res{dx};
  for (int l = 0; l < a.L; ++l) {
    HY_CHECK(zs[l].is_contiguous() && zs[l].numel() == R * a.dims[l + 1], "branch_mlp_bwd: zs[l] [R, O_l]");
    a.zs[l] = const_cast<float*>(zs[l].data_ptr<float>());
    res.push_back(at::empty({(int64_t)a.nb, R, (int64_t)a.dims[l + 1]}, x.options()));
    a.slab[l] = res.back().data_ptr<float>();
  }
  if (R > 0)
    bm::bwd_kernel<<<(int)R, 256, 0, stream()>>>(gout.data_ptr<float>(), rid.data_ptr<int>(), a, dx.data_ptr<float>());
  return res;
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def(
      "branch_mlp_fwd(Tensor x, Tensor rid, Tensor ptab, int nb, int[] dims, int[] acts, int[] trans, "
      "float[] scales, int hd, Tensor? acc=None) -> Tensor[]");
  m.def(
      "branch_mlp_bwd(Tensor gout, Tensor x, Tensor rid, Tensor ptab, int nb, int[] dims, int[] acts, "
      "int[] trans, float[] scales, int hd, Tensor[] zs) -> Tensor[]");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("branch_mlp_fwd", hy::branch_mlp_fwd);
  m.impl("branch_mlp_bwd", hy::branch_mlp_bwd);
}
