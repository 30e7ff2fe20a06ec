// Fused PNA / PNAPlus message + DegreeScalerAggregation (gfx950).
//
// Reference semantics (hydragnn/models/PNAPlusStack.py:144-286 and PyG 2.5
// DegreeScalerAggregation, aggregators [mean,min,max,std] x scalers
// [identity, amplification, attenuation, linear]):
//     m_e   = pre_nn(cat[x_i, x_j, enc_e]) * rbf_lin(rbf_e)
//     agg_n = cat_s scaler_s(deg_n) * cat[mean, min, max, std]_{e->n}(m_e)
//     Z_n   = cat[x_n, agg_n]                       (input of post_nn)
// The concat-linear decomposition pre_nn(cat[x_i,x_j,e]) = A[i] + B[j] + C_e,
// with A|B = x @ [W_i;W_j]^T computed at NODE level (N << E), turns the
// per-edge GEMM into two gathers. This kernel fuses: gather A[dst], B[src],
// add C_e, multiply by the radial gate G_e, and the 4-way segment statistics
// + 4 degree scalers + the concat with x, so m_e never touches HBM in the
// forward pass.  Edges are CSR-sorted by destination: one contiguous range
// per node, no atomics, deterministic.
//
// The backward recomputes m_e from (A, B, C, G), derives dm_e from the saved
// statistics (mean/std are read back from Z's identity block), and emits
//   dpre_e = dm_e * G_e      (== dC_e; dA = segment-sum over dst, fused here;
//                             dB = segment-sum over src, done by seg_sum with the
//                             by-source permutation)
//   dG_e   = dm_e * pre_e
#include "common.h"
#include "pna_body.h"

namespace hy {

// AB: [N, ldab] with A at column offset 0 and B at column offset F.
template <int VEC>
__global__ void __launch_bounds__(256) pna_fwd_kernel(
    const float* __restrict__ x, const float* __restrict__ AB, int ldab, const float* __restrict__ C,
    const float* __restrict__ G, const int* __restrict__ src, const int* __restrict__ rowptr,
    float* __restrict__ Z, int* __restrict__ amin, int* __restrict__ amax, int N, int F, float avg_log,
    float avg_lin, int tpr, int rpb) {
  pna_fwd_node<VEC>(x, AB, ldab, C, G, src, rowptr, Z, amin, amax, blockIdx.x * rpb + threadIdx.x / tpr,
                    threadIdx.x % tpr, N, F, avg_log, avg_lin, tpr);
}

template <int VEC>
__global__ void __launch_bounds__(256) pna_bwd_kernel(
    const float* __restrict__ dZ, const float* __restrict__ Z, const float* __restrict__ AB, int ldab,
    const float* __restrict__ C, const float* __restrict__ G, const int* __restrict__ src,
    const int* __restrict__ rowptr, const int* __restrict__ amin, const int* __restrict__ amax,
    float* __restrict__ dpre, float* __restrict__ dG, float* __restrict__ dA, int N, int F, float avg_log,
    float avg_lin, int tpr, int rpb, int ldda) {
  const int n = blockIdx.x * rpb + threadIdx.x / tpr;
  const int c = threadIdx.x % tpr;
  if (n >= N) return;
  const int beg = rowptr[n], end = rowptr[n + 1];
  const int cnt = end - beg;
  const float d = (float)max(cnt, 1);
  const float lg = logf(d + 1.f);
  const float sc[4] = {1.f, lg / avg_log, avg_log / lg, d / avg_lin};
  const int ldz = 17 * F;
  const int nv = F / VEC;
  const float invc = 1.f / d;
  for (int v = c; v < nv; v += tpr) {
    const int f0 = v * VEC;
    const float* dzr = dZ + (int64_t)n * ldz + F + f0;
    PVec<VEC> dmean, dmin, dmax, dstd;
#pragma unroll
    for (int i = 0; i < VEC; ++i) { dmean.v[i] = 0.f; dmin.v[i] = 0.f; dmax.v[i] = 0.f; dstd.v[i] = 0.f; }
#pragma unroll
    for (int sidx = 0; sidx < 4; ++sidx) {
      const float* b = dzr + sidx * 4 * F;
      const PVec<VEC> g0 = pld<VEC>(b), g1 = pld<VEC>(b + F), g2 = pld<VEC>(b + 2 * F), g3 = pld<VEC>(b + 3 * F);
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        dmean.v[i] = fmaf(sc[sidx], g0.v[i], dmean.v[i]);
        dmin.v[i] = fmaf(sc[sidx], g1.v[i], dmin.v[i]);
        dmax.v[i] = fmaf(sc[sidx], g2.v[i], dmax.v[i]);
        dstd.v[i] = fmaf(sc[sidx], g3.v[i], dstd.v[i]);
      }
    }
    const float* zr = Z + (int64_t)n * ldz + F + f0;  // identity block
    const PVec<VEC> mean = pld<VEC>(zr);
    const PVec<VEC> sd = pld<VEC>(zr + 3 * F);
    PVec<VEC> kstd;  // d std / d m_e = (m_e - mean) * kstd
    int imn[VEC], imx[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      kstd.v[i] = sd.v[i] > 0.f ? dstd.v[i] * invc / sd.v[i] : 0.f;
      dmean.v[i] *= invc;
      imn[i] = amin[(int64_t)n * F + f0 + i];
      imx[i] = amax[(int64_t)n * F + f0 + i];
    }
    const PVec<VEC> a = pld<VEC>(AB + (int64_t)n * ldab + f0);
    PVec<VEC> da;
#pragma unroll
    for (int i = 0; i < VEC; ++i) da.v[i] = 0.f;
    // edge batches as in the forward: gathers of a batch in flight together (4 edges: the
    // backward co-runs with the attention backward, and 8-edge batches doubled its registers)
    constexpr int EB = VEC == 1 ? 4 : 2;
    for (int e0 = beg; e0 < end; e0 += EB) {
      int js[EB];
#pragma unroll
      for (int k = 0; k < EB; ++k) js[k] = src[min(e0 + k, end - 1)];
      PVec<VEC> b[EB], cc[EB], g[EB];
#pragma unroll
      for (int k = 0; k < EB; ++k) {
        const int e = min(e0 + k, end - 1);
        b[k] = pld<VEC>(AB + (int64_t)js[k] * ldab + F + f0);
        if (C) cc[k] = pld<VEC>(C + (int64_t)e * F + f0); else { for (int i = 0; i < VEC; ++i) cc[k].v[i] = 0.f; }
        if (G) g[k] = pld<VEC>(G + (int64_t)e * F + f0); else { for (int i = 0; i < VEC; ++i) g[k].v[i] = 1.f; }
      }
#pragma unroll
      for (int k = 0; k < EB; ++k) {
        const int e = e0 + k;
        if (e >= end) break;
        PVec<VEC> dp, dg;
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const float pre = a.v[i] + b[k].v[i] + cc[k].v[i];
          const float m = pre * g[k].v[i];
          float dm = dmean.v[i] + (m - mean.v[i]) * kstd.v[i];
          if (e == imn[i]) dm += dmin.v[i];
          if (e == imx[i]) dm += dmax.v[i];
          dp.v[i] = dm * g[k].v[i];
          dg.v[i] = dm * pre;
          da.v[i] += dp.v[i];
        }
        pst<VEC>(dpre + (int64_t)e * F + f0, dp);
        if (dG) pst<VEC>(dG + (int64_t)e * F + f0, dg);
      }
    }
    pst<VEC>(dA + (int64_t)n * ldda + f0, da);
  }
}

static const float* opt_edge_ptr(const c10::optional<at::Tensor>& t, int64_t E, int F, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  HY_CHECK_F32(*t);
  HY_CHECK(t->is_contiguous(), name, " must be contiguous");
  HY_CHECK(t->dim() == 2 && t->size(0) == E && t->size(1) == F, name, " must be [E, F]");
  return t->data_ptr<float>();
}

// One wave per node (lane = feature, 4-byte gathers) for F = 64 instead of 16 lanes x
// float4: 4x the waves in flight for the latency-bound edge gathers (OC20 GPS step on
// MI355X: 1.438 vs 1.457 ms with the float4 layout, tools/gpu_r3_iter.sh).
static bool pna_wave_per_node(int F) { return F == 64; }

std::tuple<at::Tensor, at::Tensor, at::Tensor> pna_fwd(const at::Tensor& x, const at::Tensor& AB,
                                                       const c10::optional<at::Tensor>& C_,
                                                       const c10::optional<at::Tensor>& G_,
                                                       const at::Tensor& src, const at::Tensor& rowptr,
                                                       double avg_log, double avg_lin) {
  HY_CHECK_CUDA(x);
  HY_CHECK_F32(x); HY_CHECK_F32(AB);
  HY_CHECK_I32(src); HY_CHECK_I32(rowptr);
  HY_CHECK_CONTIG(x);
  HY_CHECK(AB.stride(1) == 1, "AB rows must be contiguous");
  const int64_t N = x.size(0);
  const int F = (int)x.size(1);
  HY_CHECK(AB.size(0) == N && AB.size(1) == 2 * F, "AB must be [N, 2F]");
  const float* Cp = opt_edge_ptr(C_, src.numel(), F, "C");
  const float* Gp = opt_edge_ptr(G_, src.numel(), F, "G");
  HY_CHECK(rowptr.numel() == N + 1, "rowptr must be [N+1]");
  auto Z = at::empty({N, 17 * F}, x.options());
  auto amin = at::empty({N, F}, x.options().dtype(at::kInt));
  auto amax = at::empty({N, F}, x.options().dtype(at::kInt));
  if (N == 0) return {Z, amin, amax};
  const int ldab = (int)AB.stride(0);
  const bool v4 = (F % 4 == 0) && (ldab % 4 == 0) &&
                  (reinterpret_cast<uintptr_t>(AB.data_ptr<float>()) % 16 == 0) && !pna_wave_per_node(F);
  auto g = row_geom(N, v4 ? F : 4 * F);
  if (v4)
    pna_fwd_kernel<4><<<g.blocks, 256, 0, stream()>>>(
        x.data_ptr<float>(), AB.data_ptr<float>(), ldab, Cp, Gp,
        src.data_ptr<int>(), rowptr.data_ptr<int>(), Z.data_ptr<float>(), amin.data_ptr<int>(),
        amax.data_ptr<int>(), N, F, (float)avg_log, (float)avg_lin, g.tpr, g.rows_per_block);
  else
    pna_fwd_kernel<1><<<g.blocks, 256, 0, stream()>>>(
        x.data_ptr<float>(), AB.data_ptr<float>(), ldab, Cp, Gp,
        src.data_ptr<int>(), rowptr.data_ptr<int>(), Z.data_ptr<float>(), amin.data_ptr<int>(),
        amax.data_ptr<int>(), N, F, (float)avg_log, (float)avg_lin, g.tpr, g.rows_per_block);
  return {Z, amin, amax};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> pna_bwd(const at::Tensor& dZ_, const at::Tensor& Z,
                                                       const at::Tensor& AB, const c10::optional<at::Tensor>& C_,
                                                       const c10::optional<at::Tensor>& G_, const at::Tensor& src,
                                                       const at::Tensor& rowptr, const at::Tensor& amin,
                                                       const at::Tensor& amax, double avg_log,
                                                       double avg_lin) {
  auto dZ = dZ_.contiguous();
  HY_CHECK_CUDA(dZ);
  const int64_t N = Z.size(0);
  const int F = (int)(Z.size(1) / 17);
  const int64_t E = src.numel();
  const float* Cp = opt_edge_ptr(C_, E, F, "C");
  const float* Gp = opt_edge_ptr(G_, E, F, "G");
  auto dpre = at::empty({E, F}, Z.options());
  auto dG = Gp ? at::empty({E, F}, Z.options()) : at::empty({0}, Z.options());
  // dA is written into the left half of a [N, 2F] buffer: the caller's seg_sum_out fills the
  // right half (dB), so dAB needs no concatenation
  auto dA = at::empty({N, 2 * F}, Z.options());
  if (N == 0) return {dpre, dG, dA};
  const int ldab = (int)AB.stride(0);
  const bool v4 = (F % 4 == 0) && (ldab % 4 == 0) &&
                  (reinterpret_cast<uintptr_t>(AB.data_ptr<float>()) % 16 == 0) && !pna_wave_per_node(F);
  auto g = row_geom(N, v4 ? F : 4 * F);
  if (v4)
    pna_bwd_kernel<4><<<g.blocks, 256, 0, stream()>>>(
        dZ.data_ptr<float>(), Z.data_ptr<float>(), AB.data_ptr<float>(), ldab, Cp,
        Gp, src.data_ptr<int>(), rowptr.data_ptr<int>(), amin.data_ptr<int>(),
        amax.data_ptr<int>(), dpre.data_ptr<float>(), Gp ? dG.data_ptr<float>() : nullptr, dA.data_ptr<float>(), N, F,
        (float)avg_log, (float)avg_lin, g.tpr, g.rows_per_block, 2 * F);
  else
    pna_bwd_kernel<1><<<g.blocks, 256, 0, stream()>>>(
        dZ.data_ptr<float>(), Z.data_ptr<float>(), AB.data_ptr<float>(), ldab, Cp,
        Gp, src.data_ptr<int>(), rowptr.data_ptr<int>(), amin.data_ptr<int>(),
        amax.data_ptr<int>(), dpre.data_ptr<float>(), Gp ? dG.data_ptr<float>() : nullptr, dA.data_ptr<float>(), N, F,
        (float)avg_log, (float)avg_lin, g.tpr, g.rows_per_block, 2 * F);
  return {dpre, dG, dA};
}

// ---------------------------------------------------------------------------------
// Derived weights of one PNAPlus conv with an edge encoder (concat-linear
// decomposition, PNAPlusStack.py:250-279).  pre_nn weight W [F, 3F] has column
// blocks (x_i | x_j | enc_e); the edge encoder maps cat[e (d), r (F)] -> F.  The
// per-step weight algebra
//     Wab = [W_i; W_j]            [2F, F]   (node GEMM  x @ Wab^T)
//     Wr  = W_e @ encW[:, d:]     [F, F]    (edge GEMM  r @ Wr^T)
//     Wd  = W_e @ encW[:, :d]     [F, d]
//     bc  = W_e @ encb + b        [F]       (pre_nn bias moved onto the edge term)
// was ~25 tiny torch kernels per layer per step (cat, slices, their zero-fill/copy
// backward, accumulation adds, mm/mv); here it is one launch forward and one
// backward.  Copies are one element per thread; every dot product is owned by ONE
// wave (lanes split the reduction, then a shuffle reduction), so each output
// costs one round of coalesced L2 loads instead of a serial K-long load chain.

// sum_k a[k * sa] * b[k * sb], k < K, reduced over the wave (all lanes get it)
__device__ __forceinline__ float wave_dot(const float* __restrict__ a, int sa, const float* __restrict__ b, int sb,
                                          int K) {
  float acc = 0.f;
  for (int k = lane_id(); k < K; k += 64) acc = fmaf(a[(int64_t)k * sa], b[(int64_t)k * sb], acc);
  return wave_sum(acc);
}

__device__ __forceinline__ void wprep_fwd_body(const float* __restrict__ W, const float* __restrict__ b,
                                               const float* __restrict__ encW, const float* __restrict__ encb,
                                               float* __restrict__ Wab, float* __restrict__ Wr, float* __restrict__ Wd,
                                               float* __restrict__ bc, int F, int d);

__global__ void __launch_bounds__(256) pna_wprep_fwd_kernel(const float* __restrict__ W, const float* __restrict__ b,
                                                            const float* __restrict__ encW,
                                                            const float* __restrict__ encb, float* __restrict__ Wab,
                                                            float* __restrict__ Wr, float* __restrict__ Wd,
                                                            float* __restrict__ bc, int F, int d) {
  wprep_fwd_body(W, b, encW, encb, Wab, Wr, Wd, bc, F, d);
}

// every layer of a stack in one launch (blockIdx.y = layer): the fused GPS encoder prepares
// all its layers' weights up front
constexpr int kWprepMaxL = 8;
struct WprepMulti {
  const float *W[kWprepMaxL], *b[kWprepMaxL], *encW[kWprepMaxL], *encb[kWprepMaxL];
  float *Wab[kWprepMaxL], *Wr[kWprepMaxL], *Wd[kWprepMaxL], *bc[kWprepMaxL];
};

__global__ void __launch_bounds__(256) pna_wprep_fwd_multi_kernel(WprepMulti m, int F, int d) {
  const int l = blockIdx.y;
  wprep_fwd_body(m.W[l], m.b[l], m.encW[l], m.encb[l], m.Wab[l], m.Wr[l], m.Wd[l], m.bc[l], F, d);
}

__device__ __forceinline__ void wprep_fwd_body(const float* __restrict__ W, const float* __restrict__ b,
                                               const float* __restrict__ encW, const float* __restrict__ encb,
                                               float* __restrict__ Wab, float* __restrict__ Wr, float* __restrict__ Wd,
                                               float* __restrict__ bc, int F, int d) {
  // one thread per output element (Wab copy, then the Wr / Wd / bc dot products of length F
  // over L1/L2-resident operands, fixed sequential order).  The round-1 form (one wave per
  // dot, 2048 workgroups) cost ~19 us on the conv branch's critical path for F = 64.
  const int ld = 3 * F, le = d + F;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nab = 2LL * F * F, nr = (int64_t)F * F, nd = (int64_t)F * d;
  if (t < nab) {
    const int r = (int)(t / F), c = (int)(t % F);
    Wab[t] = W[(r % F) * ld + (r / F) * F + c];
    return;
  }
  int64_t q = t - nab;
  if (q >= nr + nd + F) return;
  const float* wrow;
  const float* col;
  int stride;
  float* dst;
  float v = 0.f;
  if (q < nr) {
    const int o = (int)(q / F), c = (int)(q % F);
    wrow = W + o * ld + 2 * F;
    col = encW + d + c;
    stride = le;
    dst = Wr + q;
  } else if (q < nr + nd) {
    const int64_t k = q - nr;
    const int o = (int)(k / d), c = (int)(k % d);
    wrow = W + o * ld + 2 * F;
    col = encW + c;
    stride = le;
    dst = Wd + k;
  } else {
    const int o = (int)(q - nr - nd);
    wrow = W + o * ld + 2 * F;
    col = encb;
    stride = 1;
    dst = bc + o;
    v = b[o];
  }
  // 16 operand pairs in flight per chunk, 4 partial sums (fixed order): a sequential
  // load -> fma chain paid one L2 latency per k (~18 us for F = 64 on MI355X)
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int k = 0;
  for (; k + 16 <= F; k += 16) {
    float w[16], x[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      w[u] = wrow[k + u];
      x[u] = col[(int64_t)(k + u) * stride];
    }
#pragma unroll
    for (int u = 0; u < 16; u += 4) {
      a0 = fmaf(w[u], x[u], a0);
      a1 = fmaf(w[u + 1], x[u + 1], a1);
      a2 = fmaf(w[u + 2], x[u + 2], a2);
      a3 = fmaf(w[u + 3], x[u + 3], a3);
    }
  }
  for (; k < F; ++k) a0 = fmaf(wrow[k], col[(int64_t)k * stride], a0);
  *dst = ((a0 + a1) + (a2 + a3)) + v;
}

// Backward of pna_wprep_fwd: dW [F,3F], db [F], dencW [F, d+F], dencb [F].
__global__ void __launch_bounds__(256) pna_wprep_bwd_kernel(
    const float* __restrict__ dWab, const float* __restrict__ dWr, const float* __restrict__ dWd,
    const float* __restrict__ dbc, const float* __restrict__ W, const float* __restrict__ encW,
    const float* __restrict__ encb, float* __restrict__ dW, float* __restrict__ db, float* __restrict__ dencW,
    float* __restrict__ dencb, int F, int d) {
  const int ld = 3 * F, le = d + F;
  const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t idx = tid; idx < 2 * F * F + F; idx += nthreads) {  // copies: dW[:, :2F], db
    if (idx < 2 * F * F) {
      const int o = (int)(idx / (2 * F)), c = (int)(idx % (2 * F));
      dW[o * ld + c] = dWab[((c / F) * F + o) * F + (c % F)];
    } else {
      db[idx - 2 * F * F] = dbc[idx - 2 * F * F];
    }
  }
  // dots: dW_e (F*F, K = d + F + 1), dencW (F*(d+F), K = F), dencb (F, K = F)
  const int64_t nd = (int64_t)F * F + (int64_t)F * le + F;
  const int64_t nwaves = nthreads / 64;
  for (int64_t q = tid / 64; q < nd; q += nwaves) {
    float v;
    float* dst;
    if (q < F * F) {  // dW_e[o, j] = sum_c dWd[o,c] encW[j,c] + sum_c dWr[o,c] encW[j,d+c] + dbc[o] encb[j]
      const int o = (int)(q / F), j = (int)(q % F);
      v = wave_dot(dWr + o * F, 1, encW + j * le + d, 1, F) + dbc[o] * encb[j];
      if (d > 0) v += wave_dot(dWd + o * d, 1, encW + j * le, 1, d);
      dst = dW + o * ld + 2 * F + j;
    } else if (q < (int64_t)F * F + (int64_t)F * le) {  // dencW[j, c] = sum_o W_e[o, j] [dWd | dWr][o, c]
      const int64_t k = q - F * F;
      const int j = (int)(k / le), c = (int)(k % le);
      v = c < d ? wave_dot(W + 2 * F + j, ld, dWd + c, d, F) : wave_dot(W + 2 * F + j, ld, dWr + (c - d), F, F);
      dst = dencW + k;
    } else {
      const int j = (int)(q - F * F - (int64_t)F * le);
      v = wave_dot(W + 2 * F + j, ld, dbc, 1, F);
      dst = dencb + j;
    }
    if (lane_id() == 0) *dst = v;
  }
}

// one wave per dot product (64 lanes), capped at 2048 workgroups
static int wprep_grid(int64_t dots) { return (int)std::min<int64_t>(ceil_div(dots * 64, 256), 2048); }

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> pna_wprep_fwd(const at::Tensor& W_, const at::Tensor& b_,
                                                                         const at::Tensor& encW_,
                                                                         const at::Tensor& encb_) {
  HY_CHECK_CUDA(W_);
  auto W = W_.contiguous(), b = b_.contiguous(), encW = encW_.contiguous(), encb = encb_.contiguous();
  HY_CHECK_F32(W); HY_CHECK_F32(b); HY_CHECK_F32(encW); HY_CHECK_F32(encb);
  const int F = (int)W.size(0);
  HY_CHECK(W.dim() == 2 && W.size(1) == 3 * F, "pna_wprep: W must be [F, 3F]");
  HY_CHECK(encW.dim() == 2 && encW.size(0) == F && encW.size(1) > F, "pna_wprep: encW must be [F, d+F]");
  HY_CHECK(b.numel() == F && encb.numel() == F, "pna_wprep: biases must have F entries");
  const int d = (int)encW.size(1) - F;
  auto Wab = at::empty({2 * F, F}, W.options()), Wr = at::empty({F, F}, W.options());
  auto Wd = at::empty({F, d}, W.options()), bc = at::empty({F}, W.options());
  const int64_t total = 2LL * F * F + (int64_t)F * F + (int64_t)F * d + F;  // one thread per output
  pna_wprep_fwd_kernel<<<ceil_div(total, 256), 256, 0, stream()>>>(W.data_ptr<float>(), b.data_ptr<float>(),
                                                               encW.data_ptr<float>(), encb.data_ptr<float>(),
                                                               Wab.data_ptr<float>(), Wr.data_ptr<float>(),
                                                               Wd.data_ptr<float>(), bc.data_ptr<float>(), F, d);
  return {Wab, Wr, Wd, bc};
}

// [Wab_0, Wr_0, Wd_0, bc_0, Wab_1, ...] for every layer, one launch
std::vector<at::Tensor> pna_wprep_fwd_multi(at::TensorList Ws, at::TensorList bs, at::TensorList encWs,
                                            at::TensorList encbs) {
  const int L = (int)Ws.size();
  HY_CHECK(L >= 1 && L <= kWprepMaxL && (int)bs.size() == L && (int)encWs.size() == L && (int)encbs.size() == L,
           "pna_wprep_fwd_multi: 1..8 layers of (W, b, encW, encb)");
  const int F = (int)Ws[0].size(0);
  const int d = (int)encWs[0].size(1) - F;
  WprepMulti m{};
  std::vector<at::Tensor> out, keep;
  for (int l = 0; l < L; ++l) {
    HY_CHECK_CUDA(Ws[l]);
    auto W = Ws[l].contiguous(), b = bs[l].contiguous(), encW = encWs[l].contiguous(), encb = encbs[l].contiguous();
    HY_CHECK_F32(W); HY_CHECK_F32(b); HY_CHECK_F32(encW); HY_CHECK_F32(encb);
    HY_CHECK(W.dim() == 2 && W.size(0) == F && W.size(1) == 3 * F, "pna_wprep: W must be [F, 3F] (same F per layer)");
    HY_CHECK(encW.dim() == 2 && encW.size(0) == F && encW.size(1) == F + d, "pna_wprep: encW must be [F, d+F]");
    HY_CHECK(b.numel() == F && encb.numel() == F, "pna_wprep: biases must have F entries");
    auto Wab = at::empty({2 * F, F}, W.options()), Wr = at::empty({F, F}, W.options());
    auto Wd = at::empty({F, d}, W.options()), bc = at::empty({F}, W.options());
    m.W[l] = W.data_ptr<float>();
    m.b[l] = b.data_ptr<float>();
    m.encW[l] = encW.data_ptr<float>();
    m.encb[l] = encb.data_ptr<float>();
    m.Wab[l] = Wab.data_ptr<float>();
    m.Wr[l] = Wr.data_ptr<float>();
    m.Wd[l] = Wd.data_ptr<float>();
    m.bc[l] = bc.data_ptr<float>();
    keep.insert(keep.end(), {W, b, encW, encb});
    out.insert(out.end(), {Wab, Wr, Wd, bc});
  }
  const int64_t total = 2LL * F * F + (int64_t)F * F + (int64_t)F * d + F;
  pna_wprep_fwd_multi_kernel<<<dim3((unsigned)ceil_div(total, 256), (unsigned)L), 256, 0, stream()>>>(m, F, d);
  return out;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> pna_wprep_bwd(const at::Tensor& dWab_, const at::Tensor& dWr_,
                                                                         const at::Tensor& dWd_, const at::Tensor& dbc_,
                                                                         const at::Tensor& W_, const at::Tensor& encW_,
                                                                         const at::Tensor& encb_) {
  auto dWab = dWab_.contiguous(), dWr = dWr_.contiguous(), dWd = dWd_.contiguous(), dbc = dbc_.contiguous();
  auto W = W_.contiguous(), encW = encW_.contiguous(), encb = encb_.contiguous();
  const int F = (int)W.size(0), d = (int)encW.size(1) - F;
  HY_CHECK(dWab.numel() == 2 * F * F && dWr.numel() == F * F && dWd.numel() == F * d && dbc.numel() == F,
           "pna_wprep_bwd: gradient shapes do not match the forward");
  auto dW = at::empty_like(W), db = at::empty({F}, W.options());
  auto dencW = at::empty_like(encW), dencb = at::empty({F}, W.options());
  const int64_t total = (int64_t)F * F + (int64_t)F * (d + F) + F;
  pna_wprep_bwd_kernel<<<wprep_grid(total), 256, 0, stream()>>>(
      dWab.data_ptr<float>(), dWr.data_ptr<float>(), dWd.data_ptr<float>(), dbc.data_ptr<float>(),
      W.data_ptr<float>(), encW.data_ptr<float>(), encb.data_ptr<float>(), dW.data_ptr<float>(),
      db.data_ptr<float>(), dencW.data_ptr<float>(), dencb.data_ptr<float>(), F, d);
  return {dW, db, dencW, dencb};
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def(
      "pna_fwd(Tensor x, Tensor AB, Tensor? C, Tensor? G, Tensor src, Tensor rowptr, float avg_log, "
      "float avg_lin) -> (Tensor, Tensor, Tensor)");
  m.def(
      "pna_bwd(Tensor dZ, Tensor Z, Tensor AB, Tensor? C, Tensor? G, Tensor src, Tensor rowptr, Tensor amin, "
      "Tensor amax, float avg_log, float avg_lin) -> (Tensor, Tensor, Tensor)");
  m.def("pna_wprep_fwd(Tensor W, Tensor b, Tensor encW, Tensor encb) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("pna_wprep_fwd_multi(Tensor[] W, Tensor[] b, Tensor[] encW, Tensor[] encb) -> Tensor[]");
  m.def(
      "pna_wprep_bwd(Tensor dWab, Tensor dWr, Tensor dWd, Tensor dbc, Tensor W, Tensor encW, Tensor encb) -> "
      "(Tensor, Tensor, Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("pna_fwd", hy::pna_fwd);
  m.impl("pna_bwd", hy::pna_bwd);
  m.impl("pna_wprep_fwd", hy::pna_wprep_fwd);
  m.impl("pna_wprep_fwd_multi", hy::pna_wprep_fwd_multi);
  m.impl("pna_wprep_bwd", hy::pna_wprep_bwd);
}
