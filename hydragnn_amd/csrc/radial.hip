// Fused radial features of a PNAPlus stack (gfx950).
//
// Reference: PNAPlusStack (hydragnn/models/PNAPlusStack.py:40-304) computes once per
// batch  rbf = BesselBasisLayer(dist)  (DimeNet envelope u(d/c) * sin(freq_k d/c),
// learnable freq) and then, in EVERY conv layer l,
//     r_l = ReLU(rbf_emb_l(rbf))      [E, F]   (Linear(K, F) + ReLU)
//     G_l = rbf_lin_l(rbf)            [E, F]   (Linear(K, F), no bias)
// With K = num_radial ~ 6 these are K-deep dot products per output: pure memory/launch
// cost.  As torch ops the Bessel basis, 2L GEMMs, L ReLUs and their backward (2L
// weight-gradient reductions, 2L input-gradient GEMMs + accumulation, the basis'
// elementwise chain) are ~50 launches per step for a 3-layer stack.  Here:
//   forward : one kernel: the basis values are computed once per (edge, k) into LDS,
//             lanes stream the features and write r_l, G_l for all layers;
//   backward: one kernel, one pass over (R, dR, dG): per-workgroup partial sums
//             of dW_emb, db_emb, dW_lin (lanes over features) and the per-edge
//             drbf_k = sum_l sum_f dr_l W_emb_l + dG_l W_lin_l (register
//             accumulators, one wave reduction per (edge, k)), ddist and dfreq ->
//             one fixed-order partial-sum pass.
// Deterministic, no atomics.  Double backward (forces) uses the torch composite.
#include "common.h"

namespace hy {

constexpr int kRadMaxK = 8;
constexpr int kRadMaxL = 8;
constexpr int kRadBwdEdges = 64;      // edges per backward workgroup (partials per WG)

struct RadEnv {
  float inv_c;       // 1 / cutoff
  float p, a, b, c;  // envelope u(x) = 1/x + a x^(p-1) + b x^p + c x^(p+1) for x < 1
  int pe;            // p - 1 (the integer envelope exponent)
};

__device__ __forceinline__ void envelope(const RadEnv& ev, float x, float& u, float& du) {
  if (x >= 1.f || x <= 0.f) {
    u = 0.f;
    du = 0.f;
    return;
  }
  float xp0 = 1.f;
  for (int i = 0; i < ev.pe; ++i) xp0 *= x;
  const float xp1 = xp0 * x, xp2 = xp1 * x;
  u = 1.f / x + ev.a * xp0 + ev.b * xp1 + ev.c * xp2;
  du = -1.f / (x * x) + (ev.a * (ev.p - 1.f) * xp0 + ev.b * ev.p * xp1 + ev.c * (ev.p + 1.f) * xp2) / x;
}

// W layout: Wemb [L][F][K], bemb [L][F], Wlin [L][F][K];  out R, Gt: [L][E][F]
// Block: 16 edges; the 16 x K basis values are computed ONCE (one thread each) into
// LDS, then each wave streams 4 edges x F features with the (l, f) weights held in
// registers.  K is a template parameter (loops fully unrolled, no guards).
constexpr int kRadFwdEdges = 16;

template <int K>
__global__ void __launch_bounds__(256) radial_fwd_kernel(const float* __restrict__ dist, int64_t E,
                                                         const float* __restrict__ freq,
                                                         const float* __restrict__ Wemb,
                                                         const float* __restrict__ bemb,
                                                         const float* __restrict__ Wlin, int L, int F, RadEnv ev,
                                                         float* __restrict__ R, float* __restrict__ Gt) {
  __shared__ float rb[kRadFwdEdges][K];
  const int64_t e0 = (int64_t)blockIdx.x * kRadFwdEdges;
  const int ne = (int)min<int64_t>(kRadFwdEdges, E - e0);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (threadIdx.x < ne * K) {
    const int el = threadIdx.x / K, k = threadIdx.x % K;
    const float x = dist[e0 + el] * ev.inv_c;
    float u, du;
    envelope(ev, x, u, du);
    rb[el][k] = u * sinf(freq[k] * x);
  }
  __syncthreads();
  for (int f = lane; f < F; f += 64) {
    for (int l = 0; l < L; ++l) {
      float we[K], wl[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        we[k] = Wemb[((int64_t)l * F + f) * K + k];
        wl[k] = Wlin[((int64_t)l * F + f) * K + k];
      }
      const float b0 = bemb[l * F + f];
      for (int el = w; el < ne; el += 4) {
        float r = b0, g = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          r = fmaf(we[k], rb[el][k], r);
          g = fmaf(wl[k], rb[el][k], g);
        }
        const int64_t o = ((int64_t)l * E + e0 + el) * F + f;
        R[o] = fmaxf(r, 0.f);
        Gt[o] = g;
      }
    }
  }
}

// part layout per workgroup: [L][F][2K+1] (dWemb k, dWlin k, dbemb) then [K] dfreq.
// Block: 64 edges, wave w owns the 16 edges w*16 .. w*16+15; lanes own features.
// per-layer gradient bases: autograd hands the backward one [E, F] gradient per layer
// output; reading them in place avoids stacking them into [L, E, F] (two copy launches)
struct RadPtrs {
  const float* p[kRadMaxL];
};

// ONE pass over (R, dR, dG): per (f-chunk, layer) the wave's 16 rows are loaded
// at once (one latency round); each lane accumulates its features' weight
// gradients (folded over the 4 waves in LDS, fixed order) AND its share of every
// edge's input-side term  sum_f dr W_emb[f,k] + dg W_lin[f,k]  in registers
// (16 x K accumulators), which are wave-reduced once at the end.
template <int K>
__global__ void __launch_bounds__(256) radial_bwd_kernel(RadPtrs dR, RadPtrs dG,
                                                         const float* __restrict__ R,
                                                         const float* __restrict__ dist, int64_t E,
                                                         const float* __restrict__ freq,
                                                         const float* __restrict__ Wemb,
                                                         const float* __restrict__ Wlin, int L, int F, RadEnv ev,
                                                         float* __restrict__ ddist, float* __restrict__ part,
                                                         int64_t part_ld) {
  constexpr int kPer = kRadBwdEdges / 4;
  constexpr int per = 2 * K + 1;
  __shared__ float rb[kRadBwdEdges][K];
  __shared__ float drb[kRadBwdEdges][K];
  __shared__ float fold[4][64][per];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t e0 = (int64_t)blockIdx.x * kRadBwdEdges;
  const int ne = (int)min<int64_t>(kRadBwdEdges, E - e0);
  float* P = part + blockIdx.x * part_ld;
  for (int idx = threadIdx.x; idx < kRadBwdEdges * K; idx += blockDim.x) {
    const int el = idx / K, k = idx % K;
    float v = 0.f;
    if (el < ne) {
      const float x = dist[e0 + el] * ev.inv_c;
      float u, du;
      envelope(ev, x, u, du);
      v = u * sinf(freq[k] * x);
    }
    rb[el][k] = v;
  }
  __syncthreads();
  float acc[kPer][K];
#pragma unroll
  for (int i = 0; i < kPer; ++i)
#pragma unroll
    for (int k = 0; k < K; ++k) acc[i][k] = 0.f;
  for (int f0 = 0; f0 < F; f0 += 64) {
    const int f = f0 + lane;
    const bool fv = f < F;
    for (int l = 0; l < L; ++l) {
      float we[K], wl[K], aWe[K], aWl[K], ab = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int64_t wo = ((int64_t)l * F + min(f, F - 1)) * K + k;
        we[k] = fv ? Wemb[wo] : 0.f;
        wl[k] = fv ? Wlin[wo] : 0.f;
        aWe[k] = aWl[k] = 0.f;
      }
      float vr[kPer], vd[kPer], vg[kPer];
      // unconditional loads (clamped indices, masked after): a guarded load makes
      // the compiler drain the memory counter per row, serialising the 16 loads
      const int fc = min(f, F - 1);
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        const int el = min(w * kPer + i, ne - 1);
        const int64_t ol = (e0 + el) * F + fc;
        vr[i] = R[(int64_t)l * E * F + ol];
        vd[i] = dR.p[l][ol];
        vg[i] = dG.p[l][ol];
      }
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        const int el = w * kPer + i;
        const bool ok = fv && el < ne;
        const float dr = ok && vr[i] > 0.f ? vd[i] : 0.f, dg = ok ? vg[i] : 0.f;
        ab += dr;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          aWe[k] = fmaf(dr, rb[el][k], aWe[k]);
          aWl[k] = fmaf(dg, rb[el][k], aWl[k]);
          acc[i][k] = fmaf(dr, we[k], fmaf(dg, wl[k], acc[i][k]));
        }
      }
      // fold the 4 waves (fixed order) and write this block's partial
#pragma unroll
      for (int k = 0; k < K; ++k) {
        fold[w][lane][k] = aWe[k];
        fold[w][lane][K + k] = aWl[k];
      }
      fold[w][lane][2 * K] = ab;
      __syncthreads();
      if (fv) {
        for (int q = w; q < per; q += 4) {
          const float v = ((fold[0][lane][q] + fold[1][lane][q]) + fold[2][lane][q]) + fold[3][lane][q];
          P[((int64_t)l * F + f) * per + q] = v;
        }
      }
      __syncthreads();
    }
  }
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float c = wave_sum(acc[i][k]);
      if (lane == 0) drb[w * kPer + i][k] = c;
    }
  }
  __syncthreads();
  // per edge: ddist = sum_k drbf_k d rbf_k / d dist; per-edge dfreq terms into rb (reused)
  if (threadIdx.x < kRadBwdEdges) {
    const int el = threadIdx.x;
    float dd = 0.f;
    float x = 0.f, u = 0.f, du = 0.f;
    if (el < ne) {
      x = dist[e0 + el] * ev.inv_c;
      envelope(ev, x, u, du);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float sn, cs;
      sincosf(freq[k] * x, &sn, &cs);
      const float g = el < ne ? drb[el][k] : 0.f;
      dd += g * (du * sn + u * cs * freq[k]);
      rb[el][k] = g * u * cs * x;  // d rbf_k / d freq_k contribution
    }
    if (el < ne) ddist[e0 + el] = dd * ev.inv_c;
  }
  __syncthreads();
  if (threadIdx.x < K) {
    const int k = threadIdx.x;
    float a = 0.f;
    for (int el = 0; el < kRadBwdEdges; ++el) a += rb[el][k];
    P[(int64_t)L * F * per + k] = a;
  }
}

// out[j] = sum_b part[b * ld + j]: 64 columns per block, 16 waves split the partials,
// folded in a fixed order (deterministic)
constexpr int kRadSumWaves = 16;
__global__ void __launch_bounds__(64 * kRadSumWaves) radial_sum_kernel(const float* __restrict__ part, int nb,
                                                                       int64_t n, int64_t ld,
                                                                       float* __restrict__ out) {
  __shared__ float red[kRadSumWaves][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t j = (int64_t)blockIdx.x * 64 + lane;
  float a0 = 0.f, a1 = 0.f;
  if (j < n) {
    int b = w;
    for (; b + kRadSumWaves < nb; b += 2 * kRadSumWaves) {
      a0 += part[(int64_t)b * ld + j];
      a1 += part[(int64_t)(b + kRadSumWaves) * ld + j];
    }
    if (b < nb) a0 += part[(int64_t)b * ld + j];
  }
  red[w][lane] = a0 + a1;
  __syncthreads();
  if (w == 0 && j < n) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < kRadSumWaves; ++q) t += red[q][lane];
    out[j] = t;
  }
}

static RadEnv make_env(double cutoff, int64_t exponent) {
  RadEnv ev;
  const double p = (double)exponent + 1.0;
  ev.inv_c = (float)(1.0 / cutoff);
  ev.p = (float)p;
  ev.a = (float)(-(p + 1.0) * (p + 2.0) / 2.0);
  ev.b = (float)(p * (p + 2.0));
  ev.c = (float)(-p * (p + 1.0) / 2.0);
  ev.pe = (int)exponent;
  return ev;
}

static void check_w(const at::Tensor& t, int64_t L, int64_t F, int64_t K, const char* name) {
  HY_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), name, " must be contiguous fp32 on GPU");
  HY_CHECK(t.dim() == 3 && t.size(0) == L && t.size(1) == F && t.size(2) == K, name, " must be [L, F, K]");
}

std::tuple<at::Tensor, at::Tensor> radial_fwd(const at::Tensor& dist_, const at::Tensor& freq_, const at::Tensor& Wemb,
                                              const at::Tensor& bemb, const at::Tensor& Wlin, double cutoff,
                                              int64_t exponent) {
  HY_CHECK_CUDA(dist_);
  auto dist = dist_.contiguous(), freq = freq_.contiguous();
  HY_CHECK_F32(dist);
  HY_CHECK_F32(freq);
  const int64_t E = dist.numel(), K = freq.numel(), L = Wemb.size(0), F = Wemb.size(1);
  HY_CHECK(K >= 1 && K <= kRadMaxK && L >= 1 && L <= kRadMaxL, "radial: 1 <= K <= 8, 1 <= L <= 8");
  check_w(Wemb, L, F, K, "Wemb");
  check_w(Wlin, L, F, K, "Wlin");
  HY_CHECK(bemb.is_contiguous() && bemb.numel() == L * F, "bemb must be [L, F]");
  auto R = at::empty({L, E, F}, dist.options()), Gt = at::empty({L, E, F}, dist.options());
  if (E == 0) return {R, Gt};
  const auto ev = make_env(cutoff, exponent);
  const dim3 grid(ceil_div(E, kRadFwdEdges));
#define HY_RAD_FWD(KK)                                                                                            \
  radial_fwd_kernel<KK><<<grid, 256, 0, stream()>>>(dist.data_ptr<float>(), E, freq.data_ptr<float>(),            \
                                                    Wemb.data_ptr<float>(), bemb.data_ptr<float>(),               \
                                                    Wlin.data_ptr<float>(), (int)L, (int)F, ev, R.data_ptr<float>(), \
                                                    Gt.data_ptr<float>())
  switch (K) {
    case 1: HY_RAD_FWD(1); break;
    case 2: HY_RAD_FWD(2); break;
    case 3: HY_RAD_FWD(3); break;
    case 4: HY_RAD_FWD(4); break;
    case 5: HY_RAD_FWD(5); break;
    case 6: HY_RAD_FWD(6); break;
    case 7: HY_RAD_FWD(7); break;
    case 8: HY_RAD_FWD(8); break;
    default: HY_CHECK(false, "radial_fwd: unsupported basis size ", K);
  }
#undef HY_RAD_FWD
  return {R, Gt};
}

// Variant for the fused GPS encoder (ops/gps_encoder.py): per-layer weight pointers (no
// [L, F, K] stacking copies) and the basis itself written out, rbf [E, K] and its derivative
// w.r.t. the learnable frequencies drbf/dfreq [E, K] = u(x) cos(freq_k x) x, so that every
// radial parameter gradient becomes a row-reduction (dW = dY^T X) of the encoder's grouped
// weight-gradient launch: dW_emb = (dr * [r > 0])^T rbf, dW_lin = dG^T rbf, and
// dfreq = diag(drbf^T drbf/dfreq).
struct RadW {
  const float* we[kRadMaxL];
  const float* be[kRadMaxL];
  const float* wl[kRadMaxL];
  float* R[kRadMaxL];
  float* G[kRadMaxL];
};

// edge geometry for the in-kernel distance (null pos: the distances are given)
struct RadGeom {
  const float* pos;     // [N, 3]
  const int* dst;       // [E] receiver
  const int* src;       // [E] sender
  const float* shifts;  // [E, 3] or null
};

template <int K>
__global__ void __launch_bounds__(256) radial_fwd_multi_kernel(const float* __restrict__ dist, RadGeom geo,
                                                               int64_t E, const float* __restrict__ freq, RadW W,
                                                               int L, int F, RadEnv ev, float* __restrict__ rbf,
                                                               float* __restrict__ drdf) {
  __shared__ float rb[kRadFwdEdges][K];
  __shared__ float dl[kRadFwdEdges];
  const int64_t e0 = (int64_t)blockIdx.x * kRadFwdEdges;
  const int ne = (int)min<int64_t>(kRadFwdEdges, E - e0);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (threadIdx.x < ne) {
    const int64_t e = e0 + threadIdx.x;
    float d;
    if (geo.pos) {  // |pos[dst] - pos[src] + shift| (geometry.py edge_vectors_and_lengths)
      const float* pd = geo.pos + 3 * (int64_t)geo.dst[e];
      const float* ps = geo.pos + 3 * (int64_t)geo.src[e];
      float vx = pd[0] - ps[0], vy = pd[1] - ps[1], vz = pd[2] - ps[2];
      if (geo.shifts) {
        vx += geo.shifts[3 * e];
        vy += geo.shifts[3 * e + 1];
        vz += geo.shifts[3 * e + 2];
      }
      d = sqrtf(fmaf(vx, vx, fmaf(vy, vy, vz * vz)));
    } else {
      d = dist[e];
    }
    dl[threadIdx.x] = d;
  }
  __syncthreads();
  if (threadIdx.x < ne * K) {
    const int el = threadIdx.x / K, k = threadIdx.x % K;
    const float x = dl[el] * ev.inv_c;
    float u, du;
    envelope(ev, x, u, du);
    float sn, cs;
    sincosf(freq[k] * x, &sn, &cs);
    const float v = u * sn;
    rb[el][k] = v;
    rbf[(e0 + el) * K + k] = v;
    if (drdf) drdf[(e0 + el) * K + k] = u * cs * x;
  }
  __syncthreads();
  for (int f = lane; f < F; f += 64) {
    for (int l = 0; l < L; ++l) {
      float we[K], wl[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        we[k] = W.we[l][(int64_t)f * K + k];
        wl[k] = W.wl[l][(int64_t)f * K + k];
      }
      const float b0 = W.be[l][f];
      for (int el = w; el < ne; el += 4) {
        float r = b0, g = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          r = fmaf(we[k], rb[el][k], r);
          g = fmaf(wl[k], rb[el][k], g);
        }
        const int64_t o = (e0 + el) * F + f;
        W.R[l][o] = fmaxf(r, 0.f);
        W.G[l][o] = g;
      }
    }
  }
}

// returns [rbf [E, K], drbf/dfreq [E, K] (empty unless want_dfreq), R_0..R_{L-1}, G_0..G_{L-1}]
// Distances either given (dist [E]) or computed in the kernel from pos [N, 3], dst/src [E]
// int32 and optional shifts [E, 3] (no separate gather / subtract / norm launches).
std::vector<at::Tensor> radial_fwd_multi(const c10::optional<at::Tensor>& dist_, const at::Tensor& freq_,
                                         const std::vector<at::Tensor>& Wemb, const std::vector<at::Tensor>& bemb,
                                         const std::vector<at::Tensor>& Wlin, double cutoff, int64_t exponent,
                                         bool want_dfreq, const c10::optional<at::Tensor>& pos_,
                                         const c10::optional<at::Tensor>& dst_, const c10::optional<at::Tensor>& src_,
                                         const c10::optional<at::Tensor>& shifts_) {
  auto freq = freq_.contiguous();
  RadGeom geo{nullptr, nullptr, nullptr, nullptr};
  at::Tensor dist, pos, dsti, srci, shifts;
  int64_t E;
  if (pos_.has_value() && pos_->defined()) {
    pos = pos_->contiguous();
    HY_CHECK(dst_.has_value() && src_.has_value(), "radial_fwd_multi: pos needs dst and src");
    dsti = dst_->contiguous();
    srci = src_->contiguous();
    E = dsti.numel();
    HY_CHECK(pos.is_cuda() && pos.scalar_type() == at::kFloat && pos.dim() == 2 && pos.size(1) == 3 &&
                 dsti.scalar_type() == at::kInt && srci.scalar_type() == at::kInt && srci.numel() == E,
             "radial_fwd_multi: pos float [N, 3], dst/src int32 [E]");
    geo.pos = pos.data_ptr<float>();
    geo.dst = dsti.data_ptr<int>();
    geo.src = srci.data_ptr<int>();
    if (shifts_.has_value() && shifts_->defined()) {
      shifts = shifts_->contiguous();
      HY_CHECK(shifts.scalar_type() == at::kFloat && shifts.numel() == 3 * E, "radial_fwd_multi: shifts [E, 3]");
      geo.shifts = shifts.data_ptr<float>();
    }
  } else {
    HY_CHECK(dist_.has_value() && dist_->defined(), "radial_fwd_multi: dist or pos required");
    dist = dist_->contiguous();
    E = dist.numel();
  }
  const auto fopt = freq.options();
  const int64_t K = freq.numel(), L = (int64_t)Wemb.size();
  HY_CHECK(K >= 1 && K <= kRadMaxK && L >= 1 && L <= kRadMaxL && (int64_t)bemb.size() == L &&
               (int64_t)Wlin.size() == L,
           "radial_fwd_multi: 1 <= K <= 8, 1 <= L <= 8, one (Wemb, bemb, Wlin) per layer");
  const int64_t F = Wemb[0].size(0);
  RadW W{};
  std::vector<at::Tensor> out;
  auto rbf = at::empty({E, K}, fopt);
  auto drdf = want_dfreq ? at::empty({E, K}, fopt) : at::empty({0}, fopt);
  out.push_back(rbf);
  out.push_back(drdf);
  std::vector<at::Tensor> Rs, Gs;
  for (int64_t l = 0; l < L; ++l) {
    HY_CHECK(Wemb[l].is_contiguous() && Wemb[l].size(0) == F && Wemb[l].size(1) == K && Wlin[l].is_contiguous() &&
                 Wlin[l].sizes() == Wemb[l].sizes() && bemb[l].is_contiguous() && bemb[l].numel() == F,
             "radial_fwd_multi: per-layer weights [F, K], bias [F]");
    W.we[l] = Wemb[l].data_ptr<float>();
    W.be[l] = bemb[l].data_ptr<float>();
    W.wl[l] = Wlin[l].data_ptr<float>();
    Rs.push_back(at::empty({E, F}, fopt));
    Gs.push_back(at::empty({E, F}, fopt));
    W.R[l] = Rs.back().data_ptr<float>();
    W.G[l] = Gs.back().data_ptr<float>();
  }
  out.insert(out.end(), Rs.begin(), Rs.end());
  out.insert(out.end(), Gs.begin(), Gs.end());
  if (E == 0) return out;
  const auto ev = make_env(cutoff, exponent);
  const dim3 grid(ceil_div(E, kRadFwdEdges));
  float* dp = want_dfreq ? drdf.data_ptr<float>() : nullptr;
#define HY_RAD_FWDM(KK)                                                                                        \
  radial_fwd_multi_kernel<KK><<<grid, 256, 0, stream()>>>(dist.defined() ? dist.data_ptr<float>() : nullptr, geo, E, \
                                                          freq.data_ptr<float>(), W, (int)L, (int)F, ev,            \
                                                          rbf.data_ptr<float>(), dp)
  switch (K) {
    case 1: HY_RAD_FWDM(1); break;
    case 2: HY_RAD_FWDM(2); break;
    case 3: HY_RAD_FWDM(3); break;
    case 4: HY_RAD_FWDM(4); break;
    case 5: HY_RAD_FWDM(5); break;
    case 6: HY_RAD_FWDM(6); break;
    case 7: HY_RAD_FWDM(7); break;
    case 8: HY_RAD_FWDM(8); break;
    default: HY_CHECK(false, "radial_fwd_multi: unsupported basis size ", K);
  }
#undef HY_RAD_FWDM
  return out;
}

// returns ddist [E], dfreq [K], dWemb [L,F,K], dbemb [L,F], dWlin [L,F,K]
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> radial_bwd(
    const std::vector<at::Tensor>& dR_, const std::vector<at::Tensor>& dG_, const at::Tensor& R,
    const at::Tensor& dist_, const at::Tensor& freq_, const at::Tensor& Wemb, const at::Tensor& Wlin, double cutoff,
    int64_t exponent) {
  auto dist = dist_.contiguous(), freq = freq_.contiguous();
  const int64_t E = dist.numel(), K = freq.numel(), L = Wemb.size(0), F = Wemb.size(1);
  HY_CHECK(K >= 1 && K <= kRadMaxK && L >= 1 && L <= kRadMaxL, "radial_bwd: 1 <= K <= 8, 1 <= L <= 8");
  check_w(Wemb, L, F, K, "Wemb");
  check_w(Wlin, L, F, K, "Wlin");
  HY_CHECK(R.dim() == 3 && R.size(0) == L && R.size(1) == E && R.size(2) == F && R.is_contiguous(),
           "radial_bwd: R must be contiguous [L, E, F]");
  HY_CHECK((int64_t)dR_.size() == L && (int64_t)dG_.size() == L, "radial_bwd: one dR and one dG per layer");
  std::vector<at::Tensor> keep;  // contiguous copies (normally none) stay alive until launch
  RadPtrs pr{}, pg{};
  for (int64_t l = 0; l < L; ++l) {
    for (int which = 0; which < 2; ++which) {
      const at::Tensor& t = which == 0 ? dR_[l] : dG_[l];
      HY_CHECK(t.dim() == 2 && t.size(0) == E && t.size(1) == F && t.scalar_type() == at::kFloat && t.is_cuda(),
               "radial_bwd: per-layer gradients must be float [E, F] on the GPU");
      at::Tensor c = t.contiguous();
      keep.push_back(c);
      (which == 0 ? pr : pg).p[l] = c.data_ptr<float>();
    }
  }
  const int64_t per = 2 * K + 1;
  const int64_t ld = L * F * per + K;
  const int nb = std::max(1, ceil_div(E, kRadBwdEdges));
  auto part = at::empty({nb, ld}, dist.options());
  auto sums = at::empty({ld}, dist.options());
  auto ddist = at::empty({E}, dist.options());
  if (E > 0) {
    const auto ev = make_env(cutoff, exponent);
#define HY_RAD_BWD(KK)                                                                                              \
  radial_bwd_kernel<KK><<<nb, 256, 0, stream()>>>(pr, pg, R.data_ptr<float>(),                                   \
                                                  dist.data_ptr<float>(), E, freq.data_ptr<float>(),               \
                                                  Wemb.data_ptr<float>(), Wlin.data_ptr<float>(), (int)L, (int)F,   \
                                                  ev, ddist.data_ptr<float>(), part.data_ptr<float>(), ld)
    switch (K) {
      case 1: HY_RAD_BWD(1); break;
      case 2: HY_RAD_BWD(2); break;
      case 3: HY_RAD_BWD(3); break;
      case 4: HY_RAD_BWD(4); break;
      case 5: HY_RAD_BWD(5); break;
      case 6: HY_RAD_BWD(6); break;
      case 7: HY_RAD_BWD(7); break;
      case 8: HY_RAD_BWD(8); break;
      default: HY_CHECK(false, "radial_bwd: unsupported basis size ", K);
    }
#undef HY_RAD_BWD
    radial_sum_kernel<<<ceil_div(ld, 64), 64 * kRadSumWaves, 0, stream()>>>(part.data_ptr<float>(), nb, ld, ld,
                                                                            sums.data_ptr<float>());
  } else {
    sums.zero_();
  }
  auto g = sums.narrow(0, 0, L * F * per).view({L, F, per});
  auto dWemb = g.narrow(2, 0, K).contiguous();
  auto dWlin = g.narrow(2, K, K).contiguous();
  auto dbemb = g.select(2, 2 * K).contiguous();
  auto dfreq = sums.narrow(0, L * F * per, K);
  return {ddist, dfreq, dWemb, dbemb, dWlin};
}

// ---------------------------------------------------------------- MACE radial embedding
// out[e, k] = sqrt(2/rc) sin(w_k r)/r * env(r/rc) [r < rc], env(u) = 1 - (p+1)(p+2)/2 u^p +
// p(p+2) u^(p+1) - p(p+1)/2 u^(p+2): reference mace_utils/modules/radial.py:23-63 (BesselBasis),
// :98-130 (PolynomialCutoff), blocks.py:148-162 (RadialEmbeddingBlock).  As torch ops the
// basis + cutoff is ~15 elementwise launches over [E, K]; here one launch writes it, and the
// backward (edge-length gradient, first order) is one more.
struct MaceRadial {
  float pref, rc, p;
  __device__ __forceinline__ void env(float r, float& e, float& de) const {
    if (!(r < rc)) { e = 0.f; de = 0.f; return; }
    const float u = r / rc;
    const float up = powf(u, p - 1.f);  // u^(p-1); u > 0 for a real edge
    const float a = 0.5f * (p + 1.f) * (p + 2.f), b = p * (p + 2.f), c = 0.5f * p * (p + 1.f);
    const float u_p = up * u;
    e = 1.f - a * u_p + b * u_p * u - c * u_p * u * u;
    de = (-a * p * up + b * (p + 1.f) * u_p - c * (p + 2.f) * u_p * u) / rc;
  }
};

__global__ void __launch_bounds__(256) mace_radial_fwd_kernel(const float* __restrict__ r, const float* __restrict__ w,
                                                              float* __restrict__ out, int E, int K, MaceRadial m) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)E * K) return;
  const int e = (int)(t / K), k = (int)(t % K);
  const float x = r[e];
  float en, den;
  m.env(x, en, den);
  out[t] = m.pref * sinf(w[k] * x) / x * en;
}

__global__ void __launch_bounds__(256) mace_radial_bwd_kernel(const float* __restrict__ g, const float* __restrict__ r,
                                                              const float* __restrict__ w, float* __restrict__ dr,
                                                              int E, int K, MaceRadial m) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const float x = r[e];
  float en, den;
  m.env(x, en, den);
  const float inv = 1.f / x;
  float acc = 0.f;
  for (int k = 0; k < K; ++k) {
    float s, c;
    sincosf(w[k] * x, &s, &c);
    const float b = s * inv;                        // sin(w r)/r
    const float db = (w[k] * c - b) * inv;          // d/dr sin(w r)/r
    acc += g[(int64_t)e * K + k] * (db * en + b * den);
  }
  dr[e] = m.pref * acc;
}

at::Tensor mace_radial_fwd(const at::Tensor& r_, const at::Tensor& w, double rc, double p) {
  HY_CHECK_CUDA(r_);
  auto r = r_.contiguous();
  HY_CHECK_F32(r);
  HY_CHECK_F32(w);
  const int E = (int)r.numel(), K = (int)w.numel();
  auto out = at::empty({E, K}, r.options());
  MaceRadial m{(float)std::sqrt(2.0 / rc), (float)rc, (float)p};
  if ((int64_t)E * K > 0)
    mace_radial_fwd_kernel<<<ceil_div((int64_t)E * K, 256), 256, 0, stream()>>>(
        r.data_ptr<float>(), w.contiguous().data_ptr<float>(), out.data_ptr<float>(), E, K, m);
  return out;
}

at::Tensor mace_radial_bwd(const at::Tensor& g_, const at::Tensor& r_, const at::Tensor& w, double rc, double p) {
  HY_CHECK_CUDA(g_);
  auto g = g_.contiguous(), r = r_.contiguous();
  HY_CHECK_F32(g);
  HY_CHECK_F32(r);
  const int E = (int)r.numel(), K = (int)w.numel();
  HY_CHECK(g.numel() == (int64_t)E * K, "mace_radial_bwd: gradient shape");
  auto dr = at::empty_like(r);
  MaceRadial m{(float)std::sqrt(2.0 / rc), (float)rc, (float)p};
  if (E > 0)
    mace_radial_bwd_kernel<<<ceil_div((int64_t)E, 256), 256, 0, stream()>>>(
        g.data_ptr<float>(), r.data_ptr<float>(), w.contiguous().data_ptr<float>(), dr.data_ptr<float>(), E, K, m);
  return dr;
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("mace_radial_fwd(Tensor r, Tensor w, float rc, float p) -> Tensor");
  m.def("mace_radial_bwd(Tensor g, Tensor r, Tensor w, float rc, float p) -> Tensor");
  m.def(
      "radial_fwd(Tensor dist, Tensor freq, Tensor Wemb, Tensor bemb, Tensor Wlin, float cutoff, int exponent) -> "
      "(Tensor, Tensor)");
  m.def(
      "radial_fwd_multi(Tensor? dist, Tensor freq, Tensor[] Wemb, Tensor[] bemb, Tensor[] Wlin, float cutoff, "
      "int exponent, bool want_dfreq, Tensor? pos=None, Tensor? dst=None, Tensor? src=None, Tensor? shifts=None) "
      "-> Tensor[]");
  m.def(
      "radial_bwd(Tensor[] dR, Tensor[] dG, Tensor R, Tensor dist, Tensor freq, Tensor Wemb, Tensor Wlin, float cutoff, "
      "int exponent) -> (Tensor, Tensor, Tensor, Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("radial_fwd", hy::radial_fwd);
  m.impl("radial_bwd", hy::radial_bwd);
  m.impl("radial_fwd_multi", hy::radial_fwd_multi);
  m.impl("mace_radial_fwd", hy::mace_radial_fwd);
  m.impl("mace_radial_bwd", hy::mace_radial_bwd);
}
