// EGNN (E_GCL) edge / node kernels for the bf16 wide-layer path (SC25 EGNN-866,
// reference hydragnn/models/EGCLStack.py:175-289).  The GEMMs run on the MFMA engine
// (bgemm.hip); these kernels are the memory-bound pieces between them, each one pass:
//
//   gather_fwd : h1[e] = relu(AB[src_e, :H] + AB[dst_e, Hp:Hp+H] + |d_e| w_r + sum_j ea_ej w_j + b1)
//                (the edge_mlp[0] Linear over cat[x_row, x_col, radial, edge_attr], with its
//                x blocks evaluated at node level), edge geometry d_e = pos[dst]-pos[src],
//                cd_e = d_e / (|d_e| + 1), and the bf16 per-edge scalar row [|d|, ea.., 1]
//   csr_rows   : agg[n] = sum_{e: src_e = n} m[e] forward; dAB = by-source | by-destination
//                sums of dh1 backward (bf16 rows, fp32 sums, one block per (node, part))
//   pos_fwd    : pos'[n] = pos[n] + cw * mean_{e: src_e = n} clamp(cd_e tanh(s_e), +-100)
//   coord_bwd  : d(pos') -> ds_e, dcd_e; dc1 = ds_e wc2 * relu'(c1) (bf16), dwc2 partials
//   pos_bwd    : dpos[n] = dpos'[n] + sum_{dst_e = n} dvec_e - sum_{src_e = n} dvec_e, the
//                per-edge dvec_e rebuilt inline from geo, dcd and dr_e = d loss / d|d_e|
//                (dr comes from the row-dot epilogue of the dh1 GEMM, bgemm.hip)
//
// Edge-row kernels: one wave per edge row; each lane owns 4 consecutive channels (8-byte
// bf16 / 16-byte fp32 accesses), looping over the padded width Hp in steps of 256.  Column
// reductions over edges go to per-block partial rows reduced by bg_slab_reduce (no
// atomics).  Edges are stored sorted by destination (dst CSR is the identity order);
// the source CSR carries a permutation.
#include "common.h"

namespace hy {
namespace eg {

typedef __bf16 bf2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  bf2v v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ float lo_bf(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_bf(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ float4 ld_bf4(const uint16_t* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return make_float4(lo_bf(u.x), hi_bf(u.x), lo_bf(u.y), hi_bf(u.y));
}
__device__ __forceinline__ void st_bf4(uint16_t* p, float a, float b, float c, float d) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack2(a, b), pack2(c, d));
}

constexpr int MAXS = 4;  // per-edge scalar features: |d| + up to 3 edge attributes

struct GatherFwd {
  const float* AB;  // [N, 2Hp]
  const int* src;   // [E]
  const int* dst;   // [E]
  const float* pos; // [N, 3]
  const float* ea;  // [E, nea] or null
  const float* W0;  // edge_mlp[0].weight [H, ld0]; scalar columns at c0 .. c0 + nea
  const float* b1;  // [H]
  int ld0, c0, nea, H, Hp, E;
  uint16_t* h1;     // [E, Hp] (ones lane at H)
  float* geo;       // [E, 4]: cd.xyz, |d|
  uint16_t* sc;     // [E, 128]: |d|, ea..., 1 at 1 + nea
};

constexpr int GE = 32;  // edges per block (8 per wave) of the gather kernel

// One wave per edge row, 32 edges per block: the radial / edge-attribute weight columns
// and the bias are staged once per block in LDS (the strided W0 columns are never read per
// element); each lane owns channels 4l + 256 t (t < 4), all 8 row loads issued together.
__global__ __launch_bounds__(256) void gather_fwd_kernel(GatherFwd p) {
  __shared__ float wl[MAXS + 1][1024];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int k = threadIdx.x; k < p.Hp; k += 256) {
    const bool v = k < p.H;
    wl[MAXS][k] = v ? p.b1[k] : 0.f;
    for (int j = 0; j <= p.nea; ++j) wl[j][k] = v ? p.W0[(int64_t)k * p.ld0 + p.c0 + j] : 0.f;
  }
  __syncthreads();
  for (int i = 0; i < GE / 4; ++i) {
    const int e = blockIdx.x * GE + w * (GE / 4) + i;
    if (e >= p.E) break;
    const int s = p.src[e], d = p.dst[e];
    const float vx = p.pos[d * 3] - p.pos[s * 3], vy = p.pos[d * 3 + 1] - p.pos[s * 3 + 1],
                vz = p.pos[d * 3 + 2] - p.pos[s * 3 + 2];
    const float L = sqrtf(vx * vx + vy * vy + vz * vz);
    float sv[MAXS] = {L, 0.f, 0.f, 0.f};
    for (int j = 0; j < p.nea; ++j) sv[1 + j] = p.ea[(int64_t)e * p.nea + j];
    if (lane == 0) {
      const float inv = 1.f / (L + 1.f);
      *reinterpret_cast<float4*>(p.geo + (int64_t)e * 4) = make_float4(vx * inv, vy * inv, vz * inv, L);
    }
    if (lane < 32) {  // scalar row: 4 bf16 per lane over 128 columns
      float t[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = lane * 4 + r;
        t[r] = c <= p.nea ? sv[c < MAXS ? c : 0] : (c == p.nea + 1 ? 1.f : 0.f);
      }
      st_bf4(p.sc + (int64_t)e * 128 + lane * 4, t[0], t[1], t[2], t[3]);
    }
    const float* ar = p.AB + (int64_t)s * 2 * p.Hp;
    const float* br = p.AB + (int64_t)d * 2 * p.Hp + p.Hp;
    uint16_t* out = p.h1 + (int64_t)e * p.Hp;
    float4 av[4], bv[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int k = lane * 4 + t * 256;
      if (k < p.Hp) {  // AB pad columns are zero (padded weight images)
        av[t] = *reinterpret_cast<const float4*>(ar + k);
        bv[t] = *reinterpret_cast<const float4*>(br + k);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int k = lane * 4 + t * 256;
      if (k >= p.Hp) continue;
      float v[4] = {av[t].x + bv[t].x, av[t].y + bv[t].y, av[t].z + bv[t].z, av[t].w + bv[t].w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kk = k + r;
        float z = v[r] + wl[MAXS][kk] + sv[0] * wl[0][kk];
        for (int j = 1; j <= p.nea; ++j) z += sv[j] * wl[j][kk];
        v[r] = kk < p.H ? fmaxf(z, 0.f) : (kk == p.H ? 1.f : 0.f);
      }
      st_bf4(out + k, v[0], v[1], v[2], v[3]);
    }
  }
}

constexpr int EPB = 32;  // edges per block (8 per wave) for the column-partial kernels

struct CoordBwd {
  const float* dpos;  // [N, 3] gradient of pos'
  const int* src;     // [E]
  const int* srp;     // [N + 1]
  const float* geo;   // [E, 4]
  const float* s;     // [E]
  const uint16_t* c1; // [E, Hp]
  const float* wc2;   // [H]
  float cw;
  int E, H, Hp;
  uint16_t* dc1;      // [E, Hp]
  float* dcd;         // [E, 3]
  float* part;        // [nblk, Hp]: sum_e ds_e c1[e]
};

__global__ __launch_bounds__(256) void coord_bwd_kernel(CoordBwd p) {
  __shared__ float red[4][1024];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int e0 = blockIdx.x * EPB + w * (EPB / 4);
  float pa[4][4];
#pragma unroll
  for (int it = 0; it < 4; ++it)
#pragma unroll
    for (int r = 0; r < 4; ++r) pa[it][r] = 0.f;
  for (int i = 0; i < EPB / 4; ++i) {
    const int e = e0 + i;
    if (e >= p.E) break;
    const int n = p.src[e];
    const int cnt = p.srp[n + 1] - p.srp[n];
    const float sc = p.cw / (float)(cnt > 0 ? cnt : 1);
    const float4 g = *reinterpret_cast<const float4*>(p.geo + (int64_t)e * 4);
    const float t = tanhf(p.s[e]);
    const float cd[3] = {g.x, g.y, g.z};
    float dt = 0.f, dcd[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float u = cd[c] * t;
      const float dtr = (u >= -100.f && u <= 100.f) ? sc * p.dpos[n * 3 + c] : 0.f;
      dt += dtr * cd[c];
      dcd[c] = dtr * t;
    }
    const float ds = dt * (1.f - t * t);
    if (lane < 3) p.dcd[(int64_t)e * 3 + lane] = dcd[lane];
    const uint16_t* crow = p.c1 + (int64_t)e * p.Hp;
    uint16_t* orow = p.dc1 + (int64_t)e * p.Hp;
    float4 cr[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {  // the whole row in flight at once
      const int k = lane * 4 + it * 256;
      if (k < p.Hp) cr[it] = ld_bf4(crow + k);
    }
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int k = lane * 4 + it * 256;
      if (k >= p.Hp) break;
      const float4 c = cr[it];
      float o[4];
      const float cv[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float wv = (k + r < p.H) ? p.wc2[k + r] : 0.f;
        o[r] = cv[r] > 0.f ? ds * wv : 0.f;
        pa[it][r] += ds * cv[r];
      }
      st_bf4(orow + k, o[0], o[1], o[2], o[3]);
    }
  }
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int k = lane * 4 + it * 256;
    if (k < 1024) {
#pragma unroll
      for (int r = 0; r < 4; ++r) red[w][k + r] = pa[it][r];
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < p.Hp; k += 256)
    p.part[(int64_t)blockIdx.x * p.Hp + k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
}

// out[e] = g[idx[e], :H] * (gate[e] > 0) as padded bf16 (the non-equivariant layer's
// dZ2 = dagg[src] * relu'(m): no coordinate GEMM to carry the gather in its epilogue)
__global__ __launch_bounds__(256) void gather_gate_kernel(const float* __restrict__ g, int ldg,
                                                          const int* __restrict__ idx,
                                                          const uint16_t* __restrict__ gate, int E, int H, int Hp,
                                                          uint16_t* __restrict__ out) {
  const int e = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (e >= E) return;
  const float* row = g + (int64_t)idx[e] * ldg;
  for (int k = lane * 4; k < Hp; k += 256) {
    const float4 q = ld_bf4(gate + (int64_t)e * Hp + k);
    const float qv[4] = {q.x, q.y, q.z, q.w};
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (k + r < H && qv[r] > 0.f) ? row[k + r] : 0.f;
    st_bf4(out + (int64_t)e * Hp + k, v[0], v[1], v[2], v[3]);
  }
}

// ---------------------------------------------------------------- CSR row sums (bf16 rows)
// out[n, off_p + k] = sum_{i in segment n of CSR p} X[perm_p ? perm_p[i] : i, k]; one 256-thread
// block per (node, part), wave q owns channels [256 q, 256 q + 256) (4 per lane), 4 rows in
// flight: ~16 waves per SIMD on the EGNN shapes instead of one wave per node.
struct CsrParts {
  const uint16_t* X;
  int Hp;
  const int* rp[2];
  const int* perm[2];
  int off[2];
  uint16_t* out;
  int ldo;
};

__global__ __launch_bounds__(256) void csr_rows_kernel(CsrParts p) {
  const int n = blockIdx.x, part = blockIdx.y, lane = threadIdx.x & 63;
  const int k = (threadIdx.x >> 6) * 256 + lane * 4;
  if (k >= p.Hp) return;
  const int* rp = p.rp[part];
  const int* pm = p.perm[part];
  const int b = rp[n], eN = rp[n + 1];
  float4 a0 = f4zero(), a1 = f4zero();
  int i = b;
  for (; i + 3 < eN; i += 4) {
    const int e0 = pm ? pm[i] : i, e1 = pm ? pm[i + 1] : i + 1, e2 = pm ? pm[i + 2] : i + 2,
              e3 = pm ? pm[i + 3] : i + 3;
    const float4 x0 = ld_bf4(p.X + (int64_t)e0 * p.Hp + k), x1 = ld_bf4(p.X + (int64_t)e1 * p.Hp + k);
    const float4 x2 = ld_bf4(p.X + (int64_t)e2 * p.Hp + k), x3 = ld_bf4(p.X + (int64_t)e3 * p.Hp + k);
    a0 = f4add(a0, f4add(x0, x1));
    a1 = f4add(a1, f4add(x2, x3));
  }
  for (; i < eN; ++i) a0 = f4add(a0, ld_bf4(p.X + (int64_t)(pm ? pm[i] : i) * p.Hp + k));
  const float4 a = f4add(a0, a1);
  st_bf4(p.out + (int64_t)n * p.ldo + p.off[part] + k, a.x, a.y, a.z, a.w);
}

// pos'[n] = pos[n] + cw * mean_{e: src_e = n} clamp(cd_e tanh(s_e), +-100)   (wave per node,
// lanes stride the node's edges)
__global__ __launch_bounds__(256) void pos_fwd_kernel(const float* __restrict__ pos, const float* __restrict__ geo,
                                                      const float* __restrict__ s, const int* __restrict__ srp,
                                                      const int* __restrict__ sperm, float cw, int N,
                                                      float* __restrict__ pos_out) {
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (n >= N) return;
  const int b = srp[n], eN = srp[n + 1];
  float a[3] = {0.f, 0.f, 0.f};
  for (int i = b + lane; i < eN; i += 64) {
    const int e = sperm ? sperm[i] : i;
    const float4 g = *reinterpret_cast<const float4*>(geo + (int64_t)e * 4);
    const float t = tanhf(s[e]);
    a[0] += fminf(fmaxf(g.x * t, -100.f), 100.f);
    a[1] += fminf(fmaxf(g.y * t, -100.f), 100.f);
    a[2] += fminf(fmaxf(g.z * t, -100.f), 100.f);
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) a[c] = wave_sum(a[c]);
  if (lane < 3) {
    const int cnt = eN - b;
    const float v = lane == 0 ? a[0] : (lane == 1 ? a[1] : a[2]);
    pos_out[n * 3 + lane] = pos[n * 3 + lane] + cw * v / (float)(cnt > 0 ? cnt : 1);
  }
}

// per-edge position gradient d loss / d vec_e (vec = pos[dst] - pos[src]) from the radial
// gradient dr_e (|vec| feeds edge_mlp[0]) and dcd_e (normalised difference of the update)
__device__ __forceinline__ float dvec_c(const float* geo, const float* dr, const float* dcd, int64_t e, int c) {
  const float4 g = *reinterpret_cast<const float4*>(geo + e * 4);
  const float L = g.w, s1 = L + 1.f;
  if (!(L > 0.f)) return 0.f;
  const float d[3] = {g.x * s1, g.y * s1, g.z * s1};
  float v = dr[e] * d[c] / L;
  if (dcd) {
    const float q0 = dcd[e * 3], q1 = dcd[e * 3 + 1], q2 = dcd[e * 3 + 2];
    const float dot = q0 * d[0] + q1 * d[1] + q2 * d[2];
    const float qc = c == 0 ? q0 : (c == 1 ? q1 : q2);
    v += qc / s1 - d[c] * dot / (L * s1 * s1);
  }
  return v;
}

__global__ __launch_bounds__(256) void pos_bwd_kernel(const float* __restrict__ dpos_out,
                                                      const float* __restrict__ geo, const float* __restrict__ dr,
                                                      const float* __restrict__ dcd, const int* __restrict__ srp,
                                                      const int* __restrict__ sperm, const int* __restrict__ drp,
                                                      int N, float* __restrict__ dpos) {
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (n >= N) return;
  float a[3] = {0.f, 0.f, 0.f};
  for (int e = drp[n] + lane; e < drp[n + 1]; e += 64)
#pragma unroll
    for (int c = 0; c < 3; ++c) a[c] += dvec_c(geo, dr, dcd, e, c);
  for (int i = srp[n] + lane; i < srp[n + 1]; i += 64) {
    const int e = sperm ? sperm[i] : i;
#pragma unroll
    for (int c = 0; c < 3; ++c) a[c] -= dvec_c(geo, dr, dcd, e, c);
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) a[c] = wave_sum(a[c]);
  if (lane < 3) {
    const float v = lane == 0 ? a[0] : (lane == 1 ? a[1] : a[2]);
    dpos[n * 3 + lane] = v + (dpos_out ? dpos_out[n * 3 + lane] : 0.f);
  }
}

}  // namespace eg

using namespace eg;

static const int* iptr(const c10::optional<at::Tensor>& t) { return t.has_value() ? t->data_ptr<int>() : nullptr; }
static const uint16_t* cbf(const at::Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
static uint16_t* wbf(const at::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

static void chk_rows(const at::Tensor& t, int64_t rows, int64_t cols, at::ScalarType dt, const char* name) {
  HY_CHECK(t.is_cuda() && t.scalar_type() == dt && t.is_contiguous() && t.dim() == 2 && t.size(0) == rows &&
               t.size(1) == cols,
           name, ": expected contiguous [", rows, ", ", cols, "]");
}

// returns nothing; writes h1, geo, sc
void egnn_gather_fwd(const at::Tensor& AB, const at::Tensor& src, const at::Tensor& dst, const at::Tensor& pos,
                     const c10::optional<at::Tensor>& ea, const at::Tensor& W0, int64_t c0, const at::Tensor& b1,
                     const at::Tensor& h1, const at::Tensor& geo, const at::Tensor& sc) {
  const int64_t E = src.numel(), N = pos.size(0), Hp = h1.size(1), H = b1.numel();
  HY_CHECK(H < Hp && Hp % 256 != 1, "egnn_gather_fwd: H < Hp");
  chk_rows(AB, N, 2 * Hp, at::kFloat, "AB");
  HY_CHECK_I32(src);
  HY_CHECK_I32(dst);
  HY_CHECK(dst.numel() == E, "egnn_gather_fwd: dst length");
  chk_rows(pos, N, 3, at::kFloat, "pos");
  chk_rows(h1, E, Hp, at::kBFloat16, "h1");
  chk_rows(geo, E, 4, at::kFloat, "geo");
  chk_rows(sc, E, 128, at::kBFloat16, "sc");
  HY_CHECK(W0.scalar_type() == at::kFloat && W0.stride(1) == 1 && W0.size(0) == H, "egnn_gather_fwd: W0");
  GatherFwd p{};
  p.AB = AB.data_ptr<float>();
  p.src = src.data_ptr<int>();
  p.dst = dst.data_ptr<int>();
  p.pos = pos.data_ptr<float>();
  if (ea.has_value() && ea->numel()) {
    HY_CHECK(ea->scalar_type() == at::kFloat && ea->is_contiguous() && ea->size(0) == E && ea->dim() == 2 &&
                 ea->size(1) < MAXS,
             "egnn_gather_fwd: edge attributes");
    p.ea = ea->data_ptr<float>();
    p.nea = (int)ea->size(1);
  }
  HY_CHECK(c0 + 1 + p.nea <= W0.size(1), "egnn_gather_fwd: W0 scalar columns");
  p.W0 = W0.data_ptr<float>();
  p.ld0 = (int)W0.stride(0);
  p.c0 = (int)c0;
  p.b1 = b1.data_ptr<float>();
  p.H = (int)H;
  p.Hp = (int)Hp;
  p.E = (int)E;
  p.h1 = wbf(h1);
  p.geo = geo.data_ptr<float>();
  p.sc = wbf(sc);
  HY_CHECK(Hp <= 1024, "egnn_gather_fwd: Hp <= 1024");
  if (E) gather_fwd_kernel<<<ceil_div(E, GE), 256, 0, stream()>>>(p);
}

// returns the number of partial rows written to part ([nblk, Hp])
int64_t egnn_coord_bwd(const at::Tensor& dpos, const at::Tensor& src, const at::Tensor& srp, const at::Tensor& geo,
                       const at::Tensor& s, const at::Tensor& c1, const at::Tensor& wc2, double cw, const at::Tensor& dc1,
                       const at::Tensor& dcd, const at::Tensor& part) {
  const int64_t E = c1.size(0), Hp = c1.size(1), H = wc2.numel(), N = dpos.size(0);
  HY_CHECK(Hp <= 1024, "egnn_coord_bwd: Hp <= 1024");
  chk_rows(dpos, N, 3, at::kFloat, "dpos");
  chk_rows(geo, E, 4, at::kFloat, "geo");
  chk_rows(dc1, E, Hp, at::kBFloat16, "dc1");
  chk_rows(dcd, E, 3, at::kFloat, "dcd");
  HY_CHECK(s.numel() == E && src.numel() == E && srp.numel() == N + 1, "egnn_coord_bwd: lengths");
  const int64_t nblk = (E + EPB - 1) / EPB;
  HY_CHECK(part.scalar_type() == at::kFloat && part.numel() >= nblk * Hp, "egnn_coord_bwd: part");
  CoordBwd p{};
  p.dpos = dpos.data_ptr<float>();
  p.src = src.data_ptr<int>();
  p.srp = srp.data_ptr<int>();
  p.geo = geo.data_ptr<float>();
  p.s = s.data_ptr<float>();
  p.c1 = cbf(c1);
  p.wc2 = wc2.data_ptr<float>();
  p.cw = (float)cw;
  p.E = (int)E;
  p.H = (int)H;
  p.Hp = (int)Hp;
  p.dc1 = wbf(dc1);
  p.dcd = dcd.data_ptr<float>();
  p.part = part.data_ptr<float>();
  if (E) coord_bwd_kernel<<<(int)nblk, 256, 0, stream()>>>(p);
  return nblk;
}

void egnn_gather_gate(const at::Tensor& g, const at::Tensor& idx, const at::Tensor& gate, int64_t H,
                      const at::Tensor& out) {
  const int64_t E = gate.size(0), Hp = gate.size(1);
  chk_rows(gate, E, Hp, at::kBFloat16, "gate");
  chk_rows(out, E, Hp, at::kBFloat16, "out");
  HY_CHECK(g.scalar_type() == at::kFloat && g.dim() == 2 && g.stride(1) == 1 && g.size(1) >= H, "egnn_gather_gate: g");
  HY_CHECK_I32(idx);
  HY_CHECK(idx.numel() == E, "egnn_gather_gate: idx length");
  if (E)
    gather_gate_kernel<<<ceil_div(E, 4), 256, 0, stream()>>>(g.data_ptr<float>(), (int)g.stride(0),
                                                             idx.data_ptr<int>(), cbf(gate), (int)E, (int)H, (int)Hp,
                                                             wbf(out));
}

// CSR row sums of bf16 rows into column blocks of out (one or two CSR parts)
void egnn_csr_rows(const at::Tensor& X, const at::Tensor& rp0, const c10::optional<at::Tensor>& perm0, int64_t off0,
                   const c10::optional<at::Tensor>& rp1, const c10::optional<at::Tensor>& perm1, int64_t off1,
                   const at::Tensor& out) {
  const int64_t E = X.size(0), Hp = X.size(1), N = rp0.numel() - 1;
  chk_rows(X, E, Hp, at::kBFloat16, "X");
  HY_CHECK(Hp % 4 == 0 && Hp <= 1024, "egnn_csr_rows: Hp % 4 == 0, <= 1024");
  HY_CHECK(out.scalar_type() == at::kBFloat16 && out.dim() == 2 && out.stride(1) == 1 && out.size(0) == N &&
               out.size(1) >= off0 + Hp && out.stride(0) % 4 == 0,
           "egnn_csr_rows: out");
  HY_CHECK_I32(rp0);
  HY_CHECK(!perm0.has_value() || perm0->numel() == E, "egnn_csr_rows: perm0 length");
  CsrParts p{};
  p.X = cbf(X);
  p.Hp = (int)Hp;
  p.rp[0] = rp0.data_ptr<int>();
  p.perm[0] = iptr(perm0);
  p.off[0] = (int)off0;
  int parts = 1;
  if (rp1.has_value()) {
    HY_CHECK_I32(*rp1);
    HY_CHECK(rp1->numel() == N + 1 && out.size(1) >= off1 + Hp && (!perm1.has_value() || perm1->numel() == E),
             "egnn_csr_rows: second part");
    p.rp[1] = rp1->data_ptr<int>();
    p.perm[1] = iptr(perm1);
    p.off[1] = (int)off1;
    parts = 2;
  }
  p.out = wbf(out);
  p.ldo = (int)out.stride(0);
  if (N) csr_rows_kernel<<<dim3((unsigned)N, parts), 256, 0, stream()>>>(p);
}

void egnn_pos_fwd(const at::Tensor& pos, const at::Tensor& geo, const at::Tensor& s, const at::Tensor& srp,
                  const c10::optional<at::Tensor>& sperm, double cw, const at::Tensor& pos_out) {
  const int64_t N = pos.size(0);
  chk_rows(pos, N, 3, at::kFloat, "pos");
  chk_rows(pos_out, N, 3, at::kFloat, "pos_out");
  chk_rows(geo, s.numel(), 4, at::kFloat, "geo");
  HY_CHECK_I32(srp);
  HY_CHECK(srp.numel() == N + 1 && s.scalar_type() == at::kFloat, "egnn_pos_fwd: srp / s");
  if (N)
    pos_fwd_kernel<<<ceil_div(N, 4), 256, 0, stream()>>>(pos.data_ptr<float>(), geo.data_ptr<float>(),
                                                               s.data_ptr<float>(), srp.data_ptr<int>(), iptr(sperm),
                                                               (float)cw, (int)N, pos_out.data_ptr<float>());
}

void egnn_pos_bwd(const c10::optional<at::Tensor>& dpos_out, const at::Tensor& geo, const at::Tensor& dr,
                   const c10::optional<at::Tensor>& dcd, const at::Tensor& srp, const c10::optional<at::Tensor>& sperm,
                   const at::Tensor& drp, const at::Tensor& dpos) {
  const int64_t N = srp.numel() - 1;
  chk_rows(dpos, N, 3, at::kFloat, "dpos");
  HY_CHECK(dr.scalar_type() == at::kFloat && dr.numel() == geo.size(0), "egnn_pos_bwd: dr [E]");
  chk_rows(geo, dr.numel(), 4, at::kFloat, "geo");
  HY_CHECK_I32(srp);
  HY_CHECK_I32(drp);
  HY_CHECK(drp.numel() == N + 1, "egnn_pos_bwd: drp");
  if (dcd.has_value()) chk_rows(*dcd, dr.numel(), 3, at::kFloat, "dcd");
  if (dpos_out.has_value()) chk_rows(*dpos_out, N, 3, at::kFloat, "dpos_out");
  if (N)
    pos_bwd_kernel<<<ceil_div(N, 4), 256, 0, stream()>>>(
        dpos_out.has_value() ? dpos_out->data_ptr<float>() : nullptr, geo.data_ptr<float>(), dr.data_ptr<float>(),
        dcd.has_value() ? dcd->data_ptr<float>() : nullptr, srp.data_ptr<int>(), iptr(sperm), drp.data_ptr<int>(),
        (int)N, dpos.data_ptr<float>());
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def(
      "egnn_gather_fwd(Tensor AB, Tensor src, Tensor dst, Tensor pos, Tensor? ea, Tensor W0, int c0, Tensor b1, "
      "Tensor h1, Tensor geo, Tensor sc) -> ()");
  m.def(
      "egnn_coord_bwd(Tensor dpos, Tensor src, Tensor srp, Tensor geo, Tensor s, Tensor c1, Tensor wc2, float cw, "
      "Tensor dc1, Tensor dcd, Tensor part) -> int");
  m.def("egnn_gather_gate(Tensor g, Tensor idx, Tensor gate, int H, Tensor out) -> ()");
  m.def(
      "egnn_csr_rows(Tensor X, Tensor rp0, Tensor? perm0, int off0, Tensor? rp1, Tensor? perm1, int off1, Tensor out) "
      "-> ()");
  m.def("egnn_pos_fwd(Tensor pos, Tensor geo, Tensor s, Tensor srp, Tensor? sperm, float cw, Tensor pos_out) -> ()");
  m.def(
      "egnn_pos_bwd(Tensor? dpos_out, Tensor geo, Tensor dr, Tensor? dcd, Tensor srp, Tensor? sperm, Tensor drp, "
      "Tensor dpos) -> ()");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("egnn_gather_fwd", hy::egnn_gather_fwd);
  m.impl("egnn_coord_bwd", hy::egnn_coord_bwd);
  m.impl("egnn_gather_gate", hy::egnn_gather_gate);
  m.impl("egnn_csr_rows", hy::egnn_csr_rows);
  m.impl("egnn_pos_fwd", hy::egnn_pos_fwd);
  m.impl("egnn_pos_bwd", hy::egnn_pos_bwd);
}
