// PAINN force-training op families for gfx950 (reference hydragnn/models/PAINNStack.py:
// 194-263 message, :228-236 edge terms; Base.py:582-636 forces = -dE/dpos twice
// differentiated).  Host side and derivations: ops/painn_force.py (the torch twins are the
// same formulas, gradgradchecked in fp64).
//
// Geometry  (edge-parallel forward; node-parallel backward / double backward):
//   vec = pos[dst] - pos[src] (+ shift), L = |vec|
//   basis[e] = [sin(k a L) / L * cut(L) (k = 1..R) | cut(L)],  cut = (cos(a L) + 1) / 2 [L < c]
//   unit[e]  = vec / ((L + eps) L)
// Message   (one wave per node, one lane per feature; CSR views, no atomics):
//   w_e = W basis_e[:R] + b basis_e[R]  (3F),  o = w_e * phi[dst]
//   s1[n] = s[n] + sum_{src e = n} o_s,  v1[n] = v[n] + sum (v[dst] o_v + o_e unit_e)
// The backward kernels walk the dst-CSR (gathers become sums over incoming edges) and
// the double backward adds one src-CSR pass.  Weight gradients of the radial filter are
// per-workgroup partials reduced in a fixed order (deterministic).
#include "common.h"

namespace hy {
namespace pf {

constexpr int kMaxR = 32;

struct Csr {
  const int* ptr;   // [N+1]
  const int* perm;  // position -> edge id, or null (edges already in this order)
};

__device__ __forceinline__ int edge_at(const Csr& c, int p) { return c.perm ? c.perm[p] : p; }

// ------------------------------------------------------------------------ geometry
struct Geo {
  const float* pos;
  const float* shift;  // [E, 3] or null
  const int* dst;
  const int* src;
  int R;
  float a, cutoff, eps;
};

__device__ __forceinline__ void edge_vec(const Geo& g, int e, float& x, float& y, float& z) {
  const int d = g.dst[e], s = g.src[e];
  x = g.pos[3 * d] - g.pos[3 * s];
  y = g.pos[3 * d + 1] - g.pos[3 * s + 1];
  z = g.pos[3 * d + 2] - g.pos[3 * s + 2];
  if (g.shift) {
    x += g.shift[3 * e];
    y += g.shift[3 * e + 1];
    z += g.shift[3 * e + 2];
  }
}

// q(L) = 1 / ((L + eps) L) and its first two derivatives
__device__ __forceinline__ void qfun(float L, float eps, float& q, float& q1, float& q2) {
  const float D = L * L + eps * L, dD = 2.f * L + eps;
  q = 1.f / D;
  q1 = -dD * q * q;
  q2 = (-2.f * D + 2.f * dD * dD) * q * q * q;
}

struct Cut {
  float c0, c1, c2;
};
__device__ __forceinline__ Cut cutf(const Geo& g, float L) {
  const bool in = L < g.cutoff;
  float sa, ca;
  sincosf(g.a * L, &sa, &ca);
  return Cut{in ? 0.5f * (ca + 1.f) : 0.f, in ? -0.5f * g.a * sa : 0.f, in ? -0.5f * g.a * g.a * ca : 0.f};
}

// basis component k (k < R: sinc * cut, k == R: cut) and its derivatives w.r.t. L
__device__ __forceinline__ void basis_k(const Geo& g, const Cut& C, int k, float L, float iL, float& f, float& f1,
                                        float& f2, int order) {
  const float cut = C.c0, cut1 = C.c1, cut2 = C.c2;
  if (k == g.R) {
    f = cut;
    f1 = cut1;
    f2 = cut2;
    return;
  }
  const float w = (float)(k + 1) * g.a;
  float sn, cs;
  sincosf(w * L, &sn, &cs);
  const float gg = sn * iL;
  f = gg * cut;
  if (order < 1) return;
  const float g1 = w * cs * iL - sn * iL * iL;
  f1 = g1 * cut + gg * cut1;
  if (order < 2) return;
  const float g2 = -w * w * sn * iL - 2.f * w * cs * iL * iL + 2.f * sn * iL * iL * iL;
  f2 = g2 * cut + 2.f * g1 * cut1 + gg * cut2;
}

__global__ void __launch_bounds__(256) geom_fwd_kernel(Geo g, int E, float* __restrict__ basis,
                                                       float* __restrict__ unit) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= E) return;
  float x, y, z;
  edge_vec(g, e, x, y, z);
  const float L = sqrtf(x * x + y * y + z * z), iL = 1.f / L;
  const Cut C = cutf(g, L);
  float f, f1, f2;
  for (int k = 0; k <= g.R; ++k) {
    basis_k(g, C, k, L, iL, f, f1, f2, 0);
    basis[(int64_t)e * (g.R + 1) + k] = f;
  }
  float q, q1, q2;
  qfun(L, g.eps, q, q1, q2);
  unit[3 * e] = x * q;
  unit[3 * e + 1] = y * q;
  unit[3 * e + 2] = z * q;
}

// per-edge gradient w.r.t. vec of  gB . basis + gU . unit
__device__ __forceinline__ void geom_gvec(const Geo& g, int e, const float* gB, const float* gU, float& ox, float& oy,
                                          float& oz) {
  float x, y, z;
  edge_vec(g, e, x, y, z);
  const float L = sqrtf(x * x + y * y + z * z), iL = 1.f / L;
  const Cut C = cutf(g, L);
  float A = 0.f, f, f1, f2;
  for (int k = 0; k <= g.R; ++k) {
    basis_k(g, C, k, L, iL, f, f1, f2, 1);
    A += gB[(int64_t)e * (g.R + 1) + k] * f1;
  }
  float q, q1, q2;
  qfun(L, g.eps, q, q1, q2);
  const float ux = gU[3 * e], uy = gU[3 * e + 1], uz = gU[3 * e + 2];
  const float u = ux * x + uy * y + uz * z;
  const float s = (A + u * q1) * iL;
  ox = s * x + ux * q;
  oy = s * y + uy * q;
  oz = s * z + uz * q;
}

// one wave per node: lanes over incoming (+) and outgoing (-) edges
__global__ void __launch_bounds__(256) geom_vjp_kernel(Geo g, Csr din, Csr sout, int N, const float* __restrict__ gB,
                                                       const float* __restrict__ gU, float* __restrict__ gpos) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= N) return;
  float ax = 0.f, ay = 0.f, az = 0.f, x, y, z;
  for (int p = din.ptr[n] + lane; p < din.ptr[n + 1]; p += 64) {
    geom_gvec(g, edge_at(din, p), gB, gU, x, y, z);
    ax += x;
    ay += y;
    az += z;
  }
  for (int p = sout.ptr[n] + lane; p < sout.ptr[n + 1]; p += 64) {
    geom_gvec(g, edge_at(sout, p), gB, gU, x, y, z);
    ax -= x;
    ay -= y;
    az -= z;
  }
  ax = wave_sum(ax);
  ay = wave_sum(ay);
  az = wave_sum(az);
  if (lane == 0) {
    gpos[3 * n] = ax;
    gpos[3 * n + 1] = ay;
    gpos[3 * n + 2] = az;
  }
}

// second-order term of one edge: d/dvec [hv . gvec(vec)]; optionally the per-edge JVP
// outputs hB = f'(L) t / L, hU = q hv + vec q' t / L
__device__ __forceinline__ void geom_edge2(const Geo& g, int e, const float* gB, const float* gU, const float* hpos,
                                           float* hB, float* hU, bool pos_term, float& ox, float& oy, float& oz) {
  float x, y, z;
  edge_vec(g, e, x, y, z);
  const int d = g.dst[e], s = g.src[e];
  const float hx = hpos[3 * d] - hpos[3 * s], hy = hpos[3 * d + 1] - hpos[3 * s + 1],
              hz = hpos[3 * d + 2] - hpos[3 * s + 2];
  const float L = sqrtf(x * x + y * y + z * z), iL = 1.f / L;
  const float t = x * hx + y * hy + z * hz;
  float q, q1, q2;
  qfun(L, g.eps, q, q1, q2);
  const Cut C = cutf(g, L);
  float A = 0.f, A1 = 0.f, f, f1, f2;
  for (int k = 0; k <= g.R; ++k) {
    basis_k(g, C, k, L, iL, f, f1, f2, pos_term ? 2 : 1);
    if (hB) hB[(int64_t)e * (g.R + 1) + k] = f1 * t * iL;
    if (pos_term) {
      const float gb = gB[(int64_t)e * (g.R + 1) + k];
      A += gb * f1;
      A1 += gb * f2;
    }
  }
  if (hU) {
    const float c = q1 * t * iL;
    hU[3 * e] = hx * q + x * c;
    hU[3 * e + 1] = hy * q + y * c;
    hU[3 * e + 2] = hz * q + z * c;
  }
  if (pos_term) {
    const float ux = gU[3 * e], uy = gU[3 * e + 1], uz = gU[3 * e + 2];
    const float u = ux * x + uy * y + uz * z, w = ux * hx + uy * hy + uz * hz;
    const float cv = (A1 + u * q2) * t * iL * iL - (A + u * q1) * t * iL * iL * iL + q1 * w * iL;
    const float cu = q1 * t * iL, ch = (A + u * q1) * iL;
    ox = cv * x + cu * ux + ch * hx;
    oy = cv * y + cu * uy + ch * hy;
    oz = cv * z + cu * uz + ch * hz;
  } else {
    ox = oy = oz = 0.f;
  }
}

__global__ void __launch_bounds__(256) geom_vvjp_kernel(Geo g, Csr din, Csr sout, int N, const float* __restrict__ gB,
                                                        const float* __restrict__ gU, const float* __restrict__ hpos,
                                                        float* __restrict__ hB, float* __restrict__ hU,
                                                        float* __restrict__ gpos) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= N) return;
  const bool pt = gpos != nullptr;
  float ax = 0.f, ay = 0.f, az = 0.f, x, y, z;
  for (int p = din.ptr[n] + lane; p < din.ptr[n + 1]; p += 64) {
    geom_edge2(g, edge_at(din, p), gB, gU, hpos, hB, hU, pt, x, y, z);  // every edge once (by its dst)
    ax += x;
    ay += y;
    az += z;
  }
  if (!pt) return;
  for (int p = sout.ptr[n] + lane; p < sout.ptr[n + 1]; p += 64) {
    geom_edge2(g, edge_at(sout, p), gB, gU, hpos, nullptr, nullptr, true, x, y, z);
    ax -= x;
    ay -= y;
    az -= z;
  }
  ax = wave_sum(ax);
  ay = wave_sum(ay);
  az = wave_sum(az);
  if (lane == 0) {
    gpos[3 * n] = ax;
    gpos[3 * n + 1] = ay;
    gpos[3 * n + 2] = az;
  }
}

// ------------------------------------------------------------------------ message
struct Msg {
  int N, F, R;
  const int* dst;
  const int* src;
  Csr din, sout;
  const float* s;
  const float* v;
  const float* phi;
  const float* basis;
  const float* unit;
  const float* W;  // [3F][R]
  const float* b;  // [3F]
};

// RM >= R + 1 (compile-time radial width incl. the bias column), NC feature chunks of 64
// lanes: per-lane arrays are fully unrolled (registers, no scratch)
template <int RM>
struct Rows {
  float w[3][RM];  // the lane's three filter rows q F + f; column R = bias
};

template <int RM>
__device__ __forceinline__ void load_rows(const Msg& M, int f, Rows<RM>& Wr) {
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int m = q * M.F + f;
#pragma unroll
    for (int r = 0; r < RM; ++r) Wr.w[q][r] = r < M.R ? M.W[(int64_t)m * M.R + r] : (r == M.R ? M.b[m] : 0.f);
  }
}

template <int RM>
__device__ __forceinline__ void load_basis(const Msg& M, const float* src, float (&bs)[RM]) {
#pragma unroll
  for (int r = 0; r < RM; ++r) bs[r] = r <= M.R ? src[r] : 0.f;
}

template <int RM>
__device__ __forceinline__ void filt(const Rows<RM>& Wr, const float (&bs)[RM], float (&w)[3]) {
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < RM; ++r) t += Wr.w[q][r] * bs[r];
    w[q] = t;
  }
}

template <int RM, int NC>
__global__ void __launch_bounds__(256) msg_fwd_kernel(Msg M, float* __restrict__ s1, float* __restrict__ v1) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= M.N) return;
  const int F = M.F, R1 = M.R + 1;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int f = lane + 64 * c;
    if (f >= F) continue;
    Rows<RM> Wr;
    load_rows<RM>(M, f, Wr);
    float ds = 0.f, dv0 = 0.f, dv1 = 0.f, dv2 = 0.f;
    for (int p = M.sout.ptr[n]; p < M.sout.ptr[n + 1]; ++p) {
      const int e = edge_at(M.sout, p), j = M.dst[e];
      float bs[RM], w[3];
      load_basis<RM>(M, M.basis + (int64_t)e * R1, bs);
      filt<RM>(Wr, bs, w);
      const float* P = M.phi + (int64_t)j * 3 * F;
      const float ov = w[0] * P[f], oe = w[1] * P[F + f], os = w[2] * P[2 * F + f];
      const float* V = M.v + (int64_t)j * 3 * F;
      const float* U = M.unit + 3 * (int64_t)e;
      ds += os;
      dv0 += V[f] * ov + oe * U[0];
      dv1 += V[F + f] * ov + oe * U[1];
      dv2 += V[2 * F + f] * ov + oe * U[2];
    }
    s1[(int64_t)n * F + f] = M.s[(int64_t)n * F + f] + ds;
    const float* Vn = M.v + (int64_t)n * 3 * F;
    float* o = v1 + (int64_t)n * 3 * F;
    o[f] = Vn[f] + dv0;
    o[F + f] = Vn[F + f] + dv1;
    o[2 * F + f] = Vn[2 * F + f] + dv2;
  }
}

// fold the 4 waves' W-gradient accumulators (lanes = features) into this workgroup's
// partial [3F][R+1] through LDS, waves in a fixed order
template <int RM, int NC>
__device__ void wacc_store(const Rows<RM> (&A)[NC], int F, int R, float* __restrict__ part, float* lds) {
  const int R1 = R + 1, n = 3 * F * R1;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int w = 0; w < 4; ++w) {
    if (wv == w) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int f = lane + 64 * c;
        if (f >= F) continue;
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
          for (int r = 0; r < RM; ++r) {
            if (r >= R1) continue;
            const int k = (q * F + f) * R1 + r;
            lds[k] = (w == 0 ? 0.f : lds[k]) + A[c].w[q][r];
          }
      }
    }
    __syncthreads();
  }
  for (int k = threadIdx.x; k < n; k += 256) part[k] = lds[k];
}

// VJP over the dst-CSR: g_phi, g_v (= Gv + gather sums), g_basis, g_unit (+ W partials).
// One wave per destination node; incoming edges in batches of kEB whose index / basis /
// source-row loads are all issued before any of them is used (the per-edge dependent load
// chain src -> Gv[src] was the whole cost: ~3 us per edge at one edge per step).
constexpr int kEB = 4;

template <int RM, int NC>
__global__ void __launch_bounds__(256) msg_vjp_kernel(Msg M, const float* __restrict__ Gs,
                                                      const float* __restrict__ Gv, float* __restrict__ gphi,
                                                      float* __restrict__ gv, float* __restrict__ gbas,
                                                      float* __restrict__ gun, float* __restrict__ wpart) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63;
  const int F = M.F, R1 = M.R + 1;
  Rows<RM> acc[NC], Wr[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int r = 0; r < RM; ++r) acc[c].w[q][r] = 0.f;
    load_rows<RM>(M, min(lane + 64 * c, F - 1), Wr[c]);
  }
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j < M.N) {
    float aphi[NC][3], av[NC][3], P[NC][3], V[NC][3];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int f = min(lane + 64 * c, F - 1);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        aphi[c][q] = av[c][q] = 0.f;
        P[c][q] = M.phi[(int64_t)j * 3 * F + q * F + f];
        V[c][q] = M.v[(int64_t)j * 3 * F + q * F + f];
      }
    }
    const int pb = M.din.ptr[j], pe = M.din.ptr[j + 1];
    for (int p0 = pb; p0 < pe; p0 += kEB) {
      int e[kEB], n[kEB];
      float bs[kEB][RM], U[kEB][3], g[kEB][NC][4];
#pragma unroll
      for (int b = 0; b < kEB; ++b) e[b] = edge_at(M.din, min(p0 + b, pe - 1));
#pragma unroll
      for (int b = 0; b < kEB; ++b) n[b] = M.src[e[b]];
#pragma unroll
      for (int b = 0; b < kEB; ++b) {
        load_basis<RM>(M, M.basis + (int64_t)e[b] * R1, bs[b]);
#pragma unroll
        for (int q = 0; q < 3; ++q) U[b][q] = M.unit[3 * (int64_t)e[b] + q];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int f = min(lane + 64 * c, F - 1);
          const float* G = Gv + (int64_t)n[b] * 3 * F;
          g[b][c][0] = G[f];
          g[b][c][1] = G[F + f];
          g[b][c][2] = G[2 * F + f];
          g[b][c][3] = Gs[(int64_t)n[b] * F + f];
        }
      }
#pragma unroll
      for (int b = 0; b < kEB; ++b) {
        if (p0 + b >= pe) break;  // uniform
        float pbv[RM], pu[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < RM; ++r) pbv[r] = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          if (lane + 64 * c >= F) continue;
          float w[3];
          filt<RM>(Wr[c], bs[b], w);
          const float g0 = g[b][c][0], g1 = g[b][c][1], g2 = g[b][c][2];
          const float go[3] = {g0 * V[c][0] + g1 * V[c][1] + g2 * V[c][2], g0 * U[b][0] + g1 * U[b][1] + g2 * U[b][2],
                               g[b][c][3]};
#pragma unroll
          for (int q = 0; q < 3; ++q) aphi[c][q] += go[q] * w[q];
          const float ov = w[0] * P[c][0], oe = w[1] * P[c][1];
          av[c][0] += g0 * ov;
          av[c][1] += g1 * ov;
          av[c][2] += g2 * ov;
          pu[0] += g0 * oe;
          pu[1] += g1 * oe;
          pu[2] += g2 * oe;
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            const float gw = go[q] * P[c][q];
#pragma unroll
            for (int r = 0; r < RM; ++r) {
              pbv[r] += Wr[c].w[q][r] * gw;
              acc[c].w[q][r] += gw * bs[b][r];
            }
          }
        }
#pragma unroll
        for (int r = 0; r < RM; ++r) {
          if (r >= R1) continue;
          const float t = wave_sum(pbv[r]);
          if (lane == 0) gbas[(int64_t)e[b] * R1 + r] = t;
        }
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const float t = wave_sum(pu[q]);
          if (lane == 0) gun[3 * (int64_t)e[b] + q] = t;
        }
      }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int f = lane + 64 * c;
      if (f >= F) continue;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        gphi[(int64_t)j * 3 * F + q * F + f] = aphi[c][q];
        gv[(int64_t)j * 3 * F + q * F + f] = Gv[(int64_t)j * 3 * F + q * F + f] + av[c][q];
      }
    }
  }
  if (wpart) wacc_store<RM, NC>(acc, F, M.R, wpart + (int64_t)blockIdx.x * 3 * F * R1, lds);
}

// fixed-order sum of the workgroup partials into W grad [3F][R] and b grad [3F]: a block
// owns 64 outputs; its 4 waves sum interleaved quarters of the partials (8 loads in flight
// per lane), folded through LDS in a fixed order (one partial row per node quartet made a
// one-thread-per-output walk over ~256 rows a 19 us dependent-load chain)
__global__ void __launch_bounds__(256) wpart_reduce_kernel(const float* __restrict__ part, int nparts, int F, int R,
                                                           float* __restrict__ gW, float* __restrict__ gb) {
  __shared__ float red[4][64];
  const int R1 = R + 1, n = 3 * F * R1;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + lane;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (k < n) {
    int p = w;
    for (; p + 28 < nparts; p += 32) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] += part[(int64_t)(p + 4 * u) * n + k];
    }
    for (int u = 0; p < nparts; p += 4, ++u) a[u & 7] += part[(int64_t)p * n + k];
  }
  red[w][lane] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (w == 0 && k < n) {
    const float t = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    const int m = k / R1, r = k % R1;
    if (r < R)
      gW[(int64_t)m * R + r] = t;
    else
      gb[m] = t;
  }
}

// ---- double backward: (1) src-CSR pass -> gradients of the VJP's upstream (Gs, Gv)
struct Tan {
  const float* Hv;    // [N, 3F] or null
  const float* Hphi;  // [N, 3F] or null
  const float* Hbas;  // [E, R+1] or null
  const float* Hun;   // [E, 3] or null
};

template <int RM, int NC>
__global__ void __launch_bounds__(256) msg_vvjp_src_kernel(Msg M, Tan T, float* __restrict__ gGs,
                                                           float* __restrict__ gGv) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= M.N) return;
  const int F = M.F, R1 = M.R + 1;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int f = lane + 64 * c;
    if (f >= F) continue;
    Rows<RM> Wr;
    load_rows<RM>(M, f, Wr);
    float as = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f;
    for (int p = M.sout.ptr[n]; p < M.sout.ptr[n + 1]; ++p) {
      const int e = edge_at(M.sout, p), j = M.dst[e];
      float bs[RM], w[3], wp[3] = {0.f, 0.f, 0.f};
      load_basis<RM>(M, M.basis + (int64_t)e * R1, bs);
      filt<RM>(Wr, bs, w);
      if (T.Hbas) {
        float hb[RM];
        load_basis<RM>(M, T.Hbas + (int64_t)e * R1, hb);
        filt<RM>(Wr, hb, wp);
      }
      const float* P = M.phi + (int64_t)j * 3 * F;
      float o[3], op[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const float Pq = P[q * F + f];
        o[q] = w[q] * Pq;
        op[q] = wp[q] * Pq + (T.Hphi ? w[q] * T.Hphi[(int64_t)j * 3 * F + q * F + f] : 0.f);
      }
      as += op[2];
      const float* V = M.v + (int64_t)j * 3 * F;
      const float* U = M.unit + 3 * (int64_t)e;
      float t0 = V[f] * op[0] + op[1] * U[0], t1 = V[F + f] * op[0] + op[1] * U[1],
            t2 = V[2 * F + f] * op[0] + op[1] * U[2];
      if (T.Hv) {
        const float* HV = T.Hv + (int64_t)j * 3 * F;
        t0 += HV[f] * o[0];
        t1 += HV[F + f] * o[0];
        t2 += HV[2 * F + f] * o[0];
      }
      if (T.Hun) {
        const float* HU = T.Hun + 3 * (int64_t)e;
        t0 += o[1] * HU[0];
        t1 += o[1] * HU[1];
        t2 += o[1] * HU[2];
      }
      a0 += t0;
      a1 += t1;
      a2 += t2;
    }
    if (gGs) gGs[(int64_t)n * F + f] = as;
    if (gGv) {
      float* o = gGv + (int64_t)n * 3 * F;
      const float* HVn = T.Hv ? T.Hv + (int64_t)n * 3 * F : nullptr;
      o[f] = a0 + (HVn ? HVn[f] : 0.f);
      o[F + f] = a1 + (HVn ? HVn[F + f] : 0.f);
      o[2 * F + f] = a2 + (HVn ? HVn[2 * F + f] : 0.f);
    }
  }
}

// ---- double backward: (2) dst-CSR pass -> second-order terms on v, phi, basis, unit, W, b
template <int RM, int NC>
__global__ void __launch_bounds__(256) msg_vvjp_dst_kernel(Msg M, Tan T, const float* __restrict__ Gs,
                                                           const float* __restrict__ Gv, float* __restrict__ gv,
                                                           float* __restrict__ gphi, float* __restrict__ gbas,
                                                           float* __restrict__ gun, float* __restrict__ wpart) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63;
  const int F = M.F, R1 = M.R + 1;
  Rows<RM> acc[NC], Wr[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int r = 0; r < RM; ++r) acc[c].w[q][r] = 0.f;
    load_rows<RM>(M, min(lane + 64 * c, F - 1), Wr[c]);
  }
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j < M.N) {
    float aphi[NC][3], av[NC][3], P[NC][3], HP[NC][3], V[NC][3], HV[NC][3];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int f = min(lane + 64 * c, F - 1);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int64_t o = (int64_t)j * 3 * F + q * F + f;
        aphi[c][q] = av[c][q] = 0.f;
        P[c][q] = M.phi[o];
        V[c][q] = M.v[o];
        HP[c][q] = T.Hphi ? T.Hphi[o] : 0.f;
        HV[c][q] = T.Hv ? T.Hv[o] : 0.f;
      }
    }
    const int pb = M.din.ptr[j], pe = M.din.ptr[j + 1];
    for (int p0 = pb; p0 < pe; p0 += kEB) {
      int e[kEB], n[kEB];
      float bs[kEB][RM], hb[kEB][RM], U[kEB][3], HU[kEB][3], g[kEB][NC][4];
#pragma unroll
      for (int b = 0; b < kEB; ++b) e[b] = edge_at(M.din, min(p0 + b, pe - 1));
#pragma unroll
      for (int b = 0; b < kEB; ++b) n[b] = M.src[e[b]];
#pragma unroll
      for (int b = 0; b < kEB; ++b) {
        load_basis<RM>(M, M.basis + (int64_t)e[b] * R1, bs[b]);
        if (T.Hbas)
          load_basis<RM>(M, T.Hbas + (int64_t)e[b] * R1, hb[b]);
        else
#pragma unroll
          for (int r = 0; r < RM; ++r) hb[b][r] = 0.f;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          U[b][q] = M.unit[3 * (int64_t)e[b] + q];
          HU[b][q] = T.Hun ? T.Hun[3 * (int64_t)e[b] + q] : 0.f;
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int f = min(lane + 64 * c, F - 1);
          const float* G = Gv + (int64_t)n[b] * 3 * F;
          g[b][c][0] = G[f];
          g[b][c][1] = G[F + f];
          g[b][c][2] = G[2 * F + f];
          g[b][c][3] = Gs[(int64_t)n[b] * F + f];
        }
      }
#pragma unroll
      for (int b = 0; b < kEB; ++b) {
        if (p0 + b >= pe) break;  // uniform
        float pbv[RM], pu[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < RM; ++r) pbv[r] = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          if (lane + 64 * c >= F) continue;
          float w[3], wp[3];
          filt<RM>(Wr[c], bs[b], w);
          filt<RM>(Wr[c], hb[b], wp);
          const float g0 = g[b][c][0], g1 = g[b][c][1], g2 = g[b][c][2];
          const float a[3] = {g0 * HV[c][0] + g1 * HV[c][1] + g2 * HV[c][2],
                              g0 * HU[b][0] + g1 * HU[b][1] + g2 * HU[b][2], 0.f};
          const float bb[3] = {g0 * V[c][0] + g1 * V[c][1] + g2 * V[c][2], g0 * U[b][0] + g1 * U[b][1] + g2 * U[b][2],
                               g[b][c][3]};
          float op[3];
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            op[q] = wp[q] * P[c][q] + w[q] * HP[c][q];
            aphi[c][q] += a[q] * w[q] + bb[q] * wp[q];
          }
          av[c][0] += g0 * op[0];
          av[c][1] += g1 * op[0];
          av[c][2] += g2 * op[0];
          pu[0] += g0 * op[1];
          pu[1] += g1 * op[1];
          pu[2] += g2 * op[1];
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            const float gw2 = a[q] * P[c][q] + bb[q] * HP[c][q], bP = bb[q] * P[c][q];
#pragma unroll
            for (int r = 0; r < RM; ++r) {
              pbv[r] += Wr[c].w[q][r] * gw2;
              acc[c].w[q][r] += gw2 * bs[b][r] + bP * hb[b][r];
            }
          }
        }
        if (gbas)
#pragma unroll
          for (int r = 0; r < RM; ++r) {
            if (r >= R1) continue;
            const float t = wave_sum(pbv[r]);
            if (lane == 0) gbas[(int64_t)e[b] * R1 + r] = t;
          }
        if (gun)
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            const float t = wave_sum(pu[q]);
            if (lane == 0) gun[3 * (int64_t)e[b] + q] = t;
          }
      }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int f = lane + 64 * c;
      if (f >= F) continue;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        if (gphi) gphi[(int64_t)j * 3 * F + q * F + f] = aphi[c][q];
        if (gv) gv[(int64_t)j * 3 * F + q * F + f] = av[c][q];
      }
    }
  }
  if (wpart) wacc_store<RM, NC>(acc, F, M.R, wpart + (int64_t)blockIdx.x * 3 * F * R1, lds);
}

}  // namespace pf

// ------------------------------------------------------------------------ host
namespace {
using pf::Csr;

void chk(const at::Tensor& t, std::initializer_list<int64_t> shape, const char* name) {
  HY_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), "painn_force: ", name,
           " must be a contiguous fp32 GPU tensor");
  int64_t n = 1;
  for (auto s : shape) n *= s;
  HY_CHECK(t.numel() == n, "painn_force: ", name, " has ", t.numel(), " elements, expected ", n);
}

const float* optf(const c10::optional<at::Tensor>& t, std::initializer_list<int64_t> shape, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  chk(*t, shape, name);
  return t->data_ptr<float>();
}

Csr csr(const at::Tensor& ptr, const c10::optional<at::Tensor>& perm, int64_t N, int64_t E, const char* name) {
  HY_CHECK(ptr.is_cuda() && ptr.scalar_type() == at::kInt && ptr.numel() == N + 1, "painn_force: ", name,
           " rowptr must be int32 [N+1]");
  Csr c{ptr.data_ptr<int>(), nullptr};
  if (perm.has_value() && perm->defined()) {
    HY_CHECK(perm->is_cuda() && perm->scalar_type() == at::kInt && perm->numel() == E, "painn_force: ", name,
             " perm must be int32 [E]");
    c.perm = perm->data_ptr<int>();
  }
  return c;
}

pf::Geo geo(const at::Tensor& pos, const c10::optional<at::Tensor>& shift, const at::Tensor& dst,
            const at::Tensor& src, int64_t R, double a, double cutoff, double eps) {
  const int64_t N = pos.size(0), E = dst.numel();
  chk(pos, {N, 3}, "pos");
  HY_CHECK(dst.scalar_type() == at::kInt && src.scalar_type() == at::kInt && src.numel() == E && dst.is_cuda() &&
               src.is_cuda(),
           "painn_force: dst/src int32 [E]");
  HY_CHECK(R >= 1 && R < pf::kMaxR, "painn_force: num_radial out of range");
  pf::Geo g{pos.data_ptr<float>(), optf(shift, {E, 3}, "shift"), dst.data_ptr<int>(), src.data_ptr<int>(), (int)R,
            (float)a, (float)cutoff, (float)eps};
  return g;
}

pf::Msg msg(const at::Tensor& s, const at::Tensor& v, const at::Tensor& phi, const at::Tensor& basis,
            const at::Tensor& unit, const at::Tensor& W, const at::Tensor& b, const at::Tensor& dst,
            const at::Tensor& src, const at::Tensor& dptr, const c10::optional<at::Tensor>& dperm,
            const at::Tensor& sptr, const c10::optional<at::Tensor>& sperm) {
  const int64_t N = phi.size(0), F = phi.size(1) / 3, R = W.size(1), E = dst.numel();
  HY_CHECK(F >= 1 && F <= 128, "painn_force: message width must be <= 128");
  HY_CHECK(R >= 1 && R + 1 <= 32, "painn_force: num_radial out of range (<= 31)");
  HY_CHECK(dst.scalar_type() == at::kInt && src.scalar_type() == at::kInt && src.numel() == E,
           "painn_force: dst/src int32 [E]");
  if (s.defined() && s.numel()) chk(s, {N, F}, "s");
  chk(v, {N, 3, F}, "v");
  chk(phi, {N, 3 * F}, "phi");
  chk(basis, {E, R + 1}, "basis");
  chk(unit, {E, 3}, "unit");
  chk(W, {3 * F, R}, "W");
  chk(b, {3 * F}, "b");
  pf::Msg M{};
  M.N = (int)N;
  M.F = (int)F;
  M.R = (int)R;
  M.dst = dst.data_ptr<int>();
  M.src = src.data_ptr<int>();
  M.din = csr(dptr, dperm, N, E, "dst");
  M.sout = csr(sptr, sperm, N, E, "src");
  M.s = (s.defined() && s.numel()) ? s.data_ptr<float>() : nullptr;
  M.v = v.data_ptr<float>();
  M.phi = phi.data_ptr<float>();
  M.basis = basis.data_ptr<float>();
  M.unit = unit.data_ptr<float>();
  M.W = W.data_ptr<float>();
  M.b = b.data_ptr<float>();
  return M;
}

// template dispatch over (RM = padded radial width incl. bias column, NC = 64-feature chunks)
#define HY_PF_DISPATCH(M, KER, ...)                                              \
  do {                                                                           \
    const int r1_ = (M).R + 1, nc_ = (M).F > 64 ? 2 : 1;                         \
    if (r1_ <= 8) {                                                              \
      if (nc_ == 1) KER<8, 1>__VA_ARGS__; else KER<8, 2>__VA_ARGS__;             \
    } else if (r1_ <= 16) {                                                      \
      if (nc_ == 1) KER<16, 1>__VA_ARGS__; else KER<16, 2>__VA_ARGS__;           \
    } else {                                                                     \
      if (nc_ == 1) KER<32, 1>__VA_ARGS__; else KER<32, 2>__VA_ARGS__;           \
    }                                                                            \
  } while (0)

int grid_nodes(int64_t N) { return std::max(1, ceil_div(N, 4)); }
int grid_stride(int64_t N) { return std::max(1, ceil_div(N, 4)); }  // one node per wave
size_t wlds(int64_t F, int64_t R) { return (size_t)3 * F * (R + 1) * sizeof(float); }
}  // namespace

std::vector<at::Tensor> painn_geom_fwd(const at::Tensor& pos, const c10::optional<at::Tensor>& shift,
                                       const at::Tensor& dst, const at::Tensor& src, int64_t R, double a,
                                       double cutoff, double eps) {
  auto g = geo(pos, shift, dst, src, R, a, cutoff, eps);
  const int64_t E = dst.numel();
  auto basis = at::empty({E, R + 1}, pos.options());
  auto unit = at::empty({E, 3}, pos.options());
  if (E) pf::geom_fwd_kernel<<<ceil_div(E, 256), 256, 0, stream()>>>(g, (int)E, basis.data_ptr<float>(),
                                                                       unit.data_ptr<float>());
  return {basis, unit};
}

at::Tensor painn_geom_vjp(const at::Tensor& pos, const c10::optional<at::Tensor>& shift, const at::Tensor& dst,
                          const at::Tensor& src, const at::Tensor& dptr, const c10::optional<at::Tensor>& dperm,
                          const at::Tensor& sptr, const c10::optional<at::Tensor>& sperm, const at::Tensor& gB,
                          const at::Tensor& gU, int64_t R, double a, double cutoff, double eps) {
  auto g = geo(pos, shift, dst, src, R, a, cutoff, eps);
  const int64_t N = pos.size(0), E = dst.numel();
  chk(gB, {E, R + 1}, "gB");
  chk(gU, {E, 3}, "gU");
  auto din = csr(dptr, dperm, N, E, "dst"), sout = csr(sptr, sperm, N, E, "src");
  auto gpos = at::empty({N, 3}, pos.options());
  if (N) pf::geom_vjp_kernel<<<grid_nodes(N), 256, 0, stream()>>>(g, din, sout, (int)N, gB.data_ptr<float>(),
                                                                    gU.data_ptr<float>(), gpos.data_ptr<float>());
  return gpos;
}

std::vector<at::Tensor> painn_geom_vvjp(const at::Tensor& pos, const c10::optional<at::Tensor>& shift,
                                        const at::Tensor& dst, const at::Tensor& src, const at::Tensor& dptr,
                                        const c10::optional<at::Tensor>& dperm, const at::Tensor& sptr,
                                        const c10::optional<at::Tensor>& sperm, const at::Tensor& gB,
                                        const at::Tensor& gU, const at::Tensor& hpos, int64_t R, double a,
                                        double cutoff, double eps, bool need_g, bool need_pos) {
  auto g = geo(pos, shift, dst, src, R, a, cutoff, eps);
  const int64_t N = pos.size(0), E = dst.numel();
  chk(gB, {E, R + 1}, "gB");
  chk(gU, {E, 3}, "gU");
  chk(hpos, {N, 3}, "hpos");
  auto din = csr(dptr, dperm, N, E, "dst"), sout = csr(sptr, sperm, N, E, "src");
  at::Tensor hB = at::empty({0}, pos.options()), hU = hB, gp = hB;
  if (need_g) {
    hB = at::empty({E, R + 1}, pos.options());
    hU = at::empty({E, 3}, pos.options());
  }
  if (need_pos) gp = at::empty({N, 3}, pos.options());
  if (N && (need_g || need_pos))
    pf::geom_vvjp_kernel<<<grid_nodes(N), 256, 0, stream()>>>(
        g, din, sout, (int)N, gB.data_ptr<float>(), gU.data_ptr<float>(), hpos.data_ptr<float>(),
        need_g ? hB.data_ptr<float>() : nullptr, need_g ? hU.data_ptr<float>() : nullptr,
        need_pos ? gp.data_ptr<float>() : nullptr);
  return {hB, hU, gp};
}

std::vector<at::Tensor> painn_msg_fwd(const at::Tensor& s, const at::Tensor& v, const at::Tensor& phi,
                                      const at::Tensor& basis, const at::Tensor& unit, const at::Tensor& W,
                                      const at::Tensor& b, const at::Tensor& dst, const at::Tensor& src,
                                      const at::Tensor& dptr, const c10::optional<at::Tensor>& dperm,
                                      const at::Tensor& sptr, const c10::optional<at::Tensor>& sperm) {
  HY_CHECK(s.defined() && s.numel(), "painn_msg_fwd: s required");
  auto M = msg(s, v, phi, basis, unit, W, b, dst, src, dptr, dperm, sptr, sperm);
  auto s1 = at::empty_like(s), v1 = at::empty_like(v);
  if (M.N) HY_PF_DISPATCH(M, pf::msg_fwd_kernel, <<<grid_nodes(M.N), 256, 0, stream()>>>(M, s1.data_ptr<float>(), v1.data_ptr<float>()));
  return {s1, v1};
}

std::vector<at::Tensor> painn_msg_vjp(const at::Tensor& Gs, const at::Tensor& Gv, const at::Tensor& v,
                                      const at::Tensor& phi, const at::Tensor& basis, const at::Tensor& unit,
                                      const at::Tensor& W, const at::Tensor& b, const at::Tensor& dst,
                                      const at::Tensor& src, const at::Tensor& dptr,
                                      const c10::optional<at::Tensor>& dperm, const at::Tensor& sptr,
                                      const c10::optional<at::Tensor>& sperm, bool need_w) {
  auto M = msg(at::Tensor(), v, phi, basis, unit, W, b, dst, src, dptr, dperm, sptr, sperm);
  chk(Gs, {M.N, M.F}, "Gs");
  chk(Gv, {M.N, 3, M.F}, "Gv");
  const int64_t E = dst.numel();
  auto gphi = at::empty_like(phi), gv = at::empty_like(v);
  auto gbas = at::empty({E, M.R + 1}, v.options()), gun = at::empty({E, 3}, v.options());
  at::Tensor gW = at::empty({0}, v.options()), gb = gW;
  const int grid = grid_stride(M.N);
  at::Tensor part;
  if (need_w) {
    part = at::empty({grid, 3 * M.F * (M.R + 1)}, v.options());
    gW = at::empty_like(W);
    gb = at::empty_like(b);
  }
  if (M.N)
    HY_PF_DISPATCH(M, pf::msg_vjp_kernel, <<<grid, 256, need_w ? wlds(M.F, M.R) : 0, stream()>>>(
        M, Gs.data_ptr<float>(), Gv.data_ptr<float>(), gphi.data_ptr<float>(), gv.data_ptr<float>(),
        gbas.data_ptr<float>(), gun.data_ptr<float>(), need_w ? part.data_ptr<float>() : nullptr));
  if (need_w) {
    const int n = 3 * M.F * (M.R + 1);
    if (M.N)
      pf::wpart_reduce_kernel<<<ceil_div(n, 64), 256, 0, stream()>>>(part.data_ptr<float>(), grid, M.F, M.R,
                                                                       gW.data_ptr<float>(), gb.data_ptr<float>());
    else {
      gW.zero_();
      gb.zero_();
    }
  }
  return {gv, gphi, gbas, gun, gW, gb};
}

std::vector<at::Tensor> painn_msg_vvjp(const at::Tensor& Gs, const at::Tensor& Gv, const at::Tensor& v,
                                       const at::Tensor& phi, const at::Tensor& basis, const at::Tensor& unit,
                                       const at::Tensor& W, const at::Tensor& b, const at::Tensor& dst,
                                       const at::Tensor& src, const at::Tensor& dptr,
                                       const c10::optional<at::Tensor>& dperm, const at::Tensor& sptr,
                                       const c10::optional<at::Tensor>& sperm, const c10::optional<at::Tensor>& Hv,
                                       const c10::optional<at::Tensor>& Hphi, const c10::optional<at::Tensor>& Hbas,
                                       const c10::optional<at::Tensor>& Hun, at::IntArrayRef need) {
  auto M = msg(at::Tensor(), v, phi, basis, unit, W, b, dst, src, dptr, dperm, sptr, sperm);
  HY_CHECK(need.size() == 8, "painn_msg_vvjp: need flags (Gs, Gv, v, phi, basis, unit, W, b)");
  chk(Gs, {M.N, M.F}, "Gs");
  chk(Gv, {M.N, 3, M.F}, "Gv");
  const int64_t E = dst.numel(), N = M.N, F = M.F, R = M.R;
  pf::Tan T{optf(Hv, {N, 3, F}, "Hv"), optf(Hphi, {N, 3 * F}, "Hphi"), optf(Hbas, {E, R + 1}, "Hbas"),
            optf(Hun, {E, 3}, "Hun")};
  std::vector<at::Tensor> out(8, at::empty({0}, v.options()));
  if (need[0]) out[0] = at::empty({N, F}, v.options());
  if (need[1]) out[1] = at::empty_like(v);
  if (need[2]) out[2] = at::empty_like(v);
  if (need[3]) out[3] = at::empty_like(phi);
  if (need[4]) out[4] = at::empty({E, R + 1}, v.options());
  if (need[5]) out[5] = at::empty({E, 3}, v.options());
  const bool nw = need[6] || need[7];
  if (nw) {
    out[6] = at::empty_like(W);
    out[7] = at::empty_like(b);
  }
  auto fp = [](const at::Tensor& t) { return t.numel() ? t.data_ptr<float>() : nullptr; };
  if (N && (need[0] || need[1]))
    HY_PF_DISPATCH(M, pf::msg_vvjp_src_kernel, <<<grid_nodes(N), 256, 0, stream()>>>(M, T, fp(out[0]), fp(out[1])));
  const int grid = grid_stride(N);
  at::Tensor part;
  if (nw) part = at::empty({grid, 3 * F * (R + 1)}, v.options());
  if (N && (need[2] || need[3] || need[4] || need[5] || nw))
    HY_PF_DISPATCH(M, pf::msg_vvjp_dst_kernel, <<<grid, 256, nw ? wlds(F, R) : 0, stream()>>>(
        M, T, Gs.data_ptr<float>(), Gv.data_ptr<float>(), fp(out[2]), fp(out[3]), fp(out[4]), fp(out[5]),
        nw ? part.data_ptr<float>() : nullptr));
  if (nw) {
    const int n = 3 * (int)F * ((int)R + 1);
    if (N)
      pf::wpart_reduce_kernel<<<ceil_div(n, 64), 256, 0, stream()>>>(part.data_ptr<float>(), grid, (int)F, (int)R,
                                                                       out[6].data_ptr<float>(),
                                                                       out[7].data_ptr<float>());
    else {
      out[6].zero_();
      out[7].zero_();
    }
  }
  return out;
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("painn_geom_fwd(Tensor pos, Tensor? shift, Tensor dst, Tensor src, int R, float a, float cutoff, "
        "float eps) -> Tensor[]");
  m.def("painn_geom_vjp(Tensor pos, Tensor? shift, Tensor dst, Tensor src, Tensor dptr, Tensor? dperm, Tensor sptr, "
        "Tensor? sperm, Tensor gB, Tensor gU, int R, float a, float cutoff, float eps) -> Tensor");
  m.def("painn_geom_vvjp(Tensor pos, Tensor? shift, Tensor dst, Tensor src, Tensor dptr, Tensor? dperm, "
        "Tensor sptr, Tensor? sperm, Tensor gB, Tensor gU, Tensor hpos, int R, float a, float cutoff, float eps, "
        "bool need_g, bool need_pos) -> Tensor[]");
  m.def("painn_msg_fwd(Tensor s, Tensor v, Tensor phi, Tensor basis, Tensor unit, Tensor W, Tensor b, Tensor dst, "
        "Tensor src, Tensor dptr, Tensor? dperm, Tensor sptr, Tensor? sperm) -> Tensor[]");
  m.def("painn_msg_vjp(Tensor Gs, Tensor Gv, Tensor v, Tensor phi, Tensor basis, Tensor unit, Tensor W, Tensor b, "
        "Tensor dst, Tensor src, Tensor dptr, Tensor? dperm, Tensor sptr, Tensor? sperm, bool need_w) -> Tensor[]");
  m.def("painn_msg_vvjp(Tensor Gs, Tensor Gv, Tensor v, Tensor phi, Tensor basis, Tensor unit, Tensor W, Tensor b, "
        "Tensor dst, Tensor src, Tensor dptr, Tensor? dperm, Tensor sptr, Tensor? sperm, Tensor? Hv, Tensor? Hphi, "
        "Tensor? Hbas, Tensor? Hun, int[] need) -> Tensor[]");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("painn_geom_fwd", hy::painn_geom_fwd);
  m.impl("painn_geom_vjp", hy::painn_geom_vjp);
  m.impl("painn_geom_vvjp", hy::painn_geom_vvjp);
  m.impl("painn_msg_fwd", hy::painn_msg_fwd);
  m.impl("painn_msg_vjp", hy::painn_msg_vjp);
  m.impl("painn_msg_vvjp", hy::painn_msg_vvjp);
}
