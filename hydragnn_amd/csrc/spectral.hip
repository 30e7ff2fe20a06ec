// Batched Laplacian eigenvector positional encodings (gfx950) — the device version of
// PyG AddLaplacianEigenvectorPE used by the reference's GPS preprocessing
// (serialized_dataset_loader.py:90-94,183; examples qm9.py:80-84).  SURVEY N9/K17.
//
// One workgroup per graph (n <= 128 nodes): the symmetric-normalised Laplacian
// L = I - D^-1/2 A D^-1/2 and the eigenvector accumulator V live in LDS (2 x 128 x
// 129 fp32 = 132 KB of the 160 KB per CU) and are diagonalised by cyclic Jacobi
// with round-robin (tournament) pairing: every step applies n/2 disjoint rotations
// in parallel — rows first, then columns and V — so a sweep is n-1 steps of three
// barriers.  Sweeps stop when the off-diagonal norm drops below tol * ||L||_F.
// Eigenpairs are ranked by eigenvalue (ties by index), the trivial one skipped,
// and eigenvectors 1..k written to pe[node, :] (zero-padded for n <= k) with a
// per-(graph, vector) sign from `signs` (PyG's random sign flip).
#include "common.h"

namespace hy {

constexpr int kMaxPeN = 128;
constexpr int kLd = kMaxPeN + 1;  // padded row stride (bank-conflict-free columns)

// pair t (0 <= t < m/2) of round `step` in the circle method over m players
__device__ __forceinline__ void rr_pair(int step, int t, int m, int& p, int& q) {
  const int r = m - 1;
  if (t == 0) {
    p = m - 1;
    q = step % r;
  } else {
    p = (step + t) % r;
    q = (step + r - t) % r;
  }
  if (p > q) {
    const int s = p;
    p = q;
    q = s;
  }
}

__global__ void __launch_bounds__(256) lappe_jacobi_kernel(const int* __restrict__ gptr, const int* __restrict__ rowptr,
                                                           const int64_t* __restrict__ src, int k, int max_sweeps,
                                                           float tol, const float* __restrict__ signs,
                                                           float* __restrict__ pe, float* __restrict__ evals) {
  extern __shared__ float sm[];
  float* A = sm;                  // [n][kLd]
  float* V = sm + kMaxPeN * kLd;  // [n][kLd]
  __shared__ float cs[kMaxPeN / 2][2];
  __shared__ int pq[kMaxPeN / 2][2];
  __shared__ float red[256];
  __shared__ int rank_of[kMaxPeN];
  const int g = blockIdx.x, t = threadIdx.x;
  const int n0 = gptr[g], n = gptr[g + 1] - n0;
  if (n <= 0) return;
  // ---- Laplacian
  for (int e = t; e < n * kLd; e += 256) {
    A[e] = 0.f;
    V[e] = 0.f;
  }
  __syncthreads();
  for (int i = t; i < n; i += 256)
    for (int eo = rowptr[n0 + i]; eo < rowptr[n0 + i + 1]; ++eo) {
      const int j = (int)src[eo] - n0;
      if (j >= 0 && j < n) {
        A[i * kLd + j] = 1.f;
        A[j * kLd + i] = 1.f;  // symmetrise (is_undirected)
      }
    }
  __syncthreads();
  for (int i = t; i < n; i += 256) {
    float d = 0.f;
    for (int j = 0; j < n; ++j) d += A[i * kLd + j];
    red[i] = d > 0.f ? rsqrtf(d) : 0.f;
    V[i * kLd + i] = 1.f;
  }
  __syncthreads();
  for (int e = t; e < n * n; e += 256) {
    const int i = e / n, j = e % n;
    A[i * kLd + j] = (i == j ? 1.f : 0.f) - red[i] * A[i * kLd + j] * red[j];
  }
  __syncthreads();
  // ---- cyclic Jacobi (circle-method pairing over m = n rounded up to even)
  const int m = n + (n & 1);
  const int np = m / 2;
  float fro = 0.f;
  for (int e = t; e < n * n; e += 256) fro += A[(e / n) * kLd + e % n] * A[(e / n) * kLd + e % n];
  red[t] = fro;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) red[t] += red[t + s];
    __syncthreads();
  }
  const float thresh = tol * tol * fmaxf(red[0], 1e-30f);
  __syncthreads();
  for (int sweep = 0; sweep < max_sweeps && n > 1; ++sweep) {
    // off-diagonal norm
    float off = 0.f;
    for (int e = t; e < n * n; e += 256) {
      const int i = e / n, j = e % n;
      if (i != j) off += A[i * kLd + j] * A[i * kLd + j];
    }
    red[t] = off;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (t < s) red[t] += red[t + s];
      __syncthreads();
    }
    const bool done = red[0] <= thresh;
    __syncthreads();
    if (done) break;
    for (int step = 0; step < m - 1; ++step) {
      if (t < np) {
        int p, q;
        rr_pair(step, t, m, p, q);
        float c = 1.f, sn = 0.f;
        if (q < n) {  // the odd-n dummy player never rotates
          const float apq = A[p * kLd + q];
          if (fabsf(apq) > 1e-30f) {
            const float theta = (A[q * kLd + q] - A[p * kLd + p]) / (2.f * apq);
            const float tt = copysignf(1.f, theta) / (fabsf(theta) + sqrtf(theta * theta + 1.f));
            c = rsqrtf(tt * tt + 1.f);
            sn = tt * c;
          }
        }
        cs[t][0] = c;
        cs[t][1] = sn;
        pq[t][0] = p;
        pq[t][1] = q;
      }
      __syncthreads();
      // rows: A <- J^T A
      for (int w = t; w < np * n; w += 256) {
        const int pi = w / n, j = w % n;
        const int p = pq[pi][0], q = pq[pi][1];
        if (q >= n) continue;
        const float c = cs[pi][0], sn = cs[pi][1];
        const float ap = A[p * kLd + j], aq = A[q * kLd + j];
        A[p * kLd + j] = c * ap - sn * aq;
        A[q * kLd + j] = sn * ap + c * aq;
      }
      __syncthreads();
      // columns: A <- A J, V <- V J
      for (int w = t; w < np * n; w += 256) {
        const int pi = w / n, i = w % n;
        const int p = pq[pi][0], q = pq[pi][1];
        if (q >= n) continue;
        const float c = cs[pi][0], sn = cs[pi][1];
        const float ap = A[i * kLd + p], aq = A[i * kLd + q];
        A[i * kLd + p] = c * ap - sn * aq;
        A[i * kLd + q] = sn * ap + c * aq;
        const float vp = V[i * kLd + p], vq = V[i * kLd + q];
        V[i * kLd + p] = c * vp - sn * vq;
        V[i * kLd + q] = sn * vp + c * vq;
      }
      __syncthreads();
    }
  }
  // ---- rank eigenvalues, emit eigenvectors 1..k
  for (int i = t; i < n; i += 256) {
    const float di = A[i * kLd + i];
    int r = 0;
    for (int j = 0; j < n; ++j) {
      const float dj = A[j * kLd + j];
      r += (dj < di) || (dj == di && j < i);
    }
    rank_of[r] = i;
  }
  __syncthreads();
  for (int w = t; w < n * k; w += 256) {
    const int row = w / k, c = w % k;
    float v = 0.f;
    if (c + 1 < n) v = V[row * kLd + rank_of[c + 1]] * signs[(int64_t)g * k + c];
    pe[(int64_t)(n0 + row) * k + c] = v;
  }
  if (evals)
    for (int c = t; c < k; c += 256) evals[(int64_t)g * k + c] = c + 1 < n ? A[rank_of[c + 1] * kLd + rank_of[c + 1]] : 0.f;
}

// edge_index [2, E] (row 0 = source) sorted by destination with rowptr [N+1] (int32),
// gptr [G+1] (int32); signs [G, k]. -> (pe [N, k], evals [G, k])
std::tuple<at::Tensor, at::Tensor> laplacian_pe(const at::Tensor& edge_index, const at::Tensor& rowptr,
                                                const at::Tensor& gptr, int64_t k, const at::Tensor& signs,
                                                int64_t max_sweeps, double tol) {
  HY_CHECK_CUDA(edge_index);
  HY_CHECK_I32(rowptr);
  HY_CHECK_I32(gptr);
  auto ei = edge_index.to(at::kLong).contiguous();
  const int64_t G = gptr.numel() - 1, N = rowptr.numel() - 1;
  auto sg = signs.to(at::kFloat).contiguous();
  HY_CHECK(sg.numel() == G * k, "signs must be [G, k]");
  auto pe = at::zeros({N, k}, sg.options());
  auto ev = at::zeros({G, k}, sg.options());
  if (G == 0 || k == 0) return {pe, ev};
  const int64_t maxn = (gptr.narrow(0, 1, G) - gptr.narrow(0, 0, G)).max().item<int64_t>();
  HY_CHECK(maxn <= kMaxPeN, "laplacian_pe: graphs larger than ", kMaxPeN, " nodes use the host path");
  const size_t lds = 2 * (size_t)kMaxPeN * kLd * sizeof(float);
  static bool attr = [] {
    hipFuncSetAttribute((const void*)lappe_jacobi_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)(2 * kMaxPeN * kLd * sizeof(float)));
    return true;
  }();
  (void)attr;
  lappe_jacobi_kernel<<<(int)G, 256, lds, stream()>>>(gptr.data_ptr<int>(), rowptr.data_ptr<int>(),
                                                      ei.data_ptr<int64_t>(), (int)k, (int)max_sweeps, (float)tol,
                                                      sg.data_ptr<float>(), pe.data_ptr<float>(), ev.data_ptr<float>());
  return {pe, ev};
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def(
      "laplacian_pe(Tensor edge_index, Tensor rowptr, Tensor gptr, int k, Tensor signs, int max_sweeps, float tol) "
      "-> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) { m.impl("laplacian_pe", hy::laplacian_pe); }
