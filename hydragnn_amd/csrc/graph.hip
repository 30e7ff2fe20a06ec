// Device graph builders (gfx950): batched radius graph (optionally periodic) and
// DimeNet triplets.  Replace torch_cluster.radius_graph / RadiusInteractionGraph
// (reference SCFStack.py:57-61,124-128; graph_samples_checks_and_updates.py:109-138),
// ASE's periodic neighbour list (RadiusGraphPBC, :141-343) and torch_sparse's
// triplet construction (DIMEStack.py:232-256).  SURVEY N2/N3/N4, K6/K8.
//
// Both builders are two-pass (count -> exclusive scan -> fill) so that the
// output is dense, destination-sorted (CSR-ready) and deterministic:
//  * radius graph: one thread per receiver i scans the atoms of its own graph
//    (graphs are contiguous: [gptr[g], gptr[g+1])), over all periodic images
//    a in [-rx, rx] x [-ry, ry] x [-rz, rz] of that graph's cell.  Cap policy
//    "index" keeps the first max_nb sources in (image, index) order like
//    torch_cluster; "nearest" keeps the max_nb closest (RadiusGraphPBC's
//    lexsort by length) via a per-thread insertion list, emitted by distance.
//  * triplets: one thread per edge e = (j -> i) lists the in-edges (k -> j) of
//    j with k != i (in CSR order), grouped by e ascending.
#include "common.h"

namespace hy {

constexpr int kMaxNearest = 64;

struct PbcArgs {
  const float* cell;  // [G, 3, 3] (rows = lattice vectors) or nullptr
  const int* reps;    // [G, 3] image extents
};

template <bool FILL, bool NEAREST>
__global__ void __launch_bounds__(256) radius_kernel(const float* __restrict__ pos, const int* __restrict__ node_graph,
                                                     const int* __restrict__ gptr, int N, float r2, int max_nb,
                                                     int loop, PbcArgs pbc, int* __restrict__ counts,
                                                     const int64_t* __restrict__ rowptr, int64_t* __restrict__ src,
                                                     int64_t* __restrict__ dst, float* __restrict__ shifts) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const int g = node_graph[i];
  const int j0 = gptr[g], j1 = gptr[g + 1];
  const float xi = pos[3 * i], yi = pos[3 * i + 1], zi = pos[3 * i + 2];
  int rx = 0, ry = 0, rz = 0;
  float c[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (pbc.cell) {
    rx = pbc.reps[3 * g];
    ry = pbc.reps[3 * g + 1];
    rz = pbc.reps[3 * g + 2];
#pragma unroll
    for (int t = 0; t < 9; ++t) c[t] = pbc.cell[9 * g + t];
  }
  int cnt = 0;
  const int64_t base = FILL ? rowptr[i] : 0;
  // nearest policy: distance-sorted insertion list of (d2, j, image)
  float nd[NEAREST ? kMaxNearest : 1];
  int nj[NEAREST ? kMaxNearest : 1];
  int ns[NEAREST ? kMaxNearest : 1];
  int nn = 0;
  for (int a = -rx; a <= rx; ++a)
    for (int b = -ry; b <= ry; ++b)
      for (int e = -rz; e <= rz; ++e) {
        const float sx = a * c[0] + b * c[3] + e * c[6];
        const float sy = a * c[1] + b * c[4] + e * c[7];
        const float sz = a * c[2] + b * c[5] + e * c[8];
        const bool zero_img = (a == 0 && b == 0 && e == 0);
        const int img = ((a + rx) * (2 * ry + 1) + (b + ry)) * (2 * rz + 1) + (e + rz);
        for (int j = j0; j < j1; ++j) {
          if (!loop && zero_img && j == i) continue;
          const float dx = xi - (pos[3 * j] + sx), dy = yi - (pos[3 * j + 1] + sy), dz = zi - (pos[3 * j + 2] + sz);
          const float d2 = dx * dx + dy * dy + dz * dz;
          if (d2 > r2) continue;
          if constexpr (NEAREST) {
            if (nn == max_nb && d2 >= nd[nn - 1]) continue;
            int p = nn < max_nb ? nn++ : nn - 1;
            while (p > 0 && nd[p - 1] > d2) {
              nd[p] = nd[p - 1];
              nj[p] = nj[p - 1];
              ns[p] = ns[p - 1];
              --p;
            }
            nd[p] = d2;
            nj[p] = j;
            ns[p] = img;
          } else {
            if (cnt >= max_nb) continue;
            if constexpr (FILL) {
              src[base + cnt] = j;
              dst[base + cnt] = i;
              if (shifts) {  // vec = pos[dst] - pos[src] + shift  ->  shift = -(image shift)
                shifts[3 * (base + cnt)] = -sx;
                shifts[3 * (base + cnt) + 1] = -sy;
                shifts[3 * (base + cnt) + 2] = -sz;
              }
            }
            ++cnt;
          }
        }
      }
  if constexpr (NEAREST) {
    cnt = nn;
    if constexpr (FILL) {
      for (int t = 0; t < nn; ++t) {
        const int img = ns[t];
        const int e = img % (2 * rz + 1) - rz, b = (img / (2 * rz + 1)) % (2 * ry + 1) - ry,
                  a = img / ((2 * rz + 1) * (2 * ry + 1)) - rx;
        src[base + t] = nj[t];
        dst[base + t] = i;
        if (shifts) {
          shifts[3 * (base + t)] = -(a * c[0] + b * c[3] + e * c[6]);
          shifts[3 * (base + t) + 1] = -(a * c[1] + b * c[4] + e * c[7]);
          shifts[3 * (base + t) + 2] = -(a * c[2] + b * c[5] + e * c[8]);
        }
      }
    }
  }
  if constexpr (!FILL) counts[i] = cnt;
}

// returns (edge_index int64 [2, E] (row 0 = source), shifts f32 [E, 3] (empty if no cell))
std::tuple<at::Tensor, at::Tensor> radius_graph(const at::Tensor& pos_, const at::Tensor& node_graph,
                                                const at::Tensor& gptr, double r, int64_t max_nb, bool loop,
                                                bool nearest, const c10::optional<at::Tensor>& cell,
                                                const c10::optional<at::Tensor>& reps) {
  HY_CHECK_CUDA(pos_);
  auto pos = pos_.to(at::kFloat).contiguous();
  HY_CHECK(pos.dim() == 2 && pos.size(1) == 3, "pos must be [N, 3]");
  HY_CHECK_I32(node_graph);
  HY_CHECK_I32(gptr);
  HY_CHECK(!nearest || (max_nb > 0 && max_nb <= kMaxNearest),
           "nearest cap policy supports 0 < max_num_neighbors <= ", kMaxNearest);
  const int N = (int)pos.size(0);
  HY_CHECK(node_graph.numel() == N, "node_graph must have one entry per node");
  auto i64 = pos.options().dtype(at::kLong);
  const int cap = (int)std::min<int64_t>(max_nb > 0 ? max_nb : INT32_MAX, INT32_MAX);
  PbcArgs pbc{nullptr, nullptr};
  at::Tensor cellc, repsc;
  if (cell.has_value() && cell->defined()) {
    HY_CHECK(reps.has_value() && reps->defined(), "periodic radius graph needs reps");
    cellc = cell->to(at::kFloat).contiguous();
    repsc = reps->to(at::kInt).contiguous();
    HY_CHECK(cellc.numel() == 9 * (gptr.numel() - 1) && repsc.numel() == 3 * (gptr.numel() - 1),
             "cell must be [G, 3, 3] and reps [G, 3]");
    pbc = PbcArgs{cellc.data_ptr<float>(), repsc.data_ptr<int>()};
  }
  if (N == 0) return {at::empty({2, 0}, i64), at::empty({0, 3}, pos.options())};
  auto counts = at::empty({N}, pos.options().dtype(at::kInt));
  const float r2 = (float)(r * r);
  const int blocks = ceil_div(N, 256);
  const float* P = pos.data_ptr<float>();
  const int* NG = node_graph.data_ptr<int>();
  const int* GP = gptr.data_ptr<int>();
  const int lp = loop ? 1 : 0;
  if (nearest)
    radius_kernel<false, true><<<blocks, 256, 0, stream()>>>(P, NG, GP, N, r2, cap, lp, pbc, counts.data_ptr<int>(),
                                                             nullptr, nullptr, nullptr, nullptr);
  else
    radius_kernel<false, false><<<blocks, 256, 0, stream()>>>(P, NG, GP, N, r2, cap, lp, pbc, counts.data_ptr<int>(),
                                                              nullptr, nullptr, nullptr, nullptr);
  auto rowptr = at::zeros({N + 1}, i64);
  rowptr.narrow(0, 1, N).copy_(at::cumsum(counts, 0));
  const int64_t E = rowptr[N].item<int64_t>();  // host sync: the output size is data dependent
  auto ei = at::empty({2, E}, i64);
  at::Tensor sh = pbc.cell ? at::empty({E, 3}, pos.options()) : at::empty({0, 3}, pos.options());
  if (E > 0) {
    int64_t* s = ei.data_ptr<int64_t>();
    float* shp = pbc.cell ? sh.data_ptr<float>() : nullptr;
    if (nearest)
      radius_kernel<true, true><<<blocks, 256, 0, stream()>>>(P, NG, GP, N, r2, cap, lp, pbc, nullptr,
                                                              rowptr.data_ptr<int64_t>(), s, s + E, shp);
    else
      radius_kernel<true, false><<<blocks, 256, 0, stream()>>>(P, NG, GP, N, r2, cap, lp, pbc, nullptr,
                                                               rowptr.data_ptr<int64_t>(), s, s + E, shp);
  }
  return {ei, sh};
}

// ------------------------------------------------------------------ triplets
template <bool FILL>
__global__ void __launch_bounds__(256) triplet_kernel(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                      const int* __restrict__ rowptr, int64_t E,
                                                      int64_t* __restrict__ counts, const int64_t* __restrict__ tptr,
                                                      int64_t* __restrict__ idx_kj, int64_t* __restrict__ idx_ji) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int64_t j = src[e], i = dst[e];
  const int b = rowptr[j], en = rowptr[j + 1];
  int64_t c = 0;
  const int64_t o = FILL ? tptr[e] : 0;
  for (int k = b; k < en; ++k) {
    if (src[k] == i) continue;  // k != i
    if constexpr (FILL) {
      idx_kj[o + c] = k;
      idx_ji[o + c] = e;
    }
    ++c;
  }
  if constexpr (!FILL) counts[e] = c;
}

// edge_index [2, E] destination-sorted with CSR rowptr (int32 [N+1]) -> (idx_kj, idx_ji) int64
std::tuple<at::Tensor, at::Tensor> triplets(const at::Tensor& edge_index, const at::Tensor& rowptr) {
  HY_CHECK_CUDA(edge_index);
  HY_CHECK_I32(rowptr);
  auto ei = edge_index.to(at::kLong).contiguous();
  HY_CHECK(ei.dim() == 2 && ei.size(0) == 2, "edge_index must be [2, E]");
  const int64_t E = ei.size(1);
  auto o = ei.options();
  if (E == 0) return {at::empty({0}, o), at::empty({0}, o)};
  const int64_t* s = ei.data_ptr<int64_t>();
  auto counts = at::empty({E}, o);
  const int blocks = ceil_div(E, 256);
  triplet_kernel<false><<<blocks, 256, 0, stream()>>>(s, s + E, rowptr.data_ptr<int>(), E,
                                                      counts.data_ptr<int64_t>(), nullptr, nullptr, nullptr);
  auto tptr = at::zeros({E + 1}, o);
  tptr.narrow(0, 1, E).copy_(at::cumsum(counts, 0));
  const int64_t T = tptr[E].item<int64_t>();
  auto kj = at::empty({T}, o), ji = at::empty({T}, o);
  if (T > 0)
    triplet_kernel<true><<<blocks, 256, 0, stream()>>>(s, s + E, rowptr.data_ptr<int>(), E, nullptr,
                                                       tptr.data_ptr<int64_t>(), kj.data_ptr<int64_t>(),
                                                       ji.data_ptr<int64_t>());
  return {kj, ji};
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def(
      "radius_graph(Tensor pos, Tensor node_graph, Tensor gptr, float r, int max_nb, bool loop, bool nearest, "
      "Tensor? cell, Tensor? reps) -> (Tensor, Tensor)");
  m.def("triplets(Tensor edge_index, Tensor rowptr) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("radius_graph", hy::radius_graph);
  m.impl("triplets", hy::triplets);
}
