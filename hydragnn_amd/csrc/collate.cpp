// Host-side batch assembly (C++), the native counterpart of PyG's Batch.from_data_list +
// torch_sparse CSR construction that the reference's loaders call per batch
// (hydragnn/preprocess/load_data.py collate path).
//
//   collate_edges(eis, node_counts)  -> edge_index [2, E] int64 with per-sample node offsets
//                                       applied, one pass, no per-sample torch ops
//   csr_from_edges(src, dst, N)      -> (dst_rowptr, src_rowptr, src_perm) int32
//
// csr_from_edges replaces bincount + cumsum + argsort(stable) with two O(E) counting
// passes; src_perm is the stable order of edges by source (identical to
// torch.argsort(src, stable=True)).  dst_rowptr indexes the edges directly, so edges must
// be sorted by destination (collate keeps each sample's edges dst-sorted and node offsets
// increase, so a collated batch is).
#include <cstring>
#include <vector>

#include <ATen/ATen.h>
#include <torch/library.h>

namespace hy {

at::Tensor collate_edges(const std::vector<at::Tensor>& eis, const at::Tensor& node_counts) {
  TORCH_CHECK(node_counts.device().is_cpu() && node_counts.dim() == 1, "collate_edges: node_counts must be CPU [G]");
  const int64_t G = (int64_t)eis.size();
  TORCH_CHECK(node_counts.numel() == G, "collate_edges: one node count per sample");
  auto nc = node_counts.to(at::kLong).contiguous();
  const int64_t* ncp = nc.data_ptr<int64_t>();
  int64_t E = 0;
  for (const auto& e : eis) {
    TORCH_CHECK(e.device().is_cpu() && e.dim() == 2 && e.size(0) == 2, "collate_edges: edge_index must be CPU [2, E]");
    E += e.size(1);
  }
  auto out = at::empty({2, E}, at::TensorOptions().dtype(at::kLong));
  int64_t* o0 = out.data_ptr<int64_t>();
  int64_t* o1 = o0 + E;
  int64_t pos = 0, off = 0;
  for (int64_t g = 0; g < G; ++g) {
    auto e = eis[g].to(at::kLong).contiguous();
    const int64_t n = e.size(1);
    const int64_t* s = e.data_ptr<int64_t>();
    const int64_t* d = s + n;
    for (int64_t i = 0; i < n; ++i) {
      TORCH_CHECK(s[i] >= 0 && s[i] < ncp[g] && d[i] >= 0 && d[i] < ncp[g], "collate_edges: sample ", g,
                  " has an edge endpoint outside its ", ncp[g], " nodes");
      o0[pos + i] = s[i] + off;
      o1[pos + i] = d[i] + off;
    }
    pos += n;
    off += ncp[g];
  }
  return out;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> csr_from_edges(const at::Tensor& src_, const at::Tensor& dst_,
                                                             int64_t N) {
  TORCH_CHECK(src_.device().is_cpu() && dst_.device().is_cpu(), "csr_from_edges: CPU tensors expected");
  auto src = src_.to(at::kLong).contiguous(), dst = dst_.to(at::kLong).contiguous();
  const int64_t E = src.numel();
  TORCH_CHECK(dst.numel() == E, "csr_from_edges: src/dst length mismatch");
  TORCH_CHECK(N >= 0 && N < (int64_t(1) << 31) && E < (int64_t(1) << 31), "csr_from_edges: int32 index range");
  const int64_t* s = src.data_ptr<int64_t>();
  const int64_t* d = dst.data_ptr<int64_t>();
  auto i32 = at::TensorOptions().dtype(at::kInt);
  auto drow = at::zeros({N + 1}, i32), srow = at::zeros({N + 1}, i32), perm = at::empty({E}, i32);
  int32_t* dr = drow.data_ptr<int32_t>();
  int32_t* sr = srow.data_ptr<int32_t>();
  int32_t* pm = perm.data_ptr<int32_t>();
  for (int64_t i = 0; i < E; ++i) {
    TORCH_CHECK(s[i] >= 0 && s[i] < N && d[i] >= 0 && d[i] < N, "csr_from_edges: edge ", i, " outside [0, ", N, ")");
    ++dr[d[i] + 1];
    ++sr[s[i] + 1];
  }
  for (int64_t v = 0; v < N; ++v) {
    dr[v + 1] += dr[v];
    sr[v + 1] += sr[v];
  }
  std::vector<int32_t> cur(sr, sr + N);
  for (int64_t i = 0; i < E; ++i) pm[cur[s[i]]++] = (int32_t)i;
  return {drow, srow, perm};
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("collate_edges(Tensor[] eis, Tensor node_counts) -> Tensor", hy::collate_edges);
  m.def("csr_from_edges(Tensor src, Tensor dst, int N) -> (Tensor, Tensor, Tensor)", hy::csr_from_edges);
}
