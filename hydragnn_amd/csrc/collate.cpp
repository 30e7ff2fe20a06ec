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

// Packed int32 batch plan of the HBM-resident dataset store (data/device_store.py
// DeviceGraphStore.plan, the per-step host work of the captured training step): fills
//   [node_rows | edge_rows | src | dst | sperm | rowptr | srowptr | batch | gptr | aseg_id |
//    aseg_ptr | sample_idx | scalars]
// for the sample indices ``idx`` from per-sample offsets alone, with the padded layout of a
// static (Np, Ep, Gp) bucket.  Same values as the numpy reference in the store (which stays
// the CPU oracle of tests/test_device_store.py); ~15x faster (one pass per array, no
// temporaries: ~200 us of numpy per OC20 step was half the host's per-step budget).
namespace hy {

void store_plan(const at::Tensor& idx_, const at::Tensor& n_nodes_, const at::Tensor& n_edges_,
                const at::Tensor& node_off_, const at::Tensor& edge_off_, const at::Tensor& src_local_,
                const at::Tensor& dst_local_, const at::Tensor& sperm_local_, at::Tensor out, int64_t Np, int64_t Ep,
                int64_t Gp, bool padded, bool batch_scope) {
  for (const auto* t : {&idx_, &n_nodes_, &n_edges_, &node_off_, &edge_off_, &src_local_, &dst_local_, &sperm_local_})
    TORCH_CHECK(t->device().is_cpu() && t->scalar_type() == at::kLong && t->is_contiguous() && t->dim() == 1,
                "store_plan: int64 contiguous CPU vectors");
  TORCH_CHECK(out.device().is_cpu() && out.scalar_type() == at::kInt && out.is_contiguous(), "store_plan: int32 out");
  const int64_t G = idx_.numel();
  const int64_t* idx = idx_.data_ptr<int64_t>();
  const int64_t* nn = n_nodes_.data_ptr<int64_t>();
  const int64_t* ne = n_edges_.data_ptr<int64_t>();
  const int64_t* noff = node_off_.data_ptr<int64_t>();
  const int64_t* eoff = edge_off_.data_ptr<int64_t>();
  const int64_t* sl = src_local_.data_ptr<int64_t>();
  const int64_t* dl = dst_local_.data_ptr<int64_t>();
  const int64_t* pl = sperm_local_.data_ptr<int64_t>();
  const int64_t S = n_nodes_.numel();
  int64_t N = 0, E = 0;
  for (int64_t g = 0; g < G; ++g) {
    TORCH_CHECK(idx[g] >= 0 && idx[g] < S, "store_plan: sample index out of range");
    N += nn[idx[g]];
    E += ne[idx[g]];
  }
  TORCH_CHECK(N <= Np && E <= Ep && G <= Gp && (!padded || (N + 2 <= Np && G + 1 <= Gp)),
              "store_plan: batch exceeds the layout");
  const int64_t na = batch_scope ? 3 : Gp + 1;
  const int64_t sizes[13] = {Np, Ep, Ep, Ep, Ep, Np + 1, Np + 1, Np, Gp + 1, Np, na, Gp, 4};
  int64_t tot = 0;
  int32_t* v[13];
  for (int k = 0; k < 13; ++k) tot += sizes[k];
  TORCH_CHECK(out.numel() >= tot, "store_plan: out smaller than the layout");
  int32_t* o = out.data_ptr<int32_t>();
  for (int k = 0; k < 13; ++k) {
    v[k] = o;
    o += sizes[k];
  }
  int32_t *node_rows = v[0], *erows = v[1], *src = v[2], *dst = v[3], *sperm = v[4], *rowptr = v[5],
          *srowptr = v[6], *batch = v[7], *gptr = v[8], *aseg_id = v[9], *aseg_ptr = v[10], *sidx = v[11],
          *scal = v[12];
  int64_t pn_ = 0, pe_ = 0;
  for (int64_t g = 0; g < G; ++g) {
    const int64_t s = idx[g], n = nn[s], e = ne[s], nb = noff[s], eb = eoff[s];
    gptr[g] = (int32_t)pn_;
    sidx[g] = (int32_t)s;
    for (int64_t r = 0; r < n; ++r) {
      node_rows[pn_ + r] = (int32_t)(nb + r);
      batch[pn_ + r] = (int32_t)g;
    }
    for (int64_t r = 0; r < e; ++r) {
      const int64_t er = eb + r;
      erows[pe_ + r] = (int32_t)er;
      src[pe_ + r] = (int32_t)(sl[er] + pn_);
      dst[pe_ + r] = (int32_t)(dl[er] + pn_);
      sperm[pe_ + r] = (int32_t)(pl[er] + pe_);
    }
    pn_ += n;
    pe_ += e;
  }
  gptr[G] = (int32_t)N;
  if (padded) {
    for (int64_t r = N; r < Np; ++r) {
      node_rows[r] = -1;
      batch[r] = (int32_t)G;
    }
    for (int64_t r = E; r < Ep; ++r) erows[r] = -1;
    // padded edges spread evenly over the padded nodes (never self-loops), dst-sorted;
    // their source order is the stable counting sort of the sources
    const int64_t pn = Np - N, pe = Ep - E;
    if (pe > 0) {
      std::vector<int32_t> cnt(pn + 1, 0);
      for (int64_t k = 0; k < pe; ++k) {
        const int64_t pd = (k * pn) / pe, ps = (pd + 1) % pn;
        dst[E + k] = (int32_t)(N + pd);
        src[E + k] = (int32_t)(N + ps);
        ++cnt[ps + 1];
      }
      for (int64_t q = 0; q < pn; ++q) cnt[q + 1] += cnt[q];
      for (int64_t k = 0; k < pe; ++k) {
        const int64_t ps = src[E + k] - N;
        sperm[E + cnt[ps]++] = (int32_t)(E + k);
      }
    }
    for (int64_t g = G + 1; g <= Gp; ++g) gptr[g] = (int32_t)Np;
    for (int64_t g = G; g < Gp; ++g) sidx[g] = 0;
  }
  // CSR row pointers of the destination and source views (counting passes)
  std::memset(rowptr, 0, sizeof(int32_t) * (Np + 1));
  std::memset(srowptr, 0, sizeof(int32_t) * (Np + 1));
  for (int64_t k = 0; k < Ep; ++k) {
    ++rowptr[dst[k] + 1];
    ++srowptr[src[k] + 1];
  }
  for (int64_t q = 0; q < Np; ++q) {
    rowptr[q + 1] += rowptr[q];
    srowptr[q + 1] += srowptr[q];
  }
  if (batch_scope) {
    for (int64_t r = 0; r < Np; ++r) aseg_id[r] = r < N ? 0 : 1;
    aseg_ptr[0] = 0;
    aseg_ptr[1] = (int32_t)N;
    aseg_ptr[2] = (int32_t)Np;
  } else {
    std::memcpy(aseg_id, batch, sizeof(int32_t) * Np);
    std::memcpy(aseg_ptr, gptr, sizeof(int32_t) * (Gp + 1));
  }
  scal[0] = (int32_t)N;
  scal[1] = (int32_t)G;
  scal[2] = (int32_t)E;
  scal[3] = 0;
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("collate_edges(Tensor[] eis, Tensor node_counts) -> Tensor", hy::collate_edges);
  m.def("csr_from_edges(Tensor src, Tensor dst, int N) -> (Tensor, Tensor, Tensor)", hy::csr_from_edges);
  m.def(
      "store_plan(Tensor idx, Tensor n_nodes, Tensor n_edges, Tensor node_off, Tensor edge_off, Tensor src_local, "
      "Tensor dst_local, Tensor sperm_local, Tensor(a!) out, int Np, int Ep, int Gp, bool padded, bool batch_scope) -> ()",
      hy::store_plan);
}
