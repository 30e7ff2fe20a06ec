// One-launch mini-batch assembly from the HBM-resident dataset pool
// (``data/device_store.py``; replaces PyG ``Batch.from_data_list`` + H2D of the
// reference, ``train_validate_test.py:514``).
//
// Input: the packed int32 plan built on the host (node rows, edge rows, CSR
// arrays, batch, graph ptr, sample ids, [N, G, E] scalars) and the pool tensors.
// One kernel writes every per-batch tensor: node fields (x, pos, pe, forces,
// node targets) gathered by node row, edge fields (edge_attr, rel_pe, shifts)
// by edge row, graph fields (energy, graph targets) by sample id; padded rows
// are zeroed (padded nodes get distinct finite positions so padded edges never
// have zero length); plus the int64 edge_index / batch / ptr and the node and
// graph masks.  Before: ~45 small torch launches per step (index_select, mask
// multiplies, casts, stack), ~0.2 ms of a 2.8 ms step.
#include "common.h"

namespace hy {

constexpr int kAsmMaxFields = 8;

struct AsmFields {
  const float* src[kAsmMaxFields];
  float* dst[kAsmMaxFields];
  int width[kAsmMaxFields];
  int n;
};

struct AsmArgs {
  AsmFields node, edge, graph;
  const int* node_rows;
  const int* edge_rows;
  const int* src;
  const int* dst;
  const int* batch;
  const int* gptr;
  const int* sidx;
  const int* scal;
  int64_t* edge_index;  // [2, Ep]
  int64_t* batch_l;     // [Np]
  int64_t* ptr_l;       // [Gp+1]
  bool* nmask;          // [Np]
  bool* gmask;          // [Gp]
  int Np, Ep, Gp, padded, pos_field;
};

__device__ __forceinline__ void copy_row(const AsmFields& F, int out_row, int in_row, bool valid) {
  const int r = valid ? in_row : 0;
  for (int f = 0; f < F.n; ++f) {
    const int w = F.width[f];
    const float* s = F.src[f] + (int64_t)r * w;
    float* d = F.dst[f] + (int64_t)out_row * w;
    for (int c = 0; c < w; ++c) d[c] = valid ? s[c] : 0.f;
  }
}

__global__ void __launch_bounds__(256) assemble_kernel(AsmArgs a) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int stride = gridDim.x * blockDim.x;
  const int nvalid = a.scal[0], gvalid = a.scal[1];
  // nodes
  for (int n = tid; n < a.Np; n += stride) {
    const int row = a.node_rows[n];
    const bool valid = !a.padded || row >= 0;
    copy_row(a.node, n, row, valid);
    if (!valid && a.pos_field >= 0) {
      float* d = a.node.dst[a.pos_field] + (int64_t)n * a.node.width[a.pos_field];
      d[0] = 2.f * ((float)(n - nvalid) + 1.f);
    }
    a.nmask[n] = valid;
    a.batch_l[n] = a.batch[n];
  }
  // edges
  for (int e = tid; e < a.Ep; e += stride) {
    const int row = a.edge_rows[e];
    copy_row(a.edge, e, row, !a.padded || row >= 0);
    a.edge_index[e] = a.src[e];
    a.edge_index[(int64_t)a.Ep + e] = a.dst[e];
  }
  // graphs
  for (int g = tid; g <= a.Gp; g += stride) {
    a.ptr_l[g] = a.gptr[g];
    if (g == a.Gp) break;
    const bool valid = !a.padded || g < gvalid;
    copy_row(a.graph, g, a.sidx[g], valid);
    a.gmask[g] = valid;
  }
}

static void fill_fields(AsmFields& F, at::TensorList src, std::vector<at::Tensor>& outs, int64_t rows) {
  HY_CHECK((int)src.size() <= kAsmMaxFields, "store_assemble: too many fields");
  F.n = (int)src.size();
  for (int f = 0; f < F.n; ++f) {
    const auto& t = src[f];
    HY_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.dim() == 2,
             "store_assemble: pool fields must be contiguous 2-D fp32");
    auto o = at::empty({rows, t.size(1)}, t.options());
    F.src[f] = t.data_ptr<float>();
    F.dst[f] = o.data_ptr<float>();
    F.width[f] = (int)t.size(1);
    outs.push_back(o);
  }
}

std::vector<at::Tensor> store_assemble(const at::Tensor& plan, int64_t Np, int64_t Ep, int64_t Gp, bool padded,
                                       at::IntArrayRef offs, at::TensorList node_src, at::TensorList edge_src,
                                       at::TensorList graph_src, int64_t pos_field) {
  HY_CHECK_CUDA(plan);
  HY_CHECK_I32(plan);
  HY_CHECK(offs.size() == 13, "store_assemble: 13 plan offsets");
  AsmArgs a{};
  std::vector<at::Tensor> outs;
  fill_fields(a.node, node_src, outs, Np);
  fill_fields(a.edge, edge_src, outs, Ep);
  fill_fields(a.graph, graph_src, outs, Gp);
  auto li = plan.options().dtype(at::kLong);
  auto edge_index = at::empty({2, Ep}, li);
  auto batch_l = at::empty({Np}, li);
  auto ptr_l = at::empty({Gp + 1}, li);
  auto nmask = at::empty({Np}, plan.options().dtype(at::kBool));
  auto gmask = at::empty({Gp}, plan.options().dtype(at::kBool));
  const int* p = plan.data_ptr<int>();
  a.node_rows = p + offs[0];
  a.edge_rows = p + offs[1];
  a.src = p + offs[2];
  a.dst = p + offs[3];
  a.batch = p + offs[7];
  a.gptr = p + offs[8];
  a.sidx = p + offs[11];
  a.scal = p + offs[12];
  a.edge_index = edge_index.data_ptr<int64_t>();
  a.batch_l = batch_l.data_ptr<int64_t>();
  a.ptr_l = ptr_l.data_ptr<int64_t>();
  a.nmask = nmask.data_ptr<bool>();
  a.gmask = gmask.data_ptr<bool>();
  a.Np = (int)Np;
  a.Ep = (int)Ep;
  a.Gp = (int)Gp;
  a.padded = padded ? 1 : 0;
  a.pos_field = (int)pos_field;
  const int64_t work = std::max<int64_t>(std::max(Np, Ep), Gp + 1);
  const int blocks = (int)std::min<int64_t>(std::max<int64_t>(1, ceil_div(work, 256)), 2048);
  assemble_kernel<<<blocks, 256, 0, stream()>>>(a);
  outs.push_back(edge_index);
  outs.push_back(batch_l);
  outs.push_back(ptr_l);
  outs.push_back(nmask);
  outs.push_back(gmask);
  return outs;
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def(
      "store_assemble(Tensor plan, int Np, int Ep, int Gp, bool padded, int[] offs, Tensor[] node_src, "
      "Tensor[] edge_src, Tensor[] graph_src, int pos_field) -> Tensor[]");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) { m.impl("store_assemble", hy::store_assemble); }
