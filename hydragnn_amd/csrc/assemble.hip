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

// Field copies: ONE flat element index over every (field, row, column) of the batch, so
// each thread issues its 4 gathers (row index, then value) together regardless of which
// field they fall in.  (Row-per-thread copies were a chain of dependent load -> store
// pairs, ~20 us per step for the OC20 batch on MI355X; field-by-field element loops still
// paid one L2 round trip per field, ~24 us.)
constexpr int kAsmMaxSegs = 3 * kAsmMaxFields;
constexpr int kAsmDevValid = -2;
struct AsmSeg {
  const float* src;
  float* dst;
  const int* rows;  // output row -> pool row (< 0: padding)
  int width;
  int nvalid;       // rows >= nvalid are padding; kAsmDevValid: the device's valid-graph count
  int padpos;       // >= 0: position field, padding rows get distinct finite positions
  int64_t count;    // elements (rows x width)
  int blk0;         // first workgroup of this segment
};

struct AsmArgs {
  AsmSeg seg[kAsmMaxSegs];
  int nseg;
  int seg_blocks;  // workgroups [0, seg_blocks) copy fields; the rest write masks and indices
  const int* node_rows;
  const int* src;
  const int* dst;
  const int* batch;
  const int* gptr;
  const int* scal;
  int64_t* edge_index;  // [2, Ep]
  int64_t* batch_l;     // [Np]
  int64_t* ptr_l;       // [Gp+1]
  bool* nmask;          // [Np]
  bool* gmask;          // [Gp]
  int Np, Ep, Gp, padded;
};

__device__ __forceinline__ float asm_elem(const AsmSeg& g, int64_t q, int nvalid, int gvalid) {
  const int r = (int)(q / g.width), c = (int)(q % g.width);
  const int row = g.rows[r];
  const int nv = g.nvalid == kAsmDevValid ? gvalid : g.nvalid;
  if (r < nv && row >= 0) return g.src[(int64_t)row * g.width + c];
  if (g.padpos >= 0 && c == 0) return 2.f * ((float)(r - nvalid) + 1.f);  // distinct finite padding positions
  return 0.f;
}

// Workgroups are assigned to segments on the host (blk0): the segment a workgroup serves is
// uniform across it, so its parameters are scalar loads (a per-lane search of the kernel-
// argument table compiles to per-lane loads from the kernarg segment, a memory round trip
// per probe).  Each thread copies kAsmPer elements, all loads issued before the stores.
constexpr int kAsmPer = 4;

__global__ void __launch_bounds__(256) assemble_kernel(AsmArgs a) {
  const int b = blockIdx.x;
  const int nvalid = a.scal[0], gvalid = a.scal[1];
  if (b < a.seg_blocks) {
    int k = 0;
    while (k + 1 < a.nseg && b >= a.seg[k + 1].blk0) ++k;
    const AsmSeg& g = a.seg[k];
    const int64_t e0 = (int64_t)(b - g.blk0) * 256 * kAsmPer + threadIdx.x;
    float v[kAsmPer];
#pragma unroll
    for (int u = 0; u < kAsmPer; ++u) {
      const int64_t e = e0 + (int64_t)u * 256;
      v[u] = e < g.count ? asm_elem(g, e, nvalid, gvalid) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kAsmPer; ++u) {
      const int64_t e = e0 + (int64_t)u * 256;
      if (e < g.count) g.dst[e] = v[u];
    }
    return;
  }
  const int tid = (b - a.seg_blocks) * 256 + threadIdx.x;
  const int stride = (gridDim.x - a.seg_blocks) * 256;
  for (int n = tid; n < a.Np; n += stride) {
    a.nmask[n] = !a.padded || a.node_rows[n] >= 0;
    a.batch_l[n] = a.batch[n];
  }
  for (int e = tid; e < a.Ep; e += stride) {
    a.edge_index[e] = a.src[e];
    a.edge_index[(int64_t)a.Ep + e] = a.dst[e];
  }
  for (int g = tid; g <= a.Gp; g += stride) {
    a.ptr_l[g] = a.gptr[g];
    if (g < a.Gp) a.gmask[g] = !a.padded || g < gvalid;
  }
}

static void add_segs(AsmArgs& a, at::TensorList src, std::vector<at::Tensor>& outs, int64_t rows,
                     const int* rowmap, int nvalid, int pos_field) {
  HY_CHECK((int)src.size() <= kAsmMaxFields, "store_assemble: too many fields");
  for (int f = 0; f < (int)src.size(); ++f) {
    const auto& t = src[f];
    HY_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.dim() == 2,
             "store_assemble: pool fields must be contiguous 2-D fp32");
    auto o = at::empty({rows, t.size(1)}, t.options());
    outs.push_back(o);
    if (rows == 0 || t.size(1) == 0) continue;
    AsmSeg& g = a.seg[a.nseg++];
    g.src = t.data_ptr<float>();
    g.dst = o.data_ptr<float>();
    g.rows = rowmap;
    g.width = (int)t.size(1);
    g.nvalid = nvalid;
    g.padpos = f == pos_field ? 1 : -1;
    g.count = rows * t.size(1);
    g.blk0 = a.seg_blocks;
    a.seg_blocks += (int)ceil_div(g.count, (int64_t)256 * kAsmPer);
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
  const int* p = plan.data_ptr<int>();
  const int all = 1 << 30;
  add_segs(a, node_src, outs, Np, p + offs[0], all, (int)pos_field);
  add_segs(a, edge_src, outs, Ep, p + offs[1], all, -1);
  add_segs(a, graph_src, outs, Gp, p + offs[11], padded ? kAsmDevValid : all, -1);
  auto li = plan.options().dtype(at::kLong);
  auto edge_index = at::empty({2, Ep}, li);
  auto batch_l = at::empty({Np}, li);
  auto ptr_l = at::empty({Gp + 1}, li);
  auto nmask = at::empty({Np}, plan.options().dtype(at::kBool));
  auto gmask = at::empty({Gp}, plan.options().dtype(at::kBool));
  a.node_rows = p + offs[0];
  a.src = p + offs[2];
  a.dst = p + offs[3];
  a.batch = p + offs[7];
  a.gptr = p + offs[8];
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
  const int64_t tail = std::max<int64_t>(std::max(Np, Ep), Gp + 1);
  const int blocks = a.seg_blocks + (int)std::min<int64_t>(std::max<int64_t>(1, ceil_div(tail, 256)), 1024);
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
