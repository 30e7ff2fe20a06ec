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

// ------------------------------------------------------------------------------------
// Device-side batch plan (the captured step's per-step upload shrinks from the whole packed
// plan, ~0.6 MB for an OC20 batch, to the G sample ids): the same 13 arrays, with the same
// values, as the host builder (csrc/collate.cpp store_plan), expanded from per-sample tables
// that live in HBM with the dataset:
//   nn, ne [S]; noff, eoff [S]; sl, dl, pl [E_tot] (local src / dst / src-sort permutation);
//   dcum, scum [N_tot] (per-sample local dst- / src-CSR row starts).
// Every workgroup scans the G per-graph node / edge counts in LDS (G <= kPlanMaxG), then
// threads fill a flat index over nodes, edges and graphs; padded nodes / edges follow the
// host's closed forms (padded edge j: dst = N + floor(j pn / pe), src = N + (that + 1) mod pn,
// stable source order by counting).
constexpr int kPlanMaxG = 4096;
struct PlanTabs {
  const int *nn, *ne, *noff, *eoff, *sl, *dl, *pl, *dcum, *scum;
};
struct PlanOut {
  int *node_rows, *erows, *src, *dst, *sperm, *rowptr, *srowptr, *batch, *gptr, *aseg_id, *aseg_ptr, *sidx, *scal;
};

__device__ __forceinline__ int64_t ceil_q(int64_t a, int64_t b) { return (a + b - 1) / b; }

__global__ void __launch_bounds__(256) plan_expand_kernel(const int* __restrict__ seed, PlanTabs t, PlanOut o, int Np,
                                                          int Ep, int Gp, int padded, int batch_scope,
                                                          int64_t* __restrict__ rng) {
  __shared__ int pn[kPlanMaxG + 1], pe[kPlanMaxG + 1];
  // the step's dropout-counter advance rides along (ops/rng.py fold_next_advance)
  if (rng != nullptr && blockIdx.x == 0 && threadIdx.x == 0) rng[0] += 1;
  const int G = seed[0];
  const int* idx = seed + 1;
  for (int g = threadIdx.x; g < G; g += 256) {
    const int s = idx[g];
    pn[g + 1] = t.nn[s];
    pe[g + 1] = t.ne[s];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int a = 0, b = 0;
    pn[0] = 0;
    pe[0] = 0;
    for (int g = 1; g <= G; ++g) {
      a += pn[g];
      b += pe[g];
      pn[g] = a;
      pe[g] = b;
    }
  }
  __syncthreads();
  const int N = pn[G], E = pe[G];
  const int64_t pnn = (int64_t)Np - N, pee = (int64_t)Ep - E;
  // padded-edge counts below a padded node offset q (closed forms of the host's bincounts)
  auto dcount = [&](int64_t q) -> int64_t { return pee > 0 ? ceil_q(q * pee, pnn) : 0; };  // dst < N + q
  auto scount = [&](int64_t q) -> int64_t {  // src < N + q
    if (pee == 0 || q <= 0) return 0;
    return dcount(q - 1) + (pee - dcount(pnn - 1));
  };
  auto find = [&](const int* ptr, int v) {  // g with ptr[g] <= v < ptr[g + 1]
    int lo = 0, hi = G;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (ptr[mid] <= v) lo = mid; else hi = mid;
    }
    return lo;
  };
  const int64_t total = (int64_t)Np + Ep + Gp + 1;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < total; q += (int64_t)gridDim.x * 256) {
    if (q < Np) {
      const int n = (int)q;
      if (n < N) {
        const int g = find(pn, n), s = idx[g], r = n - pn[g], nr = t.noff[s] + r;
        o.node_rows[n] = nr;
        o.batch[n] = g;
        o.rowptr[n] = pe[g] + t.dcum[nr];
        o.srowptr[n] = pe[g] + t.scum[nr];
        o.aseg_id[n] = batch_scope ? 0 : g;
      } else {
        const int64_t qq = n - N;
        o.node_rows[n] = -1;
        o.batch[n] = G;
        o.rowptr[n] = (int)(E + dcount(qq));
        o.srowptr[n] = (int)(E + scount(qq));
        o.aseg_id[n] = batch_scope ? 1 : G;
      }
    } else if (q < (int64_t)Np + Ep) {
      const int k = (int)(q - Np);
      if (k < E) {
        const int g = find(pe, k), s = idx[g], er = t.eoff[s] + (k - pe[g]);
        o.erows[k] = er;
        o.src[k] = t.sl[er] + pn[g];
        o.dst[k] = t.dl[er] + pn[g];
        o.sperm[k] = t.pl[er] + pe[g];
      } else {
        const int64_t j = k - E, pd = j * pnn / pee;
        o.erows[k] = -1;
        o.dst[k] = (int)(N + pd);
        o.src[k] = (int)(N + (pd + 1) % pnn);
        // the j-th padded edge in source order: its source bucket qb (scount(qb) <= j), then the
        // bucket's edges in index order (those with pd == qb - 1 mod pn)
        int64_t lo = 0, hi = pnn;
        while (hi - lo > 1) {
          const int64_t mid = (lo + hi) >> 1;
          if (scount(mid) <= j) lo = mid; else hi = mid;
        }
        const int64_t pdb = lo == 0 ? pnn - 1 : lo - 1;
        o.sperm[k] = (int)(E + dcount(pdb) + (j - scount(lo)));
      }
    } else {
      const int g = (int)(q - Np - Ep);
      const int v = g <= G ? pn[g] : Np;
      o.gptr[g] = v;
      if (!batch_scope) o.aseg_ptr[g] = v;
      if (g < Gp) o.sidx[g] = g < G ? idx[g] : 0;
      if (g == 0) {
        o.rowptr[Np] = Ep;
        o.srowptr[Np] = Ep;
        if (batch_scope) {
          o.aseg_ptr[0] = 0;
          o.aseg_ptr[1] = N;
          o.aseg_ptr[2] = Np;
        }
        o.scal[0] = N;
        o.scal[1] = G;
        o.scal[2] = E;
        o.scal[3] = 0;
      }
    }
  }
}

// out: the packed plan [13 segments] of a (Np, Ep, Gp) layout; seed: [G, idx[0..G)] (int32,
// device); tabs: nn, ne, noff, eoff, sl, dl, pl, dcum, scum (int32, device)
void store_plan_expand(const at::Tensor& seed, at::TensorList tabs, at::Tensor out, int64_t Np, int64_t Ep, int64_t Gp,
                       bool padded, bool batch_scope, const c10::optional<at::Tensor>& rng) {
  int64_t* rp = nullptr;
  if (rng.has_value() && rng->defined()) {
    HY_CHECK(rng->is_cuda() && rng->scalar_type() == at::kLong && rng->numel() >= 1, "store_plan_expand: rng int64");
    rp = rng->data_ptr<int64_t>();
  }
  // seed: a device tensor, or the pinned host buffer itself (zero-copy: the kernel reads the
  // ids over the host link, which saves the step graph its H2D copy node)
  HY_CHECK(seed.scalar_type() == at::kInt && seed.is_contiguous(), "store_plan_expand: int32 seed");
  const int* seed_ptr = nullptr;
  if (seed.is_cuda()) {
    seed_ptr = seed.data_ptr<int>();
  } else {
    HY_CHECK(seed.is_pinned(), "store_plan_expand: a host seed must be pinned");
    void* dp = nullptr;
    HY_CHECK(hipHostGetDevicePointer(&dp, seed.data_ptr(), 0) == hipSuccess && dp != nullptr,
             "store_plan_expand: pinned seed is not device-mapped");
    seed_ptr = static_cast<const int*>(dp);
  }
  HY_CHECK_I32(out);
  HY_CHECK(tabs.size() == 9, "store_plan_expand: 9 per-sample tables");
  for (const auto& x : tabs) HY_CHECK(x.is_cuda() && x.scalar_type() == at::kInt && x.is_contiguous(),
                                      "store_plan_expand: int32 device tables");
  HY_CHECK(Gp <= kPlanMaxG && seed.numel() >= Gp + 1 && out.is_contiguous(), "store_plan_expand: Gp / seed size");
  const int64_t na = batch_scope ? 3 : Gp + 1;
  const int64_t sizes[13] = {Np, Ep, Ep, Ep, Ep, Np + 1, Np + 1, Np, Gp + 1, Np, na, Gp, 4};
  int64_t tot = 0;
  for (int k = 0; k < 13; ++k) tot += sizes[k];
  HY_CHECK(out.numel() >= tot, "store_plan_expand: out smaller than the layout");
  int* p = out.data_ptr<int>();
  int* v[13];
  for (int k = 0; k < 13; ++k) {
    v[k] = p;
    p += sizes[k];
  }
  PlanTabs t{tabs[0].data_ptr<int>(), tabs[1].data_ptr<int>(), tabs[2].data_ptr<int>(), tabs[3].data_ptr<int>(),
             tabs[4].data_ptr<int>(), tabs[5].data_ptr<int>(), tabs[6].data_ptr<int>(), tabs[7].data_ptr<int>(),
             tabs[8].data_ptr<int>()};
  PlanOut o{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], v[9], v[10], v[11], v[12]};
  const int64_t work = Np + Ep + Gp + 1;
  const int blocks = (int)std::min<int64_t>(ceil_div(work, (int64_t)256), 1024);
  plan_expand_kernel<<<blocks, 256, 0, stream()>>>(seed_ptr, t, o, (int)Np, (int)Ep, (int)Gp,
                                                   padded ? 1 : 0, batch_scope ? 1 : 0, rp);
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def(
      "store_assemble(Tensor plan, int Np, int Ep, int Gp, bool padded, int[] offs, Tensor[] node_src, "
      "Tensor[] edge_src, Tensor[] graph_src, int pos_field) -> Tensor[]");
  m.def(
      "store_plan_expand(Tensor seed, Tensor[] tabs, Tensor(a!) out, int Np, int Ep, int Gp, bool padded, "
      "bool batch_scope, Tensor(b!)? rng=None) -> ()");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("store_assemble", hy::store_assemble);
  m.impl("store_plan_expand", hy::store_plan_expand);
}
