// Fused masked regression losses of a statically padded batch (gfx950).
//
// Reference loss path: Base.loss_hpweighted (hydragnn/models/Base.py:522-562) with the
// torch losses (mse / l1 / rmse / smooth_l1).  In the captured step the padded rows
// (dummy graph, padding atoms) are masked out; the torch composite of that
// (where, mul, sum, count, div, abs/sqrt, and their backward) was ~25 one-workgroup
// launches per head per step (~70 us on MI355X).  Here: one launch forward, one
// backward.  One 1024-thread workgroup: every thread accumulates its grid-stride
// elements in fp64, the block folds through LDS in a fixed order (deterministic).
#include "common.h"

namespace hy {

enum LossKind { kMSE = 0, kMAE = 1, kRMSE = 2, kSmoothL1 = 3 };

constexpr int kLossBlk = 1024;

__device__ __forceinline__ float loss_term(int kind, float d) {
  const float a = fabsf(d);
  switch (kind) {
    case kMAE: return a;
    case kSmoothL1: return a < 1.f ? 0.5f * d * d : a - 0.5f;
    default: return d * d;
  }
}

// out[0] = loss, out[1] = number of kept elements (as float)
__global__ void __launch_bounds__(kLossBlk) masked_loss_fwd_kernel(const float* __restrict__ pred,
                                                                   const float* __restrict__ target,
                                                                   const bool* __restrict__ mask, int64_t R, int C,
                                                                   int kind, float* __restrict__ out) {
  __shared__ double red[kLossBlk];
  __shared__ double cnt[kLossBlk];
  const int t = threadIdx.x;
  double s = 0.0, c = 0.0;
  const int64_t n = R * C;
  for (int64_t i = t; i < n; i += kLossBlk) {
    const bool keep = mask == nullptr || mask[i / C];
    if (keep) {
      s += (double)loss_term(kind, pred[i] - target[i]);
      c += 1.0;
    }
  }
  red[t] = s;
  cnt[t] = c;
  __syncthreads();
  for (int w = kLossBlk / 2; w > 0; w >>= 1) {
    if (t < w) {
      red[t] += red[t + w];
      cnt[t] += cnt[t + w];
    }
    __syncthreads();
  }
  if (t == 0) {
    const double den = cnt[0] > 0.0 ? cnt[0] : 1.0;
    double l = red[0] / den;
    if (kind == kRMSE) l = sqrt(l);
    out[0] = (float)l;
    out[1] = (float)cnt[0];
  }
}

// dpred = gout * dloss/dpred on kept rows, 0 elsewhere
__global__ void __launch_bounds__(256) masked_loss_bwd_kernel(const float* __restrict__ gout,
                                                              const float* __restrict__ pred,
                                                              const float* __restrict__ target,
                                                              const bool* __restrict__ mask,
                                                              const float* __restrict__ fwd, int64_t R, int C,
                                                              int kind, float* __restrict__ dpred) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= R * C) return;
  const bool keep = mask == nullptr || mask[i / C];
  float g = 0.f;
  if (keep) {
    const float den = fwd[1] > 0.f ? fwd[1] : 1.f;
    const float d = pred[i] - target[i];
    const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
    switch (kind) {
      case kMAE: g = sgn / den; break;
      case kSmoothL1: g = (fabsf(d) < 1.f ? d : sgn) / den; break;
      case kRMSE: g = fwd[0] > 0.f ? d / (den * fwd[0]) : 0.f; break;
      default: g = 2.f * d / den; break;
    }
    g *= gout[0];
  }
  dpred[i] = g;
}

static void loss_checks(const at::Tensor& pred, const at::Tensor& target, const c10::optional<at::Tensor>& mask) {
  HY_CHECK_CUDA(pred);
  HY_CHECK_F32(pred);
  HY_CHECK_F32(target);
  HY_CHECK(pred.is_contiguous() && target.is_contiguous() && pred.sizes() == target.sizes() && pred.dim() >= 1,
           "masked_loss: contiguous pred/target of equal shape");
  if (mask.has_value() && mask->defined())
    HY_CHECK(mask->scalar_type() == at::kBool && mask->numel() == pred.size(0) && mask->is_contiguous(),
             "masked_loss: bool mask with one entry per row");
}

// returns [loss, count]
at::Tensor masked_loss_fwd(const at::Tensor& pred, const at::Tensor& target, const c10::optional<at::Tensor>& mask,
                           int64_t kind) {
  loss_checks(pred, target, mask);
  HY_CHECK(kind >= 0 && kind <= 3, "masked_loss: unknown kind");
  const int64_t R = pred.size(0);
  const int C = (int)(R > 0 ? pred.numel() / R : 1);
  auto out = at::empty({2}, pred.options());
  const bool* mp = mask.has_value() && mask->defined() ? mask->data_ptr<bool>() : nullptr;
  masked_loss_fwd_kernel<<<1, kLossBlk, 0, stream()>>>(pred.data_ptr<float>(), target.data_ptr<float>(), mp, R, C,
                                                       (int)kind, out.data_ptr<float>());
  return out;
}

at::Tensor masked_loss_bwd(const at::Tensor& gout, const at::Tensor& pred, const at::Tensor& target,
                           const c10::optional<at::Tensor>& mask, const at::Tensor& fwd, int64_t kind) {
  loss_checks(pred, target, mask);
  HY_CHECK(gout.numel() == 1 && gout.scalar_type() == at::kFloat && fwd.numel() == 2, "masked_loss_bwd: scalars");
  auto g = gout.contiguous();
  const int64_t R = pred.size(0);
  const int C = (int)(R > 0 ? pred.numel() / R : 1);
  auto dpred = at::empty_like(pred);
  const int64_t n = pred.numel();
  if (n == 0) return dpred;
  const bool* mp = mask.has_value() && mask->defined() ? mask->data_ptr<bool>() : nullptr;
  masked_loss_bwd_kernel<<<ceil_div(n, 256), 256, 0, stream()>>>(g.data_ptr<float>(), pred.data_ptr<float>(),
                                                                 target.data_ptr<float>(), mp, fwd.data_ptr<float>(),
                                                                 R, C, (int)kind, dpred.data_ptr<float>());
  return dpred;
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def("masked_loss_fwd(Tensor pred, Tensor target, Tensor? mask, int kind) -> Tensor");
  m.def("masked_loss_bwd(Tensor gout, Tensor pred, Tensor target, Tensor? mask, Tensor fwd, int kind) -> Tensor");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) {
  m.impl("masked_loss_fwd", hy::masked_loss_fwd);
  m.impl("masked_loss_bwd", hy::masked_loss_bwd);
}
