// Multi-tensor fused AdamW / Adam step (gfx950).
//
// Replaces torch.optim.AdamW's per-parameter foreach kernels (reference optimizer
// selection: hydragnn/utils/optimizer/optimizer.py:12-40; DeepSpeed FusedLamb is
// the reference's only fused optimizer).  One launch updates every parameter:
// a host-built block table maps each 2048-element chunk to (tensor, offset); the
// step counter and learning rate live in device memory so the launch can be
// captured in a hipGraph once and replayed with a changing lr / step.
#include "common.h"

#include <map>
#include <mutex>
#include <utility>

namespace hy {

struct TensorRef {
  float* p;
  const float* g;
  float* m;
  float* v;
  int64_t n;
  float* step;        // this parameter's step count (device scalar, torch's per-param "step")
  const float* used;  // optional usage flag (> 0: the parameter took part in this step); a
                      // parameter with flag 0 is skipped entirely (value, moments, step), as
                      // torch optimizers skip grad-is-None parameters
};

constexpr int kChunk = 2048;

// state: [0] = unused, [1] = lr, [2] = number of steps skipped by the non-finite guard.
// Per-parameter step counts live in the TensorRefs; every block reads its tensor's count, and
// the LAST block to finish (an agent-scope ticket) advances them all — a separate increment
// launch was one more dependent kernel at the very end of every step.
// guard (optional): the step's loss; a NaN/Inf loss skips the whole update on the device
// (no host sync, capture-safe) and is counted in state[2] (SURVEY §5.3 step guard).
__device__ __forceinline__ bool guard_bad(const float* guard) { return guard && !isfinite(*guard); }

__global__ void __launch_bounds__(256) adamw_kernel(const TensorRef* __restrict__ refs,
                                                    const int2* __restrict__ blocks, float* __restrict__ state,
                                                    float beta1, float beta2, float eps, float wd, int adamw,
                                                    float grad_scale, const float* __restrict__ guard, int nt,
                                                    int has_skip, int* __restrict__ ticket) {
  const bool bad = guard_bad(guard);
  const int2 bt = blocks[blockIdx.x];
  const TensorRef r = refs[bt.x];
  if (!bad && !(r.used && !(*r.used > 0.f))) {
    const float step = *r.step + 1.f;  // this step's count (advanced by the last block)
    const float lr = state[1];
    const float bc1 = 1.f - powf(beta1, step);
    const float bc2 = 1.f - powf(beta2, step);
    const float step_size = lr / bc1;
    const float bc2s = sqrtf(bc2);
    const int64_t base = (int64_t)bt.y * kChunk;
    for (int i = threadIdx.x; i < kChunk; i += 256) {
      const int64_t k = base + i;
      if (k >= r.n) break;
      float g = r.g[k] * grad_scale;
      float p = r.p[k];
      if (adamw) p *= (1.f - lr * wd);
      else g += wd * p;
      const float m = beta1 * r.m[k] + (1.f - beta1) * g;
      const float v = beta2 * r.v[k] + (1.f - beta2) * g * g;
      r.m[k] = m;
      r.v[k] = v;
      const float denom = sqrtf(v) / bc2s + eps;
      r.p[k] = p - step_size * m / denom;
    }
  }
  // ticket: every block's step read happened above (its value fed the update, before the
  // barrier), so the last ticket orders the increments after every read.  No fences: nothing
  // written here is read by another block of this launch (a release fence per block was an
  // L2 write-back each, +7 us on the OC20 step)
  __shared__ int last;
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) {
    *ticket = 0;  // every ticket of this launch is drawn
    if (bad && has_skip) state[2] += 1.f;
  }
  if (bad) return;
  for (int t = threadIdx.x; t < nt; t += 256) {
    const TensorRef q = refs[t];
    if (q.used && !(*q.used > 0.f)) continue;
    *q.step += 1.f;
  }
}

void adamw_step(const at::Tensor& refs, const at::Tensor& blocks, const at::Tensor& state, double beta1,
                double beta2, double eps, double wd, bool adamw, double grad_scale,
                const c10::optional<at::Tensor>& guard) {
  const float* gp = nullptr;
  if (guard.has_value() && guard->defined()) {
    HY_CHECK(guard->is_cuda() && guard->scalar_type() == at::kFloat && guard->numel() == 1, "guard: fp32 scalar");
    gp = guard->data_ptr<float>();
  }
  HY_CHECK_CUDA(refs);
  HY_CHECK(refs.scalar_type() == at::kByte && refs.numel() % sizeof(TensorRef) == 0, "refs must be a TensorRef blob");
  HY_CHECK_I32(blocks);
  HY_CHECK_F32(state);
  const int nblocks = (int)(blocks.numel() / 2);
  if (nblocks == 0) return;
  // the ticket counter: persistent per (device, stream), reset by each launch's last block
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, at::Tensor> tickets;
  at::Tensor tk;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_pair((int)state.get_device(), stream());
    auto it = tickets.find(key);
    if (it == tickets.end()) it = tickets.emplace(key, at::zeros({1}, state.options().dtype(at::kInt))).first;
    tk = it->second;
  }
  const int nt = (int)(refs.numel() / (int64_t)sizeof(TensorRef));
  adamw_kernel<<<nblocks, 256, 0, stream()>>>(reinterpret_cast<const TensorRef*>(refs.data_ptr<uint8_t>()),
                                              reinterpret_cast<const int2*>(blocks.data_ptr<int>()),
                                              state.data_ptr<float>(), (float)beta1, (float)beta2, (float)eps,
                                              (float)wd, adamw ? 1 : 0, (float)grad_scale, gp, nt,
                                              state.numel() > 2 ? 1 : 0, tk.data_ptr<int>());
}

}  // namespace hy

TORCH_LIBRARY_FRAGMENT(hydra, m) {
  m.def(
      "adamw_step(Tensor refs, Tensor blocks, Tensor state, float beta1, float beta2, float eps, float wd, "
      "bool adamw, float grad_scale, Tensor? guard=None) -> ()");
}

TORCH_LIBRARY_IMPL(hydra, CUDA, m) { m.impl("adamw_step", hy::adamw_step); }
