// Counter-based hash dropout shared by the fused kernels (norm_fused.hip, gat.hip) and the
// standalone dropout op: keep(idx) = lowbias32(idx ^ seed) >= p * 2^24, where the seed mixes
// the device step counter (advanced by a captured kernel each step) with the call-site
// salt.  Masks are recomputed in the backward instead of stored.
#pragma once

#include "common.h"

namespace hy {

__device__ __forceinline__ uint32_t hash32(uint32_t x) {  // lowbias32 finaliser
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// keep-probability test for element idx: 24-bit uniform >= p
__device__ __forceinline__ bool keep_elem(uint32_t seed, uint32_t idx, uint32_t thresh) {
  return (hash32(idx ^ seed) >> 8) >= thresh;
}

struct DropCfg {
  uint32_t seed;
  uint32_t thresh;  // p * 2^24
  float scale;      // 1 / (1 - p)
  bool on;
};

__device__ __forceinline__ DropCfg drop_cfg(const int64_t* rng, int64_t salt, float p) {
  DropCfg d;
  d.on = rng != nullptr && p > 0.f;
  const uint64_t c = d.on ? (uint64_t)rng[0] : 0;
  d.seed = d.on ? hash32(hash32((uint32_t)c ^ hash32((uint32_t)(c >> 32) + 0x9E3779B9u)) + (uint32_t)salt * 0x85EBCA6Bu)
                : 0u;
  d.thresh = (uint32_t)(p * 16777216.f);
  d.scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  return d;
}

}  // namespace hy
