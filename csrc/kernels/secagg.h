#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace idc {

// Additive-mask secure aggregation (north-star replacement of Paillier):
//   out[i] = q(x[i]) + sum_{j != rank} sign(rank, j) * PRF(seed, min, max, round, i)   (mod 2^32)
// q = round(clamp(x*scale)) as two's-complement uint32.  Summed over all clients (an RCCL uint32
// SUM all-reduce, which wraps mod 2^32) the masks cancel EXACTLY and only the fixed-point sum is
// revealed.  `alive` is the bitmask of participating clients (<= 64): a client that dropped out
// before masking is excluded from every pair, so the survivors' masks still cancel (re-keyed round).
hipError_t secagg_quantize_mask(const float* x, uint32_t* out, long long n, float scale, float clip,
                                int nclients, int rank, unsigned long long seed, unsigned long long round_,
                                unsigned long long alive, hipStream_t st);
hipError_t secagg_dequantize(const uint32_t* sum, float* out, long long n, float scale, int nclients,
                             float divisor, hipStream_t st);

}  // namespace idc
