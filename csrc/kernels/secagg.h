#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace idc {

// Additive-mask secure aggregation (north-star replacement of Paillier):
//   out[i] = q(x[i]) + sum_{j != rank, alive} sign(rank, j) * Philox(key_j; round, i)   (mod 2^32)
// q = round(clamp(x * scale_s)) as two's-complement uint32, with scale_s the fixed-point scale of
// the segment (protected weight tensor) element i belongs to: segment s covers
// [seg_end[s-1], seg_end[s]).  key_j = keys[2j], keys[2j+1] is the pair key this client shares with
// client j (derived from a Diffie-Hellman secret on the host, fed/keyagree.py; the aggregator
// cannot compute it).  Summed over all clients (an RCCL int32 SUM all-reduce, which wraps mod 2^32)
// the masks cancel EXACTLY and only the fixed-point sum is revealed.  `alive` is the bitmask of
// participating clients (<= 64): a client that dropped out before masking is excluded from every
// pair, so the survivors' masks still cancel (re-keyed round).  `accumulate`: out[i] += value
// instead of out[i] = value (a rank's running masked sum over its clients).
hipError_t secagg_quantize_mask(const float* x, uint32_t* out, long long n, const float* seg_scale,
                                const long long* seg_end, int nseg, float clip, int nclients, int rank,
                                const uint32_t* keys, unsigned long long round_, unsigned long long alive,
                                hipStream_t st, int accumulate = 0);
// out[i] = (int32)sum[i] / (scale_s * divisor)
// max |x| per segment, merged into out[] (float bits, zero-initialised by the caller)
hipError_t secagg_absmax(const float* x, long long n, const long long* seg_end, int nseg, unsigned* out,
                         hipStream_t st);
hipError_t secagg_dequantize(const uint32_t* sum, float* out, long long n, const float* seg_scale,
                             const long long* seg_end, int nseg, float divisor, hipStream_t st);

}  // namespace idc
