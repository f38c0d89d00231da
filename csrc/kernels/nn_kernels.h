#pragma once
#include "common.h"

namespace idc {

// dst = A_c*dz + B_c*x + C_c  (BatchNorm backward, coefficients from the saved statistics and the
// reductions sum(dZ), sum(dZ*xhat) accumulated by the producer of dz)
struct BnBwdApplyArgs {
  const bf16_t* dz; int lddz;
  const bf16_t* x; int ldx;
  BnArgs bn;
  const float* gsum; const float* gsumx;
  float inv_n;
  void* dst; int lddst;
  int dst_f32, accumulate;
  int M, C;
  int gsum_slots, gsum_ld;  // statistics slots of gsum/gsumx (common.h)
  float* fold_sum; float* fold_sumx;  // optional: block 0 adds the slot-summed gsum/gsumx here
};

// dZ = dy * act'(bn(x)); sums of dZ and dZ*xhat per channel; optional dZ store
struct BnBwdReduceArgs {
  const void* dy; int lddy; int dy_f32;
  const bf16_t* x; int ldx;
  BnArgs bn;
  bf16_t* dz; int lddz;   // may be null
  float* gsum; float* gsumx;
  int M, C;
  int gsum_slots, gsum_ld;
  // dz_f32: `dz` is fp32 and receives gamma*rstd*dZ (the A*dZ part of the BatchNorm backward;
  // B*x + C stays pending for the consumers, common.h BwdAff)
  int dz_f32;
};

struct PoolArgs {
  const bf16_t* x; int ldx;
  int N, H, W, C;
  BnArgs pro;          // pending BN + act applied to inputs (mode 0 & act 0: identity)
  int k, s, pt, pl;
  int Ho, Wo;
  bf16_t* y; int ldy;  // output slice
  uint8_t* argmax;     // [N*Ho*Wo*C] (max pool)
  float* stats; int stats_ld; int stats_off;  // output statistics (optional)
  int stats_slots;
  const float* stats_shift;  // shift of the output channels (pre-offset to output channel 0)
};

struct PoolBwdArgs {
  const void* dy; int lddy; int dy_f32;   // grad wrt pool output
  const uint8_t* argmax;
  int N, H, W, C, k, s, pt, pl, Ho, Wo;
  // epilogue: backward through the pending BN+act of the forward input (mode/act 0: plain)
  const bf16_t* x; int ldx;
  BnArgs bn;
  bf16_t* dx; int lddx;    // output (dZ if bn active, else plain grad)
  float* gsum; float* gsumx;
  int is_avg;
  int gsum_slots, gsum_ld;
  // backward pending affine of a LATER BatchNorm on dy (x = its forward input at the pool-output
  // positions), and dx_f32: `dx` is fp32 and receives gamma*rstd*dZ (BwdAff unit-alpha form)
  BwdAff dyaff;
  int dx_f32;
};

struct BnMovingDesc {
  const float* stats; int C; float inv_count; float unbias;  // unbias = n/(n-1)
  float* mmean; float* mvar; float momentum;
  int ld;  // statistics row length (sumsq of channel c at stats[ld + c])
  int slots;  // statistics slot copies (stride 2*ld)
  const float* shift;  // per-channel statistics shift (nullable, common.h "Shifted statistics")
};

// one statistics array whose shift is advanced to this step's batch mean (stats_shift)
struct ShiftDesc {
  const float* stats; float* shift;
  int ld; int slots; float inv_count; int pad;
};
hipError_t stats_shift(const ShiftDesc* d, int n, int maxC, hipStream_t st);

struct HeadArgs {
  const bf16_t* x; int ldx;  // [N*HW, C]
  int N, HW, C, U;
  BnArgs pro;
  const float* w;   // [C][U] fp32 master
  const float* b;   // [U]
  const float* labels;  // [N] (U==1) or [N][U]
  float* logits;    // [N][U]
  float* feats;     // [N][C]
  float* dlogits;   // [N][U]
  float* loss;      // scalar: mean loss (+= per sample when loss_vec is null)
  float loss_scale; // 1/N_global-batch-mean factor (1/N local)
  int training;
  float* loss_vec;  // [N] per-sample losses: the last block sums them in sample order and WRITES
                    // loss (run-to-run identical, no zero-fill before the head)
  unsigned* ticket; // arrival counter of loss_vec (counts modulo N, never reset)
  float dl_scale;   // dlogits factor: loss_scale x this rank's share weight of an uneven global
                    // batch (applied BEFORE the gradient all-reduce; the optimizer's scale is 1/N)
};

struct HeadBwdArgs {
  const float* feats; const float* dlogits; const float* w;
  int N, HW, C, U;
  float* dw; float* db;   // grads (accumulate)
  float* dA; int ldda;    // [N*HW, C] fp32 output: dfeat/HW broadcast
  int det;                // deterministic mode: one block row, one add per dW / db element
};

struct CastEntry {
  const float* src;  // Keras HWIO fp32
  bf16_t* fwd;       // [Cout][KH][KW][Cpad]
  bf16_t* dgrad;     // [Cin][KH][KW][Cout] flipped (may be null)
  int KH, KW, Cin, Cout, Cpad;
  int dw;            // reserved (depthwise kernels are read from the fp32 master directly)
  long long begin;   // first tile of this entry in the launch's tile space (64x64 tiles of [KH*KW*Cin][Cout])
};

// grouped-execution pointer shifts (common.h GroupArg)
__device__ __forceinline__ void gshift(BnBwdApplyArgs& a, long long o) {
  // (no early return at o == 0: gsh also moves every pointer into the global address space)
  a.dz = gsh(a.dz, o); a.x = gsh(a.x, o); gshift(a.bn, o); a.gsum = gsh(a.gsum, o); a.gsumx = gsh(a.gsumx, o);
  a.dst = gsh(a.dst, o); a.fold_sum = gsh(a.fold_sum, o); a.fold_sumx = gsh(a.fold_sumx, o);
}
__device__ __forceinline__ void gshift(BnBwdReduceArgs& a, long long o) {
  // (no early return at o == 0: gsh also moves every pointer into the global address space)
  a.dy = gsh(a.dy, o); a.x = gsh(a.x, o); gshift(a.bn, o); a.dz = gsh(a.dz, o); a.gsum = gsh(a.gsum, o);
  a.gsumx = gsh(a.gsumx, o);
}
__device__ __forceinline__ void gshift(PoolArgs& a, long long o) {
  // (no early return at o == 0: gsh also moves every pointer into the global address space)
  a.x = gsh(a.x, o); gshift(a.pro, o); a.y = gsh(a.y, o); a.argmax = gsh(a.argmax, o);
  a.stats = gsh(a.stats, o); a.stats_shift = gsh(a.stats_shift, o);
}
__device__ __forceinline__ void gshift(PoolBwdArgs& a, long long o) {
  // (no early return at o == 0: gsh also moves every pointer into the global address space)
  a.dy = gsh(a.dy, o); a.argmax = gsh(a.argmax, o); a.x = gsh(a.x, o); gshift(a.bn, o); a.dx = gsh(a.dx, o);
  a.gsum = gsh(a.gsum, o); a.gsumx = gsh(a.gsumx, o); gshift(a.dyaff, o);
}
__device__ __forceinline__ void gshift(BnMovingDesc& a, long long o) {
  // (no early return at o == 0: gsh also moves every pointer into the global address space)
  a.stats = gsh(a.stats, o); a.mmean = gsh(a.mmean, o); a.mvar = gsh(a.mvar, o); a.shift = gsh(a.shift, o);
}
__device__ __forceinline__ void gshift(ShiftDesc& a, long long o) {
  // (no early return at o == 0: gsh also moves every pointer into the global address space)
  a.stats = gsh(a.stats, o); a.shift = gsh(a.shift, o);
}
__device__ __forceinline__ void gshift(HeadArgs& a, long long o) {
  // (no early return at o == 0: gsh also moves every pointer into the global address space)
  a.x = gsh(a.x, o); gshift(a.pro, o); a.w = gsh(a.w, o); a.b = gsh(a.b, o); a.labels = gsh(a.labels, o);
  a.logits = gsh(a.logits, o); a.feats = gsh(a.feats, o); a.dlogits = gsh(a.dlogits, o); a.loss = gsh(a.loss, o);
  a.loss_vec = gsh(a.loss_vec, o); a.ticket = gsh(a.ticket, o);
}
__device__ __forceinline__ void gshift(HeadBwdArgs& a, long long o) {
  // (no early return at o == 0: gsh also moves every pointer into the global address space)
  a.feats = gsh(a.feats, o); a.dlogits = gsh(a.dlogits, o); a.w = gsh(a.w, o); a.dw = gsh(a.dw, o);
  a.db = gsh(a.db, o); a.dA = gsh(a.dA, o);
}
__device__ __forceinline__ void gshift(CastEntry& a, long long o) {
  // (no early return at o == 0: gsh also moves every pointer into the global address space)
  a.src = gsh(a.src, o); a.fwd = gsh(a.fwd, o); a.dgrad = gsh(a.dgrad, o);
}

hipError_t bn_bwd_apply(const BnBwdApplyArgs& a, hipStream_t st);
hipError_t bn_bwd_reduce(const BnBwdReduceArgs& a, hipStream_t st);
hipError_t maxpool_fwd(const PoolArgs& a, hipStream_t st);
// image-resident overlapping max pool (pool_img.hip): one workgroup per image x 16 channels
bool maxpool_img_fwd_ok(const PoolArgs& a);
bool maxpool_img_bwd_ok(const PoolBwdArgs& a);
hipError_t maxpool_img_fwd(const PoolArgs& a, hipStream_t st);
hipError_t maxpool_img_bwd(const PoolBwdArgs& a, hipStream_t st);
hipError_t avgpool_fwd(const PoolArgs& a, hipStream_t st);
hipError_t pool_bwd(const PoolBwdArgs& a, hipStream_t st);
hipError_t bn_update_moving(const BnMovingDesc* d_descs, int n, int maxC, hipStream_t st);
hipError_t head_fwd(const HeadArgs& a, hipStream_t st);
hipError_t head_bwd(const HeadBwdArgs& a, hipStream_t st);
hipError_t zero_fill(void* p, long long nbytes, hipStream_t st);
hipError_t rmsprop(float* w, const float* g, float* ms, long long n, float lr, float rho,
                   float eps, float grad_scale, const int* skip, int* hostflag, hipStream_t st);
hipError_t finite_check(const float* g, long long n, int* flag, hipStream_t st);
// status[0] = flag (last step skipped?), status[1] += flag (skipped steps), flag = 0
hipError_t finite_flag_reset(int* flag, int* status, hipStream_t st);
hipError_t cast_weights(const CastEntry* d_entries, const int* tile_entry, long long ntiles, hipStream_t st);
hipError_t group_metrics(const float* loss, const float* logits, const float* labels, long long stride, int K,
                         int B, float thr, double* acc, hipStream_t st);
hipError_t input_stage(const void* x, int x_u8, int N, int H, int W, int C, bf16_t* y, int Cpad,
                       const void* lab, int lab_code, int U, float* lab_out, hipStream_t st);
hipError_t bn_stats(const bf16_t* x, int ldx, int M, int C, float* stats, int stats_ld,
                    int stats_off, int stats_slots, hipStream_t st);
hipError_t bn_apply(const bf16_t* x, int ldx, BnArgs bn, const bf16_t* res, int ldres,
                    bf16_t* y, int ldy, int M, int C, float* stats, int stats_ld, int stats_slots,
                    hipStream_t st);
// dst[c] += sum_s src[s*ld + c] (and the same for src2/dst2 when given): folds statistics slots
// into one array (BatchNorm gamma/beta gradients in the parameter-gradient arena)
hipError_t slot_collapse(const float* src, float* dst, const float* src2, float* dst2, int slots,
                         int ld, int C, hipStream_t st);
// workgroups of the row-streaming kernels (pool / BN-reduce / BN-apply) for M rows of C channels,
// `per_thread_rows` rows per thread: one statistics slot per workgroup in the deterministic mode
int rows_grid(int M, int C, int per_thread_rows);
int pool_rows_grid(int M, int C, int per_thread_rows);  // the pool kernels' grid (IDC_POOL_GRID_DIV)

}  // namespace idc
