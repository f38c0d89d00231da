#pragma once
#include "common.h"

namespace idc {

enum OutMode : int { OUT_BF16 = 0, OUT_F32 = 1, OUT_F32_ACC = 2 };
enum Tile : int { TILE_128x128 = 0, TILE_128x64 = 1, TILE_256x32 = 2, TILE_64x64 = 3, TILE_64x32 = 4 };

struct ConvArgs {
  // input operand (A): NHWC, pointer already offset to the channel slice; element type bf16 or
  // fp32 (fp32 is converted while staging; used for fp32 gradient buffers)
  const void* x;
  int N, H, W, Cin, ldx;
  // output
  int Ho, Wo, Cout;
  void* y;
  int ldy;
  // weights [Cout][KH][KW][Cin] bf16 (k-contiguous)
  const bf16_t* w;
  int KH, KW, SH, SW, PT, PL;
  // prologue: pending BN (+act) applied to A (per input channel)
  BnArgs pro;
  // epilogue
  int epi_mode;       // 0: bias/act/store/stats   1: backward through forward-input BN+act
  const float* bias;  // [Cout] or null
  int epi_act;
  int out_mode;       // OutMode (epi 0)
  float* stats_out;   // [2*stats_ld] sum|sumsq of stored values, channel c at stats_off + c
  int stats_ld;
  int stats_off;
  // epi 1
  const bf16_t* mx;   // forward input x at output positions [M, ldmx]
  int ldmx;
  BnArgs mbn;         // the forward BN(+act) that was applied to mx
  float* gsum;        // [Cout] += sum(dZ)
  float* gsumx;       // [Cout] += sum(dZ * xhat)
  // split-K (small-M, deep-K layers are K-loop latency bound): with ksplit > 1 each output tile's
  // K range is split over `ksplit` workgroups; each publishes an fp32 partial tile to `slab`
  // ([tiles][ksplit][TM*TN][256] float4) and takes a ticket; the tile's last arriver sums the
  // partials and runs the epilogue.  Tickets count modulo ksplit (never reset in-kernel): one
  // ticket array per op, zeroed whenever the op's split factor changes.
  float* slab;
  unsigned* tickets;
  long long slab_floats;  // capacities, checked by the launcher before a split launch
  int tickets_n;
  int ksplit;
  // statistics slots (common.h): stats_out holds stats_slots copies of [sum|sumsq] (stride
  // 2*stats_ld), gsum/gsumx gsum_slots copies (stride gsum_ld); a tile adds into copy mtile % slots
  int stats_slots;
  int gsum_slots;
  int gsum_ld;
  // backward pending affine on the A operand (common.h BwdAff; bpro.mode != 0 selects it): the
  // staged operand is A*v + B*x + C with x read from bpro.x at the same pixel and channel
  BwdAff bpro;
  // epi 2 (DenseNet concat gradient): y is the fp32 stage-gradient buffer, and the epilogue adds
  //   y += gamma*rstd * dZ  +  B'*x + C'
  // where dZ = dA * act'(mbn(x)) (reduced into gsum/gsumx as in epi 1) and B', C' are the pending
  // coefficients of the PREVIOUS BatchNorm over these channels (bepi; x = mx)
  BwdAff bepi;
  // PRO 2 only (optional): the staged operand (after the affine, bf16) is also stored here, one
  // write per element (centre tap, first column tile) — the side-lane weight gradient then reads
  // a plain bf16 gradient instead of redoing the affine on the fp32 / two-tensor form
  bf16_t* aout;
  int ldaout;
  // epi 0 statistics shift of the output channels (pre-offset to output channel 0; nullable):
  // the statistics accumulate y - K (common.h "Shifted statistics")
  const float* stats_shift;
};

__device__ __forceinline__ void gshift(ConvArgs& a, long long o) {
  // (no early return at o == 0: gsh also moves every pointer into the global address space)
  a.x = gsh(a.x, o); a.y = gsh(a.y, o); a.w = gsh(a.w, o); gshift(a.pro, o); a.bias = gsh(a.bias, o);
  a.stats_out = gsh(a.stats_out, o); a.mx = gsh(a.mx, o); gshift(a.mbn, o); a.gsum = gsh(a.gsum, o);
  a.gsumx = gsh(a.gsumx, o); a.slab = gsh(a.slab, o); a.tickets = gsh(a.tickets, o); gshift(a.bpro, o);
  gshift(a.bepi, o); a.aout = gsh(a.aout, o); a.stats_shift = gsh(a.stats_shift, o);
}

// tiles TILE_BIG128 / TILE_BIG256 select the 256 x {128, 256} global_load_lds kernel for plain
// wide layers (conv_big.hip)
constexpr int TILE_BIG128 = 101;
constexpr int TILE_BIG256 = 102;
constexpr int TILE_BIG64 = 103;
constexpr int TILE_BIG128D = 104;  // 256 x 128 with three LDS buffers
// tile TILE_IMG selects the image-resident 3x3 kernel (conv_img.hip): DenseNet's 128 -> 32
// forward and 32 -> 128 data-gradient convolutions on maps up to 13 x 13
constexpr int TILE_IMG = 105;
bool conv_img_ok(const ConvArgs& a, bool a_f32);
hipError_t conv_img(const ConvArgs& a, bool a_f32, hipStream_t st);
// tile TILE_STEM selects the image-resident stem convolution (conv_stem.hip): 8-channel staged
// images, KxK stride 1/2, up to 64 output channels
constexpr int TILE_STEM = 107;
bool conv_stem_ok(const ConvArgs& a, bool a_f32);
hipError_t conv_stem(const ConvArgs& a, bool a_f32, hipStream_t st);
bool conv_big_ok(const ConvArgs& a, bool a_f32);
hipError_t conv_big(const ConvArgs& a, int bn, bool a_f32, hipStream_t st);
hipError_t conv_igemm(const ConvArgs& a, int tile, bool a_f32, hipStream_t st);
int conv_pick_tile(int M, int Cout);
int conv_num_tiles();
int conv_tile_bm(int t);
int conv_tile_bn(int t);
int conv_tile_bk(int t);

}  // namespace idc
