// Persistent dense-stage forward: every dense layer of a DenseNet stage in ONE launch.
// See dense_stage.hip for the design.
#pragma once
#include "common.h"

namespace idc {

// One dense layer (conv{s}_block{l}: BN->ReLU->1x1(128) -> BN->ReLU->3x3(32)), device table entry.
struct DenseLayerDesc {
  const bf16_t* w1;     // 1x1 kernel [128][cin] bf16 (kernel layout, k-contiguous)
  const bf16_t* w2;     // 3x3 kernel [32][k2][k2][128] bf16 (k2 = 1: centre tap only, 1x1 maps)
  const float* g1;      // _0_bn gamma / beta over the layer's input channels [0, cin)
  const float* b1;
  const float* g2;      // _1_bn gamma / beta [128]
  const float* b2;
  bf16_t* t;            // raw 1x1 output [M][128] (saved for the backward)
  float* tstats;        // [2][128] shifted statistics of t (zeroed per step; written once, whole)
  const float* tshift;  // [128] statistics shift of t (nullable)
  float eps1, eps2;
  int cin;              // input channels = this layer's slice offset in the stage buffer
  int pad_;             // bit 0 / bit 1: _0_bn / _1_bn in inference mode (frozen layer of a
                        // fine-tuned stage; the launch still produces the statistics)
  const float* mm1;     // moving mean / variance of _0_bn [cin] and _1_bn [128]: the inference-mode
  const float* mv1;     // (DenseStageArgs::infer) BatchNorms normalise with these
  const float* mm2;
  const float* mv2;
};

// Slot copies of the in-launch statistics (the per-channel float atomics of one phase are spread
// over DS_SLOTS copies so no address takes more than ~tiles/DS_SLOTS adds)
constexpr int DS_SLOTS = 8;
// floats of in-launch statistics scratch per layer: [DS_SLOTS][2][32] slice + [DS_SLOTS][2][128] t
constexpr int DS_SCRATCH_PER_LAYER = DS_SLOTS * 2 * (32 + 128);
// the widest 1x1 input a launch accepts (BN coefficient tables in LDS): DenseNet-201 stage 4 = 1888
constexpr int DS_MAX_CIN = 2048;
// staged 3x3-operand rows per tile (32 output rows plus the images' halo rows): maps up to ~8x8
constexpr int DS_MAX_STAGE_ROWS = 128;

struct DenseStageArgs {
  bf16_t* buf;                  // stage buffer [M][ld] (channels [0, c0) written before the launch)
  float* sstats;                // [2][ld] shifted statistics of the stage buffer (single copy)
  const float* sshift;          // [ld] (nullable)
  const DenseLayerDesc* layers; // device table [nlayers]
  unsigned* sync;               // [dense_stage_sync_words] ticket, per-phase completion counters,
                                // fail flag, per-tile helper counters (zeroed before every launch:
                                // the program's stats-arena memset)
  int* err;                     // persistent count of launches that gave up on a wait (nullable)
  float* scratch;               // [nlayers * DS_SCRATCH_PER_LAYER] zeroed per launch (stats arena)
  unsigned long long* stamps;   // nullable: 4 s_memrealtime stamps per work item (diagnostics)
  int N, H, W, ld, nlayers, k2;
  int act1, act2;
  float inv_count;              // 1 / (N*H*W)
  unsigned max_polls;           // bound on one wait's polls (0: default, ~0.5 s)
  int lookahead;                // queue order (set by dense_stage_fwd): 0 [A0][B0][A1][B1]...,
                                // 1 [A0][A1][B0][A2][B1]...[B_{L-1}] (see dense_stage.hip); the
                                // caller passes -1 to forbid the lookahead order (another
                                // persistent launch may share the device: the order needs more
                                // than one phase of workgroups resident)
  int infer;                    // inference-mode BatchNorms (moving statistics; frozen layers,
                                // evaluation): no statistics are produced, only data hand-offs
  int* stepflag;                // nullable: the program's per-step guard word; a launch that gives
                                // up ORs 2 into it (the optimizer then skips the step's update)
  int* hostflag;                // nullable: pinned host word set to 1 on a give-up (never shifted
                                // per group copy; the runtime polls it without a device sync)
  float* partials;              // split-K slab [2][A tiles][ksplit-1][256][8] fp32 (ksplit > 1)
  int ksplit;                   // work items per 1x1 tile (older-channel K split; 0/1: none)
  int rows;                     // 1: row-resident launch (dense_rows.hip) where its geometry fits
  int rows_ipg;                 // (set by the launcher) images per row-resident workgroup
};

// most K splits of an A tile (the helpers' partials: one slab slot each)
constexpr int DS_MAX_KSPLIT = 8;
// number of work items of one launch (the grid never needs more workgroups than this)
int dense_stage_tasks(const DenseStageArgs& a);
// work items of each phase of one layer: 1x1 items (32 rows x 64 channels x 1/ksplit of the
// older channels), 3x3 tiles (32 rows)
void dense_stage_phase_tiles(int M, int ksplit, int& nA, int& nB);
// sync words of a launch: ticket, sharded phase counters, last-slice count, fail flag, and one
// helper-arrival counter per A tile and layer
int dense_stage_sync_words(int M, int nlayers);
// floats of the split-K partial slab (0 for ksplit <= 1)
long long dense_stage_partial_floats(int M, int ksplit);
// the K split for a stage of M rows on a grid of `grid` workgroups: 1 (off) unless IDC_DS_KSPLIT
// forces a value or IDC_DS_KSPLIT_TARGET names the A items aimed at (measured slower, see .hip)
int dense_stage_default_ksplit(int M, int grid);
// whether a stage shape fits the launch (cin, staged rows)
bool dense_stage_shape_ok(int N, int H, int W, int max_cin);
hipError_t dense_stage_fwd(const DenseStageArgs& a, int grid, hipStream_t st);
// row-resident form (dense_rows.hip): each workgroup owns whole images for the whole stage and
// only the BatchNorm statistics cross workgroups (two barriers per layer; none in inference mode)
bool dense_rows_geometry(int N, int H, int W, int ld, int max_cin, int& rb, int& ipg, int& grid);
hipError_t dense_rows_fwd(const DenseStageArgs& a, hipStream_t st);

// ---------------------------------------------------------------------------------------------
// Persistent dense-stage BACKWARD (dense_stage_bwd.hip): the data gradients of every dense layer
// of a stage, its BatchNorm reductions and d gamma / d beta, in ONE launch.
struct DenseBwdLayerDesc {
  const bf16_t* w1d;    // cv1 dgrad layout [cin][128]
  const bf16_t* w2d;    // cv2 dgrad layout [128][k2][k2][32] (flipped taps)
  const float* g1;      // _0_bn gamma / beta [cin]
  const float* b1;
  const float* g2;      // _1_bn gamma / beta [128]
  const float* b2;
  const bf16_t* t;      // forward raw 1x1 output [M][128]
  const float* tstats;  // forward [2][128] shifted statistics of t
  const float* tshift;  // [128] (nullable)
  bf16_t* dO16;         // [M][32] out: the layer's staged output gradient (cv2 weight gradient)
  bf16_t* dt;           // [M][128] out: d t (cv1 weight gradient, older-channel dgrad operand)
  float* dbeta1;        // gradient arena [cin] of _0_bn
  float* dgamma1;
  float* dbeta2;        // gradient arena [128] of _1_bn
  float* dgamma2;
  float* r1;            // scratch [DS_SLOTS][2][cin]: sum dZ1, sum dZ1*xhat1 (zeroed per step)
  float* r2;            // scratch [DS_SLOTS][2][128]: sum dZ2, sum dZ2*xhat2
  float eps1, eps2;
  int cin;
  int pad_;
};

// one entry of the launch's work queue, in ticket order
struct DenseBwdPhase {
  int first;   // first ticket
  int kind;    // DSB_P / DSB_QN / DSB_G / DSB_GIN / DSB_FIN1 / DSB_FIN2
  int layer;   // P, QN: the layer; G: the slice (= the layer that produced it)
  int tiles;
};
enum { DSB_P = 1, DSB_QN = 2, DSB_G = 3, DSB_GIN = 4, DSB_FIN1 = 5, DSB_FIN2 = 6 };
constexpr int DSB_KG = 6;          // later layers gathered per G / GIN tile
constexpr int DSB_MAX_CG = 64;     // 32-channel groups of the stage input (c0 <= 2048)
// sync words: [0] ticket; layer l at 1 + 32 l: P (8 shards), QN (8 shards), G arrivals, G done;
// then GIN (8 shards), FIN1 arrivals per input channel group, FIN1 done, FIN2, fail
constexpr int DSB_SYNC_PER_LAYER = 32;
__host__ __device__ inline int dsb_sync_words(int L) { return 1 + DSB_SYNC_PER_LAYER * L + 8 + DSB_MAX_CG + 3; }

struct DenseBwdArgs {
  const bf16_t* buf;              // stage buffer [M][ld] (forward, raw)
  const float* sstats;            // [2][ld] forward shifted statistics of the stage buffer
  const float* sshift;            // [ld] (nullable)
  float* dbuf;                    // fp32 [M][ld]: on entry A*dZ of the stage's consumer BatchNorm;
                                  // the gathered older-layer terms are added in place
  float* dnew;                    // fp32 [2][M][32] scratch: newest-slice 1x1 data gradients
  bf16_t* dx16;                   // [M][c0] out: final gradient of the stage input channels (bf16)
  bf16_t* z2;                     // [M][128] scratch: dZ of the current layer's _1_bn
  BwdAff pend;                    // the consumer BatchNorm's pending B*x + C, channels [0, ld)
                                  // (its reductions complete before the launch)
  const DenseBwdLayerDesc* layers;
  const DenseBwdPhase* phases;    // work queue, nphases entries
  unsigned* sync;                 // [dsb_sync_words(nlayers)] counters (zeroed per step)
  float* btot;                    // [2][ld] scratch: each channel's summed B / C (written once)
  int* err;
  unsigned long long* stamps;     // nullable: 4 stamps per ticket
  int N, H, W, ld, c0, nlayers, k2, act, nphases, ntickets;
  float inv_count;
  unsigned max_polls;
  int* stepflag;                  // nullable: per-step guard word (as DenseStageArgs::stepflag)
  int* hostflag;                  // nullable: pinned host give-up flag (as DenseStageArgs::hostflag)
  int rows;                       // 1: row-resident launch (dense_rows_bwd.hip) where its geometry fits
  int rows_ipg;                   // (set by the launcher) images per row-resident workgroup
  float* rpart;                   // row-resident: per-workgroup bn1 sums [layer][group][2][cin]
  long long rpart_floats;         // its size (dense_rows_bwd_part_floats)
};

hipError_t dense_stage_bwd(const DenseBwdArgs& a, int grid, hipStream_t st);
// row-resident form (dense_rows_bwd.hip): whole images per workgroup, the concat gradient in LDS,
// only the BatchNorm reductions cross workgroups (two barriers per layer)
bool dense_rows_bwd_geometry(int N, int H, int W, int ld, int nlayers, int& ipg, int& grid);
hipError_t dense_rows_bwd(const DenseBwdArgs& a, hipStream_t st);
long long dense_rows_bwd_part_floats(int c0, int nlayers, int grid);

// A whole dense block in INFERENCE mode (every BatchNorm on its moving statistics: evaluation, a
// frozen base, the frozen prefix of a fine-tuned net) as ONE launch with no cross-workgroup
// traffic at all (dense_infer.hip): a workgroup owns `ipg` whole images, keeps their concat buffer
// in LDS and runs every layer's BN1+ReLU -> 1x1 -> BN2+ReLU -> 3x3 on it.  For the large maps
// (stages 1-2: 13x13 / 6x6 at 50x50) that the per-image row kernel (dense_rows.hip) cannot hold.
struct DenseInferArgs {
  bf16_t* buf;                    // stage buffer [N][H][W][ld]: channels [0, c0) in, [c0, c0 + 32 L) out
  int ld;
  int N, H, W, c0, L, ipg, act;   // act: the BatchNorms' activation (ReLU)
  const DenseLayerDesc* layers;   // L descriptors (w1, w2, g1/b1/mm1/mv1, g2/b2/mm2/mv2, eps, cin)
};
long long dense_infer_smem(const DenseInferArgs& a);  // dynamic LDS bytes, -1: shape not supported
hipError_t dense_infer(const DenseInferArgs& a, hipStream_t st);
// the same per-image block in TRAINING mode (dense_infer.hip; DenseStageArgs::rows == 2): BatchNorm
// batch statistics through slot copies and two sharded barriers per layer, outputs as the per-layer
// convs.  For stages whose images the row-resident launch cannot hold (13x13 / 6x6 at 50x50)
bool dense_img_ok(const DenseStageArgs& a);
hipError_t dense_img_fwd(const DenseStageArgs& a, hipStream_t st);

}  // namespace idc
