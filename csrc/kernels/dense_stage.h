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
  float* tstats;        // [2][128] shifted statistics of t (zeroed per step)
  const float* tshift;  // [128] statistics shift of t (nullable)
  float eps1, eps2;
  int cin;              // input channels = this layer's slice offset in the stage buffer
  int pad_;
};

struct DenseStageArgs {
  bf16_t* buf;                  // stage buffer [M][ld] (channels [0, c0) written before the launch)
  float* sstats;                // [2][ld] shifted statistics of the stage buffer
  const float* sshift;          // [ld] (nullable)
  const DenseLayerDesc* layers; // device table [nlayers]
  unsigned* sync;               // [2 + 2 * nlayers] ticket, per-phase completion counters, fail flag
                                // (zeroed before every launch: the program's stats-arena memset)
  int* err;                     // persistent count of launches that gave up on a wait (nullable)
  int N, H, W, ld, nlayers, k2;
  int act1, act2;
  float inv_count;              // 1 / (N*H*W)
  // cross-workgroup hand-off: 0 = agent-scope release/acquire fences around the completion
  // counters (an L2 writeback + invalidate per phase boundary, ~2.5 us each); bit 0 = outputs
  // stored with agent-coherent (sc1) stores, completed (vmcnt) before the counter increment, no
  // release fence; bit 1 = operands / statistics produced in this launch read with agent-coherent
  // loads (never a stale line of this XCD's L2), no acquire fence.  3 (the lowering's default):
  // DenseNet-121 bs 256 stages 3+4 4.27-4.29 ms/step vs 4.36-4.41 with fences
  int coh;
};

// number of work items of one launch (the grid never needs more workgroups than this)
int dense_stage_tasks(const DenseStageArgs& a);
hipError_t dense_stage_fwd(const DenseStageArgs& a, int grid, hipStream_t st);

}  // namespace idc
