// Persistent MobileNetV2 block chain (mb_chain.hip): the expand -> depthwise -> project convs of
// consecutive inverted-residual blocks, with every BatchNorm's batch statistics, in ONE launch.
#pragma once
#include "common.h"

namespace idc {

enum { MB_TAB = 1, MB_PW = 2, MB_DW = 3 };
constexpr int MB_MAX_PHASES = 64;     // phases of one launch (their table is copied into LDS)
constexpr int MB_MAX_SLOTS = 8;       // statistics slot copies per phase
constexpr int MB_SYNC_PER_PHASE = 10; // 8 arrival shards, shards complete, READY

// One phase of the chain (a conv, or the table of a BatchNorm whose statistics predate the launch).
// Work items ("tiles") of phase p hold tickets [first, first + tiles).
struct MbPhaseDesc {
  int kind;          // MB_TAB / MB_PW (1x1 conv) / MB_DW (3x3 depthwise conv)
  int first, tiles;  // ticket range
  int dep;           // phase whose output BatchNorm table (and data) this phase reads (-1: none)
  int pro;           // operand transform: 0 raw, 1 table + act_in (BN + ReLU6 of the producer),
                     // 2 table without act + residual `res` (a block output BN_p(p) [+ h]; MB_PW)
  int act_in;
  int tab_in;        // float offset of the operand's [scale | shift] table in `tabs` (pro != 0)
  int tab_out;       // float offset of this phase's output BatchNorm table (written once, by the
                     // phase's last tile; -1: none)
  int N, H, W, Ho, Wo, S, PT, PL;  // maps (MB_PW: H = Ho, W = Wo)
  int Cin, Cout;
  int tm, tn;        // MB_PW: rows per tile (32 / 64) and columns per tile (multiple of 64);
                     // MB_DW: images per tile and channels per tile (multiple of 8 dividing C)
  int slots;         // statistics slot copies of this phase's partial sums
  int bn_mode;       // output BatchNorm: 1 batch statistics, 2 moving statistics, 0 none
  int ldx, ldy;
  const bf16_t* x;   // operand (raw producer output)
  const bf16_t* res; // pro 2: residual (nullable)
  bf16_t* aout;      // pro 2: the materialised operand (block output) [M][Cin] (nullable)
  const bf16_t* w16; // MB_PW: kernel [Cout][Cin] bf16
  const float* w32;  // MB_DW: fp32 master kernel [3][3][C]
  bf16_t* y;         // raw output
  float* stats;      // [2][Cout] single-copy shifted statistics (the program's arena)
  const float* shift;// [Cout] statistics shift K (nullable)
  float* slotbuf;    // [slots][2][Cout] in-launch partial sums (zeroed per step)
  const float* gamma;
  const float* beta;
  const float* mmean;
  const float* mvar;
  float eps, inv_count;
  BnArgs pre;        // MB_TAB: the BatchNorm (+ act) whose table is built
};

constexpr int MB_TABLE_BYTES = (MB_MAX_PHASES * (int)sizeof(MbPhaseDesc) + 15) / 16 * 16;

struct MbChainArgs {
  const MbPhaseDesc* phases;
  unsigned* sync;             // [2 + MB_SYNC_PER_PHASE * nphases]: ticket, fail, per phase words;
                              // zeroed before every launch (the stats-arena memset)
  float* tabs;                // BatchNorm tables
  int* err;                   // persistent count of launches that gave up on a wait (nullable)
  int* stepflag;              // nullable: per-step guard word (persist.h FailSink)
  int* hostflag;              // nullable: pinned host give-up flag
  unsigned long long* stamps; // nullable: persist::NSTAMP s_memrealtime stamps per ticket
  int nphases, ntickets;
  unsigned max_polls;
  int pad_;
};

// dynamic LDS bytes a phase needs (the launch takes the maximum)
int mb_phase_smem(const MbPhaseDesc& d);
// the largest tile LDS a phase may use (the launch adds the phase table)
int mb_smem_limit();
// host-side shape rules of one phase descriptor (checked by the lowering before it emits a launch)
bool mb_phase_ok(const MbPhaseDesc& d);
hipError_t mb_chain(const MbChainArgs& a, int grid, int smem, hipStream_t st);

}  // namespace idc
