// Implicit-GEMM convolution dispatch (kernel: conv_igemm_impl.h; variants: conv_igemm_g*.hip).
#include "conv_igemm.h"

namespace idc {

hipError_t conv_igemm_group0(const ConvArgs& a, int tile, bool is1x1, bool a_f32, int pro, int epi,
                              hipStream_t st);
hipError_t conv_igemm_group1(const ConvArgs& a, int tile, bool is1x1, bool a_f32, int pro, int epi,
                              hipStream_t st);
hipError_t conv_igemm_group2(const ConvArgs& a, int tile, bool is1x1, bool a_f32, int pro, int epi,
                              hipStream_t st);
hipError_t conv_igemm_group3(const ConvArgs& a, int tile, bool is1x1, bool a_f32, int pro, int epi,
                              hipStream_t st);
hipError_t conv_igemm_group4(const ConvArgs& a, int tile, bool is1x1, bool a_f32, int pro, int epi,
                              hipStream_t st);
hipError_t conv_igemm_group5(const ConvArgs& a, int tile, bool is1x1, bool a_f32, int pro, int epi,
                              hipStream_t st);

struct TileInfo { int bm, bn, bk; };
static const TileInfo kTiles[] = {
    {128, 128, 32}, {128, 64, 32}, {256, 32, 32}, {64, 64, 32}, {64, 32, 32},  // BK 32
    {128, 128, 64}, {128, 64, 64}, {128, 32, 64}, {64, 64, 64}, {64, 32, 64},  // BK 64
    {256, 32, 64}, {64, 128, 64},                                              // BK 64
    // BK 128: half the K steps of BK 64
    {64, 32, 128}, {128, 32, 128}, {64, 64, 128}, {64, 128, 128}, {128, 64, 128},
    {64, 32, 256}, {64, 64, 256},  // BK 256: deep-K, small-M layers (stages 3-4)
    // 32-row tiles (conv_igemm_g5.hip): twice the workgroups on small-M layers
    {32, 32, 64}, {32, 32, 128}, {32, 64, 64}, {32, 64, 128}};

int conv_num_tiles() { return (int)(sizeof(kTiles) / sizeof(kTiles[0])); }
int conv_tile_bm(int t) { return kTiles[t].bm; }
int conv_tile_bn(int t) { return kTiles[t].bn; }
int conv_tile_bk(int t) { return kTiles[t].bk; }

hipError_t conv_igemm(const ConvArgs& a, int tile, bool a_f32, hipStream_t st) {
  if (tile == TILE_IMG) return conv_img(a, a_f32, st);
  if (tile == TILE_STEM) return conv_stem(a, a_f32, st);
  if (tile < 0 || (tile >= conv_num_tiles() && tile != TILE_BIG128 && tile != TILE_BIG256 && tile != TILE_BIG64 &&
                   tile != TILE_BIG128D))
    return hipErrorInvalidValue;
  const bool is1x1 = a.KH == 1 && a.KW == 1 && a.SH == 1 && a.SW == 1 && a.PT == 0 && a.PL == 0;
  const int pro = a.bpro.mode != 0 ? 2 : (a.pro.mode != 0 || a.pro.act != ACT_NONE) ? 1 : 0;
  const int epi = a.epi_mode;
  if ((a.Cin % 8) || (a.Cout % 8) || (a.ldx % 8) || (a.ldy % 8)) return hipErrorInvalidValue;
  if (pro == 2 && (a.bpro.x == nullptr || (a.bpro.ldx % 8) || a.bpro.bn.gamma == nullptr)) return hipErrorInvalidValue;
  if (epi == 2 && a.mx == nullptr) return hipErrorInvalidValue;
  if (a.ksplit > 1 && (a.slab == nullptr || a.tickets == nullptr)) return hipErrorInvalidValue;
  if (tile == TILE_BIG128 || tile == TILE_BIG256 || tile == TILE_BIG64 || tile == TILE_BIG128D)
    return conv_big(a, tile == TILE_BIG256 ? 256 : tile == TILE_BIG128 ? 128 : tile == TILE_BIG128D ? -128 : 64,
                    a_f32, st);
  const int group = tile < 4 ? 0 : tile < 8 ? 1 : tile < 12 ? 2 : tile < 16 ? 3 : tile < 19 ? 4 : 5;
  switch (group) {
    case 0: return conv_igemm_group0(a, tile, is1x1, a_f32, pro, epi, st);
    case 1: return conv_igemm_group1(a, tile, is1x1, a_f32, pro, epi, st);
    case 2: return conv_igemm_group2(a, tile, is1x1, a_f32, pro, epi, st);
    case 3: return conv_igemm_group3(a, tile, is1x1, a_f32, pro, epi, st);
    case 4: return conv_igemm_group4(a, tile, is1x1, a_f32, pro, epi, st);
    default: return conv_igemm_group5(a, tile, is1x1, a_f32, pro, epi, st);
  }
}

int conv_pick_tile(int M, int Cout) {
  auto blocks = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((Cout + bn - 1) / bn); };
  if (Cout <= 32) return blocks(128, 32) >= 256 ? 7 : 9;
  if (Cout <= 64) return blocks(128, 64) >= 256 ? 6 : 8;
  if (blocks(128, 128) >= 256) return 5;
  if (blocks(64, 128) >= 256) return 11;
  return 8;
}

}  // namespace idc
