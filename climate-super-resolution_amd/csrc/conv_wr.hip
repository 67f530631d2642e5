// 64 -> 64-channel 3x3 stride-1 convolution with the weights resident in registers (CDNA4, gfx950).
//
// Replaces nn.Conv2d on the HR-resolution / large-grid 64-channel layers: HRconv and upconv1/2 with the nearest x2
// upsample on load (climsr/models/esrgan.py:82-83,94-99), VGG19 conv1_2 (climsr/losses/perceptual.py:16), RCAN's
// residual-block convs (climsr/models/rcan.py:50-69) and their activation-backward data gradients.
//
// The 72 A fragments of the whole weight matrix (64 co x 576 k: 4 co blocks x 18 k blocks of 16 x 32 bf16) stay in
// registers for the launch -- 60 in AGPRs, read by the MFMAs from there (mfma_agpr.h), the last 12 in VGPRs -- so the
// LDS holds pixels only and every 1 KB B fragment read feeds 4 MFMAs (one per co block): 0.25 KB of LDS reads per
// MFMA, against 0.75 for conv_pw's 8-wave form that re-reads the weights from LDS.
// Waves are independent: each owns a 4 x 16-pixel output tile at a time, brings its 6 x 18-pixel input footprint
// (64 channels, pitch 80 bf16 = conflict-free b128 reads) into its own pair of LDS buffers with LDS-DMA
// (buffer_load ... lds: no staging registers, no ds_write), the next tile's footprint landing while the current one
// computes, and stores its epilogue straight from the accumulators.  No workgroup barrier anywhere: the four waves of
// a CU drift apart, so one wave's epilogue and DMA waits overlap the others' MFMAs (the lockstep of identical
// workgroups is what held conv_pw and the generic conv).
// Tiles: wave w of workgroup b (XCD-major renumbered) takes tiles 4 (b + k G) + w: the four waves of a CU work on four
// horizontally adjacent tiles (shared halo columns) and consecutive workgroups of an XCD on the next ones.
// Prologue: the 72 KB weight matrix comes into LDS once per workgroup (LDS-DMA in fragment order: one 1 KB piece per
// A fragment, lane-contiguous, so each wave's ds_read_b128 of a fragment is conflict-free), into the regions the
// second footprint buffers and the channel-sum transposes use later; every wave copies its registers from there.
// Loading them straight from global memory cost each CU four copies (296 KB) of L2 traffic before its first MFMA --
// on a small grid (RCAN's 360 x 720 LR convs: about four tiles per wave) that prologue was a third of the launch.
#include <algorithm>
#include <stdio.h>

#include "conv_ep.h"
#include "mfma_agpr.h"

namespace {

constexpr int WR_TR = 4, WR_TC = 16;                    // output rows x columns of a wave tile
constexpr int WR_PR = WR_TR + 2, WR_PC = WR_TC + 2;     // input footprint (3x3, pad 1)
constexpr int WR_XP = 80;                               // footprint pixel pitch (bf16): 64 channels + 16 pad
constexpr int WR_SPP = WR_XP / 8;                       // 16 B slots per pixel (8 data + 2 pad)
constexpr int WR_SLOTS = WR_PR * WR_PC * WR_SPP;        // 1080
constexpr int WR_NI = (WR_SLOTS + 63) / 64;             // LDS-DMA instructions per footprint (17)
constexpr int WR_BUF = WR_NI * 1024;                    // bytes per footprint buffer
constexpr int WR_LDS = 4 * 2 * WR_BUF;                  // 4 waves x 2 buffers: 139,264 B
constexpr int WR_RED = 64 * 17 * 4;                     // per wave: the channel-sum transpose [64 ch][17] (EP 3 / 4)
constexpr int WR_LDS_ALL = WR_LDS + 4 * WR_RED;         // 156,672 B
static_assert(WR_LDS_ALL <= 160 * 1024, "conv_wr LDS");
// the one-image channel sums' arrival counter: wave 3's transpose corner, row 16's pad column (never written by the
// transposes, clear of the weight pieces staged at the start of the channel-sum region)
__device__ inline uint32_t* wr_wg_count(char* smem) { return (uint32_t*)(smem + WR_LDS + 3 * WR_RED) + 16 * 17 + 16; }
static_assert(3 * WR_RED >= 4 * 1024, "conv_wr arrival counter clear of the staged weights");

struct WrArgs {
  const uint16_t* x;
  const uint16_t* w;     // packed [64 co][kpk], k = tap * 64 + channel
  const float* bias;     // may be null
  uint16_t* y;
  const uint16_t* res1;  // EP 1: residual (v = alpha1 v + beta1 r); EP 2: the activation output (act 3 / 4)
  float* ch_part;        // EP 3 / 4: per-tile channel sums [tile][64] of the fp32 values (null: none)
  int n, in_h, in_w, in_cs, in_co, up, out_h, out_w, out_cs, out_co, kpk;
  int act;  // forward: 0 none, 1 leaky relu, 2 relu; EP 2: 3 / 4 = backward of leaky relu / relu
  float slope, alpha1, beta1;
  int r1_cs, r1_co;
  int tiles_x, tiles_y, ntiles;
  int wg_sums;  // EP 3 / 4 with one image: ch_part gets one row per workgroup (its tiles' sums) instead of one per tile
  uint32_t x_bytes, y_bytes, r1_bytes;
};
typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));

// ACT: the activation as a template parameter (0 none, 1 leaky relu, 2 relu; EP 2: 3 / 4 their backward) -- as a
// kernel argument it cost a three-way uniform branch per accumulator element (~390 branch instructions per tile)
template <int EP, int ACT>
__global__ __launch_bounds__(256, 1) void conv_wr_kernel(WrArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // vector-memory operations of one epilogue (loads + stores), fixed per lane
  // EP 5: EP 0 followed by the 2x2 max pool (VGG19 conv1_2 + MaxPool2d, perceptual.py:16): 4 stores a lane
  // bf16 outputs leave as 16-B stores, two per output row m (see the epilogue): EP 0 8, EP 4 8 + 1, EP 1 / 2 16 + 8
  constexpr int NEPI = EP == 0 ? 8 : (EP == 5 ? 4 : (EP == 3 ? 17 : (EP == 4 ? 9 : 24)));
  constexpr bool SUMS = EP == 3 || EP == 4;  // per-tile channel sums (EP 3: fp32 out, EP 4: bf16 out)
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, col = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G4 = (int)gridDim.x * 4;
  int T = xcd_major(blockIdx.x, gridDim.x) * 4 + wv;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;

  // ---- the weight matrix: A fragment f = 18 t + j (co block t, k block j) = rows 16 t + col, k = 32 j + 8 g ..,
  // staged in LDS piece wr_piece(f) (see the file comment); wave w moves fragments 18 w .. 18 w + 17
  auto wr_piece = [](int f) {
    return f < 68 ? ((f / 17) * 2 + 1) * WR_BUF + (f % 17) * 1024 : WR_LDS + (f - 68) * 1024;
  };
  {
    const __amdgpu_buffer_rsrc_t wrs = buf_rsrc(a.w, (uint32_t)(64 * a.kpk * 2));
#pragma unroll
    for (int i = 0; i < 18; ++i) {
      const int f = 18 * wv + i, t = f / 18, j = f % 18;
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"((uint32_t)(((t * 16 + col) * a.kpk + j * 32 + g * 8) * 2)), "s"(wrs),
                     "s"(lds0 + (uint32_t)wr_piece(f))
                   : "memory");
    }
  }
  static_assert(WR_LDS + 4 * 1024 <= WR_LDS_ALL && 4 * 17 + 4 == 72, "conv_wr weight staging regions");
  float bias[4][4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const float4 b4 = a.bias ? *(const float4*)(a.bias + t * 16 + 4 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
    bias[t][0] = b4.x; bias[t][1] = b4.y; bias[t][2] = b4.z; bias[t][3] = b4.w;
  }

  // ---- footprint DMA: instruction i, lane l fills 16 B slot q = 64 i + l = (pixel q / 10, slot q % 10); slots 8, 9
  // of a pixel (the pitch padding) and slots past the footprint get zeros (out-of-range source offset)
  // rel: the slot's source offset from the footprint's corner pixel for an interior tile without upsampling (pad
  // slots: 2^31, past every buffer's range), so such a tile's DMA offsets are one add each
  int dg[WR_NI];
  uint32_t rel[WR_NI];
#pragma unroll
  for (int i = 0; i < WR_NI; ++i) {
    const int q = i * 64 + lane, p = q / WR_SPP, c = q - p * WR_SPP;
    const bool live = p < WR_PR * WR_PC && c < 8;
    dg[i] = live ? ((p / WR_PC) << 16) | ((p % WR_PC) << 8) | c : -1;
    rel[i] = live ? (uint32_t)((((p / WR_PC) * a.in_w + p % WR_PC) * a.in_cs + c * 8) * 2) : 0x80000000u;
  }
  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(a.x, a.x_bytes);
  const uint32_t mybuf = lds0 + (uint32_t)(wv * 2 * WR_BUF);
  const int ups = a.up == 2 ? 1 : 0, lh = a.in_h << ups, lw = a.in_w << ups;
  // in asm (not the builtin): hipcc would wait vmcnt(0) before the next ds_read for an LDS write of unknown extent;
  // the DMAs are counted by hand.  M0 = the instruction's LDS destination (wave-uniform).
  auto glds = [&](uint32_t off, uint32_t lds) {  // (retired by the second hand wait after it: tests/isa_waitcnt_lint.py)
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds ; dma-lag 2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(off), "s"(xr), "s"(lds) : "memory");
  };
  auto decode = [&](int tile, int& nimg, int& oy0, int& ox0) {
    const int tx = tile % a.tiles_x, r = tile / a.tiles_x, ty = r % a.tiles_y;
    nimg = r / a.tiles_y;
    oy0 = ty * WR_TR;
    ox0 = tx * WR_TC;
  };
  auto issue = [&](int tile, int b) {  // tile < 0: zeros (keeps the per-iteration DMA count fixed)
    int nimg = 0, oy0 = -1 << 20, ox0 = 0;
    if (tile >= 0) decode(tile, nimg, oy0, ox0);
    const uint32_t dst = mybuf + (uint32_t)(b * WR_BUF);
    if (ups == 0 && oy0 >= 1 && oy0 - 1 + WR_PR <= a.in_h && ox0 >= 1 && ox0 - 1 + WR_PC <= a.in_w) {
      // interior (wave-uniform): the corner's offset on the scalar unit, one add per instruction
      const uint32_t corner = (uint32_t)(nimg * a.in_h + oy0 - 1) * (uint32_t)a.in_w + (uint32_t)(ox0 - 1);
      const uint32_t base = (corner * (uint32_t)a.in_cs + (uint32_t)a.in_co) * 2u;
#pragma unroll
      for (int i = 0; i < WR_NI; ++i) glds(base + rel[i], dst + (uint32_t)(i * 1024));
    } else {
#pragma unroll
      for (int i = 0; i < WR_NI; ++i) {
        const int iy = oy0 - 1 + (dg[i] >> 16), ix = ox0 - 1 + ((dg[i] >> 8) & 255), c = dg[i] & 255;
        const bool ok = dg[i] >= 0 && iy >= 0 && iy < lh && ix >= 0 && ix < lw;
        const uint32_t off = (uint32_t)((((long)(nimg * a.in_h + (iy >> ups)) * a.in_w + (ix >> ups)) * a.in_cs + a.in_co + c * 8) * 2);
        glds(ok ? off : BUF_OOB, dst + (uint32_t)(i * 1024));
      }
    }
  };

  const __amdgpu_buffer_rsrc_t yr = buf_rsrc(a.y, a.y_bytes);
  const __amdgpu_buffer_rsrc_t pr = buf_rsrc(a.ch_part, SUMS && a.ch_part ? (uint32_t)a.ntiles * 256u : 0u);
  const __amdgpu_buffer_rsrc_t rr = buf_rsrc(a.res1, (EP == 1 || EP == 2) ? a.r1_bytes : 0u);
  const int lb = col * WR_XP * 2 + g * 16;  // this lane's byte offset in a footprint row: pixel col, channels 8 g ..
  if (SUMS && a.wg_sums && tid == 0) *wr_wg_count(smem) = 0u;  // (before the barriers every wave passes)
  if (T < a.ntiles) issue(T, 0);
  // the weights: this wave's 18 pieces have landed once only the footprint just requested is younger; after the
  // barrier every wave's have, and every wave copies all 72 fragments to its registers; the second barrier retires
  // those reads before any second footprint buffer (where the pieces lie) is written
  if (T < a.ntiles) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WR_NI) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  bf16x8 afb[4][18];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int j = 0; j < 18; ++j) afb[t][j] = *(const bf16x8*)(smem + wr_piece(18 * t + j) + lane * 16);
  lds_barrier();
  if (T >= a.ntiles) return;
  const int T0 = T;
  float wsum = 0.f;  // (wg_sums) this lane's channel over the wave's tiles, in tile order
  for (int it = 0;; ++it) {
    const int Tn = T + G4;
    issue(Tn < a.ntiles ? Tn : -1, (it + 1) & 1);
    // tile T's footprint has landed once at most the younger operations are outstanding: the last epilogue's and
    // the DMA just issued
    if (it == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WR_NI) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WR_NI + NEPI) : "memory");
    const char* xb = smem + (wv * 2 + (it & 1)) * WR_BUF + lb;
    f32x4 acc[4][4];  // [output row m][co block t]
    bf16x8 bq[2][4];
    auto ldb = [&](int j, int s) {  // k block j = tap j / 2, channels 32 (j % 2) ..: the 4 rows' B fragments
      const int tap = j >> 1, ky = tap / 3, kx = tap % 3;
#pragma unroll
      for (int m = 0; m < 4; ++m) bq[s][m] = *(const bf16x8*)(xb + ((m + ky) * WR_PC + kx) * WR_XP * 2 + (j & 1) * 64);
    };
    ldb(0, 0);
#pragma unroll
    for (int j = 0; j < 18; ++j) {
      if (j + 1 < 18) ldb(j + 1, (j + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        if (j == 0) mfma4x_agpr<true, false>(acc[m][0], acc[m][1], acc[m][2], acc[m][3], afb[0][j], afb[1][j], afb[2][j], afb[3][j], bq[0][m]);
        else if (j < 6) mfma4x_agpr<false, false>(acc[m][0], acc[m][1], acc[m][2], acc[m][3], afb[0][j], afb[1][j], afb[2][j], afb[3][j], bq[j & 1][m]);
        else mfma4x_agpr<false, true>(acc[m][0], acc[m][1], acc[m][2], acc[m][3], afb[0][j], afb[1][j], afb[2][j], afb[3][j], bq[j & 1][m]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    pad_mfma16(acc);
    // ---- epilogue straight from the accumulators: lane (col, g) holds co 16 t + 4 g .. + 3 of pixel (m, col);
    // every lane issues the same number of loads / stores (out-of-range offsets are dropped)
    int nimg, oy0, ox0;
    decode(T, nimg, oy0, ox0);
    const int ox = ox0 + col;
    if constexpr (EP == 5) {
      // pooled pixel (oy0 / 2 + mp, ox / 2): rows m = 2 mp, 2 mp + 1 in registers, columns col / col ^ 1 across lanes
      // (both lanes hold the result); of each co-block pair (t, t + 1) the even lane stores block t, the odd one t + 1
      const int ph = a.out_h >> 1, pw = a.out_w >> 1, px = ox >> 1, odd = col & 1;
#pragma unroll
      for (int mp = 0; mp < 2; ++mp) {
        const int py = (oy0 >> 1) + mp;
        const bool ok = py < ph && px < pw;
        const uint32_t po = ok ? (uint32_t)(((((long)nimg * ph + py) * pw + px) * a.out_cs + a.out_co + 4 * g) * 2) : BUF_OOB;
#pragma unroll
        for (int tp = 0; tp < 4; tp += 2) {
          float w[4];  // block tp + odd: both blocks' maxima are formed (the xor shuffle needs every lane), one kept
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float m2[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              float x0 = acc[2 * mp][tp + u][i] + bias[tp + u][i], x1 = acc[2 * mp + 1][tp + u][i] + bias[tp + u][i];
              if constexpr (ACT == 1) {
                x0 = fmaxf(x0, x0 * a.slope);
                x1 = fmaxf(x1, x1 * a.slope);
              } else if constexpr (ACT == 2) {
                x0 = x0 > 0.f ? x0 : 0.f;
                x1 = x1 > 0.f ? x1 : 0.f;
              }
              const float rm = fmaxf(x0, x1);
              m2[u] = fmaxf(rm, __shfl_xor(rm, 1));
            }
            w[i] = odd ? m2[1] : m2[0];
          }
          const bf16x2 p0 = {(__bf16)w[0], (__bf16)w[1]}, p1 = {(__bf16)w[2], (__bf16)w[3]};
          const v2u32 pk = {__builtin_bit_cast(uint32_t, p0), __builtin_bit_cast(uint32_t, p1)};
          __builtin_amdgcn_raw_buffer_store_b64(pk, yr, po == BUF_OOB ? BUF_OOB : po + (uint32_t)((tp + odd) * 32), 0, 0);
        }
      }
      if (Tn >= a.ntiles) break;
      T = Tn;
      continue;
    }
    uint32_t off[4];
    uint2 rv[4][4];
    v2u32 pkm[4];  // bf16 forms: this row's four packed 4-channel groups (co blocks t)
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int oy = oy0 + m;
      const bool ok = oy < a.out_h && ox < a.out_w;
      const long pix = ((long)nimg * a.out_h + oy) * a.out_w + ox;
      // fp32 (EP 3): channels 16 t + 4 g ..; bf16: the 8 channels 16 (t0 + (g & 1)) + 8 (g >> 1) .. of co-block pair t0
      off[m] = ok ? (uint32_t)((pix * a.out_cs + a.out_co + (EP == 3 ? 4 * g : 16 * (g & 1) + 8 * (g >> 1))) * (EP == 3 ? 4 : 2))
                  : BUF_OOB;
      if constexpr (EP == 1 || EP == 2) {
        const uint32_t ro = ok ? (uint32_t)((pix * a.r1_cs + a.r1_co + 4 * g) * 2) : BUF_OOB;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const auto v = __builtin_amdgcn_raw_buffer_load_b64(rr, ro == BUF_OOB ? BUF_OOB : ro + (uint32_t)(t * 32), 0, 0);
          rv[m][t] = make_uint2(v[0], v[1]);
        }
      }
    }
    float csum[4][4] = {};  // EP 3 / 4: this lane's channel sums over its 4 pixels (rows)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float x = acc[m][t][i] + bias[t][i];
          if constexpr (EP == 2) {
            const uint32_t w = i < 2 ? rv[m][t].x : rv[m][t].y;
            const float r = __uint_as_float((i & 1) ? (w & 0xFFFF0000u) : (w << 16));
            x = r > 0.f ? x : (ACT == 3 ? x * a.slope : 0.f);
          } else {
            if constexpr (ACT == 1) x = fmaxf(x, x * a.slope);  // = (x > 0 ? x : slope x) for 0 <= slope <= 1 (host)
            else if constexpr (ACT == 2) x = x > 0.f ? x : 0.f;
            if constexpr (EP == 1) {
              const uint32_t w = i < 2 ? rv[m][t].x : rv[m][t].y;
              const float r = __uint_as_float((i & 1) ? (w & 0xFFFF0000u) : (w << 16));
              x = x * a.alpha1 + a.beta1 * r;
            }
          }
          v[i] = x;
        }
        if constexpr (EP == 3) {
          const v4u32 pk = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
          __builtin_amdgcn_raw_buffer_store_b128(pk, yr, off[m] == BUF_OOB ? BUF_OOB : off[m] + (uint32_t)(t * 64), 0, 0);
          if (off[m] != BUF_OOB) {
#pragma unroll
            for (int i = 0; i < 4; ++i) csum[t][i] += v[i];
          }
        } else {
          const bf16x2 p0 = {(__bf16)v[0], (__bf16)v[1]}, p1 = {(__bf16)v[2], (__bf16)v[3]};
          pkm[t] = (v2u32){__builtin_bit_cast(uint32_t, p0), __builtin_bit_cast(uint32_t, p1)};
          if (EP == 4 && off[m] != BUF_OOB) {
#pragma unroll
            for (int i = 0; i < 4; ++i) csum[t][i] += v[i];
          }
          if (t & 1) {
            // co blocks t - 1, t: rows 1, 3 of block t - 1 <-> rows 0, 2 of block t (v_permlane16_swap), so lane (col, g)
            // holds channels 16 (t - 1 + (g & 1)) + 8 (g >> 1) .. + 7 of pixel (m, col): one 16-B store
            const auto sx = __builtin_amdgcn_permlane16_swap(pkm[t - 1][0], pkm[t][0], false, false);
            const auto sy = __builtin_amdgcn_permlane16_swap(pkm[t - 1][1], pkm[t][1], false, false);
            const v4u32 o = {sx[0], sy[0], sx[1], sy[1]};
            __builtin_amdgcn_raw_buffer_store_b128(o, yr, off[m] == BUF_OOB ? BUF_OOB : off[m] + (uint32_t)((t - 1) * 32), 0, 0);
          }
        }
      }
    if constexpr (SUMS) {
      // per-tile channel sums: the lanes' column sums transposed through this wave's LDS corner ([channel][17]: both
      // passes conflict-free), then lane l adds channel l's 16 columns in order and stores it (one 4 B store a lane;
      // the xor-shuffle tree it replaces took 64 ds_bpermute per lane).  Wave-private: LDS order within the wave suffices.
      float* red = (float*)(smem + WR_LDS) + wv * (WR_RED / 4);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) red[(16 * t + 4 * g + i) * 17 + col] = csum[t][i];
      float cs = 0.f;
#pragma unroll
      for (int c = 0; c < 16; ++c) cs += red[lane * 17 + c];
      wsum += cs;
      // (wg_sums: the store still issues, out of range, so every tile's vector-memory count stays the same)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(cs), pr, a.wg_sums ? BUF_OOB : (uint32_t)((T * 64 + lane) * 4), 0, 0);
    }
    if (Tn >= a.ntiles) break;
    T = Tn;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the zero-filling DMA past the last tile lands before the wave ends
  if constexpr (SUMS) {
    if (a.wg_sums) {  // (uniform) row blockIdx.x = the sums of the workgroup's waves with tiles, added in wave order by
                      // the last of them to arrive (the LDS counter; no barrier, so the waves without a tile may leave)
      const float* red0 = (const float*)(smem + WR_LDS);
      ((float*)red0)[wv * (WR_RED / 4) + lane] = wsum;  // (this wave's own corner: its transpose reads are behind it)
      const int nact = min(4, a.ntiles - (T0 - wv));
      uint32_t prev = 0;
      if (lane == 0) prev = __hip_atomic_fetch_add(wr_wg_count(smem), 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
      if ((int)__builtin_amdgcn_readfirstlane(prev) == nact - 1) {
        float t = 0.f;
        for (int w = 0; w < nact; ++w) t += red0[w * (WR_RED / 4) + lane];
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(t), pr, (uint32_t)((blockIdx.x * 64 + lane) * 4), 0, 0);
      }
    }
  }
}

}  // namespace

namespace climsr {

// the conv_wr epilogue for (d, ep), or -1 when the conv is not this kernel's: 0 bias / activation, bf16 out; 1 + bf16
// residual; 2 activation backward from the stored activation (no bias); 3 bias / activation, fp32 out (+ per-tile
// channel sums); 4 bias / activation, bf16 out + per-tile channel sums (of the fp32 values).  The bf16 forms store 16 B
// per lane (8 channels): their output offset and stride must be multiples of 8 channels.
int conv_wr_ep(const ClimsrConvDesc* d, const ClimsrEpilogue* ep, const float* bias) {
  const bool res = ep->res1 != nullptr;
  int epk = -1;
  if (ep->out_mode == 0 && !res && ep->act >= 0 && ep->act <= 2) epk = ep->pool2 ? 5 : (ep->ch_part ? 4 : 0);
  else if (ep->out_mode == 0 && res && ep->act == 0 && !(ep->res_f32 & 1)) epk = 1;
  else if (ep->out_mode == 0 && res && (ep->act == 3 || ep->act == 4) && !bias && !(ep->res_f32 & 1)) epk = 2;
  else if (ep->out_mode == 1 && !res && ep->act >= 0 && ep->act <= 2) epk = 3;
  const long opx = (long)d->n * d->out_h * d->out_w;
  if (epk < 0 || (ep->ch_part && epk != 3 && epk != 4) || (ep->pool2 && (epk != 5 || ep->ch_part || (d->out_h | d->out_w) & 1)) || (ep->act == 1 && !(ep->slope >= 0.f && ep->slope <= 1.f)) || d->in_c != 64 || d->out_c != 64 || d->cc != 64 || d->ks != 3 || d->stride != 1 ||
      d->pad != 1 || (d->up != 1 && d->up != 2) || d->out_h != d->in_h * d->up || d->out_w != d->in_w * d->up ||
      d->in_cstride % 8 || d->in_coff % 8 || (d->out_cstride | d->out_coff) & (epk == 3 ? 3 : 7) || ep->down2 || ep->res2 || ep->aux ||
      ep->bn_part || (res && ((ep->res1_cstride | ep->res1_coff) & 3)) ||
      (long)d->n * d->in_h * d->in_w * d->in_cstride * 2 >= (1L << 31) ||
      opx * d->out_cstride * (epk == 3 ? 4 : 2) >= (1L << 31) || (res && opx * ep->res1_cstride * 2 >= (1L << 31)) ||
      (long)ceil_div(d->out_w, WR_TC) * ceil_div(d->out_h, WR_TR) * d->n * 256 >= (1L << 31))
    return -1;
  return epk;
}

// rows of ch_part (tiles, or with one image the workgroups of the launch) of the conv, and per image; 0 when conv_wr
// does not take (d, ep)
long conv_wr_ch_parts(const ClimsrConvDesc* d, const ClimsrEpilogue* ep, int* tiles_per_image) {
  ClimsrEpilogue e = *ep;
  e.ch_part = (float*)1;  // (only its presence matters here)
  const int k = conv_wr_ep(d, &e, nullptr);
  if (k != 3 && k != 4) return 0;
  const int tpi = ceil_div(d->out_w, WR_TC) * ceil_div(d->out_h, WR_TR);
  if (d->n == 1) {  // one row per workgroup (conv_wr_launch's grid)
    const int rows = std::min(ceil_div(tpi, 4), device_cus());
    if (tiles_per_image) *tiles_per_image = rows;
    return rows;
  }
  if (tiles_per_image) *tiles_per_image = tpi;
  return (long)tpi * d->n;
}

int conv_wr_launch(const ClimsrConvDesc* d, const ClimsrEpilogue* ep, const uint16_t* x, const uint16_t* wpk, int kpk,
                   const float* bias, void* y, hipStream_t s, bool dry, char* name, int name_len) {
  const int epk = conv_wr_ep(d, ep, bias);
  const bool res = ep->res1 != nullptr;
  const long opx = (long)d->n * d->out_h * d->out_w;
  if (epk < 0 || kpk < 576) return -1;
  if (dry) {
    snprintf(name, name_len, "conv_wr_kernel<%d, %d>", epk, ep->act);
    return CLIMSR_OK;
  }
  WrArgs a;
  a.x = x; a.w = wpk; a.bias = bias; a.y = (uint16_t*)y; a.res1 = (const uint16_t*)ep->res1; a.ch_part = ep->ch_part;
  a.n = d->n; a.in_h = d->in_h; a.in_w = d->in_w; a.in_cs = d->in_cstride; a.in_co = d->in_coff; a.up = d->up;
  a.out_h = d->out_h; a.out_w = d->out_w; a.out_cs = d->out_cstride; a.out_co = d->out_coff; a.kpk = kpk;
  a.act = ep->act; a.slope = ep->slope; a.alpha1 = ep->alpha1; a.beta1 = ep->beta1;
  a.r1_cs = ep->res1_cstride; a.r1_co = ep->res1_coff;
  a.tiles_x = ceil_div(d->out_w, WR_TC); a.tiles_y = ceil_div(d->out_h, WR_TR);
  a.ntiles = a.tiles_x * a.tiles_y * d->n;
  a.wg_sums = (epk == 3 || epk == 4) && ep->ch_part && d->n == 1;
  a.x_bytes = (uint32_t)((long)d->n * d->in_h * d->in_w * d->in_cstride * 2);
  a.y_bytes = (uint32_t)((epk == 5 ? opx / 4 : opx) * d->out_cstride * (epk == 3 ? 4 : 2));
  a.r1_bytes = res ? (uint32_t)(opx * ep->res1_cstride * 2) : 0u;
  const int ncu = device_cus();
  const int grid = std::min(ceil_div(a.ntiles, 4), ncu);
  // [epilogue][activation] (EP 1: no activation; EP 2: 3 / 4)
  static void (*const kt[6][5])(WrArgs) = {
      {conv_wr_kernel<0, 0>, conv_wr_kernel<0, 1>, conv_wr_kernel<0, 2>, nullptr, nullptr},
      {conv_wr_kernel<1, 0>, nullptr, nullptr, nullptr, nullptr},
      {nullptr, nullptr, nullptr, conv_wr_kernel<2, 3>, conv_wr_kernel<2, 4>},
      {conv_wr_kernel<3, 0>, conv_wr_kernel<3, 1>, conv_wr_kernel<3, 2>, nullptr, nullptr},
      {conv_wr_kernel<4, 0>, conv_wr_kernel<4, 1>, conv_wr_kernel<4, 2>, nullptr, nullptr},
      {conv_wr_kernel<5, 0>, conv_wr_kernel<5, 1>, conv_wr_kernel<5, 2>, nullptr, nullptr}};
  void (*k)(WrArgs) = (ep->act >= 0 && ep->act < 5) ? kt[epk][ep->act] : nullptr;
  if (!k) {
    set_error("conv2d_fwd (wr): epilogue %d with activation %d", epk, ep->act);
    return CLIMSR_EINVAL;
  }
  const int lds = WR_LDS_ALL;  // (every form: the last 4 weight pieces are staged in the channel-sum region)
  if (int e = lds_opt_in((const void*)k, WR_LDS_ALL)) return e;
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, s, a);
  return check_launch("conv2d_fwd (wr)");
}

}  // namespace climsr
