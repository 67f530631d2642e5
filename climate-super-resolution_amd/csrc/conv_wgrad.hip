// Weight gradients of the implicit-GEMM convolutions for CDNA4 (gfx950): the backward of nn.Conv2d's weight and
// bias on the ESRGAN / SRCNN / RCAN / VGG-discriminator hot path (climsr/models/esrgan.py:17-102, srcnn.py:6-18,
// rfb_esrgan.py:26-61), split from conv.hip (forward and data gradient) so the two translation units compile in
// parallel and the LDS-DMA wait lint (tests/test_isa_waitcnt.py) compiles only the file that holds conv_wgrad64_glds.
// Layout and MFMA conventions are conv.hip's: activations NHWC bf16, v_mfma_f32_16x16x32_bf16.
#include <stdio.h>

#include "common.h"
#include "conv_ep.h"

using namespace climsr;

constexpr int FWD_MAXV = 8;  // 16 B staging vectors per thread held in registers (as conv.hip's forward)
// ------------------------------------------------------------------------------------------
// Weight gradient: dW[co][ci][tap] = sum_px dz[px][co] * x[px*stride + tap - pad][ci]
// GEMM: M = co (A = dz^T), N = ci (B = x), K = pixels.  Both operands are pixel-major in NHWC, so
// they are read from LDS with ds_read_b64_tr_b16 (row = pixel, any per-lane pixel address: the
// tap shift of the im2col is free).  WG tile: 16*NTC co x 16 ci x TB taps; the 4 waves split the
// pixels of each 16x16 output-pixel tile and are summed through LDS at the end; splits over
// pixel tiles write disjoint fp32 partial slabs (deterministic, reduced by wgrad_reduce).
// ------------------------------------------------------------------------------------------
constexpr int WG_TH = 16;
constexpr int WG_XP = 24;  // LDS pixel pitch (channels) of the x tile (16 + 8 pad)

struct WgArgs {
  const uint16_t* x;
  const uint16_t* dz;
  float* part;
  float* bpart;
  int n, in_h, in_w, in_c, in_cs, in_co, up, ks, stride, pad, out_h, out_w, out_c, dz_cs;
  int tph, tpw, dzp, tiles_x, tiles_y, ntiles, nsplit, ntapb, ncib, co_rows, kw;
  int lds_x;
  int xcd;  // conv_wgrad64_kernel: 1-D grid in XCD-major (split, channel block) order (else blockIdx.y = split)
};

// CI4 = 1: inputs with <= 4 real channels (srcnn.conv1 / conv_first, 3 channels).  The x tile holds 4
// channels per pixel and a B fragment's 16 columns are (4 taps x 4 channels): in the transposed read
// each lane group p points at its own tap, so 81 taps need 21 fragments instead of 81 mostly-zero ones.
// TB then counts tap groups of 4.
// WS (wave-split taps, CI4 9x9 = srcnn.conv1): one workgroup covers ALL tap groups, wave w owns groups
// [TB w, TB w + TB) over every pixel of the tile, so dz is read once per launch (the tap-blocked form re-reads it
// per block: 1 GB fetched for 0.3 GB of data) and no cross-wave reduction is needed.
template <int NTC, int TB, int CI4, bool WS = false>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* xs = (uint16_t*)smem;
  uint16_t* zs = (uint16_t*)(smem + a.lds_x);
  float* red = (float*)smem;  // reused for the cross-wave reduction at the end

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int g = lane >> 4;
  const int q = (lane & 15) >> 2;
  const int p = lane & 3;
  const int col = lane & 15;

  int bid = blockIdx.x;
  const int tb = bid % a.ntapb;
  bid /= a.ntapb;
  const int cib = bid % a.ncib;
  const int cob = bid / a.ncib;
  const int split = blockIdx.y;
  const int ci0 = cib * 16;
  const int co0 = cob * NTC * 16;
  const int tap0 = (WS ? wave : tb) * TB * (CI4 ? 4 : 1);
  constexpr int XP = CI4 ? 4 : WG_XP;  // LDS x-tile pixel pitch (channels)
  const int ks2 = a.ks * a.ks;
  const bool do_bias = (cib == 0 && tb == 0 && a.bpart != nullptr) && (!WS || wave == 0);

  f32x4 acc[NTC][TB];
  f32x4 accb[NTC];
#pragma unroll
  for (int t = 0; t < NTC; ++t) {
    accb[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < TB; ++u) acc[t][u] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  bf16x8 ones;
#pragma unroll
  for (int i = 0; i < 8; ++i) ones[i] = (__bf16)1.0f;

  int tapoff[TB];  // per-lane LDS offset of fragment u's columns (4p..4p+3)
#pragma unroll
  for (int u = 0; u < TB; ++u) {
    int tap = CI4 ? tap0 + 4 * u + p : tap0 + u;
    if (tap >= ks2) tap = 0;  // weight rows past ks*ks are never written
    tapoff[u] = ((tap / a.ks) * a.tpw + (tap % a.ks)) * XP + (CI4 ? 0 : 4 * p);
  }

  const int lh = a.in_h * a.up, lw = a.in_w * a.up;  // up in {1, 2} here
  const int upsh = a.up == 2 ? 1 : 0;
  constexpr int zvec = NTC * 2;  // 16B vectors of dz per pixel
  constexpr int XSTEP = CI4 ? 256 : 128;  // pixels advanced per 256 staging vectors
  const int x_dy = XSTEP / a.tpw, x_dx = XSTEP - x_dy * a.tpw;
  const int xpix0 = CI4 ? tid : (tid >> 1);
  const int x_ty0 = xpix0 / a.tpw, x_tx0 = xpix0 - x_ty0 * a.tpw;
  const int nvec_x = a.tph * a.tpw * (CI4 ? 1 : 2);
  const int nvec_z = WG_TH * TW * zvec;

  for (int tile = split; tile < a.ntiles; tile += a.nsplit) {
    int tt = tile;
    const int tx = tt % a.tiles_x;
    tt /= a.tiles_x;
    const int ty = tt % a.tiles_y;
    const int nimg = tt / a.tiles_y;
    const int ox0 = tx * TW, oy0 = ty * WG_TH;
    const int iy0 = oy0 * a.stride - a.pad, ix0 = ox0 * a.stride - a.pad;
    __syncthreads();
    // batched staging (all loads of a round in flight before the first LDS store); x-tile pixel
    // coordinates advance incrementally (thread's pixels are (tid>>1) + 128k, channel half tid&1)
    {
      const int h = tid & 1;
      int ty_ = x_ty0, tx_ = x_tx0;
      const int nrx = (nvec_x + 255) / 256;
      for (int base = 0; base < nrx; base += FWD_MAXV) {
        uint4 buf[FWD_MAXV];
        int dst[FWD_MAXV];
#pragma unroll
        for (int i = 0; i < FWD_MAXV; ++i) {
          dst[i] = -1;
          if (base + i < nrx && ty_ < a.tph) {
            const int iy = iy0 + ty_, ix = ix0 + tx_;
            const int c = ci0 + (CI4 ? 0 : h * 8);
            uint4 val = make_uint4(0, 0, 0, 0);
            const bool ok = iy >= 0 && iy < lh && ix >= 0 && ix < lw && c < a.in_c;
            const long src = (((long)nimg * a.in_h + (iy >> upsh)) * a.in_w + (ix >> upsh)) * a.in_cs + a.in_co + c;
            if (CI4) {
              if (ok) {
                uint2 v2 = *(const uint2*)(a.x + src);
                val.x = v2.x;
                val.y = v2.y;
              }
            } else if (ok) {
              val = *(const uint4*)(a.x + src);
            }
            buf[i] = val;
            dst[i] = (ty_ * a.tpw + tx_) * XP + (CI4 ? 0 : h * 8);
          }
          tx_ += x_dx;
          ty_ += x_dy;
          if (tx_ >= a.tpw) { tx_ -= a.tpw; ++ty_; }
        }
#pragma unroll
        for (int i = 0; i < FWD_MAXV; ++i) {
          if (dst[i] < 0) continue;
          if (CI4) *(uint2*)(xs + dst[i]) = make_uint2(buf[i].x, buf[i].y);
          else *(uint4*)(xs + dst[i]) = buf[i];
        }
      }
      const int nrz = nvec_z / 256;  // exact: 256 px x zvec vectors
      for (int base = 0; base < nrz; base += FWD_MAXV) {
        uint4 buf[FWD_MAXV];
#pragma unroll
        for (int i = 0; i < FWD_MAXV; ++i) {
          if (base + i < nrz) {
            const int vz = tid + (base + i) * 256;
            const int pix = vz / zvec;  // zvec = 2*NTC: compile-time power of two
            const int cv = vz - pix * zvec;
            const int oy = oy0 + pix / TW, ox = ox0 + (pix % TW);
            const int c = co0 + cv * 8;
            uint4 val = make_uint4(0, 0, 0, 0);
            if (oy < a.out_h && ox < a.out_w && c < a.dz_cs)
              val = *(const uint4*)(a.dz + (((long)nimg * a.out_h + oy) * a.out_w + ox) * a.dz_cs + c);
            buf[i] = val;
          }
        }
#pragma unroll
        for (int i = 0; i < FWD_MAXV; ++i) {
          if (base + i < nrz) {
            const int vz = tid + (base + i) * 256;
            const int pix = vz / zvec;
            *(uint4*)(zs + pix * a.dzp + (vz - pix * zvec) * 8) = buf[i];
          }
        }
      }
    }
    __syncthreads();
#pragma unroll 2  // (a full unroll of the WS variant's 8 k-steps made hipcc copy the accumulators AGPR<->VGPR)
    for (int s = 0; s < (WS ? 8 : 2); ++s) {
      const int kk = WS ? s : wave * 2 + s;  // k-step: output pixel rows 2kk, 2kk+1 of the tile
      // pixel handled as row q (+4) of this lane's tr reads
      const int k0 = kk * 32 + 8 * g + q;
      const int k1 = k0 + 4;
      const int r0 = k0 >> 4, c0_ = k0 & 15, r1 = k1 >> 4, c1_ = k1 & 15;
      bf16x8 af[NTC];
#pragma unroll
      for (int t = 0; t < NTC; ++t) {
        s16x4 lo = ds_read_tr16(zs + k0 * a.dzp + t * 16 + 4 * p);
        s16x4 hi = ds_read_tr16(zs + k1 * a.dzp + t * 16 + 4 * p);
        short v8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[t] = __builtin_bit_cast(bf16x8, v8);
      }
      const int xb0 = ((r0 * a.stride) * a.tpw + c0_ * a.stride) * XP;
      const int xb1 = ((r1 * a.stride) * a.tpw + c1_ * a.stride) * XP;
      if (do_bias) {
#pragma unroll
        for (int t = 0; t < NTC; ++t) accb[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], ones, accb[t], 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < TB; ++u) {
        s16x4 lo = ds_read_tr16(xs + xb0 + tapoff[u]);
        s16x4 hi = ds_read_tr16(xs + xb1 + tapoff[u]);
        short v8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bf16x8 bfr = __builtin_bit_cast(bf16x8, v8);
#pragma unroll
        for (int t = 0; t < NTC; ++t) acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bfr, acc[t][u], 0, 0, 0);
      }
    }
  }

  // cross-wave reduction through LDS (waves 1..3 -> wave 0)
  constexpr int NF = NTC * TB;
  for (int r = 1; r < (WS ? 1 : 4); ++r) {
    __syncthreads();
    if (wave == r) {
#pragma unroll
      for (int t = 0; t < NTC; ++t)
#pragma unroll
        for (int u = 0; u < TB; ++u) *(f32x4*)(red + ((t * TB + u) * 64 + lane) * 4) = acc[t][u];
#pragma unroll
      for (int t = 0; t < NTC; ++t) *(f32x4*)(red + ((NF + t) * 64 + lane) * 4) = accb[t];
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int t = 0; t < NTC; ++t) {
#pragma unroll
        for (int u = 0; u < TB; ++u) acc[t][u] += *(f32x4*)(red + ((t * TB + u) * 64 + lane) * 4);
        accb[t] += *(f32x4*)(red + ((NF + t) * 64 + lane) * 4);
      }
    }
  }
  if (!WS && wave != 0) return;
  const int ci = CI4 ? (col & 3) : ci0 + col;
  float* slab = a.part + (long)split * a.co_rows * a.kw;
#pragma unroll
  for (int t = 0; t < NTC; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = co0 + t * 16 + g * 4 + i;
      if (ci < a.in_c) {
#pragma unroll
        for (int u = 0; u < TB; ++u) {
          const int tap = CI4 ? tap0 + 4 * u + (col >> 2) : tap0 + u;
          if (tap < ks2) slab[(long)co * a.kw + ci * ks2 + tap] = acc[t][u][i];
        }
      }
      if (do_bias && col == 0) a.bpart[(long)split * a.co_rows + co] = accb[t][i];
    }
  }
}

// Weight gradient for 3x3 stride-1 convs with 64k output and 64k input channels (the RDB conv5 / the
// whole-RDB combined GEMM, trunk / upconv / HRconv): workgroup block = 64 co x 64 ci x 9 taps, wave w owns
// ci 16w..16w+15 (4 co fragments x 9 taps = 36 accumulators), so the workgroup's 4 waves never reduce with
// each other; the 8x16-pixel tiles of its split are walked with the NEXT tile's dz / x prefetched into
// registers while the current one is on the MFMA pipe.  Partials: [split][co_rows][in_c*9] (as above).
// Stride 2 (the discriminator's features.2/8/14/20): 4 x 16 output tiles whose (2*4+1) x (2*16+1) input
// footprint is staged whole; tap (r, s) of output pixel k reads tile pixel (2*row(k) + r, 2*col(k) + s).
// LDS pixel pitches (channels).  A transposed fragment read (ds_read_b64_tr_b16) is served 32 lanes at a time:
// with the k-step's pixel rows taken as 4g + q (+16), those 32 lanes read 8 consecutive tile pixels, 32 B each,
// which land in 8 disjoint 8-bank groups when one pixel step is 8 x odd banks: pitch 80 (dz tile; x tile at
// stride 1) or 72 (x tile at stride 2, where a pixel step is two tile pixels).  The old 72 / rows 8g + q left
// SQ_LDS_BANK_CONFLICT at 42 % of the LDS cycles.
constexpr int W64_P = 64 + 8;  // (dzp of the generic wgrad path's descriptor)
constexpr int W64_ZP = 80;
template <int S>
struct W64 {
  static constexpr int TH = S == 1 ? 8 : 4;                    // output tile rows (x TW = 16 columns)
  static constexpr int TPH = S * (TH - 1) + 3, TPW = S * (TW - 1) + 3;  // staged input footprint
  static constexpr int XP = S == 1 ? 80 : 72;                 // x tile pixel pitch
  static constexpr int NZ = TH * TW * 8;                      // 16 B vectors of a dz tile (TH*16 px x 64 ch)
  static constexpr int NX = TPH * TPW * 8;                    // of an x tile
  // + one spare x pixel: the stash's lanes past the tile write there (no branch in the tile loop)
  static constexpr size_t LDS = (size_t)TH * TW * W64_ZP * 2 + (size_t)(TPH * TPW + 1) * XP * 2;
};

// TS = 2: 8 waves, wave w owns ci block w & 3 and taps [0,5) or [5,9) (w >> 2): 20 accumulators instead of 36, so
// two waves share each SIMD (latency hiding) at the price of each wave re-reading the shared dz fragments.
// G (TS 1): the LDS-DMA form -- see conv_wgrad64_glds_kernel below.
template <int TS, int S, bool G>
__device__ __forceinline__ void wgrad64_body(const WgArgs& a) {
  static_assert(!G || TS == 1, "LDS-DMA form: 4-wave quads");
  // G at stride 1: two wave quads (512 threads), each walking every other tile of the split with its own two tile
  // buffers, their sums added through LDS at the end -- two waves per SIMD at the same split count (slab volume)
  constexpr int QG = (G && S == 1) ? 2 : 1;
  constexpr int NTHR = 256 * TS * QG, NU = TS == 1 ? 9 : 5;
  constexpr int TH = W64<S>::TH, TPW = W64<S>::TPW, NZ = W64<S>::NZ, NX = W64<S>::NX, XP = W64<S>::XP;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // TS 1: two buffers of W64<S>::LDS
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
  const int wave = (tid >> 6) & 3, tg = TS == 1 ? 0 : tid >> 8;  // ci block, tap group
  const int quad = QG == 2 ? __builtin_amdgcn_readfirstlane(tid >> 8) : 0;  // (wave-uniform: LDS-DMA destinations are scalar)
  const int u0 = tg * 5;
  const int q = (lane & 15) >> 2, p = lane & 3, col = lane & 15;
  // (split, 64x64 block): with a.xcd the XCD-major order in which a split's blocks are consecutive on one XCD -- they
  // walk the same pixel tiles at the same time, so each x / dz tile is fetched into that L2 once for all of them
  const int nblk = a.ncib * (a.out_c / 64);
  const int bidx = a.xcd ? xcd_major(blockIdx.x, gridDim.x) : blockIdx.x;
  const int blk = a.xcd ? bidx % nblk : bidx, split = a.xcd ? bidx / nblk : blockIdx.y;
  const int cib = blk % a.ncib, cob = blk / a.ncib;
  const int ci0 = cib * 64, co0 = cob * 64;
  const bool do_bias = cib == 0 && a.bpart != nullptr;
  const int lh = a.in_h * a.up, lw = a.in_w * a.up;
  const int upsh = a.up == 2 ? 1 : 0;

  f32x4 acc[4][NU], accb[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    accb[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < NU; ++u) acc[t][u] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  bf16x8 ones;
#pragma unroll
  for (int i = 0; i < 8; ++i) ones[i] = (__bf16)1.0f;
  int tapoff[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    if constexpr (TS == 1) {
      tapoff[u] = ((u / 3) * TPW + (u % 3)) * XP + wave * 16 + 4 * p;
    } else {
      const int tp = u0 + u < 9 ? u0 + u : 8;
      tapoff[u] = ((tp / 3) * TPW + (tp % 3)) * XP + wave * 16 + 4 * p;
    }
  }

  constexpr int VZ = NZ / NTHR, VX = (NX + NTHR - 1) / NTHR;
  uint4 pz[VZ], px[VX];
  // Branch-free tile loads: buffer loads whose byte offset is pushed out of range for halo / ragged lanes return
  // zeros (no branch around a load: hipcc waits vmcnt(0) at each one under a condition, and the per-vector 64-bit
  // address arithmetic of the branchy form was ~20 VALU a vector -- VALU-issue-bound at one wave per SIMD).  Every
  // per-vector term that does not depend on the tile is a per-thread constant.
  // dz vector i: pixel row zr + (NTHR / 128) i, column zc of the tile, channels co0 + 8 (tid & 7)
  const int zr = tid >> 7, zc = (tid >> 3) & 15, cg8 = (tid & 7) * 8;
  const uint32_t zrow_b = (uint32_t)a.out_w * a.dz_cs * 2;
  const uint32_t z_lane = (uint32_t)((zc * a.dz_cs + co0 + cg8) * 2) + (uint32_t)zr * zrow_b;
  const __amdgpu_buffer_rsrc_t zrs = buf_rsrc(a.dz, (uint32_t)((long)a.n * a.out_h * a.out_w * a.dz_cs * 2));
  // x vector i: tile pixel (xpy[i], xpx[i]), channels ci0 + 8 (tid & 7) (the upsample-on-load source: pixel >> 1)
  int xpy[VX], xpx[VX];
#pragma unroll
  for (int i = 0; i < VX; ++i) {
    const int pix = (tid + NTHR * i) >> 3;
    xpy[i] = tid + NTHR * i < NX ? pix / TPW : 1 << 20;  // past the tile: never in range
    xpx[i] = pix % TPW;
  }
  const uint32_t ximg_b = (uint32_t)a.in_h * a.in_w * a.in_cs * 2;
  const uint32_t x_lane = (uint32_t)((a.in_co + ci0 + cg8) * 2);
  const __amdgpu_buffer_rsrc_t xrs = buf_rsrc(a.x, (uint32_t)((long)a.n * a.in_h * a.in_w * a.in_cs * 2));
  // split-strided tile walk with incremental coordinates (no per-tile integer divisions on the scalar pipe)
  const int s_x = a.nsplit % a.tiles_x, s_y = (a.nsplit / a.tiles_x) % a.tiles_y, s_n = a.nsplit / (a.tiles_x * a.tiles_y);
  int ntx = split % a.tiles_x, nty = (split / a.tiles_x) % a.tiles_y, nn = split / (a.tiles_x * a.tiles_y);
  auto issue = [&](bool live) {  // the tile at (ntx, nty, nn) (zeros if !live), then advance them by nsplit tiles
    const int tx = ntx, ty = nty, nimg = nn;
    ntx += s_x;
    int c = ntx >= a.tiles_x;
    ntx -= c ? a.tiles_x : 0;
    nty += s_y + c;
    c = nty >= a.tiles_y;
    nty -= c ? a.tiles_y : 0;
    nn += s_n + c;
    const int oy0 = ty * TH, ox0 = tx * TW;
    const uint32_t zt = (uint32_t)(((nimg * a.out_h + oy0) * a.out_w + ox0) * a.dz_cs * 2) + z_lane;
    const bool zok = live && ox0 + zc < a.out_w;
#pragma unroll
    for (int i = 0; i < VZ; ++i) {
      const bool ok = zok && oy0 + zr + (NTHR / 128) * i < a.out_h;
      pz[i] = buf_load16(zrs, ok ? zt + (uint32_t)((NTHR / 128) * i) * zrow_b : BUF_OOB);
    }
    const int iy0 = S * oy0 - a.pad, ix0 = S * ox0 - a.pad;
    const uint32_t xt = (uint32_t)nimg * ximg_b + x_lane;
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      const int iy = iy0 + xpy[i], ix = ix0 + xpx[i];
      const bool ok = live && iy >= 0 && iy < lh && ix >= 0 && ix < lw;
      const uint32_t off = xt + (uint32_t)((((iy >> upsh) * a.in_w) + (ix >> upsh)) * a.in_cs * 2);
      px[i] = buf_load16(xrs, ok ? off : BUF_OOB);
    }
  };
  // buffer b of the staged tiles: dz [TH*16 px][W64_ZP], x [TPH*TPW px][XP]
  auto zbuf = [&](int b) { return (uint16_t*)(smem + b * W64<S>::LDS); };
  auto xbuf = [&](int b) { return (uint16_t*)(smem + b * W64<S>::LDS) + TH * TW * W64_ZP; };
  auto stash = [&](int b) {
    uint16_t* zs = zbuf(b);
    uint16_t* xs = xbuf(b);
#pragma unroll
    for (int i = 0; i < VZ; ++i) {
      const int v = tid + NTHR * i;
      *(uint4*)(zs + (v >> 3) * W64_ZP + (v & 7) * 8) = pz[i];
    }
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      const int v = tid + NTHR * i;
      *(uint4*)(xs + (v < NX ? v >> 3 : W64<S>::TPH * TPW) * XP + (v & 7) * 8) = px[i];  // past the tile: the spare pixel
    }
  };
  // k-step kk = 32 output pixels of the tile; lane group g's 8 k values = pixel rows 4g + q and 16 + 4g + q (a
  // permutation of the k-step's pixels, the same for both operands)
  const bool last_short = TS == 2 && tg == 1;  // tap group 1 has 4 taps (5..8)
  auto frags = [&](int b, int kk, bf16x8 (&af)[4], bf16x8 (&bf)[NU]) {
    const uint16_t* zs = zbuf(b);
    const uint16_t* xs = xbuf(b);
    const int k0 = kk * 32 + 4 * g + q, k1 = k0 + 16;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      af[t] = cat_tr(ds_read_tr16(zs + k0 * W64_ZP + t * 16 + 4 * p), ds_read_tr16(zs + k1 * W64_ZP + t * 16 + 4 * p));
    const int xb0 = (S * (k0 >> 4) * TPW + S * (k0 & 15)) * XP, xb1 = (S * (k1 >> 4) * TPW + S * (k1 & 15)) * XP;
#pragma unroll
    for (int u = 0; u < NU; ++u) bf[u] = cat_tr(ds_read_tr16(xs + xb0 + tapoff[u]), ds_read_tr16(xs + xb1 + tapoff[u]));
  };
  auto mma = [&](const bf16x8 (&af)[4], const bf16x8 (&bf)[NU]) {
    // the bias gradient (sum of dz over the pixels) on every wave: 4 more MFMAs per k-step, but no branch in the tile
    // loop (a wave-uniform branch here made hipcc copy the 144 accumulators between AGPRs and VGPRs every tile);
    // wave 0 of a bias-owning workgroup stores it
#pragma unroll
    for (int t = 0; t < 4; ++t) accb[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], ones, accb[t], 0, 0, 0);
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      if (u == NU - 1 && last_short) continue;
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bf[u], acc[t][u], 0, 0, 0);
    }
  };
  constexpr int NK = TH * TW / 32;  // 4 (stride 1) or 2 (stride 2): even
  int tile = split;
  if constexpr (G) {
    // LDS-DMA staging: buffer_load ... lds writes each wave-instruction's 64 x 16 B straight into LDS at
    // (wave-uniform base + 16 lane), so the tiles need no registers, no ds_write pass and no VALU to move them,
    // and three buffers keep two tiles in flight (the register path held one tile in 40 VGPRs, and with two whole
    // fragment sets its 160 accumulators overflowed into AGPR copies: 4.5 VALU per MFMA).  Images are lane-linear:
    // lane l of an instruction fills pixel slot 8 i + (l >> 3), 16 B position l & 7, with that pixel's channel chunk
    // (l & 7) ^ (column & 7) -- an XOR swizzle chosen on the global (source) side that spreads the 8 pixels of a
    // transposed fragment read over all 64 banks, as the register path's 80-element pitch did.
    // per wave and tile: NZI dz and NXI x instructions (stride 1: 4 + 6, stride 2: 2 + 10)
    constexpr int NZI = TH / 2, NXI = S == 1 ? 6 : 10;
    constexpr int ZB = TH * TW * 128, XB = 4 * NXI * 1024, BUF = ZB + XB, NXP = W64<S>::TPH * TPW;
    constexpr int NB = QG == 2 ? 2 : 3;  // tile buffers per quad (two quads x two, or one quad x three)
    static_assert(4 * NXI * 8 >= NXP && QG * NB * BUF <= 160 * 1024, "LDS-DMA wgrad64 tile buffers");
    const int l8 = lane >> 3, c8 = lane & 7, wv = (tid >> 6) & 3;
    // dz: wave w issues instructions w + 4 j (j < NZI): tile row (w >> 1) + 2 j, column 8 (w & 1) + l8
    const int zcol = 8 * (wv & 1) + l8, zrow0 = wv >> 1;
    const uint32_t zrow_b = (uint32_t)a.out_w * a.dz_cs * 2;
    const uint32_t z_lane = (uint32_t)((zcol * a.dz_cs + co0 + 8 * (c8 ^ (zcol & 7))) * 2) + (uint32_t)zrow0 * zrow_b;
    const __amdgpu_buffer_rsrc_t zrs = buf_rsrc(a.dz, (uint32_t)((long)a.n * a.out_h * a.out_w * a.dz_cs * 2));
    // x: instructions w + 4 j (j < NXI): footprint slot 8 (w + 4 j) + l8 of the 10 x 18 (stride 2: 9 x 33) footprint
    // (the slots past it get zeros): (row << 16) | (column << 8) | source chunk.  Stride 2 stores each footprint row's
    // 17 even columns first, then its 16 odd ones: the stride-2 pixels 2 c + dx of a fragment read then sit in
    // consecutive slots, alternating bank halves as the stride-1 reads do (in column order all of them would share one
    // half of the 64 banks: two-way conflicts)
    int xrc[NXI];
#pragma unroll
    for (int j = 0; j < NXI; ++j) {
      const int P = 8 * (wv + 4 * j) + l8, row = P < NXP ? P / TPW : 1023, slot = P % TPW;
      const int cx = S == 1 ? slot : (slot < (TPW + 1) / 2 ? 2 * slot : 2 * (slot - (TPW + 1) / 2) + 1);
      xrc[j] = (row << 16) | (cx << 8) | (c8 ^ (slot & 7));
    }
    const uint32_t ximg_b = (uint32_t)a.in_h * a.in_w * a.in_cs * 2, pxb = (uint32_t)a.in_cs * 2;
    const uint32_t x_ch = (uint32_t)((a.in_co + ci0) * 2);
    const __amdgpu_buffer_rsrc_t xrs = buf_rsrc(a.x, (uint32_t)((long)a.n * a.in_h * a.in_w * a.in_cs * 2));
    // the quad's tiles: split + (QG i + quad) nsplit
    const int qstep = QG * a.nsplit, qt0 = split + quad * a.nsplit;
    const int s_x = qstep % a.tiles_x, s_y = (qstep / a.tiles_x) % a.tiles_y, s_n = qstep / (a.tiles_x * a.tiles_y);
    int ntx = qt0 % a.tiles_x, nty = (qt0 / a.tiles_x) % a.tiles_y, nn = qt0 / (a.tiles_x * a.tiles_y);
    // in asm, not __builtin_amdgcn_raw_ptr_buffer_load_lds: hipcc treats the builtin as an LDS write of unknown
    // extent and waits vmcnt(0) before the next ds_read, i.e. for the tile just requested; hidden from it, the DMAs
    // are counted by hand (vmcnt(NZI + NXI) below) and drained before the epilogue.  M0 (the wave's LDS destination) is set
    // and restored inside the statement.
    const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;
    const int wvu = __builtin_amdgcn_readfirstlane(wv);  // provably wave-uniform: the LDS destination is an "s" operand
    // lag (tests/isa_waitcnt_lint.py): the hand wait that retires a tile's pieces is the first after their issue for the
    // prologue's tile 0, the second for every later tile (one more tile is requested behind it)
    bool lag2 = false;
    auto glds = [&](__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t lds) {
      uint32_t keep;
      if (lag2)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds ; dma-lag 2\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(off), "s"(r), "s"(lds) : "memory");
      else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(off), "s"(r), "s"(lds) : "memory");
    };
    auto issue = [&](bool live, int b) {  // the tile at (ntx, nty, nn) into buffer b (zeros if !live), then advance
      const int tx = ntx, ty = nty, nimg = nn;
      ntx += s_x;
      int c = ntx >= a.tiles_x;
      ntx -= c ? a.tiles_x : 0;
      nty += s_y + c;
      c = nty >= a.tiles_y;
      nty -= c ? a.tiles_y : 0;
      nn += s_n + c;
      const int oy0 = ty * TH, ox0 = tx * TW;
      const uint32_t zb = lds0 + (uint32_t)((quad * NB + b) * BUF);
      const uint32_t zt = (uint32_t)(((nimg * a.out_h + oy0) * a.out_w + ox0) * a.dz_cs * 2) + z_lane;
      const bool zok = live & (ox0 + zcol < a.out_w);
#pragma unroll
      for (int j = 0; j < NZI; ++j) {
        const bool ok = zok & (oy0 + zrow0 + 2 * j < a.out_h);
        glds(zrs, ok ? zt + (uint32_t)(2 * j) * zrow_b : BUF_OOB, zb + (uint32_t)((wvu + 4 * j) * 1024));
      }
      const uint32_t iy0 = (uint32_t)(S * oy0 - a.pad), ix0 = (uint32_t)(S * ox0 - a.pad), xt = (uint32_t)nimg * ximg_b + x_ch;
#pragma unroll
      for (int j = 0; j < NXI; ++j) {
        const uint32_t iy = iy0 + (uint32_t)(xrc[j] >> 16), ix = ix0 + (uint32_t)((xrc[j] >> 8) & 255);
        const bool ok = live & (iy < (uint32_t)lh) & (ix < (uint32_t)lw);
        const uint32_t off = xt + ((iy >> upsh) * (uint32_t)a.in_w + (ix >> upsh)) * pxb + (uint32_t)((xrc[j] & 7) * 16);
        glds(xrs, ok ? off : BUF_OOB, zb + (uint32_t)(ZB + (wvu + 4 * j) * 1024));
      }
    };
    // fragment reads: k-step kk, lane (g, q, p) = output pixel c0 = 4 g + q of rows 2 kk (k0) and 2 kk + 1 (k1),
    // channels 4 p.. of the 16-channel group: dz group t (chunk 2 t + (p >> 1)), x group wave (chunk 2 wave + (p >> 1));
    // tap column dx reads footprint column S c0 + dx (its slot)
    const int c0 = 4 * g + q;
    int zoff[4], xoff[3];
#pragma unroll
    for (int t = 0; t < 4; ++t) zoff[t] = c0 * 128 + (((2 * t + (p >> 1)) ^ (c0 & 7)) << 4) + 8 * (p & 1);
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int sl = S == 1 ? c0 + dx : (dx == 1 ? (TPW + 1) / 2 + c0 : c0 + dx / 2);
      xoff[dx] = sl * 128 + (((2 * wave + (p >> 1)) ^ (sl & 7)) << 4) + 8 * (p & 1);
    }
    auto ld_af = [&](const char* zb, int kk, bf16x8 (&af)[4]) {
#pragma unroll
      for (int t = 0; t < 4; ++t) af[t] = cat_tr(ds_read_tr16(zb + kk * 32 * 128 + zoff[t]), ds_read_tr16(zb + (kk * 32 + 16) * 128 + zoff[t]));
    };
    auto ld_bf = [&](const char* xb, int kk, int u) {
      const int dy = u / 3, dx = u % 3;
      return cat_tr(ds_read_tr16(xb + (S * 2 * kk + dy) * TPW * 128 + xoff[dx]), ds_read_tr16(xb + (S * (2 * kk + 1) + dy) * TPW * 128 + xoff[dx]));
    };
    // both quads run the same number of iterations (quad 0's tile count; quad 1's extra one, if any, is all zeros),
    // so their barriers pair up
    const int nit = split < a.ntiles ? (a.ntiles - split + qstep - 1) / qstep : 0;
    int tq = qt0;  // this quad's tile
    issue(tq < a.ntiles, 0);
    int cur = 0;
    // only wave 0 of each quad of a bias-owning workgroup needs the bias sums (quad 1's are added to quad 0's below): the
    // other waves skip those 4 MFMAs per k-step (-1 to -3 us per launch)
    const bool bias_wave = do_bias && __builtin_amdgcn_readfirstlane(wave) == 0;
    if constexpr (NB == 3) {
      lag2 = true;
      issue(tq + qstep < a.ntiles, 1);
    }
    // the tile loop, instantiated twice: with the bias sums (wave 0 of a bias-owning workgroup) and without (a
    // wave-uniform branch around the bias MFMAs inside it spilled registers to scratch)
    auto tiles = [&](auto with_bias) {
    constexpr bool WB = decltype(with_bias)::value;
    for (int it = 0; it < nit; ++it, tq += qstep) {
      // NB 3: this tile's NZI + NXI DMAs (per wave) have landed once at most the next tile's are outstanding; NB 2:
      // once none is.  The barrier makes that true for every wave, and every wave is past its reads of the buffer the
      // request below overwrites (the tile before last, NB 3, or the last one, NB 2)
      if constexpr (NB == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NZI + NXI) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if constexpr (NB == 3) issue(tq + 2 * qstep < a.ntiles, cur == 0 ? 2 : cur - 1);
      else issue(tq + qstep < a.ntiles, cur ^ 1);
      const char* zb = smem + (quad * NB + cur) * BUF;
      const char* xb = zb + ZB;
      // the 36 (k-step, tap) groups of 4 MFMAs read their x fragment from a 3-register ring loaded 2 groups ahead,
      // the next k-step's dz fragments half-way through the current one (one whole fragment set: 56 registers)
      constexpr int LA = 2;  // x-fragment lookahead in (k-step, tap) groups (ring of LA + 1; 3 measured neutral)
      bf16x8 af[2][4], bq[LA + 1];
      ld_af(zb, 0, af[0]);
#pragma unroll
      for (int j = 0; j < LA; ++j) bq[j] = ld_bf(xb, 0, j);
#pragma unroll
      for (int gi = 0; gi < NK * 9; ++gi) {
        const int kk = gi / 9, u = gi % 9, gn = gi + LA;
        if (gn < NK * 9) bq[gn % (LA + 1)] = ld_bf(xb, gn / 9, gn % 9);
        if (u == 4 && kk + 1 < NK) ld_af(zb, kk + 1, af[(kk + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        if (WB && u == 0) {
#pragma unroll
          for (int t = 0; t < 4; ++t) accb[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk & 1][t], ones, accb[t], 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk & 1][t], bq[gi % (LA + 1)], acc[t][u], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      cur = cur == NB - 1 ? 0 : cur + 1;
    }
    };
    if (bias_wave) tiles(std::true_type{});
    else tiles(std::false_type{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMAs past the last tile (zeros) land before the
                                                        // epilogue staging reuses the buffers
  } else {
  issue(tile < a.ntiles);
  if constexpr (TS == 1) {
    // double-buffered LDS, one barrier per tile: tile t+1 (in registers since tile t-1) is written to the other
    // buffer after the first k-step pair of tile t is on the MFMA pipe, then tile t+2 is requested -- the stash
    // no longer runs between two barriers with the MFMAs idle (one workgroup per CU: nothing else hid it).  The
    // stash and the request are unconditional (past the last tile they move zeros into the idle buffer): no branch
    // inside the tile loop, so the accumulators stay in place (the conditional form made hipcc copy all 144 of
    // them out of and back into the AGPRs every tile).  LDS-only barriers keep the register prefetch in flight.
    stash(0);
    issue(tile + a.nsplit < a.ntiles);
    lds_barrier();
    int cur = 0;
    for (; tile < a.ntiles; tile += a.nsplit) {
      bf16x8 afA[4], bfA[NU], afB[4], bfB[NU];
      frags(cur, 0, afA, bfA);
#pragma unroll
      for (int kk = 0; kk < NK; kk += 2) {
        frags(cur, kk + 1, afB, bfB);
        mma(afA, bfA);
        if (kk == 0) {
          stash(cur ^ 1);
          issue(tile + 2 * a.nsplit < a.ntiles);
        }
        if (kk + 2 < NK) frags(cur, kk + 2, afA, bfA);
        mma(afB, bfB);
      }
      lds_barrier();  // this tile's reads of buffer cur and the stash of buffer cur ^ 1 are done
      cur ^= 1;
    }
  } else {
    for (; tile < a.ntiles; tile += a.nsplit) {
      lds_barrier();  // previous tile's fragment reads done
      stash(0);
      issue(tile + a.nsplit < a.ntiles);
      lds_barrier();
      // two waves per SIMD (256 VGPRs each): one fragment set, the partner wave hides the latency
#pragma unroll 2
      for (int kk = 0; kk < NK; ++kk) {
        bf16x8 af[4], bf[NU];
        frags(0, kk, af, bf);
        mma(af, bf);
      }
    }
  }
  }
  // C[row = co][col = ci]: lane holds co = co0 + 16t + 4g + i, ci = ci0 + 16 wave + col.  The workgroup's slab block
  // (64 co rows x 576 contiguous floats each) is assembled in LDS and written with coalesced 16 B stores (the direct
  // form issued 144 scattered 4 B stores per lane, 36 B apart)
  constexpr int EPW = 9 * 64 + 4;  // staged row pitch (floats)
  float* st = (float*)smem;
  __syncthreads();  // every wave's fragment reads are done (the staging aliases the tiles)
  if constexpr (QG == 2) {  // quad 1's sums (and bias sums) through the staging area into quad 0's accumulators
    float* stb = st + 64 * EPW;
    if (quad == 1) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float* row = st + (t * 16 + g * 4 + i) * EPW + (wave * 16 + col) * 9;
#pragma unroll
          for (int u = 0; u < 9; ++u) row[u] = acc[t][u][i];
          if (wave == 0 && col == 0) stb[t * 16 + g * 4 + i] = accb[t][i];
        }
    }
    __syncthreads();
    if (quad == 0) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float* row = st + (t * 16 + g * 4 + i) * EPW + (wave * 16 + col) * 9;
#pragma unroll
          for (int u = 0; u < 9; ++u) acc[t][u][i] += row[u];
          accb[t][i] += stb[t * 16 + g * 4 + i];
        }
    }
    __syncthreads();
  }
  if (quad == 0) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float* row = st + (t * 16 + g * 4 + i) * EPW + (wave * 16 + col) * 9;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          if constexpr (TS == 1) row[u] = acc[t][u][i];
          else if (u0 + u < 9) row[u0 + u] = acc[t][u][i];
        }
        if (do_bias && wave == 0 && tg == 0 && col == 0) a.bpart[(long)split * a.co_rows + co0 + t * 16 + g * 4 + i] = accb[t][i];
      }
  }
  __syncthreads();
  float* slab = a.part + (long)split * a.co_rows * a.kw + (long)co0 * a.kw + ci0 * 9;
  for (int f = tid; f < 64 * 144; f += NTHR) {
    const int row = f / 144, c4 = f - row * 144;
    *(float4*)(slab + (long)row * a.kw + c4 * 4) = *(const float4*)(st + row * EPW + c4 * 4);
  }
}
constexpr size_t W64_EP_LDS = (size_t)64 * (9 * 64 + 4) * 4;  // the slab staging of conv_wgrad64_kernel
constexpr size_t W64G_LDS = (size_t)4 * (8 * 16 * 128 + 24 * 1024);     // two quads x two LDS-DMA tile buffers (G form)
constexpr size_t W64G2_LDS = (size_t)3 * (4 * 16 * 128 + 40 * 1024);    // (G form, stride 2)

template <int TS, int S = 1>
__global__ __launch_bounds__(256 * TS, 1) void conv_wgrad64_kernel(WgArgs a) {
  wgrad64_body<TS, S, false>(a);
}
// at most 256 registers (two waves per SIMD): the accumulators stay in VGPRs -- the 512-register form kept some of them
// in AGPRs and shuffled them every tile
__global__ __launch_bounds__(512, 1) void conv_wgrad64_glds_kernel(WgArgs a) { wgrad64_body<1, 1, true>(a); }
__global__ __launch_bounds__(256, 2) void conv_wgrad64_glds_s2_kernel(WgArgs a) { wgrad64_body<1, 2, true>(a); }

// ------------------------------------------------------------------------------------------
// Weight gradient of a 1x1 conv with 64 inputs and <= 64 outputs (srcnn.conv2): dW[co][ci] = sum_p dz[p][co]
// x[p][ci], db = sum_p dz.  One pass over the pixels: each workgroup owns a contiguous pixel range and ALL
// co x ci outputs (wave w = ci block w), 128-pixel chunks staged through LDS (next chunk prefetched into
// registers) and read back transposed (ds_read_tr16_b64) as pixel-major MFMA fragments.  The generic wgrad
// splits co x ci over workgroups that each re-read every pixel (1.6 GB fetched for 0.4 GB of data).
// ------------------------------------------------------------------------------------------
constexpr int WPT_CH = 128;

static bool wpt_shape(const ClimsrConvDesc* d) {
  return d->ks == 1 && d->stride == 1 && d->up == 1 && d->pad == 0 && d->in_c == 64 && d->out_c % 16 == 0 && d->out_c <= 64 &&
         d->out_h == d->in_h && d->out_w == d->in_w;
}

static int wpt_splits(const ClimsrConvDesc* d) {
  const long npix = (long)d->n * d->out_h * d->out_w;
  long ns = npix / (WPT_CH * 8);  // >= 8 chunks per workgroup
  if (ns > 512) ns = 512;
  return ns < 1 ? 1 : (int)ns;
}

template <int NCOF>
__global__ __launch_bounds__(256) void conv_wgrad_pt_kernel(WgArgs a) {
  constexpr int ZP = NCOF * 16 + 8, XP = 64 + 8;
  constexpr int NZV = WPT_CH * NCOF * 2 / 256, NXV = WPT_CH * 8 / 256;  // 16 B vectors per thread
  __shared__ __attribute__((aligned(16))) uint16_t zs[WPT_CH * ZP];
  __shared__ __attribute__((aligned(16))) uint16_t xs[WPT_CH * XP];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4;
  const int q = (lane & 15) >> 2, p = lane & 3, col = lane & 15;
  const long npix = (long)a.n * a.out_h * a.out_w;
  const long p0 = npix * blockIdx.x / gridDim.x, p1 = npix * (blockIdx.x + 1) / gridDim.x;
  const bool do_bias = a.bpart != nullptr && wave == 0;
  f32x4 acc[NCOF], accb[NCOF];
#pragma unroll
  for (int t = 0; t < NCOF; ++t) acc[t] = accb[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int i = 0; i < 8; ++i) ones[i] = (__bf16)1.0f;
  uint4 pz[NZV], px[NXV];
  auto issue = [&](long c0) {
#pragma unroll
    for (int i = 0; i < NZV; ++i) {
      const int v = tid + 256 * i, pix = v / (NCOF * 2), cg = v % (NCOF * 2);
      const long pp = c0 + pix;
      pz[i] = pp < p1 ? *(const uint4*)(a.dz + pp * a.dz_cs + cg * 8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NXV; ++i) {
      const int v = tid + 256 * i, pix = v >> 3, cg = v & 7;
      const long pp = c0 + pix;
      px[i] = pp < p1 ? *(const uint4*)(a.x + pp * a.in_cs + a.in_co + cg * 8) : make_uint4(0, 0, 0, 0);
    }
  };
  if (p0 < p1) issue(p0);
  for (long c0 = p0; c0 < p1; c0 += WPT_CH) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NZV; ++i) {
      const int v = tid + 256 * i;
      *(uint4*)(zs + (v / (NCOF * 2)) * ZP + (v % (NCOF * 2)) * 8) = pz[i];
    }
#pragma unroll
    for (int i = 0; i < NXV; ++i) {
      const int v = tid + 256 * i;
      *(uint4*)(xs + (v >> 3) * XP + (v & 7) * 8) = px[i];
    }
    if (c0 + WPT_CH < p1) issue(c0 + WPT_CH);
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < WPT_CH / 32; ++kk) {
      const int k0 = kk * 32 + 8 * g + q, k1 = k0 + 4;
      const s16x4 blo = ds_read_tr16(xs + k0 * XP + wave * 16 + 4 * p), bhi = ds_read_tr16(xs + k1 * XP + wave * 16 + 4 * p);
      const short b8[8] = {blo[0], blo[1], blo[2], blo[3], bhi[0], bhi[1], bhi[2], bhi[3]};
      const bf16x8 b = __builtin_bit_cast(bf16x8, b8);
#pragma unroll
      for (int t = 0; t < NCOF; ++t) {
        const s16x4 lo = ds_read_tr16(zs + k0 * ZP + t * 16 + 4 * p), hi = ds_read_tr16(zs + k1 * ZP + t * 16 + 4 * p);
        const short v8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const bf16x8 af = __builtin_bit_cast(bf16x8, v8);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, b, acc[t], 0, 0, 0);
        if (do_bias) accb[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, ones, accb[t], 0, 0, 0);
      }
    }
  }
  // D[co][ci]: lane holds co = 16t + 4g + i, ci = 16 wave + col
  float* slab = a.part + (long)blockIdx.x * a.co_rows * a.kw;
#pragma unroll
  for (int t = 0; t < NCOF; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = t * 16 + g * 4 + i;
      slab[(long)co * a.kw + wave * 16 + col] = acc[t][i];
      if (do_bias && col == 0) a.bpart[(long)blockIdx.x * a.co_rows + co] = accb[t][i];
    }
}

// ------------------------------------------------------------------------------------------
// Weight gradient of a single-output-channel conv (conv_last 64->1 3x3, srcnn.conv3 32->1 5x5).  The
// generic wgrad puts the one output channel in the MFMA M dimension (1 of 16 rows useful); here the
// horizontal taps take that role instead.  Per dz row y and input row iy = y + ky - R:
//     D_ky[kx][ci] += sum_x' dz[y][x' - kx] * X[iy][x'][ci]           (M = kx, N = ci, K = x')
// A = the dz row shifted by kx (a Toeplitz fragment: 8 consecutive dz values per lane, read 16 B-aligned
// from one of 8 pre-shifted LDS copies of the row), B = the input row transposed by ds_read_tr16_b64.
// A wave streams a segment of SEG dz rows of one 64-column strip; each staged input row feeds the KS
// dz rows it pairs with.  Block partials (4 waves summed in LDS) go to the wgrad_reduce layout
// part[split][16][in_c * ks^2] (row 0), bpart[split][16].
// ------------------------------------------------------------------------------------------
constexpr int WCO1_XT = 96, WCO1_DZL = 128;

static bool wco1_shape(const ClimsrConvDesc* d) {
  return d->out_c == 1 && d->stride == 1 && d->up == 1 && (d->ks == 3 || d->ks == 5) && d->pad == d->ks / 2 &&
         d->in_c % 16 == 0 && d->in_c <= 64 && d->out_h == d->in_h && d->out_w == d->in_w;
}

static int wco1_splits(const ClimsrConvDesc* d) {
  const long rows = (long)d->n * d->out_h * ceil_div(d->out_w, 64);
  long ns = rows / (4 * 8);  // >= 8 dz rows per wave
  if (ns > 512) ns = 512;
  return ns < 1 ? 1 : (int)ns;
}

template <int KS, int NCF>
__global__ __launch_bounds__(256, 2) void conv_wgrad_co1m_kernel(WgArgs a) {
  constexpr int R = KS / 2, CI = NCF * 16, XP = CI + 8, NV = ((64 + KS - 1) * (CI / 8) + 63) / 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, col = lane & 15;
  uint16_t* xs = (uint16_t*)smem + wave * (WCO1_XT * XP);                                   // [x'][ci]
  uint16_t* ring = (uint16_t*)smem + 4 * WCO1_XT * XP + wave * (KS * 8 * WCO1_DZL);         // [slot][copy][m]
  for (int i = lane; i < WCO1_XT * XP / 8; i += 64) ((uint4*)xs)[i] = make_uint4(0, 0, 0, 0);
  for (int i = lane; i < KS * 8 * WCO1_DZL / 8; i += 64) ((uint4*)ring)[i] = make_uint4(0, 0, 0, 0);

  f32x4 acc[KS][NCF];
#pragma unroll
  for (int k = 0; k < KS; ++k)
#pragma unroll
    for (int c = 0; c < NCF; ++c) acc[k][c] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;

  const int nstrip = (a.out_w + 63) / 64;
  const int seg_rows = a.tph;  // dz rows per segment (host-chosen)
  const int nrs = (a.out_h + seg_rows - 1) / seg_rows;
  const long nseg = (long)a.n * nstrip * nrs;
  const int gw = blockIdx.x * 4 + wave, nw = gridDim.x * 4;
  for (long seg = gw; seg < nseg; seg += nw) {
    const int rs = (int)(seg % nrs);
    const int strip = (int)((seg / nrs) % nstrip);
    const int nimg = (int)(seg / ((long)nrs * nstrip));
    const int x0 = strip * 64, ya = rs * seg_rows, yb = min(a.out_h, ya + seg_rows);
    for (int iy = ya - R; iy < yb + R; ++iy) {
      // stage input row iy: x' in [0, 64 + KS - 1) <-> input column x0 - R + x'
      uint4 v[NV];
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int e = lane + 64 * i, xq = e / (CI / 8), cg = e % (CI / 8);
        const int ix = x0 - R + xq;
        v[i] = make_uint4(0, 0, 0, 0);
        if (xq < 64 + KS - 1 && iy >= 0 && iy < a.in_h && ix >= 0 && ix < a.in_w && cg * 8 < a.in_c)
          v[i] = *(const uint4*)(a.x + (((long)nimg * a.in_h + iy) * a.in_w + ix) * a.in_cs + a.in_co + cg * 8);
      }
      // the dz row paired with tap row 0 enters the ring: 8 copies, copy q holds D[m - 16 - q]
      const int ynew = iy + R;
      float dzv = 0.f;
      if (ynew >= ya && ynew < yb && x0 + lane < a.out_w)
        dzv = bf2f(a.dz[(((long)nimg * a.out_h + ynew) * a.out_w + x0 + lane) * a.dz_cs]);
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int e = lane + 64 * i, xq = e / (CI / 8), cg = e % (CI / 8);
        if (xq < 64 + KS - 1) *(uint4*)(xs + xq * XP + cg * 8) = v[i];
      }
      if (ynew >= ya && ynew < yb) {
        bsum += dzv;
        uint16_t* slot = ring + (ynew % KS) * (8 * WCO1_DZL);
        const uint16_t b = f2bf(dzv);
#pragma unroll
        for (int q = 0; q < 8; ++q) slot[q * WCO1_DZL + lane + 16 + q] = b;
      }
      // B fragments of this input row (x' = 32 s + 8 g + j, ci = 16 c + col), shared by every tap row
      bf16x8 bx[3][NCF];
#pragma unroll
      for (int st = 0; st < 3; ++st)
#pragma unroll
        for (int c = 0; c < NCF; ++c) {
          const uint16_t* p0 = xs + (st * 32 + g * 8 + (col >> 2)) * XP + c * 16 + (col & 3) * 4;
          const s16x4 lo = ds_read_tr16(p0), hi = ds_read_tr16(p0 + 4 * XP);
          bx[st][c] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
      for (int ky = 0; ky < KS; ++ky) {
        const int y = iy - ky + R;
        if (y < ya || y >= yb) continue;
        const uint16_t* slot = ring + (y % KS) * (8 * WCO1_DZL);
#pragma unroll
        for (int st = 0; st < 3; ++st) {
          const int aoff = st * 32 + g * 8 - col;  // D index of element j = 0 (lane's kx = col)
          const int q = (-aoff) & 7;
          bf16x8 at = *(const bf16x8*)(slot + q * WCO1_DZL + aoff + 16 + q);
          if (col >= KS) at = (bf16x8){};
#pragma unroll
          for (int c = 0; c < NCF; ++c) acc[ky][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at, bx[st][c], acc[ky][c], 0, 0, 0);
        }
      }
    }
    // the next segment rewrites every ring position it reads (rows outside [ya, yb) are skipped)
  }
  // block reduction: C[kx = 4g + i][ci = 16c + col] of tap row ky
  for (int o = 32; o > 0; o >>= 1) bsum += __shfl_down(bsum, o);
  __syncthreads();
  float* red = (float*)smem;  // [wave][ky][c][lane][4]
#pragma unroll
  for (int ky = 0; ky < KS; ++ky)
#pragma unroll
    for (int c = 0; c < NCF; ++c) *(f32x4*)(red + (((wave * KS + ky) * NCF + c) * 64 + lane) * 4) = acc[ky][c];
  __shared__ float bred[4];
  if (lane == 0) bred[wave] = bsum;
  __syncthreads();
  const int ks2 = KS * KS;
  float* part = a.part + (long)blockIdx.x * 16 * a.kw;
  constexpr int PER = KS * NCF * 64 * 4;
  for (int e = tid; e < PER; e += 256) {
    const int i = e & 3, ln = (e >> 2) & 63, c = (e >> 8) % NCF, ky = (e >> 8) / NCF;
    const int kx = (ln >> 4) * 4 + i, ci = c * 16 + (ln & 15);
    if (kx >= KS || ci >= a.in_c) continue;
    const float t = red[e] + red[e + PER] + red[e + 2 * PER] + red[e + 3 * PER];
    part[ci * ks2 + ky * KS + kx] = t;
  }
  if (tid == 0 && a.bpart) a.bpart[blockIdx.x * 16] = bred[0] + bred[1] + bred[2] + bred[3];
}

template <int KS, int NCF>
static int launch_wco1(const WgArgs& a, hipStream_t s) {
  if (dry_run("conv_wgrad_co1m_kernel<%d, %d>", KS, NCF)) return CLIMSR_OK;
  auto k = conv_wgrad_co1m_kernel<KS, NCF>;  // (+16 B of static LDS: the dynamic cap leaves room for it)
  const size_t lds_x = (size_t)4 * WCO1_XT * (NCF * 16 + 8) * 2 + (size_t)4 * KS * 8 * WCO1_DZL * 2;
  const size_t lds_r = (size_t)4 * KS * NCF * 64 * 16;
  const size_t lds = lds_x > lds_r ? lds_x : lds_r;
  if (int e = lds_opt_in((const void*)k, 159 * 1024)) return e;
  hipLaunchKernelGGL(k, dim3(a.nsplit), dim3(256), lds, s, a);
  return check_launch("conv2d_wgrad (co1m)");
}

static bool w64_shape(const ClimsrConvDesc* d) {
  return d->ks == 3 && d->pad == 1 && d->out_c % 64 == 0 && d->in_c % 64 == 0 && d->in_c >= 64 &&
         (d->stride == 1 || (d->stride == 2 && d->up == 1));
}
static int w64_th(const ClimsrConvDesc* d) { return d->stride == 2 ? W64<2>::TH : W64<1>::TH; }

struct WgPlan {
  int ntc, tb, ntapb, ncib, ncob, co_rows, tiles_x, tiles_y, ntiles, tph, tpw, dzp, kw, ci4;
  size_t lds_x, lds_z, lds_total;
};

static void wg_plan(const ClimsrConvDesc* d, WgPlan* w) {
  int rows = round_up(d->out_c, 16);
  w->ntc = rows >= 64 ? 4 : (rows >= 32 ? 2 : 1);
  int ks2 = d->ks * d->ks;
  w->ci4 = d->in_c == 4;  // <= 4 real input channels: 4 taps x 4 channels per fragment
  if (w->ci4) {
    int groups = ceil_div(ks2, 4);
    w->tb = groups <= 3 ? 3 : 7;
    w->ntapb = ceil_div(groups, w->tb);
    w->ncib = 1;
  } else {
    w->tb = ks2 >= 9 ? 9 : (ks2 >= 5 ? 5 : 1);
    if (ks2 == 25) w->tb = 5;
    w->ntapb = ceil_div(ks2, w->tb);
    w->ncib = ceil_div(d->in_c, 16);
  }
  w->ncob = ceil_div(rows, w->ntc * 16);
  w->co_rows = w->ncob * w->ntc * 16;
  w->tiles_x = ceil_div(d->out_w, TW);
  w->tiles_y = ceil_div(d->out_h, WG_TH);
  w->ntiles = d->n * w->tiles_x * w->tiles_y;
  w->tph = (WG_TH - 1) * d->stride + d->ks;
  w->tpw = (TW - 1) * d->stride + d->ks;
  w->dzp = w->ntc * 16 + 8;
  w->kw = d->in_c * ks2;
  w->lds_x = (size_t)w->tph * w->tpw * (w->ci4 ? 4 : WG_XP) * 2;
  w->lds_x = (w->lds_x + 15) / 16 * 16;
  w->lds_z = (size_t)WG_TH * TW * w->dzp * 2;
  size_t red = (size_t)(w->ntc * w->tb + w->ntc) * 64 * 16;
  w->lds_total = w->lds_x + w->lds_z;
  if (red > w->lds_total) w->lds_total = red;
}

static bool wg_ws(const ClimsrConvDesc* d, const WgPlan& w) {
  return w.ci4 && d->ks == 9 && w.ncob == 1 && w.ntc == 4 && d->stride == 1;
}

extern "C" int climsr_conv2d_wgrad_splits(const ClimsrConvDesc* d) {
  if (wpt_shape(d)) return wpt_splits(d);
  if (wco1_shape(d)) return wco1_splits(d);
  if (w64_shape(d)) {  // one workgroup per CU: 256 / blocks splits
    int blocks = (d->out_c / 64) * (d->in_c / 64);
    int ntiles = d->n * ceil_div(d->out_w, TW) * ceil_div(d->out_h, w64_th(d));
    int ns = ceil_div(256, blocks);
    if (ns > ntiles) ns = ntiles;
    return ns < 1 ? 1 : ns;
  }
  WgPlan w;
  wg_plan(d, &w);
  int base = wg_ws(d, w) ? 1 : w.ntapb * w.ncib * w.ncob;
  int ns = ceil_div(512, base);
  if (ns > w.ntiles) ns = w.ntiles;
  if (ns < 1) ns = 1;
  return ns;
}

extern "C" size_t climsr_conv2d_wgrad_workspace(const ClimsrConvDesc* d, int nsplit) {
  if (wpt_shape(d)) {  // the reduce's layout: co_rows = out_c rounded to its 16/32/64 tile, kw = in_c
    const int rows = round_up(d->out_c, 16), ntc = rows >= 64 ? 4 : (rows >= 32 ? 2 : 1);
    const int co_rows = ceil_div(rows, ntc * 16) * ntc * 16;
    return (size_t)nsplit * co_rows * d->in_c + (size_t)nsplit * co_rows;
  }
  if (wco1_shape(d)) return (size_t)nsplit * 16 * d->in_c * d->ks * d->ks + (size_t)nsplit * 16;
  if (w64_shape(d)) return (size_t)nsplit * d->out_c * d->in_c * 9 + (size_t)nsplit * d->out_c;
  WgPlan w;
  wg_plan(d, &w);
  return (size_t)nsplit * w.co_rows * w.kw + (size_t)nsplit * w.co_rows;
}

template <int NTC, int TB, int CI4>
static int launch_wg(const WgArgs& a, int nblk, size_t lds, hipStream_t s) {
  if (dry_run("conv_wgrad_kernel<%d, %d, %d, false>", NTC, TB, CI4)) return CLIMSR_OK;
  auto k = conv_wgrad_kernel<NTC, TB, CI4>;
  if (int e = lds_opt_in((const void*)k, 160 * 1024)) return e;
  hipLaunchKernelGGL(k, dim3(nblk, a.nsplit), dim3(256), lds, s, a);
  return check_launch("conv2d_wgrad");
}

extern "C" int climsr_conv2d_wgrad(const ClimsrConvDesc* d, const uint16_t* x, const uint16_t* dz, int dz_cstride, float* partial,
                                   float* bias_partial, int nsplit, void* stream) {
  if (!d || !x || !dz || !partial || nsplit <= 0 || (d->in_c % 8 && d->in_c != 4) || d->in_cstride % 8 || d->in_coff % 8 ||
      dz_cstride % 8 ||
      (d->up != 1 && d->up != 2) || (d->stride != 1 && d->stride != 2)) {
    set_error("conv2d_wgrad: bad args");
    return CLIMSR_EINVAL;
  }
  if (wpt_shape(d)) {
    WgArgs a{};
    a.x = x; a.dz = dz; a.part = partial; a.bpart = bias_partial;
    a.n = d->n; a.in_c = d->in_c; a.in_cs = d->in_cstride; a.in_co = d->in_coff; a.out_h = d->out_h; a.out_w = d->out_w;
    a.out_c = d->out_c; a.dz_cs = dz_cstride; a.nsplit = nsplit; a.kw = d->in_c;
    const int rows = round_up(d->out_c, 16), ntc = rows >= 64 ? 4 : (rows >= 32 ? 2 : 1);
    a.co_rows = ceil_div(rows, ntc * 16) * ntc * 16;
    hipStream_t s = (hipStream_t)stream;
    if (dry_run("conv_wgrad_pt_kernel<%d>", d->out_c / 16 < 4 ? d->out_c / 16 : 4)) return CLIMSR_OK;
    switch (d->out_c / 16) {
      case 1: hipLaunchKernelGGL(conv_wgrad_pt_kernel<1>, dim3(nsplit), dim3(256), 0, s, a); break;
      case 2: hipLaunchKernelGGL(conv_wgrad_pt_kernel<2>, dim3(nsplit), dim3(256), 0, s, a); break;
      case 3: hipLaunchKernelGGL(conv_wgrad_pt_kernel<3>, dim3(nsplit), dim3(256), 0, s, a); break;
      default: hipLaunchKernelGGL(conv_wgrad_pt_kernel<4>, dim3(nsplit), dim3(256), 0, s, a); break;
    }
    return check_launch("conv2d_wgrad (1x1)");
  }
  if (wco1_shape(d)) {
    WgArgs a{};
    a.x = x; a.dz = dz; a.part = partial; a.bpart = bias_partial;
    a.n = d->n; a.in_h = d->in_h; a.in_w = d->in_w; a.in_c = d->in_c; a.in_cs = d->in_cstride; a.in_co = d->in_coff;
    a.out_h = d->out_h; a.out_w = d->out_w; a.out_c = 1; a.dz_cs = dz_cstride; a.ks = d->ks; a.pad = d->pad;
    a.nsplit = nsplit; a.kw = d->in_c * d->ks * d->ks; a.co_rows = 16;
    const long rows = (long)d->n * d->out_h * ceil_div(d->out_w, 64);
    a.tph = ceil_div(rows, (long)nsplit * 4);  // dz rows per wave segment (~one segment per wave)
    if (a.tph < 4) a.tph = 4;
    if (a.tph > d->out_h) a.tph = d->out_h;
    hipStream_t s = (hipStream_t)stream;
    switch (d->ks * 10 + d->in_c / 16) {
      case 31: return launch_wco1<3, 1>(a, s);
      case 32: return launch_wco1<3, 2>(a, s);
      case 33: return launch_wco1<3, 3>(a, s);
      case 34: return launch_wco1<3, 4>(a, s);
      case 51: return launch_wco1<5, 1>(a, s);
      case 52: return launch_wco1<5, 2>(a, s);
      case 53: return launch_wco1<5, 3>(a, s);
      default: return launch_wco1<5, 4>(a, s);
    }
  }
  if (w64_shape(d)) {
    if ((long)d->n * d->in_h * d->in_w * d->in_cstride * 2 >= (1L << 31) ||
        (long)d->n * d->out_h * d->out_w * dz_cstride * 2 >= (1L << 31)) {  // 32-bit buffer offsets (BUF_OOB)
      set_error("conv2d_wgrad: operands over 2 GiB (split the batch)");
      return CLIMSR_EINVAL;
    }
    WgArgs a{};
    a.x = x; a.dz = dz; a.part = partial; a.bpart = bias_partial;
    a.n = d->n; a.in_h = d->in_h; a.in_w = d->in_w; a.in_c = d->in_c; a.in_cs = d->in_cstride; a.in_co = d->in_coff;
    a.up = d->up; a.ks = 3; a.stride = 1; a.pad = 1; a.out_h = d->out_h; a.out_w = d->out_w;
    a.out_c = d->out_c; a.dz_cs = dz_cstride;
    a.tiles_x = ceil_div(d->out_w, TW); a.tiles_y = ceil_div(d->out_h, w64_th(d)); a.ntiles = d->n * a.tiles_x * a.tiles_y;
    a.nsplit = nsplit; a.ncib = d->in_c / 64; a.co_rows = d->out_c; a.kw = d->in_c * 9;
    a.dzp = W64_P; a.ntapb = 1; a.lds_x = 0;
    a.stride = d->stride;
    // 8 waves (tap-split) pay off on the large-pixel-count convs (HRconv / upconv at 256^2: +8 %) and lose on the
    // 64^2 dense-block GEMM (-19 %), measured with tools/perf_conv.py
    const bool ts2 = d->stride == 1 && (long)d->n * d->out_h * d->out_w >= (1L << 20);
    a.xcd = 1;
    const dim3 grid = dim3((d->out_c / 64) * (d->in_c / 64) * nsplit);
    if (d->stride == 2) {
      a.tph = W64<2>::TPH; a.tpw = W64<2>::TPW;
      if (dry_run("conv_wgrad64_glds_s2_kernel")) return CLIMSR_OK;
      if (int e = lds_opt_in((const void*)conv_wgrad64_glds_s2_kernel, 160 * 1024)) return e;
      hipLaunchKernelGGL(conv_wgrad64_glds_s2_kernel, grid, dim3(256), std::max(W64G2_LDS, W64_EP_LDS), (hipStream_t)stream, a);
    } else if (d->stride == 2) {
      a.tph = W64<2>::TPH; a.tpw = W64<2>::TPW;
      if (dry_run("conv_wgrad64_kernel<1, 2>")) return CLIMSR_OK;
      if (int e = lds_opt_in((const void*)conv_wgrad64_kernel<1, 2>, 160 * 1024)) return e;
      hipLaunchKernelGGL((conv_wgrad64_kernel<1, 2>), grid, dim3(256), std::max(2 * W64<2>::LDS, W64_EP_LDS), (hipStream_t)stream, a);
    } else if (ts2) {
      a.tph = W64<1>::TPH; a.tpw = W64<1>::TPW;
      if (dry_run("conv_wgrad64_kernel<2, 1>")) return CLIMSR_OK;
      if (int e = lds_opt_in((const void*)conv_wgrad64_kernel<2, 1>, 160 * 1024)) return e;
      hipLaunchKernelGGL((conv_wgrad64_kernel<2, 1>), grid, dim3(512), std::max(W64<1>::LDS, W64_EP_LDS), (hipStream_t)stream, a);
    } else {
      a.tph = W64<1>::TPH; a.tpw = W64<1>::TPW;
      if (dry_run("conv_wgrad64_glds_kernel")) return CLIMSR_OK;
      if (int e = lds_opt_in((const void*)conv_wgrad64_glds_kernel, 160 * 1024)) return e;
      static_assert(W64G_LDS <= 160 * 1024 && W64_EP_LDS + 64 * 4 <= W64G_LDS, "LDS of the two-quad wgrad64");
      hipLaunchKernelGGL(conv_wgrad64_glds_kernel, grid, dim3(512), W64G_LDS, (hipStream_t)stream, a);
    }
    return check_launch("conv2d_wgrad (64x64 block)");
  }
  WgPlan w;
  wg_plan(d, &w);
  if (w.lds_total > 160 * 1024) {
    set_error("conv2d_wgrad: LDS %zu too large", w.lds_total);
    return CLIMSR_EINVAL;
  }
  WgArgs a{};
  a.x = x; a.dz = dz; a.part = partial; a.bpart = bias_partial;
  a.n = d->n; a.in_h = d->in_h; a.in_w = d->in_w; a.in_c = d->in_c; a.in_cs = d->in_cstride; a.in_co = d->in_coff;
  a.up = d->up; a.ks = d->ks; a.stride = d->stride; a.pad = d->pad; a.out_h = d->out_h; a.out_w = d->out_w;
  a.out_c = d->out_c; a.dz_cs = dz_cstride;
  a.tph = w.tph; a.tpw = w.tpw; a.dzp = w.dzp; a.tiles_x = w.tiles_x; a.tiles_y = w.tiles_y; a.ntiles = w.ntiles;
  a.nsplit = nsplit; a.ntapb = w.ntapb; a.ncib = w.ncib; a.co_rows = w.co_rows; a.kw = w.kw;
  a.lds_x = (int)w.lds_x;
  int nblk = w.ntapb * w.ncib * w.ncob;
  hipStream_t s = (hipStream_t)stream;
  if (wg_ws(d, w)) {  // all 21 tap groups per workgroup, 6 per wave
    a.ntapb = 1;
    if (dry_run("conv_wgrad_kernel<4, 6, 1, true>")) return CLIMSR_OK;
    auto k = conv_wgrad_kernel<4, 6, 1, true>;
    if (int e = lds_opt_in((const void*)k, 160 * 1024)) return e;
    hipLaunchKernelGGL(k, dim3(1, nsplit), dim3(256), w.lds_total, s, a);
    return check_launch("conv2d_wgrad (ci4, wave-split taps)");
  }
#define WG_CASE(NTC, TB, CI4) \
  if (w.ntc == NTC && w.tb == TB && w.ci4 == CI4) return launch_wg<NTC, TB, CI4>(a, nblk, w.lds_total, s);
  WG_CASE(1, 1, 0) WG_CASE(2, 1, 0) WG_CASE(4, 1, 0)
  WG_CASE(1, 5, 0) WG_CASE(2, 5, 0) WG_CASE(4, 5, 0)
  WG_CASE(1, 9, 0) WG_CASE(2, 9, 0) WG_CASE(4, 9, 0)
  WG_CASE(1, 3, 1) WG_CASE(2, 3, 1) WG_CASE(4, 3, 1)
  WG_CASE(1, 7, 1) WG_CASE(2, 7, 1) WG_CASE(4, 7, 1)
#undef WG_CASE
  set_error("conv2d_wgrad: no kernel for ntc=%d tb=%d", w.ntc, w.tb);
  return CLIMSR_EINVAL;
}

extern "C" const char* climsr_conv2d_wgrad_kernel(const ClimsrConvDesc* d) {
  static uint16_t dummy[8];
  static float fdummy[8];
  g_dry = true;
  g_dry_name[0] = 0;
  const int rc = climsr_conv2d_wgrad(d, dummy, dummy, 8, fdummy, fdummy, climsr_conv2d_wgrad_splits(d), nullptr);
  g_dry = false;
  return rc == CLIMSR_OK ? g_dry_name : "";
}

// 256 threads = 32 consecutive outputs x 8 split groups (8 independent load chains per output,
// coalesced 128 B rows), combined in a fixed order through LDS: deterministic.
// Split group sg's share of the nsplit partials (sg, sg+8, ...): 4 independent chains so the loads are in flight
// together (one chain waited for each load in turn), combined in a fixed order.
__device__ __forceinline__ float sum_splits(const float* src, long sstride, int sg, int nsplit) {
  float a4[4] = {0.f, 0.f, 0.f, 0.f};
  int sp = sg;
  for (; sp + 24 < nsplit; sp += 32) {
#pragma unroll
    for (int u = 0; u < 4; ++u) a4[u] += src[(long)(sp + 8 * u) * sstride];
  }
  for (; sp < nsplit; sp += 8) a4[0] += src[(long)sp * sstride];
  return (a4[0] + a4[1]) + (a4[2] + a4[3]);
}

__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, const float* __restrict__ bpart,
                                                          int nsplit, int out_c, int in_c_real, int in_c, int ks2, int co_rows,
                                                          int kw, float* __restrict__ wg, float* __restrict__ bg, int accumulate) {
  __shared__ float red[8][33];
  const int lane = threadIdx.x & 31;
  const int sg = threadIdx.x >> 5;
  long idx = (long)blockIdx.x * 32 + lane;
  long nw = (long)out_c * in_c_real * ks2;
  long total = nw + (bg ? out_c : 0);
  const float* src = nullptr;
  long sstride = 0;
  if (idx < nw) {
    int co = (int)(idx / ((long)in_c_real * ks2));
    int rem = (int)(idx % ((long)in_c_real * ks2));  // ci*ks2 + tap
    src = part + (long)co * kw + rem;
    sstride = (long)co_rows * kw;
  } else if (idx < total) {
    src = bpart + (idx - nw);
    sstride = co_rows;
  }
  red[sg][lane] = src ? sum_splits(src, sstride, sg, nsplit) : 0.f;
  __syncthreads();
  if (sg == 0 && idx < total) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) t += red[i][lane];
    float* dst = (idx < nw) ? (wg + idx) : (bg + (idx - nw));
    if (accumulate) *dst += t;
    else *dst = t;
  }
}

// Row-sliced reduction of one wgrad partial matrix into several convs' OIHW gradients (the combined
// residual-dense-block weight gradient: rows [row0, row0 + out_c) of the [co_rows][kw] partial are conv
// d->wgrad's output channels, the first in_c_real*ks2 columns of each row its inputs x taps).
__global__ __launch_bounds__(256) void wgrad_reduce_rows_kernel(const float* __restrict__ part, const float* __restrict__ bpart,
                                                               int nsplit, int co_rows, int kw, int ks2,
                                                               const ClimsrReduceDesc* __restrict__ descs, int accumulate) {
  __shared__ float red[8][33];
  const ClimsrReduceDesc d = descs[blockIdx.y];
  const int lane = threadIdx.x & 31;
  const int sg = threadIdx.x >> 5;
  const long idx = (long)blockIdx.x * 32 + lane;
  const long nw = (long)d.out_c * d.in_c_real * ks2;
  const long total = nw + (d.bias_grad ? d.out_c : 0);
  if ((long)blockIdx.x * 32 >= total) return;
  const float* src = nullptr;
  long sstride = 0;
  if (idx < nw) {
    const int co = (int)(idx / ((long)d.in_c_real * ks2));
    const int rem = (int)(idx % ((long)d.in_c_real * ks2));
    src = part + (long)(d.row0 + co) * kw + rem;
    sstride = (long)co_rows * kw;
  } else if (idx < total) {
    src = bpart + d.row0 + (idx - nw);
    sstride = co_rows;
  }
  red[sg][lane] = src ? sum_splits(src, sstride, sg, nsplit) : 0.f;
  __syncthreads();
  if (sg == 0 && idx < total) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) t += red[i][lane];
    float* dst = (idx < nw) ? (d.wgrad + idx) : (d.bias_grad + (idx - nw));
    if (accumulate) *dst += t;
    else *dst = t;
  }
}

extern "C" int climsr_conv2d_wgrad_reduce_rows(const float* partial, const float* bias_partial, int nsplit, int co_rows, int kw,
                                               int ks, const ClimsrReduceDesc* descs, int ndesc, int64_t max_elems,
                                               int accumulate, void* stream) {
  if (!partial || !descs || nsplit <= 0 || ndesc <= 0 || ndesc > 65535 || ks <= 0) {
    set_error("conv2d_wgrad_reduce_rows: bad args");
    return CLIMSR_EINVAL;
  }
  hipLaunchKernelGGL(wgrad_reduce_rows_kernel, dim3(ceil_div(max_elems, 32), ndesc), dim3(256), 0, (hipStream_t)stream, partial,
                     bias_partial, nsplit, co_rows, kw, ks * ks, descs, accumulate);
  return check_launch("conv2d_wgrad_reduce_rows");
}

extern "C" int climsr_conv2d_wgrad_reduce(const float* partial, const float* bias_partial, int nsplit, int out_c, int in_c_real,
                                          int in_c, int ks, float* wgrad, float* bias_grad, int accumulate, void* stream) {
  if (!partial || !wgrad || nsplit <= 0) {
    set_error("conv2d_wgrad_reduce: bad args");
    return CLIMSR_EINVAL;
  }
  int rows = round_up(out_c, 16);
  int ntc = rows >= 64 ? 4 : (rows >= 32 ? 2 : 1);
  int co_rows = ceil_div(rows, ntc * 16) * ntc * 16;
  int ks2 = ks * ks;
  int kw = in_c * ks2;
  long total = (long)out_c * in_c_real * ks2 + (bias_grad ? out_c : 0);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(ceil_div(total, 32)), dim3(256), 0, (hipStream_t)stream, partial, bias_partial,
                     nsplit, out_c, in_c_real, in_c, ks2, co_rows, kw, wgrad, bias_grad, accumulate);
  return check_launch("conv2d_wgrad_reduce");
}
