// LDS-DMA implicit-GEMM conv for CDNA4 (gfx950): the 3x3 / stride-1 / 32-channel-chunk shapes of conv.hip's GEO 1
// path (VGG19 perceptual-loss convs climsr/losses/perceptual.py:22-36, RDB conv5 / its data gradient
// climsr/models/esrgan.py:26,32-38, the discriminator's stride-1 layers climsr/models/rfb_esrgan.py:28-52).
#include <algorithm>
#include <type_traits>

#include "conv_ep.h"

// ------------------------------------------------------------------------------------------
// LDS-DMA form of the GEO 1 conv (3x3, stride 1, 32-channel chunks: VGG19 2_1..4_4, RDB conv5 / pull-x, the
// discriminator's stride-1 layers): ONE 8-wave workgroup per CU over a 32 x 16-pixel x 64-channel output tile (wave
// w: rows 4w..4w+3, the 4 x 4 MFMA fragments of conv_fwd_body GEO 1).  Chunk operands move global -> LDS by
// `buffer_load ... lds` (no staging registers, no ds_write, no VALU) into two buffers: chunk q + 1 is requested right
// after the barrier that opens chunk q and lands under its 144 MFMAs per wave, and the two waves of each SIMD hide
// each other's fragment-read latency.  (conv_fwd_kernel's two 4-wave workgroups per CU ran in lockstep, so their
// staging and MFMA phases added up: DESIGN §3.3.)  The weights of a chunk are staged once per 512 output pixels
// instead of per 256.
// LDS images are lane-linear (one DMA instruction = 64 lanes x 16 B, contiguous): x = [34 x 18 px][4 x 16 B],
// weights = [64 rows][9 taps][4 x 16 B].  The 16 B slot s of x-tile column c / weight row r holds channel group
// s ^ 2((c >> 2) & 1) / s ^ 2((r >> 2) & 1) (the XOR is applied on the global side): every 16-lane bank group of a
// ds_read_b128 fragment read then covers the 64 banks once, and the k-steps' fragment offsets stay compile-time
// immediates on top of three per-lane x bases (one per tap column) and one weight base.
// ------------------------------------------------------------------------------------------
constexpr int DMA_TPW = TW + 2, DMA_XROW = DMA_TPW * 64;  // x-image bytes per tile row
constexpr int DMA_XU = (DMA_TH + 2) * DMA_TPW * 4;                    // 16 B units of the x image (2448)
constexpr int DMA_XI = (DMA_XU + 63) / 64;                            // its DMA instructions (39)
constexpr int DMA_WI = 64 * 36 / 64;                                  // weight DMA instructions (36)
constexpr int DMA_XB = DMA_XI * 1024, DMA_WB = DMA_WI * 1024, DMA_BUF = DMA_XB + DMA_WB;
constexpr int DMA_EPP = 64 + 4;                                       // epilogue staging pitch (floats)
constexpr size_t DMA_LDS = std::max((size_t)2 * DMA_BUF, (size_t)8 * 64 * DMA_EPP * 4);
static_assert(DMA_LDS <= 160 * 1024, "LDS-DMA conv: two chunk buffers");


// Epilogue of one wave's 64 pixels x 32 channels (staged fp32 at eb, pitch EPH) for the persistent EPs: the math of
// store_tile_lds (same helpers, same order: bit-identical results), but every lane issues the same number of buffer
// stores whatever its pixels (invalid ones get an out-of-range offset, which the hardware drops), so the next chunk's
// DMA wait can count them: NSTORE per call.
constexpr uint32_t ST_OOB = 0xFFFFFFC0u;
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
template <int EP>
struct DmaEp {
  static constexpr bool F32 = EP == 2 || EP == 7;                          // fp32 '=' output
  static constexpr int NSTORE = 4 * (F32 ? 2 : 1) + (EP == 2 ? 4 : 0);     // per call (EP 2: + the bf16 aux)
};
template <int EP>
__device__ __forceinline__ void dma_store_half(const FwdArgs& a, const float* eb, int ehp, int lane, int nimg, int oyw, int ox0, int co0) {
  static_assert(EP == 1 || EP == 2 || EP == 3 || EP == 6 || EP == 7 || EP == 8, "persistent epilogues");
  constexpr bool F32 = DmaEp<EP>::F32;
  const bool has_bias = EP == 1 || EP == 3;
  const int act = (EP == 3 || EP == 6) ? a.act : 0;
  const bool has1 = EP == 1 || EP == 2, has2 = (EP == 1 || EP == 2) && a.res2 != nullptr;
  const long opx = (long)a.n * a.out_h * a.out_w;
  const __amdgpu_buffer_rsrc_t ry = buf_rsrc(a.y, (uint32_t)(opx * a.out_cs * (F32 ? 4 : 2)));
  const __amdgpu_buffer_rsrc_t rr1 = opt_rsrc(has1 ? a.res1 : nullptr), rr2 = opt_rsrc(has2 ? a.res2 : nullptr);
  const __amdgpu_buffer_rsrc_t rax = buf_rsrc(a.aux, EP == 2 && a.aux ? (uint32_t)(opx * a.aux_cs * 2) : 0u);
  Raw8 r1[4], r2[4];
  uint32_t off[4], aoff[4];
  long pidx[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int it = j * 64 + lane, pl = it >> 2, cg = it & 3;
    const int oy = oyw + (pl >> 4), ox = ox0 + (pl & 15), co = co0 + cg * 8;
    const bool ok = oy < a.out_h && ox < a.out_w && co < a.out_c;
    pidx[j] = ok ? ((long)(nimg * a.out_h + oy) * a.out_w + ox) : 0;
    const int c = ok ? co : 0;
    off[j] = ok ? (uint32_t)((pidx[j] * a.out_cs + a.out_co + co) * (F32 ? 4 : 2)) : ST_OOB;
    aoff[j] = ok ? (uint32_t)((pidx[j] * a.aux_cs + a.aux_co + co) * 2) : ST_OOB;
    if (has1) r1[j] = load8b(rr1, EP == 2, pidx[j] * a.r1_cs + (ok ? a.r1_co : 0) + c);
    else r1[j].lo = r1[j].hi = make_uint4(0, 0, 0, 0);
    if (EP == 1 || EP == 2) r2[j] = load8b(rr2, EP == 2, pidx[j] * a.r2_cs + (ok ? a.r2_co : 0) + c);
    else r2[j].lo = r2[j].hi = make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int it = j * 64 + lane, pl = it >> 2, cg = it & 3;
    const int co = co0 + cg * 8;
    const float4 s0 = *(const float4*)(eb + pl * ehp + cg * 8), s1 = *(const float4*)(eb + pl * ehp + cg * 8 + 4);
    float v[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    float bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (has_bias && off[j] != ST_OOB) {
      const float4 b0 = *(const float4*)(a.bias + co), b1 = *(const float4*)(a.bias + co + 4);
      bb[0] = b0.x; bb[1] = b0.y; bb[2] = b0.z; bb[3] = b0.w; bb[4] = b1.x; bb[5] = b1.y; bb[6] = b1.z; bb[7] = b1.w;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
      v[i] = ep_res(act_apply(v[i] + bb[i], act, a.slope), act, a.slope, has1, raw8_at(r1[j], EP == 2, i), a.alpha1, a.beta1, has2,
                    raw8_at(r2[j], EP == 2, i), a.alpha2, a.beta2);
    if constexpr (F32) {
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, make_float4(v[0], v[1], v[2], v[3])), ry, off[j], 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, make_float4(v[4], v[5], v[6], v[7])), ry, off[j] + 16u, 0, 0);
    } else {
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, pack8_bf16(v, 1.f)), ry, off[j], 0, 0);
    }
    if constexpr (EP == 2) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, pack8_bf16(v, a.aux_scale)), rax, aoff[j], 0, 0);
  }
}


// Persistent over (tile, channel block) items v = blockIdx.x + k gridDim.x (host: gridDim.x <= #CUs, a multiple of 8,
// so v's XCD is blockIdx.x's and xcd_major keeps a tile's channel blocks on one L2): the chunks of consecutive items
// form one stream, so the next item's chunk 0 lands under the current item's last chunk, and the epilogue's stores
// drain under the next item's MFMAs.  The epilogue stages each wave's 64 pixels x 32 channels at a time through the
// chunk buffer just computed (the other one is receiving the next chunk).  EP 9 / 10 (BatchNorm partials of a whole
// 64-channel tile): one item per workgroup, the whole tile staged at once.
template <int EP, bool RF>
__global__ __launch_bounds__(512, 1) void conv_fwd_dma_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool BN = EP == 9 || EP == 10;
  // epilogues with a fixed store count per lane (dma_store_half), so the wait for the next item's chunk 0 skips them
  constexpr bool CNT = EP == 1 || EP == 2 || EP == 3 || EP == 6 || EP == 7 || EP == 8 || EP == 11;
  // EP 3 / 6 / 8 store straight from the accumulators (16 stores per lane and item): no LDS staging, no barrier --
  // VGG 256 ch @64^2 295 -> 277 us, 512 ch @32^2 263 -> 249 us against the staged form (tools/perf_diag.py, r04dd).
  // (EP 9 the same way, with its BatchNorm sums xor-shuffled over the pixel columns, measured 9 % slower in the GAN
  // step, r04h: it keeps the staged tile)
  // EP 11: EP 3 followed by the 2x2 max pool of the activated output (VGG19's conv2_2 / conv3_4 / conv4_4 + MaxPool2d,
  // perceptual.py:16): a wave's 4 rows pool to 2 in registers, column pairs across lanes col / col ^ 1, even lanes store
  constexpr bool POOL = EP == 11;
  constexpr bool DIRECT = EP == 3 || EP == 6 || EP == 8 || POOL;
  constexpr int NST_ITEM = POOL ? 4 : DIRECT ? 8 : 2 * DmaEp<CNT ? EP : 8>::NSTORE;  // (direct: 16-B stores, below)
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, col = lane & 15;
  const int wvu = __builtin_amdgcn_readfirstlane(wave);
  const int ntile = a.tiles_x * a.tiles_y * a.n, ncob = (a.out_c + 63) / 64;  // = the host's packed-row blocks
  const int nitem = ntile * ncob;
  // item v -> tile, channel block (XCD-major (channel-block group, tile, channel block) order with xgrp, as conv_fwd_body)
  auto decode = [&](int v, int& nimg, int& oy0, int& ox0, int& co0, int& tyo) {
    int tile_id, cob;
    if (a.xgrp > 0) {
      const int idx = xcd_major(v, nitem), grp = idx / (ntile * a.xgrp), rem = idx - grp * (ntile * a.xgrp);
      tile_id = rem / a.xgrp;
      cob = grp * a.xgrp + (rem - tile_id * a.xgrp);
    } else {
      cob = v / ntile;
      tile_id = v - cob * ntile;
    }
    const int tx = tile_id % a.tiles_x, ty = (tile_id / a.tiles_x) % a.tiles_y;
    nimg = tile_id / (a.tiles_x * a.tiles_y);
    ox0 = tx * TW;
    oy0 = ty * DMA_TH;
    co0 = cob * 64;
    tyo = ty;
  };

  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(a.x, (uint32_t)((long)a.n * a.in_h * a.in_w * a.in_cs * 2));
  const __amdgpu_buffer_rsrc_t wr = buf_rsrc(a.w, (uint32_t)((long)ncob * 64 * a.kpk * 2));
  // per-lane DMA source offsets of an item's chunk 0 (wave w issues x / weight instructions w + 8 i); out-of-image and
  // past-the-image lanes get BUF_OOB, which stays out of range at every chunk (zeros land in LDS)
  // 32-channel chunk j of the packed weights (packing chunks of a.cc = 32 or 64 channels, tap-major within one):
  // packing chunk j / (cc / 32) at kcpad elements each, its channels 32 (j % (cc / 32)) ..
  const int ups = a.up == 2 ? 1 : 0, cpc = a.cc >> 5;
  auto wchunk = [&](uint32_t j) { return ((j / cpc) * (uint32_t)a.kcpad + (j % cpc) * 32u) * 2u; };
  uint32_t xo[5], wo[5];
  auto offsets = [&](int nimg, int oy0, int ox0, int co0) {
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int L = (wave + 8 * i) * 64 + lane, P = L >> 2, r = P / DMA_TPW, c = P - r * DMA_TPW;
      // (up 2: nearest x2 upsample on load, source pixel = logical >> 1)
      const int iy = oy0 - a.pad + r, ix = ox0 - a.pad + c, ch = (L & 3) ^ (((c >> 2) & 1) << 1);
      const bool ok = L < DMA_XU && iy >= 0 && iy < (a.in_h << ups) && ix >= 0 && ix < (a.in_w << ups);
      xo[i] = ok ? (uint32_t)((((nimg * a.in_h + (iy >> ups)) * a.in_w + (ix >> ups)) * a.in_cs + a.in_co + ch * 8) * 2) : BUF_OOB;
      const int row = L / 36, slot = L - row * 36, wch = (slot & 3) ^ (((row >> 2) & 1) << 1);
      wo[i] = L < 64 * 36 ? (uint32_t)(((co0 + row) * a.kpk + (slot >> 2) * a.cc + wch * 8) * 2) : BUF_OOB;
    }
  };
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;
  // in asm (not the builtin): hipcc would wait vmcnt(0) before the next ds_read for an LDS write of unknown extent;
  // the DMAs are drained by hand (vmcnt(0) at each chunk barrier).  M0 = the instruction's LDS destination.
  auto glds = [&](__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(off), "s"(rs), "s"(lds) : "memory");
  };
  // DMA piece p (0..9) of chunk j into buffer b: x instruction wave + 8 p (p < 5), weight instruction wave + 8 (p - 5)
  auto piece = [&](int p, uint32_t j, int b) {
    const uint32_t base = lds0 + (uint32_t)(b * DMA_BUF);
    if (p < 5) {
      if (wvu + 8 * p < DMA_XI) glds(xr, xo[p] + j * 64u, base + (uint32_t)((wvu + 8 * p) * 1024));
    } else if (wvu + 8 * (p - 5) < DMA_WI) {
      glds(wr, wo[p - 5] + wchunk(j), base + (uint32_t)(DMA_XB + (wvu + 8 * (p - 5)) * 1024));
    }
  };
  // fragment offsets: weights row 16 t + col, tap k, group g at woff + 16 t * 576 + 64 k; x pixel (4 wave + m + dy,
  // col + dx), group g at xoff[dx] + (m + dy) * DMA_XROW
  int xoff[3];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) {
    const int c = col + dx;
    xoff[dx] = wave * 4 * DMA_XROW + c * 64 + ((g ^ (((c >> 2) & 1) << 1)) << 4);
  }
  const int woff = col * 576 + ((g ^ (((col >> 2) & 1) << 1)) << 4);

  int v = blockIdx.x;
  if (v >= nitem) return;
  int nimg, oy0, ox0, co0, ty;
  decode(v, nimg, oy0, ox0, co0, ty);
  offsets(nimg, oy0, ox0, co0);
#pragma unroll
  for (int p = 0; p < 10; ++p) piece(p, 0, 0);
  int buf = 0;  // the buffer chunk j of the current item is in
  bool later = false;  // an item after the workgroup's first (its epilogue stores were issued behind chunk 0's DMAs)
  for (;;) {
    const int vn = BN ? nitem : v + (int)gridDim.x;  // the next item (none with BatchNorm partials)
    int nimg_n = 0, oy0_n = 0, ox0_n = 0, co0_n = 0, ty_n = 0;
    f32x4 acc[4][4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[m][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < a.nchunk; ++j, buf ^= 1) {
      // chunk j's DMAs (this wave's) have landed; after the barrier every wave's have, and every wave is past its
      // fragment reads of the other buffer (and of its epilogue staging), which the next chunk now overwrites.  The
      // wait also drains the previous item's epilogue stores (issued after the DMAs of this chunk)
      if (CNT && j == 0 && later) {
        // chunk 0 of a later item: only its DMAs, not the previous item's epilogue stores issued after them
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST_ITEM) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      lds_barrier();
      // the next chunk: chunk j + 1 of this item, or chunk 0 of the next one (its offsets replace this item's: every
      // DMA of this item has been issued); its 10 DMA pieces go out between this chunk's k-steps, behind their MFMAs
      const bool last = j + 1 == a.nchunk;
      if (last && vn < nitem) {
        decode(vn, nimg_n, oy0_n, ox0_n, co0_n, ty_n);
        offsets(nimg_n, oy0_n, ox0_n, co0_n);
      }
      const bool more = !last || vn < nitem;
      const uint32_t jn = last ? 0u : (uint32_t)(j + 1);
      const char* xb = smem + buf * DMA_BUF;
      const char* wb = xb + DMA_XB;
      bf16x8 af[2][4], bf[2][4];
      auto ld = [&](int k, int s) {
        const int dy = k / 3, dx = k % 3;
#pragma unroll
        for (int t = 0; t < 4; ++t) af[s][t] = *(const bf16x8*)(wb + woff + t * 16 * 576 + k * 64);
#pragma unroll
        for (int m = 0; m < 4; ++m) bf[s][m] = *(const bf16x8*)(xb + xoff[dx] + (m + dy) * DMA_XROW);
      };
      ld(0, 0);
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        if (k + 1 < 9) ld(k + 1, (k + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[k & 1][t], bf[k & 1][m], acc[m][t], 0, 0, 0);
        if (more) {  // one piece behind each k-step's MFMAs, two at the last (2 per k-step / 3-4-3 spreads: neutral)
          piece(k, jn, buf ^ 1);
          if (k == 8) piece(9, jn, buf ^ 1);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // epilogue through the buffer just computed (buf ^ 1 after the loop's last flip); LDS-only barriers, so the
    // stores stay in flight
    if (!DIRECT) lds_barrier();  // every wave's fragment reads of it are done
    if constexpr (BN) {
      float* eb = (float*)smem + wave * (64 * DMA_EPP);  // the whole tile (aliases both buffers: no DMA in flight)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int t = 0; t < 4; ++t) *(f32x4*)(eb + (m * 16 + col) * DMA_EPP + t * 16 + g * 4) = acc[m][t];
      lds_barrier();
      // BatchNorm partials per 16 x 16 tile (the rows of waves 4h..4h+3 are 16-row tile 2 ty + h; the host takes EP 9 /
      // 10 only for out_h % 32 == 0): the sums of conv_fwd_body's bn_tile_partials in the same fixed order, bit for bit
      float ssum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, ssq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      store_tile_lds<RF, 64, 64, 64, EP>(a, eb, DMA_EPP, lane, nimg, oy0 + wave * 4, ox0, co0, ssum, ssq);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int m = 8; m < 64; m <<= 1) {
          ssum[i] += __shfl_xor(ssum[i], m);
          ssq[i] += __shfl_xor(ssq[i], m);
        }
      lds_barrier();  // every wave's epilogue reads of the staging region are done
      float* red = (float*)smem + (wave >> 2) * 512;
      if (lane < 8) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          red[(wave & 3) * 128 + lane * 8 + i] = ssum[i];
          red[(wave & 3) * 128 + 64 + lane * 8 + i] = ssq[i];
        }
      }
      lds_barrier();
      if ((wave & 3) == 0) {
        float ts = 0.f, tq = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          ts += red[w * 128 + lane];
          tq += red[w * 128 + 64 + lane];
        }
        const long tile16 = ((long)nimg * (2 * a.tiles_y) + 2 * ty + (wave >> 2)) * a.tiles_x + ox0 / TW;
        double* out = a.bn_part + tile16 * 2 * a.out_c;
        out[co0 + lane] = (double)ts;
        out[a.out_c + co0 + lane] = (double)tq;
      }
      return;
    } else if (DIRECT) {
      // lane (col, g) holds channels co0 + 16 t + 4 g .. + 3 of pixel (oy0 + 4 wave + m, ox0 + col): bias / activation,
      // bf16, one 16 B store per (m, co-block pair) -- 8 per lane per item, issued unconditionally (out-of-range offsets drop)
      const long ypx = POOL ? (long)a.n * (a.out_h >> 1) * (a.out_w >> 1) : (long)a.n * a.out_h * a.out_w;
      const __amdgpu_buffer_rsrc_t ry = buf_rsrc(a.y, (uint32_t)(ypx * a.out_cs * 2));
      float bb[4][4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float4 b4 = (EP == 3 || POOL) ? *(const float4*)(a.bias + co0 + 16 * t + 4 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
        bb[t][0] = b4.x; bb[t][1] = b4.y; bb[t][2] = b4.z; bb[t][3] = b4.w;
      }
      const int ox = ox0 + col, act = EP == 8 ? 0 : a.act;
      // the activation resolved once per item (one uniform branch) instead of per element: act_apply with a run-time
      // act compiled to a branch tree around each of the 64 values (~470 branch instructions per kernel)
      auto store_all = [&](auto actc) {
        constexpr int ACT = decltype(actc)::value;
        if constexpr (POOL) {
          // pooled output pixel (oy0 / 2 + 2 wave + mp, (ox0 + col) / 2), held by lanes col and col ^ 1 alike: of each
          // co-block pair (t, t + 1) the even lane stores block t and the odd lane block t + 1 (4 stores per lane)
          const int ph = a.out_h >> 1, pw = a.out_w >> 1, px = (ox0 + col) >> 1, odd = col & 1;
#pragma unroll
          for (int mp = 0; mp < 2; ++mp) {
            const int py = (oy0 >> 1) + 2 * wave + mp;
            const bool ok = py < ph && px < pw;
            const long pix = ((long)nimg * ph + py) * pw + px;
#pragma unroll
            for (int tp = 0; tp < 4; tp += 2) {
              float w[4];  // block tp + odd: both blocks' maxima are formed (the xor shuffle needs every lane), one kept
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                float m2[2];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                  const float r0 = act_apply(acc[2 * mp][tp + u][i] + bb[tp + u][i], ACT, a.slope);
                  const float r1 = act_apply(acc[2 * mp + 1][tp + u][i] + bb[tp + u][i], ACT, a.slope);
                  const float rm = fmaxf(r0, r1);
                  m2[u] = fmaxf(rm, __shfl_xor(rm, 1));
                }
                w[i] = odd ? m2[1] : m2[0];
              }
              const bf16x2 p0 = {(__bf16)w[0], (__bf16)w[1]}, p1 = {(__bf16)w[2], (__bf16)w[3]};
              typedef uint32_t v2u32_t __attribute__((ext_vector_type(2)));
              const v2u32_t pk = {__builtin_bit_cast(uint32_t, p0), __builtin_bit_cast(uint32_t, p1)};
              const uint32_t off = ok ? (uint32_t)((pix * a.out_cs + a.out_co + co0 + 16 * (tp + odd) + 4 * g) * 2) : BUF_OOB;
              __builtin_amdgcn_raw_buffer_store_b64(pk, ry, off, 0, 0);
            }
          }
          return;
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int oy = oy0 + wave * 4 + m;
          const bool ok = oy < a.out_h && ox < a.out_w;
          const long pix = ((long)nimg * a.out_h + oy) * a.out_w + ox;
          uint32_t pk[4][2];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            float v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = act_apply(acc[m][t][i] + bb[t][i], ACT, a.slope);
            const bf16x2 p0 = {(__bf16)v[0], (__bf16)v[1]}, p1 = {(__bf16)v[2], (__bf16)v[3]};
            pk[t][0] = __builtin_bit_cast(uint32_t, p0);
            pk[t][1] = __builtin_bit_cast(uint32_t, p1);
            if (t & 1) {
              // co blocks t - 1, t: rows 1, 3 of block t - 1 <-> rows 0, 2 of block t (v_permlane16_swap): lane (col, g)
              // then holds channels 16 (t - 1 + (g & 1)) + 8 (g >> 1) .. + 7 of its pixel, one 16-B store
              const auto sx = __builtin_amdgcn_permlane16_swap(pk[t - 1][0], pk[t][0], false, false);
              const auto sy = __builtin_amdgcn_permlane16_swap(pk[t - 1][1], pk[t][1], false, false);
              typedef uint32_t v4u32_t __attribute__((ext_vector_type(4)));
              const v4u32_t o = {sx[0], sy[0], sx[1], sy[1]};
              const uint32_t off = ok ? (uint32_t)((pix * a.out_cs + a.out_co + co0 + 16 * (t - 1 + (g & 1)) + 8 * (g >> 1)) * 2) : BUF_OOB;
              __builtin_amdgcn_raw_buffer_store_b128(o, ry, off, 0, 0);
            }
          }
        }
      };
      if (act == 1) store_all(std::integral_constant<int, 1>{});
      else if (act == 2) store_all(std::integral_constant<int, 2>{});
      else store_all(std::integral_constant<int, 0>{});
    } else {
      constexpr int EPH = 32 + 4;  // staged pitch (floats) of one 32-channel half
      float* eb = (float*)(smem + (buf ^ 1) * DMA_BUF) + wave * (64 * EPH);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h) lds_barrier();  // the first half's reads are done
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int t = 0; t < 2; ++t) *(f32x4*)(eb + (m * 16 + col) * EPH + t * 16 + g * 4) = acc[m][2 * h + t];
        lds_barrier();  // (orders the staging writes before the reads: another vector type)
        {
          if constexpr (CNT) dma_store_half<(CNT && !POOL) ? EP : 8>(a, eb, EPH, lane, nimg, oy0 + wave * 4, ox0, co0 + 32 * h);
          else store_tile_lds<RF, 64, 32, 64, EP>(a, eb, EPH, lane, nimg, oy0 + wave * 4, ox0, co0 + 32 * h);
        }
      }
    }
    if (vn >= nitem) break;
    v = vn;
    later = true;
    nimg = nimg_n; oy0 = oy0_n; ox0 = ox0_n; co0 = co0_n; ty = ty_n;
  }
}

namespace climsr {
int fwd_dma_launch(int ep, const FwdArgs& a, int ncob, hipStream_t s) {
  void (*k)(FwdArgs) = nullptr;
  const bool rf = a.res_f32 != 0;
#define DMA_EP(E) \
  case E: k = rf ? conv_fwd_dma_kernel<E, true> : conv_fwd_dma_kernel<E, false>; break;
  switch (ep) {
    DMA_EP(0) DMA_EP(3) DMA_EP(4) DMA_EP(6) DMA_EP(7) DMA_EP(8) DMA_EP(9) DMA_EP(10) DMA_EP(11)
    default: set_error("conv2d_fwd: no LDS-DMA kernel for epilogue %d", ep); return CLIMSR_EINVAL;
  }
#undef DMA_EP
  if (int e = lds_opt_in((const void*)k, 160 * 1024)) return e;
  int ncu = device_cus();
  ncu = ncu >= 8 ? ncu / 8 * 8 : 8;  // a multiple of 8: an item's XCD is its workgroup's (kernel comment)
  // one workgroup per item with BatchNorm partials, else persistent: at most one workgroup per CU
  const int nitem = a.tiles_x * a.tiles_y * a.n * ncob;
  const int grid = (ep == 9 || ep == 10) ? nitem : std::min(nitem, ncu);
  hipLaunchKernelGGL(k, dim3(grid), dim3(512), DMA_LDS, s, a);
  return CLIMSR_OK;
}
}  // namespace climsr

// ------------------------------------------------------------------------------------------
// LDS-DMA form of the 3x3 / stride-2 / pad-1 forward (the discriminator's downsampling convs rfb_esrgan.py:30-48,
// plain bf16 out, optionally with the BatchNorm partials of each 16 x 16 output tile).  The chunks are 16 channels,
// moved by LDS-DMA into three 53 KB buffers -- x = [33 x 33 px][2 x 16 B], weights = [64 rows][9 taps][2 x 16 B] --
// chunk c + 2 requested while chunk c computes (the register-staged kernel it replaced alternated staging and MFMAs
// over one buffer: MFMA busy 0.17); 8 waves, wave w owns output rows 2w, 2w+1 (x 64 channels); a k block is a PAIR
// of taps (lanes 0-31 tap 2kk, 32-63 tap 2kk+1, 16 channels each: 5 k blocks per chunk, the last half zero-weighted).
// Persistent over (tile, 64-channel block) items; the epilogue stores straight from the accumulators (8 B per lane and
// fragment) and folds the BatchNorm sums per channel through a small per-wave LDS transpose in the buffer just
// computed.
// ------------------------------------------------------------------------------------------
constexpr int S2D_TP = 33;                             // input tile side of a 16 x 16 output tile
constexpr int S2D_XI = (S2D_TP * S2D_TP * 2 + 63) / 64;  // x DMA instructions per chunk (35)
constexpr int S2D_WI = 64 * 9 * 2 / 64;                // weight DMA instructions per chunk (18)
constexpr int S2D_XB = S2D_XI * 1024, S2D_BUF = S2D_XB + S2D_WI * 1024;  // 54,272 B per buffer
constexpr int S2D_RED = 64 * 17 * 4;                   // per wave: channel-sum transpose [64][17]
constexpr int S2D_DUMMY = 3 * S2D_BUF;                 // 162,816 B: three chunk buffers, two chunks in flight,
constexpr int S2D_LDS = S2D_DUMMY + 1024;              // then one KB the padding DMA pieces write (zeros, never read)
static_assert(S2D_LDS <= 160 * 1024, "stride-2 LDS-DMA conv");
static_assert(8 * S2D_RED + 8 * 2 * 64 * 4 <= S2D_BUF, "BatchNorm scratch (aliases the buffer just computed)");

template <bool STATS>
__global__ __launch_bounds__(512, 1) void conv_fwd_s2_dma_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, col = lane & 15;
  const int wvu = __builtin_amdgcn_readfirstlane(wave);
  const int ntile = a.tiles_x * a.tiles_y * a.n, ncob = a.out_c / 64, nitem = ntile * ncob;
  const int nch = a.in_c / 16;  // 16-channel chunks
  auto decode = [&](int v, int& nimg, int& oy0, int& ox0, int& co0, int& tile) {
    const int idx = xcd_major(v, nitem);  // a tile's channel blocks consecutive on one XCD: its x chunks hit that L2
    tile = idx / ncob;
    co0 = (idx - tile * ncob) * 64;
    const int tx = tile % a.tiles_x, ty = (tile / a.tiles_x) % a.tiles_y;
    nimg = tile / (a.tiles_x * a.tiles_y);
    ox0 = tx * 16;
    oy0 = ty * 16;
  };
  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(a.x, (uint32_t)((long)a.n * a.in_h * a.in_w * a.in_cs * 2));
  const __amdgpu_buffer_rsrc_t wr = buf_rsrc(a.w, (uint32_t)((long)ncob * 64 * a.kpk * 2));
  // this wave's DMA pieces: x instructions wave + 8 j (j < 5), weight instructions wave + 8 j (j < 3)
  uint32_t xo[5], wo[3];
  auto offsets = [&](int nimg, int oy0, int ox0, int co0) {
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      // slot sl of a footprint row holds column 2 sl (sl < 17) or 2 (sl - 17) + 1: the even columns first, then the
      // odd ones, so a stride-2 fragment read (columns 2 col + kx) hits consecutive slots -- conflict-free b128 reads
      // (in column order the 16 lanes of a bank group covered half of the banks twice)
      const int u = (wave + 8 * j) * 64 + lane, p = u >> 1, h = u & 1, r = p / S2D_TP, sl = p - r * S2D_TP;
      const int c = sl < 17 ? 2 * sl : 2 * (sl - 17) + 1;
      const int iy = 2 * oy0 - 1 + r, ix = 2 * ox0 - 1 + c;
      const bool ok = p < S2D_TP * S2D_TP && iy >= 0 && iy < a.in_h && ix >= 0 && ix < a.in_w;
      xo[j] = ok ? (uint32_t)((((nimg * a.in_h + iy) * a.in_w + ix) * a.in_cs + a.in_co + 8 * h) * 2) : BUF_OOB;
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int u = (wave + 8 * j) * 64 + lane, row = u / 18, rem = u - row * 18;
      wo[j] = u < 64 * 18 ? (uint32_t)(((co0 + row) * a.kpk + (rem >> 1) * 32 + 8 * (rem & 1)) * 2) : BUF_OOB;
    }
  };
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;
  // lag (tests/isa_waitcnt_lint.py): chunk 0's pieces are retired by the first hand wait after their issue, every later
  // chunk's by the second (the next chunk is requested behind it)
  bool lag2 = false;
  auto glds = [&](__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t lds) {
    uint32_t keep;
    if (lag2)
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds ; dma-lag 2\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(off), "s"(rs), "s"(lds) : "memory");
    else
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(off), "s"(rs), "s"(lds) : "memory");
  };
  // chunk c (16 channels): x source offset + 32 c bytes; weights: packing chunk c / 2 (288 elements each), half c % 2.
  // Every wave issues all 8 pieces of a chunk: those past the 35 x / 18 weight instructions read out of range into the
  // dummy KB, so one count fits every wave's waits (with 8 / 7 / 6 real pieces per wave the waits were per-wave counts
  // that depended on the same wave index as the issue conditions).  (7 pieces per wave -- 3 padding pieces instead of
  // 11 -- leaves 10 operations behind a chunk's fourth piece, fewer than the 11 the first two chunks of a later item
  // wait for; the wait lint cannot tell those chunks from the rest, so the padding stays at 8.)
  auto piece = [&](int p, int c, int b, bool any = true) {  // any = false: nothing to request (dummy pieces only)
    const uint32_t base = lds0 + (uint32_t)(b * S2D_BUF);
    if (p < 5) {
      const bool real = any && wvu + 8 * p < S2D_XI;
      glds(xr, real && xo[p] != BUF_OOB ? xo[p] + (uint32_t)(32 * c) : BUF_OOB,
           real ? base + (uint32_t)((wvu + 8 * p) * 1024) : lds0 + (uint32_t)S2D_DUMMY);
    } else {
      const bool real = any && wvu + 8 * (p - 5) < S2D_WI;
      const uint32_t add = (uint32_t)(((c >> 1) * 288 + 16 * (c & 1)) * 2);
      glds(wr, real && wo[p - 5] != BUF_OOB ? wo[p - 5] + add : BUF_OOB,
           real ? base + (uint32_t)(S2D_XB + (wvu + 8 * (p - 5)) * 1024) : lds0 + (uint32_t)S2D_DUMMY);
    }
  };
  // fragment reads: k block kk, lane group g -> tap 2 kk + (g >> 1) (tap 9: read tap 8 under zero weights), half g & 1
  const int hh = g & 1;
  auto tap_of = [&](int kk) { return min(2 * kk + (g >> 1), 8); };

  int v = blockIdx.x;
  if (v >= nitem) return;
  int nimg, oy0, ox0, co0, tile;
  decode(v, nimg, oy0, ox0, co0, tile);
  offsets(nimg, oy0, ox0, co0);
  // chunks 0 and 1 in flight before the loop; chunk c + 2 (of this item, or of the next one) is requested during chunk
  // c into the third buffer: 8 DMA pieces per wave and chunk
#pragma unroll
  for (int p = 0; p < 8; ++p) piece(p, 0, 0);
  lag2 = true;
#pragma unroll
  for (int p = 0; p < 8; ++p) piece(p, 1, 1);
  int cur = 0;  // the buffer of the chunk being computed
  bool later = false;  // an item after the workgroup's first (its epilogue stores were issued between its chunks 0 and 1)
  for (;;) {
    const int vn = v + (int)gridDim.x;
    int nimg_n = 0, oy0_n = 0, ox0_n = 0, co0_n = 0, tile_n = 0;
    f32x4 acc[2][4];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[m][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < nch; ++c, cur = cur == 2 ? 0 : cur + 1) {
      // chunk c has landed once at most the younger requests are outstanding: the next chunk's 8 pieces (dummies behind
      // the last two chunks of the last item), and at chunks 0 / 1 of a later item also the previous item's 4 epilogue
      // stores (issued between them)
      if (c < 2 && later) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      lds_barrier();
      // the request of this chunk: chunk c + 2 of this item, or chunk c + 2 - nch of the next one (whose offsets
      // replace this item's once every piece of this item has been requested)
      if (c + 2 == nch && vn < nitem) {
        decode(vn, nimg_n, oy0_n, ox0_n, co0_n, tile_n);
        offsets(nimg_n, oy0_n, ox0_n, co0_n);
      }
      const bool more = c + 2 < nch || vn < nitem;
      const int cn = c + 2 < nch ? c + 2 : c + 2 - nch;
      const int bn = cur == 0 ? 2 : cur - 1;  // (cur + 2) % 3
      const char* xb = smem + cur * S2D_BUF;
      const char* wb = xb + S2D_XB;
      bf16x8 af[2][4], bq[2][2];
      auto ld = [&](int kk, int s) {
        const int tap = tap_of(kk), ky = tap / 3, kx = tap - ky * 3;
#pragma unroll
        for (int t = 0; t < 4; ++t) af[s][t] = *(const bf16x8*)(wb + ((16 * t + col) * 9 + tap) * 32 + 16 * hh);
        if (kk == 4 && g >= 2) {  // the pair's second tap of block 4 does not exist: zero weights (its B reads tap 8)
#pragma unroll
          for (int t = 0; t < 4; ++t) af[s][t] = (bf16x8){};
        }
#pragma unroll
        for (int m = 0; m < 2; ++m)
          bq[s][m] = *(const bf16x8*)(xb + ((2 * (2 * wave + m) + ky) * S2D_TP + col + (kx == 1 ? 17 : kx >> 1)) * 32 + 16 * hh);
      };
      ld(0, 0);
#pragma unroll
      for (int kk = 0; kk < 5; ++kk) {
        if (kk + 1 < 5) ld(kk + 1, (kk + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk & 1][t], bq[kk & 1][m], acc[m][t], 0, 0, 0);
        if (kk < 4) {  // the requested chunk's 8 DMA pieces, two per k block behind its MFMAs
          piece(2 * kk, cn, bn, more);
          piece(2 * kk + 1, cn, bn, more);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // ---- epilogue straight from the accumulators: lane (col, g) holds channels co0 + 16 t + 4 g .. + 3 of output pixel
    // (oy0 + 2 wave + m, ox0 + col); co-block pairs traded between lane rows (v_permlane16_swap) -> 4 16-B stores per
    // lane, issued unconditionally
    const __amdgpu_buffer_rsrc_t ry = buf_rsrc(a.y, (uint32_t)((long)a.n * a.out_h * a.out_w * a.out_cs * 2));
    const int ox = ox0 + col;
    float ss[4][4] = {}, sq[4][4] = {};
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int oy = oy0 + 2 * wave + m;
      const bool ok = oy < a.out_h && ox < a.out_w;
      const long pix = ((long)nimg * a.out_h + oy) * a.out_w + ox;
      uint32_t pk[4][2];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf16x2 p0 = {(__bf16)acc[m][t][0], (__bf16)acc[m][t][1]}, p1 = {(__bf16)acc[m][t][2], (__bf16)acc[m][t][3]};
        pk[t][0] = __builtin_bit_cast(uint32_t, p0);
        pk[t][1] = __builtin_bit_cast(uint32_t, p1);
        if (t & 1) {  // lane (col, g): channels co0 + 16 (t - 1 + (g & 1)) + 8 (g >> 1) .. + 7 after the trade
          const auto sx = __builtin_amdgcn_permlane16_swap(pk[t - 1][0], pk[t][0], false, false);
          const auto sy = __builtin_amdgcn_permlane16_swap(pk[t - 1][1], pk[t][1], false, false);
          typedef uint32_t v4u32_t __attribute__((ext_vector_type(4)));
          const v4u32_t o = {sx[0], sy[0], sx[1], sy[1]};
          __builtin_amdgcn_raw_buffer_store_b128(
              o, ry, ok ? (uint32_t)((pix * a.out_cs + a.out_co + co0 + 16 * (t - 1 + (g & 1)) + 8 * (g >> 1)) * 2) : BUF_OOB, 0, 0);
        }
        if (STATS && ok) {
          const float r[4] = {(float)p0[0], (float)p0[1], (float)p1[0], (float)p1[1]};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            ss[t][i] += r[i];
            sq[t][i] = fmaf(r[i], r[i], sq[t][i]);
          }
        }
      }
    }
    if constexpr (STATS) {
      // per channel over the tile's 256 pixels: each wave transposes its column sums through its own LDS corner (sum,
      // then square sum), lane l = channel l adds its 16 columns in order; the 8 waves meet in LDS, fixed order, fp64
      // scratch in the buffer just computed ((cur + 2) % 3 after the loop; the other two hold the next item's chunks 0
      // and 1 in flight), once every wave is past its fragment reads of it
      lds_barrier();
      const int fb = cur == 0 ? 2 : cur - 1;
      float* red = (float*)(smem + fb * S2D_BUF) + wave * (S2D_RED / 4);
      float* fin = (float*)(smem + fb * S2D_BUF + 8 * S2D_RED);  // [wave][2][64]
      float cs[2];
#pragma unroll
      for (int st = 0; st < 2; ++st) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) red[(16 * t + 4 * g + i) * 17 + col] = st ? sq[t][i] : ss[t][i];
        float x = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) x += red[lane * 17 + k];
        cs[st] = x;
      }
      fin[wave * 128 + lane] = cs[0];
      fin[wave * 128 + 64 + lane] = cs[1];
      lds_barrier();
      if (tid < 128) {
        const int st = tid >> 6, ch = tid & 63;
        float x = 0.f;
#pragma unroll
        for (int w = 0; w < 8; ++w) x += fin[w * 128 + st * 64 + ch];
        a.bn_part[(long)tile * 2 * a.out_c + st * a.out_c + co0 + ch] = (double)x;
      }
      lds_barrier();  // fin is reused by the next item
    }
    if (vn >= nitem) break;
    v = vn;
    later = true;
    nimg = nimg_n; oy0 = oy0_n; ox0 = ox0_n; co0 = co0_n; tile = tile_n;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

namespace climsr {
int fwd_s2_dma_launch(const FwdArgs& a, hipStream_t s) {
  void (*k)(FwdArgs) = a.bn_part ? conv_fwd_s2_dma_kernel<true> : conv_fwd_s2_dma_kernel<false>;
  if (int e = lds_opt_in((const void*)k, S2D_LDS)) return e;
  const int nitem = a.tiles_x * a.tiles_y * a.n * (a.out_c / 64);
  const int grid = std::min(nitem, device_cus());
  hipLaunchKernelGGL(k, dim3(grid), dim3(512), S2D_LDS, s, a);
  return CLIMSR_OK;
}
}  // namespace climsr
