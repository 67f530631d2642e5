// The discriminator's stem, features.0 (1 -> 64, 3x3, LeakyReLU) and features.2 (64 -> 64, 3x3 / stride 2, the
// pre-BatchNorm output with the BatchNorm partial sums of its tiles) in ONE launch (rfb_esrgan.py:28-31).
//
// features.0's output is the largest tensor of the discriminator (B x 256^2 x 64 bf16 = 268 MB at B = 32) and holds 9
// MACs per element of information: it is recomputed from the 1-channel input where features.2 needs it instead of
// being written by one launch and read back by the next (the stride-2 conv reading it was bound by that read at
// ~2.3 TB/s).  It is still written once (own pixels of each tile) when the caller keeps it for the backward.
//
// A workgroup (8 waves) walks 16 x 16 output tiles (all 64 output channels).  Per tile: the 35 x 35 input pixels go to
// LDS; each wave gathers its im2col fragments of the 33 x 33 features.0 region once (tap k of pixel p in lane group
// k / 8: 9 taps of a 32-deep K, the rest zero); then per 16-channel chunk c of features.0 one MFMA per 16 pixels
// computes that chunk (A = W0 rows 16c .. 16c + 15), LeakyReLU, bf16, into an LDS image the stride-2 conv reads,
// while the previous chunk's conv MFMAs run (two image buffers, one barrier per chunk).  features.2's weights
// (4 chunks x 18 KB) stay in LDS for the launch.  The conv part is conv_fwd_s2_dma_kernel's (conv_dma.hip): wave w
// owns output rows 2w, 2w + 1; a k block is a pair of taps x 16 channels; BatchNorm sums per 16 x 16 tile in the same
// fixed order.  Image rows keep their 17 even columns before their 16 odd ones, so the 8 pixels 2 apart that a
// stride-2 fragment read touches sit in consecutive slots (conflict-free ds_read_b128).
#include "conv_ep.h"

namespace {

constexpr int ST_TP = 33;                              // features.0 region side per 16 x 16 output tile
constexpr int ST_IN = 35;                              // input region side
constexpr int ST_NF = (ST_TP * ST_TP + 15) / 16;       // 16-pixel im2col fragments of the region (69)
constexpr int ST_FPW = (ST_NF + 7) / 8;                // per wave (9)
constexpr int ST_WCH = 64 * 9 * 32;                    // features.2 weights of one 16-channel chunk: [co][tap][2 x 16 B]
constexpr int ST_XB = ST_TP * ST_TP * 32;              // one 16-channel image of the region: [row][slot][2 x 16 B]
constexpr int ST_OFF_X = 4 * ST_WCH;                   // 73,728
constexpr int ST_OFF_IN = ST_OFF_X + 2 * ST_XB;        // 143,424
constexpr int ST_OFF_FIN = ST_OFF_IN + 2464;           // 145,888: BatchNorm [wave][2][64] fp32
constexpr int ST_LDS = ST_OFF_FIN + 8 * 2 * 64 * 4;    // 149,984
constexpr int ST_RED = 64 * 17 * 4;                    // per wave: the channel-sum transpose (in image buffer 0)
constexpr int ST_T8 = ST_TP * ST_TP * 16;              // im2col (in image buffer 1): tap 8 after taps 0..7
static_assert(ST_T8 + ST_TP * ST_TP * 2 <= ST_XB, "im2col fits one image buffer");
static_assert(8 * ST_RED <= ST_XB, "BatchNorm transpose fits one image buffer");
static_assert(ST_LDS <= 160 * 1024, "stem LDS");

struct StemArgs {
  const uint16_t* x;
  const float* w0;
  const uint16_t* w2;
  uint16_t* a0;
  uint16_t* z2;
  double* bn_part;
  int x_cs, kpk2, n, h, w, oh, ow, tiles_x, tiles_y;
  float slope;
  uint32_t x_bytes, a0_bytes, z_bytes;
};
typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int slot_of(int c) { return (c & 1) ? 17 + (c >> 1) : (c >> 1); }  // even columns first

template <bool STATS, bool KEEP>
__global__ __launch_bounds__(512, 1) void stem_s2_kernel(StemArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, col = lane & 15, hh = g & 1;
  const int ntile = a.tiles_x * a.tiles_y * a.n;
  // features.2's weights into LDS once: chunk c, row co, tap t, half hf <- packed [co][c / 2][t][32] at (c & 1) * 16
  for (int u = tid; u < 4 * 64 * 9 * 2; u += 512) {
    const int hf = u & 1, t = (u >> 1) % 9, co = (u / 18) % 64, c = u / (18 * 64);
    const uint4 v = *(const uint4*)(a.w2 + (long)co * a.kpk2 + (c >> 1) * 288 + t * 32 + (c & 1) * 16 + hf * 8);
    *(uint4*)(smem + c * ST_WCH + ((co * 9 + t) * 2 + hf) * 16) = v;
  }
  // features.0's A fragments: rows 16 c + col, lane group g: taps 8 g .. 8 g + 7 (tap 8 alone in group 1), bf16 RNE
  bf16x8 A0[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    bf16x8 v = {};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int t = 8 * g + e;
      v[e] = t < 9 ? (__bf16)a.w0[(16 * c + col) * 9 + t] : (__bf16)0.f;
    }
    A0[c] = v;
  }
  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(a.x, a.x_bytes);
  const __amdgpu_buffer_rsrc_t ar = buf_rsrc(a.a0, KEEP ? a.a0_bytes : 0u);
  const __amdgpu_buffer_rsrc_t zr = buf_rsrc(a.z2, a.z_bytes);
  const uint16_t* in = (const uint16_t*)(smem + ST_OFF_IN);

  for (int tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
    const int tx = tile % a.tiles_x, ty = (tile / a.tiles_x) % a.tiles_y, nimg = tile / (a.tiles_x * a.tiles_y);
    const int ox0 = 16 * tx, oy0 = 16 * ty, iy0 = 2 * oy0 - 1, ix0 = 2 * ox0 - 1;  // region origin (features.0 pixels)
    // the 35 x 35 input pixels around the region (zeros outside the image); the previous tile's readers of this
    // buffer are two barriers back
    for (int u = tid; u < ST_IN * ST_IN; u += 512) {
      const int r = u / ST_IN, c = u - r * ST_IN, iy = iy0 - 1 + r, ix = ix0 - 1 + c;
      const bool ok = iy >= 0 && iy < a.h && ix >= 0 && ix < a.w;
      const uint32_t off = ok ? (uint32_t)((((long)nimg * a.h + iy) * a.w + ix) * a.x_cs * 2) : BUF_OOB;
      ((uint16_t*)(smem + ST_OFF_IN))[u] = (uint16_t)__builtin_amdgcn_raw_buffer_load_b32(xr, off, 0, 0);
    }
    lds_barrier();
    // im2col of the region into image buffer 1 (free until chunk 1's features.0 is written, two barriers on): taps 0..7
    // of pixel p as 16 B at 16 p, tap 8 as 2 B at ST_T8 + 2 p
    {
      char* ic = smem + ST_OFF_X + ST_XB;
      for (int p = tid; p < ST_TP * ST_TP; p += 512) {
        const int r = p / ST_TP, c = p - r * ST_TP;
        const uint16_t* q = in + r * ST_IN + c;
        uint4 v;
        v.x = (uint32_t)q[0] | ((uint32_t)q[1] << 16);
        v.y = (uint32_t)q[2] | ((uint32_t)q[ST_IN] << 16);
        v.z = (uint32_t)q[ST_IN + 1] | ((uint32_t)q[ST_IN + 2] << 16);
        v.w = (uint32_t)q[2 * ST_IN] | ((uint32_t)q[2 * ST_IN + 1] << 16);
        *(uint4*)(ic + 16 * p) = v;
        *(uint16_t*)(ic + ST_T8 + 2 * p) = q[2 * ST_IN + 2];
      }
    }
    lds_barrier();
    // this wave's im2col fragments j = wave + 8 i of the region (pixel p = 16 j + col): lane group 0 = taps 0..7,
    // group 1 = tap 8 and zeros, groups 2 / 3 zeros (K = 9 of 32)
    bf16x8 Bs[ST_FPW];
    {
      const char* ic = smem + ST_OFF_X + ST_XB;
#pragma unroll
      for (int i = 0; i < ST_FPW; ++i) {
        const int p0 = 16 * (wave + 8 * i) + col, pv = p0 < ST_TP * ST_TP, p = pv ? p0 : 0;
        const uint4 t07 = *(const uint4*)(ic + 16 * p);
        const uint16_t t8 = *(const uint16_t*)(ic + ST_T8 + 2 * p);
        const uint4 v = !pv || g >= 2 ? make_uint4(0, 0, 0, 0) : (g == 0 ? t07 : make_uint4((uint32_t)t8, 0, 0, 0));
        Bs[i] = __builtin_bit_cast(bf16x8, v);
      }
    }
    // where each of this wave's region pixels goes: its LDS image slot (bit 30 set: outside the image, the slot gets
    // zeros) and, when kept, the byte offset of its channel 0 in a0 (own pixels only; BUF_OOB otherwise)
    uint32_t soff[ST_FPW], aoff[ST_FPW];
#pragma unroll
    for (int i = 0; i < ST_FPW; ++i) {
      const int p0 = 16 * (wave + 8 * i) + col, pv = p0 < ST_TP * ST_TP, p = pv ? p0 : 0, r = p / ST_TP, cc = p - r * ST_TP;
      const int iy = iy0 + r, ix = ix0 + cc;
      const bool in_img = iy >= 0 && iy < a.h && ix >= 0 && ix < a.w;
      soff[i] = pv ? (uint32_t)((r * ST_TP + slot_of(cc)) * 32 + g * 8) | (in_img ? 0u : 0x40000000u) : 0xFFFFFFFFu;
      aoff[i] = KEEP && pv && in_img && r >= 1 && cc >= 1 ? (uint32_t)(((nimg * a.h + iy) * a.w + ix) * 64) * 2u : BUF_OOB;
    }
    // features.0 chunk c (channels 16 c ..) of the region -> image buffer c & 1 (and the kept output), three MFMAs at a
    // time.  The kept output is stored per chunk pair, by the odd chunk: it recomputes the even chunk's values (one more
    // MFMA per fragment; holding them in registers across the conv spilled), trades the pair's channel groups between
    // lane rows g, g ^ 1 (v_permlane16_swap) so that each lane holds 8 consecutive channels, and the 4 lanes of a pixel
    // store the pair's 64 contiguous bytes as 16-B stores (8-B stores per chunk wrote 32 B of each 128-B pixel run:
    // 2.3x the tensor in WRITE_SIZE)
    auto lrelu_pack = [&](const f32x4& z) -> v2u32 {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaxf(z[e], z[e] * a.slope);  // LeakyReLU, 0 <= slope <= 1
      const bf16x2 q0 = {(__bf16)v[0], (__bf16)v[1]}, q1 = {(__bf16)v[2], (__bf16)v[3]};
      return (v2u32){__builtin_bit_cast(uint32_t, q0), __builtin_bit_cast(uint32_t, q1)};
    };
    auto stem = [&](int c) {
      char* xb = smem + ST_OFF_X + (c & 1) * ST_XB;
#pragma unroll
      for (int i0 = 0; i0 < ST_FPW; i0 += 3) {
        f32x4 z[3];
        f32x4 zp[3];  // (KEEP, odd chunk: the even chunk recomputed)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          z[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0[c], Bs[i0 + k], (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          if (KEEP && (c & 1)) zp[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0[c - 1], Bs[i0 + k], (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int i = i0 + k;
          if (wave + 8 * i < ST_NF) {
            const v2u32 pv = lrelu_pack(z[k]);
            const bool zero = soff[i] & 0x40000000u;
            const v2u32 pk = {zero ? 0u : pv[0], zero ? 0u : pv[1]};
            if (soff[i] != 0xFFFFFFFFu) *(v2u32*)(xb + (soff[i] & 0x3FFFFFFFu)) = pk;
            if constexpr (KEEP) {
              if (c & 1) {  // lane (col, g): channels 16 (c - 1 + (g & 1)) + 8 (g >> 1) .. + 7 of its pixel
                const v2u32 pe = lrelu_pack(zp[k]);
                const auto sx = __builtin_amdgcn_permlane16_swap(pe[0], pv[0], false, false);
                const auto sy = __builtin_amdgcn_permlane16_swap(pe[1], pv[1], false, false);
                typedef uint32_t v4u32_t __attribute__((ext_vector_type(4)));
                const v4u32_t o = {sx[0], sy[0], sx[1], sy[1]};
                __builtin_amdgcn_raw_buffer_store_b128(
                    o, ar, aoff[i] == BUF_OOB ? BUF_OOB : aoff[i] + (uint32_t)((16 * (c - 1 + (g & 1)) + 8 * (g >> 1)) * 2), 0, 0);
              }
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    stem(0);
    f32x4 acc[2][4];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[m][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c) {  // (unrolled: the chunk picks registers A0[c])
      lds_barrier();  // chunk c's image is complete; every wave is past its reads of the other buffer
      const char* xb = smem + ST_OFF_X + (c & 1) * ST_XB;
      const char* wb = smem + c * ST_WCH;
      // k block kk: lane group g -> tap 2 kk + (g >> 1) (tap 9: tap 8 under zero weights), channels 8 hh ..
      bf16x8 af[1][4], bq[1][2];
      auto ld = [&](int kk, int s) {
        const int tap = min(2 * kk + (g >> 1), 8), ky = tap / 3, kx = tap - ky * 3;
#pragma unroll
        for (int t = 0; t < 4; ++t) af[s][t] = *(const bf16x8*)(wb + ((16 * t + col) * 9 + tap) * 32 + 16 * hh);
        if (kk == 4 && g >= 2) {
#pragma unroll
          for (int t = 0; t < 4; ++t) af[s][t] = (bf16x8){};
        }
        const int sl = slot_of(2 * col + kx);
#pragma unroll
        for (int m = 0; m < 2; ++m) bq[s][m] = *(const bf16x8*)(xb + ((2 * (2 * wave + m) + ky) * ST_TP + sl) * 32 + 16 * hh);
      };
      
#pragma unroll
      for (int kk = 0; kk < 5; ++kk) {  // (fragments single-buffered: the SIMD's other wave covers their latency)
        ld(kk, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][t], bq[0][m], acc[m][t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (c + 1 < 4) stem(c + 1);  // into the other buffer, read by chunk c - 1 (every wave is past the barrier above)
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- epilogue straight from the accumulators: lane (col, g) holds channels 16 t + 4 g .. + 3 of output pixel
    // (oy0 + 2 wave + m, ox0 + col)
    const int ox = ox0 + col;
    float ss[4][4] = {}, sq[4][4] = {};
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int oy = oy0 + 2 * wave + m;
      const bool ok = oy < a.oh && ox < a.ow;
      const long pix = ((long)nimg * a.oh + oy) * a.ow + ox;
      uint32_t pk[4][2];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf16x2 p0 = {(__bf16)acc[m][t][0], (__bf16)acc[m][t][1]}, p1 = {(__bf16)acc[m][t][2], (__bf16)acc[m][t][3]};
        pk[t][0] = __builtin_bit_cast(uint32_t, p0);
        pk[t][1] = __builtin_bit_cast(uint32_t, p1);
        if (t & 1) {  // co-block pair traded between lane rows (v_permlane16_swap): channels 16 (t - 1 + (g & 1)) + 8 (g >> 1) ..
          const auto sx = __builtin_amdgcn_permlane16_swap(pk[t - 1][0], pk[t][0], false, false);
          const auto sy = __builtin_amdgcn_permlane16_swap(pk[t - 1][1], pk[t][1], false, false);
          typedef uint32_t v4u32_t __attribute__((ext_vector_type(4)));
          const v4u32_t o = {sx[0], sy[0], sx[1], sy[1]};
          __builtin_amdgcn_raw_buffer_store_b128(o, zr, ok ? (uint32_t)((pix * 64 + 16 * (t - 1 + (g & 1)) + 8 * (g >> 1)) * 2) : BUF_OOB, 0, 0);
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
      // per channel over the tile's 256 pixels (conv_fwd_s2_dma_kernel's order): each wave transposes its column sums
      // through its own LDS corner in image buffer 0 (free: chunk 3 read buffer 1), lane l = channel l adds its 16
      // columns in order; the 8 waves meet in LDS, fixed order, fp64 out
      float* red = (float*)(smem + ST_OFF_X) + wave * (ST_RED / 4);
      float* fin = (float*)(smem + ST_OFF_FIN);
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
        a.bn_part[(long)tile * 2 * 64 + st * 64 + ch] = (double)x;
      }
    }
    lds_barrier();  // buffer 0 / fin / the input region are rewritten by the next tile
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------------------------------------------
// VGG19 conv1_1 of the perceptual loss on its 1 -> 3 channel repeat (perceptual.py:26-31: torch.cat([x, x, x], 1)):
// conv(cat[x, x, x], W) = conv(x, W0 + W1 + W2), a 1-channel conv (+ bias, ReLU).  One launch reads the two fp32 image
// batches directly (rounded to bf16 as the packed NHWC input was) and writes the 64-channel bf16 output at its write
// floor; the 3-channel form ran the generic pointwise kernel on 8-channel pixels (51 TF/s) after two packing passes.
// The summed weight W' = bf16(W0) + bf16(W1) + bf16(W2) -- the per-channel bf16 weights the 3-channel conv (and torch
// autocast) multiply, summed exactly in fp32 -- is split w_hi = bf16(W'), w_lo = bf16(W' - w_hi) into the MFMA's idle
// K slots (9 taps of 32), so the one MFMA per 16 pixels x 16 channels computes the 3-channel conv's products.  (The
// fp32 W0 + W1 + W2 was more accurate at conv1_1 but moved the perceptual loss further from the fp64 oracle: +0.55 %
// against +0.19 %, an L1 of bf16-noisy features on a 4-image test; tools/diag_c11.py.)
// Workgroup: 16 x 64 output pixels; the 18 x 66 input region goes to LDS (bf16), then an im2col image (taps 0..7 as
// 16 B, tap 8 as 2 B per pixel); wave w computes rows 4w .. 4w + 3, 4 fragments of 16 pixels each, 4 MFMAs per
// fragment (16 channels each), and stores each pixel's 128 contiguous bytes as two 64-B chunk pairs of 16-B stores
// (channel groups traded between lane rows g, g ^ 1 by v_permlane16_swap).
constexpr int C11_TR = 16, C11_TC = 64, C11_IR = C11_TR + 2, C11_IC = C11_TC + 2;
constexpr int C11_NP = C11_TR * C11_TC;                               // 1024 output pixels per tile
constexpr int C11_OFF_IC = (C11_IR * C11_IC * 2 + 15) / 16 * 16;     // im2col image after the input region
constexpr int C11_OFF_T8 = C11_OFF_IC + C11_NP * 16;
constexpr int C11_LDS = C11_OFF_T8 + C11_NP * 2;                      // 20,832 B

struct C11Args {
  const float* xa;
  const float* xb;
  const float* wt;    // [64][3][3][3] fp32 (OIHW)
  const float* bias;  // [64]
  uint16_t* y;        // [2 n_half][h][w][64] bf16
  int n_half, h, w, tiles_x, tiles_y;
  uint32_t y_bytes;
};

__global__ __launch_bounds__(256) void vgg_conv1_1_kernel(C11Args a) {
  __shared__ __attribute__((aligned(16))) char smem[C11_LDS];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, col = lane & 15;
  const int tile = blockIdx.x, tx = tile % a.tiles_x, ty = (tile / a.tiles_x) % a.tiles_y, img = tile / (a.tiles_x * a.tiles_y);
  const int oy0 = C11_TR * ty, ox0 = C11_TC * tx;
  const float* src = img < a.n_half ? a.xa + (long)img * a.h * a.w : a.xb + (long)(img - a.n_half) * a.h * a.w;
  // the input region (zeros outside the image: conv1_1's padding), bf16 RNE
  uint16_t* in = (uint16_t*)smem;
  for (int u = tid; u < C11_IR * C11_IC; u += 256) {
    const int r = u / C11_IC, c = u - r * C11_IC, iy = oy0 - 1 + r, ix = ox0 - 1 + c;
    const float v = iy >= 0 && iy < a.h && ix >= 0 && ix < a.w ? src[(long)iy * a.w + ix] : 0.f;
    in[u] = f2bf(v);
  }
  // A fragments (rows 16 c + col): lane groups 0 / 1 = taps 0..7 / tap 8 of w_hi, 2 / 3 the same of w_lo
  bf16x8 A[4];
  float bb[4][4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    bf16x8 v = {};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int t = 8 * (g & 1) + e, co = 16 * c + col;
      const float wf = t < 9 ? ((float)(__bf16)a.wt[(co * 3 + 0) * 9 + t] + (float)(__bf16)a.wt[(co * 3 + 1) * 9 + t]) +
                                   (float)(__bf16)a.wt[(co * 3 + 2) * 9 + t]
                             : 0.f;
      const __bf16 hi = (__bf16)wf;
      v[e] = g < 2 ? hi : (__bf16)(wf - (float)hi);
    }
    A[c] = v;
#pragma unroll
    for (int e = 0; e < 4; ++e) bb[c][e] = a.bias[16 * c + 4 * g + e];
  }
  __syncthreads();
  // im2col: output pixel p = (r, c) of the tile -> taps 0..7 (16 B at 16 p), tap 8 (2 B)
  for (int p = tid; p < C11_NP; p += 256) {
    const int r = p / C11_TC, c = p - r * C11_TC;
    const uint16_t* q = in + r * C11_IC + c;
    uint4 v;
    v.x = (uint32_t)q[0] | ((uint32_t)q[1] << 16);
    v.y = (uint32_t)q[2] | ((uint32_t)q[C11_IC] << 16);
    v.z = (uint32_t)q[C11_IC + 1] | ((uint32_t)q[C11_IC + 2] << 16);
    v.w = (uint32_t)q[2 * C11_IC] | ((uint32_t)q[2 * C11_IC + 1] << 16);
    *(uint4*)(smem + C11_OFF_IC + 16 * p) = v;
    *(uint16_t*)(smem + C11_OFF_T8 + 2 * p) = q[2 * C11_IC + 2];
  }
  __syncthreads();
  const __amdgpu_buffer_rsrc_t yr = buf_rsrc(a.y, a.y_bytes);
  typedef uint32_t v4u32_t __attribute__((ext_vector_type(4)));
#pragma unroll 2
  for (int fr = 0; fr < 16; ++fr) {  // this wave's fragments: row 4 wave + fr / 4, columns 16 (fr % 4) ..
    const int r = 4 * wave + (fr >> 2), c = 16 * (fr & 3) + col, p = r * C11_TC + c;
    const uint4 t07 = *(const uint4*)(smem + C11_OFF_IC + 16 * p);
    const uint16_t t8 = *(const uint16_t*)(smem + C11_OFF_T8 + 2 * p);
    const bf16x8 B = __builtin_bit_cast(bf16x8, (g & 1) == 0 ? t07 : make_uint4((uint32_t)t8, 0, 0, 0));
    f32x4 z[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) z[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[k], B, (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    const int oy = oy0 + r, ox = ox0 + c;
    const bool ok = oy < a.h && ox < a.w;
    const uint32_t pix = (uint32_t)(((long)img * a.h + oy) * a.w + ox);
    uint32_t pk[4][2];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float v0 = fmaxf(z[k][0] + bb[k][0], 0.f), v1 = fmaxf(z[k][1] + bb[k][1], 0.f);
      const float v2 = fmaxf(z[k][2] + bb[k][2], 0.f), v3 = fmaxf(z[k][3] + bb[k][3], 0.f);
      const bf16x2 q0 = {(__bf16)v0, (__bf16)v1}, q1 = {(__bf16)v2, (__bf16)v3};
      pk[k][0] = __builtin_bit_cast(uint32_t, q0);
      pk[k][1] = __builtin_bit_cast(uint32_t, q1);
      if (k & 1) {  // lane (col, g): channels 16 (k - 1 + (g & 1)) + 8 (g >> 1) .. + 7 of its pixel
        const auto sx = __builtin_amdgcn_permlane16_swap(pk[k - 1][0], pk[k][0], false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(pk[k - 1][1], pk[k][1], false, false);
        const v4u32_t o = {sx[0], sy[0], sx[1], sy[1]};
        __builtin_amdgcn_raw_buffer_store_b128(o, yr, ok ? (pix * 64u + (uint32_t)(16 * (k - 1 + (g & 1)) + 8 * (g >> 1))) * 2u : BUF_OOB, 0, 0);
      }
    }
  }
}

}  // namespace

extern "C" int climsr_d_stem_s2(const ClimsrStemDesc* d, void* stream) {
  if (!d || !d->x || !d->w0 || !d->w2 || !d->z2 || d->n <= 0 || d->h <= 0 || d->w <= 0 || d->x_cs <= 0 || d->x_cs % 8 ||
      d->kpk2 != 2 * 288 || !(d->slope >= 0.f && d->slope <= 1.f)) {
    set_error("d_stem_s2: bad args");
    return CLIMSR_EINVAL;
  }
  const long px = (long)d->n * d->h * d->w, opx = (long)d->n * ((d->h + 1) / 2) * ((d->w + 1) / 2);
  if (px * d->x_cs * 2 >= (1L << 31) || px * 64 * 2 >= (1L << 31) || opx * 64 * 2 >= (1L << 31)) {
    set_error("d_stem_s2: tensors over 2 GiB (32-bit buffer offsets)");
    return CLIMSR_EINVAL;
  }
  StemArgs a{};
  a.x = d->x; a.w0 = d->w0; a.w2 = d->w2; a.a0 = d->a0; a.z2 = d->z2; a.bn_part = d->bn_part;
  a.x_cs = d->x_cs; a.kpk2 = d->kpk2; a.n = d->n; a.h = d->h; a.w = d->w;
  a.oh = (d->h + 1) / 2; a.ow = (d->w + 1) / 2;
  a.tiles_x = ceil_div(a.ow, 16); a.tiles_y = ceil_div(a.oh, 16);
  a.slope = d->slope;
  a.x_bytes = (uint32_t)(px * d->x_cs * 2); a.a0_bytes = (uint32_t)(px * 64 * 2); a.z_bytes = (uint32_t)(opx * 64 * 2);
  void (*k)(StemArgs) = d->bn_part ? (d->a0 ? stem_s2_kernel<true, true> : stem_s2_kernel<true, false>)
                                   : (d->a0 ? stem_s2_kernel<false, true> : stem_s2_kernel<false, false>);
  if (int e = lds_opt_in((const void*)k, ST_LDS)) return e;
  const int ntile = a.tiles_x * a.tiles_y * a.n;
  const int grid = ntile < device_cus() ? ntile : device_cus();
  hipLaunchKernelGGL(k, dim3(grid), dim3(512), ST_LDS, (hipStream_t)stream, a);
  return check_launch("d_stem_s2");
}

extern "C" int64_t climsr_d_stem_s2_bn_parts(int32_t n, int32_t h, int32_t w) {
  return (int64_t)n * ((((h + 1) / 2) + 15) / 16) * ((((w + 1) / 2) + 15) / 16);
}

extern "C" int climsr_vgg_conv1_1(const float* xa, const float* xb, int n_half, int h, int w, const float* weight, const float* bias,
                                  uint16_t* y, void* stream) {
  if (!xa || !xb || !weight || !bias || !y || n_half <= 0 || h <= 0 || w <= 0) {
    set_error("vgg_conv1_1: bad args");
    return CLIMSR_EINVAL;
  }
  const long ybytes = 2L * n_half * h * w * 64 * 2;
  if (ybytes >= (1L << 31)) {
    set_error("vgg_conv1_1: output over 2 GiB (32-bit buffer offsets)");
    return CLIMSR_EINVAL;
  }
  C11Args a{};
  a.xa = xa; a.xb = xb; a.wt = weight; a.bias = bias; a.y = y;
  a.n_half = n_half; a.h = h; a.w = w;
  a.tiles_x = ceil_div(w, C11_TC); a.tiles_y = ceil_div(h, C11_TR);
  a.y_bytes = (uint32_t)ybytes;
  hipLaunchKernelGGL(vgg_conv1_1_kernel, dim3(a.tiles_x * a.tiles_y * 2 * n_half), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("vgg_conv1_1");
}
