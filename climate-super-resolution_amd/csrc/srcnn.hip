// The SRCNN tail of the ESRGAN generator as ONE launch (CDNA4, gfx950): conv1 9x9 (in_c <= 4 -> 64) + ReLU, conv2
// 1x1 (64 -> 32) + ReLU, conv3 5x5 (32 -> 1) (climsr/models/srcnn.py:9-18) over the generator's
// cat[conv_last(out), elev, mask] (climsr/models/esrgan.py:99-100), with the 64- and 32-channel HR intermediates kept
// on chip.
//
// A workgroup (4 waves, one per SIMD) owns a 32 x 32 output tile at a time.  conv3 needs conv2's output over the
// 36 x 36 region around it, which needs the 44 x 44 input footprint (4 channels x bf16 = 8 B per pixel in LDS).  The
// region is walked in 81 groups of 4 x 4 pixels; per group a wave runs three MFMA chains back to back without leaving
// registers:
//   conv1  C1[64 co][16 px]  = 4 co blocks x 11 k blocks (81 taps x 4 channels, the 4th channel and taps 81..87 carry
//                              zero weights); B = two 8 B LDS reads (two taps x 4 channels) per lane and k block
//   conv2  C2[32 co][16 px]  = 2 co blocks x 2 k blocks; its B fragments are conv1's accumulators after bias + ReLU,
//                              converted in place: the C layout (lane: co 4g..4g+3 of each 16-row block) IS a B layout
//                              once the packed A operand permutes K the same way (srcnn_pack_kernel)
//   conv3  Q[32 taps][16 px] = W3^T x relu(C2): the 25 per-tap partial products of every region pixel (1 k block),
//                              written to LDS in fp32
// and after a barrier each output pixel sums its 25 shifted Q entries in a fixed order (deterministic, fp32) + bias.
// The 44 weight fragments of conv1 (plus conv2's and Q's 6) stay in AGPRs for the launch (mfma_agpr.h).
// LDS: Q 25 x 1300 floats (pitch 1300: the 4 lane groups' tap rows land 16 banks apart) + the footprint.  The next
// tile's footprint is fetched into registers while the current tile computes.
// keep (training): the tile's own pixels of relu(conv1) and relu(conv2) are also stored (bf16 NHWC, 64 / 32 channels)
// for the backward's weight gradients and ReLU masks.
#include <algorithm>
#include <stdio.h>

#include "conv_ep.h"
#include "mfma_agpr.h"

namespace {

constexpr int ST = 32;                        // output tile side
constexpr int SR = ST + 4;                    // region (conv1 / conv2 outputs = conv3 inputs): 36
constexpr int SI = SR + 8;                    // input footprint: 44
constexpr int SGX = SR / 4;                   // 4 x 4-pixel groups per region row: 9
constexpr int SG = SGX * SGX;                 // groups per region: 81
constexpr int NK1 = 11;                       // conv1 k blocks (81 taps x 4 channels = 324 -> 352)
constexpr int NTAP3 = 25;                     // conv3 taps
constexpr int QP = 1300;                      // Q row pitch (floats)
constexpr int Q_BYTES = NTAP3 * QP * 4;       // 130,000
constexpr int IN_BYTES = SI * SI * 8;         // 15,488
constexpr int S_LDS = Q_BYTES + IN_BYTES;     // 145,488
constexpr int NFRAG = 4 * NK1 + 4 + 2;        // packed A fragments: conv1 44, conv2 4, conv3 (Q) 2
constexpr int NLD = (SI * SI + 255) / 256;    // footprint loads per thread (8 B each)
static_assert(S_LDS <= 160 * 1024, "srcnn LDS");
static_assert(Q_BYTES % 16 == 0, "footprint alignment");

struct SrcnnArgs {
  const uint16_t* x;      // bf16 NHWC, channels x_co .. x_co + 3 used
  const uint16_t* wpk;    // NFRAG x 64 lanes x 8 bf16
  const float *b1, *b2, *b3;
  float* out;             // fp32 [n][h][w] (= NCHW with one channel)
  uint16_t* s1;           // keep: relu(conv1) bf16 [n][h][w][64]
  uint16_t* s2;           // keep: relu(conv2) bf16 [n][h][w][32]
  int n, h, w, x_cs, x_co;
  int tiles_x, tiles_y, ntiles;
  uint32_t x_bytes, out_bytes, s1_bytes, s2_bytes;
};

typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void pad_mfma2(f32x4& c0, f32x4& c1) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+v"(c0), "+v"(c1));
}

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  const bf16x2 p = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, p);
}

template <bool KEEP>
__global__ __launch_bounds__(256, 1) void srcnn_tail_kernel(SrcnnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* q = (float*)smem;
  char* xin = smem + Q_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, col = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = (int)gridDim.x;
  int T = xcd_major(blockIdx.x, G);
  if (T >= a.ntiles) return;

  // ---- weights: fragment f, lane l = 16 B at wpk + (f * 64 + l) * 16
  const bf16x8* wf = (const bf16x8*)a.wpk + lane;
  bf16x8 a1[4][NK1], a2[2][2], aq[2];
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int s = 0; s < NK1; ++s) a1[b][s] = wf[(b * NK1 + s) * 64];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int s = 0; s < 2; ++s) a2[b][s] = wf[(4 * NK1 + b * 2 + s) * 64];
#pragma unroll
  for (int b = 0; b < 2; ++b) aq[b] = wf[(4 * NK1 + 4 + b) * 64];
  float bias1[4][4], bias2[2][4];
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int i = 0; i < 4; ++i) bias1[b][i] = a.b1[16 * b + 4 * g + i];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int i = 0; i < 4; ++i) bias2[b][i] = a.b2[16 * b + 4 * g + i];
  const float bias3 = a.b3[0];

  // per-lane footprint offsets (bytes) of k block s: taps 8 s + 2 g and 8 s + 2 g + 1 (taps past 80 read tap 80,
  // under zero weights)
  int toff[NK1][2];
#pragma unroll
  for (int s = 0; s < NK1; ++s)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int t = min(8 * s + 2 * g + hh, 80);
      toff[s][hh] = ((t / 9) * SI + t % 9) * 8;
    }

  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(a.x, a.x_bytes);
  const __amdgpu_buffer_rsrc_t orr = buf_rsrc(a.out, a.out_bytes);
  const __amdgpu_buffer_rsrc_t s1r = buf_rsrc(a.s1, KEEP ? a.s1_bytes : 0u);
  const __amdgpu_buffer_rsrc_t s2r = buf_rsrc(a.s2, KEEP ? a.s2_bytes : 0u);
  auto decode = [&](int tile, int& nimg, int& oy0, int& ox0) {
    const int tx = tile % a.tiles_x, r = tile / a.tiles_x, ty = r % a.tiles_y;
    nimg = r / a.tiles_y;
    oy0 = ty * ST;
    ox0 = tx * ST;
  };
  // footprint pixel p = tid + 256 k: image (oy0 - 6 + p / SI, ox0 - 6 + p % SI); outside the image -> zeros
  v2u32 pre[NLD];
  auto fetch = [&](int tile) {
    int nimg, oy0, ox0;
    decode(tile, nimg, oy0, ox0);
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int p = tid + 256 * k, iy = p / SI, ix = p - iy * SI;
      const int yy = oy0 - 6 + iy, xx = ox0 - 6 + ix;
      const bool ok = p < SI * SI && yy >= 0 && yy < a.h && xx >= 0 && xx < a.w;
      const uint32_t off = ok ? (uint32_t)((((long)nimg * a.h + yy) * a.w + xx) * a.x_cs + a.x_co) * 2u : BUF_OOB;
      pre[k] = __builtin_amdgcn_raw_buffer_load_b64(xr, off, 0, 0);
    }
  };

  fetch(T);
  for (;;) {
    // the footprint of tile T -> LDS.  Every wave has passed the previous tile's Q barrier (its footprint reads are
    // done) and finished its gather before it writes here, and the barrier below orders these writes before any read.
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int p = tid + 256 * k;
      if (p < SI * SI) *(v2u32*)(xin + p * 8) = pre[k];
    }
    lds_barrier();
    const int Tn = T + G;
    if (Tn < a.ntiles) fetch(Tn);
    int nimg, oy0, ox0;
    decode(T, nimg, oy0, ox0);

    for (int gi = wv; gi < SG; gi += 4) {
      const int gy = gi / SGX, gx = gi - gy * SGX;
      const int ry = 4 * gy + (col >> 2), rx = 4 * gx + (col & 3);
      const char* xb = xin + (ry * SI + rx) * 8;
      // ---- conv1: 4 co blocks x 11 k blocks, B double-buffered one k block ahead
      f32x4 c1[4];
      bf16x8 bq[2];
      auto ldb = [&](int s, int buf) {
        const v2u32 lo = *(const v2u32*)(xb + toff[s][0]);
        const v2u32 hi = *(const v2u32*)(xb + toff[s][1]);
        const uint32_t u[4] = {lo[0], lo[1], hi[0], hi[1]};
        bq[buf] = __builtin_bit_cast(bf16x8, u);
      };
      ldb(0, 0);
#pragma unroll
      for (int s = 0; s < NK1; ++s) {
        if (s + 1 < NK1) ldb(s + 1, (s + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
        if (s == 0) mfma4x_agpr<true, false>(c1[0], c1[1], c1[2], c1[3], a1[0][s], a1[1][s], a1[2][s], a1[3][s], bq[0]);
        else mfma4x_agpr<false, false>(c1[0], c1[1], c1[2], c1[3], a1[0][s], a1[1][s], a1[2][s], a1[3][s], bq[s & 1]);
        __builtin_amdgcn_sched_barrier(0);
      }
      pad_mfma(c1);
      // ---- bias + ReLU -> conv2's B fragments (k block s2: co blocks 2 s2, 2 s2 + 1)
      const int yy = oy0 - 2 + ry, xx = ox0 - 2 + rx;
      const bool inimg = yy >= 0 && yy < a.h && xx >= 0 && xx < a.w;
      const bool own = inimg && ry >= 2 && ry < 2 + ST && rx >= 2 && rx < 2 + ST;
      const long pix = ((long)nimg * a.h + yy) * a.w + xx;
      uint32_t u1[4][2];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = fmaxf(c1[b][i] + bias1[b][i], 0.f);
        u1[b][0] = pack2(v[0], v[1]);
        u1[b][1] = pack2(v[2], v[3]);
        if constexpr (KEEP) {
          const v2u32 pk = {u1[b][0], u1[b][1]};
          __builtin_amdgcn_raw_buffer_store_b64(pk, s1r, own ? (uint32_t)((pix * 64 + 16 * b + 4 * g) * 2) : BUF_OOB, 0, 0);
        }
      }
      bf16x8 b2f[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const uint32_t u[4] = {u1[2 * s][0], u1[2 * s][1], u1[2 * s + 1][0], u1[2 * s + 1][1]};
        b2f[s] = __builtin_bit_cast(bf16x8, u);
      }
      // ---- conv2
      f32x4 c2[2];
      mfma2x_agpr<true, false>(c2[0], c2[1], a2[0][0], a2[1][0], b2f[0]);
      mfma2x_agpr<false, false>(c2[0], c2[1], a2[0][1], a2[1][1], b2f[1]);
      pad_mfma2(c2[0], c2[1]);
      uint32_t u2[2][2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = fmaxf(c2[b][i] + bias2[b][i], 0.f);
        u2[b][0] = pack2(v[0], v[1]);
        u2[b][1] = pack2(v[2], v[3]);
        if constexpr (KEEP) {
          const v2u32 pk = {u2[b][0], u2[b][1]};
          __builtin_amdgcn_raw_buffer_store_b64(pk, s2r, own ? (uint32_t)((pix * 32 + 16 * b + 4 * g) * 2) : BUF_OOB, 0, 0);
        }
      }
      const uint32_t uq[4] = {u2[0][0], u2[0][1], u2[1][0], u2[1][1]};
      const bf16x8 bqf = __builtin_bit_cast(bf16x8, uq);
      // ---- conv3's per-tap partial products; conv3 pads its input with zeros: none from outside the image
      f32x4 cq[2];
      mfma2x_agpr<true, false>(cq[0], cq[1], aq[0], aq[1], bqf);
      pad_mfma2(cq[0], cq[1]);
      const int p = ry * SR + rx;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int tap = 16 * b + 4 * g + i;
          if (tap < NTAP3) q[tap * QP + p] = inimg ? cq[b][i] : 0.f;
        }
    }
    lds_barrier();  // Q complete (and every footprint read done)
    // ---- conv3: out(oy, ox) = b3 + sum over taps (ky, kx) of Q[tap][(oy + ky, ox + kx)], fixed order
#pragma unroll
    for (int k = 0; k < ST * ST / 256; ++k) {
      const int ox = tid & (ST - 1), oy = (tid >> 5) + k * (256 / ST);
      float acc = 0.f;
#pragma unroll
      for (int ky = 0; ky < 5; ++ky)
#pragma unroll
        for (int kx = 0; kx < 5; ++kx) acc += q[(ky * 5 + kx) * QP + (oy + ky) * SR + ox + kx];
      const int yy = oy0 + oy, xx = ox0 + ox;
      const bool ok = yy < a.h && xx < a.w;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc + bias3), orr,
                                            ok ? (uint32_t)((((long)nimg * a.h + yy) * a.w + xx) * 4) : BUF_OOB, 0, 0);
    }
    if (Tn >= a.ntiles) break;
    T = Tn;
  }
}

// A fragments in lane order: element e = (f * 64 + lane) * 8 + j, A[row = lane & 15][k = 8 (lane >> 4) + j]
__global__ __launch_bounds__(256) void srcnn_pack_kernel(const float* __restrict__ w1, const float* __restrict__ w2,
                                                         const float* __restrict__ w3, int cin, uint16_t* __restrict__ out) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= NFRAG * 512) return;
  const int f = e >> 9, lane = (e >> 3) & 63, j = e & 7, r = lane & 15, g = lane >> 4;
  float v = 0.f;
  if (f < 4 * NK1) {  // conv1: co = 16 b + r, k = 32 s + 8 g + j = tap * 4 + channel
    const int b = f / NK1, s = f % NK1, co = 16 * b + r, tap = 8 * s + 2 * g + (j >> 2), c = j & 3;
    if (tap < 81 && c < cin) v = w1[((co * cin + c) * 9 + tap / 9) * 9 + tap % 9];
  } else if (f < 4 * NK1 + 4) {  // conv2: k j of block s2 = conv1 channel 16 (2 s2 + j / 4) + 4 g + j % 4
    const int ff = f - 4 * NK1, b = ff >> 1, s2 = ff & 1, co = 16 * b + r;
    const int ch = 16 * (2 * s2 + (j >> 2)) + 4 * g + (j & 3);
    v = w2[co * 64 + ch];
  } else {  // Q: rows = conv3 taps 16 b + r, k j = conv2 channel 16 (j / 4) + 4 g + j % 4
    const int b = f - 4 * NK1 - 4, tap = 16 * b + r, ch = 16 * (j >> 2) + 4 * g + (j & 3);
    if (tap < NTAP3) v = w3[ch * NTAP3 + tap];
  }
  out[e] = climsr::f2bf(v);
}

}  // namespace

using namespace climsr;

extern "C" int64_t climsr_srcnn_packed_elems(void) { return (int64_t)NFRAG * 512; }

extern "C" int climsr_srcnn_pack(const float* w1, const float* w2, const float* w3, int in_c, uint16_t* out, void* stream) {
  if (!w1 || !w2 || !w3 || !out || in_c < 1 || in_c > 4) {
    set_error("srcnn_pack: bad args (in_c 1..4)");
    return CLIMSR_EINVAL;
  }
  hipLaunchKernelGGL(srcnn_pack_kernel, dim3(NFRAG * 2), dim3(256), 0, (hipStream_t)stream, w1, w2, w3, in_c, out);
  return check_launch("srcnn_pack");
}

extern "C" const char* climsr_srcnn_fwd_kernel(const ClimsrSrcnnDesc* d) {
  if (!d) return "";
  return d->s1 ? "srcnn_tail_kernel<true>" : "srcnn_tail_kernel<false>";
}

extern "C" int climsr_srcnn_fwd(const ClimsrSrcnnDesc* d, void* stream) {
  if (!d || !d->x || !d->wpk || !d->b1 || !d->b2 || !d->b3 || !d->out || d->n <= 0 || d->h <= 0 || d->w <= 0 ||
      d->x_cs % 4 || d->x_co % 4 || d->x_co + 4 > d->x_cs || (!d->s1) != (!d->s2)) {
    set_error("srcnn_fwd: bad args (x channel stride / offset multiples of 4, offset + 4 <= stride; s1, s2 both or neither)");
    return CLIMSR_EINVAL;
  }
  const long npx = (long)d->n * d->h * d->w;
  const long xb = npx * d->x_cs * 2, s1b = d->s1 ? npx * 128 : 0;
  if (xb >= (1L << 31) || s1b >= (1L << 31)) {
    set_error("srcnn_fwd: buffers past 2 GiB (32-bit buffer offsets)");
    return CLIMSR_EINVAL;
  }
  SrcnnArgs a;
  a.x = d->x;
  a.wpk = d->wpk;
  a.b1 = d->b1;
  a.b2 = d->b2;
  a.b3 = d->b3;
  a.out = d->out;
  a.s1 = d->s1;
  a.s2 = d->s2;
  a.n = d->n;
  a.h = d->h;
  a.w = d->w;
  a.x_cs = d->x_cs;
  a.x_co = d->x_co;
  a.tiles_x = ceil_div(d->w, ST);
  a.tiles_y = ceil_div(d->h, ST);
  a.ntiles = a.tiles_x * a.tiles_y * d->n;
  a.x_bytes = (uint32_t)xb;
  a.out_bytes = (uint32_t)(npx * 4);
  a.s1_bytes = (uint32_t)s1b;
  a.s2_bytes = (uint32_t)(s1b / 2);
  const int grid = std::min(a.ntiles, device_cus());
  if (d->s1) {
    if (int e = lds_opt_in((const void*)srcnn_tail_kernel<true>, S_LDS)) return e;
    hipLaunchKernelGGL(srcnn_tail_kernel<true>, dim3(grid), dim3(256), S_LDS, (hipStream_t)stream, a);
  } else {
    if (int e = lds_opt_in((const void*)srcnn_tail_kernel<false>, S_LDS)) return e;
    hipLaunchKernelGGL(srcnn_tail_kernel<false>, dim3(grid), dim3(256), S_LDS, (hipStream_t)stream, a);
  }
  return check_launch("srcnn_fwd");
}
