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
// Nothing else is stored: the backward (srcnn_bwd_kernel below) recomputes relu(conv1) / relu(conv2).
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
constexpr int NFRAG_ALL = NFRAG + 4 + 2;      // + the backward's: conv2^T 4, conv3^T 2
constexpr int NLD = (SI * SI + 255) / 256;    // footprint loads per thread (8 B each)
static_assert(S_LDS <= 160 * 1024, "srcnn LDS");
static_assert(Q_BYTES % 16 == 0, "footprint alignment");

struct SrcnnArgs {
  const uint16_t* x;      // bf16 NHWC, channels x_co .. x_co + 3 used
  const uint16_t* wpk;    // NFRAG_ALL x 64 lanes x 8 bf16
  const float *b1, *b2, *b3;
  float* out;             // fp32 [n][h][w] (= NCHW with one channel)
  int n, h, w, x_cs, x_co;
  int tiles_x, tiles_y, ntiles;
  uint32_t x_bytes, out_bytes;
};

typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void pad_mfma2(f32x4& c0, f32x4& c1) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+v"(c0), "+v"(c1));
}

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  const bf16x2 p = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, p);
}

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

    // groups in pairs (gi, gi + 4): the two groups' conv1 chains interleave, so each k block's two B reads are covered
    // by eight MFMAs (one wave per SIMD: nothing else hides the LDS latency); a wave's odd last group pairs with itself
    auto finish = [&](int gi, f32x4 (&c1)[4]) {
      const int gy = gi / SGX, gx = gi - gy * SGX;
      const int ry = 4 * gy + (col >> 2), rx = 4 * gx + (col & 3);
      // ---- bias + ReLU -> conv2's B fragments (k block s2: co blocks 2 s2, 2 s2 + 1)
      const int yy = oy0 - 2 + ry, xx = ox0 - 2 + rx;
      const bool inimg = yy >= 0 && yy < a.h && xx >= 0 && xx < a.w;
      uint32_t u1[4][2];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = fmaxf(c1[b][i] + bias1[b][i], 0.f);
        u1[b][0] = pack2(v[0], v[1]);
        u1[b][1] = pack2(v[2], v[3]);
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
    };
    for (int ga = wv; ga < SG; ga += 8) {
      const int gb = ga + 4 < SG ? ga + 4 : ga;
      const char* xa = xin + ((4 * (ga / SGX) + (col >> 2)) * SI + 4 * (ga % SGX) + (col & 3)) * 8;
      const char* xq = xin + ((4 * (gb / SGX) + (col >> 2)) * SI + 4 * (gb % SGX) + (col & 3)) * 8;
      // ---- conv1 of both groups: 4 co blocks x 11 k blocks each, B double-buffered one k block ahead
      f32x4 ca[4], cb[4];
      bf16x8 ba[2], bb[2];
      auto ldb = [&](const char* xb, int s) {
        const v2u32 lo = *(const v2u32*)(xb + toff[s][0]);
        const v2u32 hi = *(const v2u32*)(xb + toff[s][1]);
        const uint32_t u[4] = {lo[0], lo[1], hi[0], hi[1]};
        return __builtin_bit_cast(bf16x8, u);
      };
      ba[0] = ldb(xa, 0);
      bb[0] = ldb(xq, 0);
#pragma unroll
      for (int s = 0; s < NK1; ++s) {
        if (s + 1 < NK1) {
          ba[(s + 1) & 1] = ldb(xa, s + 1);
          bb[(s + 1) & 1] = ldb(xq, s + 1);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (s == 0) {
          mfma4x_agpr<true, false>(ca[0], ca[1], ca[2], ca[3], a1[0][s], a1[1][s], a1[2][s], a1[3][s], ba[0]);
          mfma4x_agpr<true, false>(cb[0], cb[1], cb[2], cb[3], a1[0][s], a1[1][s], a1[2][s], a1[3][s], bb[0]);
        } else {
          mfma4x_agpr<false, false>(ca[0], ca[1], ca[2], ca[3], a1[0][s], a1[1][s], a1[2][s], a1[3][s], ba[s & 1]);
          mfma4x_agpr<false, false>(cb[0], cb[1], cb[2], cb[3], a1[0][s], a1[1][s], a1[2][s], a1[3][s], bb[s & 1]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      pad_mfma(ca);
      pad_mfma(cb);
      finish(ga, ca);
      if (gb != ga) finish(gb, cb);
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

// ------------------------------------------------------------------------------------------
// Backward of the tail below conv1 (srcnn.py:13-18 under autograd), recomputing the forward instead of reading
// stored intermediates: per 32 x 32 tile of OWN pixels (no halo recompute: conv1 / conv2 outputs are needed at the own
// pixels only), per group of 4 x 4 pixels
//   s1 = relu(conv1(x)), s2 = relu(conv2(s1))                    (the forward's two chains, same packing)
//   dA2 = conv3^T(g)  [32 ch]  = W3^T x G, G[tap][px] = g(px - tap + 2) gathered from the tile's gout image (bf16)
//   dZ2 = dA2 * (s2 > 0)  ->  dA1 = W2^T dZ2 [64 ch]  ->  dZ1 = dA1 * (s1 > 0), stored bf16 (conv1's gradients read it)
// and the weight gradients of conv2 / conv3 over the own pixels, two groups (32 pixels = one MFMA k block) at a time
// from a wave-private LDS staging of [pixel][channel] rows read back transposed (ds_read_tr16_b64):
//   dW2[co][ci] += dZ2^T s1,  db2 += dZ2^T 1,  dW3[c][tap] += s2^T G,  db3 += sum g (= 1^T G at the centre tap)
// Per-workgroup partial gradients go to a workspace slab, summed over the workgroups in a fixed order by
// srcnn_bwd_reduce_kernel (deterministic).  g outside the image and pixels outside it contribute zeros (conv3's
// zero padding of its input, the image border).
// ------------------------------------------------------------------------------------------
constexpr int BT = 32;                         // own tile side
constexpr int BI = BT + 8;                     // conv1 input footprint: 40
constexpr int BGO = BT + 4;                    // gout image side (halo 2): 36
constexpr int BGX = BT / 4;                    // 4 x 4 groups per tile row: 8 (64 groups, 16 per wave)
constexpr int B_IN = BI * BI * 8;              // footprint bytes (12,800)
constexpr int B_GO = (BGO * BGO * 2 + 15) / 16 * 16;  // gout image bytes, bf16 (2,592)
constexpr int S1P = 64 + 8, S2P = 32 + 8;      // staging pitches (bf16)
constexpr int B_STG = 32 * (S1P + 2 * S2P) * 2;  // per wave: s1 [32][72] + dZ2 [32][40] + s2 [32][40] (9,728)
constexpr int NPART = 32 * 64 + 32 + 32 * NTAP3 + 1;  // dW2, db2, dW3, db3
constexpr int NPART_P = (NPART + 3) / 4 * 4;
constexpr int B_LDS = B_IN + B_GO + 4 * B_STG; // 54,304 (the per-wave partial sums alias it at the end: 4 x NPART_P x 4)
constexpr int B_LDS_ALL = B_LDS + 96 * 4;      // + the conv1 / conv2 biases
constexpr int NLDB = (BI * BI + 255) / 256, NLDG = (BGO * BGO + 255) / 256;
static_assert(4 * NPART_P * 4 <= B_LDS, "srcnn bwd partial staging");

struct SrcnnBwdArgs {
  const uint16_t* x;      // the tail input (as the forward)
  const float* gout;      // fp32 [n][h][w]
  const uint16_t* wpk;
  const float *b1, *b2;
  uint16_t* dz1;          // bf16 [n][h][w][64]
  float* part;            // [gridDim.x][NPART_P]
  int n, h, w, x_cs, x_co;
  int tiles_x, tiles_y, ntiles;
  uint32_t x_bytes, g_bytes, dz1_bytes;
};

// (the weight-gradient accumulators live in AGPRs for the whole launch, beside conv1's weights: "+a")
// acc[co block][ci block] += A[co] B[ci] for the two dZ2 fragments x four s1 fragments, and the db2 sums (B = ones)
__device__ __forceinline__ void mfma_dw2(f32x4 (&acc)[2][4], f32x4 (&accb)[2], const bf16x8 (&a)[2], const bf16x8 (&b)[4],
                                         const bf16x8& ones) {
  asm volatile(
      "s_nop 3\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %10, %12, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %1, %10, %13, %1\n\t"
      "v_mfma_f32_16x16x32_bf16 %2, %10, %14, %2\n\t"
      "v_mfma_f32_16x16x32_bf16 %3, %10, %15, %3\n\t"
      "v_mfma_f32_16x16x32_bf16 %4, %11, %12, %4\n\t"
      "v_mfma_f32_16x16x32_bf16 %5, %11, %13, %5\n\t"
      "v_mfma_f32_16x16x32_bf16 %6, %11, %14, %6\n\t"
      "v_mfma_f32_16x16x32_bf16 %7, %11, %15, %7\n\t"
      "v_mfma_f32_16x16x32_bf16 %8, %10, %16, %8\n\t"
      "v_mfma_f32_16x16x32_bf16 %9, %11, %16, %9"
      : "+a"(acc[0][0]), "+a"(acc[0][1]), "+a"(acc[0][2]), "+a"(acc[0][3]), "+a"(acc[1][0]), "+a"(acc[1][1]),
        "+a"(acc[1][2]), "+a"(acc[1][3]), "+a"(accb[0]), "+a"(accb[1])
      : "v"(a[0]), "v"(a[1]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(ones));
}
// acc[c block][tap block] += A[c] B[tap] (s2 fragments x G fragments), accd += ones x G[0] (db3 at the centre tap)
__device__ __forceinline__ void mfma_dw3(f32x4 (&acc)[2][2], f32x4& accd, const bf16x8 (&a)[2], const bf16x8 (&b)[2],
                                         const bf16x8& ones) {
  asm volatile(
      "s_nop 3\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %5, %7, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %1, %5, %8, %1\n\t"
      "v_mfma_f32_16x16x32_bf16 %2, %6, %7, %2\n\t"
      "v_mfma_f32_16x16x32_bf16 %3, %6, %8, %3\n\t"
      "v_mfma_f32_16x16x32_bf16 %4, %9, %7, %4"
      : "+a"(acc[0][0]), "+a"(acc[0][1]), "+a"(acc[1][0]), "+a"(acc[1][1]), "+a"(accd)
      : "v"(a[0]), "v"(a[1]), "v"(b[0]), "v"(b[1]), "v"(ones));
}
__device__ __forceinline__ void pad_dw(f32x4 (&d2)[2][4], f32x4 (&b2)[2], f32x4 (&d3)[2][2], f32x4& b3) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3"
               : "+a"(d2[0][0]), "+a"(d2[0][1]), "+a"(d2[0][2]), "+a"(d2[0][3]), "+a"(d2[1][0]), "+a"(d2[1][1]), "+a"(d2[1][2]),
                 "+a"(d2[1][3]), "+a"(b2[0]), "+a"(b2[1]), "+a"(d3[0][0]), "+a"(d3[0][1]), "+a"(d3[1][0]), "+a"(d3[1][1]),
                 "+a"(b3));
}
// c[t] = A[t] B from a literal zero accumulator, the A fragments in VGPRs (conv2^T / conv3^T: the AGPRs are full)
__device__ __forceinline__ void mfma2_first_v(f32x4 (&c)[2], const bf16x8 (&a)[2], const bf16x8& b) {
  asm volatile("s_nop 3\n\tv_mfma_f32_16x16x32_bf16 %0, %2, %4, 0\n\tv_mfma_f32_16x16x32_bf16 %1, %3, %4, 0"
               : "=&v"(c[0]), "=&v"(c[1]) : "v"(a[0]), "v"(a[1]), "v"(b));
}
__device__ __forceinline__ void mfma4_first_v(f32x4 (&c)[4], const bf16x8 (&a)[4], const bf16x8& b) {
  asm volatile(
      "s_nop 3\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %4, %8, 0\n\t"
      "v_mfma_f32_16x16x32_bf16 %1, %5, %8, 0\n\t"
      "v_mfma_f32_16x16x32_bf16 %2, %6, %8, 0\n\t"
      "v_mfma_f32_16x16x32_bf16 %3, %7, %8, 0"
      : "=&v"(c[0]), "=&v"(c[1]), "=&v"(c[2]), "=&v"(c[3])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(b));
}
__device__ __forceinline__ void pad_mfma4(f32x4 (&c)[4]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]));
}

__global__ __launch_bounds__(256, 1) void srcnn_bwd_kernel(SrcnnBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* xin = smem;
  uint16_t* gimg = (uint16_t*)(smem + B_IN);
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, col = lane & 15, q4 = col >> 2, p4 = col & 3;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  char* stg = smem + B_IN + B_GO + wv * B_STG;
  uint16_t* st1 = (uint16_t*)stg;            // s1 [32 px][S1P]
  uint16_t* stz = st1 + 32 * S1P;            // dZ2 [32 px][S2P]
  uint16_t* st2 = stz + 32 * S2P;            // s2 [32 px][S2P]
  const int G = (int)gridDim.x;
  int T = xcd_major(blockIdx.x, G);

  const bf16x8* wf = (const bf16x8*)a.wpk + lane;
  bf16x8 a1[4][NK1], a2[2][2], a2t[4], a3t[2];
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int s = 0; s < NK1; ++s) a1[b][s] = wf[(b * NK1 + s) * 64];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int s = 0; s < 2; ++s) a2[b][s] = wf[(4 * NK1 + b * 2 + s) * 64];
#pragma unroll
  for (int b = 0; b < 4; ++b) a2t[b] = wf[(NFRAG + b) * 64];
#pragma unroll
  for (int b = 0; b < 2; ++b) a3t[b] = wf[(NFRAG + 4 + b) * 64];
  // biases in LDS (read per group: registers are the scarce resource here); per-thread index math is recomputed where
  // it is used (an empty asm makes its input opaque, so hipcc cannot hoist and keep -- and spill -- it)
  float* bsm = (float*)(smem + B_LDS);
  if (tid < 64) bsm[tid] = a.b1[tid];
  else if (tid < 96) bsm[tid] = a.b2[tid - 64];
  bf16x8 ones;
#pragma unroll
  for (int i = 0; i < 8; ++i) ones[i] = (__bf16)1.0f;
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  f32x4 dw2[2][4], db2[2], dw3[2][2], db3 = z4;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    db2[b] = z4;
#pragma unroll
    for (int c = 0; c < 4; ++c) dw2[b][c] = z4;
#pragma unroll
    for (int c = 0; c < 2; ++c) dw3[b][c] = z4;
  }

  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(a.x, a.x_bytes);
  const __amdgpu_buffer_rsrc_t gr = buf_rsrc(a.gout, a.g_bytes);
  const __amdgpu_buffer_rsrc_t zr = buf_rsrc(a.dz1, a.dz1_bytes);
  auto decode = [&](int tile, int& nimg, int& oy0, int& ox0) {
    const int tx = tile % a.tiles_x, r = tile / a.tiles_x, ty = r % a.tiles_y;
    nimg = r / a.tiles_y;
    oy0 = ty * BT;
    ox0 = tx * BT;
  };
  v2u32 pre[NLDB];
  uint32_t pg[NLDG];
  auto fetch = [&](int tile) {  // footprint (origin own - 4) and gout image (origin own - 2); zeros outside the image
    int nimg = 0, oy0 = -(1 << 20), ox0 = 0;
    if (tile < a.ntiles) decode(tile, nimg, oy0, ox0);
    int t0 = tid;
    asm volatile("" : "+v"(t0));
#pragma unroll
    for (int k = 0; k < NLDB; ++k) {
      const int p = t0 + 256 * k, iy = p / BI, ix = p - iy * BI;
      const int yy = oy0 - 4 + iy, xx = ox0 - 4 + ix;
      const bool ok = p < BI * BI && yy >= 0 && yy < a.h && xx >= 0 && xx < a.w;
      const uint32_t off = ok ? (uint32_t)((((long)nimg * a.h + yy) * a.w + xx) * a.x_cs + a.x_co) * 2u : BUF_OOB;
      pre[k] = __builtin_amdgcn_raw_buffer_load_b64(xr, off, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < NLDG; ++k) {
      const int p = t0 + 256 * k, iy = p / BGO, ix = p - iy * BGO;
      const int yy = oy0 - 2 + iy, xx = ox0 - 2 + ix;
      const bool ok = p < BGO * BGO && yy >= 0 && yy < a.h && xx >= 0 && xx < a.w;
      pg[k] = __builtin_amdgcn_raw_buffer_load_b32(gr, ok ? (uint32_t)((((long)nimg * a.h + yy) * a.w + xx) * 4) : BUF_OOB, 0, 0);
    }
  };

  // transposed staging reads (rows = pixels 4 g + q4 and 16 + 4 g + q4, the MFMA k order; lane col = channel)
  auto tr_frag = [&](const uint16_t* base, int pitch, int c0) {
    const uint16_t* p0 = base + (4 * g + q4) * pitch + c0 + 4 * p4;
    return cat_tr(ds_read_tr16(p0), ds_read_tr16(p0 + 16 * pitch));
  };

  fetch(T);
  for (; T < a.ntiles; T += G) {
#pragma unroll
    for (int k = 0; k < NLDB; ++k) {
      const int p = tid + 256 * k;
      if (p < BI * BI) *(v2u32*)(xin + p * 8) = pre[k];
    }
#pragma unroll
    for (int k = 0; k < NLDG; ++k) {
      const int p = tid + 256 * k;
      if (p < BGO * BGO) gimg[p] = f2bf(__uint_as_float(pg[k]));
    }
    lds_barrier();
    fetch(T + G);
    int nimg, oy0, ox0;
    decode(T, nimg, oy0, ox0);
    for (int pr = 0; pr < 16; pr += 2) {
      int gyp[2], gxp[2];
#pragma unroll
      for (int ps = 0; ps < 2; ++ps) {
        const int gi = wv + 4 * (pr + ps);
        gyp[ps] = gi / BGX;
        gxp[ps] = gi - gyp[ps] * BGX;
      }
      // ---- recompute conv1 at both groups' pixels, the two chains interleaved (8 MFMAs cover each k block's reads)
      int g2 = 2 * g;
      asm volatile("" : "+v"(g2));
      auto toff = [&](int s, int hh) {  // footprint offset of tap 8 s + 2 g + hh (taps past 80 read tap 80)
        const int t = min(8 * s + g2 + hh, 80), ky = (t * 57) >> 9;  // t / 9 for t < 128
        return (ky * (BI - 9) + t) * 8;
      };
      const char* xa = xin + ((4 * gyp[0] + q4) * BI + 4 * gxp[0] + p4) * 8;
      const char* xq = xin + ((4 * gyp[1] + q4) * BI + 4 * gxp[1] + p4) * 8;
      auto ldb = [&](const char* xb, int s) {
        const v2u32 lo = *(const v2u32*)(xb + toff(s, 0));
        const v2u32 hi = *(const v2u32*)(xb + toff(s, 1));
        const uint32_t u[4] = {lo[0], lo[1], hi[0], hi[1]};
        return __builtin_bit_cast(bf16x8, u);
      };
      f32x4 c1p[2][4];
      bf16x8 ba[2], bb[2];
      ba[0] = ldb(xa, 0);
      bb[0] = ldb(xq, 0);
#pragma unroll
      for (int s = 0; s < NK1; ++s) {
        if (s + 1 < NK1) {
          ba[(s + 1) & 1] = ldb(xa, s + 1);
          bb[(s + 1) & 1] = ldb(xq, s + 1);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (s == 0) {
          mfma4x_agpr<true, false>(c1p[0][0], c1p[0][1], c1p[0][2], c1p[0][3], a1[0][s], a1[1][s], a1[2][s], a1[3][s], ba[0]);
          mfma4x_agpr<true, false>(c1p[1][0], c1p[1][1], c1p[1][2], c1p[1][3], a1[0][s], a1[1][s], a1[2][s], a1[3][s], bb[0]);
        } else {
          mfma4x_agpr<false, false>(c1p[0][0], c1p[0][1], c1p[0][2], c1p[0][3], a1[0][s], a1[1][s], a1[2][s], a1[3][s], ba[s & 1]);
          mfma4x_agpr<false, false>(c1p[1][0], c1p[1][1], c1p[1][2], c1p[1][3], a1[0][s], a1[1][s], a1[2][s], a1[3][s], bb[s & 1]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      pad_mfma(c1p[0]);
      pad_mfma(c1p[1]);
#pragma unroll
      for (int ps = 0; ps < 2; ++ps) {
        const int ry = 4 * gyp[ps] + q4, rx = 4 * gxp[ps] + p4;
        const int yy = oy0 + ry, xx = ox0 + rx;
        const bool inimg = yy < a.h && xx < a.w;
        f32x4 (&c1)[4] = c1p[ps];
        uint32_t u1[4][2];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = fmaxf(c1[b][i] + bsm[16 * b + 4 * g + i], 0.f);
          u1[b][0] = pack2(v[0], v[1]);
          u1[b][1] = pack2(v[2], v[3]);
        }
        bf16x8 b2f[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const uint32_t u[4] = {u1[2 * s][0], u1[2 * s][1], u1[2 * s + 1][0], u1[2 * s + 1][1]};
          b2f[s] = __builtin_bit_cast(bf16x8, u);
        }
        f32x4 c2[2];
        mfma2x_agpr<true, false>(c2[0], c2[1], a2[0][0], a2[1][0], b2f[0]);
        mfma2x_agpr<false, false>(c2[0], c2[1], a2[0][1], a2[1][1], b2f[1]);
        pad_mfma2(c2[0], c2[1]);
        uint32_t u2[2][2];
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = inimg ? fmaxf(c2[b][i] + bsm[64 + 16 * b + 4 * g + i], 0.f) : 0.f;  // conv3's zero padding
          u2[b][0] = pack2(v[0], v[1]);
          u2[b][1] = pack2(v[2], v[3]);
        }
        // ---- dA2 = W3^T G: B element j = g at (ry - ky + 2, rx - kx + 2) for tap 8 g + j (image index + 2)
        bf16x8 bg;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int t = min(8 * g + j, NTAP3 - 1), ky = t / 5, kx = t - ky * 5;
          bg[j] = __builtin_bit_cast(__bf16, gimg[(ry - ky + 4) * BGO + rx - kx + 4]);
        }
        f32x4 d2[2];
        mfma2_first_v(d2, a3t, bg);
        pad_mfma2(d2[0], d2[1]);
        // ---- dZ2 = dA2 * (s2 > 0) (zero outside the image) -> dA1 = W2^T dZ2
        uint32_t uz[2][2];
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t w2 = u2[b][i >> 1];
            const float sv = __uint_as_float((i & 1) ? (w2 & 0xFFFF0000u) : (w2 << 16));
            v[i] = sv > 0.f ? d2[b][i] : 0.f;
          }
          uz[b][0] = pack2(v[0], v[1]);
          uz[b][1] = pack2(v[2], v[3]);
        }
        const uint32_t uzq[4] = {uz[0][0], uz[0][1], uz[1][0], uz[1][1]};
        const bf16x8 bz = __builtin_bit_cast(bf16x8, uzq);
        f32x4 d1[4];
        mfma4_first_v(d1, a2t, bz);
        pad_mfma4(d1);
        // ---- dZ1 = dA1 * (s1 > 0), stored bf16
        const long pix = ((long)nimg * a.h + yy) * a.w + xx;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t w1 = u1[b][i >> 1];
            const float sv = __uint_as_float((i & 1) ? (w1 & 0xFFFF0000u) : (w1 << 16));
            v[i] = sv > 0.f ? d1[b][i] : 0.f;
          }
          const v2u32 pk = {pack2(v[0], v[1]), pack2(v[2], v[3])};
          __builtin_amdgcn_raw_buffer_store_b64(pk, zr, inimg ? (uint32_t)((pix * 64 + 16 * b + 4 * g) * 2) : BUF_OOB, 0, 0);
        }
        // ---- stage this group's rows (pixel 16 ps + col): s1 (zero outside the image), dZ2, s2
        const int row = 16 * ps + col;
#pragma unroll
        for (int b = 0; b < 4; ++b)
          *(v2u32*)(st1 + row * S1P + 16 * b + 4 * g) = inimg ? (v2u32){u1[b][0], u1[b][1]} : (v2u32){0u, 0u};
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          *(v2u32*)(stz + row * S2P + 16 * b + 4 * g) = (v2u32){uz[b][0], uz[b][1]};
          *(v2u32*)(st2 + row * S2P + 16 * b + 4 * g) = (v2u32){u2[b][0], u2[b][1]};
        }
      }
      // ---- weight gradients of the pair (32 pixels): k element j = staged row 4 g + j (j < 4) / 16 + 4 g + j - 4,
      // i.e. group ps = j >> 2's pixel (4 gy + g, 4 gx + (j & 3))
      bf16x8 fz[2], fs1[4], fs2[2], fg[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) fz[b] = tr_frag(stz, S2P, 16 * b);
#pragma unroll
      for (int b = 0; b < 4; ++b) fs1[b] = tr_frag(st1, S1P, 16 * b);
#pragma unroll
      for (int b = 0; b < 2; ++b) fs2[b] = tr_frag(st2, S2P, 16 * b);
#pragma unroll
      for (int b = 0; b < 2; ++b) {  // G[q][tap], tap = 16 b + col (zero past 24), q = the k element's pixel
        const int t = 16 * b + col, tc = min(t, NTAP3 - 1), ky = tc / 5, kx = tc - ky * 5;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int ps = j >> 2, ry = 4 * gyp[ps] + g, rx = 4 * gxp[ps] + (j & 3);
          const uint16_t gv = gimg[(ry - ky + 4) * BGO + rx - kx + 4];
          fg[b][j] = __builtin_bit_cast(__bf16, t < NTAP3 ? gv : (uint16_t)0);
        }
      }
      mfma_dw2(dw2, db2, fz, fs1, ones);
      mfma_dw3(dw3, db3, fs2, fg, ones);
      pad_dw(dw2, db2, dw3, db3);
    }
    lds_barrier();  // every wave is past its reads of the footprint / gout image before the next tile's land
  }
  // ---- the workgroup's partial gradients: per-wave values staged, summed over the 4 waves in a fixed order
  float* pw = (float*)smem + wv * NPART_P;
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = 16 * b + 4 * g + i;
#pragma unroll
      for (int c = 0; c < 4; ++c) pw[co * 64 + 16 * c + col] = dw2[b][c][i];
      if (col == 0) pw[2048 + co] = db2[b][i];
#pragma unroll
      for (int tb = 0; tb < 2; ++tb) {
        const int t = 16 * tb + col;
        if (t < NTAP3) pw[2048 + 32 + co * NTAP3 + t] = dw3[b][tb][i];
      }
    }
  if (lane == 12) pw[NPART - 1] = db3[0];  // row 0, centre tap 12: sum of g over the own pixels
  lds_barrier();
  for (int e = tid; e < NPART; e += 256) {
    const float* ps = (const float*)smem;
    a.part[(long)blockIdx.x * NPART_P + e] = ((ps[e] + ps[NPART_P + e]) + ps[2 * NPART_P + e]) + ps[3 * NPART_P + e];
  }
}

// grads (+)= sum over the workgroup slabs in a fixed order: thread (q, e) sums slabs q, q + 4, .. of element e, the
// four chains then combine in order (one serial chain over every slab took 62 us)
__global__ __launch_bounds__(256) void srcnn_bwd_reduce_kernel(const float* __restrict__ part, int nparts, float* gw2, float* gb2,
                                                               float* gw3, float* gb3, int accumulate) {
  __shared__ float red[4][64];
  const int q = threadIdx.x >> 6, e = blockIdx.x * 64 + (threadIdx.x & 63);
  float s = 0.f;
  if (e < NPART)
    for (int k = q; k < nparts; k += 4) s += part[(long)k * NPART_P + e];
  red[q][threadIdx.x & 63] = s;
  __syncthreads();
  if (q != 0 || e >= NPART) return;
  const int l = threadIdx.x & 63;
  s = ((red[0][l] + red[1][l]) + red[2][l]) + red[3][l];
  float* dst = e < 2048 ? gw2 + e : (e < 2080 ? gb2 + (e - 2048) : (e < NPART - 1 ? gw3 + (e - 2080) : gb3));
  *dst = accumulate ? *dst + s : s;
}

// A fragments in lane order: element e = (f * 64 + lane) * 8 + j, A[row = lane & 15][k = 8 (lane >> 4) + j]
__global__ __launch_bounds__(256) void srcnn_pack_kernel(const float* __restrict__ w1, const float* __restrict__ w2,
                                                         const float* __restrict__ w3, int cin, uint16_t* __restrict__ out) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= NFRAG_ALL * 512) return;
  const int f = e >> 9, lane = (e >> 3) & 63, j = e & 7, r = lane & 15, g = lane >> 4;
  float v = 0.f;
  if (f < 4 * NK1) {  // conv1: co = 16 b + r, k = 32 s + 8 g + j = tap * 4 + channel
    const int b = f / NK1, s = f % NK1, co = 16 * b + r, tap = 8 * s + 2 * g + (j >> 2), c = j & 3;
    if (tap < 81 && c < cin) v = w1[((co * cin + c) * 9 + tap / 9) * 9 + tap % 9];
  } else if (f < 4 * NK1 + 4) {  // conv2: k j of block s2 = conv1 channel 16 (2 s2 + j / 4) + 4 g + j % 4
    const int ff = f - 4 * NK1, b = ff >> 1, s2 = ff & 1, co = 16 * b + r;
    const int ch = 16 * (2 * s2 + (j >> 2)) + 4 * g + (j & 3);
    v = w2[co * 64 + ch];
  } else if (f < NFRAG) {  // Q: rows = conv3 taps 16 b + r, k j = conv2 channel 16 (j / 4) + 4 g + j % 4
    const int b = f - 4 * NK1 - 4, tap = 16 * b + r, ch = 16 * (j >> 2) + 4 * g + (j & 3);
    if (tap < NTAP3) v = w3[ch * NTAP3 + tap];
  } else if (f < NFRAG + 4) {  // conv2^T: rows = conv1 channels 16 b + r, k j = conv2 channel 16 (j / 4) + 4 g + j % 4
    const int b = f - NFRAG, ci = 16 * b + r, co = 16 * (j >> 2) + 4 * g + (j & 3);
    v = w2[co * 64 + ci];
  } else {  // conv3^T: rows = conv2 channels 16 b + r, k = the tap 8 g + j
    const int b = f - NFRAG - 4, c = 16 * b + r, tap = 8 * g + j;
    if (tap < NTAP3) v = w3[c * NTAP3 + tap];
  }
  out[e] = climsr::f2bf(v);
}

}  // namespace

using namespace climsr;

extern "C" int64_t climsr_srcnn_packed_elems(void) { return (int64_t)NFRAG_ALL * 512; }

extern "C" int climsr_srcnn_pack(const float* w1, const float* w2, const float* w3, int in_c, uint16_t* out, void* stream) {
  if (!w1 || !w2 || !w3 || !out || in_c < 1 || in_c > 4) {
    set_error("srcnn_pack: bad args (in_c 1..4)");
    return CLIMSR_EINVAL;
  }
  hipLaunchKernelGGL(srcnn_pack_kernel, dim3(NFRAG_ALL * 2), dim3(256), 0, (hipStream_t)stream, w1, w2, w3, in_c, out);
  return check_launch("srcnn_pack");
}

extern "C" int climsr_srcnn_fwd(const ClimsrSrcnnDesc* d, void* stream) {
  if (!d || !d->x || !d->wpk || !d->b1 || !d->b2 || !d->b3 || !d->out || d->n <= 0 || d->h <= 0 || d->w <= 0 ||
      d->x_cs % 4 || d->x_co % 4 || d->x_co + 4 > d->x_cs) {
    set_error("srcnn_fwd: bad args (x channel stride / offset multiples of 4, offset + 4 <= stride)");
    return CLIMSR_EINVAL;
  }
  const long npx = (long)d->n * d->h * d->w;
  const long xb = npx * d->x_cs * 2;
  if (xb >= (1L << 31)) {
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
  const int grid = std::min(a.ntiles, device_cus());
  if (int e = lds_opt_in((const void*)srcnn_tail_kernel, S_LDS)) return e;
  hipLaunchKernelGGL(srcnn_tail_kernel, dim3(grid), dim3(256), S_LDS, (hipStream_t)stream, a);
  return check_launch("srcnn_fwd");
}

static int srcnn_bwd_grid(int n, int h, int w) {
  const long nt = (long)ceil_div(w, BT) * ceil_div(h, BT) * n;
  return (int)std::min<long>(nt, device_cus());
}

extern "C" int64_t climsr_srcnn_bwd_workspace(int n, int h, int w) {
  if (n <= 0 || h <= 0 || w <= 0) return 0;
  return (int64_t)srcnn_bwd_grid(n, h, w) * NPART_P * 4;
}

extern "C" int climsr_srcnn_bwd(const ClimsrSrcnnBwdDesc* d, void* stream) {
  if (!d || !d->x || !d->gout || !d->wpk || !d->b1 || !d->b2 || !d->dz1 || !d->part || !d->gw2 || !d->gb2 || !d->gw3 ||
      !d->gb3 || d->n <= 0 || d->h <= 0 || d->w <= 0 || d->x_cs % 4 || d->x_co % 4 || d->x_co + 4 > d->x_cs) {
    set_error("srcnn_bwd: bad args (x channel stride / offset multiples of 4, offset + 4 <= stride)");
    return CLIMSR_EINVAL;
  }
  const long npx = (long)d->n * d->h * d->w;
  if (npx * d->x_cs * 2 >= (1L << 31) || npx * 128 >= (1L << 31)) {
    set_error("srcnn_bwd: buffers past 2 GiB (32-bit buffer offsets)");
    return CLIMSR_EINVAL;
  }
  SrcnnBwdArgs a;
  a.x = d->x;
  a.gout = d->gout;
  a.wpk = d->wpk;
  a.b1 = d->b1;
  a.b2 = d->b2;
  a.dz1 = d->dz1;
  a.part = d->part;
  a.n = d->n;
  a.h = d->h;
  a.w = d->w;
  a.x_cs = d->x_cs;
  a.x_co = d->x_co;
  a.tiles_x = ceil_div(d->w, BT);
  a.tiles_y = ceil_div(d->h, BT);
  a.ntiles = a.tiles_x * a.tiles_y * d->n;
  a.x_bytes = (uint32_t)(npx * d->x_cs * 2);
  a.g_bytes = (uint32_t)(npx * 4);
  a.dz1_bytes = (uint32_t)(npx * 128);
  const int grid = srcnn_bwd_grid(d->n, d->h, d->w);
  hipStream_t s = (hipStream_t)stream;
  if (int e = lds_opt_in((const void*)srcnn_bwd_kernel, B_LDS_ALL)) return e;
  hipLaunchKernelGGL(srcnn_bwd_kernel, dim3(grid), dim3(256), B_LDS_ALL, s, a);
  if (int e = check_launch("srcnn_bwd")) return e;
  hipLaunchKernelGGL(srcnn_bwd_reduce_kernel, dim3(ceil_div(NPART, 64)), dim3(256), 0, s, d->part, grid, d->gw2, d->gb2, d->gw3,
                     d->gb3, d->accumulate);
  return check_launch("srcnn_bwd_reduce");
}
