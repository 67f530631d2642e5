// Residual-dense-block chain for images up to 64 columns wide (16, 32, 48, 64): the four 16-output 3x3 convs of an
// RDB in ONE launch (esrgan.py:22-37), forward (conv1..conv4 -> x1..x4) and pull backward (pull4..pull1 -> dZ4..dZ1);
// wider images take rdb_chain.hip's column-windowed kernel.
//
// One workgroup owns R full-width image rows and streams down them, one barrier per step.  Each level ingests one
// input row per step and reuses it for all three kernel rows: the B fragment of (row i, tap column kx) is multiplied
// by the weights of taps (0, kx), (1, kx), (2, kx) into the accumulators of output rows i + 1, i, i - 1 (three rows
// rotate), so a 1 KB fragment read from LDS feeds three MFMAs instead of one -- a level computed one output row at a
// time needs a fresh fragment per MFMA, which is the whole LDS read rate of the CU (1 KB per 16-cycle MFMA per SIMD).
// Output row i - 1 of a level is complete once its row i is in; it goes through the epilogue into that level's LDS ring
// and, for the strip's own rows, to HBM.  Level L + 1 ingests that row in the next step, so level L ingests row
// r0 - 2 - 2L + s in step s.  Only the rows the next levels consume are computed: level L finishes rows
// [r0 - 4 + L, r1 + 4 - L) (3 + 2 + 1 halo rows above / below a strip are recomputed by its neighbours).
// LDS: an 8-row ring of the base (64 ch, 160 B pixel pitch: the 16 lanes of each ds_read_b128 bank group cover the 64
// banks once) filled by LDS-DMA one step ahead, and rings of the level outputs x1 / x2 / x3 (16 ch, 32 B pitch; 6 / 4
// / 2 rows: the steps until their last reader).
// Eight waves, two per SIMD: wave w < 4 computes level w + 1, wave w >= 4 level 8 - w (each SIMD pairs a light and a
// heavy level: 36 + 66 / 48 + 54 MFMAs per row); waves 0-3 cover column fragments 0, 1 and waves 4-7 fragments 2, 3.
// A wave keeps its level's A fragments (16 co x 32 k: 18 base + 6 / 9 / 15 dense per level) in registers for the
// launch.  Dense blocks: x1 | x2 of one tap in one block, a 16-channel group alone as a PAIR of tap columns (lanes
// 0-31 column a, 32-63 column b; the third column pairs with zero weights).
// MFMA v_mfma_f32_16x16x32_bf16: A = weights [16 co][32 k], B = [32 k][16 pixels], C lane = 4 co of one pixel.
#include "common.h"

using namespace climsr;


namespace {

struct ChainArgs {
  const uint16_t* base;
  int bcs, boff;
  uint16_t* out;
  int ocs;
  int ooff[4];
  const uint16_t* wt[4];  // packed [16][9*KP_L], k = tap*KP_L + channel (base | out1 | out2 | out3)
  const float* bias[4];
  const uint16_t* mask;
  int mcs;
  int moff[4];
  float slope;
  int n, h, w, rows, strips_y;
  uint32_t base_bytes, mask_bytes, out_bytes;
};
typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));

// 32-channel blocks of a level's packed K row (KP = 64 + 16 (L - 1) rounded up to 32)
__host__ __device__ constexpr int kp_blocks(int L) { return L == 1 ? 2 : (L == 4 ? 4 : 3); }

constexpr int RR_PX = 66;                               // pixel slots per row: image columns -1 .. 64
constexpr int RR_BP = 160;                              // base pixel pitch: 64 ch + 32 B pad (10 units of 16 B)
constexpr int RR_BNI = (RR_PX * 10 + 63) / 64;          // base-row DMA instructions (11)
constexpr int RR_BSLOT = RR_BNI * 1024;                 // 11,264 B per base row (whole DMA instructions)
constexpr int RR_NB = 9;                                // base ring rows (requested two steps ahead, read until L4)
constexpr int RR_DP = 32;                               // dense pixel pitch (16 ch)
constexpr int RR_DROW = RR_PX * RR_DP;                  // 2,112 B
constexpr int RR_N1 = 6, RR_N2 = 4, RR_N3 = 2;          // x1 / x2 / x3 ring rows
constexpr int RR_OFF_D = RR_NB * RR_BSLOT;              // 90,112
constexpr int RR_OFF_2 = RR_OFF_D + RR_N1 * RR_DROW, RR_OFF_3 = RR_OFF_2 + RR_N2 * RR_DROW;
constexpr int RR_OFF_DUMMY = RR_OFF_3 + RR_N3 * RR_DROW;  // one KB the padding DMA pieces write (zeros, never read)
constexpr int RR_LDS = RR_OFF_DUMMY + 1024;             // 127,744 B
constexpr int RR_K = 2;                                 // base-row DMA pieces per wave (11 real + 5 padding)

__device__ __forceinline__ uint32_t pack2_bf16(float a, float b) {
  const bf16x2 v = {(__bf16)a, (__bf16)b};  // v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(uint32_t, v);
}

// dense block groups per kernel row of level L (see the file comment)
__host__ __device__ constexpr int rr_nd(int L) { return L == 1 ? 0 : (L == 2 ? 2 : (L == 3 ? 3 : 5)); }

// One wave's whole strip walk: level L, column fragments 2 fp and 2 fp + 1.  Every wave runs the same steps (base-row
// DMA + one barrier each).  MODE 0: forward (bias + leaky relu); 1: pull (leaky-relu derivative of the stored
// activation, no bias).
template <int MODE, int L>
__device__ __forceinline__ void run_level(const ChainArgs& a, char* smem, int tid, int nimg, int r0, int r1) {
  constexpr int ND = rr_nd(L), NG = 6 + ND, KP = kp_blocks(L) * 32;
  const int lane = tid & 63, g = lane >> 4, col = lane & 15;
  const int wvu = __builtin_amdgcn_readfirstlane(tid >> 6), fp = wvu >> 2;
  const bool live0 = 32 * fp < a.w, live1 = 32 * fp + 16 < a.w;
  const __amdgpu_buffer_rsrc_t br = buf_rsrc(a.base, a.base_bytes);
  const __amdgpu_buffer_rsrc_t mr = buf_rsrc(a.mask, MODE == 1 ? a.mask_bytes : 0u);
  const __amdgpu_buffer_rsrc_t orr = buf_rsrc(a.out, a.out_bytes);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;

  // base-row DMA: instructions wvu and wvu + 8 (< 11); lane -> 16-B unit 64 k + lane = (pixel slot p, chunk j < 8)
  uint32_t po[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int k = wvu + 8 * j, u = 64 * k + lane, p = u / 10, jj = u - 10 * p, ix = p - 1;
    po[j] = (k < RR_BNI && jj < 8 && p < RR_PX && ix >= 0 && ix < a.w) ? (uint32_t)((ix * a.bcs + a.boff + 8 * jj) * 2) : BUF_OOB;
  }
  const uint32_t brow = (uint32_t)a.w * (uint32_t)a.bcs * 2u;
  // base row `row` into ring slot (row - r0 + 4) % 9; every wave issues exactly RR_K pieces (rows outside the strip's
  // range or the image, and pieces past the 11th, read out of range into the dummy KB)
  auto dma_row = [&](int row) {
    const bool ok = row >= r0 - 4 && row <= r1 + 3 && row >= 0 && row < a.h;
    const uint32_t rb = ok ? (uint32_t)(nimg * a.h + row) * brow : 0u;
    const uint32_t slot = lds0 + (uint32_t)((ok ? (row - r0 + 4) % RR_NB : 0) * RR_BSLOT);
#pragma unroll
    for (int j = 0; j < RR_K; ++j) {
      const bool real = ok && wvu + 8 * j < RR_BNI;
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds ; dma-lag 2\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(real && po[j] != BUF_OOB ? po[j] + rb : BUF_OOB), "s"(br),
                     "s"(real ? slot + (uint32_t)((wvu + 8 * j) * 1024) : lds0 + (uint32_t)RR_OFF_DUMMY)
                   : "memory");
    }
  };

  // A fragments: base [ky][kx][cb] (fragment 6 ky + 2 kx + cb) and dense [ky][d] (fragment 18 + ND ky + d) from the
  // packed [16][9 KP] weights (k = tap KP + channel: base | out1 | out2 | out3 at channels 0 / 64 / 80 / 96), staged
  // through LDS once per workgroup: the level's two waves move its fragments by LDS-DMA (one lane-linear 1 KB piece
  // each, into the ring space before the rings are used) and both read all of them.  Loaded straight from global
  // memory, every wave fetched its level's whole weight set: 2 x 110 KB per CU ahead of the first MFMA.
  constexpr int NF = 18 + 3 * ND, PB = L == 1 ? 0 : (L == 2 ? 18 : (L == 3 ? 42 : 69));  // fragments, first piece
  static_assert((69 + 33) * 1024 <= RR_OFF_DUMMY, "chain weight staging fits the ring space");
  {
    const __amdgpu_buffer_rsrc_t wrs = buf_rsrc(a.wt[L - 1], (uint32_t)(16 * 9 * KP * 2));
    for (int f = fp; f < NF; f += 2) {
      int ky, kx, ch;
      bool zero = false;
      if (f < 18) {
        ky = f / 6;
        kx = (f % 6) >> 1;
        ch = (f & 1) * 32 + 8 * g;
      } else {
        const int e = f - 18, d = e % (ND > 0 ? ND : 1);
        ky = e / (ND > 0 ? ND : 1);
        if (L == 2 || d >= 3) {  // a 16-channel group (x1 at level 2, x3 at level 4) as a pair of tap columns
          const int pr = L == 2 ? d : d - 3;
          kx = pr == 0 ? (g < 2 ? 0 : 1) : 2;
          zero = pr == 1 && g >= 2;
          ch = (L == 2 ? 64 : 96) + 8 * (g & 1);
        } else {  // x1 | x2 of tap column d
          kx = d;
          ch = 64 + 8 * g;
        }
      }
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(zero ? BUF_OOB : (uint32_t)((col * 9 * KP + (3 * ky + kx) * KP + ch) * 2)), "s"(wrs),
                     "s"(lds0 + (uint32_t)((PB + f) * 1024))
                   : "memory");
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();  // every level's pieces have landed
  bf16x8 Ab[3][3][2], Ad[3][ND > 0 ? ND : 1];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) Ab[ky][kx][cb] = *(const bf16x8*)(smem + (PB + 6 * ky + 2 * kx + cb) * 1024 + lane * 16);
#pragma unroll
    for (int d = 0; d < ND; ++d) Ad[ky][d] = *(const bf16x8*)(smem + (PB + 18 + ND * ky + d) * 1024 + lane * 16);
  }
  lds_barrier();  // every wave's reads are done: the rings may be written
  // the level-output rings start zeroed: their pixel slots of image columns -1 and >= w are never written (padding)
  for (int i = tid; i < (RR_LDS - RR_OFF_D) / 16; i += 512) *(uint4*)(smem + RR_OFF_D + 16 * i) = make_uint4(0, 0, 0, 0);
  float bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // channels 8 (g >> 1) .. + 7 (the epilogue's traded layout)
  if constexpr (MODE == 0) {
    const float4 b0 = *(const float4*)(a.bias[L - 1] + 8 * (g >> 1)), b1 = *(const float4*)(a.bias[L - 1] + 8 * (g >> 1) + 4);
    bb[0] = b0.x; bb[1] = b0.y; bb[2] = b0.z; bb[3] = b0.w; bb[4] = b1.x; bb[5] = b1.y; bb[6] = b1.z; bb[7] = b1.w;
  }
  // per-lane LDS offsets: base pixel slot col (+ 16 f + kx), chunk 4 cb + g; dense pixel slot col (+ ...), chunk g & 1
  const int lb = col * RR_BP + g * 16;
  const int ldn = col * RR_DP + (g & 1) * 16;
  // completed-row epilogue, after the fragment halves are traded between lane rows g and g ^ 1 (v_permlane16_swap):
  // lane (col, g) holds channels 8 (g >> 1) .. + 7 of fragment g & 1's pixel col -- one 16-B ring store (slot 1 + the
  // pixel) and one 16-B HBM row store
  const int fq = g & 1;
  const bool liveq = fq == 0 ? live0 : live1;
  const int dl = (1 + 32 * fp + 16 * fq + col) * RR_DP + (g >> 1) * 16;
  const int ol = (32 * fp + 16 * fq + col) * a.ocs + a.ooff[L - 1] + 8 * (g >> 1);
  const int ml = (32 * fp + 16 * fq + col) * a.mcs + a.moff[L - 1] + 8 * (g >> 1);  // (the traded layout, as ol)
  const uint32_t orow = (uint32_t)a.w * (uint32_t)a.ocs * 2u, mrow = (uint32_t)a.w * (uint32_t)a.mcs * 2u;

  // Per step every wave issues, in this order: the pull's mask load (the activation of the row it finishes two steps
  // later, when that row is one the level finishes), RR_K DMA pieces (the base row level 1 ingests two steps later)
  // and, on the steps that finish one of the strip's own rows, one row store.  Step s needs the DMA of step s - 2;
  // younger are step s - 2's store and step s - 1's operations: at least RR_K of them, so that is what the wait leaves.
  constexpr int NW = RR_K;
  f32x4 acc[3][2];  // accumulator row of output row y: (y - r0) mod 3 (phase-resolved at compile time)
#pragma unroll
  for (int r = 0; r < 3; ++r) acc[r][0] = acc[r][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  v4u32 msk[3];  // pull: this lane's 8 channels of the stored activation of the row finished in step s, loaded in
                 // step s - 2 (set s mod 3; traded layout)
  // rows of this level: ingested [r0 - 5 + L, r1 + 4 - L], finished [r0 - 4 + L, r1 + 4 - L)
  const int ilo = r0 - 5 + L, ihi = r1 + 4 - L, clo = r0 - 4 + L, chi = r1 + 4 - L;
  const int nsteps = r1 - r0 + 11;
  dma_row(r0 - 4);  // level 1's rows of steps 0 and 1
  dma_row(r0 - 3);
  // step s (phase K = s mod 3): level L ingests row i = r0 - 2 - 2L + s and finishes row i - 1
  auto step = [&](auto kc, int s) {
    constexpr int K = decltype(kc)::value;
    const int i = r0 - 2 - 2 * L + s;
    if (s == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NW) : "memory");
    lds_barrier();
    if constexpr (MODE == 1) {  // the activation of row i + 1 (finished two steps later)
      const int y2 = i + 1;
      if (y2 >= clo && y2 < chi && y2 >= 0 && y2 < a.h)  // (wave-uniform)
        msk[K] = __builtin_bit_cast(v4u32, __builtin_amdgcn_raw_buffer_load_b128(
                                               mr, liveq ? (uint32_t)(nimg * a.h + y2) * mrow + (uint32_t)(ml * 2) : BUF_OOB, 0, 0));
    }
    dma_row(r0 - 2 + s);  // the base row level 1 ingests in step s + 2
    // ingest row i.  All three kernel rows and both fragments are computed unconditionally: a target row outside this
    // level's finished range or outside the image is never finished from its accumulator (the rows a finished row
    // needs are all ingested), and the pixel slots of a fragment past the image width hold zeros
    constexpr int SN = (K + 2) % 3, SI = (K + 1) % 3, SP = K;  // accumulator rows of output rows i + 1, i, i - 1
    if (i >= ilo && i <= ihi && i >= 0 && i < a.h) {
      const char* bsl = smem + ((i - r0 + 4) % RR_NB) * RR_BSLOT + lb;
      const char* x1r = smem + RR_OFF_D + ((i - r0 + 3 + RR_N1) % RR_N1) * RR_DROW + ldn;
      const char* x2r = smem + RR_OFF_2 + ((i - r0 + 2 + RR_N2) % RR_N2) * RR_DROW + ldn;
      const char* x3r = smem + RR_OFF_3 + ((i - r0 + 1 + RR_N3) % RR_N3) * RR_DROW + ldn;
      bf16x8 B[2][2];
      auto ldB = [&](int grp, int buf) {
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          const int px = 16 * (2 * fp + f);
          if (grp < 6) {
            const int kx = grp >> 1, cb = grp & 1;
            B[buf][f] = *(const bf16x8*)(bsl + (px + kx) * RR_BP + cb * 64);
          } else {
            const int d = grp - 6;
            const char* src;
            int kx;
            if (L == 2 || d >= 3) {
              const int pr = L == 2 ? d : d - 3;
              kx = pr == 0 ? (g < 2 ? 0 : 1) : 2;
              src = L == 2 ? x1r : x3r;
            } else {
              kx = d;
              src = g < 2 ? x1r : x2r;
            }
            B[buf][f] = *(const bf16x8*)(src + (px + kx) * RR_DP);
          }
        }
      };
      ldB(0, 0);
#pragma unroll
      for (int grp = 0; grp < NG; ++grp) {
        if (grp + 1 < NG) ldB(grp + 1, (grp + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const bf16x8 af = grp < 6 ? Ab[ky][grp >> 1][grp & 1] : Ad[ky][grp < 6 ? 0 : grp - 6];
          constexpr int SL[3] = {SN, SI, SP};
#pragma unroll
          for (int f = 0; f < 2; ++f)
            acc[SL[ky]][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, B[grp & 1][f], acc[SL[ky]][f], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // row y = i - 1 is complete: epilogue into this level's ring (zeros outside the image: the next level's padding)
    // and the strip's own rows to HBM (2 raw stores, unconditional; an out-of-range offset drops them)
    const int y = i - 1;
    const bool fin = y >= clo && y < chi, yin = y >= 0 && y < a.h;
    // rows 1, 3 of fragment 0 <-> rows 0, 2 of fragment 1 (v_permlane16_swap on the fp32 sums): lane (col, g) then holds
    // channels 8 (g >> 1) .. + 7 of fragment g & 1's pixel col
    float t8[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[SP][0][e]), __float_as_uint(acc[SP][1][e]), false, false);
      t8[e] = __uint_as_float(sw[0]);
      t8[4 + e] = __uint_as_float(sw[1]);
    }
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float t = t8[e] + bb[e];
      if (MODE == 0) {
        v[e] = fmaxf(t, t * a.slope);  // leaky relu, 0 <= slope <= 1 (checked on the host)
      } else {
        const uint32_t mw = msk[(K + 1) % 3][e >> 1];
        const float mv = __uint_as_float((e & 1) ? (mw & 0xFFFF0000u) : (mw << 16));
        v[e] = mv > 0.f ? t : t * a.slope;
      }
    }
    const uint4 o8 = yin ? make_uint4(pack2_bf16(v[0], v[1]), pack2_bf16(v[2], v[3]), pack2_bf16(v[4], v[5]), pack2_bf16(v[6], v[7]))
                         : make_uint4(0u, 0u, 0u, 0u);
    if constexpr (L < 4) {
      if (fin) {
        char* ring = smem + (L == 1 ? RR_OFF_D + ((y - r0 + 3) % RR_N1) * RR_DROW
                                    : (L == 2 ? RR_OFF_2 + ((y - r0 + 2) % RR_N2) * RR_DROW : RR_OFF_3 + ((y - r0 + 1) % RR_N3) * RR_DROW));
        if (liveq) *(uint4*)(ring + dl) = o8;
      }
    }
    if (fin && yin && y >= r0 && y < r1)  // (wave-uniform) one of the strip's own rows
      __builtin_amdgcn_raw_buffer_store_b128((v4u32){o8.x, o8.y, o8.z, o8.w}, orr,
                                             liveq ? (uint32_t)(nimg * a.h + y) * orow + (uint32_t)(ol * 2) : BUF_OOB, 0, 0);
#pragma unroll
    for (int f = 0; f < 2; ++f) acc[SP][f] = (f32x4){0.f, 0.f, 0.f, 0.f};  // becomes row i + 2's next step
  };
  for (int s = 0; s < nsteps; s += 3) {
    step(std::integral_constant<int, 0>{}, s);
    if (s + 1 < nsteps) step(std::integral_constant<int, 1>{}, s + 1);
    if (s + 2 < nsteps) step(std::integral_constant<int, 2>{}, s + 2);
  }
}

// Waves w and w + 4 share a SIMD (a workgroup's waves go round the 4 SIMDs in a fixed cyclic order).  Wave w < 4
// computes level w + 1, wave w >= 4 level 8 - w; wave w covers column fragments 2 (w >> 2) and 2 (w >> 2) + 1.
template <int MODE>
__global__ __launch_bounds__(512, 1) void rdb_chain_rr_kernel(ChainArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int nimg = blockIdx.x / a.strips_y, r0 = (blockIdx.x % a.strips_y) * a.rows;
  const int r1 = min(r0 + a.rows, a.h);
  const int w = tid >> 6;
  switch (w < 4 ? w : 7 - w) {
    case 0: run_level<MODE, 1>(a, smem, tid, nimg, r0, r1); break;
    case 1: run_level<MODE, 2>(a, smem, tid, nimg, r0, r1); break;
    case 2: run_level<MODE, 3>(a, smem, tid, nimg, r0, r1); break;
    default: run_level<MODE, 4>(a, smem, tid, nimg, r0, r1); break;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

namespace climsr {

// the launch for an already validated descriptor of width 16 / 32 / 48 / 64 (climsr_rdb_chain, rdb_chain.hip)
int rdb_chain_narrow(const ClimsrChainDesc* d, hipStream_t stream) {
  const long px = (long)d->n * d->h * d->w;
  ChainArgs a;
  a.base = d->base; a.bcs = d->bcs; a.boff = d->boff;
  a.out = d->out; a.ocs = d->ocs;
  a.mask = d->mask; a.mcs = d->mcs;
  for (int L = 0; L < 4; ++L) {
    a.ooff[L] = d->ooff[L];
    a.wt[L] = d->wt[L];
    a.bias[L] = d->bias[L];
    a.moff[L] = d->moff[L];
  }
  a.slope = d->slope;
  a.n = d->n; a.h = d->h; a.w = d->w;
  a.base_bytes = (uint32_t)(px * d->bcs * 2);
  a.out_bytes = (uint32_t)(px * d->ocs * 2);
  a.mask_bytes = d->act == 3 ? (uint32_t)(px * d->mcs * 2) : 0u;
  // strip height: enough strips to give every CU one (a strip recomputes 3 + 2 + 1 halo rows per level)
  int rows = ceil_div((long)d->n * d->h, device_cus());
  if (rows < 2) rows = 2;
  if (rows > 32) rows = 32;
  if (rows > d->h) rows = d->h;
  a.rows = rows;
  a.strips_y = ceil_div(d->h, rows);
  if (d->act == 1) {
    if (int e = lds_opt_in((const void*)rdb_chain_rr_kernel<0>, RR_LDS)) return e;
    hipLaunchKernelGGL(rdb_chain_rr_kernel<0>, dim3(a.strips_y * a.n), dim3(512), RR_LDS, stream, a);
  } else {
    if (int e = lds_opt_in((const void*)rdb_chain_rr_kernel<1>, RR_LDS)) return e;
    hipLaunchKernelGGL(rdb_chain_rr_kernel<1>, dim3(a.strips_y * a.n), dim3(512), RR_LDS, stream, a);
  }
  return check_launch("rdb_chain");
}

}  // namespace climsr
