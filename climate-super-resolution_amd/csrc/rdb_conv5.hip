// The 128 -> 64 3x3 conv of a residual dense block: conv5 over the dense concatenation [x | x1 | x2 | x3 | x4] with
// its fused `x5 * 0.2 + x` (and the RRDB's `out * 0.2 + x`) epilogue (esrgan.py:26,38,54), and the same shape in the
// backward, pull-x: the gradient of the block input as ONE conv over the side-by-side output gradients
// [dZ1 | .. | dZ5] (fp32 out + skip gradients + the previous block's bf16 dZ5).
//
// Row streaming with input-row reuse.  A workgroup owns a strip of R output rows x 64 columns and ingests the R + 2
// input rows it needs one at a time (LDS-DMA into three row slots: two rows in flight under the current row's MFMAs).
// An ingested row feeds all three kernel rows at once: B fragment (row i, tap column kx) is multiplied by the weights
// of taps (0, kx), (1, kx), (2, kx) into the accumulators of output rows i + 1, i, i - 1, so each 1 KB fragment read
// from LDS feeds three MFMAs (a per-output-row implicit GEMM reads it three times).  Output row i - 1 is complete
// once row i is in; three accumulator rows rotate.
// Eight waves: wave w owns output channels 16 (w & 3) .. + 15 and input channels 64 (w >> 2) .. + 63 for all four
// 16-pixel fragments of a row; its 18 weight fragments (3 x 3 taps x 2 channel blocks of 32) stay in registers for
// the launch.  The two channel halves of an output block are summed through LDS (each wave finishes two of the four
// fragments, in a fixed order: half 0 + half 1, deterministic) before the epilogue.  The epilogue trades halves of
// the two fragments between lane rows g and g ^ 1 (v_permlane16_swap) so that each lane holds 8 consecutive channels
// of one pixel: residuals and outputs move as 16-B loads / stores (8-B ones cost twice the issue per byte).
// One barrier per row; the residual operands of a row are loaded one step before it is finished, and the waits are
// counted by hand (see the step loop) so that the next row's DMA stays in flight across them.
// LDS pixel slots are 288 B (128 channels + 32 B pad): the 16-B unit of channel chunk c of slot p is 18 p + c, so
// the 16 lanes of each ds_read_b128 bank group (two channel groups, 8 pixels each) cover the 64 banks once.
// MFMA v_mfma_f32_16x16x32_bf16: A = weights [16 co][32 channels], B = [32 channels][16 pixels].
#include "conv_ep.h"

namespace {

constexpr int R5_PX = 66;                          // pixel slots per row: image columns c0 - 1 .. c0 + 64
constexpr int R5_PITCH = 288;                      // bytes per pixel slot (18 units of 16 B)
constexpr int R5_UNITS = R5_PX * 18;               // 1188
constexpr int R5_NI = (R5_UNITS + 63) / 64;        // DMA instructions per row (19)
constexpr int R5_SLOT = R5_NI * 1024;              // 19,456 B
constexpr int R5_NSLOT = 3;                        // row slots: the row being read, and two in flight
constexpr int R5_PART = 16 * 1024;                 // one partial-sum exchange region: [co block][fragment][lane] f32x4
constexpr int R5_OFF_P = R5_NSLOT * R5_SLOT;       // 58,368
constexpr int R5_OFF_DUMMY = R5_OFF_P + 2 * R5_PART;  // one KB the padding DMA pieces write (zeros, never read)
constexpr int R5_LDS = R5_OFF_DUMMY + 1024;        // 92,160 B
constexpr int R5_K = 3;                            // DMA pieces per wave and row (19 real + 5 padding over 8 waves)
#ifndef CLIMSR_R5_EXP  // timing experiments of diagnostic builds only (tools/gpu_r05f.sh): 1 no step DMA, 2 no residual
#define CLIMSR_R5_EXP 0  // loads, 3 no stores, 4 none of the three, 5 no MFMAs -- their results are wrong
#endif

#ifdef CLIMSR_R5_STAMP
// Timing diagnostic (tools/stamp_r5.py; never in the product build): waves 0 and 4 record (s_memrealtime, s_memtime)
// at R5_NST points into LDS past the kernel's own bytes; the block copies them to r5_stamps at the end.
constexpr int R5_NST = 48, R5_STAMP_BLOCKS = 1024;
constexpr int R5_LDS_ALL = R5_LDS + 2 * R5_NST * 16;
__device__ unsigned long long r5_stamps[R5_STAMP_BLOCKS * 2 * R5_NST * 2];
#define R5_STAMP(k)                                                                                              \
  do {                                                                                                           \
    if (lane == 0 && (wvu & 3) == 0 && (k) < R5_NST) {                                                           \
      unsigned long long* sl_ = (unsigned long long*)(smem + R5_LDS + ((wvu >> 2) * R5_NST + (k)) * 16);          \
      sl_[0] = __builtin_amdgcn_s_memrealtime();                                                                 \
      sl_[1] = __builtin_amdgcn_s_memtime();                                                                     \
    }                                                                                                            \
  } while (0)
#else
constexpr int R5_LDS_ALL = R5_LDS;
#define R5_STAMP(k) \
  do {              \
  } while (0)
#endif

struct R5Args {
  const uint16_t* x;
  const uint16_t* wt;
  const float* bias;
  void* y;
  const void* res1;
  const void* res2;
  uint16_t* aux;
  int xcs, xco, kpk, ycs, yco, r1cs, r1co, r2cs, r2co, auxcs, auxco;
  float alpha1, beta1, alpha2, beta2, aux_scale;
  int n, h, w, rows, strips, tiles_x;
  uint32_t x_bytes, y_bytes, r1_bytes, r2_bytes, aux_bytes;
};
typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t pk2(float a, float b) {
  const bf16x2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// MODE 1: conv5 (bias, bf16 residuals, bf16 out); MODE 2: pull-x (no bias, fp32 residuals, fp32 out, optional bf16 aux)
template <int MODE, bool R2>
__global__ __launch_bounds__(512, 1) void rdb5_kernel(R5Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool F32 = MODE == 2;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, col = lane & 15;
  const int wvu = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = wvu & 3, hh = wvu >> 2;  // output channel block, input channel half
  const int tile = blockIdx.x % a.tiles_x, rest = blockIdx.x / a.tiles_x;
  const int strip = rest % a.strips, nimg = rest / a.strips;
  const int r0 = strip * a.rows, r1 = min(r0 + a.rows, a.h);  // output rows [r0, r1)
  const int c0 = tile * 64;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;
  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(a.x, a.x_bytes);
  R5_STAMP(0);

  // this wave's DMA pieces of a row: instructions wvu, wvu + 8, wvu + 16 (< 19); lane -> 16-B unit 64 k + lane =
  // (pixel slot p, channel chunk j); pad units and out-of-image pixels get BUF_OOB (zeros land)
  uint32_t po[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int k = wvu + 8 * j, u = 64 * k + lane, p = u / 18, jj = u - 18 * p, ix = c0 - 1 + p;
    po[j] = (k < R5_NI && jj < 16 && p < R5_PX && ix >= 0 && ix < a.w) ? (uint32_t)((ix * a.xcs + a.xco + 8 * jj) * 2) : BUF_OOB;
  }
  const uint32_t xrow = (uint32_t)a.w * (uint32_t)a.xcs * 2u;
  auto glds = [&](uint32_t off, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(off), "s"(xr), "s"(lds) : "memory");
  };
  // the 18 weight fragments: tap (ky, kx), channel block 2 hh + cb (packed [co][chunk][tap][32], chunk pitch 288)
  bf16x8 A[3][3][2];
  {
    const uint16_t* wr = a.wt + (long)(16 * q + col) * a.kpk + 8 * g;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) A[ky][kx][cb] = *(const bf16x8*)(wr + (2 * hh + cb) * 288 + (3 * ky + kx) * 32);
  }
  // after the swap (see finish) lane (col, g) holds channels co8 .. co8 + 7 of fragment 2 hh + (g & 1), pixel col
  const int co8 = 16 * q + 8 * (g >> 1), fm = g & 1;
  float bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if constexpr (MODE == 1) {
    const float4 b0 = *(const float4*)(a.bias + co8), b1 = *(const float4*)(a.bias + co8 + 4);
    bb[0] = b0.x; bb[1] = b0.y; bb[2] = b0.z; bb[3] = b0.w; bb[4] = b1.x; bb[5] = b1.y; bb[6] = b1.z; bb[7] = b1.w;
  }
  const bool has_aux = MODE == 2 && a.aux != nullptr;
  const __amdgpu_buffer_rsrc_t rr1 = buf_rsrc(a.res1, a.r1_bytes), rr2 = buf_rsrc(a.res2, R2 ? a.r2_bytes : 0u);
  const __amdgpu_buffer_rsrc_t ry = buf_rsrc(a.y, a.y_bytes), rax = buf_rsrc(a.aux, has_aux ? a.aux_bytes : 0u);
  f32x4 acc[3][4];
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int f = 0; f < 4; ++f) acc[s][f] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // residual operands of this lane's 8 channels of the row it finishes: two sets, loaded one step ahead; 16 B each
  // (bf16), two 16-B halves (fp32)
  constexpr int NR = F32 ? 2 : 1;
  struct Rv {
    v4u32 v[NR];
  };
  Rv rs1[2], rs2[2];
  const bool col_ok = c0 + 16 * (2 * hh + fm) + col < a.w;
  auto pidx = [&](int y) { return (uint32_t)((nimg * a.h + y) * a.w + c0 + 16 * (2 * hh + fm) + col); };
  auto load_res = [&](int y, Rv& r1v, Rv& r2v) {
    const bool ok = y >= r0 && y < r1 && col_ok;
    const uint32_t p = ok ? pidx(y) : 0u;
#pragma unroll
    for (int h = 0; h < NR; ++h) {
      r1v.v[h] = __builtin_bit_cast(v4u32, __builtin_amdgcn_raw_buffer_load_b128(
                                               rr1, ok ? (p * a.r1cs + a.r1co + co8 + 4 * h) * (F32 ? 4u : 2u) : BUF_OOB, 0, 0));
      if constexpr (R2)
        r2v.v[h] = __builtin_bit_cast(v4u32, __builtin_amdgcn_raw_buffer_load_b128(
                                                 rr2, ok ? (p * a.r2cs + a.r2co + co8 + 4 * h) * (F32 ? 4u : 2u) : BUF_OOB, 0, 0));
    }
  };
  auto rval = [&](const Rv& r, int i) -> float {  // channel co8 + i
    if constexpr (F32) return __uint_as_float(r.v[i >> 2][i & 3]);
    else return bf2f((uint16_t)((i & 1) ? (r.v[0][i >> 1] >> 16) : r.v[0][i >> 1]));
  };
  const int lb = col * R5_PITCH + (8 * hh + g) * 16;  // this lane's B offset: pixel slot col (+ 16 f + kx), chunk 8 hh + 4 cb + g

  // Hand-counted waits.  Per step every wave issues, in this order, RL residual loads (for the row it finishes in the
  // next step), ST stores (the row it finishes now) and R5_K DMA pieces (the row it ingests two steps later), all
  // unconditionally (out-of-range offsets / the dummy KB where there is nothing to move).  Step s needs the DMA of
  // step s - 2: younger are step s - 1's RL + ST + R5_K operations.  (hipcc's own wait for the residuals of step s - 1,
  // which counts only loads and stores, may also cover step s - 1's DMA: issued half a step earlier, landed by then.)
  constexpr int RL = NR * (R2 ? 2 : 1), ST = F32 ? 3 : 1, NW = RL + ST + R5_K;
  const int nsteps = r1 - r0 + 3;  // ingest rows r0 - 1 .. r1, finish rows r0 .. r1 - 1 one step after completion
  auto dma_step = [&](int row, int slot) {
    // rows of the strip's window [r0 - 1, r1] land in their slot (zeros outside the image); any other row's pieces go
    // to the dummy KB (the MFMAs of that step only touch accumulator rows that are never finished)
    const bool win = row >= r0 - 1 && row <= r1, img = row >= 0 && row < a.h;
    const uint32_t rb = img ? (uint32_t)(nimg * a.h + row) * xrow : 0u;
#pragma unroll
    for (int j = 0; j < R5_K; ++j) {
      const bool real = win && wvu + 8 * j < R5_NI;
      glds(real && img && po[j] != BUF_OOB ? po[j] + rb : BUF_OOB,
           lds0 + (uint32_t)(real ? slot * R5_SLOT + (wvu + 8 * j) * 1024 : R5_OFF_DUMMY));
    }
  };
  dma_step(r0 - 1, 0);
  dma_step(r0, 1);
  R5_STAMP(1);

  // the epilogue of row yf: this wave's two fragments (own channel half + the partner's, fixed order), the fragment
  // halves traded so that each lane holds 8 channels of one pixel, bias / residuals, one 16-B store (fp32: two, and the
  // bf16 aux)
  auto finish = [&](int yf, bool fin, const f32x4 (&own)[2], const f32x4 (&other)[2], const Rv& r1v, const Rv& r2v) {
    f32x4 s0 = hh == 0 ? own[0] + other[0] : other[0] + own[0];
    f32x4 s1 = hh == 0 ? own[1] + other[1] : other[1] + own[1];
#pragma unroll
    for (int e = 0; e < 4; ++e) {  // rows 1, 3 of fragment 0 <-> rows 0, 2 of fragment 1
      const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(s0[e]), __float_as_uint(s1[e]), false, false);
      s0[e] = __uint_as_float(sw[0]);
      s1[e] = __uint_as_float(sw[1]);
    }
    const bool ok = fin && col_ok;
    const uint32_t p = ok ? pidx(yf) : 0u;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = (e < 4 ? s0[e] : s1[e - 4]) + bb[e];
      t = t * a.alpha1 + a.beta1 * rval(r1v, e);
      if (R2) t = t * a.alpha2 + a.beta2 * rval(r2v, e);
      v[e] = t;
    }
    if constexpr (F32) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const v4u32 o = {__float_as_uint(v[4 * h]), __float_as_uint(v[4 * h + 1]), __float_as_uint(v[4 * h + 2]),
                         __float_as_uint(v[4 * h + 3])};
        __builtin_amdgcn_raw_buffer_store_b128(o, ry, ok ? (p * a.ycs + a.yco + co8 + 4 * h) * 4u : BUF_OOB, 0, 0);
      }
      const v4u32 x4 = {pk2(a.aux_scale * v[0], a.aux_scale * v[1]), pk2(a.aux_scale * v[2], a.aux_scale * v[3]),
                        pk2(a.aux_scale * v[4], a.aux_scale * v[5]), pk2(a.aux_scale * v[6], a.aux_scale * v[7])};
      __builtin_amdgcn_raw_buffer_store_b128(x4, rax, ok ? (p * a.auxcs + a.auxco + co8) * 2u : BUF_OOB, 0, 0);
    } else {
      const v4u32 o = {pk2(v[0], v[1]), pk2(v[2], v[3]), pk2(v[4], v[5]), pk2(v[6], v[7])};
      __builtin_amdgcn_raw_buffer_store_b128(o, ry, ok ? (p * a.ycs + a.yco + co8) * 2u : BUF_OOB, 0, 0);
    }
  };

  // step s (compile-time phase K = s mod 6: row slot, residual set and accumulator row by K % 3, partial region by K & 1).
  // One basic block from the barrier to the partial-sum hand-off: the residual loads, the epilogue of row i - 2 and
  // the DMA of row i + 2 are issued between the MFMA groups of row i, so the MFMA pipe does not idle behind them
  auto step = [&](auto kc, int s) {
    constexpr int K = decltype(kc)::value;
    constexpr int SA = K % 3;         // accumulator row of output row r0 + s (ky = 0 target) == the row finished here
    constexpr int SC = (K + 1) % 3;   // accumulator row of output row r0 + s - 2 (completed in this step)
    const int i = r0 - 1 + s;         // the row ingested in this step (slot K % 3)
    R5_STAMP(2 + 3 * s);
    if (s == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NW) : "memory");
    lds_barrier();
    R5_STAMP(3 + 3 * s);
    // row i - 2 (completed last step): this wave's two fragments and the partner's halves of them
    const int yf = i - 2;
    const bool fin = yf >= r0 && yf < r1;
    f32x4 own[2], other[2];
    {
      const char* part = smem + R5_OFF_P + ((K + 1) & 1) * R5_PART;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        other[m] = *(const f32x4*)(part + (q * 4 + 2 * hh + m) * 1024 + lane * 16);
        own[m] = hh == 0 ? acc[SA][m] : acc[SA][2 + m];  // (a register select: acc is never indexed at run time)
      }
    }
#pragma unroll
    for (int f = 0; f < 4; ++f) acc[SA][f] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // ingest row i.  Every MFMA is issued: rows of the window outside the image are zeros in their slot, and the
    // last step's row (r1 + 1) only reaches accumulator rows that are never finished
    const char* xs = smem + (K % 3) * R5_SLOT + lb;
    bf16x8 B[2][4];
    auto ldB = [&](int grp, int buf) {
      const int kx = grp >> 1, cb = grp & 1;
#pragma unroll
      for (int f = 0; f < 4; ++f) B[buf][f] = *(const bf16x8*)(xs + (16 * f + kx) * R5_PITCH + cb * 64);
    };
    ldB(0, 0);
#pragma unroll
    for (int grp = 0; grp < 6; ++grp) {
      const int kx = grp >> 1, cb = grp & 1;
      if (grp + 1 < 6) ldB(grp + 1, (grp + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        constexpr int SL[3] = {SA, (K + 2) % 3, SC};  // rows r0 + s, r0 + s - 1, r0 + s - 2
#pragma unroll
        for (int f = 0; f < 4; ++f)
          if (CLIMSR_R5_EXP != 5)
            acc[SL[ky]][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ky][kx][cb], B[grp & 1][f], acc[SL[ky]][f], 0, 0, 0);
          else
            acc[SL[ky]][f] += __builtin_bit_cast(f32x4, B[grp & 1][f]);
      }
      // the step's memory work, in the hand-counted order RL, ST, DMA (see above)
      constexpr int X = CLIMSR_R5_EXP;
      if (grp == 0 && X != 2 && X != 4) load_res(i - 1, rs1[K & 1], rs2[K & 1]);  // residuals of row i - 1 (finished next step)
      if (grp == 1 && X != 3 && X != 4) finish(yf, fin, own, other, rs1[(K + 1) & 1], rs2[(K + 1) & 1]);
      if (grp == 3 && X != 1 && X != 4) dma_step(i + 2, (K + 2) % 3);  // row i + 2 into the slot of row i - 1 (last read last step)
      __builtin_amdgcn_sched_barrier(0);
    }
    R5_STAMP(4 + 3 * s);
    // row i - 1 is complete: hand the partner the two fragments it finishes
    if (i - 1 >= r0 && i - 1 < r1) {
      char* part = smem + R5_OFF_P + (K & 1) * R5_PART;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int f = 2 * (1 - hh) + m;
        *(f32x4*)(part + (q * 4 + f) * 1024 + lane * 16) = hh == 0 ? acc[SC][2 + m] : acc[SC][m];
      }
    }
  };
  for (int s = 0; s < nsteps; s += 6) {
    step(std::integral_constant<int, 0>{}, s);
    if (s + 1 < nsteps) step(std::integral_constant<int, 1>{}, s + 1);
    if (s + 2 < nsteps) step(std::integral_constant<int, 2>{}, s + 2);
    if (s + 3 < nsteps) step(std::integral_constant<int, 3>{}, s + 3);
    if (s + 4 < nsteps) step(std::integral_constant<int, 4>{}, s + 4);
    if (s + 5 < nsteps) step(std::integral_constant<int, 5>{}, s + 5);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef CLIMSR_R5_STAMP
  R5_STAMP(R5_NST - 1);
  __syncthreads();
  if (tid < 4 * R5_NST && blockIdx.x < R5_STAMP_BLOCKS)
    r5_stamps[(long)blockIdx.x * 4 * R5_NST + tid] = ((const unsigned long long*)(smem + R5_LDS))[tid];
#endif
}

}  // namespace

namespace climsr {

// The route (climsr_conv2d_fwd): 1 = conv5 form, 2 = pull-x form, 0 = not this kernel
int rdb5_route(const ClimsrConvDesc* d, const ClimsrEpilogue* ep, const float* bias, int kcpad) {
  if (!(d->ks == 3 && d->stride == 1 && d->pad == 1 && d->up == 1 && d->in_c == 128 && d->out_c == 64 && d->cc == 32 &&
        kcpad == 288 && d->out_h == d->in_h && d->out_w == d->in_w && d->in_cstride % 8 == 0 && d->in_coff % 8 == 0 &&
        !ep->down2 && ep->act == 0 && !ep->bn_part && !ep->bn_z && !ep->ch_part && ep->res1 &&
        ((d->out_cstride | d->out_coff) & 3) == 0 && ((ep->res1_cstride | ep->res1_coff) & 3) == 0 &&
        (!ep->res2 || ((ep->res2_cstride | ep->res2_coff) & 3) == 0) && (!ep->aux || ((ep->aux_cstride | ep->aux_coff) & 3) == 0)))
    return 0;
  const long px = (long)d->n * d->in_h * d->in_w;
  if (px * d->in_cstride * 2 >= (1L << 31)) return 0;  // 32-bit DMA offsets
  if (bias && ep->res_f32 == 0 && ep->out_mode == 0 && !ep->aux) return 1;
  if (!bias && (ep->res_f32 & 1) && (!ep->res2 || (ep->res_f32 & 2)) && ep->out_mode == 1) return 2;
  return 0;
}

int rdb5_launch(int mode, const ClimsrConvDesc* d, const ClimsrEpilogue* ep, const uint16_t* x, const uint16_t* wpk, int kpk,
                const float* bias, void* y, hipStream_t s, bool dry, char* name, int name_len) {
  R5Args a{};
  a.x = x; a.wt = wpk; a.bias = bias; a.y = y; a.res1 = ep->res1; a.res2 = ep->res2; a.aux = (uint16_t*)ep->aux;
  a.xcs = d->in_cstride; a.xco = d->in_coff; a.kpk = kpk; a.ycs = d->out_cstride; a.yco = d->out_coff;
  a.r1cs = ep->res1_cstride; a.r1co = ep->res1_coff; a.r2cs = ep->res2_cstride; a.r2co = ep->res2_coff;
  a.auxcs = ep->aux_cstride; a.auxco = ep->aux_coff;
  a.alpha1 = ep->alpha1; a.beta1 = ep->beta1; a.alpha2 = ep->alpha2; a.beta2 = ep->beta2; a.aux_scale = ep->aux_scale;
  a.n = d->n; a.h = d->in_h; a.w = d->in_w;
  const long px = (long)d->n * d->in_h * d->in_w;
  const int eb = mode == 2 ? 4 : 2;
  a.x_bytes = (uint32_t)(px * d->in_cstride * 2);
  a.y_bytes = (uint32_t)(px * d->out_cstride * eb);
  a.r1_bytes = (uint32_t)(px * ep->res1_cstride * eb);
  a.r2_bytes = ep->res2 ? (uint32_t)(px * ep->res2_cstride * eb) : 0u;
  a.aux_bytes = ep->aux ? (uint32_t)(px * ep->aux_cstride * 2) : 0u;
  a.tiles_x = ceil_div(d->in_w, 64);
  // strip height: one strip per CU where the rows allow (an input row costs the same whatever the strip height; the
  // two halo rows are ingested once per strip), 4..64 rows
  int rows = ceil_div((long)d->n * d->in_h * a.tiles_x, device_cus());
  rows = rows < 4 ? 4 : (rows > 64 ? 64 : rows);
  if (rows > d->in_h) rows = d->in_h;
  a.rows = rows;
  a.strips = ceil_div(d->in_h, rows);
  if (dry) {
    snprintf(name, name_len, "rdb5_kernel<%d, %s>", mode, ep->res2 ? "true" : "false");
    return CLIMSR_OK;
  }
  const bool r2 = ep->res2 != nullptr;
  void (*k)(R5Args) = mode == 2 ? (r2 ? rdb5_kernel<2, true> : rdb5_kernel<2, false>) : (r2 ? rdb5_kernel<1, true> : rdb5_kernel<1, false>);
  if (int e = lds_opt_in((const void*)k, R5_LDS_ALL)) return e;
  hipLaunchKernelGGL(k, dim3(a.tiles_x * a.strips * a.n), dim3(512), R5_LDS_ALL, s, a);
  return check_launch("conv2d_fwd (rdb5)");
}

}  // namespace climsr

#ifdef CLIMSR_R5_STAMP
extern "C" int climsr_diag_r5_stamps(void* dst, long bytes) {
  const long cap = (long)sizeof(unsigned long long) * R5_STAMP_BLOCKS * 2 * R5_NST * 2;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(r5_stamps), bytes < cap ? bytes : cap, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
