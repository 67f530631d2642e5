// Residual-dense-block chain for images up to 64 columns wide (16, 32, 48, 64): the four 16-output 3x3 convs of an
// RDB in ONE launch (esrgan.py:22-37), forward (conv1..conv4 -> x1..x4) and pull backward (pull4..pull1 -> dZ4..dZ1);
// wider images take rdb_chain.hip's column-windowed kernel.
//
// One workgroup owns R full-width image rows and streams down them.  Step s: level 1 computes row y1 = r0 - 3 + s,
// level L row y1 - 2(L - 1) (every row it reads from level L-1 was written in an earlier step: one barrier per step).
// LDS holds a 10-row ring of the base (64 ch: each level reads the base rows around its own row) and an 8-row ring
// of the level outputs [out1|out2|out3] (48 ch); only the strip's own rows are stored to HBM, the 3 + 2 + 1 halo rows
// above / below each strip are recomputed by the neighbouring strips.
// Eight waves, two per SIMD: wave w < 4 computes level w + 1, wave w >= 4 level 8 - w, so each SIMD pairs a light and
// a heavy level (1 + 4, 2 + 3: 50 of the 100 MFMA blocks per row each); waves 0-3 cover column fragments 0, 1 and
// waves 4-7 fragments 2, 3.  A wave keeps its level's A fragments (16 co x 32 k, 18 + dense blocks) in registers for
// the launch, and every A fragment feeds two MFMAs (its two column fragments); B = one 16-pixel x 32-channel
// ds_read_b128 per MFMA.  The second wave of a SIMD hides the other's LDS latency (the column-windowed kernel's one
// wave per SIMD measured 43 / 52 us per forward / pull launch at B=32 64x64 against 32 / 40 us here).
// K blocking: the base part of a level is 9 taps x 2 blocks of 32 channels; the dense part is one block per tap for
// 32 channels (out1|out2) and, for a 16-channel group (out1 of level 2, out3 of level 4), PAIRS of taps in one block
// (lanes 0-31 read tap 2p, lanes 32-63 tap 2p+1): 5 blocks instead of 9 half-empty ones.
// MFMA v_mfma_f32_16x16x32_bf16: A = weights [16 co][32 k], B = [32 k][16 pixels], C lane = 4 co of one pixel.
#include "common.h"

using namespace climsr;


namespace {

constexpr int RC_W = 64;                         // widest image row (4 fragments)
constexpr int RC_COLS = RC_W + 2;                // LDS pixel slots per row: image columns -1 .. 64
constexpr int RC_XP = 64 + 16;                   // base pixel pitch (bf16): == 16 (mod 32), conflict-free b128 reads
constexpr int RC_DP = 48;                        // dense pixel pitch: out1 | out2 | out3 (== 16 mod 32)
constexpr int RC_XD = 10;                        // base ring rows (y1-7 .. y1+1 read, y1+2 staged)
constexpr int RC_DD = 8;                         // dense ring rows (y1-7 .. y1-1 read, y1 written)
constexpr int RC_XROW = RC_COLS * RC_XP;
constexpr int RC_DROW = RC_COLS * RC_DP;
constexpr int RC_OFF_D = RC_XD * RC_XROW;        // elements
constexpr int RC_LDS = (RC_OFF_D + RC_DD * RC_DROW) * 2;  // 156,288 B
constexpr int RC_XCH = RC_COLS * 8;              // 16 B chunks of one base row (528)

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

__host__ __device__ constexpr int kp_blocks(int L) { return L == 1 ? 2 : (L == 4 ? 4 : 3); }
__host__ __device__ constexpr int nd_blocks(int L) { return L == 1 ? 0 : (L == 2 ? 5 : (L == 3 ? 9 : 14)); }
__host__ __device__ constexpr int n_blocks(int L) { return 18 + nd_blocks(L); }

// The (tap, channel offset in the dense pixel) of lane group g in dense block j of level L; tap < 0: padding
// (zero weights; the B read goes to tap 8 of the same block so every value read is finite).
__device__ __forceinline__ void dense_src(int L, int j, int g, int& tap, int& ch) {
  if (L == 3 || (L == 4 && j < 9)) {
    tap = j;
    ch = 8 * g;
  } else {
    const int p = L == 2 ? j : j - 9;
    tap = 2 * p + (g >> 1);
    ch = (L == 2 ? 0 : 32) + 8 * (g & 1);
    if (tap > 8) tap = -1;
  }
}

// A fragments of level L (16 co x 32 k per block) straight from the packed global weights ([16][9*KP], row pitch
// 9*KP) into registers, kept for the whole launch: no LDS weight image, no workgroup barrier before the first base
// rows are staged (the two waves of a level each fetch their 18-32 x 1 KB, L2-resident across the grid).
template <int L>
__device__ __forceinline__ void load_af_global(const uint16_t* __restrict__ wt, int lane, bf16x8 (&af)[n_blocks(L)]) {
  constexpr int KP = kp_blocks(L) * 32;
  const int g = lane >> 4, col = lane & 15;
  const uint16_t* wr = wt + col * 9 * KP;
#pragma unroll
  for (int j = 0; j < 18; ++j) af[j] = *(const bf16x8*)(wr + (j >> 1) * KP + (j & 1) * 32 + g * 8);
#pragma unroll
  for (int j = 0; j < nd_blocks(L); ++j) {
    int tap, ch;
    dense_src(L, j, g, tap, ch);
    af[18 + j] = tap >= 0 ? *(const bf16x8*)(wr + tap * KP + 64 + ch) : (bf16x8){};
  }
}

// One level row, two column fragments (16 pixels apart): acc0/acc1 = sum over the level's blocks.  xr[ky] / dr[ky]:
// LDS element offsets of the base / dense ring rows y-1+ky; lx / ld / lp: this lane's pixel-column (+ channel
// group) offsets within a row.  Every A fragment feeds two independent accumulators.
template <int L>
__device__ __forceinline__ const uint16_t* block_src(const uint16_t* lds, const int (&xr)[3], const int (&dr)[3], int lx,
                                                     int ld, int lp, int g, int j) {
  if (j < 18) {
    const int t = j >> 1, ky = t / 3, kx = t % 3;
    return lds + xr[ky] + lx + kx * RC_XP + (j & 1) * 32;
  }
  j -= 18;
  int off;
  if (L == 3 || (L == 4 && j < 9)) {
    off = dr[j / 3] + ld + (j % 3) * RC_DP;
  } else {
    const int p = L == 2 ? j : j - 9;
    const int ta = 2 * p, tb = 2 * p + 1 <= 8 ? 2 * p + 1 : 2 * p;
    const int oa = dr[ta / 3] + (ta % 3) * RC_DP, ob = dr[tb / 3] + (tb % 3) * RC_DP;
    off = (g >= 2 ? ob : oa) + lp + (L == 2 ? 0 : 32);
  }
  return lds + RC_OFF_D + off;
}

// Blocks run in groups of rc_group(L): the B fragments of group k+1 are read while group k is on the MFMA pipe, so
// 2 x rc_group reads stay in flight (the group size is what each level's weight registers leave room for).
__host__ __device__ constexpr int rc_group(int L) { return L <= 2 ? 6 : (L == 3 ? 5 : 4); }

template <int L>
__device__ __forceinline__ void level_acc(const uint16_t* lds, const bf16x8 (&af)[n_blocks(L)], const int (&xr)[3],
                                          const int (&dr)[3], int lx, int ld, int lp, int g, f32x4& acc0, f32x4& acc1) {
  constexpr int NB = n_blocks(L), G = rc_group(L), NG = (NB + G - 1) / G;
  acc0 = (f32x4){0.f, 0.f, 0.f, 0.f};
  acc1 = acc0;
  bf16x8 b[2][G][2];
  auto load = [&](int gi, bf16x8 (&bb)[G][2]) {
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int j = gi * G + i;
      if (j < NB) {
        const uint16_t* p = block_src<L>(lds, xr, dr, lx, ld, lp, g, j);
        bb[i][0] = *(const bf16x8*)p;
        bb[i][1] = *(const bf16x8*)(p + (j < 18 ? 16 * RC_XP : 16 * RC_DP));  // the second fragment: 16 pixels on
      }
    }
  };
  load(0, b[0]);
#pragma unroll
  for (int gi = 0; gi < NG; ++gi) {
    if (gi + 1 < NG) load(gi + 1, b[(gi + 1) & 1]);
    __builtin_amdgcn_sched_barrier(0);  // the next group's reads go out before this group's MFMAs
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int j = gi * G + i;
      if (j < NB) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[j], b[gi & 1][i][0], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[j], b[gi & 1][i][1], acc1, 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

__device__ __forceinline__ int xslot(int y) { return (y + 4 * RC_XD) % RC_XD; }  // y >= -8
__device__ __forceinline__ int dslot(int y) { return (y + 4 * RC_DD) & (RC_DD - 1); }

__device__ __forceinline__ uint32_t pack2_bf16(float a, float b) {
  const bf16x2 v = {(__bf16)a, (__bf16)b};  // v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(uint32_t, v);
}

// The whole strip walk of one wave: level L, column fragments 2h and 2h+1.  Every wave runs the same step loop
// (base-row staging + one barrier per step); level L computes in steps 3(L-1) .. R+4+L.
// MODE 0: forward (bias + leaky relu); 1: pull (leaky-relu derivative of the stored activation, no bias).
// Address arithmetic is split into per-lane constants (computed once) and per-step wave-uniform row offsets.
template <int MODE, int L>
__device__ __forceinline__ void run_level(const ChainArgs& a, uint16_t* lds, int tid, int nimg, int r0) {
  const int lane = tid & 63, g = lane >> 4, col = lane & 15, h = tid >> 8;
  const int px0 = 32 * h + col;                  // this lane's image column in fragment 2h (fragment 2h+1: + 16)
  const bool live0 = 32 * h < a.w, live1 = 32 * h + 16 < a.w;
  const __amdgpu_buffer_rsrc_t br = buf_rsrc(a.base, a.base_bytes);
  const __amdgpu_buffer_rsrc_t mr = buf_rsrc(a.mask, MODE == 1 ? a.mask_bytes : 0u);
  const int R = a.rows, row0 = nimg * a.h;       // row0: this image's first row in the batch

  // base row staging: chunk q = tid (+ 512) of a row is (slot q / 8 = image column + 1, 16 B channel group q % 8)
  int xg[2], xl[2];  // byte offset within a base row in HBM (-1: zero chunk) / element offset within a ring row (-1: none)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = tid + 512 * i, p = q >> 3, c = q & 7, ix = p - 1;
    xl[i] = q < RC_XCH ? p * RC_XP + c * 8 : -1;
    xg[i] = q < RC_XCH && ix >= 0 && ix < a.w ? (ix * a.bcs + a.boff + c * 8) * 2 : -1;
  }
  const uint32_t xrow_bytes = (uint32_t)(a.w * a.bcs * 2);
  auto issue_row = [&](int y, uint4 (&v)[2]) {
    const bool rok = y >= 0 && y < a.h;
    const uint32_t rb = (uint32_t)(row0 + y) * xrow_bytes;
#pragma unroll
    for (int i = 0; i < 2; ++i) v[i] = buf_load16(br, rok && xg[i] >= 0 ? rb + (uint32_t)xg[i] : BUF_OOB);
  };
  auto store_row = [&](int y, const uint4 (&v)[2]) {
    uint16_t* row = lds + xslot(y) * RC_XROW;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      if (xl[i] >= 0) *(uint4*)(row + xl[i]) = v[i];
  };
  // pull: the activation x_j of this level's row in step s for both fragments (zeros outside), one step ahead
  int ml[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int px = px0 + 16 * k;
    ml[k] = px < a.w ? (px * a.mcs + a.moff[L - 1] + 4 * g) * 2 : -1;
  }
  const uint32_t mrow_bytes = (uint32_t)(a.w * a.mcs * 2);
  auto issue_mask = [&](int s, uint2 (&m)[2]) {
    const int y = r0 - 3 + s - 2 * (L - 1);
    const bool rok = y >= 0 && y < a.h;
    const uint32_t rb = (uint32_t)(row0 + y) * mrow_bytes;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(mr, rok && ml[k] >= 0 ? rb + (uint32_t)ml[k] : BUF_OOB, 0, 0);
      m[k] = make_uint2(v[0], v[1]);
    }
  };
  // Prologue: the first base rows are in flight while each wave loads its level's A fragments.
  // Base rows are loaded one step before the step that stores them (two steps before their first use) and masks
  // one step before their use; the loop is unrolled x2 with alternating register sets, so no register copy of a
  // load still in flight (which would wait for it) is ever needed.
  uint4 v0[2], v1[2], v2[2], ra[2], rb[2];
  issue_row(r0 - 4, v0);
  issue_row(r0 - 3, v1);
  issue_row(r0 - 2, v2);
  issue_row(r0 - 1, ra);
  uint2 ma[2] = {}, mb[2] = {};
  if constexpr (MODE == 1) issue_mask(0, ma);
  const float4 bias = MODE == 0 ? *(const float4*)(a.bias[L - 1] + 4 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
  bf16x8 af[n_blocks(L)];
  load_af_global<L>(a.wt[L - 1], lane, af);
  // dense ring: the slots of image columns -1 and >= w are never written, they are the zero padding
  for (int i = tid; i < RC_DD * (RC_COLS - a.w) * (RC_DP / 8); i += 512) {
    const int c = i % (RC_DP / 8), k = (i / (RC_DP / 8)) % (RC_COLS - a.w), r = i / (RC_DP / 8) / (RC_COLS - a.w);
    const int p = k == 0 ? 0 : a.w + k;
    *(uint4*)(lds + RC_OFF_D + r * RC_DROW + p * RC_DP + c * 8) = make_uint4(0, 0, 0, 0);
  }
  store_row(r0 - 4, v0);
  store_row(r0 - 3, v1);
  store_row(r0 - 2, v2);
  lds_barrier();
  // retire the remaining loads here: with no VMEM result carried into the loop, hipcc's wait counting inside it
  // stays exact (otherwise every step waits with a count that also drains the base-row prefetch)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)

  const int lx = px0 * RC_XP + 8 * g;  // + kx * RC_XP: input column px - 1 + kx sits in slot px + kx
  const int ld = px0 * RC_DP + 8 * g;
  const int lp = px0 * RC_DP + 8 * (g & 1);
  const int dl = (px0 + 1) * RC_DP + 16 * (L - 1) + 4 * g;    // this lane's dense-ring store (fragment 2h)
  const int ol = px0 * a.ocs + a.ooff[L - 1] + 4 * g;          // and HBM store, elements within an image row
  const long orow = (long)a.w * a.ocs;
  const float bb[4] = {bias.x, bias.y, bias.z, bias.w};
  // step s: `cur` holds base row y1 + 2 (stored after the MFMAs), `nxt` receives row y1 + 3; `mcur` = this step's
  // masks, `mnxt` receives the next step's
  // output stores are raw buffer stores issued unconditionally every step (an out-of-range offset drops them): a store
  // under the step's level-active / own-row branches made the compiler's vmcnt for the next base-row wait count it as
  // maybe-not-issued, so that wait also drained this step's stores (measured: 7 of 31 us per forward launch)
  const __amdgpu_buffer_rsrc_t orr = buf_rsrc(a.out, a.out_bytes);
  auto step = [&](int s, uint4 (&cur)[2], uint4 (&nxt)[2], const uint2 (&mcur)[2], uint2 (&mnxt)[2]) {
    const int y1 = r0 - 3 + s;
    issue_row(y1 + 3, nxt);
    if constexpr (MODE == 1) issue_mask(s + 1, mnxt);
    const bool active = live0 && s >= 3 * (L - 1) && s <= R + 4 + L;
    const int y = y1 - 2 * (L - 1);
    const bool own = active && y >= 0 && y < a.h && y >= r0 && y < r0 + R;
    uint2 pko[2] = {make_uint2(0, 0), make_uint2(0, 0)};
    if (active) {
      int xr[3], dr[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        xr[k] = xslot(y - 1 + k) * RC_XROW;
        dr[k] = dslot(y - 1 + k) * RC_DROW;
      }
      f32x4 acc[2];
      level_acc<L>(lds, af, xr, dr, lx, ld, lp, g, acc[0], acc[1]);
      const bool in = y >= 0 && y < a.h;  // rows outside the image: zeros, the next level's padding
      uint16_t* drow = lds + RC_OFF_D + dslot(y) * RC_DROW + dl;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float t = acc[k][i] + bb[i];
          if (MODE == 0) {
            v[i] = fmaxf(t, t * a.slope);  // leaky relu, 0 <= slope <= 1 (checked on the host)
          } else {
            const uint32_t mw = i < 2 ? mcur[k].x : mcur[k].y;
            const float m = __uint_as_float((i & 1) ? (mw & 0xFFFF0000u) : (mw << 16));  // the stored activation
            v[i] = m > 0.f ? t : t * a.slope;
          }
        }
        uint2 pk = make_uint2(pack2_bf16(v[0], v[1]), pack2_bf16(v[2], v[3]));
        if (!in) pk = make_uint2(0, 0);
        if (L < 4 && (k == 0 || live1)) *(uint2*)(drow + 16 * k * RC_DP) = pk;
        pko[k] = pk;
      }
    }
    const uint32_t ob = (uint32_t)((row0 + y) * orow + ol) * 2u;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const bool ok = own && (k == 0 || live1);
      __builtin_amdgcn_raw_buffer_store_b64((v2u32){pko[k].x, pko[k].y}, orr, ok ? ob + (uint32_t)(16 * k * a.ocs * 2) : BUF_OOB, 0, 0);
    }
    store_row(y1 + 2, cur);  // its slot held row y1 - 8, which no level reads in this step
    lds_barrier();
  };
  for (int s = 0; s < R + 9; s += 2) {
    step(s, ra, rb, ma, mb);
    if (s + 1 < R + 9) step(s + 1, rb, ra, mb, ma);
  }
}

// Waves w and w + 4 share a SIMD (a workgroup's waves go round the 4 SIMDs in a fixed cyclic order).  Wave w < 4
// computes level w + 1, wave w >= 4 level 8 - w, so each SIMD pairs a light and a heavy level (1+4, 2+3: 50 of the
// 100 MFMA blocks per row each) instead of carrying one level: the per-step critical path is the slowest SIMD.
// Wave w covers column fragments 2 (w >> 2) and 2 (w >> 2) + 1.
template <int MODE>
__global__ __launch_bounds__(512, 1) void rdb_chain_kernel(ChainArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* lds = (uint16_t*)smem;
  const int tid = threadIdx.x;
  const int nimg = blockIdx.x / a.strips_y, r0 = (blockIdx.x % a.strips_y) * a.rows;
  const int w = tid >> 6;
  switch (w < 4 ? w : 7 - w) {
    case 0: run_level<MODE, 1>(a, lds, tid, nimg, r0); break;
    case 1: run_level<MODE, 2>(a, lds, tid, nimg, r0); break;
    case 2: run_level<MODE, 3>(a, lds, tid, nimg, r0); break;
    default: run_level<MODE, 4>(a, lds, tid, nimg, r0); break;
  }
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
  // strip height: enough strips to give every CU one (a strip recomputes 3 + 2 + 1 halo rows per level chain)
  int rows = ceil_div((long)d->n * d->h, device_cus());
  if (rows < 2) rows = 2;
  if (rows > 32) rows = 32;
  if (rows > d->h) rows = d->h;
  a.rows = rows;
  a.strips_y = ceil_div(d->h, rows);
  if (d->act == 1) {
    if (int e = lds_opt_in((const void*)rdb_chain_kernel<0>, RC_LDS)) return e;
    hipLaunchKernelGGL(rdb_chain_kernel<0>, dim3(a.strips_y * a.n), dim3(512), RC_LDS, stream, a);
  } else {
    if (int e = lds_opt_in((const void*)rdb_chain_kernel<1>, RC_LDS)) return e;
    hipLaunchKernelGGL(rdb_chain_kernel<1>, dim3(a.strips_y * a.n), dim3(512), RC_LDS, stream, a);
  }
  return check_launch("rdb_chain");
}

}  // namespace climsr
