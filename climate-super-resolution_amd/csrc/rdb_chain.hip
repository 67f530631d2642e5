// Residual-dense-block chain: the four 16-output 3x3 convs of an RDB in ONE launch (esrgan.py:22-37), for images
// of any width (column windows); widths 16 / 32 / 48 / 64 take rdb_chain_narrow.hip's level-per-wave kernel, which
// is faster there (two waves per SIMD).
//
// Forward:        x1 = lrelu(conv1(x)),  x2 = lrelu(conv2([x,x1])),  x3 = ...,  x4 = lrelu(conv4([x,x1,x2,x3]))
// Pull backward:  dZ4 = lrelu'(x4) * pull4(dZ5),  dZ3 = lrelu'(x3) * pull3([dZ5,dZ4]),  ...  (climsr_hip.h)
// Both are "level L reads a 64-channel base plus the 16-channel outputs of levels < L".
//
// A level is a skinny GEMM (16 output channels): every MFMA needs a fresh 1 KB B fragment of pixels (16 px x 32 k)
// while its A fragment (weights) can stay in registers, so computed level by level the LDS read rate, not the matrix
// core, bounds it (1 KB per 16-cycle MFMA per SIMD = the whole 256 B/clk of the CU).  But the base part of the four
// levels (K = 9 x 64 of K = 9 x (64 + 16(L-1))) does not depend on the chain: it is ONE 64 -> 64-channel conv.  So
// here a wave owns a 16-pixel column fragment for ALL four levels: when base row y arrives it computes the base part
// of row y for all four levels at once (each B fragment feeds four MFMAs), keeps the partial sums of the levels that
// finish row y later in registers, and each level adds its dense part (the outputs of the earlier levels, from an LDS
// ring) when that row's inputs exist: level L finishes row y1 - 2(L-1) in step y1 (one barrier per step).
//
// A workgroup (4 waves, one per SIMD) streams down R rows of a 64-column window (4 fragments).  Images up to 64
// columns wide are one window (zero padding at the image edges); wider ones are cut into strips of 48 own columns,
// whose window adds 8 columns each side (the halo of 3 + 2 + 1 columns the chain consumes; the window's edge values
// are wrong and never stored).  The 3 + 2 + 1 halo rows above / below a strip are recomputed by its neighbours.
// LDS: a 4-row ring of the base (64 ch), an 8-row ring of the level outputs [out1|out2|out3] (48 ch), the dense-part
// A fragments of levels 3 and 4 (23 KB) and per wave the fp32 partial sums of levels 3 / 4 in flight (4 / 6 rows, one
// 1 KB lane-linear slot each); registers: the base-part A fragments of all four levels (72 x 16 B per lane), level 2's
// dense A fragments and its partial sums (two rows: the step loop runs two steps per iteration, so they never move).
// MFMA v_mfma_f32_16x16x32_bf16: A = weights [16 co][32 k], B = [32 k][16 pixels], C lane = 4 co of one pixel.
#include "common.h"
#include "mfma_agpr.h"

using namespace climsr;

namespace {

constexpr int NFR = 4;                          // 16-pixel column fragments per window = waves per workgroup
constexpr int WIN = 16 * NFR;                   // window columns
constexpr int HALO_X = 8;                       // window columns on each side of a strip's own columns (wide images)
constexpr int COLS = WIN + 2;                   // LDS pixel slots per ring row: window columns -1 .. WIN
constexpr int XP = 64 + 16;                     // base pixel pitch (bf16): == 16 (mod 32), conflict-free b128 reads
constexpr int DP = 48;                          // dense pixel pitch: out1 | out2 | out3 (== 16 mod 32)
constexpr int XD = 4;                           // base ring rows (y1-1 .. y1+1 read, y1+2 staged)
constexpr int DD = 8;                           // dense ring rows (y1-7 .. y1-1 read, y1 written)
constexpr int XROW = COLS * XP, DROW = COLS * DP;
constexpr int OFF_D = XD * XROW;                // elements
constexpr int OFF_A = OFF_D + DD * DROW;        // dense-part A fragments of levels 3, 4 [block][lane][8 bf16]
constexpr int NDA = 9 + 14;                     // their dense blocks
constexpr int OFF_P = OFF_A + NDA * 512;        // partial sums: per wave 4 (level 3) + 6 (level 4) slots of 64 x f32x4
constexpr int NPS = 4 + 6;
constexpr int LDS_BYTES = OFF_P * 2 + NFR * NPS * 1024;  // 157,440 B
constexpr int XCH = COLS * 8;                   // 16 B chunks of one base row
constexpr int XIT = (XCH + 255) / 256;          // of them per thread
static_assert(LDS_BYTES <= 160 * 1024, "rdb chain LDS");

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
  int n, h, w, rows, strips_y, strips_x, own_w, x_halo;
  uint32_t base_bytes, mask_bytes, out_bytes;
};
typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));

__host__ __device__ constexpr int kp_blocks(int L) { return L == 1 ? 2 : (L == 4 ? 4 : 3); }
__host__ __device__ constexpr int nd_blocks(int L) { return L == 1 ? 0 : (L == 2 ? 5 : (L == 3 ? 9 : 14)); }
__host__ __device__ constexpr int da_base(int L) { return L == 3 ? 0 : 9; }

// The (tap, channel offset in the dense pixel) of lane group g in dense block j of level L; tap < 0: padding
// (zero weights; the B read goes to tap 8 of the same block so every value read is finite).  A block is 32 k: one
// tap of 32 channels (out1|out2), or for a 16-channel group (out1 of level 2, out3 of level 4) PAIRS of taps (lanes
// 0-31 read tap 2p, lanes 32-63 tap 2p+1): 5 blocks instead of 9 half-empty ones.
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

// element offset (from the dense ring) of dense block j of level L for this lane: dr[ky] = ring row y-1+ky, ld / lp
// = this lane's pixel (+ channel group) offsets within a row
template <int L>
__device__ __forceinline__ int dense_off(const int (&dr)[3], int ld, int lp, int g, int j) {
  if (L == 3 || (L == 4 && j < 9)) return dr[j / 3] + ld + (j % 3) * DP;
  const int p = L == 2 ? j : j - 9;
  const int ta = 2 * p, tb = 2 * p + 1 <= 8 ? 2 * p + 1 : 2 * p;
  const int oa = dr[ta / 3] + (ta % 3) * DP, ob = dr[tb / 3] + (tb % 3) * DP;
  return (g >= 2 ? ob : oa) + lp + (L == 2 ? 0 : 32);
}

__device__ __forceinline__ int xslot(int y) { return (y + 64) & (XD - 1); }  // y >= -64
__device__ __forceinline__ int dslot(int y) { return (y + 64) & (DD - 1); }

__device__ __forceinline__ uint32_t pack2_bf16(float a, float b) {
  const bf16x2 v = {(__bf16)a, (__bf16)b};  // v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(uint32_t, v);
}

// The dense part of level L added to acc: B from the ring, A from registers (level 2: ar) or LDS (levels 3, 4).
// Blocks go in groups of 3: the next group's fragments are read while this group is on the MFMA pipe.
template <int L>
__device__ __forceinline__ void dense_acc(const uint16_t* lds, const bf16x8 (&ar)[5], int y, int ld, int lp, int g, int lane,
                                          f32x4& acc) {
  constexpr int NB = nd_blocks(L), G = 3, NG = (NB + G - 1) / G;
  int dr[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) dr[k] = OFF_D + dslot(y - 1 + k) * DROW;
  const uint16_t* ab = lds + OFF_A + da_base(L) * 512 + lane * 8;
  bf16x8 fa[2][G], fb[2][G];
  auto load = [&](int gi, int s) {
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int j = gi * G + i;
      if (j < NB) {
        fa[s][i] = L == 2 ? ar[j < 5 ? j : 0] : *(const bf16x8*)(ab + j * 512);
        fb[s][i] = *(const bf16x8*)(lds + dense_off<L>(dr, ld, lp, g, j));
      }
    }
  };
  load(0, 0);
#pragma unroll
  for (int gi = 0; gi < NG; ++gi) {
    if (gi + 1 < NG) load(gi + 1, (gi + 1) & 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < G; ++i)
      if (gi * G + i < NB) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[gi & 1][i], fb[gi & 1][i], acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Base part of one row for levels 1..M (pn[L-1] += conv_L restricted to the 64 base channels): 18 blocks (tap t = j / 2,
// 32-channel half j % 2), in groups of 3 whose B fragments are read under the previous group's MFMAs; every fragment
// feeds M MFMAs.  The A fragments of levels 1..3 and blocks 0..5 of level 4 come from AGPRs (mfma3_agpr), level 4's
// blocks 6..17 from VGPRs (mfma3_vgpr; the 256 AGPRs hold 60 of the 72).  Every MFMA of the loop is in asm: hipcc must
// never see an MFMA that could make it move an accumulator between the register halves mid-chain.
template <int M>
__device__ __forceinline__ void base_part(const uint16_t* lds, const bf16x8 (&afb)[4][18], const int (&xr)[3], int lx, f32x4 (&pn)[4]) {
  constexpr int G = 3, NG = 18 / G;
  bf16x8 b[2][G];
  auto load = [&](int gi, int st) {
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int j = gi * G + i, t = j >> 1, ky = t / 3, kx = t % 3;
      b[st][i] = *(const bf16x8*)(lds + xr[ky] + lx + kx * XP + (j & 1) * 32);
    }
  };
  load(0, 0);
#pragma unroll
  for (int gi = 0; gi < NG; ++gi) {
    if (gi + 1 < NG) load(gi + 1, (gi + 1) & 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int L = 0; L < M; ++L) {
      if (gi == 0) {
        mfma3_agpr<true>(pn[L], afb[L][0], afb[L][1], afb[L][2], b[0][0], b[0][1], b[0][2]);
      } else if (L < 3 || gi < 2) {
        mfma3_agpr<false>(pn[L], afb[L][gi * G], afb[L][gi * G + 1], afb[L][gi * G + 2], b[gi & 1][0], b[gi & 1][1], b[gi & 1][2]);
      } else {
        mfma3_vgpr(pn[L], afb[L][gi * G], afb[L][gi * G + 1], afb[L][gi * G + 2], b[gi & 1][0], b[gi & 1][1], b[gi & 1][2]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// MODE 0: forward (bias + leaky relu); 1: pull (leaky-relu derivative of the stored activation, no bias).
template <int MODE>
__global__ __launch_bounds__(256, 1) void rdb_chain_wide_kernel(ChainArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* lds = (uint16_t*)smem;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, col = lane & 15;
  const int f = __builtin_amdgcn_readfirstlane(tid >> 6);  // this wave's column fragment
  int bi = blockIdx.x;
  const int sx = bi % a.strips_x;
  bi /= a.strips_x;
  const int sy = bi % a.strips_y, nimg = bi / a.strips_y;
  const int r0 = sy * a.rows, R = min(a.rows, a.h - r0);
  const int c0 = sx * a.own_w, x0 = c0 - a.x_halo;  // window column 0 = image column x0
  const int row0 = nimg * a.h;                       // this image's first row in the batch
  const __amdgpu_buffer_rsrc_t br = buf_rsrc(a.base, a.base_bytes);

  // ---- dense-part A fragments of levels 3, 4 into LDS, lane-linear per block; the dense ring zeroed (its edge slots
  // and the columns of fragments outside the image are the zero padding of the level convs)
  for (int i = tid; i < NDA * 64; i += 256) {
    const int blk = i >> 6, l = i & 63, gg = l >> 4, cc = l & 15;
    const int L = blk < 9 ? 3 : 4, j = blk - (L == 3 ? 0 : 9);
    const int KP = kp_blocks(L) * 32;
    const uint16_t* wp = L == 3 ? a.wt[2] : a.wt[3];
    int tap, ch;
    dense_src(L, j, gg, tap, ch);
    *(bf16x8*)(lds + OFF_A + i * 8) = tap >= 0 ? *(const bf16x8*)(wp + cc * 9 * KP + tap * KP + 64 + ch) : (bf16x8){};
  }
  for (int i = tid; i < DD * DROW / 8; i += 256) *(uint4*)(lds + OFF_D + i * 8) = make_uint4(0, 0, 0, 0);

  // ---- base row staging: chunk q = tid + 256 i of a row is (slot q / 8 = window column + 1, 16 B channel group q % 8)
  int xg[XIT], xl[XIT];
#pragma unroll
  for (int i = 0; i < XIT; ++i) {
    const int q = tid + 256 * i, p = q >> 3, c = q & 7, ix = x0 + p - 1;
    xl[i] = q < XCH ? p * XP + c * 8 : -1;
    xg[i] = q < XCH && ix >= 0 && ix < a.w ? (ix * a.bcs + a.boff + c * 8) * 2 : -1;
  }
  const uint32_t xrow_bytes = (uint32_t)(a.w * a.bcs * 2);
  auto issue_row = [&](int y, uint4 (&v)[XIT]) {
    const bool rok = y >= 0 && y < a.h;
    const uint32_t rb = (uint32_t)(row0 + y) * xrow_bytes;
#pragma unroll
    for (int i = 0; i < XIT; ++i) v[i] = buf_load16(br, rok && xg[i] >= 0 ? rb + (uint32_t)xg[i] : BUF_OOB);
  };
  auto store_row = [&](int y, const uint4 (&v)[XIT]) {
    uint16_t* row = lds + xslot(y) * XROW;
#pragma unroll
    for (int i = 0; i < XIT; ++i)
      if (xl[i] >= 0) *(uint4*)(row + xl[i]) = v[i];
  };
  {
    uint4 v0[XIT], v1[XIT], v2[XIT];
    issue_row(r0 - 4, v0);
    issue_row(r0 - 3, v1);
    issue_row(r0 - 2, v2);
    store_row(r0 - 4, v0);
    store_row(r0 - 3, v1);
    store_row(r0 - 2, v2);
  }

  // ---- base-part A fragments of the four levels, kept in registers for the whole launch
  bf16x8 afb[4][18];
#pragma unroll
  for (int L = 0; L < 4; ++L) {
    const int KP = kp_blocks(L + 1) * 32;
    const uint16_t* wr = a.wt[L] + col * 9 * KP;
#pragma unroll
    for (int j = 0; j < 18; ++j) afb[L][j] = *(const bf16x8*)(wr + (j >> 1) * KP + (j & 1) * 32 + g * 8);
  }
  bf16x8 ad2[5];  // level 2's dense A fragments
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    int tap, ch;
    dense_src(2, j, g, tap, ch);
    ad2[j] = tap >= 0 ? *(const bf16x8*)(a.wt[1] + col * 9 * 96 + tap * 96 + 64 + ch) : (bf16x8){};
  }
  float bias[4][4];
#pragma unroll
  for (int L = 0; L < 4; ++L) {
    const float4 b4 = MODE == 0 ? *(const float4*)(a.bias[L] + 4 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
    bias[L][0] = b4.x; bias[L][1] = b4.y; bias[L][2] = b4.z; bias[L][3] = b4.w;
  }
  lds_barrier();

  // this lane's pixel: window column px = 16 f + col = image column x
  const int px = 16 * f + col, x = x0 + px;
  const bool fact = x0 + 16 * f < a.w && x0 + 16 * f + 16 > 0;  // wave-uniform: the fragment touches the image
  const bool xin = x >= 0 && x < a.w, xown = xin && x >= c0 && x < c0 + a.own_w;
  const int lx = px * XP + 8 * g;                      // + kx * XP: window column px - 1 + kx sits in slot px + kx
  const int ld = px * DP + 8 * g, lp = px * DP + 8 * (g & 1);
  const int dl = (px + 1) * DP + 4 * g;                // dense-ring store (+ 16 (L-1))
  const __amdgpu_buffer_rsrc_t orr = buf_rsrc(a.out, a.out_bytes);
  const __amdgpu_buffer_rsrc_t mr = buf_rsrc(a.mask, MODE == 1 ? a.mask_bytes : 0u);

  // partial sums (base part) of rows still to finish: level 2 in registers (P2e / P2o: the row of the last even / odd
  // step), levels 3 / 4 in this wave's LDS slots (row of step s in slot s % 4 / s % 6)
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  f32x4 P2e = z4, P2o = z4;
  f32x4* ps = (f32x4*)(smem + OFF_P * 2 + f * (NPS * 1024)) + lane;  // slot k: ps[64 k]

  // level L's epilogue for row y: leaky relu (forward, + bias) or its derivative from the stored activation (pull);
  // zeros outside the image (the next level's padding); the dense-ring store (levels 1..3) and the HBM store of the
  // strip's own pixels, a raw buffer store issued unconditionally (an out-of-range offset drops it)
  auto finish = [&](int L, int y, bool act, const f32x4& acc, uint2 m) {
    const bool in = act && xin && y >= 0 && y < a.h;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float t = acc[i] + bias[L - 1][i];
      if (MODE == 0) {
        v[i] = fmaxf(t, t * a.slope);  // leaky relu, 0 <= slope <= 1 (checked on the host)
      } else {
        const uint32_t mw = i < 2 ? m.x : m.y;
        const float mv = __uint_as_float((i & 1) ? (mw & 0xFFFF0000u) : (mw << 16));  // the stored activation
        v[i] = mv > 0.f ? t : t * a.slope;
      }
    }
    uint2 pk = make_uint2(pack2_bf16(v[0], v[1]), pack2_bf16(v[2], v[3]));
    if (!in) pk = make_uint2(0, 0);
    if (L < 4 && act && fact) *(uint2*)(lds + OFF_D + dslot(y) * DROW + dl + 16 * (L - 1)) = pk;
    const bool own = in && xown && y >= r0 && y < r0 + R;
    const uint32_t ob = (uint32_t)(((long)(row0 + y) * a.w + x) * a.ocs + a.ooff[L - 1] + 4 * g) * 2u;
    __builtin_amdgcn_raw_buffer_store_b64((v2u32){pk.x, pk.y}, orr, own ? ob : BUF_OOB, 0, 0);
  };

  // pull: the stored activations of the four levels' rows in step s (issued a step ahead)
  auto issue_mask = [&](int s, uint2 (&mk)[4]) {
    if constexpr (MODE == 1) {
      const int y1 = r0 - 3 + s;
#pragma unroll
      for (int L = 1; L <= 4; ++L) {
        const int y = y1 - 2 * (L - 1);
        const bool ok = xin && y >= 0 && y < a.h;
        const uint32_t mo = (uint32_t)(((long)(row0 + y) * a.w + x) * a.mcs + a.moff[L - 1] + 4 * g) * 2u;
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(mr, ok ? mo : BUF_OOB, 0, 0);
        mk[L - 1] = make_uint2(v[0], v[1]);
      }
    }
  };

  // step s: base rows are loaded two steps before they are staged (row y1 + 2, stored at the end of step s, was issued
  // in step s - 1 into cur; row y1 + 3 goes into nxt now) and the pull's activation rows one step before their use,
  // so the HBM latency hides under a step's MFMAs
  auto step = [&](int s, f32x4& P2, uint4 (&cur)[XIT], uint4 (&nxt)[XIT], const uint2 (&mk)[4], uint2 (&mkn)[4]) {
    const int y1 = r0 - 3 + s;
    issue_row(y1 + 3, nxt);
    issue_mask(s + 1, mkn);
    // levels whose base part is computed in this step: level L's rows are computed 2(L-1) steps before it finishes
    // them, for s in [L-1, R + 6 - L] -- always the prefix 1..m of the levels (none for rows outside the image)
    const bool yin = fact && y1 >= 0 && y1 < a.h;
    const int m = yin ? min(4, min(s + 1, R + 6 - s)) : 0;
    // ---- base part of row y1 for levels 1..m: 18 blocks (9 taps x 2 x 32 channels), each B fragment feeding the
    // MFMAs of every such level; one branch-free copy of the loop per m
    f32x4 pn[4];
    if (m > 0) {
      int xr[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) xr[k] = xslot(y1 - 1 + k) * XROW;
      switch (m) {
        case 4: base_part<4>(lds, afb, xr, lx, pn); break;
        case 3: base_part<3>(lds, afb, xr, lx, pn); break;
        case 2: base_part<2>(lds, afb, xr, lx, pn); break;
        default: base_part<1>(lds, afb, xr, lx, pn); break;
      }
      pad_mfma(pn);
    }
    // levels past m: zero partials
#pragma unroll
    for (int L = 0; L < 4; ++L)
      if (L >= m) pn[L] = z4;
    // ---- level 1 (row y1): base part only
    finish(1, y1, s <= R + 5, pn[0], mk[0]);
    // ---- level 2 (row y1 - 2), 3 (y1 - 4), 4 (y1 - 6): + the dense part from the ring (rows of earlier steps)
    const bool a2 = s >= 3 && s <= R + 6, a3 = s >= 6 && s <= R + 7, a4 = s >= 9 && s <= R + 8;
    f32x4* p3 = ps + 64 * (s & 3);        // level 3: the row of step s - 4 (read), then this step's row (written)
    f32x4* p4 = ps + 64 * (4 + s % 6);    // level 4: the row of step s - 6, then this step's
    {
      f32x4 acc = P2;  // the row of step s - 2 (same parity)
      if (a2 && fact) dense_acc<2>(lds, ad2, y1 - 2, ld, lp, g, lane, acc);
      finish(2, y1 - 2, a2, acc, mk[1]);
    }
    {
      f32x4 acc = a3 ? *p3 : z4;
      if (a3 && fact) dense_acc<3>(lds, ad2, y1 - 4, ld, lp, g, lane, acc);
      finish(3, y1 - 4, a3, acc, mk[2]);
    }
    {
      f32x4 acc = a4 ? *p4 : z4;
      if (a4 && fact) dense_acc<4>(lds, ad2, y1 - 6, ld, lp, g, lane, acc);
      finish(4, y1 - 6, a4, acc, mk[3]);
    }
    P2 = pn[1];
    *p3 = pn[2];  // (this wave's own slots: no barrier between its read and its write)
    *p4 = pn[3];
    store_row(y1 + 2, cur);  // its slot held row y1 - 2, which no level reads in this step
    lds_barrier();
  };
  uint4 ra[XIT], rb[XIT];
  uint2 ma[4] = {}, mb[4] = {};
  issue_row(r0 - 1, ra);
  issue_mask(0, ma);
  for (int s = 0; s < R + 9; s += 2) {
    step(s, P2e, ra, rb, ma, mb);
    if (s + 1 < R + 9) step(s + 1, P2o, rb, ra, mb, ma);
  }
}

}  // namespace

namespace climsr {
int rdb_chain_narrow(const ClimsrChainDesc* d, hipStream_t stream);
}

static bool narrow_width(int w) { return w <= 64 && w % 16 == 0; }

extern "C" const char* climsr_rdb_chain_kernel(const ClimsrChainDesc* d) {
  if (!d || d->w <= 0) return "";
  if (narrow_width(d->w)) return d->act == 1 ? "rdb_chain_rr_kernel<0>" : "rdb_chain_rr_kernel<1>";
  return d->act == 1 ? "rdb_chain_wide_kernel<0>" : "rdb_chain_wide_kernel<1>";
}

extern "C" int climsr_rdb_chain(const ClimsrChainDesc* d, void* stream) {
  if (!d || !d->base || !d->out || d->n <= 0 || d->h <= 0 || d->w <= 0 || d->bcs % 8 || d->boff % 8 || d->ocs % 4 ||
      (d->act != 1 && d->act != 3) || (d->act == 3 && (!d->mask || d->mcs % 4)) || !(d->slope >= 0.f && d->slope <= 1.f)) {
    set_error("rdb_chain: bad args");
    return CLIMSR_EINVAL;
  }
  for (int L = 0; L < 4; ++L) {
    if (!d->wt[L] || d->ooff[L] % 4 || (d->act == 1 && !d->bias[L]) || (d->act == 3 && d->moff[L] % 4)) {
      set_error("rdb_chain: bad level %d", L + 1);
      return CLIMSR_EINVAL;
    }
  }
  const long px = (long)d->n * d->h * d->w;
  if (px * d->bcs * 2 >= (1L << 31) || px * d->ocs * 2 >= (1L << 31) || (d->act == 3 && px * d->mcs * 2 >= (1L << 31))) {
    set_error("rdb_chain: tensors over 2 GiB");
    return CLIMSR_EINVAL;
  }
  if (narrow_width(d->w)) return rdb_chain_narrow(d, (hipStream_t)stream);
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
  // columns: one window when the image fits it, else strips of WIN - 2 HALO_X own columns
  if (d->w <= WIN) {
    a.strips_x = 1; a.own_w = d->w; a.x_halo = 0;
  } else {
    a.own_w = WIN - 2 * HALO_X; a.x_halo = HALO_X; a.strips_x = ceil_div(d->w, a.own_w);
  }
  // rows: about one strip per CU (a strip recomputes 3 + 2 + 1 halo rows per level chain)
  const int ncu = device_cus();
  const long bands = (long)d->n * a.strips_x;
  int rows = ceil_div(bands * d->h, ncu);
  if (rows < 2) rows = 2;
  if (rows > 64) rows = 64;
  if (rows > d->h) rows = d->h;
  a.rows = rows;
  a.strips_y = ceil_div(d->h, rows);
  const long grid = bands * a.strips_y;
  if (grid >= (1L << 31)) {
    set_error("rdb_chain: grid too large");
    return CLIMSR_EINVAL;
  }
  if (d->act == 1) {
    if (int e = lds_opt_in((const void*)rdb_chain_wide_kernel<0>, LDS_BYTES)) return e;
    hipLaunchKernelGGL(rdb_chain_wide_kernel<0>, dim3((unsigned)grid), dim3(256), LDS_BYTES, (hipStream_t)stream, a);
  } else {
    if (int e = lds_opt_in((const void*)rdb_chain_wide_kernel<1>, LDS_BYTES)) return e;
    hipLaunchKernelGGL(rdb_chain_wide_kernel<1>, dim3((unsigned)grid), dim3(256), LDS_BYTES, (hipStream_t)stream, a);
  }
  return check_launch("rdb_chain");
}

extern "C" int climsr_rdb_chain_kp(int level) { return level >= 1 && level <= 4 ? kp_blocks(level) * 32 : -1; }
