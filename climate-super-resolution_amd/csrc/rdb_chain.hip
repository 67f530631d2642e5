// Residual-dense-block chain: the four 16-output 3x3 convs of an RDB in ONE launch.
//
// Forward (esrgan.py:22-37):   x1 = lrelu(conv1(x)),  x2 = lrelu(conv2([x,x1])),  ...,  x4 = lrelu(conv4([x,x1,x2,x3]))
// Pull backward (the data-gradient chain of the same block, see climsr_hip.h ClimsrPullPackDesc):
//                              dZ4 = lrelu'(x4) * pull4(dZ5),  dZ3 = lrelu'(x3) * pull3([dZ5,dZ4]),  ...
// Both are "level L reads a base tensor (64 ch) plus the outputs of levels < L (16 ch each)".  Run as four
// separate convs, every level re-reads its whole input from HBM and pays a launch; here one workgroup owns a
// 16-row x 32-column output strip and streams down it: wave L computes level L one row per step, lagging
// level L-1 by two rows (so everything it reads was produced in earlier steps), with ring buffers of the
// rows still needed in LDS, the base rows prefetched two steps ahead, and each wave's weights in VGPRs.
// Halo rows / columns of levels 1-3 are recomputed by neighbouring strips; only owned pixels are stored.
// MFMA v_mfma_f32_16x16x32_bf16: A = weights [16 co][32 k], B = 16 pixels of one row x 32 channels.
#include "common.h"

using namespace climsr;

namespace {

constexpr int CH_SW = 32;           // owned output columns per strip
constexpr int CH_R = 16;            // owned output rows per strip
constexpr int CH_COLS = 52;         // LDS columns (image column c0 - 5 + j)
constexpr int CH_BP = 64 + 8;       // base pixel pitch (bf16)
constexpr int CH_OP = 16 + 8;       // 16-channel ring pixel pitch
constexpr int CH_RB = 10;           // base ring rows
constexpr int CH_R1 = 8, CH_R2 = 6, CH_R3 = 4;  // ring rows of levels 1..3
constexpr int CH_STEPS = CH_R + 9;

struct ChainArgs {
  const uint16_t* base;  // bf16 NHWC, 64 channels at boff
  int bcs, boff;
  uint16_t* out;         // bf16 NHWC; level L writes 16 channels at ooff[L-1]
  int ocs;
  int ooff[4];
  const uint16_t* wt[4];  // packed [16][9*KP_L] (k = tap*KP_L + c), channel order base | out1 | out2 | out3
  const float* bias[4];  // forward: conv biases; pull: null
  const uint16_t* mask;  // pull: activation outputs x_j (act 3), level L uses channels moff[L-1]
  int mcs;
  int moff[4];
  int act;               // 1 = leaky relu (forward), 3 = leaky relu backward with mask
  float slope;
  int n, h, w, strips_x, strips_y;
};

__host__ __device__ constexpr int kp_blocks(int L) { return L == 1 ? 2 : (L == 4 ? 4 : 3); }

// LDS layout (bf16 elements)
constexpr int OFF_BASE = 0;
constexpr int OFF_R1 = OFF_BASE + CH_RB * CH_COLS * CH_BP;
constexpr int OFF_R2 = OFF_R1 + CH_R1 * CH_COLS * CH_OP;
constexpr int OFF_R3 = OFF_R2 + CH_R2 * CH_COLS * CH_OP;
constexpr int OFF_ZERO = OFF_R3 + CH_R3 * CH_COLS * CH_OP;
constexpr int LDS_ELEMS = OFF_ZERO + 40 * CH_OP;  // zero block covers every fragment offset

__device__ __forceinline__ int wrap(int r, int m) { return ((r % m) + m) % m; }

// One level's row: acc over its K blocks, 3 frags of 16 columns (level 4: 2)
// Fragments [F0, F0 + NF) of level L's row y (a level computes 3 fragments of 16 columns, level 4 two)
template <int L, int F0, int NF>
__device__ __forceinline__ void level_row(const ChainArgs& a, const uint16_t* lds, uint16_t* ldsw, const bf16x8 (&af)[9][4],
                                          int lane, int nimg, int r0, int c0, int y, const uint2 (&mk)[2]) {
  constexpr int NB = kp_blocks(L);
  constexpr int col0 = (L == 4 ? 5 : L) + 16 * F0;  // first LDS column of this wave's fragments
  const int g = lane >> 4, col = lane & 15;
  f32x4 acc[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) acc[f] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const int yy = y + ky - 1;
    const int sb = wrap(yy, CH_RB), s1 = wrap(yy, CH_R1), s2 = wrap(yy, CH_R2), s3 = wrap(yy, CH_R3);
    // per-lane row pointers of this ky; every (kx, fragment, block) read is then a compile-time offset
    const int cc = col0 + col - 1;
    const uint16_t* pb = lds + OFF_BASE + (sb * CH_COLS + cc) * CH_BP + g * 8;
    const uint16_t* p2 = g < 2 ? lds + OFF_R1 + (s1 * CH_COLS + cc) * CH_OP + g * 8
                               : (L >= 3 ? lds + OFF_R2 + (s2 * CH_COLS + cc) * CH_OP + (g - 2) * 8 : lds + OFF_ZERO);
    const uint16_t* p3 = g < 2 ? lds + OFF_R3 + (s3 * CH_COLS + cc) * CH_OP + g * 8 : lds + OFF_ZERO;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      bf16x8 b[NB][NF];
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const int dx = kx + 16 * f;
#pragma unroll
        for (int blk = 0; blk < NB; ++blk) {
          if (blk < 2) b[blk][f] = *(const bf16x8*)(pb + dx * CH_BP + blk * 32);
          else if (blk == 2) b[blk][f] = *(const bf16x8*)(p2 + dx * CH_OP);
          else b[blk][f] = *(const bf16x8*)(p3 + dx * CH_OP);
        }
      }
#pragma unroll
      for (int blk = 0; blk < NB; ++blk)
#pragma unroll
        for (int f = 0; f < NF; ++f)
          acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ky * 3 + kx][blk], b[blk][f], acc[f], 0, 0, 0);
    }
  }
  // epilogue: lane holds channels 4g..4g+3 of column col0 + 16 f + col, row y
  const int co = 4 * g;
  float bb[4] = {0.f, 0.f, 0.f, 0.f};
  if (a.bias[L - 1]) {
    const float4 t = *(const float4*)(a.bias[L - 1] + co);
    bb[0] = t.x; bb[1] = t.y; bb[2] = t.z; bb[3] = t.w;
  }
  const bool row_in = y >= 0 && y < a.h;
  const bool own_row = y >= r0 && y < r0 + CH_R && row_in;
  uint16_t* ring = L == 1 ? ldsw + OFF_R1 : (L == 2 ? ldsw + OFF_R2 : ldsw + OFF_R3);
  const int rs = L == 1 ? CH_R1 : (L == 2 ? CH_R2 : CH_R3);
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const int cx = col0 + 16 * f + col;
    const int ix = c0 - 5 + cx;
    const bool in = row_in && ix >= 0 && ix < a.w;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float t = acc[f][i] + bb[i];
      if (a.act == 1) t = t > 0.f ? t : t * a.slope;
      else if (a.act == 3) {
        const uint32_t mw = i < 2 ? mk[f].x : mk[f].y;
        const float m = bf2f((uint16_t)((i & 1) ? (mw >> 16) : mw));
        t = m > 0.f ? t : t * a.slope;
      }
      v[i] = in ? t : 0.f;  // outside the image: zero padding for the next levels
    }
    uint2 pk;
    pk.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    pk.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    if (L < 4) *(uint2*)(ring + (wrap(y, rs) * CH_COLS + cx) * CH_OP + co) = pk;
    if (own_row && in && cx >= 5 && cx < 5 + CH_SW)
      *(uint2*)(a.out + (((long)nimg * a.h + y) * a.w + ix) * a.ocs + a.ooff[L - 1] + co) = pk;
  }
}

template <int L>
__device__ __forceinline__ void load_af(const ChainArgs& a, int lane, bf16x8 (&af)[9][4]) {
  constexpr int NB = kp_blocks(L), KP = NB * 32;
  const int g = lane >> 4, col = lane & 15;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int blk = 0; blk < 4; ++blk)
      af[t][blk] = blk < NB ? *(const bf16x8*)(a.wt[L - 1] + (long)col * 9 * KP + t * KP + blk * 32 + g * 8) : (bf16x8){};
}

// mask (act 3) of level L's row y for this lane's 3 fragments, loaded before the MFMAs of the step
template <int L, int F0, int NF>
__device__ __forceinline__ void load_mask(const ChainArgs& a, int lane, int nimg, int c0, int y, uint2 (&mk)[2]) {
  constexpr int col0 = (L == 4 ? 5 : L) + 16 * F0;
  const int g = lane >> 4, col = lane & 15;
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    mk[f] = make_uint2(0, 0);
    const int ix = c0 - 5 + col0 + 16 * f + col;
    if (f < NF && a.act == 3 && y >= 0 && y < a.h && ix >= 0 && ix < a.w)
      mk[f] = *(const uint2*)(a.mask + (((long)nimg * a.h + y) * a.w + ix) * a.mcs + a.moff[L - 1] + 4 * g);
  }
}

// Wave w (8 per workgroup, two per SIMD) computes level (w & 3) + 1; w < 4 takes its first two fragments
// (level 4: the first), w >= 4 the rest.
template <int L, int HALF>
__device__ __forceinline__ void wave_step(const ChainArgs& a, uint16_t* lds, const bf16x8 (&af)[9][4], int lane, int nimg, int r0,
                                          int c0, int y) {
  constexpr int F0 = HALF == 0 ? 0 : (L == 4 ? 1 : 2);
  constexpr int NF = HALF == 0 ? (L == 4 ? 1 : 2) : 1;
  uint2 mk[2];
  load_mask<L, F0, NF>(a, lane, nimg, c0, y, mk);
  level_row<L, F0, NF>(a, lds, lds, af, lane, nimg, r0, c0, y, mk);
}

__global__ __launch_bounds__(512, 1) void rdb_chain_kernel(ChainArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* lds = (uint16_t*)smem;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  int bid = blockIdx.x;
  const int sx = bid % a.strips_x;
  bid /= a.strips_x;
  const int sy = bid % a.strips_y;
  const int nimg = bid / a.strips_y;
  const int c0 = sx * CH_SW, r0 = sy * CH_R;
  const int L = (wave & 3) + 1;

  for (int i = tid; i < LDS_ELEMS / 8; i += 512) *(uint4*)(lds + i * 8) = make_uint4(0, 0, 0, 0);

  bf16x8 af[9][4];
  switch (L) {
    case 1: load_af<1>(a, lane, af); break;
    case 2: load_af<2>(a, lane, af); break;
    case 3: load_af<3>(a, lane, af); break;
    default: load_af<4>(a, lane, af); break;
  }

  // base staging: one LDS row = CH_COLS x 8 vectors (416), one per thread
  auto load_base = [&](int yy, uint4& pre) {
    const int cx = tid >> 3, cg = tid & 7;
    const int ix = c0 - 5 + cx;
    pre = make_uint4(0, 0, 0, 0);
    if (tid < CH_COLS * 8 && yy >= 0 && yy < a.h && ix >= 0 && ix < a.w)
      pre = *(const uint4*)(a.base + (((long)nimg * a.h + yy) * a.w + ix) * a.bcs + a.boff + cg * 8);
  };
  auto store_base = [&](int yy, const uint4& pre) {
    if (tid < CH_COLS * 8) *(uint4*)(lds + OFF_BASE + (wrap(yy, CH_RB) * CH_COLS + (tid >> 3)) * CH_BP + (tid & 7) * 8) = pre;
  };
  __syncthreads();  // zero fill done
  // prologue: base rows r0-4 .. r0-2 (level 1's first row r0-3 reads r0-4..r0-2)
  for (int yy = r0 - 4; yy <= r0 - 2; ++yy) {
    uint4 pre;
    load_base(yy, pre);
    store_base(yy, pre);
  }
  uint4 pa, pb;  // base rows for steps s+1 and s+2
  load_base(r0 - 1, pa);
  load_base(r0, pb);
  __syncthreads();

  for (int s = 0; s < CH_STEPS; ++s) {
    // level L computes row y_L = r0 - 3 + s - 2(L-1) during steps 3L-3 .. R+L+4
    const int y = r0 - 3 + s - 2 * (L - 1);
    if (s >= 3 * L - 3 && s <= CH_R + L + 4) {
      switch (wave) {
        case 0: wave_step<1, 0>(a, lds, af, lane, nimg, r0, c0, y); break;
        case 1: wave_step<2, 0>(a, lds, af, lane, nimg, r0, c0, y); break;
        case 2: wave_step<3, 0>(a, lds, af, lane, nimg, r0, c0, y); break;
        case 3: wave_step<4, 0>(a, lds, af, lane, nimg, r0, c0, y); break;
        case 4: wave_step<1, 1>(a, lds, af, lane, nimg, r0, c0, y); break;
        case 5: wave_step<2, 1>(a, lds, af, lane, nimg, r0, c0, y); break;
        case 6: wave_step<3, 1>(a, lds, af, lane, nimg, r0, c0, y); break;
        default: wave_step<4, 1>(a, lds, af, lane, nimg, r0, c0, y); break;
      }
    }
    // base row needed from step s+1 on (level 1 at step s+1 reads up to row r0 - 1 + s)
    store_base(r0 - 1 + s, pa);
    pa = pb;
    load_base(r0 + 1 + s, pb);
    __syncthreads();
  }
}

}  // namespace

extern "C" int climsr_rdb_chain(const ClimsrChainDesc* d, void* stream) {
  if (!d || !d->base || !d->out || d->n <= 0 || d->h <= 0 || d->w <= 0 || d->bcs % 8 || d->boff % 8 || d->ocs % 4 ||
      (d->act != 1 && d->act != 3) || (d->act == 3 && (!d->mask || d->mcs % 4))) {
    set_error("rdb_chain: bad args");
    return CLIMSR_EINVAL;
  }
  for (int L = 0; L < 4; ++L) {
    if (!d->wt[L] || d->ooff[L] % 4 || (d->act == 3 && d->moff[L] % 4)) {
      set_error("rdb_chain: bad level %d", L + 1);
      return CLIMSR_EINVAL;
    }
  }
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
  a.act = d->act; a.slope = d->slope;
  a.n = d->n; a.h = d->h; a.w = d->w;
  a.strips_x = ceil_div(d->w, CH_SW);
  a.strips_y = ceil_div(d->h, CH_R);
  const size_t lds = (size_t)LDS_ELEMS * 2;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)rdb_chain_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  hipLaunchKernelGGL(rdb_chain_kernel, dim3(a.strips_x * a.strips_y * a.n), dim3(512), lds, (hipStream_t)stream, a);
  return check_launch("rdb_chain");
}

extern "C" int climsr_rdb_chain_kp(int level) { return level >= 1 && level <= 4 ? kp_blocks(level) * 32 : -1; }
