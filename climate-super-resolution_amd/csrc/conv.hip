// Implicit-GEMM convolution for CDNA4 (gfx950): forward / data-gradient and weight-gradient.
//
// Replaces nn.Conv2d (+ fused F.interpolate(nearest), LeakyReLU/ReLU, residual adds) on the
// ESRGAN hot path: climsr/models/esrgan.py:17-102, srcnn.py:6-18, rfb_esrgan.py:26-61.
//
// Layout: activations NHWC bf16; a conv reads channels [in_coff, in_coff+in_c) of a buffer with
// in_cstride channels per pixel (the RDB dense concatenation is one 128-channel buffer, so
// torch.cat is free).  GEMM view: M = output channels (MFMA A = packed weights), N = output pixels
// (MFMA B = input pixels staged in LDS, im2col done by LDS addressing), K = taps x channels.
// MFMA: v_mfma_f32_16x16x32_bf16.  Lane l: A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15],
// C[row 4(l>>4)+i][col l&15].
#include <algorithm>
#include <atomic>
#include <mutex>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include "common.h"
#include "conv_ep.h"

namespace climsr {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// dry run (climsr_conv2d_fwd_kernel): the dispatcher records the kernel it would launch instead of launching
thread_local bool g_dry = false;
thread_local char g_dry_name[96] = "";

// true (and the kernel's name recorded) when the dispatcher runs dry: the caller returns before launching
bool dry_run(const char* fmt, ...) {
  if (!g_dry) return false;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_dry_name, sizeof(g_dry_name), fmt, ap);
  va_end(ap);
  return true;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return CLIMSR_EHIP;
  }
  return CLIMSR_OK;
}

// Per-device launch facts, shared by every dispatcher (one process may drive several devices from several threads):
// the CU count of the CURRENT device and the dynamic-LDS opt-in of a kernel on it, each settled once per device
// under a mutex; readers of a settled entry take no lock.
static constexpr int MAX_DEV = 64;
static std::mutex g_rt_mu;
static std::atomic<int> g_ncu[MAX_DEV];

static int current_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEV) dev = 0;
  return dev;
}

int device_cus() {
  const int dev = current_device();
  int n = g_ncu[dev].load(std::memory_order_acquire);
  if (n > 0) return n;
  std::lock_guard<std::mutex> lk(g_rt_mu);
  n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  g_ncu[dev].store(n, std::memory_order_release);
  return n;
}

int lds_opt_in(const void* fn, int bytes) {
  struct Key {
    const void* fn;
    int dev;
  };
  static Key done[1024];
  static std::atomic<int> ndone{0};
  const int dev = current_device();
  const int seen = ndone.load(std::memory_order_acquire);
  for (int i = 0; i < seen; ++i)
    if (done[i].fn == fn && done[i].dev == dev) return CLIMSR_OK;
  std::lock_guard<std::mutex> lk(g_rt_mu);
  const int m = ndone.load(std::memory_order_relaxed);
  for (int i = 0; i < m; ++i)
    if (done[i].fn == fn && done[i].dev == dev) return CLIMSR_OK;
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e != hipSuccess) {
    set_error("hipFuncSetAttribute(MaxDynamicSharedMemorySize=%d): %s", bytes, hipGetErrorString(e));
    return CLIMSR_EHIP;
  }
  if (m < 1024) {
    done[m] = Key{fn, dev};
    ndone.store(m + 1, std::memory_order_release);
  }
  return CLIMSR_OK;
}

// ------------------------------------------------------------------------------------------
// Tiling constants
// ------------------------------------------------------------------------------------------
// LDS pitches of the staged operand tiles.  A 16 x 32-channel MFMA fragment is read with ds_read_b128 (lane
// 16g + col: row col, channels 8g..8g+7); its four 16-lane bank groups are conflict-free when the row pitch
// is 16 (mod 32) bf16 elements, and 2-way conflicted at 8 (mod 32) (measured SQ_LDS_BANK_CONFLICT 43 % of
// the LDS cycles of conv5 with the old +8 pads).
static inline int xpitch(int cc) { return cc + ((16 - cc % 32) + 32) % 32; }  // >= cc, == 16 (mod 32)
// Stride 2: a fragment's 16 pixels sit 2 pixels apart in the tile, so the lane pitch is 2 * ccp and ccp == 8 (mod 16)
// keeps it at 16 (mod 32) (the stride-1 pitch left every stride-2 read 4-way conflicted: SQ_LDS_BANK_CONFLICT 35 %).
static inline int xpitch_s2(int cc) { return cc + ((8 - cc % 16) + 16) % 16; }
constexpr int WPAD = 16;          // k padding of the LDS weight tile rows (kcpad is a multiple of 32)
constexpr int FWD_LDS_BUDGET = 80 * 1024;  // two workgroups per CU
constexpr int FWD_MAXV = 8;             // 16 B staging vectors per thread held in registers (prefetch)

struct FwdGeom {
  int th, tph, tpw, ccp, kc, kcpad, nchunk, kpk, nt, mw;
  size_t lds_tab, lds_x, lds_w, lds_total;
};

static int fwd_nt(int out_c) {
  int nt = (out_c + 15) / 16;
  return nt > 4 ? 4 : (nt == 3 ? 4 : nt);
}

__device__ inline int climsr_rows_dev(int out_c) {
  int nt = (out_c + 15) / 16;
  nt = nt > 4 ? 4 : (nt == 3 ? 4 : nt);
  return (out_c + nt * 16 - 1) / (nt * 16) * (nt * 16);
}

static void fwd_geom(int in_c, int ks, int stride, int out_c, int cc, int mw, FwdGeom* g) {
  g->mw = mw;
  g->th = 4 * mw;
  g->tph = (g->th - 1) * stride + ks;
  g->tpw = (TW - 1) * stride + ks;
  g->ccp = stride == 2 ? xpitch_s2(cc) : xpitch(cc);
  g->kc = ks * ks * cc;
  g->kcpad = round_up(g->kc, 32);
  g->nchunk = ceil_div(in_c, cc);
  g->kpk = g->nchunk * g->kcpad;
  g->nt = fwd_nt(out_c);
  g->lds_tab = (size_t)(g->kcpad / 8) * 4;
  g->lds_tab = (g->lds_tab + 15) / 16 * 16;
  g->lds_x = (size_t)g->tph * g->tpw * g->ccp * 2;
  g->lds_w = (size_t)g->nt * 16 * (g->kcpad + WPAD) * 2;
  g->lds_total = g->lds_tab + g->lds_x + g->lds_w;
}

}  // namespace climsr

using namespace climsr;

extern "C" const char* climsr_last_error(void) { return g_err; }
extern "C" int climsr_version(void) { return 2; }

// Convs with <= 16 outputs, 3x3 and <= 128 inputs (the residual dense block's conv1-4 and their pull data
// gradients) run on conv_n16_kernel, whose packed K is tap-major with the channels padded to 32 per tap.
static bool n16_shape(int in_c, int ks, int out_c) { return out_c <= 16 && ks == 3 && in_c <= 128; }

static bool pw_fits(int in_c, int ks, int out_c);

extern "C" int climsr_conv_chunk_ex(int in_c, int ks, int out_c, int stride) {
  // <= 4 real input channels (conv_first, srcnn.conv1, VGG conv1_1, RCAN head): taps packed 4 channels apart
  // (conv_pw GEO 2) -- K = ks^2 * 4 instead of ks^2 * 8 (9x9: 11 k-steps instead of 21)
  if (in_c == 4 && stride == 1 && out_c == 64 && (ks == 3 || ks == 9)) return 4;
  if (stride == 1 && n16_shape(in_c, ks, out_c))  // conv_n16: one chunk, padded to 32/64/128
    return in_c <= 32 ? 32 : (in_c <= 64 ? 64 : 128);
  if (stride == 1 && pw_fits(in_c, ks, out_c)) return round_up(in_c, 8);  // conv_pw: the whole K in one chunk
  int cc = round_up(in_c, 8);
  FwdGeom g;
  while (cc > 8) {
    fwd_geom(in_c, ks, 1, out_c, cc, 4, &g);
    long nvec = (long)g.tph * g.tpw * (cc / 8) + (long)g.nt * 16 * (g.kcpad / 8);
    if (g.lds_total <= (size_t)FWD_LDS_BUDGET) break;
    (void)nvec;
    cc = round_up((cc + 1) / 2, 8);
  }
  return cc;
}

extern "C" int climsr_conv_chunk(int in_c, int ks, int out_c) { return climsr_conv_chunk_ex(in_c, ks, out_c, 1); }

extern "C" int climsr_conv_packed_k(int in_c, int ks, int cc) {
  return ceil_div(in_c, cc) * round_up(ks * ks * cc, 32);
}

extern "C" int climsr_conv_packed_rows(int out_c) {
  int nt = fwd_nt(out_c);
  return round_up(out_c, nt * 16);
}

// ------------------------------------------------------------------------------------------
// Weight packing: fp32 OIHW -> bf16 [co_pad16][nchunk][kcpad], k' = tap*cc + c (zeros elsewhere)
// ------------------------------------------------------------------------------------------
__global__ void pack_kernel(const float* __restrict__ w, int rows, int kpk, int in_c_real, int out_c_real, int ks, int cc,
                            int kcpad, int tflip, uint16_t* __restrict__ out) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)rows * kpk;
  if (idx >= total) return;
  int co = (int)(idx / kpk);
  int kk = (int)(idx % kpk);
  int j = kk / kcpad;
  int kr = kk % kcpad;
  int tap = kr / cc;
  int c = j * cc + kr % cc;
  float v = 0.f;
  int kk2 = ks * ks;
  if (co < out_c_real && tap < kk2 && c < in_c_real) {
    int ky = tap / ks, kx = tap % ks;
    if (!tflip) {
      v = w[(((long)co * in_c_real + c) * ks + ky) * ks + kx];
    } else {  // src W[c][co][ks-1-ky][ks-1-kx] with src dims [in_c_real][out_c_real]
      v = w[(((long)c * out_c_real + co) * ks + (ks - 1 - ky)) * ks + (ks - 1 - kx)];
    }
  }
  out[idx] = f2bf(v);
}

extern "C" int climsr_pack_conv_weight(const float* w, int out_c, int in_c, int in_c_real, int out_c_real, int ks, int cc,
                                       int transpose_flip, uint16_t* wpk, void* stream) {
  if (!w || !wpk || (in_c % 8 && !(in_c == 4 && cc == 4)) || (cc % 8 && cc != 4) || cc <= 0 || ks <= 0) {
    set_error("pack_conv_weight: bad args (in_c=%d cc=%d ks=%d)", in_c, cc, ks);
    return CLIMSR_EINVAL;
  }
  int rows = climsr_conv_packed_rows(out_c);
  int kcpad = round_up(ks * ks * cc, 32);
  int kpk = climsr_conv_packed_k(in_c, ks, cc);
  long total = (long)rows * kpk;
  hipLaunchKernelGGL(pack_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, w, rows, kpk, in_c_real,
                     out_c_real, ks, cc, kcpad, transpose_flip, wpk);
  return check_launch("pack_conv_weight");
}

// Batched form: one launch packs every conv of a network (blockIdx.y = descriptor).  Each thread writes 8
// consecutive packed elements (one 16 B store; cc and kcpad are multiples of 8, so the 8 share the chunk and
// the tap) with 32-bit index math (a packed matrix is < 2^31 elements).
__device__ __forceinline__ uint4 pack8(const float (&v)[8]) {
  uint4 o;
  o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
  o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
  return o;
}
__global__ void pack_batched_kernel(const ClimsrPackDesc* __restrict__ descs) {
  const ClimsrPackDesc d = descs[blockIdx.y];
  const int rows = climsr_rows_dev(d.out_c);
  const int kcpad = (d.ks * d.ks * d.cc + 31) / 32 * 32;
  const int kpk = (d.in_c + d.cc - 1) / d.cc * kcpad;
  const int total8 = rows * kpk / 8, kpk8 = kpk / 8, kc8 = kcpad / 8;
  const int kk2 = d.ks * d.ks;
  for (int i8 = blockIdx.x * blockDim.x + threadIdx.x; i8 < total8; i8 += gridDim.x * blockDim.x) {
    const int co = i8 / kpk8, kk8 = i8 - co * kpk8;
    const int j = kk8 / kc8, kr = (kk8 - j * kc8) * 8;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {  // (cc = 4: the 8 elements span two taps)
      const int tap = (kr + e) / d.cc, c = j * d.cc + (kr + e) - tap * d.cc;
      const bool ok = co < d.out_c_real && tap < kk2;
      const int ky = tap / d.ks, kx = tap - (tap / d.ks) * d.ks;
      v[e] = 0.f;
      if (ok && c < d.in_c_real) {
        if (!d.tflip) v[e] = d.w[((co * d.in_c_real + c) * d.ks + ky) * d.ks + kx];
        else v[e] = d.w[((c * d.out_c_real + co) * d.ks + (d.ks - 1 - ky)) * d.ks + (d.ks - 1 - kx)];
      }
    }
    *(uint4*)(d.out + (long)i8 * 8) = pack8(v);
  }
}

extern "C" int climsr_pack_conv_weights_batched(const ClimsrPackDesc* descs, int ndesc, int64_t max_elems, void* stream) {
  if (!descs || ndesc <= 0 || ndesc > 65535) {
    set_error("pack_conv_weights_batched: bad args");
    return CLIMSR_EINVAL;
  }
  int gx = ceil_div(max_elems / 8, 256);
  if (gx > 64) gx = 64;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL(pack_batched_kernel, dim3(gx, ndesc), dim3(256), 0, (hipStream_t)stream, descs);
  return check_launch("pack_conv_weights_batched");
}

// Pull data-gradient weights of a residual dense block (see climsr_hip.h), all the pull convs of a network in
// one launch, row-per-workgroup (blockIdx.x strides over the packed rows co, blockIdx.y = descriptor): the
// row's source weights W_s[c][ci_off + co][.][.] are 9 contiguous floats per input channel c, read in
// those runs into an LDS [tap][channel] image (tap flipped), then the packed row is written as coalesced
// 16 B vectors.  (An element-per-thread gather of 8 floats 36*seg_ic bytes apart per output vector took
// 128 us per step for the generator's 165 pull convs.)
constexpr int PULL_ROW_MAX = 4096;  // in_c * ks^2 floats staged per row
__global__ __launch_bounds__(256) void pack_pull_row_kernel(const ClimsrPullPackDesc* __restrict__ descs) {
  __shared__ float img[PULL_ROW_MAX];
  // the segment arrays are indexed dynamically: read them from the descriptor in global memory (a private
  // copy of the struct would live in scratch)
  const ClimsrPullPackDesc* dp = descs + blockIdx.y;
  const ClimsrPullPackDesc d = *dp;
  const int rows = climsr_rows_dev(d.out_c);
  const int kk2 = d.ks * d.ks;
  const int kcpad = (kk2 * d.cc + 31) / 32 * 32;
  const int kpk = (d.in_c + d.cc - 1) / d.cc * kcpad;
  const int kc8 = kcpad / 8;
  const bool staged = d.in_c * kk2 <= PULL_ROW_MAX;
  // source of (channel cabs, source tap t) of row co, 0 past the segments
  auto src_at = [&](int co, int cabs, int t) -> float {
    int c = cabs, s = 0;
    while (s < d.nseg - 1 && c >= dp->seg_oc[s]) c -= dp->seg_oc[s++];
    return c < dp->seg_oc[s] ? dp->seg_w[s][((long)c * dp->seg_ic[s] + d.ci_off + co) * kk2 + t] : 0.f;
  };
  for (int co = blockIdx.x; co < rows; co += gridDim.x) {
    if (staged) {
      __syncthreads();  // the previous row's reads of img are done
      if (co < d.out_c)
        for (int e = threadIdx.x; e < d.in_c * kk2; e += blockDim.x) {
          const int cabs = e / kk2, t = e - cabs * kk2;
          img[(kk2 - 1 - t) * d.in_c + cabs] = src_at(co, cabs, t);  // (ks-1-ky, ks-1-kx) = tap kk2-1-t
        }
      __syncthreads();
    }
    uint16_t* out = d.out + (long)co * kpk;
    for (int i8 = threadIdx.x; i8 < kpk / 8; i8 += blockDim.x) {
      const int j = i8 / kc8, kr = (i8 - j * kc8) * 8;
      const int tap = kr / d.cc, cabs = j * d.cc + kr - tap * d.cc;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool ok = co < d.out_c && tap < kk2 && cabs + e < d.in_c;
        v[e] = !ok ? 0.f : staged ? img[tap * d.in_c + cabs + e] : src_at(co, cabs + e, kk2 - 1 - tap);
      }
      *(uint4*)(out + i8 * 8) = pack8(v);
    }
  }
}

extern "C" int climsr_pack_pull_weights_batched(const ClimsrPullPackDesc* descs, int ndesc, int64_t max_elems, void* stream) {
  if (!descs || ndesc <= 0 || ndesc > 65535) {
    set_error("pack_pull_weights_batched: bad args");
    return CLIMSR_EINVAL;
  }
  (void)max_elems;
  // rows per descriptor are on the device: 64 row slots (the RDB pulls have 16 or 64 rows), more rows loop
  hipLaunchKernelGGL(pack_pull_row_kernel, dim3(64, ndesc), dim3(256), 0, (hipStream_t)stream, descs);
  return check_launch("pack_pull_weights_batched");
}

// PF > 0: software-pipelined chunks.  Chunk j+1's input and weight vectors (at most PFX + PFW per thread) are
// loaded into registers while chunk j is on the MFMA pipe, so a multi-chunk tile (RDB conv5 / pull-x: four
// 32-channel chunks) pays one staging latency instead of one per chunk.
// GEO (host-checked geometry specialisation, 0 = runtime geometry): 1 / 2 = 3x3 taps over 32-channel chunks at
// stride 1 / 2 with 16x16 output tiles (MW 4): every tap / row / fragment LDS offset is a compile-time immediate,
// so the unrolled k-steps read their fragments with no address arithmetic and no tap-table lookup (the runtime
// form waited on a dependent ds_read of the table each k-step, and the compiler then issued the fragment reads
// just before their MFMAs: the compute phase alone ran at ~55 % of the MFMA rate).
template <int MW, int NT, bool RF, int MV, int PFX, int PFW, int EP, int GEO>
__device__ __forceinline__ void conv_fwd_body(const FwdArgs& a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* tab = (int*)smem;
  uint16_t* xs = (uint16_t*)(smem + a.lds_tab);
  uint16_t* ws = (uint16_t*)(smem + a.lds_tab + a.lds_x);

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int g = lane >> 4;
  const int col = lane & 15;

  // (tile, output-channel block): blockIdx, or with xgrp the XCD-major order in which the xgrp channel blocks of a
  // tile are consecutive on one XCD (the x tile is fetched into that L2 once for all of them, not once per XCD)
  // Stagger: the two workgroups that share a CU run the same program and start together, so they stage (global
  // loads, LDS stores, barriers) and compute (MFMA) in lockstep -- diagnostic builds measured staging + MFMA-only
  // times that simply add (VGG 256 @64^2: 141 + 147 us = 288 us).  The second workgroup of each CU (the second
  // dispatch round, [stag_lo, stag_hi)) starts about half a chunk late; the blocks that replace them inherit the
  // offset.  Speed only: nothing depends on which workgroups share a CU.
  if (a.stag_n && (int)blockIdx.x >= a.stag_lo && (int)blockIdx.x < a.stag_hi)
    for (int i = 0; i < a.stag_n; ++i) __builtin_amdgcn_s_sleep(32);
  int tile_id = blockIdx.x, cob = blockIdx.y;
  if (a.xgrp > 0) {
    const int ntile = a.tiles_x * a.tiles_y * a.n, idx = xcd_major(blockIdx.x, gridDim.x);
    const int grp = idx / (ntile * a.xgrp), rem = idx - grp * (ntile * a.xgrp);
    tile_id = rem / a.xgrp;
    cob = grp * a.xgrp + (rem - tile_id * a.xgrp);
  }
  int bid = tile_id;
  const int tx = bid % a.tiles_x;
  bid /= a.tiles_x;
  const int ty = bid % a.tiles_y;
  const int nimg = bid / a.tiles_y;
  const int ox0 = tx * TW;
  const int oy0 = ty * (4 * MW);
  const int co_blk0 = cob * NT * 16;
  const int wpitch = a.kcpad + WPAD;
  const int ks2 = a.ks * a.ks;

  // tap table: LDS element offset of k-group (8 channels) within a chunk
  for (int i = tid; i < (GEO > 0 ? 0 : a.kcpad / 8); i += 256) {
    int kr = i * 8;
    int tap = kr / a.cc;
    int c = kr - tap * a.cc;
    if (tap >= ks2) { tap = 0; c = 0; }
    int ky = tap / a.ks, kx = tap - (tap / a.ks) * a.ks;
    tab[i] = (ky * a.tpw + kx) * a.ccp + c;
  }

  f32x4 acc[MW][NT];
#pragma unroll
  for (int m = 0; m < MW; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[m][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

  int pixbase[MW];
#pragma unroll
  for (int m = 0; m < MW; ++m) pixbase[m] = ((wave * MW + m) * a.stride * a.tpw + col * a.stride) * a.ccp;

  // up = 2: nearest x2 upsample on load (src = j >> 1); up = -2: zero insertion (src = j >> 1 for even j,
  // else 0) = the input of the data gradient of a stride-2 conv
  const int ufac = a.up < 0 ? -a.up : a.up;
  const int lh = a.in_h * ufac, lw = a.in_w * ufac;
  const int iy0 = oy0 * a.stride - a.pad, ix0 = ox0 * a.stride - a.pad;
  const int cvec = a.cc / 8;
  const int dilmask = a.up < 0 ? 1 : 0;
  const int nvec_x = a.tph * a.tpw * cvec;
  const int wvec_row = a.kcpad / 8;
  const int nvec_w = NT * 16 * wvec_row;
  const int upsh = ufac == 2 ? 1 : 0;

  // Staging index math is incremental: each thread's k-th vector is (tid + 256k); the pixel /
  // channel-group / row decomposition of the first one costs a few divisions once per kernel, every
  // later one only adds constants with carries (runtime integer division is ~40 VALU ops).
  const int x_dp = 256 / cvec, x_dc = 256 - x_dp * cvec;  // +256 vectors = x_dp pixels + x_dc groups
  const int x_dy = x_dp / a.tpw, x_dx = x_dp - x_dy * a.tpw;
  const int x_pix0 = tid / cvec, x_cg0 = tid - x_pix0 * cvec;
  const int x_ty0 = x_pix0 / a.tpw, x_tx0 = x_pix0 - x_ty0 * a.tpw;
  const int w_dr = 256 / wvec_row, w_dk = 256 - w_dr * wvec_row;
  const int w_r0 = tid / wvec_row, w_k0 = tid - w_r0 * wvec_row;
  const int nrx = (nvec_x + 255) / 256, nrw = (nvec_w + 255) / 256;
  // k-steps software-pipelined two deep: the fragments of k-step s+1 are read from LDS while the MFMAs of
  // k-step s run (one wave per SIMD pair cannot hide the ds_read latency otherwise)
  auto compute = [&]() {
    if constexpr (GEO > 0) {
      static_assert(MW == 4, "GEO tiles are 16 x 16");
      constexpr int S = GEO, TPW = (TW - 1) * S + 3, CCP = S == 1 ? 48 : 40, WP = 9 * 32 + WPAD;
      const uint16_t* xb = xs + ((wave * MW * TPW + col) * S) * CCP + g * 8;
      const uint16_t* wb = ws + col * WP + g * 8;
      bf16x8 af[2][NT], bf[2][MW];
      auto ld = [&](int k, int b) {
        const int off = ((k / 3) * TPW + (k % 3)) * CCP;
#pragma unroll
        for (int t = 0; t < NT; ++t) af[b][t] = *(const bf16x8*)(wb + t * 16 * WP + k * 32);
#pragma unroll
        for (int m = 0; m < MW; ++m) bf[b][m] = *(const bf16x8*)(xb + m * S * TPW * CCP + off);
      };
      ld(0, 0);
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        if (k + 1 < 9) ld(k + 1, (k + 1) & 1);
        // the next k-step's NT + MW fragment reads go out as one burst ahead of this k-step's MW x NT MFMAs (the
        // compiler otherwise sinks each read next to its first MFMA and waits lgkmcnt(0) there: the LDS latency was
        // exposed at nearly every k-step of the unrolled loop)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < MW; ++m)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[k & 1][t], bf[k & 1][m], acc[m][t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      return;
    }
    const int nks = a.kcpad / 32;
    bf16x8 afA[NT], bfA[MW], afB[NT], bfB[MW];
    auto ld = [&](int ks, bf16x8(&af)[NT], bf16x8(&bf)[MW]) {
      const int off = tab[ks * 4 + g];
#pragma unroll
      for (int t = 0; t < NT; ++t) af[t] = *(const bf16x8*)(ws + (t * 16 + col) * wpitch + ks * 32 + g * 8);
#pragma unroll
      for (int m = 0; m < MW; ++m) bf[m] = *(const bf16x8*)(xs + pixbase[m] + off);
    };
    auto mm = [&](const bf16x8(&af)[NT], const bf16x8(&bf)[MW]) {
#pragma unroll
      for (int m = 0; m < MW; ++m)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bf[m], acc[m][t], 0, 0, 0);
    };
    ld(0, afA, bfA);
    int ks = 0;
    for (; ks + 2 <= nks; ks += 2) {
      ld(ks + 1, afB, bfB);
      mm(afA, bfA);
      ld(ks + 2 < nks ? ks + 2 : nks - 1, afA, bfA);  // unconditional (clamped): no branch around the reads
      mm(afB, bfB);
    }
    if (ks < nks) mm(afA, bfA);  // odd k-step count: the last one is already loaded
  };

  if constexpr (PFX > 0 && GEO == 1) {
    // Compile-time staging geometry (18 x 18-pixel x tile of 4 x 16 B channel vectors, 64 x 36 weight vectors per
    // chunk): each thread's vector i is (tid + 256 i), so its pixel / channel group / weight row are per-thread
    // constants; the chunk-0 byte offset of every vector is computed once (out-of-image vectors get BUF_OOB, which
    // stays out of range at every chunk), and a chunk's loads are buffer loads at offset + j * chunk bytes -- one add
    // per vector.  The runtime-geometry walk below spent ~570 VALU per chunk on index carries, bounds checks and
    // 64-bit addresses (4 VALU per MFMA: the chunk loop was VALU-issue bound, conv5 / pull-x most of all).
    // The host takes GEO 1 only for up == 1, in_c % 32 == 0 and tensors under 2 GiB.
    constexpr int CV = 4, TPWc = TW + 2, CCPc = 48, NXV = (TW + 2) * (TW + 2) * CV, WV = 36, WPc = 9 * 32 + WPAD, NWV = NT * 16 * WV;
    static_assert(PFX * 256 >= NXV && PFW * 256 >= NWV, "GEO 1 staging: not enough prefetch vectors");
    uint4 px[PFX], pw[PFW];
    const int cg8 = (tid & 3) * 8;  // 256 % CV == 0: every vector of a thread has the same channel group
    const __amdgpu_buffer_rsrc_t xr = buf_rsrc(a.x, (uint32_t)((long)a.n * a.in_h * a.in_w * a.in_cs * 2));
    const __amdgpu_buffer_rsrc_t wr = buf_rsrc(a.w, (uint32_t)((long)(cob + 1) * NT * 16 * a.kpk * 2));
    uint32_t xo[PFX], wo[PFW];
#pragma unroll
    for (int i = 0; i < PFX; ++i) {
      const int v = tid + 256 * i, pix = v >> 2, ty_ = pix / TPWc, tx_ = pix - ty_ * TPWc;
      const int iy = iy0 + ty_, ix = ix0 + tx_;
      const bool ok = v < NXV && iy >= 0 && iy < a.in_h && ix >= 0 && ix < a.in_w;
      xo[i] = ok ? (uint32_t)((((nimg * a.in_h + iy) * a.in_w + ix) * a.in_cs + a.in_co + cg8) * 2) : BUF_OOB;
    }
#pragma unroll
    for (int i = 0; i < PFW; ++i) {
      const int v = tid + 256 * i, r = v / WV, kv = v - r * WV;
      wo[i] = v < NWV ? (uint32_t)(((co_blk0 + r) * a.kpk + kv * 8) * 2) : BUF_OOB;
    }
    auto issue = [&](int j) {
#pragma unroll
      for (int i = 0; i < PFX; ++i) px[i] = buf_load16(xr, xo[i] + (uint32_t)j * 64u);
#pragma unroll
      for (int i = 0; i < PFW; ++i) pw[i] = buf_load16(wr, wo[i] + (uint32_t)j * (uint32_t)(a.kcpad * 2));
    };
    auto stash = [&]() {
      // pixel (v >> 2) = (tid >> 2) + 64 i: compile-time steps; lanes past the tile dump into the pad channels 32..39
      // of pixel 0, which no fragment reads
      const int xl0 = (tid >> 2) * CCPc + cg8;
#pragma unroll
      for (int i = 0; i < PFX; ++i) {
        const int v = tid + 256 * i;
        *(uint4*)(xs + ((NXV % 256 == 0 || v < NXV) ? xl0 + 64 * CCPc * i : 32)) = px[i];
      }
#pragma unroll
      for (int i = 0; i < PFW; ++i) {
        const int v = tid + 256 * i, r = v / WV, kv = v - r * WV;
        if (NWV % 256 == 0 || v < NWV) *(uint4*)(ws + r * WPc + kv * 8) = pw[i];
      }
    };
    issue(0);
    for (int j = 0; j < a.nchunk; ++j) {
      lds_barrier();  // chunk j-1's fragment reads are done
      stash();
      if (j + 1 < a.nchunk) issue(j + 1);  // lands while chunk j computes
      lds_barrier();
      compute();
    }
  } else if constexpr (PFX > 0) {
    uint4 px[PFX], pw[PFW];
    auto issue = [&](int j) {
      int ty_ = x_ty0, tx_ = x_tx0, cg = x_cg0;
#pragma unroll
      for (int i = 0; i < PFX; ++i) {
        px[i] = make_uint4(0, 0, 0, 0);
        if (i < nrx && ty_ < a.tph) {
          const int iy = iy0 + ty_, ix = ix0 + tx_;
          const int c = j * a.cc + cg * 8;
          if (iy >= 0 && iy < lh && ix >= 0 && ix < lw && c < a.in_c && !((iy | ix) & dilmask))
            px[i] = *(const uint4*)(a.x + (((long)nimg * a.in_h + (iy >> upsh)) * a.in_w + (ix >> upsh)) * a.in_cs + a.in_co + c);
        }
        cg += x_dc;
        tx_ += x_dx;
        ty_ += x_dy;
        if (cg >= cvec) { cg -= cvec; ++tx_; }
        if (tx_ >= a.tpw) { tx_ -= a.tpw; ++ty_; }
      }
      int r = w_r0, kv = w_k0;
#pragma unroll
      for (int i = 0; i < PFW; ++i) {
        pw[i] = make_uint4(0, 0, 0, 0);
        if (i < nrw && r < NT * 16)
          pw[i] = *(const uint4*)(a.w + (long)(co_blk0 + r) * a.kpk + (long)j * a.kcpad + kv * 8);
        kv += w_dk;
        r += w_dr;
        if (kv >= wvec_row) { kv -= wvec_row; ++r; }
      }
    };
    auto stash = [&]() {
      int ty_ = x_ty0, tx_ = x_tx0, cg = x_cg0;
#pragma unroll
      for (int i = 0; i < PFX; ++i) {
        if (i < nrx && ty_ < a.tph) *(uint4*)(xs + (ty_ * a.tpw + tx_) * a.ccp + cg * 8) = px[i];
        cg += x_dc;
        tx_ += x_dx;
        ty_ += x_dy;
        if (cg >= cvec) { cg -= cvec; ++tx_; }
        if (tx_ >= a.tpw) { tx_ -= a.tpw; ++ty_; }
      }
      int r = w_r0, kv = w_k0;
#pragma unroll
      for (int i = 0; i < PFW; ++i) {
        if (i < nrw && r < NT * 16) *(uint4*)(ws + r * wpitch + kv * 8) = pw[i];
        kv += w_dk;
        r += w_dr;
        if (kv >= wvec_row) { kv -= wvec_row; ++r; }
      }
    };
    issue(0);
    for (int j = 0; j < a.nchunk; ++j) {
      __syncthreads();  // chunk j-1's fragment reads are done
      stash();
      if (j + 1 < a.nchunk) issue(j + 1);  // lands while chunk j computes
      __syncthreads();
      compute();
    }
  } else {
  // batched staging: every thread issues up to MV input + MV weight 16 B global loads before the first
  // LDS store, so a chunk pays ~one memory latency instead of one per vector
  const int nbatch = nrx > nrw ? nrx : nrw;
  for (int j = 0; j < a.nchunk; ++j) {
    __syncthreads();
    int ty_ = x_ty0, tx_ = x_tx0, cg = x_cg0;  // input tile (logical coordinates: upsampled / zero-inserted)
    int r = w_r0, kv = w_k0;                  // weight chunk rows [co_blk0, co_blk0 + 16*NT) x kcpad
    for (int base = 0; base < nbatch; base += MV) {
      uint4 bx[MV], bw[MV];
      int dx[MV], dw[MV];
#pragma unroll
      for (int i = 0; i < MV; ++i) {
        dx[i] = -1;
        if (base + i < nrx && ty_ < a.tph) {
          const int iy = iy0 + ty_, ix = ix0 + tx_;
          const int c = j * a.cc + cg * 8;
          uint4 val = make_uint4(0, 0, 0, 0);
          if (iy >= 0 && iy < lh && ix >= 0 && ix < lw && c < a.in_c && !((iy | ix) & dilmask))
            val = *(const uint4*)(a.x + (((long)nimg * a.in_h + (iy >> upsh)) * a.in_w + (ix >> upsh)) * a.in_cs + a.in_co + c);
          bx[i] = val;
          dx[i] = (ty_ * a.tpw + tx_) * a.ccp + cg * 8;
        }
        cg += x_dc;
        tx_ += x_dx;
        ty_ += x_dy;
        if (cg >= cvec) { cg -= cvec; ++tx_; }
        if (tx_ >= a.tpw) { tx_ -= a.tpw; ++ty_; }
      }
#pragma unroll
      for (int i = 0; i < MV; ++i) {
        dw[i] = -1;
        if (base + i < nrw && r < NT * 16) {
          bw[i] = *(const uint4*)(a.w + (long)(co_blk0 + r) * a.kpk + (long)j * a.kcpad + kv * 8);
          dw[i] = r * wpitch + kv * 8;
        }
        kv += w_dk;
        r += w_dr;
        if (kv >= wvec_row) { kv -= wvec_row; ++r; }
      }
#pragma unroll
      for (int i = 0; i < MV; ++i)
        if (dx[i] >= 0) *(uint4*)(xs + dx[i]) = bx[i];
#pragma unroll
      for (int i = 0; i < MV; ++i)
        if (dw[i] >= 0) *(uint4*)(ws + dw[i]) = bw[i];
    }
    __syncthreads();
    compute();
  }
  }

  // ---------------- epilogue ----------------
  // All global reads of the epilogue (bias, residuals, accumulate targets) are issued for every
  // fragment before the first store, so their latencies overlap instead of serialising.
  const int ox = ox0 + col;
  if (EP == 0 && a.down2) {
    // sum the 2x2 block: rows (m, m+1) are in this wave (MW even, oy0 even); columns pair via lane^1.
    // Optional activation backward (act 3/4, res1 = the activation output at the LOW-res pixel), bf16 or
    // fp32 (=, +=) store and a bf16 aux copy.
    const int dh = a.out_h >> 1, dw = a.out_w >> 1;
    const bool mask = a.act == 3 || a.act == 4;
    float4 old[MW / 2][NT];
    uint2 r1v[MW / 2][NT];
    const __amdgpu_buffer_rsrc_t ry2 = opt_rsrc(a.out_mode == 2 ? a.y : nullptr), rm1 = opt_rsrc(mask ? a.res1 : nullptr);
#pragma unroll
    for (int m = 0; m < MW; m += 2) {
      const int oy = oy0 + wave * MW + m;
      const long pidx = ((long)nimg * dh + (oy >> 1)) * dw + (ox >> 1);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int co = co_blk0 + t * 16 + g * 4;
        const bool ok = (col & 1) == 0 && oy < a.out_h && ox < a.out_w && co + 3 < a.out_c;
        const long q = ok ? pidx : 0;
        const uint4 o4 = buf_load16(ry2, (uint32_t)((q * a.out_cs + (ok ? a.out_co + co : 0)) * 4));
        old[m / 2][t] = make_float4(__uint_as_float(o4.x), __uint_as_float(o4.y), __uint_as_float(o4.z), __uint_as_float(o4.w));
        r1v[m / 2][t] = buf_load8(rm1, (uint32_t)((q * a.r1_cs + (ok ? a.r1_co + co : 0)) * 2));
      }
    }
#pragma unroll
    for (int m = 0; m < MW; m += 2) {
      const int oy = oy0 + wave * MW + m;
      const long pidx = ((long)nimg * dh + (oy >> 1)) * dw + (ox >> 1);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float sm = acc[m][t][i] + acc[m + 1][t][i];
          sm += __shfl_xor(sm, 1);
          v[i] = sm;
        }
        const int co = co_blk0 + t * 16 + g * 4;
        if ((col & 1) == 0 && oy < a.out_h && ox < a.out_w) {
          const long ob = pidx * a.out_cs + a.out_co + co;
          if (co + 3 < a.out_c) {
            const uint4 r1 = make_uint4(r1v[m / 2][t].x, r1v[m / 2][t].y, 0, 0);
            if (mask) {
#pragma unroll
              for (int i = 0; i < 4; ++i) v[i] = ep_res(v[i], a.act, a.slope, true, res4_at(r1, false, i), 1.f, 1.f, false, 0.f, 1.f, 1.f);
            }
            if (a.out_mode == 0) {
              uint2 pk;
              pk.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
              pk.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
              *(uint2*)((uint16_t*)a.y + ob) = pk;
            } else {
              float4 o = old[m / 2][t];
              *(float4*)((float*)a.y + ob) = make_float4(o.x + v[0], o.y + v[1], o.z + v[2], o.w + v[3]);
            }
            if (a.aux) {
              uint2 pk;
              pk.x = (uint32_t)f2bf(a.aux_scale * v[0]) | ((uint32_t)f2bf(a.aux_scale * v[1]) << 16);
              pk.y = (uint32_t)f2bf(a.aux_scale * v[2]) | ((uint32_t)f2bf(a.aux_scale * v[3]) << 16);
              *(uint2*)(a.aux + pidx * a.aux_cs + a.aux_co + co) = pk;
            }
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              if (co + i >= a.out_c) continue;
              float x = v[i];
              if (mask) x = ep_res(x, a.act, a.slope, true, res_at(a.res1, false, pidx * a.r1_cs + a.r1_co + co + i), 1.f, 1.f, false,
                                   0.f, 1.f, 1.f);
              if (a.out_mode == 0) ((uint16_t*)a.y)[ob + i] = f2bf(x);
              else if (a.out_mode == 2) ((float*)a.y)[ob + i] += x;
              else ((float*)a.y)[ob + i] = x;
              if (a.aux) a.aux[pidx * a.aux_cs + a.aux_co + co + i] = f2bf(a.aux_scale * x);
            }
          }
        }
      }
    }
    return;
  }
  // coalesced epilogue: the wave's MW x 16 pixels x 16 NT channels go through its own LDS region
  constexpr int EPP = NT * 16 + 4;  // LDS pitch (floats) of a staged pixel
  float* eb = (float*)smem + wave * (MW * 16 * EPP);
  __syncthreads();  // every wave is done with the staged operands (the regions alias them)
#pragma unroll
  for (int m = 0; m < MW; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t) *(f32x4*)(eb + (m * 16 + col) * EPP + t * 16 + g * 4) = acc[m][t];
  __syncthreads();  // orders the staging writes before the transposed reads (they use another vector type)
  if constexpr (EP == 9 || EP == 10) {
    static_assert(MW == 4 && NT == 4, "BatchNorm partials: 16x16 x 64-channel tiles");
    float ssum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, ssq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    store_tile_lds<RF, MW * 16, NT * 16, 64, EP>(a, eb, EPP, lane, nimg, oy0 + wave * MW, ox0, co_blk0, ssum, ssq);
    bn_tile_partials(a, ssum, ssq, true, wave, lane, tile_id, co_blk0, (float*)smem);
  } else {
    store_tile_lds<RF, MW * 16, NT * 16, 64, EP>(a, eb, EPP, lane, nimg, oy0 + wave * MW, ox0, co_blk0);
  }
}

// two workgroups per CU (<= 80 KiB LDS each): at most 256 registers so that two waves share each SIMD
template <int MW, int NT, bool RF, int MV, int PFX = 0, int PFW = 0, int EP = 0, int GEO = 0>
__global__ __launch_bounds__(256, 2) void conv_fwd_kernel(FwdArgs a) {
  conv_fwd_body<MW, NT, RF, MV, PFX, PFW, EP, GEO>(a);
}
// large stride-2 input tiles (one workgroup per CU): the deep prefetch may use the whole register file
template <int MW, int NT, bool RF, int MV, int PFX = 0, int PFW = 0, int EP = 0, int GEO = 0>
__global__ __launch_bounds__(256) void conv_fwd_wide_kernel(FwdArgs a) {
  conv_fwd_body<MW, NT, RF, MV, PFX, PFW, EP, GEO>(a);
}

// ------------------------------------------------------------------------------------------
// Dense-block conv with <= 16 output channels (RDB conv1-4, esrgan.py:22-25, and their pull data
// gradients): 3x3, stride 1, pad 1, <= 128 input channels.  One 16-row MFMA tile of outputs leaves the
// generic kernel staging- and latency-bound; this one is built for memory-level parallelism:
//  * workgroups are persistent (grid-stride over 8x16-pixel output tiles, 3 per CU) and the NEXT tile's
//    input is loaded into registers while the current one is computed (one pixel per staging thread,
//    compile-time channel offsets: no per-vector index math);
//  * the 4 waves split the K dimension (32-channel blocks; NCB = blocks) x the tile rows (4/NCB groups),
//    so a wave keeps only its 9 weight fragments in VGPRs (loaded once per workgroup);
//  * a B fragment (16 pixels x 32 channels of one input row) is read from LDS once and feeds the three
//    output rows that use it (ky = 0..2);
//  * the per-channel-block partial sums meet in LDS; each wave finishes 2 output rows (fused epilogue).
// Channels are padded to NCB*32 (zero weights, zero LDS pixels).
// ------------------------------------------------------------------------------------------
constexpr int N16_TH = 8;
constexpr int N16_TPH = N16_TH + 2, N16_TPW = TW + 2;

// Persistent tile walk, XCD-aware.  Workgroups are dispatched round-robin over the 8 XCDs and each XCD
// has its own L2, so block b walks a contiguous span of tiles owned by XCD b % 8: tiles that run at the
// same time on one XCD are spatial neighbours and share their input halo rows in that L2.
struct TileWalk {
  int first, step, end;
  __device__ explicit TileWalk(int ntiles) {
    const int grid = (int)gridDim.x, b = (int)blockIdx.x;
    if (grid % 8 == 0 && grid >= 64) {
      const int span = (ntiles + 7) / 8, xcd = b % 8;
      first = xcd * span + b / 8;
      step = grid / 8;
      end = min(ntiles, (xcd + 1) * span);
    } else {
      first = b;
      step = grid;
      end = ntiles;
    }
  }
};

static int n16_ncb(int in_c) { return in_c <= 32 ? 1 : (in_c <= 64 ? 2 : 4); }

// EP: epilogue specialisation (the per-tile epilogue is branch- and SALU-heavy when every option is a runtime
// flag): 0 = generic (runtime flags), 1 = forward (bias + leaky relu, bf16 out), 2 = pull (leaky-relu
// derivative from the bf16 activation res1, no bias, bf16 out).  The host picks 1/2 only when they match.
template <int NCB, int EP>
__global__ __launch_bounds__(256, NCB == 4 ? 2 : 3) void conv_n16_kernel(FwdArgs a) {
  const bool has_bias = EP == 1 ? true : EP == 2 ? false : a.bias != nullptr;
  const bool has_r1 = EP == 1 ? false : EP == 2 ? true : a.res1 != nullptr;
  const bool has_r2 = EP != 0 ? false : a.res2 != nullptr;
  const bool has_aux = EP != 0 ? false : a.aux != nullptr;
  const int out_mode = EP != 0 ? 0 : a.out_mode;
  const int act = EP == 1 ? 1 : EP == 2 ? 3 : a.act;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* xs = (uint16_t*)smem;
  float* part = (float*)smem;  // partial sums [cb][row][lane] (aliases the input tile after compute)
  constexpr int CINP = NCB * 32, P = CINP + 16, CV = CINP / 8;  // P == 16 (mod 32): conflict-free fragment reads
  constexpr int RG = 4 / NCB, MW = N16_TH / RG;  // row groups, output rows per wave
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, col = lane & 15;
  const int cb = wave % NCB, rg = wave / NCB;
  const int cvec = a.in_c / 8, cvec32 = (a.in_c + 31) / 32 * 4;  // real / 32-block-rounded 16 B channel groups

  float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
  const int co = g * 4;
  if (has_bias) {
    bv.x = co < a.out_c ? a.bias[co] : 0.f;
    bv.y = co + 1 < a.out_c ? a.bias[co + 1] : 0.f;
    bv.z = co + 2 < a.out_c ? a.bias[co + 2] : 0.f;
    bv.w = co + 3 < a.out_c ? a.bias[co + 3] : 0.f;
  }
  const int ntiles = a.tiles_x * a.tiles_y * a.n;
  const bool valign = EP != 0 || (((a.out_cs | a.out_co) & 3) == 0 && (!a.res1 || ((a.r1_cs | a.r1_co) & 3) == 0) &&
                                   (!a.res2 || ((a.r2_cs | a.r2_co) & 3) == 0) && co + 3 < a.out_c);

  // staging: vector v = tid + 256 i of the tile is (pixel v / CV, channel group v % CV); CV is a power of
  // two, so consecutive lanes read consecutive 16 B of a pixel (coalesced) and the pad groups (>= cvec)
  // are stored as zeros without a load
  constexpr int NPIX = N16_TPH * N16_TPW, NV = (NPIX * CV + 255) / 256;
  uint4 pre[NV];
  // buffer loads: out-of-image / pad-channel vectors take an out-of-range offset and read as zeros, so the
  // next tile's loads stay in flight through the current tile's compute (no branch, no early vmcnt wait)
  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(a.x, (uint32_t)((long)a.n * a.in_h * a.in_w * a.in_cs * 2));
  auto issue = [&](int tile) {  // tile < 0: no next tile, every lane takes the out-of-range offset
    const bool live = tile >= 0;
    int tt = live ? tile : 0;
    const int tx = tt % a.tiles_x;
    tt /= a.tiles_x;
    const int ty = tt % a.tiles_y;
    const int nimg = tt / a.tiles_y;
    const int iy0 = ty * N16_TH - 1, ix0 = tx * TW - 1;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = tid + 256 * i;
      const int pix = v / CV, j = v % CV;
      const int py = pix / N16_TPW, px = pix - py * N16_TPW;
      const int iy = iy0 + py, ix = ix0 + px;
      const bool ok = live && v < NPIX * CV && j < cvec && iy >= 0 && iy < a.in_h && ix >= 0 && ix < a.in_w;
      const uint32_t off = (uint32_t)(((((nimg * a.in_h + iy) * a.in_w + ix) * a.in_cs) + a.in_co + j * 8) * 2);
      pre[i] = buf_load16(xr, ok ? off : BUF_OOB);
    }
  };
  const TileWalk walk(ntiles);
  if (walk.first < walk.end) issue(walk.first);
  const __amdgpu_buffer_rsrc_t er1 = opt_rsrc(has_r1 ? a.res1 : nullptr), er2 = opt_rsrc(has_r2 ? a.res2 : nullptr),
                               ery = opt_rsrc(out_mode == 2 ? a.y : nullptr);
  // this wave's A fragments (channel block cb, 9 taps; packed rows are tap-major with CINP channels per
  // tap), loaded once per workgroup straight into VGPRs while the first tile's input is in flight
  bf16x8 af[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) af[t] = *(const bf16x8*)(a.w + (long)col * a.kpk + t * CINP + cb * 32 + g * 8);
  // retire them here: the loop below then has no loop-carried VMEM results, and hipcc's wait counting
  // inside it stays exact (no vmcnt(0) before the prefetch can land)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)

  for (int tile = walk.first; tile < walk.end; tile += walk.step) {
    int tt = tile;
    const int tx = tt % a.tiles_x;
    tt /= a.tiles_x;
    const int ty = tt % a.tiles_y;
    const int nimg = tt / a.tiles_y;
    const int oy0 = ty * N16_TH, ox0 = tx * TW;
    lds_barrier();  // the previous tile's LDS reads (partials) are done
    {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int v = tid + 256 * i;
        // channel groups of fully padded 32-channel blocks are never read (their waves skip the MFMAs)
        if (v < NPIX * CV && (v % CV) < cvec32) *(uint4*)(xs + (v / CV) * P + (v % CV) * 8) = pre[i];
      }
    }
    issue(tile + walk.step < walk.end ? tile + walk.step : -1);  // lands while this tile computes (unconditional:
                                                                  // a branch around it makes hipcc drain it)
    lds_barrier();
    f32x4 acc[MW];
#pragma unroll
    for (int m = 0; m < MW; ++m) acc[m] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (cb * 32 < a.in_c) {  // a wave whose 32-channel block is all padding adds zeros
      const uint16_t* xb = xs + ((rg * MW) * N16_TPW + col) * P + cb * 32 + g * 8;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        bf16x8 b[MW + 2];  // all input rows of this kx in flight before the first MFMA
#pragma unroll
        for (int ir = 0; ir < MW + 2; ++ir) b[ir] = *(const bf16x8*)(xb + (ir * N16_TPW + kx) * P);
        __builtin_amdgcn_sched_barrier(0);  // keep the reads batched (the scheduler would re-serialise them)
#pragma unroll
        for (int ir = 0; ir < MW + 2; ++ir)
#pragma unroll
          for (int ky = 0; ky < 3; ++ky) {
            const int m = ir - ky;
            if (m >= 0 && m < MW) acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ky * 3 + kx], b[ir], acc[m], 0, 0, 0);
          }
      }
    }
    lds_barrier();  // input tile reads done: the partials overwrite it
#pragma unroll
    for (int m = 0; m < MW; ++m) *(f32x4*)(part + ((cb * N16_TH + rg * MW + m) * 64 + lane) * 4) = acc[m];
    lds_barrier();
    // epilogue: wave w finishes output rows 2w, 2w+1; lane owns channels co..co+3 of column ox0 + col
    const int ox = ox0 + col;
    f32x4 sum[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      sum[h] = *(const f32x4*)(part + ((0 * N16_TH + wave * 2 + h) * 64 + lane) * 4);
#pragma unroll
      for (int c = 1; c < NCB; ++c) sum[h] += *(const f32x4*)(part + ((c * N16_TH + wave * 2 + h) * 64 + lane) * 4);
    }
    uint2 r1v[2], r2v[2];
    float4 old[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // branch-free (opt_rsrc): both rows' operand loads in flight together
      const int oy = oy0 + wave * 2 + h;
      const bool ld = oy < a.out_h && ox < a.out_w && valign;
      const long pidx = ld ? ((long)nimg * a.out_h + oy) * a.out_w + ox : 0;
      const int c = ld ? co : 0;
      r1v[h] = has_r1 ? buf_load8(er1, (uint32_t)((pidx * a.r1_cs + (ld ? a.r1_co : 0) + c) * 2)) : make_uint2(0, 0);
      r2v[h] = has_r2 ? buf_load8(er2, (uint32_t)((pidx * a.r2_cs + (ld ? a.r2_co : 0) + c) * 2)) : make_uint2(0, 0);
      const uint4 o4 = out_mode == 2 ? buf_load16(ery, (uint32_t)((pidx * a.out_cs + (ld ? a.out_co : 0) + c) * 4))
                                     : make_uint4(0, 0, 0, 0);
      old[h] = make_float4(__uint_as_float(o4.x), __uint_as_float(o4.y), __uint_as_float(o4.z), __uint_as_float(o4.w));
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int oy = oy0 + wave * 2 + h;
      if (oy >= a.out_h || ox >= a.out_w || co >= a.out_c) continue;
      const long pidx = ((long)nimg * a.out_h + oy) * a.out_w + ox;
      const float bb[4] = {bv.x, bv.y, bv.z, bv.w};
      float v[4];
      const long ob = pidx * a.out_cs + a.out_co + co;
      if (valign) {
        const uint4 r1 = make_uint4(r1v[h].x, r1v[h].y, 0, 0), r2 = make_uint4(r2v[h].x, r2v[h].y, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          v[i] = ep_res(act_apply(sum[h][i] + bb[i], act, a.slope), act, a.slope, has_r1, res4_at(r1, false, i), a.alpha1,
                        a.beta1, has_r2, res4_at(r2, false, i), a.alpha2, a.beta2);
        if (out_mode == 0) {
          uint2 pk;
          pk.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          pk.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
          *(uint2*)((uint16_t*)a.y + ob) = pk;
        } else {
          *(float4*)((float*)a.y + ob) = make_float4(old[h].x + v[0], old[h].y + v[1], old[h].z + v[2], old[h].w + v[3]);
        }
        if (has_aux) {
          uint2 pk;
          pk.x = (uint32_t)f2bf(a.aux_scale * v[0]) | ((uint32_t)f2bf(a.aux_scale * v[1]) << 16);
          pk.y = (uint32_t)f2bf(a.aux_scale * v[2]) | ((uint32_t)f2bf(a.aux_scale * v[3]) << 16);
          *(uint2*)(a.aux + pidx * a.aux_cs + a.aux_co + co) = pk;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (co + i >= a.out_c) continue;
          const float r1 = a.res1 ? res_at(a.res1, false, pidx * a.r1_cs + a.r1_co + co + i) : 0.f;
          const float r2 = a.res2 ? res_at(a.res2, false, pidx * a.r2_cs + a.r2_co + co + i) : 0.f;
          const float x = ep_res(act_apply(sum[h][i] + bb[i], a.act, a.slope), a.act, a.slope, a.res1 != nullptr, r1, a.alpha1,
                                 a.beta1, a.res2 != nullptr, r2, a.alpha2, a.beta2);
          if (a.out_mode == 0) ((uint16_t*)a.y)[ob + i] = f2bf(x);
          else if (a.out_mode == 2) ((float*)a.y)[ob + i] += x;
          else ((float*)a.y)[ob + i] = x;
          if (a.aux) a.aux[pidx * a.aux_cs + a.aux_co + co + i] = f2bf(a.aux_scale * x);
        }
      }
    }
  }
}

template <int NCB, int EP>
static int launch_n16(const FwdArgs& a, hipStream_t s) {
  if (g_dry) {
    snprintf(g_dry_name, sizeof(g_dry_name), "conv_n16_kernel<%d, %d>", NCB, EP);
    return CLIMSR_OK;
  }
  auto k = conv_n16_kernel<NCB, EP>;
  size_t lds = (size_t)N16_TPH * N16_TPW * (NCB * 32 + 16) * 2;
  const size_t lds_p = (size_t)NCB * N16_TH * 64 * 16;             // partial sums (aliased)
  if (lds_p > lds) lds = lds_p;
  if (int e = lds_opt_in((const void*)k, 160 * 1024)) return e;
  const int ncu = device_cus();
  static std::atomic<int> occ{0};  // workgroups per CU: a property of the kernel and the architecture
  int per_cu = occ.load(std::memory_order_relaxed);
  if (!per_cu) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k, 256, lds) != hipSuccess || per_cu <= 0) per_cu = 2;
    occ.store(per_cu, std::memory_order_relaxed);
  }
  int ntiles = a.tiles_x * a.tiles_y * a.n;
  int grid = ntiles < per_cu * ncu ? ntiles : per_cu * ncu;
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, s, a);
  return check_launch("conv2d_fwd (n16)");
}

// ------------------------------------------------------------------------------------------
// Single-output-channel conv on MFMA (conv_last 64->1 3x3, srcnn.conv3 32->1 5x5 and the data gradient
// of srcnn.conv1 w.r.t. its first input channel, 64->1 9x9).  The horizontal taps go into the MFMA N
// dimension: per output row y and input column x',
//     T[y][x'][kx] = sum_{ky, ci} x[y + ky - R][x'][ci] * w[ky][kx][ci]        (M = x', N = kx, K = ky x ci)
//     out[y][x]    = sum_kx T[y][x + kx - R][kx]                               (shift-sum through LDS)
// so the 16-wide N tile carries KS useful columns instead of 1 (KS/16 vs 1/16 of the MFMA).  A wave
// computes ROWS output rows x 64 columns (5 M-fragments of x'), streaming its ROWS + KS - 1 input rows straight
// from global memory (16 B per lane, next row in flight during the current row's MFMAs); every input row
// feeds the up-to-KS output rows it touches.  Output row r is complete once input row r + KS - 1 is in: its
// shift-sum and store run right there and its accumulators take row r + KS, so a ring of min(KS, ROWS) rows is
// live -- which lets the 3x3 / 5x5 forms stream 16 rows per wave (input rows fetched 18/16 or 20/16 times instead
// of 6/4 or 8/4: conv_last read 1.76x its input at 4 rows).  Weights sit in VGPRs for the whole wave.
// ------------------------------------------------------------------------------------------
constexpr int CO1M_NF = 5, CO1M_COLS = 64;
template <int KS>
struct Co1m {
  static constexpr int ROWS = KS <= 5 ? 16 : 4;                  // output rows per wave
  static constexpr int NSLOT = KS < ROWS ? KS : ROWS;            // live accumulator rows
};

static bool co1m_shape(const ClimsrConvDesc* d) {
  return d->out_c == 1 && d->stride == 1 && d->up == 1 && (d->ks == 3 || d->ks == 5 || d->ks == 9) && d->pad == d->ks / 2 &&
         d->in_c <= 64 && d->in_c % 8 == 0 && d->cc % 8 == 0 && d->out_h == d->in_h && d->out_w == d->in_w;
}

template <int KS, int NCH>
__global__ __launch_bounds__(256, 2) void conv_co1m_kernel(FwdArgs a) {
  constexpr int R = KS / 2, ROWS = Co1m<KS>::ROWS, NSLOT = Co1m<KS>::NSLOT, NR = ROWS + KS - 1;
  __shared__ float sc[4][CO1M_NF * 16][17];  // per-wave T rows (x' x kx), padded pitch
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, col = lane & 15;
  const int x0 = blockIdx.x * CO1M_COLS, y0 = (blockIdx.y * 4 + wave) * ROWS, nimg = blockIdx.z;
  // B fragments: B[k = ci][n = kx] of tap row ky, channel block c (packed row 0: k = (ci/cc)*kcpad + tap*cc + ci%cc)
  bf16x8 bw[KS][NCH];
#pragma unroll
  for (int ky = 0; ky < KS; ++ky)
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int ci = c * 32 + g * 8;
      bw[ky][c] = (bf16x8){};
      if (col < KS && ci < a.in_c)
        bw[ky][c] = *(const bf16x8*)(a.w + (long)(ci / a.cc) * a.kcpad + (ky * KS + col) * a.cc + (ci % a.cc));
    }
  f32x4 acc[NSLOT][CO1M_NF];
#pragma unroll
  for (int r = 0; r < NSLOT; ++r)
#pragma unroll
    for (int f = 0; f < CO1M_NF; ++f) acc[r][f] = (f32x4){0.f, 0.f, 0.f, 0.f};

  bf16x8 xa[2][CO1M_NF][NCH];
  auto load_row = [&](int buf, int iyr) {
    const int iy = y0 - R + iyr;
    const bool rowok = iy >= 0 && iy < a.in_h;
#pragma unroll
    for (int f = 0; f < CO1M_NF; ++f) {
      const int ix = x0 - R + f * 16 + col;
      const bool ok = rowok && ix >= 0 && ix < a.in_w;
      const long base = (((long)nimg * a.in_h + iy) * a.in_w + ix) * a.in_cs + a.in_co;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int ci = c * 32 + g * 8;
        xa[buf][f][c] = (bf16x8){};
        if (ok && ci < a.in_c) xa[buf][f][c] = *(const bf16x8*)(a.x + base + ci);
      }
    }
  };
  // shift-sum of output row r (slot r % NSLOT): out[x0 + l] = sum_kx T[x' = l + kx][kx]; then the fused epilogue
  // (same as conv_co1_kernel); the slot is cleared for row r + NSLOT
  const float bias = a.bias ? a.bias[0] : 0.f;
  const bool f1 = a.res_f32 & 1;
  auto finish = [&](int r) {
    const int sl = r % NSLOT;
#pragma unroll
    for (int f = 0; f < CO1M_NF; ++f)
#pragma unroll
      for (int i = 0; i < 4; ++i) sc[wave][f * 16 + g * 4 + i][col] = acc[sl][f][i];
#pragma unroll
    for (int f = 0; f < CO1M_NF; ++f) acc[sl][f] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float v = 0.f;
#pragma unroll
    for (int kx = 0; kx < KS; ++kx) v += sc[wave][lane + kx][kx];
    const int oy = y0 + r, ox = x0 + lane;
    if (oy < a.out_h && ox < a.out_w) {
      v = act_apply(v + bias, a.act, a.slope);
      const long pidx = ((long)nimg * a.out_h + oy) * a.out_w + ox;
      const float r1 = a.res1 ? res_at(a.res1, f1, pidx * a.r1_cs + a.r1_co) : 0.f;
      v = ep_res(v, a.act, a.slope, a.res1 != nullptr, r1, a.alpha1, a.beta1, false, 0.f, 1.f, 1.f);
      const long ob = pidx * a.out_cs + a.out_co;
      if (a.out_mode == 0) ((uint16_t*)a.y)[ob] = f2bf(v);
      else if (a.out_mode == 2) ((float*)a.y)[ob] += v;
      else ((float*)a.y)[ob] = v;
      if (a.aux) a.aux[pidx * a.aux_cs + a.aux_co] = f2bf(a.aux_scale * v);
    }
  };
  load_row(0, 0);
#pragma unroll
  for (int iyr = 0; iyr < NR; ++iyr) {
    if (iyr + 1 < NR) load_row((iyr + 1) & 1, iyr + 1);
#pragma unroll
    for (int ky = KS - 1; ky >= 0; --ky) {  // oldest row first: row iyr - KS + 1 completes here
      const int r = iyr - ky;  // output row fed by input row iyr through tap row ky
      if (r < 0 || r >= ROWS) continue;
#pragma unroll
      for (int f = 0; f < CO1M_NF; ++f)
#pragma unroll
        for (int c = 0; c < NCH; ++c)
          acc[r % NSLOT][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[iyr & 1][f][c], bw[ky][c], acc[r % NSLOT][f], 0, 0, 0);
      if (NSLOT < ROWS && ky == KS - 1) finish(r);
    }
  }
  if constexpr (NSLOT == ROWS) {  // no slot reuse (9x9): every row finishes after the stream, as fewer registers stay live
#pragma unroll
    for (int r = 0; r < ROWS; ++r) finish(r);
  }
}

template <int KS, int NCH>
static int launch_co1m(const FwdArgs& a, hipStream_t s) {
  if (g_dry) {
    snprintf(g_dry_name, sizeof(g_dry_name), "conv_co1m_kernel<%d, %d>", KS, NCH);
    return CLIMSR_OK;
  }
  dim3 grid(ceil_div(a.out_w, CO1M_COLS), ceil_div(a.out_h, 4 * Co1m<KS>::ROWS), a.n);
  hipLaunchKernelGGL((conv_co1m_kernel<KS, NCH>), grid, dim3(256), 0, s, a);
  return check_launch("conv2d_fwd (co1m)");
}

static int dispatch_co1m(const ClimsrConvDesc* d, const FwdArgs& a, hipStream_t s) {
  const int nch = d->in_c <= 32 ? 1 : 2;
  switch (d->ks * 10 + nch) {
    case 31: return launch_co1m<3, 1>(a, s);
    case 32: return launch_co1m<3, 2>(a, s);
    case 51: return launch_co1m<5, 1>(a, s);
    case 52: return launch_co1m<5, 2>(a, s);
    case 91: return launch_co1m<9, 1>(a, s);
    default: return launch_co1m<9, 2>(a, s);
  }
}

// ------------------------------------------------------------------------------------------
// Single-output-channel conv on VALU (v_dot2_f32_bf16): conv_last (64->1), srcnn.conv3 (32->1) and
// the data gradient of srcnn.conv1 w.r.t. its first input channel (64->1, 9x9).  With Cout = 1 an
// MFMA tile would waste 15 of 16 rows; here each thread owns one output pixel of a 16x16 tile, the
// input tile (CO1_CC channels at a time) sits in LDS and the weights are wave-uniform scalar loads.
// ------------------------------------------------------------------------------------------
constexpr int CO1_CC = 32;

__global__ __launch_bounds__(256) void conv_co1_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* xs = (uint16_t*)smem;
  constexpr int XPITCH = CO1_CC + 8;
  uint16_t* wsm = (uint16_t*)(smem + (size_t)(15 + a.ks) * (15 + a.ks) * XPITCH * 2);  // [tap][CO1_CC]
  const int tid = threadIdx.x;
  int bid = blockIdx.x;
  const int tx = bid % a.tiles_x;
  bid /= a.tiles_x;
  const int ty = bid % a.tiles_y;
  const int nimg = bid / a.tiles_y;
  const int ox0 = tx * 16, oy0 = ty * 16;
  const int py = tid >> 4, px = tid & 15;
  const int tph = 15 + a.ks, tpw = 15 + a.ks;
  const int iy0 = oy0 - a.pad, ix0 = ox0 - a.pad;
  const int kcpad = a.kcpad;
  float acc = 0.f;
  constexpr int cvec = CO1_CC / 8;
  const int nvec = tph * tpw * cvec;
  for (int c0 = 0; c0 < a.in_c; c0 += CO1_CC) {
    __syncthreads();
    for (int base = 0; base < nvec; base += 256 * FWD_MAXV) {
      uint4 buf[FWD_MAXV];
#pragma unroll
      for (int i = 0; i < FWD_MAXV; ++i) {
        const int v = base + tid + i * 256;
        uint4 val = make_uint4(0, 0, 0, 0);
        if (v < nvec) {
          const int pix = v / cvec, cg = v % cvec;  // cvec compile-time
          const int yy = pix / tpw, xx = pix - (pix / tpw) * tpw;
          const int iy = iy0 + yy, ix = ix0 + xx, c = c0 + cg * 8;
          if (iy >= 0 && iy < a.in_h && ix >= 0 && ix < a.in_w && c < a.in_c)
            val = *(const uint4*)(a.x + (((long)nimg * a.in_h + iy) * a.in_w + ix) * a.in_cs + a.in_co + c);
        }
        buf[i] = val;
      }
#pragma unroll
      for (int i = 0; i < FWD_MAXV; ++i) {
        const int v = base + tid + i * 256;
        if (v < nvec) {
          const int pix = v / cvec, cg = v % cvec;
          *(uint4*)(xs + pix * XPITCH + cg * 8) = buf[i];
        }
      }
    }
    // weights of this channel chunk, [tap][CO1_CC] (packed row 0: k = (c/cc)*kcpad + tap*cc + c%cc)
    for (int v = tid; v < a.ks * a.ks * cvec; v += 256) {
      const int tap = v / cvec, cg = v % cvec, c = c0 + cg * 8;
      uint4 val = make_uint4(0, 0, 0, 0);
      if (c < a.in_c) val = *(const uint4*)(a.w + (c / a.cc) * kcpad + tap * a.cc + (c % a.cc));
      *(uint4*)(wsm + tap * CO1_CC + cg * 8) = val;
    }
    __syncthreads();
    const int cn = min(CO1_CC, a.in_c - c0);
    for (int ky = 0; ky < a.ks; ++ky) {
      for (int kx = 0; kx < a.ks; ++kx) {
        const int tap = ky * a.ks + kx;
        const uint16_t* xp = xs + ((py + ky) * tpw + px + kx) * XPITCH;
        const uint16_t* wp = wsm + tap * CO1_CC;
        for (int cg = 0; cg < cn; cg += 8) {
          const uint4 wv = *(const uint4*)(wp + cg);  // same address in every lane: LDS broadcast
          const uint4 xv = *(const uint4*)(xp + cg);
          const uint32_t xw[4] = {xv.x, xv.y, xv.z, xv.w}, ww[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
          for (int q = 0; q < 4; ++q)
            acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, xw[q]), __builtin_bit_cast(bf16x2, ww[q]), acc, false);
        }
      }
    }
  }
  const int oy = oy0 + py, ox = ox0 + px;
  if (oy >= a.out_h || ox >= a.out_w) return;
  float v = acc + (a.bias ? a.bias[0] : 0.f);
  v = act_apply(v, a.act, a.slope);
  const long pidx = ((long)nimg * a.out_h + oy) * a.out_w + ox;
  const bool f1 = a.res_f32 & 1, f2 = (a.res_f32 >> 1) & 1;
  const float r1 = a.res1 ? res_at(a.res1, f1, pidx * a.r1_cs + a.r1_co) : 0.f;
  const float r2 = a.res2 ? res_at(a.res2, f2, pidx * a.r2_cs + a.r2_co) : 0.f;
  v = ep_res(v, a.act, a.slope, a.res1 != nullptr, r1, a.alpha1, a.beta1, a.res2 != nullptr, r2, a.alpha2, a.beta2);
  const long ob = pidx * a.out_cs + a.out_co;
  if (a.out_mode == 0) ((uint16_t*)a.y)[ob] = f2bf(v);
  else if (a.out_mode == 2) ((float*)a.y)[ob] += v;
  else ((float*)a.y)[ob] = v;
  if (a.aux) a.aux[pidx * a.aux_cs + a.aux_co] = f2bf(a.aux_scale * v);
}

// ------------------------------------------------------------------------------------------
// Weights-resident persistent conv: one workgroup per CU stages the WHOLE packed weight matrix
// (<= 64 output channels, one channel chunk) into LDS once and walks its share of the output tiles,
// the next tile's input prefetched into registers while the current one is on the MFMA pipe.  For the
// HR-resolution convs (HRconv / upconv1-2 with the upsample on load, srcnn.conv1 9x9 and conv2 5x5,
// their data gradients, trunk_conv / conv_first) the generic kernel restages the weights for every
// 256-pixel tile (8k tiles per launch at 256^2).  Stride 1 only; epilogue = the generic one.
// ------------------------------------------------------------------------------------------
constexpr int PW_PV = 12;  // prefetched 16 B input vectors per thread (tile <= 3072 vectors)

struct PwGeom {
  int mw, tph, tpw, ccp, kcpad, nvx;
  size_t lds_tab, lds_w, lds_x, lds_ep, lds_total;
};

static bool pw_geom(const ClimsrConvDesc* d, int nt, int mw, PwGeom* g, int nw = 4) {
  if (d->stride != 1 || d->cc < d->in_c) return false;
  g->mw = mw;
  g->tph = nw * mw + d->ks - 1;
  g->tpw = TW + d->ks - 1;
  const int ccs = d->cc < 8 ? 8 : d->cc;  // staged channels per pixel (cc 4: 16 B loads, 4 of 8 channels used)
  g->ccp = xpitch(ccs);
  g->kcpad = round_up(d->ks * d->ks * d->cc, 32);
  g->nvx = g->tph * g->tpw * (ccs / 8);
  g->lds_tab = ((size_t)(g->kcpad / (d->cc < 8 ? 4 : 8)) * 4 + 15) / 16 * 16;
  g->lds_w = (size_t)nt * 16 * (g->kcpad + WPAD) * 2;
  g->lds_x = (size_t)g->tph * g->tpw * g->ccp * 2;
  g->lds_ep = (size_t)nw * mw * 16 * (nt * 16 + 4) * 4;
  g->lds_total = g->lds_tab + g->lds_w + (g->lds_x > g->lds_ep ? g->lds_x : g->lds_ep);
  return g->nvx <= 64 * nw * PW_PV && g->lds_total <= 160 * 1024;
}

static bool pw_fits(int in_c, int ks, int out_c) {
  const int nt = fwd_nt(out_c);
  if (out_c <= 16 || out_c > 64 || (nt != 2 && nt != 4)) return false;
  ClimsrConvDesc d{};
  d.in_c = round_up(in_c, 8);
  d.cc = d.in_c;
  d.ks = ks;
  d.stride = 1;
  PwGeom g;
  return pw_geom(&d, nt, 2, &g, 4);
}

// GEO = 1: 3x3 taps over one 64-channel chunk with 8 waves x 2 rows (the 64 -> 64 HR-resolution / VGG conv1_2
// shapes): the 18 k-steps unrolled with compile-time LDS offsets (no tap table; see conv_fwd_kernel's GEO)
template <int NW, int MW, int NT, bool RF, int PV, int EP = 0, int GEO = 0>
__global__ __launch_bounds__(64 * NW, 1) void conv_pw_kernel(FwdArgs a) {
  constexpr int NTHR = 64 * NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* tab = (int*)smem;
  uint16_t* ws = (uint16_t*)(smem + a.lds_tab);
  uint16_t* xs = (uint16_t*)(smem + a.lds_tab + a.lds_x);  // lds_x carries the weight region size here
  float* ebase = (float*)xs;                               // epilogue staging aliases the input tile

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, col = lane & 15;
  const int wpitch = a.kcpad + WPAD;
  const int ks2 = a.ks * a.ks;
  if constexpr (GEO == 2) {  // 4-channel taps: table of tap offsets, one per 4 k values
    for (int i = tid; i < a.kcpad / 4; i += NTHR) {
      const int tap = i < ks2 ? i : 0, ky = tap / a.ks, kx = tap - ky * a.ks;
      tab[i] = (ky * a.tpw + kx) * a.ccp;
    }
  }
  for (int i = tid; i < (GEO ? 0 : a.kcpad / 8); i += NTHR) {  // tap table (one chunk)
    const int kr = i * 8;
    int tap = kr / a.cc, c = kr - tap * a.cc;
    if (tap >= ks2) { tap = 0; c = 0; }
    const int ky = tap / a.ks, kx = tap - ky * a.ks;
    tab[i] = (ky * a.tpw + kx) * a.ccp + c;
  }
  {  // the whole weight matrix, once: 8 vectors per thread in flight per batch (buffer loads, no branch)
    const int wvec_row = a.kcpad / 8, nvw = NT * 16 * wvec_row;
    const __amdgpu_buffer_rsrc_t wr = buf_rsrc(a.w, 0xFFFFFFFFu);
    for (int v0 = 0; v0 < nvw; v0 += 8 * NTHR) {
      uint4 wv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int v = v0 + tid + i * NTHR;
        const int r = v / wvec_row, kv = v - r * wvec_row;
        wv[i] = buf_load16(wr, v < nvw ? (uint32_t)((r * a.kpk + kv * 8) * 2) : 0u);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int v = v0 + tid + i * NTHR;
        const int r = v / wvec_row, kv = v - r * wvec_row;
        if (v < nvw) *(uint4*)(ws + r * wpitch + kv * 8) = wv[i];
      }
    }
  }
  const int ufac = a.up, upsh = a.up == 2 ? 1 : 0;
  const int lh = a.in_h * ufac, lw = a.in_w * ufac;
  const int cvec = a.cc / 8;
  const int nvec_x = a.tph * a.tpw * cvec;
  const int x_dp = NTHR / cvec, x_dc = NTHR - x_dp * cvec;
  const int x_dy = x_dp / a.tpw, x_dx = x_dp - x_dy * a.tpw;
  const int x_pix0 = tid / cvec, x_cg0 = tid - x_pix0 * cvec;
  const int x_ty0 = x_pix0 / a.tpw, x_tx0 = x_pix0 - x_ty0 * a.tpw;
  const int ntiles = a.tiles_x * a.tiles_y * a.n;

  uint4 pre[PV];
  // buffer loads (zeros out of range) and an unconditional call: the next tile's loads stay in flight
  // through this tile's compute (see conv_n16_kernel)
  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(a.x, (uint32_t)((long)a.n * a.in_h * a.in_w * a.in_cs * 2));
  // tile coordinates advance incrementally by the walk's step (no per-tile integer divisions: wave-uniform
  // divisions by runtime tile counts cost ~40 SALU each, 8 per tile, on the CU's shared scalar pipe)
  auto issue = [&](bool live, int tx, int ty, int nimg) {  // !live: nothing to load
    const int iy0 = ty * (NW * MW) - a.pad, ix0 = tx * TW - a.pad;
    int ty_ = x_ty0, tx_ = x_tx0, cg = x_cg0;
#pragma unroll
    for (int i = 0; i < PV; ++i) {
      {
        const int iy = iy0 + ty_, ix = ix0 + tx_;
        const int c = cg * 8;
        const bool ok = live && tid + NTHR * i < nvec_x && iy >= 0 && iy < lh && ix >= 0 && ix < lw && c < a.in_c;
        const uint32_t off = (uint32_t)((((nimg * a.in_h + (iy >> upsh)) * a.in_w + (ix >> upsh)) * a.in_cs + a.in_co + c) * 2);
        pre[i] = buf_load16(xr, ok ? off : BUF_OOB);
      }
      cg += x_dc;
      tx_ += x_dx;
      ty_ += x_dy;
      if (cg >= cvec) { cg -= cvec; ++tx_; }
      if (tx_ >= a.tpw) { tx_ -= a.tpw; ++ty_; }
    }
  };
  const TileWalk walk(ntiles);
  const int s_x = walk.step % a.tiles_x, s_y = (walk.step / a.tiles_x) % a.tiles_y, s_n = walk.step / (a.tiles_x * a.tiles_y);
  auto advance = [&](int& tx, int& ty, int& n) {
    tx += s_x;
    int c = tx >= a.tiles_x;
    tx -= c ? a.tiles_x : 0;
    ty += s_y + c;
    c = ty >= a.tiles_y;
    ty -= c ? a.tiles_y : 0;
    n += s_n + c;
  };
  int ctx = walk.first % a.tiles_x, cty = (walk.first / a.tiles_x) % a.tiles_y, cn = walk.first / (a.tiles_x * a.tiles_y);
  if (walk.first < walk.end) issue(true, ctx, cty, cn);

  int pixbase[MW];
#pragma unroll
  for (int m = 0; m < MW; ++m) pixbase[m] = ((wave * MW + m) * a.tpw + col) * a.ccp;

  for (int tile = walk.first; tile < walk.end; tile += walk.step) {
    const int tx = ctx, ty = cty, nimg = cn;
    advance(ctx, cty, cn);  // the next tile of this workgroup
    const int ox0 = tx * TW, oy0 = ty * (NW * MW);
    lds_barrier();  // previous tile's epilogue reads of the aliased region are done
    {
      int ty_ = x_ty0, tx_ = x_tx0, cg = x_cg0;
#pragma unroll
      for (int i = 0; i < PV; ++i) {
        if (tid + NTHR * i < nvec_x) *(uint4*)(xs + (ty_ * a.tpw + tx_) * a.ccp + cg * 8) = pre[i];
        cg += x_dc;
        tx_ += x_dx;
        ty_ += x_dy;
        if (cg >= cvec) { cg -= cvec; ++tx_; }
        if (tx_ >= a.tpw) { tx_ -= a.tpw; ++ty_; }
      }
    }
    issue(tile + walk.step < walk.end, ctx, cty, cn);  // lands while this tile computes
    lds_barrier();
    f32x4 acc[MW][NT];
#pragma unroll
    for (int m = 0; m < MW; ++m)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[m][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    {
      // k-steps two deep: k-step s+1's tap offset and fragments are read while s is on the MFMA pipe (one k-step at
      // a time serialised tab read -> B read -> MFMAs, 3 lgkmcnt waits per 8 MFMAs)
      if constexpr (GEO == 1) {
        static_assert(NW * MW == 16, "GEO 1: 16-row tiles");
        constexpr int TPW = TW + 2, CCP = 80, WP = 9 * 64 + WPAD;
        const uint16_t* xb = xs + ((wave * MW) * TPW + col) * CCP + g * 8;
        const uint16_t* wb = ws + col * WP + g * 8;
        bf16x8 af[2][NT], bf[2][MW];
        auto ldk = [&](int k, int b) {  // k-step k: tap k / 2, channels (k & 1) * 32 + 8 g
          const int tap = k >> 1, off = ((tap / 3) * TPW + tap % 3) * CCP + (k & 1) * 32;
#pragma unroll
          for (int t = 0; t < NT; ++t) af[b][t] = *(const bf16x8*)(wb + t * 16 * WP + k * 32);
#pragma unroll
          for (int m = 0; m < MW; ++m) bf[b][m] = *(const bf16x8*)(xb + m * TPW * CCP + off);
        };
        ldk(0, 0);
#pragma unroll
        for (int k = 0; k < 18; ++k) {
          if (k + 1 < 18) ldk(k + 1, (k + 1) & 1);
          __builtin_amdgcn_sched_barrier(0);  // the next k-step's reads as one burst ahead of this k-step's MFMAs
#pragma unroll
          for (int m = 0; m < MW; ++m)
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[k & 1][t], bf[k & 1][m], acc[m][t], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
      const int nks = a.kcpad / 32;
      bf16x8 afA[NT], bfA[MW], afB[NT], bfB[MW];
      auto ld = [&](int ks, bf16x8 (&af)[NT], bf16x8 (&bf)[MW]) {
#pragma unroll
        for (int t = 0; t < NT; ++t) af[t] = *(const bf16x8*)(ws + (t * 16 + col) * wpitch + ks * 32 + g * 8);
        if constexpr (GEO == 2) {  // k values 8g..8g+7 of the step = taps 8 ks + 2g, +1, 4 channels each
          const int off0 = tab[ks * 8 + 2 * g], off1 = tab[ks * 8 + 2 * g + 1];
#pragma unroll
          for (int m = 0; m < MW; ++m)
            bf[m] = cat_tr(*(const s16x4*)(xs + pixbase[m] + off0), *(const s16x4*)(xs + pixbase[m] + off1));
        } else {
          const int off = tab[ks * 4 + g];
#pragma unroll
          for (int m = 0; m < MW; ++m) bf[m] = *(const bf16x8*)(xs + pixbase[m] + off);
        }
      };
      auto mm = [&](const bf16x8 (&af)[NT], const bf16x8 (&bf)[MW]) {
#pragma unroll
        for (int m = 0; m < MW; ++m)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bf[m], acc[m][t], 0, 0, 0);
      };
      ld(0, afA, bfA);
      int ks = 0;
      for (; ks + 2 <= nks; ks += 2) {
        ld(ks + 1, afB, bfB);
        mm(afA, bfA);
        ld(ks + 2 < nks ? ks + 2 : nks - 1, afA, bfA);  // clamped: no branch around the reads
        mm(afB, bfB);
      }
      if (ks < nks) mm(afA, bfA);
      }
    }
    const int ox = ox0 + col;
    if constexpr (EP == 5) {  // 2x2 sum + activation backward (act' of the bf16 low-res activation res1), bf16 out,
                              // 4 channels (8 B) per lane; all operand loads issued before the first store
      const int dh = a.out_h >> 1, dw = a.out_w >> 1;
      const __amdgpu_buffer_rsrc_t rm1 = opt_rsrc(a.res1);
      uint2 r1v[MW / 2][NT];
#pragma unroll
      for (int m = 0; m < MW; m += 2) {
        const int oy = oy0 + wave * MW + m;
        const bool ok = !(col & 1) && oy < a.out_h && ox < a.out_w;
        const long q = ok ? ((long)nimg * dh + (oy >> 1)) * dw + (ox >> 1) : 0;
#pragma unroll
        for (int t = 0; t < NT; ++t) r1v[m / 2][t] = buf_load8(rm1, (uint32_t)((q * a.r1_cs + (ok ? a.r1_co + t * 16 + g * 4 : 0)) * 2));
      }
#pragma unroll
      for (int m = 0; m < MW; m += 2) {
        const int oy = oy0 + wave * MW + m;
        const long pidx = ((long)nimg * dh + (oy >> 1)) * dw + (ox >> 1);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float sm = acc[m][t][i] + acc[m + 1][t][i];
            sm += __shfl_xor(sm, 1);
            v[i] = sm;
          }
          if ((col & 1) || oy >= a.out_h || ox >= a.out_w) continue;
          const uint4 r1 = make_uint4(r1v[m / 2][t].x, r1v[m / 2][t].y, 0, 0);
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = ep_res(v[i], a.act, a.slope, true, res4_at(r1, false, i), 1.f, 1.f, false, 0.f, 1.f, 1.f);
          uint2 pk;
          pk.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          pk.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
          *(uint2*)((uint16_t*)a.y + pidx * a.out_cs + a.out_co + t * 16 + g * 4) = pk;
        }
      }
      continue;
    }
    if (EP == 0 && a.down2) {  // 2x2 sum (data gradient of the nearest upsample): rows (m, m+1), columns via lane ^ 1
      const int dh = a.out_h >> 1, dw = a.out_w >> 1;
      const bool mask = a.act == 3 || a.act == 4;
#pragma unroll
      for (int m = 0; m < MW; m += 2) {
        const int oy = oy0 + wave * MW + m;
        const long pidx = ((long)nimg * dh + (oy >> 1)) * dw + (ox >> 1);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float sm = acc[m][t][i] + acc[m + 1][t][i];
            sm += __shfl_xor(sm, 1);
            v[i] = sm;
          }
          const int co = t * 16 + g * 4;
          if ((col & 1) || oy >= a.out_h || ox >= a.out_w) continue;
          const long ob = pidx * a.out_cs + a.out_co + co;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (co + i >= a.out_c) continue;
            float x = v[i];
            if (mask) x = ep_res(x, a.act, a.slope, true, res_at(a.res1, false, pidx * a.r1_cs + a.r1_co + co + i), 1.f, 1.f, false, 0.f,
                                 1.f, 1.f);
            if (a.out_mode == 0) ((uint16_t*)a.y)[ob + i] = f2bf(x);
            else if (a.out_mode == 2) ((float*)a.y)[ob + i] += x;
            else ((float*)a.y)[ob + i] = x;
            if (a.aux) a.aux[pidx * a.aux_cs + a.aux_co + co + i] = f2bf(a.aux_scale * x);
          }
        }
      }
      continue;
    }
    constexpr int EPP = NT * 16 + 4;
    float* eb = ebase + wave * (MW * 16 * EPP);
    lds_barrier();  // all waves are done reading the input tile (the staging region aliases it)
#pragma unroll
    for (int m = 0; m < MW; ++m)
#pragma unroll
      for (int t = 0; t < NT; ++t) *(f32x4*)(eb + (m * 16 + col) * EPP + t * 16 + g * 4) = acc[m][t];
    lds_barrier();
    store_tile_lds<RF, MW * 16, NT * 16, 64, EP>(a, eb, EPP, lane, nimg, oy0 + wave * MW, ox0, 0);
  }
}

template <int NW, int MW, int NT, int PV, int EP, int GEO>
static int launch_pw_geo(const FwdArgs& a0, const PwGeom& g, hipStream_t s) {
  if (g_dry) {
    snprintf(g_dry_name, sizeof(g_dry_name), "conv_pw_kernel<%d, %d, %d, %s, %d, %d, %d>", NW, MW, NT, a0.res_f32 ? "true" : "false", PV, EP,
             GEO);
    return CLIMSR_OK;
  }
  FwdArgs a = a0;
  a.tph = g.tph; a.tpw = g.tpw; a.ccp = g.ccp; a.kcpad = g.kcpad;
  a.tiles_x = ceil_div(a.out_w, TW);
  a.tiles_y = ceil_div(a.out_h, NW * MW);
  a.lds_tab = (int)g.lds_tab;
  a.lds_x = (int)g.lds_w;  // offset of the input tile = tab + weights
  auto k = a.res_f32 ? conv_pw_kernel<NW, MW, NT, true, PV, EP, GEO> : conv_pw_kernel<NW, MW, NT, false, PV, EP, GEO>;
  if (int e = lds_opt_in((const void*)k, 160 * 1024)) return e;
  const int ncu = device_cus();
  const int ntiles = a.tiles_x * a.tiles_y * a.n;
  const int grid = ntiles < ncu ? ntiles : ncu;
  hipLaunchKernelGGL(k, dim3(grid), dim3(64 * NW), g.lds_total, s, a);
  return check_launch("conv2d_fwd (pw)");
}

template <int NW, int MW, int NT, int PV, int EP = 0>
static int launch_pw(const FwdArgs& a, const PwGeom& g, hipStream_t s) {
  if (a.cc == 4) {  // 4-channel taps: staged as 8-channel pixels (16 B loads)
    FwdArgs b = a;
    b.cc = 8;
    b.in_c = 8;
    // one 16 B vector per pixel: the 24 x 24 (9x9) / 18 x 18 (3x3) input tile is <= 2 vectors per thread, and the
    // staging loops run PV iterations of address math whether or not their vectors exist
    if (g.nvx <= 2 * 64 * NW) return launch_pw_geo<NW, MW, NT, 2, EP, 2>(b, g, s);
    return launch_pw_geo<NW, MW, NT, PV, EP, 2>(b, g, s);
  }
  if constexpr (NW * MW == 16) {
    if (a.ks == 3 && a.cc == 64 && g.kcpad == 9 * 64 && g.ccp == 80 && g.tpw == TW + 2 && g.tph == 18)
      return launch_pw_geo<NW, MW, NT, PV, EP, 1>(a, g, s);
  }
  return launch_pw_geo<NW, MW, NT, PV, EP, 0>(a, g, s);
}

// ------------------------------------------------------------------------------------------
// 1x1 conv as a streaming GEMM (srcnn.conv2 64->32 and its 32->64 data gradient with the ReLU mask):
// out[p][co] = epilogue(sum_ci x[p][ci] w[co][ci]).  Nothing is reused across pixels except the weights, so
// nothing goes through LDS: the weight fragments sit in VGPRs, each lane loads its 16 B channel slice of a
// pixel straight into the B fragment (16 pixels x 32 channels per load round), U groups of 16 pixels are in
// flight per wave, and the fused epilogue stores 4 consecutive channels per lane.  HBM-bound by design.
// ------------------------------------------------------------------------------------------
constexpr int PT_U = 4;  // 16-pixel groups per wave iteration

static bool pt_shape(const ClimsrConvDesc* d, const ClimsrEpilogue* ep) {
  return d->ks == 1 && d->stride == 1 && d->up == 1 && d->pad == 0 && !ep->down2 && d->in_c % 32 == 0 && d->in_c <= 128 &&
         d->cc == d->in_c && d->out_c % 16 == 0 && d->out_c <= 64 && d->out_h == d->in_h && d->out_w == d->in_w &&
         ((d->out_cstride | d->out_coff) & 3) == 0 && (!ep->res1 || ((ep->res1_cstride | ep->res1_coff) & 3) == 0) &&
         (!ep->res2 || ((ep->res2_cstride | ep->res2_coff) & 3) == 0);
}

// EP: 0 generic (runtime flags); 3 activation forward (bias + leaky relu / relu, bf16 out); 4 activation backward
// (act' from the bf16 activation res1, no bias, bf16 out) -- srcnn.conv2's forward and data gradient.
template <int NCOF, int NKC, int EP = 0>
__global__ __launch_bounds__(256) void conv_pt_kernel(FwdArgs a, long npix) {
  __shared__ float tsm[NCOF == 4 ? 4 * 16 * 68 : 1];
  const int lane = threadIdx.x & 63, g = lane >> 4, col = lane & 15;
  bf16x8 af[NCOF][NKC];
#pragma unroll
  for (int f = 0; f < NCOF; ++f)
#pragma unroll
    for (int k = 0; k < NKC; ++k) af[f][k] = *(const bf16x8*)(a.w + (long)(f * 16 + col) * a.kpk + k * 32 + g * 8);
  float bb[NCOF][4];
#pragma unroll
  for (int f = 0; f < NCOF; ++f)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      bb[f][i] = ((EP == 3 || (EP == 0 && a.bias)) && f * 16 + g * 4 + i < a.out_c) ? a.bias[f * 16 + g * 4 + i] : 0.f;
  const bool f1 = EP != 0 ? false : (a.res_f32 & 1) != 0, f2 = EP != 0 ? false : ((a.res_f32 >> 1) & 1) != 0;
  const bool has_bias = EP == 3 ? true : EP == 4 ? false : a.bias != nullptr;
  const bool has1 = EP == 3 ? false : EP == 4 ? true : a.res1 != nullptr;
  const bool has2 = EP != 0 ? false : a.res2 != nullptr;
  const bool has_aux = EP != 0 ? false : a.aux != nullptr;
  const int out_mode = EP != 0 ? 0 : a.out_mode;
  const long ngroups = (npix + 15) / 16;
  const long wave_id = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  // input groups are loaded one iteration ahead with range-checked buffer loads (zeros past npix, no branch),
  // so the next group's loads are in flight through this group's epilogue
  const __amdgpu_buffer_rsrc_t xr = buf_rsrc(a.x, (uint32_t)(npix * a.in_cs * 2));
  const __amdgpu_buffer_rsrc_t rr1 = opt_rsrc(has1 ? a.res1 : nullptr), rr2 = opt_rsrc(has2 ? a.res2 : nullptr);
  bf16x8 bn[PT_U][NKC];
  auto ldx = [&](long g0) {
#pragma unroll
    for (int u = 0; u < PT_U; ++u) {
      const long p = (g0 + u) * 16 + col;
#pragma unroll
      for (int k = 0; k < NKC; ++k) {
        const uint4 v = buf_load16(xr, p < npix ? (uint32_t)((p * a.in_cs + a.in_co + k * 32 + g * 8) * 2) : BUF_OOB);
        bn[u][k] = __builtin_bit_cast(bf16x8, v);
      }
    }
  };
  ldx(wave_id * PT_U);
  for (long g0 = wave_id * PT_U; g0 < ngroups; g0 += nwaves * PT_U) {
    bf16x8 bx[PT_U][NKC];
#pragma unroll
    for (int u = 0; u < PT_U; ++u)
#pragma unroll
      for (int k = 0; k < NKC; ++k) bx[u][k] = bn[u][k];
    ldx(g0 + nwaves * PT_U);
#pragma unroll
    for (int u = 0; u < PT_U; ++u) {
      const long p = (g0 + u) * 16 + col;
      f32x4 acc[NCOF];
#pragma unroll
      for (int f = 0; f < NCOF; ++f) {
        acc[f] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < NKC; ++k) acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[f][k], bx[u][k], acc[f], 0, 0, 0);
      }
      if (NCOF == 4) {  // transpose through this wave's LDS so each lane owns 16 channels of one pixel and a store
                        // instruction covers whole lines (the 8 B-per-lane MFMA layout touches 16 lines per store)
        float* tw = tsm + (threadIdx.x >> 6) * (16 * 68);
#pragma unroll
        for (int f = 0; f < NCOF; ++f)
#pragma unroll
          for (int i = 0; i < 4; ++i) tw[col * 68 + f * 16 + g * 4 + i] = acc[f][i];
        const int pp = lane / NCOF, c0 = (lane % NCOF) * 16;  // NCOF lanes per pixel
        const long q = (g0 + u) * 16 + pp;
        float v[16];
        const int ppr = pp < 16 ? pp : 15;  // lanes beyond the 16 pixels (NCOF 2) read a valid row and store nothing
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x4 t4 = *(const f32x4*)(tw + ppr * 68 + c0 + 4 * j);
#pragma unroll
          for (int i = 0; i < 4; ++i) v[4 * j + i] = t4[i];
        }
        const bool okq = pp < 16 && q < npix;
        uint4 r1s[4], r2s[4];  // every residual load of this pixel before the first use (branch-free)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const long qq = okq ? q : 0;
          const int co = okq ? c0 + 4 * j : 0;
          if (EP == 0 || has1) {
            if (f1) r1s[j] = buf_load16(rr1, (uint32_t)((qq * a.r1_cs + (okq ? a.r1_co : 0) + co) * 4));
            else { const uint2 t2 = buf_load8(rr1, (uint32_t)((qq * a.r1_cs + (okq ? a.r1_co : 0) + co) * 2)); r1s[j] = make_uint4(t2.x, t2.y, 0, 0); }
          } else r1s[j] = make_uint4(0, 0, 0, 0);
          if (EP == 0 || has2) {
            if (f2) r2s[j] = buf_load16(rr2, (uint32_t)((qq * a.r2_cs + (okq ? a.r2_co : 0) + co) * 4));
            else { const uint2 t2 = buf_load8(rr2, (uint32_t)((qq * a.r2_cs + (okq ? a.r2_co : 0) + co) * 2)); r2s[j] = make_uint4(t2.x, t2.y, 0, 0); }
          } else r2s[j] = make_uint4(0, 0, 0, 0);
        }
        if (okq) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int co = c0 + 4 * j;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float bsv = has_bias ? a.bias[co + i] : 0.f;
              v[4 * j + i] = ep_res(act_apply(v[4 * j + i] + bsv, a.act, a.slope), a.act, a.slope, has1, res4_at(r1s[j], f1, i),
                                    a.alpha1, a.beta1, has2, res4_at(r2s[j], f2, i), a.alpha2, a.beta2);
            }
          }
          const long ob = q * a.out_cs + a.out_co + c0;
          if (out_mode == 0) {
            uint4 w0, w1;
            w0.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
            w0.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
            w0.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
            w0.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
            w1.x = (uint32_t)f2bf(v[8]) | ((uint32_t)f2bf(v[9]) << 16);
            w1.y = (uint32_t)f2bf(v[10]) | ((uint32_t)f2bf(v[11]) << 16);
            w1.z = (uint32_t)f2bf(v[12]) | ((uint32_t)f2bf(v[13]) << 16);
            w1.w = (uint32_t)f2bf(v[14]) | ((uint32_t)f2bf(v[15]) << 16);
            *(uint4*)((uint16_t*)a.y + ob) = w0;
            *(uint4*)((uint16_t*)a.y + ob + 8) = w1;
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
              if (out_mode == 2) o = *(const float4*)((const float*)a.y + ob + 4 * j);
              *(float4*)((float*)a.y + ob + 4 * j) =
                  make_float4(o.x + v[4 * j], o.y + v[4 * j + 1], o.z + v[4 * j + 2], o.w + v[4 * j + 3]);
            }
          }
          if (has_aux) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              uint2 pk;
              pk.x = (uint32_t)f2bf(a.aux_scale * v[4 * j]) | ((uint32_t)f2bf(a.aux_scale * v[4 * j + 1]) << 16);
              pk.y = (uint32_t)f2bf(a.aux_scale * v[4 * j + 2]) | ((uint32_t)f2bf(a.aux_scale * v[4 * j + 3]) << 16);
              *(uint2*)(a.aux + q * a.aux_cs + a.aux_co + c0 + 4 * j) = pk;
            }
          }
        }
        continue;
      }
      uint4 r1s[NCOF], r2s[NCOF];  // all residual loads of this pixel first (branch-free)
#pragma unroll
      for (int f = 0; f < NCOF; ++f) {
        const int co = f * 16 + g * 4;
        const bool okf = p < npix && co < a.out_c;
        const long pp = okf ? p : 0;
        const int cc = okf ? co : 0;
        if (EP == 0 || has1) {
          if (f1) r1s[f] = buf_load16(rr1, (uint32_t)((pp * a.r1_cs + (okf ? a.r1_co : 0) + cc) * 4));
          else { const uint2 t2 = buf_load8(rr1, (uint32_t)((pp * a.r1_cs + (okf ? a.r1_co : 0) + cc) * 2)); r1s[f] = make_uint4(t2.x, t2.y, 0, 0); }
        } else r1s[f] = make_uint4(0, 0, 0, 0);
        if (EP == 0 || has2) {
          if (f2) r2s[f] = buf_load16(rr2, (uint32_t)((pp * a.r2_cs + (okf ? a.r2_co : 0) + cc) * 4));
          else { const uint2 t2 = buf_load8(rr2, (uint32_t)((pp * a.r2_cs + (okf ? a.r2_co : 0) + cc) * 2)); r2s[f] = make_uint4(t2.x, t2.y, 0, 0); }
        } else r2s[f] = make_uint4(0, 0, 0, 0);
      }
      if (p >= npix) continue;
#pragma unroll
      for (int f = 0; f < NCOF; ++f) {
        const int co = f * 16 + g * 4;
        if (co >= a.out_c) continue;
        const uint4 r1 = r1s[f], r2 = r2s[f];
        const long ob = p * a.out_cs + a.out_co + co;
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          v[i] = ep_res(act_apply(acc[f][i] + bb[f][i], a.act, a.slope), a.act, a.slope, has1, res4_at(r1, f1, i), a.alpha1,
                        a.beta1, has2, res4_at(r2, f2, i), a.alpha2, a.beta2);
        if (out_mode == 0) {
          uint2 pk;
          pk.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          pk.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
          *(uint2*)((uint16_t*)a.y + ob) = pk;
        } else {
          float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
          if (out_mode == 2) o = *(const float4*)((const float*)a.y + ob);
          *(float4*)((float*)a.y + ob) = make_float4(o.x + v[0], o.y + v[1], o.z + v[2], o.w + v[3]);
        }
        if (has_aux) {
          uint2 pk;
          pk.x = (uint32_t)f2bf(a.aux_scale * v[0]) | ((uint32_t)f2bf(a.aux_scale * v[1]) << 16);
          pk.y = (uint32_t)f2bf(a.aux_scale * v[2]) | ((uint32_t)f2bf(a.aux_scale * v[3]) << 16);
          *(uint2*)(a.aux + p * a.aux_cs + a.aux_co + co) = pk;
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Data gradient of a conv with ONE output channel (conv_last 64->1 3x3, srcnn.conv3 32->1 5x5; esrgan.py:99,
// srcnn.py:17): g[q][c] = act'(res1[q][c]) * sum_{ky,kx} W[0][c][ky][kx] * dz[q - (ky,kx) + pad].  A 1 -> C
// stencil, not a GEMM (K = ks^2 taps of one channel): one 16x16-pixel tile per workgroup, the dz tile (+halo)
// and the fp32 weights in LDS, each thread one pixel x 8 channels per step (16 B residual load, 16 B store).
// Bound by HBM (the residual read and the output write).  The implicit-GEMM path padded K to 32 and ran the
// epilogue of a 64-output MFMA tile per 2 input channels (conv_last dgrad 222 us, srcnn.conv3 dgrad 144 us).
// ------------------------------------------------------------------------------------------
constexpr int S1_T = 16;
// LPP = C / 8 lanes share a pixel (8 channels each), so a wave's 16 B stores / residual loads cover whole
// 128 B (C = 64) or 64 B (C = 32) pixel rows; weights in LDS as [tap][C] (two 16 B reads per tap).
// FWD: the same stencil as the FORWARD of a 1 -> C conv (the discriminator's features.0, rfb_esrgan.py:28: 1 -> 64,
// 3x3, no bias, LeakyReLU): out[q][c] = act(sum W[c][0][ky][kx] * x[q + (ky,kx) - pad] + bias[c]), act 1 / 2 =
// leaky relu / relu forward.  The implicit-GEMM path pads the single input channel to 8 (K = 72 of 96) and is
// bound by its LDS-staged epilogue (156 us per B=32 256^2 launch for a 268 MB output).
template <int KS, int LPP, bool FWD = false>
__global__ __launch_bounds__(256) void dgrad_ci1_kernel(int n, int h, int w, int pad, const uint16_t* __restrict__ dz, int dz_cs,
                                                        int dz_co, const float* __restrict__ wt, int act, float slope,
                                                        const uint16_t* __restrict__ res1, int r1_cs, int r1_co, uint16_t* __restrict__ out,
                                                        int out_cs, int out_co, const float* __restrict__ bias = nullptr) {
  constexpr int TP = S1_T + KS - 1, C = LPP * 8, PPS = 256 / LPP, NPASS = S1_T * S1_T / PPS;
  __shared__ float dzt[TP * TP];
  __shared__ __attribute__((aligned(16))) float wl[KS * KS * C];
  const int tid = threadIdx.x, cg = tid % LPP, ps = tid / LPP;
  const int tiles_x = (w + S1_T - 1) / S1_T, tiles_y = (h + S1_T - 1) / S1_T;
  int b = blockIdx.x;
  const int bx = b % tiles_x;
  b /= tiles_x;
  const int by = b % tiles_y, img = b / tiles_y;
  const int x0 = bx * S1_T, y0 = by * S1_T;
  // tile row r <-> dz row y0 - (KS - 1) + pad + r (same for columns); forward: x row y0 - pad + r
  const int ry0 = FWD ? y0 - pad : y0 - (KS - 1) + pad, rx0 = FWD ? x0 - pad : x0 - (KS - 1) + pad;
  // every residual load of this thread first (they land while the tile is staged and the sums computed)
  uint4 rv[NPASS];
#pragma unroll
  for (int k = 0; k < NPASS; ++k) {
    const int pix = k * PPS + ps, qy = y0 + pix / S1_T, qx = x0 + pix % S1_T;
    const bool ok = !FWD && act && qy < h && qx < w;
    rv[k] = ok ? *(const uint4*)(res1 + (((long)img * h + qy) * w + qx) * r1_cs + r1_co + cg * 8) : make_uint4(0, 0, 0, 0);
  }
  for (int i = tid; i < TP * TP; i += 256) {
    const int r = i / TP, c = i - r * TP;
    const int yy = ry0 + r, xx = rx0 + c;
    dzt[i] = (yy >= 0 && yy < h && xx >= 0 && xx < w) ? bf2f(dz[(((long)img * h + yy) * w + xx) * dz_cs + dz_co]) : 0.f;
  }
  for (int i = tid; i < C * KS * KS; i += 256) {  // OIHW [c][tap] -> [tap][c]
    const int c = i / (KS * KS), t = i - c * (KS * KS);
    wl[t * C + c] = wt[i];
  }
  __syncthreads();
  // 3x3: this thread's 8 channels x 9 taps of weights held in registers across the passes (72 VGPRs); 5x5 re-reads LDS
  constexpr bool WREG = KS == 3;
  float4 wr0[WREG ? KS * KS : 1], wr1[WREG ? KS * KS : 1];
  if constexpr (WREG) {
#pragma unroll
    for (int t = 0; t < KS * KS; ++t) {
      wr0[t] = *(const float4*)(wl + t * C + cg * 8);
      wr1[t] = *(const float4*)(wl + t * C + cg * 8 + 4);
    }
  }
#pragma unroll
  for (int k = 0; k < NPASS; ++k) {
    const int pix = k * PPS + ps, ty = pix / S1_T, tx = pix % S1_T;
    const int qy = y0 + ty, qx = x0 + tx;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ky = 0; ky < KS; ++ky)
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) {  // out[q] += W[c][ky][kx] * dz[q - (ky, kx) + pad]  (FWD: x[q + (ky, kx) - pad])
        const float d = FWD ? dzt[(ty + ky) * TP + tx + kx] : dzt[(ty + KS - 1 - ky) * TP + tx + KS - 1 - kx];
        const int t = ky * KS + kx;
        const float4 w0 = WREG ? wr0[WREG ? t : 0] : *(const float4*)(wl + t * C + cg * 8);
        const float4 w1 = WREG ? wr1[WREG ? t : 0] : *(const float4*)(wl + t * C + cg * 8 + 4);
        v[0] += w0.x * d; v[1] += w0.y * d; v[2] += w0.z * d; v[3] += w0.w * d;
        v[4] += w1.x * d; v[5] += w1.y * d; v[6] += w1.z * d; v[7] += w1.w * d;
      }
    if (qy >= h || qx >= w) continue;
    if (FWD) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (bias) v[i] += bias[cg * 8 + i];
        v[i] = act_apply(v[i], act, slope);
      }
    } else if (act) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t wd = i < 2 ? rv[k].x : i < 4 ? rv[k].y : i < 6 ? rv[k].z : rv[k].w;
        const float r = bf2f((uint16_t)((i & 1) ? (wd >> 16) : wd));
        v[i] = r > 0.f ? v[i] : (act == 3 ? v[i] * slope : 0.f);
      }
    }
    *(uint4*)(out + (((long)img * h + qy) * w + qx) * out_cs + out_co + cg * 8) = pack8_bf16(v, 1.f);
  }
}

extern "C" int climsr_dgrad_single_output(int n, int h, int w, int ks, int pad, const uint16_t* dz, int dz_cstride, int dz_coff,
                                          const float* weight, int c, int act, float slope, const uint16_t* res1, int res1_cstride,
                                          int res1_coff, uint16_t* out, int out_cstride, int out_coff, void* stream) {
  if (!dz || !weight || !out || n <= 0 || h <= 0 || w <= 0 || (ks != 3 && ks != 5) || pad != ks / 2 || c <= 0 || c > 64 || c % 8 ||
      (out_cstride | out_coff) % 8 || (act != 0 && act != 3 && act != 4) || (act && (!res1 || (res1_cstride | res1_coff) % 8))) {
    set_error("dgrad_single_output: unsupported arguments (ks %d pad %d c %d act %d)", ks, pad, c, act);
    return CLIMSR_EINVAL;
  }
  const long tiles = (long)n * ((h + S1_T - 1) / S1_T) * ((w + S1_T - 1) / S1_T);
  if (dry_run("dgrad_ci1_kernel<%d, %d>", ks, c / 8)) return CLIMSR_OK;
#define CLIMSR_CI1(KS_, LPP_)                                                                                              \
  hipLaunchKernelGGL((dgrad_ci1_kernel<KS_, LPP_>), dim3((unsigned)tiles), dim3(256), 0, (hipStream_t)stream, n, h, w, pad, dz, \
                     dz_cstride, dz_coff, weight, act, slope, res1, res1_cstride, res1_coff, out, out_cstride, out_coff)
  switch (ks * 100 + c / 8) {
    case 308: CLIMSR_CI1(3, 8); break;
    case 304: CLIMSR_CI1(3, 4); break;
    case 508: CLIMSR_CI1(5, 8); break;
    case 504: CLIMSR_CI1(5, 4); break;
    default: set_error("dgrad_single_output: no instance for ks %d, %d channels (32 or 64)", ks, c); return CLIMSR_EINVAL;
  }
#undef CLIMSR_CI1
  return check_launch("dgrad_single_output");
}

extern "C" int climsr_conv_single_input(int n, int h, int w, int ks, int pad, const uint16_t* x, int x_cstride, int x_coff,
                                        const float* weight, const float* bias, int c, int act, float slope, uint16_t* out,
                                        int out_cstride, int out_coff, void* stream) {
  if (!x || !weight || !out || n <= 0 || h <= 0 || w <= 0 || (ks != 3 && ks != 5) || pad != ks / 2 || c % 8 || (c != 32 && c != 64) ||
      (out_cstride | out_coff) % 8 || act < 0 || act > 2) {
    set_error("conv_single_input: unsupported arguments (ks %d pad %d c %d act %d)", ks, pad, c, act);
    return CLIMSR_EINVAL;
  }
  const long tiles = (long)n * ((h + S1_T - 1) / S1_T) * ((w + S1_T - 1) / S1_T);
  if (dry_run("dgrad_ci1_kernel<%d, %d, true>", ks, c / 8)) return CLIMSR_OK;
#define CLIMSR_CI1F(KS_, LPP_)                                                                                                   \
  hipLaunchKernelGGL((dgrad_ci1_kernel<KS_, LPP_, true>), dim3((unsigned)tiles), dim3(256), 0, (hipStream_t)stream, n, h, w, pad, x, \
                     x_cstride, x_coff, weight, act, slope, nullptr, 0, 0, out, out_cstride, out_coff, bias)
  switch (ks * 100 + c / 8) {
    case 308: CLIMSR_CI1F(3, 8); break;
    case 304: CLIMSR_CI1F(3, 4); break;
    case 508: CLIMSR_CI1F(5, 8); break;
    default: CLIMSR_CI1F(5, 4); break;
  }
#undef CLIMSR_CI1F
  return check_launch("conv_single_input");
}

template <int NCOF, int NKC>
static int launch_pt(const FwdArgs& a, hipStream_t s) {
  // epilogue specialisations: activation forward (3) / activation backward from a bf16 activation (4)
  const bool plain = !a.res2 && !a.aux && a.out_mode == 0 && a.res_f32 == 0 && a.out_c == NCOF * 16;
  const int ep = (plain && a.bias && !a.res1 && (a.act == 1 || a.act == 2)) ? 3
                 : (plain && !a.bias && a.res1 && (a.act == 3 || a.act == 4)) ? 4 : 0;
  if (g_dry) {
    snprintf(g_dry_name, sizeof(g_dry_name), "conv_pt_kernel<%d, %d, %d>", NCOF, NKC, ep);
    return CLIMSR_OK;
  }
  const long npix = (long)a.n * a.out_h * a.out_w;
  const long groups = (npix + 15) / 16;
  long blocks = (groups + 4 * PT_U - 1) / (4 * PT_U);
  if (blocks > 4096) blocks = 4096;
  if (ep == 3) hipLaunchKernelGGL((conv_pt_kernel<NCOF, NKC, 3>), dim3((unsigned)blocks), dim3(256), 0, s, a, npix);
  else if (ep == 4) hipLaunchKernelGGL((conv_pt_kernel<NCOF, NKC, 4>), dim3((unsigned)blocks), dim3(256), 0, s, a, npix);
  else hipLaunchKernelGGL((conv_pt_kernel<NCOF, NKC, 0>), dim3((unsigned)blocks), dim3(256), 0, s, a, npix);
  return check_launch("conv2d_fwd (pt)");
}

static int dispatch_pt(const ClimsrConvDesc* d, const FwdArgs& a, hipStream_t s) {
  const int ncof = (d->out_c + 15) / 16, nkc = d->in_c / 32;
  switch (ncof * 10 + nkc) {
    case 11: return launch_pt<1, 1>(a, s);
    case 12: return launch_pt<1, 2>(a, s);
    case 14: return launch_pt<1, 4>(a, s);
    case 21: return launch_pt<2, 1>(a, s);
    case 22: return launch_pt<2, 2>(a, s);
    case 24: return launch_pt<2, 4>(a, s);
    case 41: return launch_pt<4, 1>(a, s);
    case 42: return launch_pt<4, 2>(a, s);
    case 44: return launch_pt<4, 4>(a, s);
    default: set_error("conv_pt: no instance for %d outputs / %d inputs", d->out_c, d->in_c); return CLIMSR_EINVAL;
  }
}

// ------------------------------------------------------------------------------------------
// Data gradient of a 3x3 / stride-2 / pad-1 conv (the discriminator's downsampling convs, rfb_esrgan.py:30-48),
// phase-decomposed.  The zero-inserted form (a stride-1 conv over the 2x-upsampled dz, up = -2) spends 3 of every
// 4 MFMAs on inserted zeros; here a dx pixel (2i+a, 2j+b) sums only its own taps: with the transposed, flipped
// weights of wpk_t (tap (ky, kx) = forward tap (2-ky, 2-kx)), tap (ky, kx) feeds phase (ky != 1, kx != 1) from dz
// pixel (i + (ky == 2), j + (kx == 2)).  Every tap is one k-step (32-channel chunks), 9 k-steps per chunk in all.
// Workgroup: 16 x 16 dz positions (32 x 32 dx pixels) x 32 dx channels; wave w owns dz rows 4w..4w+3 and keeps
// 4 phases x 4 rows x 2 channel blocks of accumulators.  The taps are walked grouped by dz offset, so a B fragment
// (16 dz pixels x 32 channels) is read once per offset (4 per chunk, not 9).  dz tile 17 x 17 pixels (+ right /
// bottom halo) and the weight chunk are staged in LDS, the next chunk prefetched into registers during the
// MFMAs.  Epilogue per phase through LDS (fp32), 16 B bf16 stores, optional LeakyReLU/ReLU backward from the
// bf16 activation res1 at the dx pixel (EP 4: the layer-1 data gradient writing layer 0's output gradient).
// ------------------------------------------------------------------------------------------
constexpr int S2D_TPW = 17, S2D_CCP = 48, S2D_WP = 9 * 32 + WPAD;
template <int MW>
constexpr int s2d_lds(int nt) { return (4 * MW + 1) * S2D_TPW * S2D_CCP * 2 + nt * 16 * S2D_WP * 2; }

// MW dz rows per wave x NT 16-channel blocks (MW * NT = 8: 4 x 2 for >= 128 dx channels, 2 x 4 -- whole 128 B
// pixel lines per workgroup -- for 64)
template <int EP, int MW, int NT>
__global__ __launch_bounds__(256, 2) void conv_dgrad_s2_kernel(FwdArgs a) {
  constexpr int TPH = 4 * MW + 1, CO = NT * 16, EPP = CO + 4;
  constexpr int NRX = (TPH * S2D_TPW * 4 + 255) / 256, NRW = (CO * 36 + 255) / 256;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* xs = (uint16_t*)smem;
  uint16_t* ws = (uint16_t*)(smem + TPH * S2D_TPW * S2D_CCP * 2);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, col = lane & 15;
  // XCD-paired order: the channel blocks of one tile are 8 workgroups apart, i.e. on the same XCD (round-robin
  // dispatch) at about the same time, so they share the dz tile in that L2 and complete each other's partial
  // dx lines there (a block writes 64 of a pixel's 128 B at 64 channels)
  const int ncob = a.out_c / CO, grp = blockIdx.x / (8 * ncob), r8 = blockIdx.x % (8 * ncob);
  int bid = grp * 8 + (r8 & 7);
  if (bid >= a.tiles_x * a.tiles_y * a.n) return;
  const int tx = bid % a.tiles_x;
  bid /= a.tiles_x;
  const int ty = bid % a.tiles_y;
  const int nimg = bid / a.tiles_y;
  const int j0 = tx * 16, i0 = ty * 4 * MW, co0 = (r8 >> 3) * CO;

  f32x4 acc[4][MW][NT];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int m = 0; m < MW; ++m)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[p][m][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

  uint4 px[NRX], pw[NRW];
  auto issue = [&](int j) {
#pragma unroll
    for (int r = 0; r < NRX; ++r) {
      const int v = tid + 256 * r, pix = v >> 2, cg = v & 3;
      const int yy = i0 + pix / S2D_TPW, xx = j0 + pix % S2D_TPW;
      px[r] = make_uint4(0, 0, 0, 0);
      if (pix < TPH * S2D_TPW && yy < a.in_h && xx < a.in_w)
        px[r] = *(const uint4*)(a.x + (((long)nimg * a.in_h + yy) * a.in_w + xx) * a.in_cs + a.in_co + j * 32 + cg * 8);
    }
#pragma unroll
    for (int r = 0; r < NRW; ++r) {
      const int v = tid + 256 * r, row = v / 36, kv = v % 36;
      pw[r] = make_uint4(0, 0, 0, 0);
      if (row < CO) pw[r] = *(const uint4*)(a.w + (long)(co0 + row) * a.kpk + (long)j * 288 + kv * 8);
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int r = 0; r < NRX; ++r) {
      const int v = tid + 256 * r, pix = v >> 2, cg = v & 3;
      if (pix < TPH * S2D_TPW) *(uint4*)(xs + pix * S2D_CCP + cg * 8) = px[r];
    }
#pragma unroll
    for (int r = 0; r < NRW; ++r) {
      const int v = tid + 256 * r, row = v / 36, kv = v % 36;
      if (row < CO) *(uint4*)(ws + row * S2D_WP + kv * 8) = pw[r];
    }
  };
  // taps grouped by dz offset (dy, dx): (0,0): ky,kx in {0,1}; (0,1): kx = 2; (1,0): ky = 2; (1,1): (2,2)
  constexpr int TKY[9] = {0, 0, 1, 1, 0, 1, 2, 2, 2}, TKX[9] = {0, 1, 0, 1, 2, 2, 0, 1, 2};
  const uint16_t* xb = xs + (wave * MW * S2D_TPW + col) * S2D_CCP + g * 8;
  const uint16_t* wb = ws + col * S2D_WP + g * 8;
  auto compute = [&]() {
    bf16x8 af[2][NT], bf[2][MW];
    auto lda = [&](int st, int b) {
      const int tap = TKY[st] * 3 + TKX[st];
#pragma unroll
      for (int t = 0; t < NT; ++t) af[b][t] = *(const bf16x8*)(wb + t * 16 * S2D_WP + tap * 32);
    };
    auto ldb = [&](int st, int b) {
      const int off = ((TKY[st] == 2) * S2D_TPW + (TKX[st] == 2)) * S2D_CCP;
#pragma unroll
      for (int m = 0; m < MW; ++m) bf[b][m] = *(const bf16x8*)(xb + m * S2D_TPW * S2D_CCP + off);
    };
    lda(0, 0);
    ldb(0, 0);
    int bb = 0;
#pragma unroll
    for (int st = 0; st < 9; ++st) {
      const bool newb = st + 1 < 9 && (st + 1 == 4 || st + 1 == 6 || st + 1 == 8);
      if (st + 1 < 9) lda(st + 1, (st + 1) & 1);
      if (newb) ldb(st + 1, bb ^ 1);
      const int ph = (TKY[st] != 1) * 2 + (TKX[st] != 1);
#pragma unroll
      for (int m = 0; m < MW; ++m)
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[ph][m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[st & 1][t], bf[bb][m], acc[ph][m][t], 0, 0, 0);
      if (newb) bb ^= 1;
    }
  };
  issue(0);
  for (int j = 0; j < a.nchunk; ++j) {
    __syncthreads();  // chunk j-1's fragment reads are done
    stash();
    if (j + 1 < a.nchunk) issue(j + 1);  // lands while chunk j computes
    __syncthreads();
    compute();
  }

  // epilogue, one phase at a time: fp32 [64 px][32 ch] per wave in LDS, then 8 channels (16 B bf16) per item
  float* eb = (float*)smem + wave * (MW * 16 * EPP);
  constexpr int NG = CO / 8;  // 16 B channel groups per pixel
  const __amdgpu_buffer_rsrc_t rr1 = opt_rsrc(EP == 4 ? a.res1 : nullptr);
  // item (phase ph, k): pixel it / NG of the wave's MW x 16 dz positions, channels (it % NG) * 8, it = lane + 64 k;
  // the activation operand of all 4 phases is loaded up front (one HBM latency, not four)
  auto item_pidx = [&](int ph, int k, bool& ok) -> long {
    const int it = lane + 64 * k, pl = it / NG;
    const int py = 2 * (i0 + wave * MW + (pl >> 4)) + (ph >> 1), pxx = 2 * (j0 + (pl & 15)) + (ph & 1);
    ok = py < a.out_h && pxx < a.out_w;
    return ok ? ((long)nimg * a.out_h + py) * a.out_w + pxx : 0;
  };
  uint4 r1[4][4];
  // EP 10: the BatchNorm-backward partials of the stored dx (store_tile_lds EP 10): z is loaded per phase (not up
  // front like the activation operand: 64 more registers beside the 128 accumulators spilled); the lane's 8
  // channels are the same for all of its items (64 % NG == 0)
  const __amdgpu_buffer_rsrc_t rrz = opt_rsrc(EP == 10 ? (const void*)a.bz : nullptr);
  const int cgl = lane % NG;
  float bmu[8], brs[8], bsc[8], bsh[8], ssum[8], ssq[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ssum[i] = 0.f;
    ssq[i] = 0.f;
    if constexpr (EP == 10) {
      const int c = co0 + cgl * 8 + i;
      bmu[i] = a.bmean[c];
      brs[i] = a.brstd[c];
      bsc[i] = a.bgamma[c] * brs[i];
      bsh[i] = a.bbeta[c] - bmu[i] * bsc[i];
    }
  }
#pragma unroll
  for (int ph = 0; ph < 4; ++ph)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      r1[ph][k] = make_uint4(0, 0, 0, 0);
      if (EP == 4) {
        bool ok;
        const long pidx = item_pidx(ph, k, ok);
        r1[ph][k] = buf_load16(rr1, (uint32_t)((pidx * a.r1_cs + (ok ? a.r1_co + co0 + ((lane + 64 * k) % NG) * 8 : 0)) * 2));
      }
    }
#pragma unroll
  for (int ph = 0; ph < 4; ++ph) {
    uint4 zv[4];
    if constexpr (EP == 10) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        bool ok;
        const long pidx = item_pidx(ph, k, ok);
        // (opt_rsrc has no range limit: a pixel outside the image reads pixel 0, whose d is 0)
        zv[k] = buf_load16(rrz, (uint32_t)((pidx * a.bz_cs + co0 + cgl * 8) * 2));
      }
    }
    __syncthreads();  // operands (first phase) / the previous phase's reads are done
#pragma unroll
    for (int m = 0; m < MW; ++m)
#pragma unroll
      for (int t = 0; t < NT; ++t) *(f32x4*)(eb + (m * 16 + col) * EPP + t * 16 + g * 4) = acc[ph][m][t];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int it = lane + 64 * k, pl = it / NG, cg = it % NG;
      bool ok;
      const long oidx = item_pidx(ph, k, ok) * a.out_cs + a.out_co + co0 + cg * 8;
      const float4 s0 = *(const float4*)(eb + pl * EPP + cg * 8), s1 = *(const float4*)(eb + pl * EPP + cg * 8 + 4);
      float v[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      if (EP == 4) {
        Raw8 rr;
        rr.lo = r1[ph][k];
        rr.hi = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float r = raw8_at(rr, false, i);
          v[i] = a.act == 3 ? (r > 0.f ? v[i] : v[i] * a.slope) : (r > 0.f ? v[i] : 0.f);
        }
      }
      const uint4 pk = pack8_bf16(v, 1.f);
      if (ok) *(uint4*)((uint16_t*)a.y + oidx) = pk;
      if constexpr (EP == 10) {
        Raw8 rr, rz;
        rr.lo = pk;
        rz.lo = zv[k];
        rr.hi = rz.hi = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float r = ok ? raw8_at(rr, false, i) : 0.f, z = raw8_at(rz, false, i);
          const float d = fmaf(z, bsc[i], bsh[i]) > 0.f ? r : r * a.bslope;
          ssum[i] += d;
          ssq[i] = fmaf(d, (z - bmu[i]) * brs[i], ssq[i]);
        }
      }
    }
  }
  if constexpr (EP == 10) {
    // lanes with equal lane % NG hold the same 8 channels: xor-shuffles over the other lane bits, then the 4 waves
    // meet in LDS (the staging is free after a barrier) and part[tile][0 / 1][co0 + ch] gets fixed-order fp64 sums
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int m = NG; m < 64; m <<= 1) {
        ssum[i] += __shfl_xor(ssum[i], m);
        ssq[i] += __shfl_xor(ssq[i], m);
      }
    float* red = (float*)smem;
    lds_barrier();  // every wave's reads of the last phase's staging are done
    if (lane < NG) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        red[wave * 2 * CO + lane * 8 + i] = ssum[i];
        red[wave * 2 * CO + CO + lane * 8 + i] = ssq[i];
      }
    }
    lds_barrier();
    if (tid < CO) {
      float ts = 0.f, tq = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        ts += red[w * 2 * CO + tid];
        tq += red[w * 2 * CO + CO + tid];
      }
      const long tile = ((long)nimg * a.tiles_y + ty) * a.tiles_x + tx;
      double* out = a.bn_part + tile * 2 * a.out_c;
      out[co0 + tid] = (double)ts;
      out[a.out_c + co0 + tid] = (double)tq;
    }
  }
}

static int plain_ep(const FwdArgs& a);
static bool fwd_s2_shape(const ClimsrConvDesc* d, const FwdArgs& a) {
  return d->stride == 2 && d->ks == 3 && d->pad == 1 && d->up == 1 && d->cc == 32 && d->in_c % 32 == 0 && d->out_c % 64 == 0 &&
         d->in_coff % 8 == 0 && d->in_cstride % 8 == 0 && a.kcpad == 288 && plain_ep(a) == 8 &&
         // the LDS-DMA kernel's buffer offsets are 32-bit (BUF_OOB past every buffer): larger tensors take the generic conv
         (long)a.n * a.in_h * a.in_w * a.in_cs * 2 < (1L << 31) && (long)a.n * a.out_h * a.out_w * a.out_cs * 2 < (1L << 31) &&
         (long)d->out_c * a.kpk * 2 < (1L << 31);
}

// the LDS-DMA kernel (conv_dma.hip conv_fwd_s2_dma_kernel); the register-staged 8-wave kernel it replaced measured
// 352 against 332 us over the four discriminator stride-2 layers at B=32 (tools/perf_s2.py A/B, r04l)
static int launch_fwd_s2(const ClimsrConvDesc* d, FwdArgs a, hipStream_t s) {
  a.tiles_x = ceil_div(d->out_w, 16);
  a.tiles_y = ceil_div(d->out_h, 16);
  if (g_dry) {
    snprintf(g_dry_name, sizeof(g_dry_name), "conv_fwd_s2_dma_kernel<%s>", a.bn_part ? "true" : "false");
    return CLIMSR_OK;
  }
  const int rc = fwd_s2_dma_launch(a, s);
  return rc == CLIMSR_OK ? check_launch("conv2d_fwd (s2 LDS-DMA)") : rc;
}

static bool dgrad_s2_shape(const ClimsrConvDesc* d, const ClimsrEpilogue* ep, const float* bias) {
  const bool act_ok = ep->act == 0 ? !ep->res1 : ((ep->act == 3 || ep->act == 4) && ep->res1 && !(ep->res_f32 & 1) &&
                                                   ((ep->res1_cstride | ep->res1_coff) & 7) == 0);
  return d->up == -2 && d->stride == 1 && d->ks == 3 && d->pad == 1 && d->cc == 32 && d->in_c % 32 == 0 && d->out_c % 32 == 0 &&
         d->in_coff % 8 == 0 && d->in_cstride % 8 == 0 && ((d->out_cstride | d->out_coff) & 7) == 0 && d->out_h == 2 * d->in_h &&
         d->out_w == 2 * d->in_w && ep->out_mode == 0 && !bias && !ep->res2 && !ep->aux && !ep->down2 && act_ok;
}

// channel blocks grouped per tile in the XCD-major order: the largest divisor of ncob (>= 2) whose weight blocks
// together stay within ~2.5 MB of the XCD's 4 MB L2 (they are re-read by every tile of the group), else 0
// the second dispatch round of a two-workgroups-per-CU launch starts late (conv_fwd_body 'Stagger')
static void set_stagger(FwdArgs& a) {
  const int ncu = device_cus();
  a.stag_lo = ncu;
  a.stag_hi = 2 * ncu;
  a.stag_n = 2;  // 2 x 2048 cycles: GAN step 25.25 -> 24.98 ms (same box, 2 + 6 runs)
}

template <int MW, int NT>
static int launch_dgrad_s2_t(const ClimsrConvDesc* d, FwdArgs a, hipStream_t s) {
  a.tiles_x = ceil_div(d->in_w, 16);
  a.tiles_y = ceil_div(d->in_h, 4 * MW);
  const bool ep4 = a.act == 3 || a.act == 4;
  if (g_dry) {
    snprintf(g_dry_name, sizeof(g_dry_name), "conv_dgrad_s2_kernel<%d, %d, %d>", ep4 ? 4 : a.bz ? 10 : 0, MW, NT);
    return CLIMSR_OK;
  }
  dim3 grid(ceil_div(a.tiles_x * a.tiles_y * a.n, 8) * 8 * (d->out_c / (NT * 16)));
  const int lds = s2d_lds<MW>(NT);

  if (ep4) hipLaunchKernelGGL((conv_dgrad_s2_kernel<4, MW, NT>), grid, dim3(256), lds, s, a);
  else if (a.bz) hipLaunchKernelGGL((conv_dgrad_s2_kernel<10, MW, NT>), grid, dim3(256), lds, s, a);
  else hipLaunchKernelGGL((conv_dgrad_s2_kernel<0, MW, NT>), grid, dim3(256), lds, s, a);
  return check_launch("conv2d_fwd (dgrad s2)");
}

static int launch_dgrad_s2(const ClimsrConvDesc* d, const FwdArgs& a, hipStream_t s) {
  // 64 dx channels: one workgroup per 128 B pixel line (layer 1 with LeakyReLU': 158 -> 150 us at B=32; for wider
  // layers the 4 x 2 form is 2-8 % faster)
  if (d->out_c == 64) return launch_dgrad_s2_t<2, 4>(d, a, s);
  return launch_dgrad_s2_t<4, 2>(d, a, s);
}

static int conv_xcd_group(int ncob, long wblk_bytes) {
  if (ncob < 2) return 0;
  for (int gsz = ncob; gsz >= 2; --gsz)
    if (ncob % gsz == 0 && gsz * wblk_bytes <= (5L << 19)) return gsz;
  return 0;
}

// the LDS-DMA conv (conv_dma.hip)
template <int EP>
static int launch_fwd_dma(const FwdArgs& a0, int ncob, hipStream_t s) {
  FwdArgs a = a0;
  a.tiles_y = ceil_div(a.out_h, DMA_TH);
  a.nchunk = a.in_c / 32;  // 32-channel chunks (of a 32- or 64-channel packing)
  a.xgrp = conv_xcd_group(ncob, (long)64 * a.kpk * 2);
  a.stag_n = 0;
  if (g_dry) {
    snprintf(g_dry_name, sizeof(g_dry_name), "conv_fwd_dma_kernel<%d, %s>", EP, a.res_f32 ? "true" : "false");
    return CLIMSR_OK;
  }
  const int rc = fwd_dma_launch(EP, a, ncob, s);
  return rc == CLIMSR_OK ? check_launch("conv2d_fwd (LDS-DMA)") : rc;
}

#define WIDE_GEO(pfx) ((pfx) == 18)
template <int MW, int NT, int PFX, int PFW, int EP, int GEO>
static int launch_fwd_geo(const FwdArgs& a0, int ncob, size_t lds, hipStream_t s) {
  if constexpr (GEO == 1 && !WIDE_GEO(PFX) && MW == 4 && NT == 4) {
    // the LDS-DMA form for the tiles it fills (32-row tiles: not the 16^2 VGG conv5 layers); with BatchNorm partials
    // (per 16 x 16 tile) only when every 32-row tile holds two whole 16-row tiles
    // RDB conv5 / pull-x (EP 1 / 2: 256 items at B=32 64^2, one round of one workgroup per CU) measured 7 % slower in
    // the GAN step than the two-workgroups-per-CU form (its chunk-0 latency and epilogue are not hidden in a single
    // round)
    const bool fits = (EP == 9 || EP == 10) ? a0.out_h % DMA_TH == 0 : (a0.out_h % DMA_TH == 0 || a0.out_h >= 3 * DMA_TH);
    if (EP != 1 && EP != 2 && !a0.down2 && fits) return launch_fwd_dma<EP>(a0, ncob, s);
  }
  FwdArgs a = a0;
  a.xgrp = GEO == 1 ? conv_xcd_group(ncob, (long)NT * 16 * a.kpk * 2) : 0;
  set_stagger(a);
  if (GEO != 1 || WIDE_GEO(PFX)) a.stag_n = 0;
  const dim3 grid = a.xgrp ? dim3(a.tiles_x * a.tiles_y * a.n * ncob) : dim3(a.tiles_x * a.tiles_y * a.n, ncob);
  const size_t lds_ep = (size_t)4 * MW * 16 * (NT * 16 + 4) * 4;  // epilogue staging (aliases the operands)
  if (lds_ep > lds) lds = lds_ep;
  constexpr int MV = NT == 1 ? 6 : (NT == 2 ? 8 : 4);
  constexpr bool WIDE = PFX == 18;
  if (g_dry) {
    snprintf(g_dry_name, sizeof(g_dry_name), "%s<%d, %d, %s, %d, %d, %d, %d, %d>", WIDE ? "conv_fwd_wide_kernel" : "conv_fwd_kernel", MW, NT,
             a.res_f32 ? "true" : "false", MV, PFX, PFW, EP, GEO);
    return CLIMSR_OK;
  }
  void (*kt)(FwdArgs);
  void (*kf)(FwdArgs);
  if constexpr (WIDE) {
    kt = conv_fwd_wide_kernel<MW, NT, true, MV, PFX, PFW, EP, GEO>;
    kf = conv_fwd_wide_kernel<MW, NT, false, MV, PFX, PFW, EP, GEO>;
  } else {
    kt = conv_fwd_kernel<MW, NT, true, MV, PFX, PFW, EP, GEO>;
    kf = conv_fwd_kernel<MW, NT, false, MV, PFX, PFW, EP, GEO>;
  }
  auto k = a.res_f32 ? kt : kf;
  if (int e = lds_opt_in((const void*)k, 160 * 1024)) return e;
  hipLaunchKernelGGL(k, grid, dim3(256), lds, s, a);
  return check_launch("conv2d_fwd");
}

// the GEO specialisation matching a's geometry (conv_fwd_kernel): 16x16 tiles of 3x3 taps over 32-channel chunks
template <int MW, int NT, int PFX = 0, int PFW = 0, int EP = 0>
static int launch_fwd_ep(const FwdArgs& a, int ncob, size_t lds, hipStream_t s) {
  const bool base = MW == 4 && a.cc == 32 && a.ks == 3 && a.kcpad == 9 * 32;
  if constexpr (MW == 4 && PFX != 18) {
    if (base && a.stride == 1 && a.tpw == TW + 2 && a.ccp == 48 && a.up == 1 && a.in_c % 32 == 0 && a.nchunk * 32 == a.in_c &&
        (long)a.n * a.in_h * a.in_w * a.in_cs * 2 < (1L << 31) && (long)ncob * NT * 16 * a.kpk * 2 < (1L << 31))
      return launch_fwd_geo<MW, NT, PFX, PFW, EP, 1>(a, ncob, lds, s);
  }
  if constexpr (MW == 4 && PFX == 18) {
    if (base && a.stride == 2 && a.tpw == 2 * TW + 1 && a.ccp == 40) return launch_fwd_geo<MW, NT, PFX, PFW, EP, 2>(a, ncob, lds, s);
  }
  return launch_fwd_geo<MW, NT, PFX, PFW, EP, 0>(a, ncob, lds, s);
}

template <int MW, int NT, int PFX = 0, int PFW = 0>
static int launch_fwd(const FwdArgs& a, int ncob, size_t lds, hipStream_t s) {
  return launch_fwd_ep<MW, NT, PFX, PFW, 0>(a, ncob, lds, s);
}


// Epilogue specialisations without residuals (store_tile_lds EP 3 / 6 / 7 / 8), or 0: activation forward with
// (3) / without (6) bias, plain fp32 '=' output (7), plain bf16 output (8).  Needs 8-channel-aligned slices.
static int plain_ep(const FwdArgs& a) {
  if ((a.out_c & 7) || ((a.out_cs | a.out_co) & 7) || a.down2 || a.res1 || a.res2 || a.aux || a.res_f32) return 0;
  if (a.out_mode == 0 && (a.act == 1 || a.act == 2)) return a.bias ? 3 : 6;
  if (a.act == 0 && !a.bias) return a.out_mode == 1 ? 7 : a.out_mode == 0 ? 8 : 0;
  return 0;
}

// The convs whose epilogue can emit BatchNorm partials (EP 9 / conv_fwd_s2_dma_kernel<true>): plain bf16 out over 16x16
// tiles of 64-channel blocks -- the stride-2 kernel, or the chunk-pipelined generic kernel with >= 2 channel blocks
// (so neither conv_pw nor conv_n16 takes it).  Mirrors the dispatch below.
static bool bn_parts_ok(const ClimsrConvDesc* d, const FwdArgs& a, const FwdGeom& g) {
  if (plain_ep(a) != 8 || d->out_c % 64) return false;
  if (d->stride == 2) return fwd_s2_shape(d, a);
  const int nrx = ceil_div(g.tph * g.tpw * (d->cc / 8), 256), nrw = ceil_div(g.nt * 16 * (g.kcpad / 8), 256);
  return d->stride == 1 && d->up == 1 && d->ks == 3 && g.mw == 4 && g.nt == 4 && d->out_c >= 128 && g.nchunk > 1 && nrx <= 6 &&
         nrw <= 9 && g.lds_total <= 160 * 1024;
}

// Backward partials (ep->bn_z): the stride-1 16x16-tile path (EP 10) or the phase-decomposed stride-2 data gradient
static bool bn_bwd_parts_ok(const ClimsrConvDesc* d, const ClimsrEpilogue* ep, const FwdArgs& a, const FwdGeom& g) {
  if (plain_ep(a) != 8) return false;
  if (d->up == -2) return dgrad_s2_shape(d, ep, nullptr);
  return d->stride == 1 && bn_parts_ok(d, a, g);
}

extern "C" int climsr_conv2d_fwd(const ClimsrConvDesc* d, const uint16_t* x, const uint16_t* wpk, const float* bias,
                                 const ClimsrEpilogue* ep, void* y, void* stream);
namespace climsr {
int conv_wr_launch(const ClimsrConvDesc* d, const ClimsrEpilogue* ep, const uint16_t* x, const uint16_t* wpk, int kpk,
                   const float* bias, void* y, hipStream_t s, bool dry, char* name, int name_len);
long conv_wr_ch_parts(const ClimsrConvDesc* d, const ClimsrEpilogue* ep, int* tiles_per_image);
int conv_wr_ep(const ClimsrConvDesc* d, const ClimsrEpilogue* ep, const float* bias);
}

extern "C" int64_t climsr_conv2d_fwd_ch_parts(const ClimsrConvDesc* d, const ClimsrEpilogue* ep, int32_t* tiles_per_image) {
  if (!d || !ep) return 0;
  return conv_wr_ch_parts(d, ep, tiles_per_image);
}

extern "C" int64_t climsr_conv2d_fwd_bn_parts(const ClimsrConvDesc* d, const ClimsrEpilogue* ep) {
  if (!d || !ep || d->cc % 8 || d->cc <= 0 || d->stride < 1) return 0;
  const int mw = (d->out_h >= 12 && fwd_nt(d->out_c) == 4) ? 4 : 2;
  FwdGeom g;
  fwd_geom(d->in_c, d->ks, d->stride, d->out_c, d->cc, mw, &g);
  FwdArgs a{};
  a.act = ep->act; a.out_mode = ep->out_mode; a.down2 = ep->down2; a.res1 = ep->res1; a.res2 = ep->res2; a.aux = (uint16_t*)ep->aux;
  a.res_f32 = ep->res_f32; a.out_c = d->out_c; a.out_cs = d->out_cstride; a.out_co = d->out_coff; a.kcpad = g.kcpad;
  if (ep->bn_z) {
    if (!bn_bwd_parts_ok(d, ep, a, g)) return 0;
    if (d->up == -2) return (int64_t)ceil_div(d->in_w, 16) * ceil_div(d->in_h, 4 * (d->out_c == 64 ? 2 : 4)) * d->n;  // dz tiles
    return (int64_t)ceil_div(d->out_w, TW) * ceil_div(d->out_h, 16) * d->n;
  }
  if (!bn_parts_ok(d, a, g)) return 0;
  return (int64_t)ceil_div(d->out_w, TW) * ceil_div(d->out_h, 16) * d->n;
}

// the LDS-DMA conv's pooled epilogue (EP 11): its GEO-1 shapes (3x3 / stride 1 / 32-channel chunks, 64-channel
// blocks, 32-row tiles) with bias + activation, bf16 out
static bool pool_dma_ok(const ClimsrConvDesc* d, const FwdArgs& a, const FwdGeom& g, int ncob) {
  return d->ks == 3 && d->stride == 1 && d->pad == 1 && d->up == 1 && d->cc == 32 && d->in_c % 32 == 0 && g.kcpad == 288 &&
         g.nchunk * 32 == d->in_c && d->out_c % 64 == 0 && ncob * 64 == d->out_c && d->in_coff % 8 == 0 && d->in_cstride % 8 == 0 &&
         ((d->out_cstride | d->out_coff) & 7) == 0 && a.bias != nullptr && (a.act == 1 || a.act == 2) &&
         (d->out_h % DMA_TH == 0 || d->out_h >= 3 * DMA_TH) && d->out_w % 2 == 0 &&
         (long)d->n * d->in_h * d->in_w * d->in_cstride * 2 < (1L << 31) && (long)d->out_c * g.kpk * 2 < (1L << 31);
}

extern "C" int climsr_conv2d_fwd(const ClimsrConvDesc* d, const uint16_t* x, const uint16_t* wpk, const float* bias,
                                 const ClimsrEpilogue* ep, void* y, void* stream);

extern "C" int climsr_conv2d_fwd_pool_ok(const ClimsrConvDesc* d, const ClimsrEpilogue* ep) {
  if (!d || !ep || !ep->pool2) return 0;
  static uint16_t dummy[8];
  static float fdummy[64];
  g_dry = true;
  const int rc = climsr_conv2d_fwd(d, dummy, dummy, fdummy, ep, dummy, nullptr);
  g_dry = false;
  return rc == CLIMSR_OK ? 1 : 0;
}

extern "C" int climsr_conv2d_fwd(const ClimsrConvDesc* d, const uint16_t* x, const uint16_t* wpk, const float* bias,
                                 const ClimsrEpilogue* ep, void* y, void* stream) {
  if (!d || !x || !wpk || !ep || !y) {
    set_error("conv2d_fwd: null argument");
    return CLIMSR_EINVAL;
  }
  const bool cc4 = d->cc == 4 && d->in_c == 4;  // conv_pw GEO 2 (climsr_conv_chunk_ex)
  if ((d->in_c % 8 && !cc4) || d->in_cstride % 8 || d->in_coff % 8 || (d->cc % 8 && !cc4) || d->cc <= 0 ||
      (d->up != 1 && d->up != 2 && d->up != -2) ||
      (d->stride != 1 && d->stride != 2) || d->ks < 1 || d->n <= 0 || d->out_c <= 0 || d->in_coff + d->in_c > d->in_cstride) {
    set_error("conv2d_fwd: unsupported geometry (in_c=%d cs=%d coff=%d cc=%d up=%d stride=%d ks=%d)", d->in_c, d->in_cstride,
              d->in_coff, d->cc, d->up, d->stride, d->ks);
    return CLIMSR_EINVAL;
  }
  if (ep->down2 && (ep->res2 || ep->res_f32 || bias || ep->act == 1 || ep->act == 2 || (ep->res1 && ep->act < 3) ||
                    (d->out_h & 1) || (d->out_w & 1))) {
    set_error("conv2d_fwd: down2 epilogue: no bias / forward activation / residual (act 3/4 mask only), even output size");
    return CLIMSR_EINVAL;
  }
  if (ep->act < 0 || ep->act > 4 || ((ep->act == 3 || ep->act == 4) && !ep->res1)) {
    set_error("conv2d_fwd: act %d invalid (3/4 need res1 = the activation output)", ep->act);
    return CLIMSR_EINVAL;
  }
  if (ep->ch_part && conv_wr_ep(d, ep, bias) != 3 && conv_wr_ep(d, ep, bias) != 4) {
    set_error("conv2d_fwd: per-tile channel sums only from the 64 -> 64 3x3 register-resident conv "
              "(climsr_conv2d_fwd_ch_parts)");
    return CLIMSR_EINVAL;
  }
  if (ep->aux && ((ep->aux_cstride | ep->aux_coff) & 3)) {
    set_error("conv2d_fwd: aux channel stride/offset must be multiples of 4");
    return CLIMSR_EINVAL;
  }
  {  // epilogue operands are read through 32-bit buffer offsets (opt_rsrc)
    const long opx = (long)d->n * d->out_h * d->out_w;
    const long r1b = ep->res1 ? opx * ep->res1_cstride * ((ep->res_f32 & 1) ? 4 : 2) : 0;
    const long r2b = ep->res2 ? opx * ep->res2_cstride * ((ep->res_f32 & 2) ? 4 : 2) : 0;
    const long yb = opx * d->out_cstride * (ep->out_mode == 0 ? 2 : 4);
    if (r1b >= (1L << 32) - 64 || r2b >= (1L << 32) - 64 || yb >= (1L << 32) - 64) {
      set_error("conv2d_fwd: output / residual operand of %ld B exceeds 32-bit buffer addressing (split the batch)",
                r1b > r2b ? (r1b > yb ? r1b : yb) : (r2b > yb ? r2b : yb));
      return CLIMSR_EINVAL;
    }
  }
  if (ep->pool2 && (ep->out_mode != 0 || ep->act < 0 || ep->act > 2 || ep->res1 || ep->res2 || ep->aux || ep->bn_part || ep->bn_z ||
                    ep->ch_part || ep->down2 || ((d->out_h | d->out_w) & 1))) {
    set_error("conv2d_fwd: pool2 takes bf16 out, bias / activation only, even output size");
    return CLIMSR_EINVAL;
  }
  FwdGeom g;
  // 16x16 output tiles (64 px per wave) for the 64-channel layers; 8x16 otherwise
  const int mw = (d->out_h >= 12 && fwd_nt(d->out_c) == 4) ? 4 : 2;
  fwd_geom(d->in_c, d->ks, d->stride, d->out_c, d->cc, mw, &g);
  FwdArgs a{};  // zero: the optional operands (bz, bn_part, xgrp, ...) default to absent
  a.x = x; a.w = wpk; a.bias = bias; a.y = y;
  a.res1 = ep->res1; a.res2 = ep->res2; a.aux = (uint16_t*)ep->aux;
  a.res_f32 = ep->res_f32; a.beta1 = ep->beta1; a.beta2 = ep->beta2;
  a.aux_cs = ep->aux_cstride; a.aux_co = ep->aux_coff; a.aux_scale = ep->aux_scale;
  a.n = d->n; a.in_h = d->in_h; a.in_w = d->in_w; a.in_c = d->in_c; a.in_cs = d->in_cstride; a.in_co = d->in_coff;
  a.up = d->up; a.ks = d->ks; a.stride = d->stride; a.pad = d->pad; a.out_h = d->out_h; a.out_w = d->out_w;
  a.out_c = d->out_c; a.out_cs = d->out_cstride; a.out_co = d->out_coff; a.cc = d->cc;
  a.tph = g.tph; a.tpw = g.tpw; a.ccp = g.ccp; a.kcpad = g.kcpad; a.nchunk = g.nchunk; a.kpk = g.kpk;
  a.tiles_x = ceil_div(d->out_w, TW); a.tiles_y = ceil_div(d->out_h, g.th);
  a.act = ep->act; a.out_mode = ep->out_mode; a.down2 = ep->down2;
  a.slope = ep->slope; a.alpha1 = ep->alpha1; a.alpha2 = ep->alpha2;
  a.r1_cs = ep->res1_cstride; a.r1_co = ep->res1_coff; a.r2_cs = ep->res2_cstride; a.r2_co = ep->res2_coff;
  a.lds_tab = (int)g.lds_tab; a.lds_x = (int)g.lds_x;
  a.bn_part = ep->bn_part;
  if (ep->bn_part && ep->bn_z) {
    if (!ep->bn_mean || !ep->bn_rstd || !ep->bn_gamma || !ep->bn_beta || ep->bn_z_cstride < d->out_c || ep->bn_z_cstride % 8 ||
        (long)d->n * d->out_h * d->out_w * ep->bn_z_cstride * 2 >= (1L << 31)) {
      set_error("conv2d_fwd: BatchNorm-backward partials need z (channel stride >= out_c, 8-aligned, < 2 GiB) and its statistics");
      return CLIMSR_EINVAL;
    }
    a.bz = ep->bn_z; a.bz_cs = ep->bn_z_cstride; a.bslope = ep->bn_slope;
    a.bmean = ep->bn_mean; a.brstd = ep->bn_rstd; a.bgamma = ep->bn_gamma; a.bbeta = ep->bn_beta;
  }
  int rows = climsr_conv_packed_rows(d->out_c);
  int ncob = rows / (g.nt * 16);
  hipStream_t s = (hipStream_t)stream;
  if (ep->pool2) {  // conv + 2x2 max pool: the register-resident 64 -> 64 conv, or the LDS-DMA conv (EP 11)
    const int rc = conv_wr_launch(d, ep, x, wpk, g.kpk, bias, y, s, g_dry, g_dry_name, (int)sizeof(g_dry_name));
    if (rc != -1) return rc;
    if (pool_dma_ok(d, a, g, ncob)) return launch_fwd_dma<11>(a, ncob, s);
    set_error("conv2d_fwd: no conv + max-pool kernel for this shape (climsr_conv2d_fwd_pool_ok)");
    return CLIMSR_EINVAL;
  }
  if (ep->bn_part && !(ep->bn_z ? bn_bwd_parts_ok(d, ep, a, g) : bn_parts_ok(d, a, g))) {
    set_error("conv2d_fwd: BatchNorm partials only for the 16x16-tile bf16 paths (climsr_conv2d_fwd_bn_parts)");
    return CLIMSR_EINVAL;
  }
  if (d->out_c == 1 && d->stride == 1 && d->up == 1 && !ep->down2 && !ep->res2 && co1m_shape(d))
    return dispatch_co1m(d, a, s);
  if (d->out_c == 1 && d->stride == 1 && d->up == 1 && !ep->down2 && !ep->res2) {
    a.tiles_x = ceil_div(d->out_w, 16);
    a.tiles_y = ceil_div(d->out_h, 16);
    size_t lds = (size_t)(15 + d->ks) * (15 + d->ks) * (CO1_CC + 8) * 2 + (size_t)d->ks * d->ks * CO1_CC * 2;
    if (g_dry) {
      snprintf(g_dry_name, sizeof(g_dry_name), "conv_co1_kernel");
      return CLIMSR_OK;
    }
    hipLaunchKernelGGL(conv_co1_kernel, dim3(a.tiles_x * a.tiles_y * a.n), dim3(256), lds, s, a);
    return check_launch("conv2d_fwd (co1)");
  }
  if (n16_shape(d->in_c, d->ks, d->out_c) && d->cc == 32 * n16_ncb(d->in_c) && d->stride == 1 && d->up == 1 && d->pad == 1 &&
      !ep->down2 && !ep->res_f32 && d->out_h == d->in_h && d->out_w == d->in_w &&
      (long)d->n * d->in_h * d->in_w * d->in_cstride * 2 < (1L << 31)) {  // 32-bit buffer offsets
    a.tiles_x = ceil_div(d->out_w, TW);
    a.tiles_y = ceil_div(d->out_h, N16_TH);
    // epilogue specialisations (see conv_n16_kernel): forward conv1-4 and the pull data gradients
    const bool al = ((a.out_cs | a.out_co) & 3) == 0 && d->out_c == 16;
    const int ep_mode = (al && a.act == 1 && a.bias && !a.res1 && !a.res2 && !a.aux && a.out_mode == 0) ? 1
                        : (al && a.act == 3 && !a.bias && a.res1 && !(a.res_f32 & 1) && ((a.r1_cs | a.r1_co) & 3) == 0 &&
                           !a.res2 && !a.aux && a.out_mode == 0)
                            ? 2
                            : 0;
    switch ((d->cc / 32) * 4 + ep_mode) {
      case 4: return launch_n16<1, 0>(a, s);
      case 5: return launch_n16<1, 1>(a, s);
      case 6: return launch_n16<1, 2>(a, s);
      case 8: return launch_n16<2, 0>(a, s);
      case 9: return launch_n16<2, 1>(a, s);
      case 10: return launch_n16<2, 2>(a, s);
      case 17: return launch_n16<4, 1>(a, s);
      case 18: return launch_n16<4, 2>(a, s);
      default: return launch_n16<4, 0>(a, s);
    }
  }
  if (dgrad_s2_shape(d, ep, bias) && (long)d->n * d->out_h * d->out_w * ep->res1_cstride * 2 < (1L << 32) - 64)
    return launch_dgrad_s2(d, a, s);
  if (fwd_s2_shape(d, a)) return launch_fwd_s2(d, a, s);
  // RDB conv5 / pull-x (128 -> 64 3x3): row streaming with input-row reuse (rdb_conv5.hip)

  if (pt_shape(d, ep) && (d->out_c == 16 || d->out_c == 32 || d->out_c == 64) &&
      (d->in_c == 32 || d->in_c == 64 || d->in_c == 128))
    return dispatch_pt(d, a, s);
  {  // 64 -> 64 3x3: the weights resident in registers, wave-independent tiles (conv_wr.hip)
    const int rc = conv_wr_launch(d, ep, x, wpk, g.kpk, bias, y, s, g_dry, g_dry_name, (int)sizeof(g_dry_name));
    if (rc != -1) return rc;
  }
  {  // weights-resident persistent kernel for one-chunk convs with 17..64 outputs (large-pixel-count layers)
    const int nt = fwd_nt(d->out_c);
    const long npx = (long)d->n * d->out_h * d->out_w;
    PwGeom pg;
    if (ncob == 1 && (nt == 4 || nt == 2) && d->up != -2 && (npx >= 4096 || cc4) &&
        (long)d->n * d->in_h * d->in_w * d->in_cstride * 2 < (1L << 31)) {  // 32-bit buffer offsets
      // 8 waves x 2 rows (two waves per SIMD) when the LDS allows, else 4 waves x 2 rows
      if (pw_geom(d, nt, 2, &pg, 8) && pg.nvx <= 512 * 7 && (d->out_h >= 16 || cc4)) {
        // epilogue specialisations (store_tile_lds EP 3 / 4): activation forward / activation backward
        const bool v8 = (a.out_c & 7) == 0 && ((a.out_cs | a.out_co) & 7) == 0 && !a.down2 && !a.res2 && !a.aux &&
                        a.out_mode == 0 && a.res_f32 == 0;
        const bool d2 = a.down2 && a.out_c == 64 && ((a.out_cs | a.out_co) & 3) == 0 && !a.bias && a.res1 && a.res_f32 == 0 &&
                        ((a.r1_cs | a.r1_co) & 3) == 0 && (a.act == 3 || a.act == 4) && !a.res2 && !a.aux && a.out_mode == 0;
        const int epm = (v8 && a.bias && !a.res1 && (a.act == 1 || a.act == 2)) ? 3
                        : (v8 && !a.bias && a.res1 && ((a.r1_cs | a.r1_co) & 7) == 0 && (a.act == 3 || a.act == 4)) ? 4
                        : d2 ? 5 : 0;
        if (nt == 4 && epm == 0) {
          switch (plain_ep(a)) {
            case 6: return launch_pw<8, 2, 4, 7, 6>(a, pg, s);
            case 7: return launch_pw<8, 2, 4, 7, 7>(a, pg, s);
            case 8: return launch_pw<8, 2, 4, 7, 8>(a, pg, s);
            default: break;
          }
        }
        if (nt == 4) return epm == 3 ? launch_pw<8, 2, 4, 7, 3>(a, pg, s) : epm == 4 ? launch_pw<8, 2, 4, 7, 4>(a, pg, s)
                            : epm == 5 ? launch_pw<8, 2, 4, 7, 5>(a, pg, s) : launch_pw<8, 2, 4, 7>(a, pg, s);
        return epm == 3 ? launch_pw<8, 2, 2, 7, 3>(a, pg, s) : epm == 4 ? launch_pw<8, 2, 2, 7, 4>(a, pg, s)
                                                                        : launch_pw<8, 2, 2, 7>(a, pg, s);
      }
      if (pw_geom(d, nt, 2, &pg, 4)) return nt == 4 ? launch_pw<4, 2, 4, 12>(a, pg, s) : launch_pw<4, 2, 2, 12>(a, pg, s);
    }
  }
  if (cc4) {
    set_error("conv2d_fwd: 4-channel chunks need the conv_pw path (stride 1, up 1/2, 64 outputs, 32-bit offsets)");
    return CLIMSR_EINVAL;
  }
  if (g.lds_total > 160 * 1024) {
    set_error("conv2d_fwd: LDS %zu exceeds 160 KiB (cc=%d)", g.lds_total, d->cc);
    return CLIMSR_EINVAL;
  }
  if (mw == 4) {
    // multi-chunk tiles whose per-thread staging fits 6 input + 9 weight vectors: chunk-pipelined variant
    const int nrx = ceil_div(g.tph * g.tpw * (d->cc / 8), 256), nrw = ceil_div(g.nt * 16 * (g.kcpad / 8), 256);
    if (g.nchunk > 1 && nrx <= 6 && nrw <= 9) {
      // epilogue specialisations (store_tile_lds EP): residual forward (conv5, trunk_conv) / fp32 pull-x
      const bool v8 = (a.out_c & 7) == 0 && ((a.out_cs | a.out_co) & 7) == 0 && ((a.r1_cs | a.r1_co) & 7) == 0 &&
                      (!a.res2 || ((a.r2_cs | a.r2_co) & 7) == 0) && (!a.aux || ((a.aux_cs | a.aux_co) & 7) == 0) && !a.down2 &&
                      a.act == 0 && a.res1;
      if (v8 && a.bias && a.res_f32 == 0 && a.out_mode == 0 && !a.aux) return launch_fwd_ep<4, 4, 6, 9, 1>(a, ncob, g.lds_total, s);
      if (v8 && !a.bias && (a.res_f32 & 1) && (!a.res2 || (a.res_f32 & 2)) && a.out_mode == 1)
        return launch_fwd_ep<4, 4, 6, 9, 2>(a, ncob, g.lds_total, s);
      // activation backward from a bf16 activation, bf16 out (the discriminator's layer-1 data gradient)
      if (!a.bias && a.res1 && (a.act == 3 || a.act == 4) && a.res_f32 == 0 && !a.res2 && !a.aux && !a.down2 && a.out_mode == 0 &&
          (a.out_c & 7) == 0 && ((a.out_cs | a.out_co | a.r1_cs | a.r1_co) & 7) == 0)
        return launch_fwd_ep<4, 4, 6, 9, 4>(a, ncob, g.lds_total, s);
      switch (plain_ep(a)) {
        case 3: return launch_fwd_ep<4, 4, 6, 9, 3>(a, ncob, g.lds_total, s);
        case 6: return launch_fwd_ep<4, 4, 6, 9, 6>(a, ncob, g.lds_total, s);
        case 7: return launch_fwd_ep<4, 4, 6, 9, 7>(a, ncob, g.lds_total, s);
        case 8: return a.bz ? launch_fwd_ep<4, 4, 6, 9, 10>(a, ncob, g.lds_total, s)
                       : a.bn_part ? launch_fwd_ep<4, 4, 6, 9, 9>(a, ncob, g.lds_total, s) : launch_fwd_ep<4, 4, 6, 9, 8>(a, ncob, g.lds_total, s);
        default: return launch_fwd<4, 4, 6, 9>(a, ncob, g.lds_total, s);
      }
    }
    // large input tiles (stride 2: 33x33 pixels per 16x16 outputs) with several chunks: the deeper-prefetch
    // variant (one workgroup per CU already, so the 18 staging vectors per thread cost no occupancy)
    if (g.nchunk > 1 && nrx <= 18 && nrw <= 9) {
      if (plain_ep(a) == 8) return launch_fwd_ep<4, 4, 18, 9, 8>(a, ncob, g.lds_total, s);
      return launch_fwd<4, 4, 18, 9>(a, ncob, g.lds_total, s);
    }
    switch (plain_ep(a)) {
      case 3: return launch_fwd_ep<4, 4, 0, 0, 3>(a, ncob, g.lds_total, s);
      case 6: return launch_fwd_ep<4, 4, 0, 0, 6>(a, ncob, g.lds_total, s);
      case 7: return launch_fwd_ep<4, 4, 0, 0, 7>(a, ncob, g.lds_total, s);
      case 8: return launch_fwd_ep<4, 4, 0, 0, 8>(a, ncob, g.lds_total, s);
      default: break;
    }
    return launch_fwd<4, 4>(a, ncob, g.lds_total, s);
  }
  switch (g.nt) {
    case 1: return launch_fwd<2, 1>(a, ncob, g.lds_total, s);
    case 2: return launch_fwd<2, 2>(a, ncob, g.lds_total, s);
    default: return launch_fwd<2, 4>(a, ncob, g.lds_total, s);
  }
}

extern "C" const char* climsr_conv2d_fwd_kernel(const ClimsrConvDesc* d, const float* bias, const ClimsrEpilogue* ep) {
  static uint16_t dummy[8];
  g_dry = true;
  g_dry_name[0] = 0;
  const int rc = climsr_conv2d_fwd(d, dummy, dummy, bias, ep, dummy, nullptr);
  g_dry = false;
  return rc == CLIMSR_OK ? g_dry_name : "";
}

extern "C" int climsr_dgrad_single_output(int n, int h, int w, int ks, int pad, const uint16_t* dz, int dz_cstride, int dz_coff,
                                          const float* weight, int c, int act, float slope, const uint16_t* res1, int res1_cstride,
                                          int res1_coff, uint16_t* out, int out_cstride, int out_coff, void* stream);

extern "C" const char* climsr_dgrad_single_output_kernel(int ks, int c, int act) {
  static uint16_t dummy[8];
  static float wdummy[8];
  g_dry = true;
  g_dry_name[0] = 0;
  const int rc = climsr_dgrad_single_output(1, 1, 1, ks, ks / 2, dummy, 8, 0, wdummy, c, act, 0.2f, dummy, 8, 0, dummy, c, 0, nullptr);
  g_dry = false;
  return rc == CLIMSR_OK ? g_dry_name : "";
}
