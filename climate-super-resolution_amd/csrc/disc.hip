// Discriminator / perceptual-loss / GAN-loss kernels for CDNA4 (gfx950).
//
// Replaces, on the RFB-ESRGAN discriminator path (climsr/models/rfb_esrgan.py:26-69) and the GAN
// task (climsr/task/pl_gan.py:28-61): nn.BatchNorm2d (train-mode batch statistics, running-stat
// update), nn.AdaptiveAvgPool2d((14,14)), nn.Linear(100352,1024) + LeakyReLU + Linear(1024,1) +
// Sigmoid, BCEWithLogitsLoss on the relativistic logits, and for the perceptual loss
// (climsr/losses/perceptual.py) VGG's MaxPool2d(2,2) and the L1 between bf16 feature maps.
// Deterministic: every reduction is a fixed-shape tree with fp64 partials.
#include <math.h>

#include "common.h"

using namespace climsr;

namespace {

__device__ inline void unpack8(uint4 u, float* f) {
  uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = bf2f((uint16_t)(w[i >> 1] >> ((i & 1) * 16)));
}

__device__ inline uint4 pack8(const float* f) {
  uint4 u;
  u.x = f2bf(f[0]) | ((uint32_t)f2bf(f[1]) << 16);
  u.y = f2bf(f[2]) | ((uint32_t)f2bf(f[3]) << 16);
  u.z = f2bf(f[4]) | ((uint32_t)f2bf(f[5]) << 16);
  u.w = f2bf(f[6]) | ((uint32_t)f2bf(f[7]) << 16);
  return u;
}

// ---------------------------------------------------------------------------------------------
// BatchNorm2d (train mode) over an NHWC [npix][c] bf16 tensor (rfb_esrgan.py:32-50; discriminator.py:17-18).
//
// Thread layout shared by the statistics and apply kernels: G = c/8 channel groups (one uint4 = 8 bf16
// channels per load), R = 256/G pixel rows per 256-thread block; thread (cg = tid % G, r = tid / G) owns the
// 8 channels cg*8.. for every R-th pixel of its block's range, so each block streams one contiguous
// [pixels x c] slab (coalesced) and a thread's per-channel constants live in registers.  Pixel counts fit
// in 32 bits (npix * c < 2^31 is checked on the host), so there is no 64-bit division anywhere.
//
// Statistics: every thread accumulates fp32 over <= BN_PX_PER_THREAD pixels (4 loads in flight), the block
// combines its R rows in fp64 in a fixed order and writes fp64 partials [P][2][c]; the finish kernel sums the
// P partials (8 slices per channel, fixed order) -> deterministic for a given shape.
// mode 0 (forward): sums of z and z^2.  mode 1 (backward): d = da * lrelu'(a); sums of d and d * xhat,
// xhat = (z - mean) * rstd.
// ---------------------------------------------------------------------------------------------
constexpr int BN_MAX_PARTS = 2048;
constexpr long BN_TARGET_BLOCKS = 1024;  // >= 4 blocks (16 waves) per CU in flight for these streaming kernels

struct BnGrid {
  int parts;    // statistics blocks P
  int per_blk;  // pixels per statistics block (multiple of R)
};

// Pixels per thread: as many as keep >= BN_TARGET_BLOCKS blocks (4..64), so small late layers (512 ch x 8 K px)
// still fill the chip and large early ones amortise the partials.
static inline int bn_px_per_thread(long npix, int c) {
  const long threads_px = npix * (c / 8) / (BN_TARGET_BLOCKS * 256);
  return (int)(threads_px < 4 ? 4 : threads_px > 64 ? 64 : threads_px);
}

static inline BnGrid bn_grid(long npix, int c) {
  const int G = c / 8;
  const int R = 256 / G;
  long per = (long)R * bn_px_per_thread(npix, c);
  const long need = (npix + BN_MAX_PARTS - 1) / BN_MAX_PARTS;
  if (per < need) per = (need + R - 1) / R * R;
  return BnGrid{(int)((npix + per - 1) / per), (int)per};
}

// 8 consecutive channels of an output gradient held as fp32 (32 B) or bf16 (16 B)
__device__ inline void load_da8(const float* da, size_t off, float* d) {
  const float4* dp = (const float4*)(da + off);
  const float4 d0 = dp[0], d1 = dp[1];
  d[0] = d0.x; d[1] = d0.y; d[2] = d0.z; d[3] = d0.w; d[4] = d1.x; d[5] = d1.y; d[6] = d1.z; d[7] = d1.w;
}
__device__ inline void load_da8(const uint16_t* da, size_t off, float* d) { unpack8(*(const uint4*)(da + off), d); }

// BN affine of the forward (bn_apply_kernel): y = z * sc + sh, sc = gamma*rstd, sh = beta - mean*sc, the same
// fmaf, so sign(y) -- hence lrelu'(a) -- is recomputed bit-identically from z without reading a.
template <int MODE, typename DA = float>
__global__ __launch_bounds__(256) void bn_stats_kernel(int npix, int c, int per_blk, const uint16_t* __restrict__ z,
                                                       const DA* __restrict__ da, const uint16_t* __restrict__ a,
                                                       const float* __restrict__ mean, const float* __restrict__ rstd,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       float slope, double* __restrict__ part) {
  __shared__ float ls[2][2048];  // [sum | sumsq][R][c] (R * c <= 2048)
  const int G = c >> 3;
  const int R = 256 / G;
  const int tid = threadIdx.x;
  const int cg = tid % G;
  const int r = tid / G;
  const int p0 = blockIdx.x * per_blk;
  const int p1 = min(p0 + per_blk, npix);
  float s[8], q[8], mu[8], rs[8], sc[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { s[i] = 0.f; q[i] = 0.f; mu[i] = 0.f; rs[i] = 0.f; sc[i] = 0.f; sh[i] = 0.f; }
  if (r < R) {
    if (MODE >= 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) { mu[i] = mean[cg * 8 + i]; rs[i] = rstd[cg * 8 + i]; }
    }
    if (MODE == 2) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        sc[i] = gamma[cg * 8 + i] * rs[i];
        sh[i] = beta[cg * 8 + i] - mu[i] * sc[i];
      }
    }
    auto accum = [&](int p) {
      float zf[8];
      unpack8(*(const uint4*)(z + (size_t)p * c + cg * 8), zf);
      if (MODE == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) { s[i] += zf[i]; q[i] = fmaf(zf[i], zf[i], q[i]); }
      } else {
        float af[8], dd[8];
        if (MODE == 1) {
          unpack8(*(const uint4*)(a + (size_t)p * c + cg * 8), af);
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) af[i] = fmaf(zf[i], sc[i], sh[i]);
        }
        load_da8(da, (size_t)p * c + cg * 8, dd);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float d = af[i] > 0.f ? dd[i] : dd[i] * slope;
          s[i] += d;
          q[i] = fmaf(d, (zf[i] - mu[i]) * rs[i], q[i]);
        }
      }
    };
    int p = p0 + r;
    for (; p + 3 * R < p1; p += 4 * R) {
      accum(p);
      accum(p + R);
      accum(p + 2 * R);
      accum(p + 3 * R);
    }
    for (; p < p1; p += R) accum(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      ls[0][r * c + cg * 8 + i] = s[i];
      ls[1][r * c + cg * 8 + i] = q[i];
    }
  }
  __syncthreads();
  for (int ch = tid; ch < c; ch += 256) {
    double ts = 0.0, tq = 0.0;
    for (int rr = 0; rr < R; ++rr) {
      ts += (double)ls[0][rr * c + ch];
      tq += (double)ls[1][rr * c + ch];
    }
    double* out = part + (size_t)blockIdx.x * 2 * c;
    out[ch] = ts;
    out[c + ch] = tq;
  }
}

// Sum of the P partials of channel ch: a block owns 8 channels (one 64 B row segment) x 32 slices; slice sl sums
// partials sl, sl+32, ... with 4 independent chains, then the 32 slice sums are added in a fixed order.
__device__ inline void bn_sum_parts(const double* __restrict__ part, int parts, int c, double* red, double& s, double& q,
                                    int& ch) {
  const int lane = threadIdx.x & 7, sl = threadIdx.x >> 3;
  ch = blockIdx.x * 8 + lane;
  double ts[4] = {0.0, 0.0, 0.0, 0.0}, tq[4] = {0.0, 0.0, 0.0, 0.0};
  if (ch < c) {
    int b = sl;
    for (; b + 96 < parts; b += 128) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        ts[u] += part[(size_t)(b + 32 * u) * 2 * c + ch];
        tq[u] += part[(size_t)(b + 32 * u) * 2 * c + c + ch];
      }
    }
    for (; b < parts; b += 32) {
      ts[0] += part[(size_t)b * 2 * c + ch];
      tq[0] += part[(size_t)b * 2 * c + c + ch];
    }
  }
  red[threadIdx.x] = (ts[0] + ts[1]) + (ts[2] + ts[3]);
  red[256 + threadIdx.x] = (tq[0] + tq[1]) + (tq[2] + tq[3]);
  __syncthreads();
  s = 0.0;
  q = 0.0;
  if (sl == 0) {
    for (int k = 0; k < 32; ++k) {
      s += red[k * 8 + lane];
      q += red[256 + k * 8 + lane];
    }
  }
}

__global__ __launch_bounds__(256) void bn_finish_stats_kernel(const double* __restrict__ part, int parts, int c, int npix,
                                                              float eps, float momentum, float* mean, float* rstd,
                                                              float* run_mean, float* run_var, int64_t* nbt) {
  __shared__ double red[512];
  double s, q;
  int ch;
  bn_sum_parts(part, parts, c, red, s, q, ch);
  if ((threadIdx.x >> 3) != 0 || ch >= c) return;
  const double m = s / (double)npix;
  double var = q / (double)npix - m * m;
  if (var < 0.0) var = 0.0;
  mean[ch] = (float)m;
  rstd[ch] = (float)(1.0 / sqrt(var + (double)eps));
  if (run_mean) {
    const double unb = npix > 1 ? var * (double)npix / (double)(npix - 1) : var;
    run_mean[ch] = (float)((1.0 - momentum) * run_mean[ch] + momentum * m);
    run_var[ch] = (float)((1.0 - momentum) * run_var[ch] + momentum * unb);
  }
  if (nbt && ch == 0) *nbt += 1;  // BatchNorm2d.num_batches_tracked
}

// y = act(z * scale + shift) with scale = gamma*rstd, shift = beta - mean*scale (mode 0: batch statistics
// mean/rstd; mode 1: running statistics, rstd = rsqrt(var + eps)).  ACT (0 none, 1 leaky relu, 2 relu) a template
// parameter: as an argument it compiled to a uniform three-way branch per element (165 branches in the loop).
template <int MODE, int ACT>
__global__ __launch_bounds__(256) void bn_apply_kernel(int npix, int c, int per_blk, const uint16_t* __restrict__ z,
                                                       const float* __restrict__ mean, const float* __restrict__ var_or_rstd,
                                                       float eps, const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       float slope, uint16_t* __restrict__ y) {
  const int G = c >> 3;
  const int R = 256 / G;
  const int cg = threadIdx.x % G;
  const int r = threadIdx.x / G;
  if (r >= R) return;
  float sc[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int ch = cg * 8 + i;
    const float rs = MODE == 0 ? var_or_rstd[ch] : rsqrtf(var_or_rstd[ch] + eps);
    sc[i] = gamma[ch] * rs;
    sh[i] = beta[ch] - mean[ch] * sc[i];
  }
  const int p0 = blockIdx.x * per_blk;
  const int p1 = min(p0 + per_blk, npix);
  auto one = [&](int p) {
    float f[8];
    const size_t off = (size_t)p * c + cg * 8;
    unpack8(*(const uint4*)(z + off), f);
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = act_apply(fmaf(f[i], sc[i], sh[i]), ACT, slope);
    *(uint4*)(y + off) = pack8(f);
  };
  int p = p0 + r;
  for (; p + 3 * R < p1; p += 4 * R) {
    one(p);
    one(p + R);
    one(p + 2 * R);
    one(p + 3 * R);
  }
  for (; p < p1; p += R) one(p);
}

// Backward coefficients: dgamma (+)= sum(d*xhat), dbeta (+)= sum(d); coef = {gamma*rstd, mean(d), mean(d*xhat)}.
__global__ __launch_bounds__(256) void bn_bwd_finish_kernel(const double* __restrict__ part, int parts, int c, int npix,
                                                            const float* __restrict__ gamma, const float* __restrict__ rstd,
                                                            float* dgamma, float* dbeta, int accumulate, float* coef) {
  __shared__ double red[512];
  double s, q;
  int ch;
  bn_sum_parts(part, parts, c, red, s, q, ch);
  if ((threadIdx.x >> 3) != 0 || ch >= c) return;
  if (dgamma) dgamma[ch] = (accumulate ? dgamma[ch] : 0.f) + (float)q;
  if (dbeta) dbeta[ch] = (accumulate ? dbeta[ch] : 0.f) + (float)s;
  coef[ch] = gamma[ch] * rstd[ch];
  coef[c + ch] = (float)(s / (double)npix);
  coef[2 * c + ch] = (float)(q / (double)npix);
}

// dz = gamma*rstd * (d - mean(d) - xhat * mean(d*xhat)), d = da * lrelu'(a); out_slope != 1: z is itself a
// LeakyReLU output (plain discriminator) and dz carries its derivative too.
// FROM_Z: lrelu'(a) from the recomputed BN output (no read of a; MODE 2 of the statistics kernel).
template <typename DA = float, bool FROM_Z = false>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(int npix, int c, int per_blk, const DA* __restrict__ da,
                                                           const uint16_t* __restrict__ a, const uint16_t* __restrict__ z,
                                                           const float* __restrict__ mean, const float* __restrict__ rstd,
                                                           const float* __restrict__ gamma, const float* __restrict__ beta,
                                                           const float* __restrict__ coef, float slope, float out_slope,
                                                           uint16_t* __restrict__ dz) {
  const int G = c >> 3;
  const int R = 256 / G;
  const int cg = threadIdx.x % G;
  const int r = threadIdx.x / G;
  if (r >= R) return;
  float k[8], m1[8], m2[8], mu[8], rs[8], sc[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int ch = cg * 8 + i;
    k[i] = coef[ch];
    m1[i] = coef[c + ch];
    m2[i] = coef[2 * c + ch];
    mu[i] = mean[ch];
    rs[i] = rstd[ch];
    sc[i] = FROM_Z ? gamma[ch] * rs[i] : 0.f;
    sh[i] = FROM_Z ? beta[ch] - mu[i] * sc[i] : 0.f;
  }
  const int p0 = blockIdx.x * per_blk;
  const int p1 = min(p0 + per_blk, npix);
  auto one = [&](int p) {
    const size_t off = (size_t)p * c + cg * 8;
    float zf[8], af[8], o[8], dd[8];
    unpack8(*(const uint4*)(z + off), zf);
    if (FROM_Z) {
#pragma unroll
      for (int i = 0; i < 8; ++i) af[i] = fmaf(zf[i], sc[i], sh[i]);
    } else {
      unpack8(*(const uint4*)(a + off), af);
    }
    load_da8(da, off, dd);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float d = af[i] > 0.f ? dd[i] : dd[i] * slope;
      const float xh = (zf[i] - mu[i]) * rs[i];
      o[i] = k[i] * (d - m1[i] - xh * m2[i]);
      if (out_slope != 1.f && zf[i] <= 0.f) o[i] *= out_slope;
    }
    *(uint4*)(dz + off) = pack8(o);
  };
  int p = p0 + r;
  for (; p + 3 * R < p1; p += 4 * R) {
    one(p);
    one(p + R);
    one(p + 2 * R);
    one(p + 3 * R);
  }
  for (; p < p1; p += R) one(p);
}

template <int MODE>
static void launch_bn_apply(hipStream_t s, int nb, int npix, int c, int per, const uint16_t* z, const float* mean, const float* v,
                            float eps, const float* gamma, const float* beta, int act, float slope, uint16_t* y) {
  if (act == 1)
    hipLaunchKernelGGL((bn_apply_kernel<MODE, 1>), dim3(nb), dim3(256), 0, s, npix, c, per, z, mean, v, eps, gamma, beta, slope, y);
  else if (act == 2)
    hipLaunchKernelGGL((bn_apply_kernel<MODE, 2>), dim3(nb), dim3(256), 0, s, npix, c, per, z, mean, v, eps, gamma, beta, slope, y);
  else
    hipLaunchKernelGGL((bn_apply_kernel<MODE, 0>), dim3(nb), dim3(256), 0, s, npix, c, per, z, mean, v, eps, gamma, beta, slope, y);
}

static inline int bn_apply_grid(long npix, int c, int* per_blk) {
  const int R = 256 / (c / 8);
  *per_blk = R * bn_px_per_thread(npix, c);
  return ceil_div(npix, *per_blk);
}

static bool bn_shape_ok(int64_t npix, int c) { return c > 0 && c % 8 == 0 && c <= 2048 && npix > 0 && npix * (int64_t)c < (1ll << 31); }

}  // namespace

extern "C" int64_t climsr_bn_workspace_doubles(int64_t npix, int c) {
  if (!bn_shape_ok(npix, c)) return 0;
  return (int64_t)bn_grid(npix, c).parts * 2 * c;
}

extern "C" int climsr_bn_forward(const uint16_t* z, int64_t npix, int c, const float* gamma, const float* beta, int act, float slope,
                                 float eps, float momentum, double* workspace, float* mean, float* rstd, float* run_mean,
                                 float* run_var, int64_t* num_batches_tracked, uint16_t* y, void* stream) {
  if (!z || !gamma || !beta || !workspace || !mean || !rstd || !y || !bn_shape_ok(npix, c)) {
    set_error("bn_forward: bad args (c=%d, npix=%lld)", c, (long long)npix);
    return CLIMSR_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  const BnGrid g = bn_grid(npix, c);
  hipLaunchKernelGGL(bn_stats_kernel<0>, dim3(g.parts), dim3(256), 0, s, (int)npix, c, g.per_blk, z, (const float*)nullptr, nullptr,
                     nullptr, nullptr, nullptr, nullptr, 0.f, workspace);
  hipLaunchKernelGGL(bn_finish_stats_kernel, dim3(ceil_div(c, 8)), dim3(256), 0, s, workspace, g.parts, c, (int)npix, eps,
                     momentum, mean, rstd, run_mean, run_var, num_batches_tracked);
  int per;
  const int nb = bn_apply_grid(npix, c, &per);
  launch_bn_apply<0>(s, nb, (int)npix, c, per, z, mean, rstd, 0.f, gamma, beta, act, slope, y);
  return check_launch("bn_forward");
}

extern "C" int climsr_bn_forward_parts(const double* parts, int64_t nparts, const uint16_t* z, int64_t npix, int c, const float* gamma,
                                       const float* beta, int act, float slope, float eps, float momentum, float* mean, float* rstd,
                                       float* run_mean, float* run_var, int64_t* num_batches_tracked, uint16_t* y, void* stream) {
  if (!parts || nparts <= 0 || nparts > (1L << 30) || !z || !gamma || !beta || !mean || !rstd || !y || !bn_shape_ok(npix, c)) {
    set_error("bn_forward_parts: bad args (c=%d, npix=%lld, parts=%lld)", c, (long long)npix, (long long)nparts);
    return CLIMSR_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_finish_stats_kernel, dim3(ceil_div(c, 8)), dim3(256), 0, s, parts, (int)nparts, c, (int)npix, eps, momentum,
                     mean, rstd, run_mean, run_var, num_batches_tracked);
  int per;
  const int nb = bn_apply_grid(npix, c, &per);
  launch_bn_apply<0>(s, nb, (int)npix, c, per, z, mean, rstd, 0.f, gamma, beta, act, slope, y);
  return check_launch("bn_forward_parts");
}

extern "C" int climsr_bn_inference(const uint16_t* z, int64_t npix, int c, const float* run_mean, const float* run_var, float eps,
                                   const float* gamma, const float* beta, int act, float slope, uint16_t* y, void* stream) {
  if (!z || !run_mean || !run_var || !gamma || !beta || !y || !bn_shape_ok(npix, c)) {
    set_error("bn_inference: bad args");
    return CLIMSR_EINVAL;
  }
  int per;
  const int nb = bn_apply_grid(npix, c, &per);
  launch_bn_apply<1>((hipStream_t)stream, nb, (int)npix, c, per, z, run_mean, run_var, eps, gamma, beta, act, slope, y);
  return check_launch("bn_inference");
}

extern "C" int climsr_bn_backward(const float* da, const uint16_t* a, const uint16_t* z, int64_t npix, int c, const float* mean,
                                  const float* rstd, const float* gamma, float slope, float out_slope, double* workspace, float* coef,
                                  float* dgamma, float* dbeta, int accumulate, uint16_t* dz, void* stream) {
  if (!da || !a || !z || !mean || !rstd || !gamma || !workspace || !coef || !dz || !bn_shape_ok(npix, c)) {
    set_error("bn_backward: bad args");
    return CLIMSR_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  const BnGrid g = bn_grid(npix, c);
  hipLaunchKernelGGL(bn_stats_kernel<1>, dim3(g.parts), dim3(256), 0, s, (int)npix, c, g.per_blk, z, da, a, mean, rstd, nullptr,
                     nullptr, slope, workspace);
  hipLaunchKernelGGL(bn_bwd_finish_kernel, dim3(ceil_div(c, 8)), dim3(256), 0, s, workspace, g.parts, c, (int)npix, gamma, rstd,
                     dgamma, dbeta, accumulate, coef);
  int per;
  const int nb = bn_apply_grid(npix, c, &per);
  hipLaunchKernelGGL((bn_bwd_apply_kernel<float, false>), dim3(nb), dim3(256), 0, s, (int)npix, c, per, da, a, z, mean, rstd, nullptr,
                     nullptr, coef, slope, out_slope, dz);
  return check_launch("bn_backward");
}

// BatchNorm2d + LeakyReLU backward without the activation: lrelu'(a) comes from sign(z * gamma*rstd + beta -
// mean*gamma*rstd), recomputed exactly as the forward applied it; da is bf16 (da_bf16 = 1: what the data gradient
// of the next conv writes) or fp32.  Per element 4 B (bf16 da + z) read by each of the two passes, not 8.
extern "C" int climsr_bn_backward_z(const void* da, int da_bf16, const uint16_t* z, int64_t npix, int c, const float* mean,
                                    const float* rstd, const float* gamma, const float* beta, float slope, double* workspace,
                                    float* coef, float* dgamma, float* dbeta, int accumulate, uint16_t* dz, void* stream) {
  if (!da || !z || !mean || !rstd || !gamma || !beta || !workspace || !coef || !dz || !bn_shape_ok(npix, c)) {
    set_error("bn_backward_z: bad args");
    return CLIMSR_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  const BnGrid g = bn_grid(npix, c);
  if (da_bf16)
    hipLaunchKernelGGL((bn_stats_kernel<2, uint16_t>), dim3(g.parts), dim3(256), 0, s, (int)npix, c, g.per_blk, z,
                       (const uint16_t*)da, nullptr, mean, rstd, gamma, beta, slope, workspace);
  else
    hipLaunchKernelGGL((bn_stats_kernel<2, float>), dim3(g.parts), dim3(256), 0, s, (int)npix, c, g.per_blk, z, (const float*)da,
                       nullptr, mean, rstd, gamma, beta, slope, workspace);
  hipLaunchKernelGGL(bn_bwd_finish_kernel, dim3(ceil_div(c, 8)), dim3(256), 0, s, workspace, g.parts, c, (int)npix, gamma, rstd,
                     dgamma, dbeta, accumulate, coef);
  int per;
  const int nb = bn_apply_grid(npix, c, &per);
  if (da_bf16)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<uint16_t, true>), dim3(nb), dim3(256), 0, s, (int)npix, c, per, (const uint16_t*)da,
                       nullptr, z, mean, rstd, gamma, beta, coef, slope, 1.f, dz);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<float, true>), dim3(nb), dim3(256), 0, s, (int)npix, c, per, (const float*)da, nullptr,
                       z, mean, rstd, gamma, beta, coef, slope, 1.f, dz);
  return check_launch("bn_backward_z");
}

// climsr_bn_backward_z with the statistics pass replaced by the producing data gradient's epilogue partials
// (ClimsrEpilogue.bn_z / bn_part, nparts = climsr_conv2d_fwd_bn_parts): finish + apply only.
extern "C" int climsr_bn_backward_parts(const double* parts, int64_t nparts, const uint16_t* da, const uint16_t* z, int64_t npix,
                                        int c, const float* mean, const float* rstd, const float* gamma, const float* beta,
                                        float slope, float* coef, float* dgamma, float* dbeta, int accumulate, uint16_t* dz,
                                        void* stream) {
  if (!parts || nparts <= 0 || nparts > (1L << 30) || !da || !z || !mean || !rstd || !gamma || !beta || !coef || !dz ||
      !bn_shape_ok(npix, c)) {
    set_error("bn_backward_parts: bad args (c=%d, npix=%lld, parts=%lld)", c, (long long)npix, (long long)nparts);
    return CLIMSR_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_bwd_finish_kernel, dim3(ceil_div(c, 8)), dim3(256), 0, s, parts, (int)nparts, c, (int)npix, gamma, rstd,
                     dgamma, dbeta, accumulate, coef);
  int per;
  const int nb = bn_apply_grid(npix, c, &per);
  hipLaunchKernelGGL((bn_bwd_apply_kernel<uint16_t, true>), dim3(nb), dim3(256), 0, s, (int)npix, c, per, da, nullptr, z, mean, rstd,
                     gamma, beta, coef, slope, 1.f, dz);
  return check_launch("bn_backward_parts");
}

// ---------------------------------------------------------------------------------------------
// nn.AdaptiveAvgPool2d((oh, ow)) on NHWC bf16, output flattened in torch's NCHW order
// (torch.flatten(out, 1), rfb_esrgan.py:65-66): out[n][(c*oh + i)*ow + j]; optional transposed
// copy out_t[(c*oh+i)*ow+j][n_pad] for the fc weight gradient.  Window i = [i*H/oh, ceil((i+1)*H/oh)).
// ---------------------------------------------------------------------------------------------
__global__ void adaptive_pool_fwd_kernel(const uint16_t* __restrict__ x, int n, int h, int w, int c, int oh, int ow,
                                         uint16_t* __restrict__ out, uint16_t* __restrict__ out_t, int n_pad) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;  // over n * oh * ow * c (c fastest: coalesced reads)
  long total = (long)n * oh * ow * c;
  if (idx >= total) return;
  const int ch = (int)(idx % c);
  long t = idx / c;
  const int j = (int)(t % ow);
  t /= ow;
  const int i = (int)(t % oh);
  const int b = (int)(t / oh);
  const int y0 = (i * h) / oh, y1 = ((i + 1) * h + oh - 1) / oh;
  const int x0 = (j * w) / ow, x1 = ((j + 1) * w + ow - 1) / ow;
  float s = 0.f;
  for (int yy = y0; yy < y1; ++yy)
    for (int xx = x0; xx < x1; ++xx) s += bf2f(x[(((long)b * h + yy) * w + xx) * c + ch]);
  s /= (float)((y1 - y0) * (x1 - x0));
  const long f = ((long)ch * oh + i) * ow + j;
  const uint16_t v = f2bf(s);
  out[(long)b * c * oh * ow + f] = v;
  if (out_t) out_t[f * n_pad + b] = v;
}

__global__ void adaptive_pool_bwd_kernel(const float* __restrict__ dp, int n, int h, int w, int c, int oh, int ow,
                                         float* __restrict__ dx) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;  // over n*h*w*c
  long total = (long)n * h * w * c;
  if (idx >= total) return;
  const int ch = (int)(idx % c);
  long t = idx / c;
  const int xx = (int)(t % w);
  t /= w;
  const int yy = (int)(t % h);
  const int b = (int)(t / h);
  float s = 0.f;
  // output windows containing (yy, xx): i with floor(i*h/oh) <= yy < ceil((i+1)*h/oh); the candidates
  // lie in [floor(yy*oh/h) - 1, ceil((yy+1)*oh/h)] (covers both shrinking and growing pools)
  const int ilo = max(0, (yy * oh) / h - 1), ihi = min(oh - 1, ((yy + 1) * oh + h - 1) / h);
  const int jlo = max(0, (xx * ow) / w - 1), jhi = min(ow - 1, ((xx + 1) * ow + w - 1) / w);
  for (int i = ilo; i <= ihi; ++i) {
    const int y0 = (i * h) / oh, y1 = ((i + 1) * h + oh - 1) / oh;
    if (yy < y0 || yy >= y1) continue;
    for (int j = jlo; j <= jhi; ++j) {
      const int x0 = (j * w) / ow, x1 = ((j + 1) * w + ow - 1) / ow;
      if (xx < x0 || xx >= x1) continue;
      s += dp[(long)b * c * oh * ow + ((long)ch * oh + i) * ow + j] / (float)((y1 - y0) * (x1 - x0));
    }
  }
  dx[idx] = s;
}

// Tiled forms (the discriminator's 16x16 -> 14x14 over 512 channels, 32 images): one workgroup per (image, AP_CB
// channels).  The element-per-thread kernels above gather / scatter with a 196-element stride between neighbouring
// lanes (NCHW flatten vs NHWC), 33 / 72 us per launch for 16 MB.
constexpr int AP_CB = 64;
constexpr size_t AP_LDS = 64 * 1024;

// Window tables (integer divisions once per workgroup, not per element): output row / column windows [y0, y1) /
// [x0, x1); for the backward, the (at most AP_MAXC) output rows / columns whose windows contain each input row /
// column, with the window extents.  Element loops read them with independent lookups (no per-element division
// chains: a dependent LDS lookup chain per element kept these kernels latency-bound at 4 waves per CU).
constexpr int AP_MAXD = 64, AP_MAXC = 3, AP_SPLIT = 4;
__device__ __forceinline__ void ap_win_tables(int h, int w, int oh, int ow, int* y0, int* y1, int* x0, int* x1) {
  for (int i = threadIdx.x; i < oh; i += blockDim.x) { y0[i] = (i * h) / oh; y1[i] = ((i + 1) * h + oh - 1) / oh; }
  for (int j = threadIdx.x; j < ow; j += blockDim.x) { x0[j] = (j * w) / ow; x1[j] = ((j + 1) * w + ow - 1) / ow; }
}
// cand[p][k] = k-th output index whose window [lo, hi) contains input p (or -1), ext[p][k] = hi - lo
__device__ __forceinline__ void ap_cand_tables(int in, int out, int (*cand)[AP_MAXC], int (*ext)[AP_MAXC]) {
  for (int p = threadIdx.x; p < in; p += blockDim.x) {
    int k = 0;
    const int lo = max(0, (p * out) / in - 1), hi = min(out - 1, ((p + 1) * out + in - 1) / in);
    for (int o = lo; o <= hi && k < AP_MAXC; ++o) {
      const int s0 = (o * in) / out, s1 = ((o + 1) * in + out - 1) / out;
      if (p >= s0 && p < s1) { cand[p][k] = o; ext[p][k] = s1 - s0; ++k; }
    }
    for (; k < AP_MAXC; ++k) { cand[p][k] = -1; ext[p][k] = 1; }
  }
}

// grid (c / AP_CB, n, AP_SPLIT): workgroup z computes output positions [z*no/S, (z+1)*no/S) of 64 channels
__global__ __launch_bounds__(256) void adaptive_pool_fwd_tile_kernel(const uint16_t* __restrict__ x, int h, int w, int c, int oh, int ow,
                                                                    uint16_t* __restrict__ out) {
  __shared__ uint16_t xs[AP_LDS / 2];  // [channel][h*w] bf16, channel pitch h*w + 1
  __shared__ int ty0[AP_MAXD], ty1[AP_MAXD], tx0[AP_MAXD], tx1[AP_MAXD];
  const int b = blockIdx.y, c0 = blockIdx.x * AP_CB, hw = h * w, pitch = hw + 1, no = oh * ow;
  ap_win_tables(h, w, oh, ow, ty0, ty1, tx0, tx1);
  const uint16_t* xb = x + (long)b * hw * c + c0;
  for (int i = threadIdx.x; i < hw * (AP_CB / 8); i += 256) {  // coalesced NHWC read, 16 B (8 channels) per lane
    const int px = i >> 3, cv = i & 7;
    const uint4 u = *(const uint4*)(xb + (long)px * c + cv * 8);
    const uint32_t wd[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) xs[(cv * 8 + j) * pitch + px] = (uint16_t)(wd[j >> 1] >> (16 * (j & 1)));
  }
  __syncthreads();
  const int r0 = no * blockIdx.z / AP_SPLIT, r1 = no * (blockIdx.z + 1) / AP_SPLIT, nr = r1 - r0;
  uint16_t* ob = out + (long)b * c * no + (long)c0 * no;
  for (int i = threadIdx.x; i < AP_CB * nr; i += 256) {  // (channel, position) with position fastest: contiguous runs
    const int ch = i / nr, r = r0 + i - ch * nr, oi = r / ow, oj = r - oi * ow;
    const int y0 = ty0[oi], y1 = ty1[oi], x0 = tx0[oj], x1 = tx1[oj];
    float sm = 0.f;
    for (int yy = y0; yy < y1; ++yy)
      for (int xx = x0; xx < x1; ++xx) sm += bf2f(xs[ch * pitch + yy * w + xx]);
    ob[(long)ch * no + r] = f2bf(sm / (float)((y1 - y0) * (x1 - x0)));
  }
}

// out_t[f][b] = out[b][f] for b < n, 0 for n <= b < n_pad: 64 x 64 tiles through LDS
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const uint16_t* __restrict__ in, int n, long feat, int n_pad,
                                                             uint16_t* __restrict__ out) {
  __shared__ uint16_t t[64][66];
  const long f0 = (long)blockIdx.x * 64;
  const int b0 = blockIdx.y * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int bb = i / 64, ff = i % 64;
    const long f = f0 + ff;
    t[bb][ff] = (b0 + bb < n && f < feat) ? in[(long)(b0 + bb) * feat + f] : (uint16_t)0;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int ff = i / 64, bb = i % 64;
    const long f = f0 + ff;
    if (f < feat && b0 + bb < n_pad) out[f * n_pad + b0 + bb] = t[bb][ff];
  }
}

// grid (c / AP_CB, n, AP_SPLIT): workgroup z writes input rows [z*h/S, (z+1)*h/S) of 64 channels
__global__ __launch_bounds__(256) void adaptive_pool_bwd_tile_kernel(const float* __restrict__ dp, int h, int w, int c, int oh, int ow,
                                                                    float* __restrict__ dx) {
  __shared__ float ds[AP_LDS / 4];  // [channel][oh*ow], channel pitch oh*ow + 1 (conflict-free column reads)
  __shared__ int rc[AP_MAXD][AP_MAXC], re[AP_MAXD][AP_MAXC], cc_[AP_MAXD][AP_MAXC], ce[AP_MAXD][AP_MAXC];
  const int b = blockIdx.y, c0 = blockIdx.x * AP_CB, no = oh * ow, pitch = no + 1;
  ap_cand_tables(h, oh, rc, re);
  ap_cand_tables(w, ow, cc_, ce);
  const float* db = dp + (long)b * c * no + (long)c0 * no;
  for (int i4 = threadIdx.x * 4; i4 < AP_CB * no; i4 += 1024) {  // contiguous 16 B reads of the pooled gradients
    const float4 f = *(const float4*)(db + i4);
    const float fv[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = i4 + j, ch = i / no;
      ds[ch * pitch + (i - ch * no)] = fv[j];
    }
  }
  __syncthreads();
  const int y0 = h * blockIdx.z / AP_SPLIT, y1 = h * (blockIdx.z + 1) / AP_SPLIT;
  float* xb = dx + (long)b * h * w * c + c0;
  const int cq = threadIdx.x % (AP_CB / 4);  // 4 channels per lane: one 16 B store per pixel
  for (int q = threadIdx.x / (AP_CB / 4); q < (y1 - y0) * w; q += 256 / (AP_CB / 4)) {  // (pixel, channel quad)
    const int yy = y0 + q / w, xx = q - (q / w) * w;
    float sm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < AP_MAXC; ++u) {
      const int oi = rc[yy][u];
      if (oi < 0) break;
#pragma unroll
      for (int v = 0; v < AP_MAXC; ++v) {
        const int oj = cc_[xx][v];
        if (oj < 0) break;
        const float den = (float)(re[yy][u] * ce[xx][v]);
#pragma unroll
        for (int j = 0; j < 4; ++j) sm[j] += ds[(cq * 4 + j) * pitch + oi * ow + oj] / den;
      }
    }
    *(float4*)(xb + ((long)yy * w + xx) * c + cq * 4) = make_float4(sm[0], sm[1], sm[2], sm[3]);
  }
}

extern "C" int climsr_adaptive_pool_fwd(const uint16_t* x, int n, int h, int w, int c, int oh, int ow, uint16_t* out,
                                        uint16_t* out_t, int n_pad, void* stream) {
  if (!x || !out || oh <= 0 || ow <= 0 || (out_t && n_pad < n)) {
    set_error("adaptive_pool_fwd: bad args");
    return CLIMSR_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  if (c % AP_CB == 0 && ((size_t)h * w + 1) * AP_CB * 2 <= AP_LDS && oh <= AP_MAXD && ow <= AP_MAXD) {
    // one workgroup per (image, 64 channels): NHWC tile staged once, NCHW-flattened output written contiguously;
    // the [feat][n_pad] copy by a tiled transpose (both sides coalesced)
    hipLaunchKernelGGL(adaptive_pool_fwd_tile_kernel, dim3(c / AP_CB, n, AP_SPLIT), dim3(256), 0, st, x, h, w, c, oh, ow, out);
    if (out_t) {
      const long feat = (long)c * oh * ow;
      hipLaunchKernelGGL(transpose_bf16_kernel, dim3(ceil_div(feat, 64), ceil_div(n_pad, 64)), dim3(256), 0, st, out, n, feat, n_pad,
                         out_t);
    }
    return check_launch("adaptive_pool_fwd");
  }
  long total = (long)n * oh * ow * c;
  hipLaunchKernelGGL(adaptive_pool_fwd_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, st, x, n, h, w, c, oh, ow, out, out_t, n_pad);
  return check_launch("adaptive_pool_fwd");
}

extern "C" int climsr_adaptive_pool_bwd(const float* dp, int n, int h, int w, int c, int oh, int ow, float* dx, void* stream) {
  if (!dp || !dx || oh <= 0 || ow <= 0) {
    set_error("adaptive_pool_bwd: bad args");
    return CLIMSR_EINVAL;
  }
  if (c % AP_CB == 0 && ((size_t)oh * ow + 1) * AP_CB * 4 <= AP_LDS && h <= AP_MAXD && w <= AP_MAXD && oh <= AP_MAXD &&
      ow <= AP_MAXD && oh <= 2 * h && ow <= 2 * w && h >= AP_SPLIT) {
    hipLaunchKernelGGL(adaptive_pool_bwd_tile_kernel, dim3(c / AP_CB, n, AP_SPLIT), dim3(256), 0, (hipStream_t)stream, dp, h, w, c, oh,
                       ow, dx);
    return check_launch("adaptive_pool_bwd");
  }
  long total = (long)n * h * w * c;
  hipLaunchKernelGGL(adaptive_pool_bwd_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, dp, n, h, w, c, oh,
                     ow, dx);
  return check_launch("adaptive_pool_bwd");
}

// ---------------------------------------------------------------------------------------------
// Linear layers (nn.Linear(100352, 1024), rfb_esrgan.py:57) on MFMA 16x16x32 bf16.
// forward: y[n][o] = act(sum_k x[n][k] W[o][k] + b[o]); split-K partials, then reduce.
//   A = W rows (o), B = x rows (n); both k-contiguous -> straight 16 B global loads, no LDS.
//   Workgroup = 4 waves x 16 o; each wave keeps NF = n_pad/16 accumulators.
// ---------------------------------------------------------------------------------------------
template <int NF>
__global__ __launch_bounds__(256) void linear_fwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, int n, int k,
                                                         int o, int ksplit, float* __restrict__ part) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, col = lane & 15;
  const int o0 = blockIdx.x * 64 + wave * 16;
  const int split = blockIdx.y;
  const int kb = split * ksplit, ke = min(k, kb + ksplit);
  f32x4 acc[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) acc[f] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const uint16_t* wrow = w + (long)(o0 + col) * k + g * 8;
  const bool orow_ok = o0 + col < o;
  // LU k-steps per round, every load of a round issued before its MFMAs: 16 weight rows x LU*64 B contiguous per
  // wave in flight (one k-step at a time kept a single 64 B segment per row outstanding: 2.4 TB/s)
  constexpr int LU = 8;
  int kk = kb;
  for (; kk + 32 * LU <= ke; kk += 32 * LU) {
    bf16x8 af[LU], bfr[LU][NF];
#pragma unroll
    for (int u = 0; u < LU; ++u) af[u] = orow_ok ? *(const bf16x8*)(wrow + kk + 32 * u) : (bf16x8){};
#pragma unroll
    for (int u = 0; u < LU; ++u)
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const int nn = f * 16 + col;
        bfr[u][f] = nn < n ? *(const bf16x8*)(x + (long)nn * k + kk + 32 * u + g * 8) : (bf16x8){};
      }
#pragma unroll
    for (int u = 0; u < LU; ++u)
#pragma unroll
      for (int f = 0; f < NF; ++f) acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[u], bfr[u][f], acc[f], 0, 0, 0);
  }
  for (; kk < ke; kk += 32) {
    bf16x8 af = orow_ok ? *(const bf16x8*)(wrow + kk) : (bf16x8){};
    bf16x8 bfr[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int nn = f * 16 + col;
      bfr[f] = nn < n ? *(const bf16x8*)(x + (long)nn * k + kk + g * 8) : (bf16x8){};
    }
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[f], acc[f], 0, 0, 0);
  }
  // C: row = o (4g+i), col = n
  float* dst = part + (long)split * n * o;
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const int nn = f * 16 + col;
    if (nn >= n) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int oo = o0 + g * 4 + i;
      if (oo < o) dst[(long)nn * o + oo] = acc[f][i];
    }
  }
}

// Wide-row form (o % 256 == 0): a wave owns 64 weight rows (4 A fragments), so each B fragment (the 32 x rows) read
// per k-step feeds 4 MFMAs instead of one -- the x operand (re-read by every workgroup of a K slice) was 2/3 of the
// load instructions of the form above.  Workgroup = 256 rows, grid = (o / 256) x nsplit.  Measured at fc.0 (n 32,
// k 100352, o 1024): 65 us = 3.2 TB/s of weights with 3 workgroups per CU; 8 or 16 waves per workgroup splitting K
// inside it (partials met in LDS) were slower (68-110 us), as were 1.5 or 6 workgroups per CU.  (A fragment-order copy
// of W -- 4 KB contiguous per wave and k-step -- ran 53 instead of 64 us, but the AdamW pass that writes the copy gave
// the time back: DESIGN.md 3.6; removed.)
template <int NF>
__global__ __launch_bounds__(256) void linear_fwd_wide_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, int n,
                                                              int k, int o, int ksplit, float* __restrict__ part) {
  constexpr int NA = 4, LU = 4;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, col = lane & 15;
  const int o0 = blockIdx.x * 256 + wave * 64;
  const int split = blockIdx.y;
  const int kb = split * ksplit, ke = min(k, kb + ksplit);
  f32x4 acc[NA][NF];
#pragma unroll
  for (int t = 0; t < NA; ++t)
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[t][f] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // A fragment t of k-step kk: w[(o0 + 16t + col) * k + kk + 8g]
  const uint16_t* wrow = w + (long)(o0 + col) * k + g * 8;
  auto wfrag = [&](int t, int kk) -> bf16x8 { return *(const bf16x8*)(wrow + (long)t * 16 * k + kk); };
  int kk = kb;
  for (; kk + 32 * LU <= ke; kk += 32 * LU) {
    bf16x8 af[LU][NA], bfr[LU][NF];
#pragma unroll
    for (int u = 0; u < LU; ++u)
#pragma unroll
      for (int t = 0; t < NA; ++t) af[u][t] = wfrag(t, kk + 32 * u);
#pragma unroll
    for (int u = 0; u < LU; ++u)
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const int nn = f * 16 + col;
        bfr[u][f] = nn < n ? *(const bf16x8*)(x + (long)nn * k + kk + 32 * u + g * 8) : (bf16x8){};
      }
#pragma unroll
    for (int u = 0; u < LU; ++u)
#pragma unroll
      for (int t = 0; t < NA; ++t)
#pragma unroll
        for (int f = 0; f < NF; ++f) acc[t][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[u][t], bfr[u][f], acc[t][f], 0, 0, 0);
  }
  for (; kk < ke; kk += 32) {
    bf16x8 af[NA], bfr[NF];
#pragma unroll
    for (int t = 0; t < NA; ++t) af[t] = wfrag(t, kk);
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int nn = f * 16 + col;
      bfr[f] = nn < n ? *(const bf16x8*)(x + (long)nn * k + kk + g * 8) : (bf16x8){};
    }
#pragma unroll
    for (int t = 0; t < NA; ++t)
#pragma unroll
      for (int f = 0; f < NF; ++f) acc[t][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bfr[f], acc[t][f], 0, 0, 0);
  }
  float* dst = part + (long)split * n * o;
#pragma unroll
  for (int t = 0; t < NA; ++t)
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int nn = f * 16 + col;
      if (nn >= n) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[(long)nn * o + o0 + t * 16 + g * 4 + i] = acc[t][f][i];
    }
}

__global__ void linear_reduce_kernel(const float* __restrict__ part, int nsplit, int n, int o, const float* __restrict__ bias, int act,
                                     float slope, float* __restrict__ y, uint16_t* __restrict__ ybf) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)n * o) return;
  // 8 independent partial sums (loads in flight together), combined in a fixed order: deterministic
  const long stride = (long)n * o;
  float a8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int sp = 0;
  for (; sp + 8 <= nsplit; sp += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) a8[u] += part[(long)(sp + u) * stride + idx];
  }
  for (; sp < nsplit; ++sp) a8[0] += part[(long)sp * stride + idx];
  float s = ((a8[0] + a8[1]) + (a8[2] + a8[3])) + ((a8[4] + a8[5]) + (a8[6] + a8[7]));
  if (bias) s += bias[idx % o];
  s = act_apply(s, act, slope);
  y[idx] = s;
  if (ybf) ybf[idx] = f2bf(s);
}

extern "C" int climsr_linear_fwd(const uint16_t* x, const uint16_t* w, const float* bias, int n, int k, int o, int act, float slope,
                                 float* workspace, int64_t ws_floats, float* y, void* stream) {
  const char* who = "linear_fwd";
  if (!x || !w || !y || !workspace || n <= 0 || n > 64 || k % 32 || o % 16) {
    set_error("%s: bad args (n=%d k=%d o=%d; need n<=64, k%%32==0, o%%16==0)", who, n, k, o);
    return CLIMSR_EINVAL;
  }
  const bool wide = o % 256 == 0;
  const int oblk = wide ? o / 256 : ceil_div(o, 64);
  // ~6 (narrow) / 3 (wide: 4x the rows per workgroup) workgroups per CU, K slices of whole rounds where possible
  const int rnd = wide ? 128 : 256;
  int nsplit = wide ? ceil_div(768, oblk) : ceil_div(1536, oblk);
  int ksplit = round_up(ceil_div(k, nsplit), k >= rnd * nsplit ? rnd : 32);
  nsplit = ceil_div(k, ksplit);
  if ((int64_t)nsplit * n * o > ws_floats) {
    set_error("%s: workspace too small (%lld floats needed)", who, (long long)nsplit * n * o);
    return CLIMSR_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  const int nf = (n + 15) / 16;
  dim3 grid(oblk, nsplit);
  if (wide) {
    if (nf == 1) hipLaunchKernelGGL(linear_fwd_wide_kernel<1>, grid, dim3(256), 0, s, x, w, n, k, o, ksplit, workspace);
    else if (nf == 2) hipLaunchKernelGGL(linear_fwd_wide_kernel<2>, grid, dim3(256), 0, s, x, w, n, k, o, ksplit, workspace);
    else hipLaunchKernelGGL(linear_fwd_wide_kernel<4>, grid, dim3(256), 0, s, x, w, n, k, o, ksplit, workspace);
  } else if (nf == 1) hipLaunchKernelGGL(linear_fwd_kernel<1>, grid, dim3(256), 0, s, x, w, n, k, o, ksplit, workspace);
  else if (nf == 2) hipLaunchKernelGGL(linear_fwd_kernel<2>, grid, dim3(256), 0, s, x, w, n, k, o, ksplit, workspace);
  else hipLaunchKernelGGL(linear_fwd_kernel<4>, grid, dim3(256), 0, s, x, w, n, k, o, ksplit, workspace);
  hipLaunchKernelGGL(linear_reduce_kernel, dim3(ceil_div((long)n * o, 256)), dim3(256), 0, s, workspace, nsplit, n, o, bias, act, slope,
                     y, (uint16_t*)nullptr);
  return check_launch(who);
}

// data gradient dx[n][k] = sum_o dy[n][o] W[o][k]:  A = dy rows (n, o-contiguous), B = W^T taken
// from an LDS tile of W [o][64 k] with ds_read_b64_tr_b16.  Workgroup: 64 k (one 16-col frag per
// wave) x n_pad rows, loop over o in 128-row LDS tiles.
template <int NF>
__global__ __launch_bounds__(256) void linear_dgrad_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ w, int n, int k,
                                                           int o, float* __restrict__ dx, int accumulate) {
  __shared__ __attribute__((aligned(16))) uint16_t ws_[128 * 72];  // 128 o rows x 64 k (+8 pad)
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, col = lane & 15;
  const int q = (lane & 15) >> 2, p = lane & 3;
  const int k0 = blockIdx.x * 64;
  f32x4 acc[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) acc[f] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // W[ob..ob+128][k0..k0+64] tiles: 128 rows x 8 vectors; the next tile's loads are in flight (registers) while the
  // current one is on the MFMA pipe
  uint4 buf[4];
  auto issue = [&](int ob) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int v = tid + i * 256;
      const int r = v >> 3, cv = v & 7;
      buf[i] = (ob + r < o && k0 + cv * 8 < k) ? *(const uint4*)(w + (long)(ob + r) * k + k0 + cv * 8) : make_uint4(0, 0, 0, 0);
    }
  };
  issue(0);
  for (int ob = 0; ob < o; ob += 128) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int v = tid + i * 256;
      *(uint4*)(ws_ + (v >> 3) * 72 + (v & 7) * 8) = buf[i];
    }
    if (ob + 128 < o) issue(ob + 128);
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {  // 4 k-steps of 32 o
      const int orow = ks * 32 + 8 * g + q;
      s16x4 lo = ds_read_tr16(ws_ + orow * 72 + wave * 16 + 4 * p);
      s16x4 hi = ds_read_tr16(ws_ + (orow + 4) * 72 + wave * 16 + 4 * p);
      short v8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      bf16x8 bfr = __builtin_bit_cast(bf16x8, v8);
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const int nn = f * 16 + col;
        const int oo = ob + ks * 32 + g * 8;
        bf16x8 af = (nn < n && oo < o) ? *(const bf16x8*)(dy + (long)nn * o + oo) : (bf16x8){};
        acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[f], 0, 0, 0);
      }
    }
  }
  // C: row = n (4g+i within frag f), col = k
  const int kk = k0 + wave * 16 + col;
  if (kk >= k) return;
#pragma unroll
  for (int f = 0; f < NF; ++f) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int nn = f * 16 + g * 4 + i;
      if (nn < n) {
        float* d = dx + (long)nn * k + kk;
        *d = (accumulate ? *d : 0.f) + acc[f][i];
      }
    }
  }
}

// Wide form (k % 128 == 0, the fc.0 case): a workgroup owns 128 k columns (two 16-column fragments per wave), so a W
// tile row is 256 contiguous bytes, and the dy fragments of the next 128-row o tile are loaded into registers together
// with the next W tile (the form above reads them from global memory right before each MFMA).
template <int NF>
__global__ __launch_bounds__(256) void linear_dgrad_wide_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ w, int n,
                                                                int k, int o, float* __restrict__ dx, int accumulate) {
  constexpr int WP = 128 + 8;  // LDS row pitch (bf16)
  __shared__ __attribute__((aligned(16))) uint16_t ws_[128 * WP];  // 128 o rows x 128 k
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = lane >> 4, col = lane & 15;
  const int q = (lane & 15) >> 2, p = lane & 3;
  const int k0 = blockIdx.x * 128;
  f32x4 acc[2][NF];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[b][f] = (f32x4){0.f, 0.f, 0.f, 0.f};
  uint4 buf[8];
  bf16x8 dyf[4][NF];
  // vector v (16 B) of a tile: row v / 16, k 8 (v % 16)
  auto lds_pos = [&](int v) -> int { return (v >> 4) * WP + (v & 15) * 8; };
  auto issue = [&](int ob) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int v = tid + i * 256;
      const int r = v >> 4, cv = v & 15;
      buf[i] = ob + r < o ? *(const uint4*)(w + (long)(ob + r) * k + k0 + cv * 8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const int nn = f * 16 + col, oo = ob + ks * 32 + g * 8;
        dyf[ks][f] = (nn < n && oo < o) ? *(const bf16x8*)(dy + (long)nn * o + oo) : (bf16x8){};
      }
  };
  issue(0);
  for (int ob = 0; ob < o; ob += 128) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) *(uint4*)(ws_ + lds_pos(tid + i * 256)) = buf[i];
    bf16x8 af[4][NF];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int f = 0; f < NF; ++f) af[ks][f] = dyf[ks][f];
    if (ob + 128 < o) issue(ob + 128);
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {  // 4 k-steps of 32 o
      const int orow = ks * 32 + 8 * g + q;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int c0 = wave * 32 + b * 16 + 4 * p;
        const bf16x8 bfr = cat_tr(ds_read_tr16(ws_ + orow * WP + c0), ds_read_tr16(ws_ + (orow + 4) * WP + c0));
#pragma unroll
        for (int f = 0; f < NF; ++f) acc[b][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][f], bfr, acc[b][f], 0, 0, 0);
      }
    }
  }
  // C: row = n (4g+i within frag f), col = k
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int kk = k0 + wave * 32 + b * 16 + col;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int nn = f * 16 + g * 4 + i;
        if (nn < n) {
          float* d = dx + (long)nn * k + kk;
          *d = (accumulate ? *d : 0.f) + acc[b][f][i];
        }
      }
    }
  }
}

extern "C" int climsr_linear_dgrad(const uint16_t* dy, const uint16_t* w, int n, int k, int o, float* dx, int accumulate,
                                   void* stream) {
  if (!dy || !w || !dx || n <= 0 || n > 64 || k % 64 || o % 32) {
    set_error("linear_dgrad: bad args (n=%d k=%d o=%d)", n, k, o);
    return CLIMSR_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  const int nf = (n + 15) / 16;
  if (k % 128 == 0) {
    dim3 gw(k / 128);
    if (nf == 1) hipLaunchKernelGGL(linear_dgrad_wide_kernel<1>, gw, dim3(256), 0, s, dy, w, n, k, o, dx, accumulate);
    else if (nf == 2) hipLaunchKernelGGL(linear_dgrad_wide_kernel<2>, gw, dim3(256), 0, s, dy, w, n, k, o, dx, accumulate);
    else hipLaunchKernelGGL(linear_dgrad_wide_kernel<4>, gw, dim3(256), 0, s, dy, w, n, k, o, dx, accumulate);
    return check_launch("linear_dgrad");
  }
  dim3 grid(k / 64);
  if (nf == 1) hipLaunchKernelGGL(linear_dgrad_kernel<1>, grid, dim3(256), 0, s, dy, w, n, k, o, dx, accumulate);
  else if (nf == 2) hipLaunchKernelGGL(linear_dgrad_kernel<2>, grid, dim3(256), 0, s, dy, w, n, k, o, dx, accumulate);
  else hipLaunchKernelGGL(linear_dgrad_kernel<4>, grid, dim3(256), 0, s, dy, w, n, k, o, dx, accumulate);
  return check_launch("linear_dgrad");
}

// weight gradient dW[o][k] (+)= sum_n dy[n][o] x[n][k] with K = n_pad (multiple of 32):
// A = dy^T [o][n_pad], B = x^T [k][n_pad] (both n-contiguous).  Each wave: 16 o x 64 k.
// Optional second pair (dyt2, xt2, n_pad2): the same sum continued over a second batch, so two backward passes through
// the layer (the discriminator's real and fake calls, pl_gan.py:51-61) write dW once instead of a write plus a
// read-modify-write of the 411 MB fp32 gradient.
__global__ __launch_bounds__(256) void linear_wgrad_kernel(const uint16_t* __restrict__ dyt, const uint16_t* __restrict__ xt, int n_pad,
                                                           const uint16_t* __restrict__ dyt2, const uint16_t* __restrict__ xt2,
                                                           int n_pad2, int k, int o, float* __restrict__ dw, int accumulate) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, col = lane & 15;
  const int o0 = blockIdx.y * 64 + wave * 16;
  const int k0 = blockIdx.x * 64;
  // one accumulator set per batch, added in the order two separate launches would: (old + a) + b, bit-identical to
  // them and to torch DDP's AccumulateGrad sum of the two calls' gradients
  f32x4 acc[2][4];
#pragma unroll
  for (int sidx = 0; sidx < 2; ++sidx)
#pragma unroll
    for (int f = 0; f < 4; ++f) acc[sidx][f] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // A = x^T rows (k), B = dy^T columns (o): C[row = k (4g+i)][col = o], so a lane holds 4 consecutive k of one dW row
  // and stores (and, accumulating, loads) them as one 16 B vector (the dy-as-A form wrote 4 B per lane, k floats apart)
  auto run = [&](const uint16_t* dy_, const uint16_t* x_, int np, f32x4* ac) {
    for (int nb = 0; nb < np; nb += 32) {
      const bf16x8 bo = *(const bf16x8*)(dy_ + (long)(o0 + col) * np + nb + g * 8);
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const bf16x8 ak = *(const bf16x8*)(x_ + (long)(k0 + f * 16 + col) * np + nb + g * 8);
        ac[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ak, bo, ac[f], 0, 0, 0);
      }
    }
  };
  run(dyt, xt, n_pad, acc[0]);
  if (dyt2) run(dyt2, xt2, n_pad2, acc[1]);
  float* row = dw + (long)(o0 + col) * k + k0 + g * 4;
  float4 old[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) old[f] = accumulate ? *(const float4*)(row + f * 16) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    float4 r = make_float4(old[f].x + acc[0][f][0], old[f].y + acc[0][f][1], old[f].z + acc[0][f][2], old[f].w + acc[0][f][3]);
    if (dyt2) r = make_float4(r.x + acc[1][f][0], r.y + acc[1][f][1], r.z + acc[1][f][2], r.w + acc[1][f][3]);
    *(float4*)(row + f * 16) = r;
  }
}

extern "C" int climsr_linear_wgrad(const uint16_t* dy_t, const uint16_t* x_t, int n_pad, int k, int o, float* dw, int accumulate,
                                   void* stream) {
  if (!dy_t || !x_t || !dw || n_pad % 32 || k % 64 || o % 64) {
    set_error("linear_wgrad: bad args (n_pad=%d k=%d o=%d)", n_pad, k, o);
    return CLIMSR_EINVAL;
  }
  hipLaunchKernelGGL(linear_wgrad_kernel, dim3(k / 64, o / 64), dim3(256), 0, (hipStream_t)stream, dy_t, x_t, n_pad,
                     (const uint16_t*)nullptr, (const uint16_t*)nullptr, 0, k, o, dw, accumulate);
  return check_launch("linear_wgrad");
}

extern "C" int climsr_linear_wgrad2(const uint16_t* dy_t, const uint16_t* x_t, int n_pad, const uint16_t* dy_t2, const uint16_t* x_t2,
                                    int n_pad2, int k, int o, float* dw, int accumulate, void* stream) {
  if (!dy_t || !x_t || !dy_t2 || !x_t2 || !dw || n_pad % 32 || n_pad2 % 32 || k % 64 || o % 64) {
    set_error("linear_wgrad2: bad args (n_pad=%d n_pad2=%d k=%d o=%d)", n_pad, n_pad2, k, o);
    return CLIMSR_EINVAL;
  }
  hipLaunchKernelGGL(linear_wgrad_kernel, dim3(k / 64, o / 64), dim3(256), 0, (hipStream_t)stream, dy_t, x_t, n_pad, dy_t2, x_t2,
                     n_pad2, k, o, dw, accumulate);
  return check_launch("linear_wgrad2");
}

// ---------------------------------------------------------------------------------------------
// Discriminator head after fc.0 + LeakyReLU: s = sigmoid(h . w2 + b2) (rfb_esrgan.py:59-60), and its
// backward: du = ds*s*(1-s); dw2 += sum_n du h; db2 += sum du; du0 = du*w2*lrelu'(h);
// db0 += sum_n du0; du0 written as bf16 [n][o] and transposed [o][n_pad] for the fc.0 grads.
// One workgroup, n <= 64, fixed reduction order.
// ---------------------------------------------------------------------------------------------
// one workgroup per image (blockIdx.x = b), fixed-order tree reduction
__global__ __launch_bounds__(256) void d_head_fwd_kernel(const float* __restrict__ h, const float* __restrict__ w2,
                                                         const float* __restrict__ b2, int n, int o, int sigmoid, float* __restrict__ s) {
  __shared__ float red[256];
  const int b = blockIdx.x;
  float t = 0.f;
  for (int j = threadIdx.x; j < o; j += 256) t += h[(long)b * o + j] * w2[j];
  red[threadIdx.x] = t;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float u = red[0] + b2[0];
    s[b] = sigmoid ? 1.f / (1.f + expf(-u)) : u;
  }
}

__global__ __launch_bounds__(256) void d_head_bwd_kernel(const float* __restrict__ h, const float* __restrict__ s, const float* __restrict__ ds,
                                                         const float* __restrict__ w2, int n, int o, int n_pad, float slope, int sigmoid,
                                                         float* dw2, float* db2, float* db0, int accumulate, uint16_t* __restrict__ du0,
                                                         uint16_t* __restrict__ du0_t) {
  const int j = blockIdx.x * 256 + threadIdx.x;  // one hidden unit per thread over the grid
  if (j < o) {
    float a_w2 = 0.f, a_b0 = 0.f;
    uint4* trow = (uint4*)(du0_t + (long)j * n_pad);  // n_pad % 32 == 0: whole 16 B vectors per row
    for (int b8 = 0; b8 < n_pad; b8 += 8) {
      uint32_t pk[4];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int b = b8 + q;
        float v = 0.f;
        if (b < n) {
          const float du = sigmoid ? ds[b] * s[b] * (1.f - s[b]) : ds[b];
          const float hv = h[(long)b * o + j];
          a_w2 += du * hv;
          v = du * w2[j] * (hv > 0.f ? 1.f : slope);
          a_b0 += v;
          du0[(long)b * o + j] = f2bf(v);
        }
        if (q & 1) pk[q >> 1] |= (uint32_t)f2bf(v) << 16;
        else pk[q >> 1] = f2bf(v);
      }
      trow[b8 / 8] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    }
    if (dw2) dw2[j] = (accumulate ? dw2[j] : 0.f) + a_w2;
    if (db0) db0[j] = (accumulate ? db0[j] : 0.f) + a_b0;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && db2) {
    float t = 0.f;
    for (int b = 0; b < n; ++b) t += sigmoid ? ds[b] * s[b] * (1.f - s[b]) : ds[b];
    db2[0] = (accumulate ? db2[0] : 0.f) + t;
  }
}

extern "C" int climsr_d_head_fwd(const float* h, const float* w2, const float* b2, int n, int o, int sigmoid, float* s,
                                 void* stream) {
  if (!h || !w2 || !b2 || !s || n <= 0) {
    set_error("d_head_fwd: bad args");
    return CLIMSR_EINVAL;
  }
  hipLaunchKernelGGL(d_head_fwd_kernel, dim3(n), dim3(256), 0, (hipStream_t)stream, h, w2, b2, n, o, sigmoid, s);
  return check_launch("d_head_fwd");
}

extern "C" int climsr_d_head_bwd(const float* h, const float* s, const float* ds, const float* w2, int n, int o, int n_pad, float slope,
                                 int sigmoid, float* dw2, float* db2, float* db0, int accumulate, uint16_t* du0, uint16_t* du0_t,
                                 void* stream) {
  if (!h || !s || !ds || !w2 || !du0 || !du0_t || n_pad < n || n_pad % 32) {
    set_error("d_head_bwd: bad args");
    return CLIMSR_EINVAL;
  }
  hipLaunchKernelGGL(d_head_bwd_kernel, dim3(ceil_div(o, 256)), dim3(256), 0, (hipStream_t)stream, h, s, ds, w2, n, o, n_pad, slope, sigmoid,
                     dw2, db2, db0, accumulate, du0, du0_t);
  return check_launch("d_head_bwd");
}

// ---------------------------------------------------------------------------------------------
// Relativistic-average BCE-with-logits on the (sigmoid) scores (pl_gan.py:31-38 and :52-59):
//   rf = s_r - mean(s_f), fr = s_f - mean(s_r)
//   L = ( BCEwl(fr, t_fr) + BCEwl(rf, t_rf) ) / 2
// loss_g: t_fr = 1, t_rf = 0;  loss_d: t_fr = 0, t_rf = 1.  With gscale != NULL also writes
// g_r = gscale * dL/ds_r and g_f = gscale * dL/ds_f.  One workgroup, n <= 1024.
// ---------------------------------------------------------------------------------------------
__device__ inline double bcewl(double x, double t) { return fmax(x, 0.0) - x * t + log1p(exp(-fabs(x))); }

__global__ void rel_bce_kernel(const float* __restrict__ sr, const float* __restrict__ sf, int n, float t_rf, float t_fr,
                               float* __restrict__ loss, const float* __restrict__ gscale, float* __restrict__ gr,
                               float* __restrict__ gf) {
  // one wave; lane l owns samples l, l+64, ... (summed in that order), then a fixed butterfly: deterministic
  const int l = threadIdx.x;
  auto wsum = [](double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
    return v;
  };
  double pr = 0.0, pf = 0.0;
  for (int i = l; i < n; i += 64) { pr += sr[i]; pf += sf[i]; }
  const double mr = wsum(pr) / n, mf = wsum(pf) / n;
  double l_rf = 0.0, l_fr = 0.0, s_drf = 0.0, s_dfr = 0.0;
  for (int i = l; i < n; i += 64) {
    const double rf = sr[i] - mf, fr = sf[i] - mr;
    l_rf += bcewl(rf, t_rf);
    l_fr += bcewl(fr, t_fr);
    s_drf += 0.5 / n * (1.0 / (1.0 + exp(-rf)) - t_rf);
    s_dfr += 0.5 / n * (1.0 / (1.0 + exp(-fr)) - t_fr);
  }
  l_rf = wsum(l_rf);
  l_fr = wsum(l_fr);
  const double sum_drf = wsum(s_drf), sum_dfr = wsum(s_dfr);
  if (loss && l == 0) loss[0] = (float)((l_rf / n + l_fr / n) / 2.0);
  if (gscale) {
    const double gs = gscale[0];
    for (int i = l; i < n; i += 64) {
      const double rf = sr[i] - mf, fr = sf[i] - mr;
      const double drf = 0.5 / n * (1.0 / (1.0 + exp(-rf)) - t_rf);
      const double dfr = 0.5 / n * (1.0 / (1.0 + exp(-fr)) - t_fr);
      gr[i] = (float)(gs * (drf - sum_dfr / n));
      gf[i] = (float)(gs * (dfr - sum_drf / n));
    }
  }
}

extern "C" int climsr_relativistic_bce(const float* s_real, const float* s_fake, int n, float t_rf, float t_fr, float* loss,
                                       const float* gscale, float* g_real, float* g_fake, void* stream) {
  if (!s_real || !s_fake || n <= 0 || (gscale && (!g_real || !g_fake))) {
    set_error("relativistic_bce: bad args");
    return CLIMSR_EINVAL;
  }
  hipLaunchKernelGGL(rel_bce_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, s_real, s_fake, n, t_rf, t_fr, loss, gscale, g_real,
                     g_fake);
  return check_launch("relativistic_bce");
}

// ---------------------------------------------------------------------------------------------
// VGG19 helpers (perceptual.py): MaxPool2d(2,2) on NHWC bf16, L1 mean between two bf16 tensors.
// ---------------------------------------------------------------------------------------------
__global__ void maxpool2_kernel(const uint16_t* __restrict__ x, int n, int h, int w, int c, uint16_t* __restrict__ y) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int oh = h / 2, ow = w / 2, groups = c / 8;
  long total = (long)n * oh * ow * groups;
  if (idx >= total) return;
  const int cg = (int)(idx % groups);
  long t = idx / groups;
  const int j = (int)(t % ow);
  t /= ow;
  const int i = (int)(t % oh);
  const int b = (int)(t / oh);
  float m[8], f[8];
  unpack8(*(const uint4*)(x + (((long)b * h + 2 * i) * w + 2 * j) * c + cg * 8), m);
  const int dy[3] = {0, 1, 1}, dx[3] = {1, 0, 1};
  for (int r = 0; r < 3; ++r) {
    unpack8(*(const uint4*)(x + (((long)b * h + 2 * i + dy[r]) * w + 2 * j + dx[r]) * c + cg * 8), f);
#pragma unroll
    for (int q = 0; q < 8; ++q) m[q] = fmaxf(m[q], f[q]);
  }
  *(uint4*)(y + (((long)b * oh + i) * ow + j) * c + cg * 8) = pack8(m);
}

extern "C" int climsr_maxpool2_bf16(const uint16_t* x, int n, int h, int w, int c, uint16_t* y, void* stream) {
  if (!x || !y || c % 8 || h % 2 || w % 2) {
    set_error("maxpool2_bf16: bad args");
    return CLIMSR_EINVAL;
  }
  long total = (long)n * (h / 2) * (w / 2) * (c / 8);
  hipLaunchKernelGGL(maxpool2_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, x, n, h, w, c, y);
  return check_launch("maxpool2_bf16");
}

__global__ void l1_bf16_partial_kernel(const uint16_t* __restrict__ a, const uint16_t* __restrict__ b, long n8, double* ws) {
  __shared__ double sh[256];
  double s = 0.0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float fa[8], fb[8];
    unpack8(((const uint4*)a)[i], fa);
    unpack8(((const uint4*)b)[i], fb);
#pragma unroll
    for (int q = 0; q < 8; ++q) s += fabsf(fa[q] - fb[q]);
  }
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) sh[threadIdx.x] += sh[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) ws[blockIdx.x] = sh[0];
}

// one wave: lane l sums ws[l], ws[l + 64], .. in order, then a fixed xor tree (deterministic; a single thread summing
// the 512 partials serially took 31 us)
__global__ void l1_bf16_final_kernel(const double* ws, int nb, long n, float* out) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += 64) s += ws[i];
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) s += __shfl_xor(s, m);
  if (threadIdx.x == 0) out[0] = (float)(s / (double)n);
}

extern "C" int climsr_l1_loss_bf16(const uint16_t* a, const uint16_t* b, int64_t n, double* workspace, float* out, void* stream) {
  if (!a || !b || !workspace || !out || n <= 0 || n % 8) {
    set_error("l1_loss_bf16: bad args");
    return CLIMSR_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(l1_bf16_partial_kernel, dim3(512), dim3(256), 0, s, a, b, (long)(n / 8), workspace);
  hipLaunchKernelGGL(l1_bf16_final_kernel, dim3(1), dim3(64), 0, s, workspace, 512, (long)n, out);
  return check_launch("l1_loss_bf16");
}

// bf16 copy of an fp32 matrix (the fc.0 weight's MFMA copy), vectorised
__global__ void f32_to_bf16_kernel(const float* __restrict__ x, long n, uint16_t* __restrict__ y) {
  long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i + 7 < n) {
    float4 a = *(const float4*)(x + i), b = *(const float4*)(x + i + 4);
    float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    *(uint4*)(y + i) = pack8(f);
  } else {
    for (long j = i; j < n; ++j) y[j] = f2bf(x[j]);
  }
}

__global__ void inc_i64_kernel(int64_t* p) {
  if (threadIdx.x == 0) p[0] += 1;
}

extern "C" int climsr_increment_i64(int64_t* p, void* stream) {
  if (!p) {
    set_error("increment_i64: null");
    return CLIMSR_EINVAL;
  }
  hipLaunchKernelGGL(inc_i64_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, p);
  return check_launch("increment_i64");
}

extern "C" int climsr_f32_to_bf16(const float* x, int64_t n, uint16_t* y, void* stream) {
  if (!x || !y || n < 0) {
    set_error("f32_to_bf16: bad args");
    return CLIMSR_EINVAL;
  }
  long threads = (n + 7) / 8;
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(ceil_div(threads > 0 ? threads : 1, 256)), dim3(256), 0, (hipStream_t)stream, x, (long)n, y);
  return check_launch("f32_to_bf16");
}

// ---------------------------------------------------------------------------------------------
// nn.ReflectionPad2d(1) (discriminator.py:15,21) on NHWC bf16 and its backward (fp32 fold): padded
// row -1 mirrors row 1, row h mirrors row h-2 (same for columns).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int refl1(int i, int n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); }

__global__ void reflect_pad1_kernel(const uint16_t* __restrict__ x, int n, int h, int w, int cs, uint16_t* __restrict__ y) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;  // over n*(h+2)*(w+2)*(cs/8)
  const int groups = cs / 8;
  const long total = (long)n * (h + 2) * (w + 2) * groups;
  if (idx >= total) return;
  const int cg = (int)(idx % groups);
  long t = idx / groups;
  const int px = (int)(t % (w + 2));
  t /= (w + 2);
  const int py = (int)(t % (h + 2));
  const int b = (int)(t / (h + 2));
  const int sy = refl1(py - 1, h), sx = refl1(px - 1, w);
  *(uint4*)(y + idx * 8) = *(const uint4*)(x + (((long)b * h + sy) * w + sx) * cs + cg * 8);
}

__global__ void reflect_pad1_bwd_kernel(const float* __restrict__ gp, int n, int h, int w, int c, float* __restrict__ g) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;  // over n*h*w*c
  const long total = (long)n * h * w * c;
  if (idx >= total) return;
  const int ch = (int)(idx % c);
  long t = idx / c;
  const int x = (int)(t % w);
  t /= w;
  const int y = (int)(t % h);
  const int b = (int)(t / h);
  // padded rows / columns that read (y, x): p = y+1, plus the mirror p = 0 (y == 1) and p = h+1 (y == h-2)
  int rows[3], cols[3], nr = 0, nc = 0;
  rows[nr++] = y + 1;
  if (y == 1) rows[nr++] = 0;
  if (y == h - 2) rows[nr++] = h + 1;
  cols[nc++] = x + 1;
  if (x == 1) cols[nc++] = 0;
  if (x == w - 2) cols[nc++] = w + 1;
  float s = 0.f;
  for (int i = 0; i < nr; ++i)
    for (int j = 0; j < nc; ++j) s += gp[(((long)b * (h + 2) + rows[i]) * (w + 2) + cols[j]) * c + ch];
  g[idx] = s;
}

extern "C" int climsr_reflect_pad1_bf16(const uint16_t* x, int n, int h, int w, int cstride, uint16_t* y, void* stream) {
  if (!x || !y || n <= 0 || h < 2 || w < 2 || cstride % 8) {
    set_error("reflect_pad1_bf16: bad args");
    return CLIMSR_EINVAL;
  }
  const long total = (long)n * (h + 2) * (w + 2) * (cstride / 8);
  hipLaunchKernelGGL(reflect_pad1_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, x, n, h, w, cstride, y);
  return check_launch("reflect_pad1_bf16");
}

extern "C" int climsr_reflect_pad1_bwd_f32(const float* gp, int n, int h, int w, int c, float* g, void* stream) {
  if (!gp || !g || n <= 0 || h < 3 || w < 3 || c <= 0) {
    set_error("reflect_pad1_bwd_f32: bad args");
    return CLIMSR_EINVAL;
  }
  const long total = (long)n * h * w * c;
  hipLaunchKernelGGL(reflect_pad1_bwd_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, gp, n, h, w, c, g);
  return check_launch("reflect_pad1_bwd_f32");
}
