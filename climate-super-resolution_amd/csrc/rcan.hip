// RCAN pieces that are not convolutions (climsr/models/rcan.py):
//  * channel attention of an RCAB (CALayer, rcan.py:50-69): global average pool -> 1x1 conv -> ReLU ->
//    1x1 conv -> sigmoid -> x * y, and the block residual (RCAB.forward, rcan.py:104-107) fused with the
//    scaling into one pass that also emits the bf16 copy the next conv reads;
//  * nn.PixelShuffle(r) of the Upsampler (rcan.py:17-47) on NHWC bf16: a pure index map, bit-exact.
// All HBM-bound elementwise / reduction work: 16 B per lane where the layout allows, deterministic
// fixed-order reductions.
#include "common.h"

using namespace climsr;

namespace {
constexpr int POOL_SPLIT = 256;  // pixel slices per image of the pooling pass (>= 1 block per CU for one grid)
constexpr int TILE_DIRECT = 1024;  // at most this many fp32 rows per image (64 channels): ca_mlp_kernel reads them itself
constexpr int TILE_SPLIT = 256;  // slices per image of the per-tile sums (channel_attention_parts; 64 measured neutral)
}

// part[n][split][c] = sum over the split's pixels of x[n][p][c] (fp32 NHWC, cstride).  A block is
// (c/4 float4 lanes) x (256 / (c/4) pixel lanes); fp32 per-thread sums, fp64 across the block.
__global__ __launch_bounds__(256) void channel_sum_partial_kernel(const float* __restrict__ x, long hw, int c, int cs,
                                                                  double* __restrict__ part) {
  const int nimg = blockIdx.y, sp = blockIdx.x;
  const long p0 = hw * sp / POOL_SPLIT, p1 = hw * (sp + 1) / POOL_SPLIT;
  __shared__ double sh[256 * 4];
  const int cg = c / 4;  // host guarantees c % 4 == 0, cs % 4 == 0, cg <= 256
  const int plan = 256 / cg;
  const int g = threadIdx.x % cg, pl = threadIdx.x / cg;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (pl < plan)
    for (long p = p0 + pl; p < p1; p += plan) {
      const float4 v = *(const float4*)(x + ((long)nimg * hw + p) * cs + g * 4);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  sh[threadIdx.x * 4 + 0] = acc.x;
  sh[threadIdx.x * 4 + 1] = acc.y;
  sh[threadIdx.x * 4 + 2] = acc.z;
  sh[threadIdx.x * 4 + 3] = acc.w;
  __syncthreads();
  for (int ch = threadIdx.x; ch < c; ch += 256) {
    const int gg = ch / 4, q = ch % 4;
    double t = 0.0;
    for (int k = 0; k < plan; ++k) t += sh[(k * cg + gg) * 4 + q];
    part[((long)nimg * POOL_SPLIT + sp) * c + ch] = t;
  }
}

// s[n][c] = sigmoid(W2 relu(W1 mean + b1) + b2)  (conv_du of CALayer on the pooled [n, c, 1, 1] map)
// The slice sums of a slice group are loaded 4 at a time (independent fp64 chains, combined in a fixed order); W1 / W2
// are staged in LDS by every thread at once when they fit; a hidden unit is one wave's strided dot product finished
// by a fixed xor-shuffle tree (the serial per-thread loops over global W1 / W2 took most of this kernel's 8.9 us).
constexpr int CA_STAGE_MAX = 8192;  // floats of W1 + W2 staged in LDS
// P: the slice sums' type -- fp64 slices of the fold kernels, or fp32 rows straight from the conv epilogue (c == 64: a
// thread's float4 loads are all in flight at once, 16 channel quads x 64 row lanes; a wave's 4 row lanes are combined by
// a fixed xor-shuffle tree, the 16 waves in order)
template <typename P>
__global__ __launch_bounds__(1024) void ca_mlp_kernel(const P* __restrict__ part, int nsl, long hw, int c, int cr, const float* __restrict__ w1,
                              const float* __restrict__ b1, const float* __restrict__ w2, const float* __restrict__ b2,
                              float* __restrict__ s, float* __restrict__ mean_out) {
  extern __shared__ float sm[];
  float* mean = sm;      // [c]
  float* hid = sm + c;   // [cr]
  __shared__ float wst[CA_STAGE_MAX];
  constexpr int NT = 1024;
  __shared__ double grp[NT];
  const int nimg = blockIdx.x, t = threadIdx.x;
  const bool staged = 2 * cr * c <= CA_STAGE_MAX;
  if (staged)
    for (int i = t; i < cr * c; i += NT) {
      wst[i] = w1[i];
      wst[cr * c + i] = w2[i];
    }
  const float* W1 = staged ? wst : w1;
  const float* W2 = staged ? wst + cr * c : w2;
  const int cw = c < NT ? c : NT;  // channels per round
  const int G = NT / cw;           // split groups summed in parallel, then combined in a fixed order
  if constexpr (sizeof(P) == 4) {
    const int q = t & 15, rl = t >> 4;  // channel quad, row lane (0..63)
    const float4* pp = (const float4*)(part + (long)nimg * nsl * 64) + q;
    double a[8][4] = {};
    int r = rl;
    for (; r + 7 * 64 < nsl; r += 8 * 64) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = pp[(long)(r + u * 64) * 16];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a[u][0] += v[u].x; a[u][1] += v[u].y; a[u][2] += v[u].z; a[u][3] += v[u].w;
      }
    }
#pragma unroll
    for (int u = 0; u < 7; ++u)
      if (r + u * 64 < nsl) {
        const float4 v = pp[(long)(r + u * 64) * 16];
        a[u][0] += v.x; a[u][1] += v.y; a[u][2] += v.z; a[u][3] += v.w;
      }
    double m4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      double v = ((a[0][k] + a[1][k]) + (a[2][k] + a[3][k])) + ((a[4][k] + a[5][k]) + (a[6][k] + a[7][k]));
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      m4[k] = v;
    }
    const int wave = t >> 6, lane = t & 63;
    if (lane < 16)
#pragma unroll
      for (int k = 0; k < 4; ++k) grp[wave * 64 + q * 4 + k] = m4[k];
    __syncthreads();
    if (t < 64) {
      double m = 0.0;
      for (int w = 0; w < NT / 64; ++w) m += grp[w * 64 + t];
      mean[t] = (float)(m / (double)hw);
      if (mean_out) mean_out[(long)nimg * 64 + t] = mean[t];
    }
    __syncthreads();
  } else
  for (int c0 = 0; c0 < c; c0 += cw) {
    const int i = c0 + t % cw, gi = t / cw;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    if (i < c && gi < G) {
      const P* pp = part + (long)nimg * nsl * c + i;
      int sp = gi;
      for (; sp + 3 * G < nsl; sp += 4 * G) {
        a0 += (double)pp[(long)sp * c];
        a1 += (double)pp[(long)(sp + G) * c];
        a2 += (double)pp[(long)(sp + 2 * G) * c];
        a3 += (double)pp[(long)(sp + 3 * G) * c];
      }
      for (; sp < nsl; sp += G) a0 += (double)pp[(long)sp * c];
    }
    grp[t] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (t < cw && c0 + t < c) {
      double m = 0.0;
      for (int k = 0; k < G; ++k) m += grp[k * cw + t];
      mean[c0 + t] = (float)(m / (double)hw);
      if (mean_out) mean_out[(long)nimg * c + c0 + t] = mean[c0 + t];  // kept for the backward (climsr_ca_backward)
    }
    __syncthreads();
  }
  const int wave = t >> 6, lane = t & 63;
  for (int j = wave; j < cr; j += NT / 64) {
    float v = 0.f;
    for (int i = lane; i < c; i += 64) v += W1[j * c + i] * mean[i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) {
      v += b1 ? b1[j] : 0.f;
      hid[j] = v > 0.f ? v : 0.f;
    }
  }
  __syncthreads();
  for (int i = t; i < c; i += NT) {
    float v = b2 ? b2[i] : 0.f;
    for (int j = 0; j < cr; ++j) v += W2[i * cr + j] * hid[j];
    s[nimg * c + i] = 1.f / (1.f + expf(-v));
  }
}

extern "C" int climsr_channel_attention_mean(const float* u, int n, int64_t hw, int c, int u_cstride, const float* w1, const float* b1,
                                             const float* w2, const float* b2, int cr, double* workspace, float* s, float* mean_out,
                                             void* stream) {
  if (!u || !w1 || !w2 || !workspace || !s || n <= 0 || hw <= 0 || c <= 0 || cr <= 0 || u_cstride < c || c % 4 || u_cstride % 4 ||
      c > 1024) {
    set_error("channel_attention: bad args (c, u_cstride multiples of 4, c <= 1024)");
    return CLIMSR_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(channel_sum_partial_kernel, dim3(POOL_SPLIT, n), dim3(256), 0, st, u, (long)hw, c, u_cstride, workspace);
  hipLaunchKernelGGL(ca_mlp_kernel<double>, dim3(n), dim3(1024), (size_t)(c + cr) * sizeof(float), st, workspace, POOL_SPLIT, (long)hw, c, cr, w1, b1,
                     w2, b2, s, mean_out);
  return check_launch("channel_attention");
}

extern "C" int climsr_channel_attention(const float* u, int n, int64_t hw, int c, int u_cstride, const float* w1, const float* b1,
                                        const float* w2, const float* b2, int cr, double* workspace, float* s, void* stream) {
  return climsr_channel_attention_mean(u, n, hw, c, u_cstride, w1, b1, w2, b2, cr, workspace, s, nullptr, stream);
}

extern "C" size_t climsr_channel_attention_workspace(int n, int c) { return (size_t)n * POOL_SPLIT * c * sizeof(double); }

// channel_attention from per-tile channel sums: the image's tile rows folded into TILE_SPLIT fp64 slices (slice sp =
// tiles [tpi sp / TILE_SPLIT, tpi (sp + 1) / TILE_SPLIT), summed in order), then ca_mlp_kernel over the slices -- the
// same fixed order every run.  One workgroup per (slice, image): 256 threads = 4 tile lanes x 64 channels per round.
__global__ __launch_bounds__(256) void tile_parts_fold_kernel(const float* __restrict__ part, int tpi, int c, double* __restrict__ out) {
  const int nimg = blockIdx.y, sp = blockIdx.x;
  const long t0 = (long)tpi * sp / TILE_SPLIT, t1 = (long)tpi * (sp + 1) / TILE_SPLIT;
  __shared__ double sh[256];
  for (int c0 = 0; c0 < c; c0 += 64) {
    const int ch = c0 + (threadIdx.x & 63), tl = threadIdx.x >> 6;
    double t = 0.0;
    if (ch < c)
      for (long k = t0 + tl; k < t1; k += 4) t += (double)part[((long)nimg * tpi + k) * c + ch];
    sh[threadIdx.x] = t;
    __syncthreads();
    if (threadIdx.x < 64 && ch < c)
      out[((long)nimg * TILE_SPLIT + sp) * c + ch] = ((sh[threadIdx.x] + sh[64 + threadIdx.x]) + sh[128 + threadIdx.x]) + sh[192 + threadIdx.x];
    __syncthreads();
  }
}

extern "C" int climsr_channel_attention_parts_mean(const float* part, int n, int tiles_per_image, int64_t hw, int c, const float* w1,
                                                   const float* b1, const float* w2, const float* b2, int cr, double* workspace, float* s,
                                                   float* mean_out, void* stream) {
  if (!part || !w1 || !w2 || !s || !workspace || n <= 0 || tiles_per_image <= 0 || hw <= 0 || c <= 0 || c > 1024 || cr <= 0) {
    set_error("channel_attention_parts: bad args");
    return CLIMSR_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  if (tiles_per_image <= TILE_DIRECT && c == 64) {  // few rows (one per conv workgroup, or small images): the MLP folds them
    hipLaunchKernelGGL(ca_mlp_kernel<float>, dim3(n), dim3(1024), (size_t)(c + cr) * sizeof(float), st, part, tiles_per_image, (long)hw, c,
                       cr, w1, b1, w2, b2, s, mean_out);
    return check_launch("channel_attention_parts");
  }
  hipLaunchKernelGGL(tile_parts_fold_kernel, dim3(TILE_SPLIT, n), dim3(256), 0, st, part, tiles_per_image, c, workspace);
  hipLaunchKernelGGL(ca_mlp_kernel<double>, dim3(n), dim3(1024), (size_t)(c + cr) * sizeof(float), st, workspace, TILE_SPLIT, (long)hw, c, cr, w1, b1,
                     w2, b2, s, mean_out);
  return check_launch("channel_attention_parts");
}

extern "C" int climsr_channel_attention_parts(const float* part, int n, int tiles_per_image, int64_t hw, int c, const float* w1,
                                              const float* b1, const float* w2, const float* b2, int cr, double* workspace, float* s,
                                              void* stream) {
  return climsr_channel_attention_parts_mean(part, n, tiles_per_image, hw, c, w1, b1, w2, b2, cr, workspace, s, nullptr, stream);
}

// xres[p][c] = u[p][c] * s[n][c] + xres[p][c];  xb[p][c] = bf16(xres[p][c])   (RCAB: body(x) + x); u fp32 or bf16
template <bool UB>
__global__ __launch_bounds__(256) void ca_scale_add_kernel(const void* __restrict__ u, int u_cs, const float* __restrict__ s,
                                                           float* __restrict__ xres, uint16_t* __restrict__ xb, int xb_cs, long hw,
                                                           int c, long total4) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total4) return;
  const int cg = c / 4;
  const long pix = i / cg;
  const int c0 = (int)(i % cg) * 4;
  const int nimg = (int)(pix / hw);
  float4 uv;
  if constexpr (UB) {
    const uint2 raw = *(const uint2*)((const uint16_t*)u + pix * u_cs + c0);
    uv = make_float4(__uint_as_float(raw.x << 16), __uint_as_float(raw.x & 0xFFFF0000u), __uint_as_float(raw.y << 16),
                     __uint_as_float(raw.y & 0xFFFF0000u));
  } else {
    uv = *(const float4*)((const float*)u + pix * u_cs + c0);
  }
  const float4 sv = *(const float4*)(s + (long)nimg * c + c0);
  float4 r = *(const float4*)(xres + pix * c + c0);
  r.x = uv.x * sv.x + r.x;
  r.y = uv.y * sv.y + r.y;
  r.z = uv.z * sv.z + r.z;
  r.w = uv.w * sv.w + r.w;
  *(float4*)(xres + pix * c + c0) = r;
  uint2 pk;
  pk.x = (uint32_t)f2bf(r.x) | ((uint32_t)f2bf(r.y) << 16);
  pk.y = (uint32_t)f2bf(r.z) | ((uint32_t)f2bf(r.w) << 16);
  *(uint2*)(xb + pix * xb_cs + c0) = pk;
}

extern "C" int climsr_ca_scale_add(const void* u, int u_bf16, int u_cstride, const float* s, float* xres, uint16_t* xb, int xb_cstride,
                                   int n, int64_t hw, int c, void* stream) {
  if (!u || !s || !xres || !xb || n <= 0 || hw <= 0 || c % 4 || u_cstride % 4 || xb_cstride % 4 || u_cstride < c ||
      xb_cstride < c) {
    set_error("ca_scale_add: bad args (c, strides multiples of 4)");
    return CLIMSR_EINVAL;
  }
  const long total4 = (long)n * hw * (c / 4);
  if (u_bf16)
    hipLaunchKernelGGL(ca_scale_add_kernel<true>, dim3(ceil_div(total4, 256)), dim3(256), 0, (hipStream_t)stream, u, u_cstride, s,
                       xres, xb, xb_cstride, (long)hw, c, total4);
  else
    hipLaunchKernelGGL(ca_scale_add_kernel<false>, dim3(ceil_div(total4, 256)), dim3(256), 0, (hipStream_t)stream, u, u_cstride, s,
                       xres, xb, xb_cstride, (long)hw, c, total4);
  return check_launch("ca_scale_add");
}

// nn.PixelShuffle(r) on NHWC: y[n][y*r+i][x*r+j][co] = x[n][y][x][co*r*r + i*r + j]; one thread per output
// (pixel, 8 channels): 8 gathered 2 B reads from one input pixel's channel vector, one 16 B store.
__global__ __launch_bounds__(256) void pixel_shuffle_kernel(const uint16_t* __restrict__ x, int h, int w, int c_out, int r,
                                                            int in_cs, uint16_t* __restrict__ y, int out_cs, long total) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int cg = c_out / 8;
  const long opix = i / cg;
  const int co0 = (int)(i % cg) * 8;
  const int ow = w * r, oh = h * r;
  const int ox = (int)(opix % ow);
  const long t = opix / ow;
  const int oy = (int)(t % oh);
  const long nimg = t / oh;
  const int yy = oy / r, ii = oy - yy * r, xx = ox / r, jj = ox - xx * r;
  const uint16_t* src = x + ((nimg * h + yy) * w + xx) * in_cs + ii * r + jj;
  const int rr = r * r;
  uint32_t v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = (uint32_t)src[(co0 + 2 * k) * rr] | ((uint32_t)src[(co0 + 2 * k + 1) * rr] << 16);
  *(uint4*)(y + opix * out_cs + co0) = make_uint4(v[0], v[1], v[2], v[3]);
}

extern "C" int climsr_pixel_shuffle_bf16(const uint16_t* x, int n, int h, int w, int c_out, int r, int in_cstride, uint16_t* y,
                                         int out_cstride, void* stream) {
  if (!x || !y || n <= 0 || h <= 0 || w <= 0 || r < 1 || c_out % 8 || out_cstride % 8 || out_cstride < c_out ||
      in_cstride < c_out * r * r) {
    set_error("pixel_shuffle: bad args (c_out, out_cstride multiples of 8; in_cstride >= c_out*r*r)");
    return CLIMSR_EINVAL;
  }
  const long total = (long)n * h * r * w * r * (c_out / 8);
  hipLaunchKernelGGL(pixel_shuffle_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, x, h, w, c_out, r,
                     in_cstride, y, out_cstride, total);
  return check_launch("pixel_shuffle");
}

// ------------------------------------------------------------------------------------------------------------------
// RCAN training (the reference trains RCAN under the L1 pre-training task,
// conf/experiment/rcan_pre_training.yaml): the backward of the RCAB's channel attention + residual and of the
// Upsampler's PixelShuffle.  With y = u * s + x (rcan.py:65-68, 98-101), s = sigmoid(W2 relu(W1 m + b1) + b2) and
// m = mean_p u (rcan.py:56-63), for the incoming gradient gy:
//   g_s[c]  = sum_p gy[p][c] u[p][c]                                     (ca_bwd_parts_kernel: fixed-order slices)
//   g_a2    = g_s s (1 - s);  g_h = W2^T g_a2;  g_a1 = g_h [W1 m + b1 > 0];  g_m = W1^T g_a1      (ca_bwd_mlp_kernel)
//   dW2 += g_a2 h^T, db2 += g_a2, dW1 += g_a1 m^T, db1 += g_a1, summed over the images in order    (ca_bwd_wsum_kernel)
//   g_u[p][c] = gy[p][c] s[c] + g_m[c] / hw   (bf16: what the RCAB's second conv's gradients read) (ca_bwd_apply_kernel)
// (the direct path of the residual, dL/dx += gy, is the caller's: the first conv's data gradient accumulates into gy).
// ------------------------------------------------------------------------------------------------------------------
namespace {
constexpr int CA_BWD_PX_PER_SLICE = 64;  // pixels per slice of the g_s pass (slices per image <= CA_BWD_MAX_SLICES)
constexpr int CA_BWD_MAX_SLICES = 256;
int ca_bwd_slices(int64_t hw) {
  const int64_t s = (hw + CA_BWD_PX_PER_SLICE - 1) / CA_BWD_PX_PER_SLICE;
  return (int)(s < 1 ? 1 : s > CA_BWD_MAX_SLICES ? CA_BWD_MAX_SLICES : s);
}
}  // namespace

// part[n][sl][c] = sum over the slice's pixels of gy * u (gy fp32, u fp32 or bf16; NHWC with channel strides).
// A block = (c / 4 float4 channel lanes) x (256 / (c / 4) pixel lanes): per-thread fp32 sums in pixel order, fp64
// across the block's pixel lanes in a fixed order.
template <bool UB>
__global__ __launch_bounds__(256) void ca_bwd_parts_kernel(const float* __restrict__ gy, int gy_cs, const void* __restrict__ u, int u_cs,
                                                           long hw, int c, int nsl, double* __restrict__ part) {
  const int nimg = blockIdx.y, sp = blockIdx.x;
  const long p0 = hw * sp / nsl, p1 = hw * (sp + 1) / nsl;
  __shared__ double sh[256 * 4];
  const int cg = c / 4;
  const int plan = 256 / cg;
  const int g = threadIdx.x % cg, pl = threadIdx.x / cg;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (pl < plan)
    for (long p = p0 + pl; p < p1; p += plan) {
      const long pix = (long)nimg * hw + p;
      const float4 gv = *(const float4*)(gy + pix * gy_cs + g * 4);
      float uv[4];
      if constexpr (UB) {
        const uint2 raw = *(const uint2*)((const uint16_t*)u + pix * u_cs + g * 4);
        uv[0] = __uint_as_float(raw.x << 16);
        uv[1] = __uint_as_float(raw.x & 0xFFFF0000u);
        uv[2] = __uint_as_float(raw.y << 16);
        uv[3] = __uint_as_float(raw.y & 0xFFFF0000u);
      } else {
        const float4 v = *(const float4*)((const float*)u + pix * u_cs + g * 4);
        uv[0] = v.x; uv[1] = v.y; uv[2] = v.z; uv[3] = v.w;
      }
      a[0] = fmaf(gv.x, uv[0], a[0]);
      a[1] = fmaf(gv.y, uv[1], a[1]);
      a[2] = fmaf(gv.z, uv[2], a[2]);
      a[3] = fmaf(gv.w, uv[3], a[3]);
    }
#pragma unroll
  for (int q = 0; q < 4; ++q) sh[threadIdx.x * 4 + q] = a[q];
  __syncthreads();
  for (int ch = threadIdx.x; ch < c; ch += 256) {
    const int gg = ch / 4, q = ch % 4;
    double t = 0.0;
    for (int k = 0; k < plan; ++k) t += sh[(k * cg + gg) * 4 + q];
    part[((long)nimg * nsl + sp) * c + ch] = t;
  }
}

// One workgroup per image: fold the slices (fixed order), then the MLP backward.  Writes ga2[n][c], hid[n][cr]
// (= relu(W1 m + b1), recomputed exactly as ca_mlp_kernel computed it: one wave's lane-strided dot product + the same
// xor tree), ga1[n][cr] and gm[n][c] = g_m / hw.
__global__ __launch_bounds__(256) void ca_bwd_mlp_kernel(const double* __restrict__ part, int nsl, long hw, int c, int cr,
                                                         const float* __restrict__ s, const float* __restrict__ mean,
                                                         const float* __restrict__ w1, const float* __restrict__ b1,
                                                         const float* __restrict__ w2, float* __restrict__ ga2, float* __restrict__ hid,
                                                         float* __restrict__ ga1, float* __restrict__ gm) {
  extern __shared__ float sm[];
  float* g2 = sm;           // [c]
  float* mm = sm + c;       // [c]
  float* g1 = sm + 2 * c;   // [cr]
  const int nimg = blockIdx.x, t = threadIdx.x;
  for (int ch = t; ch < c; ch += 256) {
    const double* pp = part + (long)nimg * nsl * c + ch;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    int sp = 0;
    for (; sp + 3 < nsl; sp += 4) {
      a0 += pp[(long)sp * c];
      a1 += pp[(long)(sp + 1) * c];
      a2 += pp[(long)(sp + 2) * c];
      a3 += pp[(long)(sp + 3) * c];
    }
    for (; sp < nsl; ++sp) a0 += pp[(long)sp * c];
    const float gs = (float)((a0 + a1) + (a2 + a3));
    const float sv = s[(long)nimg * c + ch];
    const float v = gs * sv * (1.f - sv);
    g2[ch] = v;
    ga2[(long)nimg * c + ch] = v;
    mm[ch] = mean[(long)nimg * c + ch];
  }
  __syncthreads();
  const int wave = t >> 6, lane = t & 63;
  for (int j = wave; j < cr; j += 4) {
    float a = 0.f, gh = 0.f;
    for (int i = lane; i < c; i += 64) {
      a += w1[j * c + i] * mm[i];
      gh += w2[i * cr + j] * g2[i];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      a += __shfl_xor(a, off);
      gh += __shfl_xor(gh, off);
    }
    if (lane == 0) {
      a += b1 ? b1[j] : 0.f;
      const float ga = a > 0.f ? gh : 0.f;
      g1[j] = ga;
      hid[(long)nimg * cr + j] = a > 0.f ? a : 0.f;
      ga1[(long)nimg * cr + j] = ga;
    }
  }
  __syncthreads();
  const float inv = (float)(1.0 / (double)hw);
  for (int ch = t; ch < c; ch += 256) {
    float v = 0.f;
    for (int j = 0; j < cr; ++j) v += w1[j * c + ch] * g1[j];
    gm[(long)nimg * c + ch] = v * inv;
  }
}

// The four parameter gradients of conv_du, each element a sum over the images in order (fp32), '=' or '+='.
// Element e: [0, cr c) dW1[j][i] = sum ga1[j] m[i];  [cr c, cr c + cr) db1;  then dW2[i][j] = sum ga2[i] hid[j];  db2.
__global__ __launch_bounds__(256) void ca_bwd_wsum_kernel(int n, int c, int cr, const float* __restrict__ ga2, const float* __restrict__ hid,
                                                          const float* __restrict__ ga1, const float* __restrict__ mean,
                                                          float* __restrict__ gw1, float* __restrict__ gb1, float* __restrict__ gw2,
                                                          float* __restrict__ gb2, int accumulate) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int n_w1 = cr * c, n_b1 = cr, n_w2 = c * cr, n_b2 = c;
  float v = 0.f;
  float* dst = nullptr;
  if (e < n_w1) {
    const int j = e / c, i = e - j * c;
    for (int k = 0; k < n; ++k) v = fmaf(ga1[(long)k * cr + j], mean[(long)k * c + i], v);
    dst = gw1 + e;
  } else if (e < n_w1 + n_b1) {
    const int j = e - n_w1;
    for (int k = 0; k < n; ++k) v += ga1[(long)k * cr + j];
    dst = gb1 ? gb1 + j : nullptr;
  } else if (e < n_w1 + n_b1 + n_w2) {
    const int f = e - n_w1 - n_b1, i = f / cr, j = f - i * cr;
    for (int k = 0; k < n; ++k) v = fmaf(ga2[(long)k * c + i], hid[(long)k * cr + j], v);
    dst = gw2 + f;
  } else if (e < n_w1 + n_b1 + n_w2 + n_b2) {
    const int i = e - n_w1 - n_b1 - n_w2;
    for (int k = 0; k < n; ++k) v += ga2[(long)k * c + i];
    dst = gb2 ? gb2 + i : nullptr;
  }
  if (dst) *dst = accumulate ? *dst + v : v;
}

// gu[p][c0..c0+7] = bf16(gy[p][c] * s[n][c] + gm[n][c]): one thread per (pixel, 8 channels), one 16 B store.
__global__ __launch_bounds__(256) void ca_bwd_apply_kernel(const float* __restrict__ gy, int gy_cs, const float* __restrict__ s,
                                                           const float* __restrict__ gm, long hw, int c, uint16_t* __restrict__ gu, int gu_cs,
                                                           long total8) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total8) return;
  const int cg = c / 8;
  const long pix = i / cg;
  const int c0 = (int)(i - pix * cg) * 8;
  const long nimg = pix / hw;
  const float4 g0 = *(const float4*)(gy + pix * gy_cs + c0), g1 = *(const float4*)(gy + pix * gy_cs + c0 + 4);
  const float4 s0 = *(const float4*)(s + nimg * c + c0), s1 = *(const float4*)(s + nimg * c + c0 + 4);
  const float4 m0 = *(const float4*)(gm + nimg * c + c0), m1 = *(const float4*)(gm + nimg * c + c0 + 4);
  uint4 o;
  o.x = (uint32_t)f2bf(fmaf(g0.x, s0.x, m0.x)) | ((uint32_t)f2bf(fmaf(g0.y, s0.y, m0.y)) << 16);
  o.y = (uint32_t)f2bf(fmaf(g0.z, s0.z, m0.z)) | ((uint32_t)f2bf(fmaf(g0.w, s0.w, m0.w)) << 16);
  o.z = (uint32_t)f2bf(fmaf(g1.x, s1.x, m1.x)) | ((uint32_t)f2bf(fmaf(g1.y, s1.y, m1.y)) << 16);
  o.w = (uint32_t)f2bf(fmaf(g1.z, s1.z, m1.z)) | ((uint32_t)f2bf(fmaf(g1.w, s1.w, m1.w)) << 16);
  *(uint4*)(gu + pix * gu_cs + c0) = o;
}

namespace {
struct CaBwdWs {  // byte offsets into the caller's workspace (every piece 256 B aligned)
  size_t part, ga2, hid, ga1, gm, total;
};
CaBwdWs ca_bwd_ws(int n, int64_t hw, int c, int cr) {
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  CaBwdWs w;
  w.part = 0;
  w.ga2 = al((size_t)n * ca_bwd_slices(hw) * c * sizeof(double));
  w.hid = w.ga2 + al((size_t)n * c * sizeof(float));
  w.ga1 = w.hid + al((size_t)n * cr * sizeof(float));
  w.gm = w.ga1 + al((size_t)n * cr * sizeof(float));
  w.total = w.gm + al((size_t)n * c * sizeof(float));
  return w;
}
}  // namespace

extern "C" size_t climsr_ca_backward_workspace(int n, int64_t hw, int c, int cr) {
  if (n <= 0 || hw <= 0 || c <= 0 || cr <= 0) return 0;
  return ca_bwd_ws(n, hw, c, cr).total;
}

extern "C" int climsr_ca_backward(const float* gy, int gy_cstride, const void* u, int u_bf16, int u_cstride, const float* s, const float* mean,
                                  int n, int64_t hw, int c, const float* w1, const float* b1, const float* w2, int cr, float* gw1, float* gb1,
                                  float* gw2, float* gb2, int accumulate, void* workspace, uint16_t* gu, int gu_cstride, void* stream) {
  if (!gy || !u || !s || !mean || !w1 || !w2 || !gw1 || !gw2 || !workspace || !gu || n <= 0 || hw <= 0 || c <= 0 || cr <= 0 ||
      c % 8 || c > 1024 || cr > 256 || gy_cstride % 8 || u_cstride % 4 || gu_cstride % 8 || gy_cstride < c || u_cstride < c ||
      gu_cstride < c || (b1 == nullptr) != (gb1 == nullptr)) {
    set_error("ca_backward: bad args (c multiple of 8 and <= 1024, cr <= 256, gy / gu strides multiples of 8, u stride of 4; b1 and gb1 "
              "both given or both null)");
    return CLIMSR_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  const CaBwdWs w = ca_bwd_ws(n, hw, c, cr);
  char* base = (char*)workspace;
  double* part = (double*)(base + w.part);
  float *ga2 = (float*)(base + w.ga2), *hid = (float*)(base + w.hid), *ga1 = (float*)(base + w.ga1), *gm = (float*)(base + w.gm);
  const int nsl = ca_bwd_slices(hw);
  if (u_bf16)
    hipLaunchKernelGGL(ca_bwd_parts_kernel<true>, dim3(nsl, n), dim3(256), 0, st, gy, gy_cstride, u, u_cstride, (long)hw, c, nsl, part);
  else
    hipLaunchKernelGGL(ca_bwd_parts_kernel<false>, dim3(nsl, n), dim3(256), 0, st, gy, gy_cstride, u, u_cstride, (long)hw, c, nsl, part);
  hipLaunchKernelGGL(ca_bwd_mlp_kernel, dim3(n), dim3(256), (size_t)(2 * c + cr) * sizeof(float), st, part, nsl, (long)hw, c, cr, s, mean,
                     w1, b1, w2, ga2, hid, ga1, gm);
  const int nel = 2 * cr * c + cr + c;
  hipLaunchKernelGGL(ca_bwd_wsum_kernel, dim3(ceil_div(nel, 256)), dim3(256), 0, st, n, c, cr, ga2, hid, ga1, mean, gw1, gb1, gw2, gb2,
                     accumulate);
  const long total8 = (long)n * hw * (c / 8);
  hipLaunchKernelGGL(ca_bwd_apply_kernel, dim3(ceil_div(total8, 256)), dim3(256), 0, st, gy, gy_cstride, s, gm, (long)hw, c, gu, gu_cstride,
                     total8);
  return check_launch("ca_backward");
}

// Backward of nn.PixelShuffle(r) on NHWC bf16 (the inverse index map, bit-exact):
//   gx[n][y][x][co*r*r + i*r + j] = gy[n][y*r+i][x*r+j][co]
// one thread per (low-resolution pixel, 8 consecutive channels of gx): 8 gathered 2 B reads, one 16 B store.
__global__ __launch_bounds__(256) void pixel_unshuffle_kernel(const uint16_t* __restrict__ gy, int h, int w, int c_out, int r, int gy_cs,
                                                              uint16_t* __restrict__ gx, int gx_cs, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int rr = r * r, c4 = c_out * rr, kg = c4 / 8;
  const long pix = i / kg;
  const int k0 = (int)(i - pix * kg) * 8;
  const int xx = (int)(pix % w);
  const long t = pix / w;
  const int yy = (int)(t % h);
  const long nimg = t / h;
  const int ow = w * r;
  uint32_t v[4];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int k = k0 + q, co = k / rr, ij = k - co * rr, ii = ij / r, jj = ij - ii * r;
    const uint16_t e = gy[((nimg * h * r + yy * r + ii) * ow + xx * r + jj) * (long)gy_cs + co];
    if (q & 1) v[q >> 1] |= (uint32_t)e << 16;
    else v[q >> 1] = e;
  }
  *(uint4*)(gx + pix * gx_cs + k0) = make_uint4(v[0], v[1], v[2], v[3]);
}

extern "C" int climsr_pixel_unshuffle_bf16(const uint16_t* gy, int n, int h, int w, int c_out, int r, int gy_cstride, uint16_t* gx,
                                           int gx_cstride, void* stream) {
  if (!gy || !gx || n <= 0 || h <= 0 || w <= 0 || r < 1 || c_out <= 0 || (c_out * r * r) % 8 || gx_cstride % 8 ||
      gx_cstride < c_out * r * r || gy_cstride < c_out) {
    set_error("pixel_unshuffle: bad args (c_out*r*r and gx_cstride multiples of 8, gx_cstride >= c_out*r*r, gy_cstride >= c_out)");
    return CLIMSR_EINVAL;
  }
  const long total = (long)n * h * w * (c_out * r * r / 8);
  hipLaunchKernelGGL(pixel_unshuffle_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, gy, h, w, c_out, r, gy_cstride,
                     gx, gx_cstride, total);
  return check_launch("pixel_unshuffle");
}
