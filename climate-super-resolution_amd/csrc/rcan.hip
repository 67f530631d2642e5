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
__global__ __launch_bounds__(1024) void ca_mlp_kernel(const double* __restrict__ part, int nsl, long hw, int c, int cr, const float* __restrict__ w1,
                              const float* __restrict__ b1, const float* __restrict__ w2, const float* __restrict__ b2,
                              float* __restrict__ s) {
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
  for (int c0 = 0; c0 < c; c0 += cw) {
    const int i = c0 + t % cw, gi = t / cw;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    if (i < c && gi < G) {
      const double* pp = part + (long)nimg * nsl * c + i;
      int sp = gi;
      for (; sp + 3 * G < nsl; sp += 4 * G) {
        a0 += pp[(long)sp * c];
        a1 += pp[(long)(sp + G) * c];
        a2 += pp[(long)(sp + 2 * G) * c];
        a3 += pp[(long)(sp + 3 * G) * c];
      }
      for (; sp < nsl; sp += G) a0 += pp[(long)sp * c];
    }
    grp[t] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (t < cw && c0 + t < c) {
      double m = 0.0;
      for (int k = 0; k < G; ++k) m += grp[k * cw + t];
      mean[c0 + t] = (float)(m / (double)hw);
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

extern "C" int climsr_channel_attention(const float* u, int n, int64_t hw, int c, int u_cstride, const float* w1, const float* b1,
                                        const float* w2, const float* b2, int cr, double* workspace, float* s, void* stream) {
  if (!u || !w1 || !w2 || !workspace || !s || n <= 0 || hw <= 0 || c <= 0 || cr <= 0 || u_cstride < c || c % 4 || u_cstride % 4 ||
      c > 1024) {
    set_error("channel_attention: bad args (c, u_cstride multiples of 4, c <= 1024)");
    return CLIMSR_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(channel_sum_partial_kernel, dim3(POOL_SPLIT, n), dim3(256), 0, st, u, (long)hw, c, u_cstride, workspace);
  hipLaunchKernelGGL(ca_mlp_kernel, dim3(n), dim3(1024), (size_t)(c + cr) * sizeof(float), st, workspace, POOL_SPLIT, (long)hw, c, cr, w1, b1,
                     w2, b2, s);
  return check_launch("channel_attention");
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

extern "C" int climsr_channel_attention_parts(const float* part, int n, int tiles_per_image, int64_t hw, int c, const float* w1,
                                              const float* b1, const float* w2, const float* b2, int cr, double* workspace, float* s,
                                              void* stream) {
  if (!part || !w1 || !w2 || !s || !workspace || n <= 0 || tiles_per_image <= 0 || hw <= 0 || c <= 0 || c > 1024 || cr <= 0) {
    set_error("channel_attention_parts: bad args");
    return CLIMSR_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(tile_parts_fold_kernel, dim3(TILE_SPLIT, n), dim3(256), 0, st, part, tiles_per_image, c, workspace);
  hipLaunchKernelGGL(ca_mlp_kernel, dim3(n), dim3(1024), (size_t)(c + cr) * sizeof(float), st, workspace, TILE_SPLIT, (long)hw, c, cr, w1, b1,
                     w2, b2, s);
  return check_launch("channel_attention_parts");
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
