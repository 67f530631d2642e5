// Memory-bound kernels of the ESRGAN step: activation gradients, layout conversion at the
// torch (NCHW fp32) boundary, gradient routing, L1 loss, OneCycleLR + AdamW.
// All vectorised 16 B per lane where the layout allows (Guideline 13).
#include <math.h>

#include "common.h"

using namespace climsr;

// ------------------------------------------------------------------------------------------
// activation gradient -> bf16 dZ (MFMA operand of the following dgrad / wgrad)
// ------------------------------------------------------------------------------------------
__global__ void act_grad_kernel(long npix, int c_real, const float* __restrict__ g, int gcs, int gco,
                                const uint16_t* __restrict__ y, int ycs, int yco, int act, float slope, float scale,
                                uint16_t* __restrict__ dz, int dzcs, int vec) {
  // one thread per (pixel, group of 8 dz channels); vec: g/y slices are 16 B aligned and c_real % 8 == 0
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  int groups = dzcs / 8;
  if (idx >= npix * groups) return;
  long p = idx / groups;
  int c0 = (int)(idx % groups) * 8;
  float v[8];
  if (vec && c0 < c_real) {
    const float4* gp = (const float4*)(g + p * gcs + gco + c0);
    float4 a = gp[0], b = gp[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    if (act) {
      uint4 yy = *(const uint4*)(y + p * ycs + yco + c0);
      uint32_t w[4] = {yy.x, yy.y, yy.z, yy.w};
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        uint16_t u = (uint16_t)(w[i >> 1] >> ((i & 1) * 16));
        float yf = bf2f(u);
        v[i] *= scale;
        if (!(yf > 0.f)) v[i] = (act == 1) ? v[i] * slope : 0.f;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] *= scale;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      int c = c0 + i;
      float t = 0.f;
      if (c < c_real) {
        t = g[p * gcs + gco + c] * scale;
        if (act) {
          float yy = bf2f(y[p * ycs + yco + c]);
          if (!(yy > 0.f)) t = (act == 1) ? t * slope : 0.f;
        }
      }
      v[i] = t;
    }
  }
  uint4 pk;
  pk.x = f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  pk.y = f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  pk.z = f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
  pk.w = f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
  *(uint4*)(dz + p * dzcs + c0) = pk;
}

extern "C" int climsr_act_grad(int64_t npix, int c_real, const float* g, int g_cstride, int g_coff, const uint16_t* y,
                               int y_cstride, int y_coff, int act, float slope, float scale, uint16_t* dz, int dz_cstride,
                               void* stream) {
  if (!g || !dz || dz_cstride % 8 || c_real > dz_cstride || (act && !y)) {
    set_error("act_grad: bad args");
    return CLIMSR_EINVAL;
  }
  long total = (long)npix * (dz_cstride / 8);
  int vec = (c_real % 8 == 0) && (g_cstride % 4 == 0) && (g_coff % 4 == 0) && (!act || (y_cstride % 8 == 0 && y_coff % 8 == 0)) &&
            ((uintptr_t)g % 16 == 0) && (!act || (uintptr_t)y % 16 == 0);
  hipLaunchKernelGGL(act_grad_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, (long)npix, c_real, g,
                     g_cstride, g_coff, y, y_cstride, y_coff, act, slope, scale, dz, dz_cstride, vec);
  return check_launch("act_grad");
}

// ------------------------------------------------------------------------------------------
// layout conversion at the torch boundary
// ------------------------------------------------------------------------------------------
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ src, int n, int c, int h, int w, uint16_t* __restrict__ dst,
                                    int cs, int co) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;  // over n*h*w pixels (coalesced source reads per channel)
  long npix = (long)n * h * w;
  if (idx >= npix) return;
  long hw = (long)h * w;
  long b = idx / hw, r = idx % hw;
  for (int ch = 0; ch < c; ++ch) dst[idx * cs + co + ch] = f2bf(src[(b * c + ch) * hw + r]);
}

extern "C" int climsr_nchw_to_nhwc_bf16(const float* src, int n, int c, int h, int w, uint16_t* dst, int cstride, int coff,
                                        void* stream) {
  if (!src || !dst || coff + c > cstride) {
    set_error("nchw_to_nhwc_bf16: bad args");
    return CLIMSR_EINVAL;
  }
  long npix = (long)n * h * w;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(ceil_div(npix, 256)), dim3(256), 0, (hipStream_t)stream, src, n, c, h, w, dst,
                     cstride, coff);
  return check_launch("nchw_to_nhwc_bf16");
}

// Up to 8 fp32 planes ([n] images of h*w, image stride per plane) -> one bf16 NHWC pixel of 8 channels per thread, a
// single 16 B store (channel k = plane k, zero where the plane is absent): the padded network inputs (G's lr /
// elevation / mask, D's input, the perceptual loss's 3-channel repeat) in one pass, no zero fill beforehand and no
// 2-byte strided stores.
__global__ void pack_planes8_kernel(ClimsrPlanes8 pl, int n, long hw, uint16_t* __restrict__ dst) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)n * hw) return;
  const long b = idx / hw, r = idx - b * hw;
  uint32_t v[4];
#pragma unroll
  for (int k = 0; k < 8; k += 2) {
    const uint16_t lo = pl.p[k] ? f2bf(pl.p[k][b * pl.img_stride[k] + r]) : (uint16_t)0;
    const uint16_t hi = pl.p[k + 1] ? f2bf(pl.p[k + 1][b * pl.img_stride[k + 1] + r]) : (uint16_t)0;
    v[k >> 1] = (uint32_t)lo | ((uint32_t)hi << 16);
  }
  *(uint4*)(dst + idx * 8) = make_uint4(v[0], v[1], v[2], v[3]);
}

extern "C" int climsr_pack_planes_nhwc8_bf16(const ClimsrPlanes8* planes, int n, int h, int w, uint16_t* dst, void* stream) {
  if (!planes || !dst || n <= 0 || h <= 0 || w <= 0) {
    set_error("pack_planes_nhwc8_bf16: bad args");
    return CLIMSR_EINVAL;
  }
  const long total = (long)n * h * w;
  hipLaunchKernelGGL(pack_planes8_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, *planes, n, (long)h * w, dst);
  return check_launch("pack_planes_nhwc8_bf16");
}

__global__ void nhwc_to_nchw_kernel(const void* __restrict__ src, int is_bf16, int n, int c, int h, int w, int cs, int co,
                                    float* __restrict__ dst) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long npix = (long)n * h * w;
  if (idx >= npix) return;
  long hw = (long)h * w;
  long b = idx / hw, r = idx % hw;
  for (int ch = 0; ch < c; ++ch) {
    long s = idx * cs + co + ch;
    float v = is_bf16 ? bf2f(((const uint16_t*)src)[s]) : ((const float*)src)[s];
    dst[(b * c + ch) * hw + r] = v;
  }
}

extern "C" int climsr_nhwc_to_nchw_f32(const void* src, int src_is_bf16, int n, int c, int h, int w, int cstride, int coff,
                                       float* dst, void* stream) {
  if (!src || !dst || coff + c > cstride) {
    set_error("nhwc_to_nchw_f32: bad args");
    return CLIMSR_EINVAL;
  }
  long npix = (long)n * h * w;
  hipLaunchKernelGGL(nhwc_to_nchw_kernel, dim3(ceil_div(npix, 256)), dim3(256), 0, (hipStream_t)stream, src, src_is_bf16, n, c,
                     h, w, cstride, coff, dst);
  return check_launch("nhwc_to_nchw_f32");
}

// y = a*x + b*y over channel slices (fp32); x may be NULL (then y = b*y).  4 channels per thread when aligned.
__global__ void axpby_kernel(long npix, int c, float a, const float* __restrict__ x, int xcs, int xco, float b, float* y,
                             int ycs, int yco, int vec) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (vec) {
    int groups = c / 4;
    if (idx >= npix * groups) return;
    long p = idx / groups;
    int ch = (int)(idx % groups) * 4;
    float4* yp = (float4*)(y + p * ycs + yco + ch);
    float4 xv = x ? *(const float4*)(x + p * xcs + xco + ch) : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 yv = (b != 0.f) ? *yp : make_float4(0.f, 0.f, 0.f, 0.f);
    *yp = make_float4(a * xv.x + b * yv.x, a * xv.y + b * yv.y, a * xv.z + b * yv.z, a * xv.w + b * yv.w);
    return;
  }
  if (idx >= npix * c) return;
  long p = idx / c;
  int ch = (int)(idx % c);
  float* yp = y + p * ycs + yco + ch;
  float xv = x ? x[p * xcs + xco + ch] : 0.f;
  float yv = (b != 0.f) ? *yp * b : 0.f;
  *yp = a * xv + yv;
}

extern "C" int climsr_axpby_f32(int64_t npix, int c, float a, const float* x, int x_cstride, int x_coff, float b, float* y,
                                int y_cstride, int y_coff, void* stream) {
  if (!y) {
    set_error("axpby_f32: null y");
    return CLIMSR_EINVAL;
  }
  int vec = (c % 4 == 0) && (y_cstride % 4 == 0) && (y_coff % 4 == 0) && ((uintptr_t)y % 16 == 0) &&
            (!x || (x_cstride % 4 == 0 && x_coff % 4 == 0 && (uintptr_t)x % 16 == 0));
  long total = (long)npix * (vec ? c / 4 : c);
  hipLaunchKernelGGL(axpby_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, (long)npix, c, a, x, x_cstride,
                     x_coff, b, y, y_cstride, y_coff, vec);
  return check_launch("axpby_f32");
}

// ------------------------------------------------------------------------------------------
// Residual-dense-block backward prologue (esrgan.py:38,54), one pass over the block's pixels:
//   g_o = a_o * gout (a_o = 0.2 for the 3rd RDB of an RRDB, whose output is out*0.2 + x)
//   save_skip: gskip = gout (the RRDB skip gradient);   gy[:, :nf] = g_o (+ gskip if add_skip)
//   gy[:, nf:dc] = 0;   dz5 = bf16(0.2 * g_o)  (conv5 output x5 enters as x5*0.2)
// ------------------------------------------------------------------------------------------
__global__ void rdb_bwd_init_kernel(long npix, int nf, int dc, const float* __restrict__ gx, float* __restrict__ gy,
                                    float* __restrict__ gskip, uint16_t* __restrict__ dz, float a_o, int save_skip, int add_skip) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  int groups = dc / 4;
  if (idx >= npix * groups) return;
  long p = idx / groups;
  int c = (int)(idx % groups) * 4;
  float4* yp = (float4*)(gy + p * dc + c);
  if (c >= nf) {
    *yp = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  float4 g = *(const float4*)(gx + p * dc + c);
  float4* sp = (float4*)(gskip + p * nf + c);
  if (save_skip) *sp = g;
  float4 o = make_float4(a_o * g.x, a_o * g.y, a_o * g.z, a_o * g.w);
  float4 r = o;
  if (add_skip) {
    float4 s = *sp;
    r.x += s.x; r.y += s.y; r.z += s.z; r.w += s.w;
  }
  *yp = r;
  uint2 pk;
  pk.x = f2bf(0.2f * o.x) | ((uint32_t)f2bf(0.2f * o.y) << 16);
  pk.y = f2bf(0.2f * o.z) | ((uint32_t)f2bf(0.2f * o.w) << 16);
  *(uint2*)(dz + p * nf + c) = pk;
}

extern "C" int climsr_rdb_bwd_init(int64_t npix, int nf, int dc, const float* gx, float* gy, float* gskip, uint16_t* dz, float a_o,
                                   int save_skip, int add_skip, void* stream) {
  if (!gx || !gy || !gskip || !dz || nf % 8 || dc % 4 || nf > dc) {
    set_error("rdb_bwd_init: bad args");
    return CLIMSR_EINVAL;
  }
  long total = (long)npix * (dc / 4);
  hipLaunchKernelGGL(rdb_bwd_init_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, (long)npix, nf, dc, gx, gy,
                     gskip, dz, a_o, save_skip, add_skip);
  return check_launch("rdb_bwd_init");
}

// ------------------------------------------------------------------------------------------
// L1 loss (mean): deterministic two-pass reduction with fp64 partials
// ------------------------------------------------------------------------------------------
constexpr int RED_BLOCKS = 512;

__device__ double block_sum(double v) {
  __shared__ double sh[4];
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o);
  int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  double r = 0.0;
  if (threadIdx.x == 0) r = sh[0] + sh[1] + sh[2] + sh[3];
  return r;
}

__global__ void l1_partial_kernel(const float* __restrict__ a, const float* __restrict__ b, long n, double* ws) {
  double s = 0.0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) s += fabs((double)a[i] - (double)b[i]);
  double r = block_sum(s);
  if (threadIdx.x == 0) ws[blockIdx.x] = r;
}

__global__ void l1_final_kernel(const double* ws, int nb, long n, float* out) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) s += ws[i];
  double r = block_sum(s);
  if (threadIdx.x == 0) out[0] = (float)(r / (double)n);
}

extern "C" int climsr_l1_loss(const float* a, const float* b, int64_t n, double* workspace, float* out, void* stream) {
  if (!a || !b || !workspace || !out || n <= 0) {
    set_error("l1_loss: bad args");
    return CLIMSR_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(l1_partial_kernel, dim3(RED_BLOCKS), dim3(256), 0, s, a, b, (long)n, workspace);
  hipLaunchKernelGGL(l1_final_kernel, dim3(1), dim3(256), 0, s, workspace, RED_BLOCKS, (long)n, out);
  return check_launch("l1_loss");
}

__global__ void l1_grad_kernel(const float* __restrict__ a, const float* __restrict__ b, long n, const float* gscale,
                               float* __restrict__ ga) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float d = a[i] - b[i];
  float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
  ga[i] = sg * (gscale ? gscale[0] : 1.f) / (float)n;
}

extern "C" int climsr_l1_loss_grad(const float* a, const float* b, int64_t n, const float* gscale, float* ga, void* stream) {
  if (!a || !b || !ga || n <= 0) {
    set_error("l1_loss_grad: bad args");
    return CLIMSR_EINVAL;
  }
  hipLaunchKernelGGL(l1_grad_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, a, b, (long)n, gscale, ga);
  return check_launch("l1_loss_grad");
}

// ------------------------------------------------------------------------------------------
// OneCycleLR (torch semantics, cos anneal, beta1 cycling 0.95 <-> 0.85) + AdamW scalars, on device
// so a captured hipGraph replays the schedule without host round trips.
// ------------------------------------------------------------------------------------------
__device__ double cos_anneal(double start, double end, double pct) { return end + (start - end) / 2.0 * (cos(M_PI * pct) + 1.0); }

__global__ void adamw_hparams_kernel(double* state, int total_steps, double max_lr, double pct_start, double div_factor,
                                     double final_div_factor, double beta2, double eps, double wd, float* hp) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double step = state[0] + 1.0;  // optimizer step about to be taken (torch increments before use)
  double sched = state[1];       // scheduler last_epoch
  double initial_lr = max_lr / div_factor;
  double min_lr = initial_lr / final_div_factor;
  double end0 = pct_start * total_steps - 1.0, end1 = (double)total_steps - 1.0;
  double lr, b1;
  if (sched <= end0) {
    double pct = sched / end0;
    lr = cos_anneal(initial_lr, max_lr, pct);
    b1 = cos_anneal(0.95, 0.85, pct);
  } else {
    double pct = (sched - end0) / (end1 - end0);
    lr = cos_anneal(max_lr, min_lr, pct);
    b1 = cos_anneal(0.85, 0.95, pct);
  }
  double bc1 = 1.0 - pow(b1, step);
  double bc2 = 1.0 - pow(beta2, step);
  hp[0] = (float)lr;
  hp[1] = (float)b1;
  hp[2] = (float)beta2;
  hp[3] = (float)eps;
  hp[4] = (float)wd;
  hp[5] = (float)(lr / bc1);
  hp[6] = (float)sqrt(bc2);
  hp[7] = 0.f;
  state[0] = step;
  state[1] = sched + 1.0;
}

extern "C" int climsr_adamw_hparams(double* state, int total_steps, double max_lr, double pct_start, double div_factor,
                                    double final_div_factor, double beta2, double eps, double wd, float* hp, void* stream) {
  if (!state || !hp || total_steps < 2) {
    set_error("adamw_hparams: bad args");
    return CLIMSR_EINVAL;
  }
  hipLaunchKernelGGL(adamw_hparams_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, state, total_steps, max_lr, pct_start,
                     div_factor, final_div_factor, beta2, eps, wd, hp);
  return check_launch("adamw_hparams");
}

// torch.optim.AdamW (amsgrad=False) single-tensor semantics in fp32:
//   p *= 1 - lr*wd; m = b1*m + (1-b1)*g; v = b2*v + (1-b2)*g*g; p -= (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)
// mirror (optional): bf16 copy of the updated p[lo, lo + mn) into mirror[0, mn) -- the MFMA operand of a layer whose
// weights are read straight from the flat buffer (the discriminator's fc.0), written by this pass instead of a
// separate fp32 -> bf16 sweep of the same 411 MB.
__device__ __forceinline__ void adamw_mirror(long i, float v, uint16_t* mirror, long lo, long mn) {
  if (mirror && i >= lo && i < lo + mn) mirror[i - lo] = f2bf(v);
}
// four consecutive elements at p + i (16 B aligned); returns the updated p
__device__ __forceinline__ float4 adamw_update4(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                                float* __restrict__ v, long i, const float* __restrict__ hp) {
  const float lr = hp[0], b1 = hp[1], b2 = hp[2], eps = hp[3], wd = hp[4], step_size = hp[5], bc2s = hp[6];
  float4 pp = *(float4*)(p + i), gg = *(const float4*)(g + i), mm = *(float4*)(m + i), vv = *(float4*)(v + i);
  float* P = (float*)&pp; const float* G = (const float*)&gg; float* M = (float*)&mm; float* V = (float*)&vv;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    P[k] *= 1.f - lr * wd;
    M[k] = M[k] + (G[k] - M[k]) * (1.f - b1);
    V[k] = V[k] * b2 + G[k] * G[k] * (1.f - b2);
    P[k] -= step_size * (M[k] / (sqrtf(V[k]) / bc2s + eps));
  }
  *(float4*)(p + i) = pp; *(float4*)(m + i) = mm; *(float4*)(v + i) = vv;
  return pp;
}

__device__ __forceinline__ uint2 bf16x4_pack(float4 a) {
  return make_uint2((uint32_t)f2bf(a.x) | ((uint32_t)f2bf(a.y) << 16), (uint32_t)f2bf(a.z) | ((uint32_t)f2bf(a.w) << 16));
}

__global__ void adamw_kernel(long n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, const float* __restrict__ hp, uint16_t* __restrict__ mirror = nullptr,
                             long mlo = 0, long mn = 0) {
  const float lr = hp[0], b1 = hp[1], b2 = hp[2], eps = hp[3], wd = hp[4], step_size = hp[5], bc2s = hp[6];
  long i4 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 + 3 < n) {
    const float4 pp = adamw_update4(p, g, m, v, i4, hp);
    const float* P = (const float*)&pp;
    if (mirror && i4 >= mlo && i4 + 3 < mlo + mn && ((i4 - mlo) & 3) == 0) {  // 8 B store of 4 bf16
      *(uint2*)(mirror + (i4 - mlo)) = bf16x4_pack(pp);
    } else if (mirror) {
#pragma unroll
      for (int k = 0; k < 4; ++k) adamw_mirror(i4 + k, P[k], mirror, mlo, mn);
    }
  } else {
    for (long i = i4; i < n; ++i) {
      float pi = p[i] * (1.f - lr * wd);
      float mi = m[i] + (g[i] - m[i]) * (1.f - b1);
      float vi = v[i] * b2 + g[i] * g[i] * (1.f - b2);
      p[i] = pi - step_size * (mi / (sqrtf(vi) / bc2s + eps));
      m[i] = mi; v[i] = vi;
      adamw_mirror(i, p[i], mirror, mlo, mn);
    }
  }
}

extern "C" int climsr_adamw_step(int64_t n, float* p, const float* g, float* m, float* v, const float* hp, void* stream) {
  if (!p || !g || !m || !v || !hp || n <= 0) {
    set_error("adamw_step: bad args");
    return CLIMSR_EINVAL;
  }
  long threads = (n + 3) / 4;
  hipLaunchKernelGGL(adamw_kernel, dim3(ceil_div(threads, 256)), dim3(256), 0, (hipStream_t)stream, (long)n, p, g, m, v, hp,
                     (uint16_t*)nullptr, 0L, 0L);
  return check_launch("adamw_step");
}

extern "C" int climsr_adamw_step_mirror(int64_t n, float* p, const float* g, float* m, float* v, const float* hp, int64_t mirror_lo,
                                        int64_t mirror_n, uint16_t* mirror, void* stream) {
  if (!p || !g || !m || !v || !hp || n <= 0 || !mirror || mirror_lo < 0 || mirror_n <= 0 || mirror_lo + mirror_n > n) {
    set_error("adamw_step_mirror: bad args");
    return CLIMSR_EINVAL;
  }
  long threads = (n + 3) / 4;
  hipLaunchKernelGGL(adamw_kernel, dim3(ceil_div(threads, 256)), dim3(256), 0, (hipStream_t)stream, (long)n, p, g, m, v, hp, mirror,
                     (long)mirror_lo, (long)mirror_n);
  return check_launch("adamw_step_mirror");
}
