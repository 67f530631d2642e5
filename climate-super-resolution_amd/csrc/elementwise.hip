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
                                uint16_t* __restrict__ dz, int dzcs) {
  // one thread per (pixel, group of 8 dz channels)
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  int groups = dzcs / 8;
  if (idx >= npix * groups) return;
  long p = idx / groups;
  int c0 = (int)(idx % groups) * 8;
  uint16_t o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    int c = c0 + i;
    float v = 0.f;
    if (c < c_real) {
      v = g[p * gcs + gco + c] * scale;
      if (act) {
        float yy = bf2f(y[p * ycs + yco + c]);
        if (!(yy > 0.f)) v = (act == 1) ? v * slope : 0.f;
      }
    }
    o[i] = f2bf(v);
  }
  uint4 pk;
  pk.x = o[0] | ((uint32_t)o[1] << 16);
  pk.y = o[2] | ((uint32_t)o[3] << 16);
  pk.z = o[4] | ((uint32_t)o[5] << 16);
  pk.w = o[6] | ((uint32_t)o[7] << 16);
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
  hipLaunchKernelGGL(act_grad_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, (long)npix, c_real, g,
                     g_cstride, g_coff, y, y_cstride, y_coff, act, slope, scale, dz, dz_cstride);
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

// y = a*x + b*y over channel slices (fp32); x may be NULL (then y = b*y)
__global__ void axpby_kernel(long npix, int c, float a, const float* __restrict__ x, int xcs, int xco, float b, float* y,
                             int ycs, int yco) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
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
  long total = (long)npix * c;
  hipLaunchKernelGGL(axpby_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, (long)npix, c, a, x, x_cstride,
                     x_coff, b, y, y_cstride, y_coff);
  return check_launch("axpby_f32");
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
__global__ void adamw_kernel(long n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, const float* __restrict__ hp) {
  const float lr = hp[0], b1 = hp[1], b2 = hp[2], eps = hp[3], wd = hp[4], step_size = hp[5], bc2s = hp[6];
  long i4 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 + 3 < n) {
    float4 pp = *(float4*)(p + i4), gg = *(const float4*)(g + i4), mm = *(float4*)(m + i4), vv = *(float4*)(v + i4);
    float* P = (float*)&pp; const float* G = (const float*)&gg; float* M = (float*)&mm; float* V = (float*)&vv;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      P[k] *= 1.f - lr * wd;
      M[k] = M[k] + (G[k] - M[k]) * (1.f - b1);
      V[k] = V[k] * b2 + G[k] * G[k] * (1.f - b2);
      P[k] -= step_size * (M[k] / (sqrtf(V[k]) / bc2s + eps));
    }
    *(float4*)(p + i4) = pp; *(float4*)(m + i4) = mm; *(float4*)(v + i4) = vv;
  } else {
    for (long i = i4; i < n; ++i) {
      float pi = p[i] * (1.f - lr * wd);
      float mi = m[i] + (g[i] - m[i]) * (1.f - b1);
      float vi = v[i] * b2 + g[i] * g[i] * (1.f - b2);
      p[i] = pi - step_size * (mi / (sqrtf(vi) / bc2s + eps));
      m[i] = mi; v[i] = vi;
    }
  }
}

extern "C" int climsr_adamw_step(int64_t n, float* p, const float* g, float* m, float* v, const float* hp, void* stream) {
  if (!p || !g || !m || !v || !hp || n <= 0) {
    set_error("adamw_step: bad args");
    return CLIMSR_EINVAL;
  }
  long threads = (n + 3) / 4;
  hipLaunchKernelGGL(adamw_kernel, dim3(ceil_div(threads, 256)), dim3(256), 0, (hipStream_t)stream, (long)n, p, g, m, v, hp);
  return check_launch("adamw_step");
}
