// On-device tile pipeline and validation metrics.
//
// Tile pipeline: the per-sample work of ClimateDataset.__getitem__ / _get_training_sample /
// _get_val_test_sample (climsr/data/sr/climate_dataset.py:144-189, 191-218, 220-275) and the
// MinMaxScaler / StandardScaler arithmetic (climsr/data/normalization.py:37-61, 99-116), done for a
// whole batch of raw tiles already resident in HBM: v-flip, h-flip, rot90, normalisation with NaN
// substitution, land mask, nearest decimation to LR (cv2.INTER_NEAREST with an integer ratio picks
// [::s, ::s]) and the channel concatenation of _concat_if_needed (:95-118).  One thread per HR
// output pixel; every output is written once with unit stride.  HBM-bound byte shuffling: no MFMA.
//
// Metrics: TaskSuperResolutionModule.common_val_test_step + compute_metrics (climsr/core/task.py:
// 262-294, 336-372): denormalise, mask sea pixels to 0, then RegressionAccuracy x8, PSNR, SSIM,
// MAE, MSE, RMSE, MAPE, SMAPE, R2 and the normalised L1, as one fused deterministic reduction (fixed
// block partials, single-block final sum) plus a separable-Gaussian SSIM pass.  Nothing syncs the
// host: SSIM's data range and constants are read from the first pass's device results.
//
// Built with -ffp-contract=off (Makefile): the normalisation reproduces numpy's one-rounding-per-
// operation arithmetic bit for bit, which a fused multiply-add would break.
#include <math.h>

#include "common.h"

using namespace climsr;

// ------------------------------------------------------------------------------------------
// per-tile nanmin / nanmax (np.nanmin / np.nanmax after missing_indicator -> NaN)
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) tile_minmax_kernel(const float* __restrict__ x, long count, float missing,
                                                           int use_missing, float* __restrict__ out) {
  const float* t = x + (long)blockIdx.x * count;
  float mn = INFINITY, mx = -INFINITY;
  int any = 0;
  for (long i = threadIdx.x; i < count; i += blockDim.x) {
    float v = t[i];
    if (isnan(v) || (use_missing && v == missing)) continue;
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
    any = 1;
  }
  for (int o = 32; o > 0; o >>= 1) {
    mn = fminf(mn, __shfl_down(mn, o));
    mx = fmaxf(mx, __shfl_down(mx, o));
    any |= __shfl_down(any, o);
  }
  __shared__ float smn[16], smx[16];
  __shared__ int sany[16];
  int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    smn[wv] = mn;
    smx[wv] = mx;
    sany[wv] = any;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) {
      mn = fminf(mn, smn[i]);
      mx = fmaxf(mx, smx[i]);
      any |= sany[i];
    }
    out[2 * blockIdx.x] = any ? mn : NAN;  // all-NaN slice: numpy returns nan
    out[2 * blockIdx.x + 1] = any ? mx : NAN;
  }
}

extern "C" int climsr_tile_minmax_f32(const float* x, int n, int64_t count, float missing, int use_missing, float* out,
                                      void* stream) {
  if (!x || !out || n <= 0 || count <= 0) {
    set_error("tile_minmax: bad args (n=%d count=%lld)", n, (long long)count);
    return CLIMSR_EINVAL;
  }
  hipLaunchKernelGGL(tile_minmax_kernel, dim3(n), dim3(1024), 0, (hipStream_t)stream, x, (long)count, missing, use_missing, out);
  return check_launch("tile_minmax");
}

// ------------------------------------------------------------------------------------------
// tile pipeline
// ------------------------------------------------------------------------------------------
struct Scale32 {
  float mul, add;
};

// Output pixel (y, x) of the transformed tile -> pixel of the raw tile.  The reference applies, in
// order, np.flipud, np.fliplr, np.rot90(., k) (climate_dataset.py:149-166); invert rot first.
__device__ __forceinline__ void source_of(int y, int x, int h, int w, int code, int& sy, int& sx) {
  int k = (code >> 2) & 3;
  int fy, fx;  // position in the flipped (pre-rotation) array, which is h x w
  if (k == 0) {
    fy = y; fx = x;
  } else if (k == 1) {  // rot90 k=1: out[i, j] = in[j, W-1-i]
    fy = x; fx = w - 1 - y;
  } else if (k == 2) {  // out[i, j] = in[H-1-i, W-1-j]
    fy = h - 1 - y; fx = w - 1 - x;
  } else {              // k=3: out[i, j] = in[H-1-j, i]
    fy = h - 1 - x; fx = y;
  }
  sy = (code & 1) ? h - 1 - fy : fy;
  sx = (code & 2) ? w - 1 - fx : fx;
}

// MinMaxScaler._normalize with min/max given as float64 (the per-file / global stats of the feather
// tables): numpy computes scale and offset in float64 and, under NEP 50 (numpy >= 2), the float32
// tile is promoted by the np.float64 scalars, so the value is rounded to float32 once at the end.
__device__ __forceinline__ float minmax_f64(float v, double scale, double add, float nan_sub) {
  double r = __dadd_rn(__dmul_rn((double)v, scale), add);  // two double roundings, as numpy (no fma)
  float f = (float)r;
  return isnan(f) ? nan_sub : f;
}

// MinMaxScaler._normalize with min/max from np.nanmin/np.nanmax of a float32 array (elevation):
// everything stays float32 under NEP 50, with one rounding per numpy operation.
// Python-float operands (a, b - a, eps) are weak scalars: converted to float32 at each use.
__device__ __forceinline__ Scale32 minmax_f32_params(float mn, float mx, double a, double b, double eps) {
  float range = __fsub_rn(mx, mn);
  float den = __fadd_rn(range, (float)eps);
  float scale = __fdiv_rn((float)(b - a), den);
  float add = __fsub_rn((float)a, __fmul_rn(mn, scale));
  return {scale, add};
}

__device__ __forceinline__ float normalize_hr(float v, const ClimsrTileDesc& d, double scale, double add) {
  if (d.method == 0) return minmax_f64(v, scale, add, (float)d.nan_sub);
  if (d.method == 1) {  // StandardScaler: (arr - mean) / (std + eps) in float64 (np.float64 stats)
    double r = __ddiv_rn(__dsub_rn((double)v, d.zs_hr_mean), __dadd_rn(d.zs_hr_std, d.eps));
    float f = (float)r;
    if (isnan(f) && d.zs_hr_nan_sub != 0.0) f = (float)d.zs_hr_nan_sub;  // `if self.nan_substitution:`
    return f;
  }
  return v;
}

__device__ __forceinline__ float normalize_elev(float v, const ClimsrTileDesc& d, Scale32 es) {
  if (v == d.elev_missing) v = NAN;  // `out_arr[arr == missing_indicator] = np.nan`
  if (d.method == 0) {
    float f = __fadd_rn(__fmul_rn(v, es.mul), es.add);
    return isnan(f) ? (float)d.nan_sub : f;
  }
  if (d.method == 1) {
    double r = __ddiv_rn(__dsub_rn((double)v, d.zs_elev_mean), __dadd_rn(d.zs_elev_std, d.eps));
    float f = (float)r;
    if (isnan(f) && d.zs_elev_nan_sub != 0.0) f = (float)d.zs_elev_nan_sub;
    return f;
  }
  return v;
}

__global__ void __launch_bounds__(256) tile_prepare_kernel(ClimsrTileDesc d) {
  const int hw = d.h * d.w;
  long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long)d.n * hw) return;
  const int t = (int)(gid / hw);
  const int rem = (int)(gid - (long)t * hw);
  const int y = rem / d.w, x = rem - (rem / d.w) * d.w;
  const int code = d.xform ? d.xform[t] : 0;
  const float* hr_raw = d.hr_raw + (long)t * hw;
  const float* el_raw = d.elev_raw ? d.elev_raw + (long)t * hw : nullptr;

  double hs = 0.0, ha = 0.0;
  if (d.method == 0) {  // normalization.py:51-56 in float64
    double mn = d.hr_min[t], mx = d.hr_max[t];
    hs = __ddiv_rn(d.range_b - d.range_a, __dadd_rn(__dsub_rn(mx, mn), d.eps));
    ha = __dsub_rn(d.range_a, __dmul_rn(mn, hs));
  }
  Scale32 es = {0.f, 0.f};
  if (el_raw && d.method == 0) es = minmax_f32_params(d.elev_minmax[2 * t], d.elev_minmax[2 * t + 1], d.range_a, d.range_b, d.eps);

  int sy, sx;
  source_of(y, x, d.h, d.w, code, sy, sx);
  const float raw = hr_raw[sy * d.w + sx];
  const float hv = normalize_hr(raw, d, hs, ha);
  const float mv = isnan(raw) ? 0.f : 1.f;  // mask = ~np.isnan(original_image)
  const float ev = el_raw ? normalize_elev(el_raw[sy * d.w + sx], d, es) : 0.f;

  const long o = (long)t * hw + rem;
  d.hr[o] = hv;
  if (d.elev) d.elev[o] = ev;
  if (d.mask) d.mask[o] = mv;

  const int s = d.scale, lh = d.h / s, lw = d.w / s;
  // nearest decimation (A.Resize INTER_NEAREST, integer ratio) and nearest upscale of the LR tile
  const int ny = (y / s) * s, nx = (x / s) * s;
  float near = hv;
  if (ny != y || nx != x) {
    int qy, qx;
    source_of(ny, nx, d.h, d.w, code, qy, qx);
    near = normalize_hr(hr_raw[qy * d.w + qx], d, hs, ha);
  }
  if (d.nearest) d.nearest[o] = near;
  if (d.srcnn) {  // _concat_if_needed, SRCNN branch: [nearest(lr), elev, mask] at HR size
    float* l = d.lr + (long)t * d.lr_c * hw + rem;
    int c = 0;
    l[(long)(c++) * hw] = near;
    if (d.use_elev) l[(long)(c++) * hw] = ev;
    if (d.use_mask) l[(long)(c++) * hw] = mv;
  } else if (ny == y && nx == x) {  // [lr, elev_lr, mask_lr] at LR size
    const int lhw = lh * lw;
    const int lo = (y / s) * lw + (x / s);
    float* l = d.lr + (long)t * d.lr_c * lhw + lo;
    int c = 0;
    l[(long)(c++) * lhw] = hv;
    if (d.use_elev) l[(long)(c++) * lhw] = ev;
    if (d.use_mask) l[(long)(c++) * lhw] = mv;
  }
  if (d.elev_lr && ny == y && nx == x) d.elev_lr[(long)t * lh * lw + (y / s) * lw + (x / s)] = ev;
  if (d.hr_lr && ny == y && nx == x) d.hr_lr[(long)t * lh * lw + (y / s) * lw + (x / s)] = hv;
}

extern "C" int climsr_tile_prepare(const ClimsrTileDesc* d, void* stream) {
  if (!d || !d->hr_raw || !d->hr || !d->lr || d->n <= 0 || d->h <= 0 || d->w <= 0 || d->scale <= 0 ||
      d->h % d->scale || d->w % d->scale) {
    set_error("tile_prepare: bad args (h and w must be positive multiples of scale)");
    return CLIMSR_EINVAL;
  }
  int want_c = 1 + (d->use_elev ? 1 : 0) + (d->use_mask ? 1 : 0);
  if (d->lr_c != want_c || (d->use_elev && !d->elev_raw) || (d->method == 0 && (!d->hr_min || !d->hr_max)) ||
      (d->method == 0 && d->elev_raw && !d->elev_minmax) || d->method < 0 || d->method > 2) {
    set_error("tile_prepare: lr_c=%d (expected %d) / missing elevation, stats or min-max inputs", d->lr_c, want_c);
    return CLIMSR_EINVAL;
  }
  if (d->h != d->w && d->xform) {
    // rot90 with an odd factor changes the shape; the reference tiles are square (128 or 452)
    set_error("tile_prepare: random rotation needs square tiles (got %dx%d)", d->h, d->w);
    return CLIMSR_EINVAL;
  }
  long total = (long)d->n * d->h * d->w;
  hipLaunchKernelGGL(tile_prepare_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, *d);
  return check_launch("tile_prepare");
}

// ------------------------------------------------------------------------------------------
// cv2.resize(INTER_CUBIC) upscale, float32 path (the `cubic` baseline of the val/test batch,
// climate_dataset.py:195).  cv2: fx = (dx + 0.5) * (src/dst) - 0.5, sx = floor(fx), A = -0.75,
// taps sx-1..sx+2 clamped to the border (replicate), horizontal pass then vertical, float math.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void cubic_coeffs(float x, float c[4]) {
  const float A = -0.75f;
  c[0] = ((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A;
  c[1] = ((A + 2) * x - (A + 3)) * x * x + 1;
  c[2] = ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1;
  c[3] = 1.f - c[0] - c[1] - c[2];
}

__global__ void __launch_bounds__(256) resize_cubic_kernel(const float* __restrict__ src, int n, int sh, int sw,
                                                           float* __restrict__ dst, int dh, int dw) {
  long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long dhw = (long)dh * dw;
  if (gid >= (long)n * dhw) return;
  int t = (int)(gid / dhw);
  int rem = (int)(gid - (long)t * dhw);
  int dy = rem / dw, dx = rem - (rem / dw) * dw;
  float fy = (float)((dy + 0.5) * ((double)sh / dh) - 0.5);
  float fx = (float)((dx + 0.5) * ((double)sw / dw) - 0.5);
  int y0 = (int)floorf(fy), x0 = (int)floorf(fx);
  float cy[4], cx[4];
  cubic_coeffs(fy - y0, cy);
  cubic_coeffs(fx - x0, cx);
  const float* s = src + (long)t * sh * sw;
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int yy = min(max(y0 - 1 + i, 0), sh - 1);
    const float* row = s + (long)yy * sw;
    float r = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) r = __fadd_rn(r, __fmul_rn(row[min(max(x0 - 1 + j, 0), sw - 1)], cx[j]));
    acc = __fadd_rn(acc, __fmul_rn(r, cy[i]));
  }
  dst[gid] = acc;
}

extern "C" int climsr_resize_cubic_f32(const float* src, int n, int sh, int sw, float* dst, int dh, int dw, void* stream) {
  if (!src || !dst || n <= 0 || sh <= 0 || sw <= 0 || dh <= 0 || dw <= 0) {
    set_error("resize_cubic: bad args");
    return CLIMSR_EINVAL;
  }
  long total = (long)n * dh * dw;
  hipLaunchKernelGGL(resize_cubic_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, src, n, sh, sw, dst,
                     dh, dw);
  return check_launch("resize_cubic");
}

// ------------------------------------------------------------------------------------------
// validation / test metrics
// ------------------------------------------------------------------------------------------
namespace {
constexpr int MET_BLOCKS = 1024;  // 4 blocks of 4 waves per CU: the fused pass is load-latency bound
constexpr int SSIM_BLOCKS = 1024;
constexpr int SSIM_T = 32;                 // output tile edge
constexpr int SSIM_K = 11, SSIM_R = 5;     // torchmetrics SSIM defaults: kernel 11, sigma 1.5
constexpr int SSIM_IN = SSIM_T + 2 * SSIM_R;
// per-block partial slots
enum {
  P_ABS = 0, P_SQ, P_ACC0, P_MAPE = P_ACC0 + 8, P_SMAPE, P_T, P_TT, P_L1N, P_NSUM,
  P_TD_MIN = P_NSUM, P_TD_MAX, P_PN_MIN, P_PN_MAX, P_TN_MIN, P_TN_MAX, P_SLOTS
};
// stats after the first pass (workspace tail)
constexpr int WS_STATS = MET_BLOCKS * P_SLOTS;
constexpr int WS_SSIM = WS_STATS + 32;
}  // namespace

struct Denorm {
  int t = -1;
  double scale = 1.0, add = 0.0;
};

__device__ __forceinline__ void masked_values(const ClimsrMetricsDesc& d, long i, Denorm& dn, float& pn, float& tn, double& pd,
                                              double& td) {
  const int hw = d.h * d.w;
  const int t = (int)(i / hw);
  const bool land = d.mask[i] != 0.f;  // `(~mask.bool())` -> 0
  const float sr = d.sr[i];
  pn = land ? sr : 0.f;
  tn = land ? d.hr[i] : 0.f;
  double den;
  if (d.method == 0) {  // MinMaxScaler._denormalize with float64 min/max tensors (task.py:281-285)
    if (t != dn.t) {    // per-sample constants, recomputed only when the grid-stride loop crosses a sample
      double mn = d.min[t], mx = d.max[t];
      dn.scale = __ddiv_rn(d.range_b - d.range_a, __dadd_rn(__dsub_rn(mx, mn), d.eps));
      dn.add = __dsub_rn(d.range_a, __dmul_rn(mn, dn.scale));
      dn.t = t;
    }
    den = __ddiv_rn(__dsub_rn((double)sr, dn.add), dn.scale);
  } else if (d.method == 1) {  // StandardScaler._denormalize: float32 tensor * python float
    den = (double)__fadd_rn(__fmul_rn(sr, (float)d.zs_std), (float)d.zs_mean);
  } else {
    den = (double)sr;
  }
  pd = land ? den : 0.0;
  td = land ? (double)d.original[i] : 0.0;
}

__global__ void __launch_bounds__(256) metrics_partial_kernel(ClimsrMetricsDesc d) {
  double acc[P_NSUM];
#pragma unroll
  for (int k = 0; k < P_NSUM; ++k) acc[k] = 0.0;
  double tdmin = INFINITY, tdmax = -INFINITY;
  float pnmin = INFINITY, pnmax = -INFINITY, tnmin = INFINITY, tnmax = -INFINITY;
  const long total = (long)d.n * d.h * d.w;
  const float MEPS = 1.17e-06f;  // torchmetrics MAPE / SMAPE epsilon
  Denorm dn_cache;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    float pn, tn;
    double pd, td;
    masked_values(d, i, dn_cache, pn, tn, pd, td);
    double dd = pd - td;
    double ad = fabs(dd);
    acc[P_ABS] += ad;
    acc[P_SQ] += dd * dd;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[P_ACC0 + k] += (ad <= (double)d.acc_eps[k]) ? 1.0 : 0.0;
    float dn = fabsf(pn - tn);
    acc[P_MAPE] += (double)(dn / fmaxf(fabsf(tn), MEPS));
    acc[P_SMAPE] += ad / fmax(fabs(td) + fabs(pd), (double)MEPS);
    acc[P_T] += td;
    acc[P_TT] += td * td;
    acc[P_L1N] += (double)dn;
    tdmin = fmin(tdmin, td);
    tdmax = fmax(tdmax, td);
    pnmin = fminf(pnmin, pn);
    pnmax = fmaxf(pnmax, pn);
    tnmin = fminf(tnmin, tn);
    tnmax = fmaxf(tnmax, tn);
  }
  __shared__ double sh[P_SLOTS][4];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double v[P_SLOTS];
#pragma unroll
  for (int k = 0; k < P_NSUM; ++k) v[k] = acc[k];
  v[P_TD_MIN] = tdmin;
  v[P_TD_MAX] = tdmax;
  v[P_PN_MIN] = pnmin;
  v[P_PN_MAX] = pnmax;
  v[P_TN_MIN] = tnmin;
  v[P_TN_MAX] = tnmax;
#pragma unroll
  for (int k = 0; k < P_SLOTS; ++k) {
    double x = v[k];
    for (int o = 32; o > 0; o >>= 1) {
      double y = __shfl_down(x, o);
      if (k < P_NSUM) x += y;
      else if ((k - P_NSUM) % 2 == 0) x = fmin(x, y);
      else x = fmax(x, y);
    }
    if (lane == 0) sh[k][wv] = x;
  }
  __syncthreads();
  if (threadIdx.x < P_SLOTS) {
    int k = threadIdx.x;
    double x = sh[k][0];
    for (int i = 1; i < 4; ++i) {
      double y = sh[k][i];
      if (k < P_NSUM) x += y;
      else if ((k - P_NSUM) % 2 == 0) x = fmin(x, y);
      else x = fmax(x, y);
    }
    d.workspace[(long)blockIdx.x * P_SLOTS + k] = x;
  }
}

__device__ __forceinline__ double combine(int k, double x, double y) {
  if (k < P_NSUM) return x + y;
  return ((k - P_NSUM) % 2 == 0) ? fmin(x, y) : fmax(x, y);
}

// One block of 16 waves; wave w combines slots w, w+16: lane l folds partials l, l+64, ... in order, then a
// fixed shuffle tree -> deterministic, no block-wide barriers.
__global__ void __launch_bounds__(1024) metrics_stats_kernel(ClimsrMetricsDesc d) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int k = wv; k < P_SLOTS; k += 16) {
    double x = d.workspace[(long)lane * P_SLOTS + k];
    for (int b = lane + 64; b < MET_BLOCKS; b += 64) x = combine(k, x, d.workspace[(long)b * P_SLOTS + k]);
    for (int o = 32; o > 0; o >>= 1) x = combine(k, x, __shfl_down(x, o));
    if (lane == 0) d.workspace[WS_STATS + k] = x;
  }
}

// SSIM over the masked normalised maps: 5 Gaussian-filtered maps (p, t, p², t², pt), reflect padding
// (only the cropped interior [5, h-5) x [5, w-5) is averaged, whose windows never touch the pad).
__global__ void __launch_bounds__(256) ssim_kernel(ClimsrMetricsDesc d) {
  __shared__ float sp[SSIM_IN][SSIM_IN + 1], st[SSIM_IN][SSIM_IN + 1];
  __shared__ float hsum[5][SSIM_IN][SSIM_T + 1];
  __shared__ float g[SSIM_K];
  __shared__ double red[4];
  const int oh = d.h - 2 * SSIM_R, ow = d.w - 2 * SSIM_R;
  const int tiles_y = (oh + SSIM_T - 1) / SSIM_T, tiles_x = (ow + SSIM_T - 1) / SSIM_T;
  const long ntiles = (long)d.n * tiles_y * tiles_x;
  if (threadIdx.x < SSIM_K) {  // torchmetrics _gaussian: exp(-(dist/sigma)^2 / 2), normalised
    float s = 0.f, gv = 0.f;
    for (int i = 0; i < SSIM_K; ++i) {
      float dist = (float)(i - SSIM_R);
      float e = expf(-((dist / 1.5f) * (dist / 1.5f)) / 2.f);
      s += e;
      if (i == (int)threadIdx.x) gv = e;
    }
    g[threadIdx.x] = gv / s;
  }
  const double* stats = d.workspace + WS_STATS;
  const float dr = fmaxf((float)stats[P_PN_MAX] - (float)stats[P_PN_MIN], (float)stats[P_TN_MAX] - (float)stats[P_TN_MIN]);
  const float c1 = (0.01f * dr) * (0.01f * dr), c2 = (0.03f * dr) * (0.03f * dr);
  double part = 0.0;
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int b = (int)(tile / (tiles_y * tiles_x));
    const int r = (int)(tile - (long)b * tiles_y * tiles_x);
    const int oy0 = (r / tiles_x) * SSIM_T, ox0 = (r % tiles_x) * SSIM_T;  // cropped-output origin
    __syncthreads();
    for (int e = threadIdx.x; e < SSIM_IN * SSIM_IN; e += blockDim.x) {
      int iy = e / SSIM_IN, ix = e % SSIM_IN;
      int gy = oy0 + iy, gx = ox0 + ix;  // input row/col (crop offset cancels the window radius)
      float pn = 0.f, tn = 0.f;
      if (gy < d.h && gx < d.w) {  // normalised maps only: SSIM never sees the denormalised values
        long i = ((long)b * d.h + gy) * d.w + gx;
        if (d.mask[i] != 0.f) {
          pn = d.sr[i];
          tn = d.hr[i];
        }
      }
      sp[iy][ix] = pn;
      st[iy][ix] = tn;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < SSIM_IN * SSIM_T; e += blockDim.x) {
      int iy = e / SSIM_T, ox = e % SSIM_T;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, a4 = 0.f;
#pragma unroll
      for (int k = 0; k < SSIM_K; ++k) {
        float p = sp[iy][ox + k], q = st[iy][ox + k], w = g[k];
        a0 += w * p;
        a1 += w * q;
        a2 += w * (p * p);
        a3 += w * (q * q);
        a4 += w * (p * q);
      }
      hsum[0][iy][ox] = a0;
      hsum[1][iy][ox] = a1;
      hsum[2][iy][ox] = a2;
      hsum[3][iy][ox] = a3;
      hsum[4][iy][ox] = a4;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < SSIM_T * SSIM_T; e += blockDim.x) {
      int oy = e / SSIM_T, ox = e % SSIM_T;
      if (oy0 + oy >= oh || ox0 + ox >= ow) continue;
      float m[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < SSIM_K; ++k) {
        float w = g[k];
#pragma unroll
        for (int q = 0; q < 5; ++q) m[q] += w * hsum[q][oy + k][ox];
      }
      float mu_p2 = m[0] * m[0], mu_t2 = m[1] * m[1], mu_pt = m[0] * m[1];
      float s_p = m[2] - mu_p2, s_t = m[3] - mu_t2, s_pt = m[4] - mu_pt;
      float upper = 2.f * s_pt + c2, lower = s_p + s_t + c2;
      part += (double)(((2.f * mu_pt + c1) * upper) / ((mu_p2 + mu_t2 + c1) * lower));
    }
  }
  for (int o = 32; o > 0; o >>= 1) part += __shfl_down(part, o);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = part;
  __syncthreads();
  if (threadIdx.x == 0) d.workspace[WS_SSIM + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void __launch_bounds__(SSIM_BLOCKS) metrics_final_kernel(ClimsrMetricsDesc d, int ssim_blocks) {
  __shared__ double sh[SSIM_BLOCKS];
  sh[threadIdx.x] = (int)threadIdx.x < ssim_blocks ? d.workspace[WS_SSIM + threadIdx.x] : 0.0;
  __syncthreads();
  for (int o = SSIM_BLOCKS / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const double* s = d.workspace + WS_STATS;
  const double n = (double)d.n * d.h * d.w;
  double* out = d.out;
  for (int k = 0; k < 8; ++k) out[k] = s[P_ACC0 + k] / n;  // RegressionAccuracy: correct / total
  const double mse = s[P_SQ] / n;
  const double range = s[P_TD_MAX] - s[P_TD_MIN];           // PSNR(data_range=None): target max - min
  out[8] = (2.0 * log(range) - log(mse)) * (10.0 / log(10.0));
  out[9] = sh[0] / ((double)d.n * (d.h - 2 * SSIM_R) * (d.w - 2 * SSIM_R));
  out[10] = s[P_ABS] / n;       // MAE
  out[11] = mse;                // MSE
  out[12] = sqrt(mse);          // RMSE (MeanSquaredError(squared=False))
  out[13] = s[P_MAPE] / n;      // MAPE on the normalised maps
  out[14] = 2.0 * s[P_SMAPE] / n;
  const double mean_t = s[P_T] / n;  // R2Score: 1 - SS_res / (sum t^2 - sum t * mean t)
  out[15] = 1.0 - s[P_SQ] / (s[P_TT] - s[P_T] * mean_t);
  out[16] = s[P_L1N] / n;       // normalised L1 (`{prefix}/normalized_loss`, `{prefix}/loss`)
}

extern "C" size_t climsr_sr_metrics_workspace(void) { return (size_t)(WS_SSIM + SSIM_BLOCKS) * sizeof(double); }

extern "C" int climsr_sr_metrics(const ClimsrMetricsDesc* d, void* stream) {
  if (!d || !d->sr || !d->hr || !d->original || !d->mask || !d->workspace || !d->out || d->n <= 0 ||
      d->h < SSIM_K || d->w < SSIM_K || (d->method == 0 && (!d->min || !d->max)) || d->method < 0 || d->method > 2) {
    set_error("sr_metrics: bad args (h, w >= %d for the 11x11 SSIM window; min/max needed for minmax)", SSIM_K);
    return CLIMSR_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  const ClimsrMetricsDesc dd = *d;
  hipLaunchKernelGGL(metrics_partial_kernel, dim3(MET_BLOCKS), dim3(256), 0, s, dd);
  hipLaunchKernelGGL(metrics_stats_kernel, dim3(1), dim3(1024), 0, s, dd);
  const int oh = d->h - 2 * SSIM_R, ow = d->w - 2 * SSIM_R;
  long ntiles = (long)d->n * ((oh + SSIM_T - 1) / SSIM_T) * ((ow + SSIM_T - 1) / SSIM_T);
  int sb = (int)(ntiles < SSIM_BLOCKS ? ntiles : SSIM_BLOCKS);
  hipLaunchKernelGGL(ssim_kernel, dim3(sb), dim3(256), 0, s, dd);
  hipLaunchKernelGGL(metrics_final_kernel, dim3(1), dim3(SSIM_BLOCKS), 0, s, dd, sb);
  return check_launch("sr_metrics");
}

// ------------------------------------------------------------------------------------------
// RegressionAccuracy.update (climsr/metrics/regression_accuracy.py:15-19): count |p - t| <= eps in
// the inputs' float32 arithmetic; int64 counters (exact, order-independent).
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) regression_accuracy_kernel(const float* __restrict__ p, const float* __restrict__ t,
                                                                  long n, float eps, unsigned long long* counts) {
  unsigned long long c = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    c += (fabsf(p[i] - t[i]) <= eps) ? 1ull : 0ull;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(counts, c);
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(counts + 1, (unsigned long long)n);
}

extern "C" int climsr_regression_accuracy_update(const float* preds, const float* target, int64_t n, float eps, int64_t* counts,
                                                 void* stream) {
  if (!preds || !target || !counts || n < 0) {
    set_error("regression_accuracy: bad args");
    return CLIMSR_EINVAL;
  }
  if (n == 0) return 0;
  int blocks = (int)((n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024);
  hipLaunchKernelGGL(regression_accuracy_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, preds, target, (long)n, eps,
                     (unsigned long long*)counts);
  return check_launch("regression_accuracy");
}

// ------------------------------------------------------------------------------------------
// Inference output (inference.py:73-80): MinMaxScaler.denormalize of the SR map with the grid's float64
// min / max (numpy float64 arithmetic, one rounding to float32 at the end), NaN where the land mask is 0.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void denormalize_mask_kernel(const float* __restrict__ sr, const float* __restrict__ mask,
                                                               const double* __restrict__ mn, const double* __restrict__ mx,
                                                               double a, double b, double eps, long hw, long total,
                                                               float* __restrict__ out) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int t = (int)(i / hw);
  const double scale = __ddiv_rn(b - a, __dadd_rn(__dsub_rn(mx[t], mn[t]), eps));
  const double add = __dsub_rn(a, __dmul_rn(mn[t], scale));
  const float v = (float)__ddiv_rn(__dsub_rn((double)sr[i], add), scale);
  out[i] = (mask && mask[i] == 0.f) ? NAN : v;
}

extern "C" int climsr_denormalize_mask(const float* sr, const float* mask, const double* min, const double* max, double range_a,
                                       double range_b, int n, int64_t hw, float* out, void* stream) {
  if (!sr || !min || !max || !out || n <= 0 || hw <= 0) {
    set_error("denormalize_mask: bad args");
    return CLIMSR_EINVAL;
  }
  const long total = (long)n * hw;
  hipLaunchKernelGGL(denormalize_mask_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, sr, mask, min, max,
                     range_a, range_b, 1e-8, (long)hw, total, out);
  return check_launch("denormalize_mask");
}
