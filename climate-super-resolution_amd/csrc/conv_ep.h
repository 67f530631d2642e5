// Shared by the conv translation units (conv.hip, conv_dma.hip): the forward / data-gradient kernel arguments and
// the coalesced store epilogue (store_tile_lds) with its BatchNorm-partial helpers.
#pragma once
#include "common.h"

namespace climsr {
constexpr int TW = 16;  // output tile width (one MFMA N-fragment of pixels)
}  // namespace climsr
using namespace climsr;

// ------------------------------------------------------------------------------------------
// Forward / data-gradient kernel
// ------------------------------------------------------------------------------------------
struct FwdArgs {
  const uint16_t* x;
  const uint16_t* w;
  const float* bias;
  void* y;
  const void* res1;
  const void* res2;
  uint16_t* aux;
  int n, in_h, in_w, in_c, in_cs, in_co, up, ks, stride, pad, out_h, out_w, out_c, out_cs, out_co, cc;
  int tph, tpw, ccp, kcpad, nchunk, kpk, tiles_x, tiles_y;
  int act, out_mode, down2;
  float slope, alpha1, alpha2;
  int r1_cs, r1_co, r2_cs, r2_co;
  int res_f32;
  float beta1, beta2;
  int aux_cs, aux_co;
  float aux_scale;
  int lds_tab, lds_x;
  double* bn_part;  // EP 9: per-tile BatchNorm partial sums [tile][2][out_c] of the bf16 outputs (climsr_conv2d_fwd_bn_parts)
  int xgrp;         // > 0: 1-D grid in XCD-major (channel-block group, tile, channel block) order, xgrp blocks a group
  int stag_lo, stag_hi, stag_n;  // blocks [stag_lo, stag_hi) start stag_n x 2048 cycles late (conv_fwd_body, GEO 1)
  // EP 10: BatchNorm-backward partials of the stored data gradient (ClimsrEpilogue.bn_z ...) into bn_part
  const uint16_t* bz;
  int bz_cs;
  float bslope;
  const float *bmean, *brstd, *bgamma, *bbeta;
};

// Blocks are dealt round-robin over the 8 XCDs (blocks b and b + 8 share one, MI355X_MICROARCH.md 'Workgroup
// dispatch'; for speed only, nothing depends on it).  xcd_major(b, n) renumbers a grid of n so that each XCD's
// blocks form one contiguous index range (bijective for any n): blocks that read the same operand tiles and sit
// next to each other in that order share an L2 instead of fetching the tiles once per XCD.
__device__ __forceinline__ int xcd_major(int b, int n) {
  const int x = b & 7, j = b >> 3, q = n >> 3, r = n & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + j;
}

// Epilogue residual operands: 4 consecutive channels, bf16 (8 B) or fp32 (16 B), kept raw until use so
// that all loads of a round are in flight together.
__device__ __forceinline__ uint4 load_res4(const void* p, bool f32, long idx) {
  if (f32) return *(const uint4*)((const float*)p + idx);
  const uint2 v = *(const uint2*)((const uint16_t*)p + idx);
  return make_uint4(v.x, v.y, 0, 0);
}
__device__ __forceinline__ float res4_at(const uint4& r, bool f32, int i) {
  if (f32) return __uint_as_float(i == 0 ? r.x : i == 1 ? r.y : i == 2 ? r.z : r.w);
  const uint32_t w = (i < 2) ? r.x : r.y;
  return bf2f((uint16_t)((i & 1) ? (w >> 16) : w));
}
__device__ __forceinline__ float res_at(const void* p, bool f32, long idx) {
  return f32 ? ((const float*)p)[idx] : bf2f(((const uint16_t*)p)[idx]);
}
// v after bias (+ forward activation): apply res1 (residual, or activation-backward mask for act 3/4), res2
__device__ __forceinline__ float ep_res(float v, int act, float slope, bool has1, float r1, float alpha1, float beta1, bool has2,
                                        float r2, float alpha2, float beta2) {
  if (act == 3) v = r1 > 0.f ? v : v * slope;
  else if (act == 4) v = r1 > 0.f ? v : 0.f;
  else if (has1) v = v * alpha1 + beta1 * r1;
  if (has2) v = v * alpha2 + beta2 * r2;
  return v;
}

// RF: the epilogue may read fp32 residuals (then one output row per round, to stay within 256 registers)
// MV: staging vectors (16 B) per thread and stream held in registers per batch
// 8 consecutive channels of a residual / output operand (16 B bf16 or 32 B fp32)
struct Raw8 {
  uint4 lo, hi;
};
__device__ __forceinline__ Raw8 load8(const void* p, bool f32, long idx) {
  Raw8 r;
  if (f32) {
    r.lo = *(const uint4*)((const float*)p + idx);
    r.hi = *(const uint4*)((const float*)p + idx + 4);
  } else {
    r.lo = *(const uint4*)((const uint16_t*)p + idx);
    r.hi = make_uint4(0, 0, 0, 0);
  }
  return r;
}
// Branch-free epilogue operand loads: an optional operand (null pointer) gets a zero-record buffer resource,
// whose loads return 0 without touching memory, and lanes without a valid pixel load at offset 0 (their
// values are never used).  No branch around a load, so every load of a round is in flight together
// (hipcc waits vmcnt(0) at each load that sits under a condition, even a wave-uniform one).  Operand
// extents are < 4 GiB (checked on the host: climsr_conv2d_fwd).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t opt_rsrc(const void* p) { return buf_rsrc(p, p ? 0xFFFFFFFFu : 0u); }
__device__ __forceinline__ Raw8 load8b(__amdgpu_buffer_rsrc_t r, bool f32, long idx) {
  Raw8 v;
  if (f32) {
    v.lo = buf_load16(r, (uint32_t)(idx * 4));
    v.hi = buf_load16(r, (uint32_t)(idx * 4 + 16));
  } else {
    v.lo = buf_load16(r, (uint32_t)(idx * 2));
    v.hi = make_uint4(0, 0, 0, 0);
  }
  return v;
}
__device__ __forceinline__ uint2 buf_load8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  return make_uint2(v[0], v[1]);
}
__device__ __forceinline__ float raw8_at(const Raw8& r, bool f32, int i) {
  if (f32) {
    const uint4& q = i < 4 ? r.lo : r.hi;
    const int k = i & 3;
    return __uint_as_float(k == 0 ? q.x : k == 1 ? q.y : k == 2 ? q.z : q.w);
  }
  const int k = i >> 1;
  const uint32_t w = k == 0 ? r.lo.x : k == 1 ? r.lo.y : k == 2 ? r.lo.z : r.lo.w;
  return bf2f((uint16_t)((i & 1) ? (w >> 16) : w));
}
__device__ __forceinline__ uint4 pack8_bf16(const float* v, float scale) {
  uint4 o;
  o.x = (uint32_t)f2bf(scale * v[0]) | ((uint32_t)f2bf(scale * v[1]) << 16);
  o.y = (uint32_t)f2bf(scale * v[2]) | ((uint32_t)f2bf(scale * v[3]) << 16);
  o.z = (uint32_t)f2bf(scale * v[4]) | ((uint32_t)f2bf(scale * v[5]) << 16);
  o.w = (uint32_t)f2bf(scale * v[6]) | ((uint32_t)f2bf(scale * v[7]) << 16);
  return o;
}

// Store epilogue for a tile of fp32 results staged in LDS as [pixel][channel] (pitch ep floats): each lane
// owns 8 consecutive channels of one pixel, so global stores / residual loads are 16 B (bf16) or 32 B
// (fp32) per lane and 8 lanes cover a 64-channel pixel row (8 B per lane stores are issue-bound).
// npx pixels (pixel p -> output (oy0 + p / 16, ox0 + p % 16)), nch channels starting at co0.
// EP (epilogue specialisation, picked on the host only when the arguments match; 0 = every option a runtime
// flag): 1 = residual forward (bias, no activation, bf16 residual(s), bf16 output: RDB conv5, trunk_conv),
// 2 = fp32 data gradient (no bias / activation, fp32 residual(s), fp32 '=' output, optional bf16 aux: pull-x).
template <bool RF, int NPX, int NCH, int NLANE, int EP = 0>
__device__ __forceinline__ void store_tile_lds(const FwdArgs& a, const float* eb, int ep, int lane, int nimg, int oy0, int ox0,
                                               int co0, float* ssum = nullptr, float* ssq = nullptr) {
  constexpr int NG = NCH / 8, NIT = NPX * NG;
  // EP 3 = activation forward (bias + leaky relu / relu, bf16 out); 4 = activation backward (act' read from
  // the bf16 activation res1, no bias, bf16 out): the HR-resolution layers (conv_pw_kernel); 6 = activation
  // forward without bias (discriminator convs); 7 = plain fp32 '=' output (data gradients feeding a BN /
  // activation backward); 8 = plain bf16 output (pre-BN discriminator convs).
  const bool f1 = EP == 2 ? true : EP != 0 ? false : RF && (a.res_f32 & 1);
  const bool f2 = EP == 2 ? true : EP != 0 ? false : RF && ((a.res_f32 >> 1) & 1);
  const bool has_bias = (EP == 1 || EP == 3) ? true : EP != 0 ? false : a.bias != nullptr;
  // EP 9 = EP 8 + sums / sums of squares of the stored (bf16-rounded) values per lane (ssum / ssq [8]: the lane's
  // 8 channels, the same for all of its items when NCH / 8 divides NLANE)
  // EP 10 = EP 8 + BatchNorm-backward partials (ssum += d, ssq += d * xhat; d = stored value * lrelu'(BN(z)), z read
  // from a.bz at the output pixel: the layer's affine is recomputed as bn_stats_kernel MODE 2 does, bit for bit)
  const int act = (EP == 1 || EP == 2 || EP == 7 || EP == 8 || EP == 9 || EP == 10) ? 0 : a.act;
  const bool has1 = (EP == 1 || EP == 2 || EP == 4) ? true : EP != 0 ? false : a.res1 != nullptr;
  const bool has2 = (EP == 0 || EP == 1 || EP == 2) ? a.res2 != nullptr : false;
  const int out_mode = (EP == 2 || EP == 7) ? 1 : EP != 0 ? 0 : a.out_mode;
  const bool has_aux = (EP == 0 || EP == 2) ? a.aux != nullptr : false;
  const bool vec = EP != 0 || ((a.out_c & 7) == 0 && ((a.out_cs | a.out_co) & 7) == 0 && (!a.res1 || ((a.r1_cs | a.r1_co) & 7) == 0) &&
                               (!a.res2 || ((a.r2_cs | a.r2_co) & 7) == 0) && (!a.aux || ((a.aux_cs | a.aux_co) & 7) == 0));
  constexpr int IB = RF ? 2 : 4;  // items per round: their global loads are in flight together
  const __amdgpu_buffer_rsrc_t rr1 = opt_rsrc(EP == 10 ? (const void*)a.bz : has1 ? a.res1 : nullptr),
                               rr2 = opt_rsrc(has2 ? a.res2 : nullptr), rry = opt_rsrc(out_mode == 2 ? a.y : nullptr);
  float bmu[8], brs[8], bsc[8], bsh[8];  // EP 10: the lane's 8 channels (the same for all of its items, as for EP 9)
  if constexpr (EP == 10) {
    static_assert(NLANE % NG == 0, "EP 10: one channel group per lane");
    const int c = co0 + (lane % NG) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      bmu[i] = a.bmean[c + i];
      brs[i] = a.brstd[c + i];
      bsc[i] = a.bgamma[c + i] * brs[i];
      bsh[i] = a.bbeta[c + i] - bmu[i] * bsc[i];
    }
  }
#pragma unroll
  for (int base = 0; base < (NIT + NLANE - 1) / NLANE; base += IB) {
    Raw8 r1[IB], r2[IB], old[IB];
    int pidxs[IB];
    bool ok[IB];
#pragma unroll
    for (int j = 0; j < IB; ++j) {
      const int it = (base + j) * NLANE + lane;
      const int pl = it / NG, cg = it - (it / NG) * NG;
      const int oy = oy0 + pl / 16, ox = ox0 + (pl & 15);
      const int co = co0 + cg * 8;
      ok[j] = it < NIT && oy < a.out_h && ox < a.out_w && co < a.out_c;
      pidxs[j] = ((nimg * a.out_h + oy) * a.out_w + ox);
      const bool ld = ok[j] && vec && co + 7 < a.out_c;  // else the values are unused
      const long pidx = ld ? pidxs[j] : 0;
      const int c = ld ? co : 0;
      // (EP 0: unconditional, a null operand reads zeros; EP > 0: compile-time known)
      if (EP == 10) r1[j] = load8b(rr1, false, pidx * a.bz_cs + c);  // the layer's z
      else if (EP == 0 || has1) r1[j] = load8b(rr1, f1, pidx * a.r1_cs + (ld ? a.r1_co : 0) + c);
      else r1[j].lo = r1[j].hi = make_uint4(0, 0, 0, 0);
      if (EP == 0 || has2) r2[j] = load8b(rr2, f2, pidx * a.r2_cs + (ld ? a.r2_co : 0) + c);
      else r2[j].lo = r2[j].hi = make_uint4(0, 0, 0, 0);
      if (EP == 0 || out_mode == 2) old[j] = load8b(rry, true, pidx * a.out_cs + (ld ? a.out_co : 0) + c);
      else old[j].lo = old[j].hi = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < IB; ++j) {
      if (!ok[j]) continue;
      const int it = (base + j) * NLANE + lane;
      const int pl = it / NG, cg = it - (it / NG) * NG;
      const int co = co0 + cg * 8;
      const long pidx = pidxs[j];
      const float4 s0 = *(const float4*)(eb + pl * ep + cg * 8), s1 = *(const float4*)(eb + pl * ep + cg * 8 + 4);
      float v[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      const long ob = pidx * a.out_cs + a.out_co + co;
      if (vec && co + 7 < a.out_c) {
        float4 b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0;
        if (has_bias) {
          b0 = *(const float4*)(a.bias + co);
          b1 = *(const float4*)(a.bias + co + 4);
        }
        const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i)
          v[i] = ep_res(act_apply(v[i] + bb[i], act, a.slope), act, a.slope, has1, raw8_at(r1[j], f1, i), a.alpha1, a.beta1, has2,
                        raw8_at(r2[j], f2, i), a.alpha2, a.beta2);
        if (out_mode == 0) {
          const uint4 pk = pack8_bf16(v, 1.f);
          *(uint4*)((uint16_t*)a.y + ob) = pk;
          if constexpr (EP == 9) {
            Raw8 rr;
            rr.lo = pk;
            rr.hi = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const float r = raw8_at(rr, false, i);
              ssum[i] += r;
              ssq[i] = fmaf(r, r, ssq[i]);
            }
          }
          if constexpr (EP == 10) {
            Raw8 rr;
            rr.lo = pk;
            rr.hi = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const float r = raw8_at(rr, false, i), z = raw8_at(r1[j], false, i);
              const float d = fmaf(z, bsc[i], bsh[i]) > 0.f ? r : r * a.bslope;
              ssum[i] += d;
              ssq[i] = fmaf(d, (z - bmu[i]) * brs[i], ssq[i]);
            }
          }
        } else {
          float o[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] = v[i] + (out_mode == 2 ? raw8_at(old[j], true, i) : 0.f);
          *(float4*)((float*)a.y + ob) = make_float4(o[0], o[1], o[2], o[3]);
          *(float4*)((float*)a.y + ob + 4) = make_float4(o[4], o[5], o[6], o[7]);
        }
        if (has_aux) *(uint4*)(a.aux + pidx * a.aux_cs + a.aux_co + co) = pack8_bf16(v, a.aux_scale);
      } else if (EP == 0) {  // scalar tail (channel counts / slices not multiples of 8)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (co + i >= a.out_c) continue;
          const float r1v = a.res1 ? res_at(a.res1, f1, pidx * a.r1_cs + a.r1_co + co + i) : 0.f;
          const float r2v = a.res2 ? res_at(a.res2, f2, pidx * a.r2_cs + a.r2_co + co + i) : 0.f;
          const float x = ep_res(act_apply(v[i] + (a.bias ? a.bias[co + i] : 0.f), a.act, a.slope), a.act, a.slope,
                                 a.res1 != nullptr, r1v, a.alpha1, a.beta1, a.res2 != nullptr, r2v, a.alpha2, a.beta2);
          if (a.out_mode == 0) ((uint16_t*)a.y)[ob + i] = f2bf(x);
          else if (a.out_mode == 2) ((float*)a.y)[ob + i] += x;
          else ((float*)a.y)[ob + i] = x;
          if (a.aux) a.aux[pidx * a.aux_cs + a.aux_co + co + i] = f2bf(a.aux_scale * x);
        }
      }
    }
  }
}

// BatchNorm partials of one 16x16-pixel x 64-channel output tile (EP 9): the lanes with equal lane % 8 own the same
// 8 channels (store_tile_lds items), so three xor-shuffles (8, 16, 32) give each wave's sums in lanes 0..7; the 4
// row waves meet in LDS and wave 0 writes fp64 part[tile][0 / 1][co0 + ch] -- fixed order, deterministic.  Every
// wave of the workgroup calls it (`live` = the wave stored rows); red = 2 KB of LDS no wave reads any more.
__device__ __forceinline__ void bn_tile_partials(const FwdArgs& a, float* ssum, float* ssq, bool live, int wave4, int lane, long tile,
                                                 int co0, float* red) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (!live) { ssum[i] = 0.f; ssq[i] = 0.f; }
#pragma unroll
    for (int m = 8; m < 64; m <<= 1) {
      ssum[i] += __shfl_xor(ssum[i], m);
      ssq[i] += __shfl_xor(ssq[i], m);
    }
  }
  // LDS-only barriers: __syncthreads()' release fence would also wait for this wave's output stores
  lds_barrier();  // every wave's epilogue reads of the staging region are done
  if (live && lane < 8) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[wave4 * 128 + lane * 8 + i] = ssum[i];
      red[wave4 * 128 + 64 + lane * 8 + i] = ssq[i];
    }
  }
  lds_barrier();
  if (threadIdx.x < 64) {
    const int ch = threadIdx.x;
    float ts = 0.f, tq = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      ts += red[w * 128 + ch];
      tq += red[w * 128 + 64 + ch];
    }
    double* out = a.bn_part + tile * 2 * a.out_c;
    out[co0 + ch] = (double)ts;
    out[a.out_c + co0 + ch] = (double)tq;
  }
}


// LDS-DMA conv (conv_dma.hip): 32-row output tiles; launches conv_fwd_dma_kernel<ep, a.res_f32 != 0> (EP 0, 1, 2, 3,
// 4, 6, 7, 8) over the grid a.xgrp / a.tiles_y describe; CLIMSR_EINVAL for an EP it has no kernel for
namespace climsr {
constexpr int DMA_TH = 32;
int fwd_dma_launch(int ep, const FwdArgs& a, int ncob, hipStream_t s);
// stride-2 3x3 forward, plain bf16 out (+ BatchNorm partials when a.bn_part), 16 x 16 tiles (a.tiles_x / tiles_y)
int fwd_s2_dma_launch(const FwdArgs& a, hipStream_t s);
}  // namespace climsr
