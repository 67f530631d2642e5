/*
 * climsr_hip.h — C ABI of libclimsr_hip.so, the MI355X (gfx950) hot path of
 * xultaeculcis/climate-super-resolution (ESRGAN generator / discriminator forward + backward,
 * losses, optimiser).
 *
 * The reference has no native boundary: every op below replaces a stock PyTorch op that the
 * reference calls from Python (cited per entry point as reference file:line).  The Python
 * mirror of the reference's module/step API (climsr_amd.*) binds these with ctypes
 * (climate-super-resolution_amd/_lib.py); INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - Every pointer is a DEVICE pointer; the caller allocates every output and workspace (the
 *    library never allocates or frees).  Activations are NHWC; `cstride` = channels per pixel of
 *    the buffer, `coff` = first channel used, so channel slices of one buffer (the RDB dense
 *    concatenation, esrgan.py:34-37) are addressed without copies.
 *  - bf16 tensors are raw uint16 bit patterns (bfloat16); accumulation is fp32 (MFMA).
 *  - All calls are asynchronous on `stream` (a hipStream_t passed as void*), never synchronise,
 *    and are graph-capturable.
 *  - Return 0 on success, CLIMSR_EINVAL (-1) for a bad shape/argument, CLIMSR_EHIP (-2) when
 *    the launch failed; climsr_last_error() returns a thread-local message.
 */
#ifndef CLIMSR_HIP_H
#define CLIMSR_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CLIMSR_OK 0
#define CLIMSR_EINVAL (-1)
#define CLIMSR_EHIP (-2)

/* Geometry of one 2-D convolution (square kernel) over NHWC buffers. */
typedef struct ClimsrConvDesc {
  int32_t n;                   /* batch */
  int32_t in_h, in_w;          /* SOURCE spatial size (before the nearest upsample) */
  int32_t in_c;                /* channels consumed (multiple of 8) */
  int32_t in_cstride, in_coff; /* input buffer channels per pixel / first channel (multiples of 8) */
  int32_t up;                  /* 1, or 2 = nearest x2 upsample on load (esrgan.py:94,97: src = dst >> 1) */
  int32_t ks, stride, pad;     /* kernel size (1,3,5,9), stride (1,2), zero padding */
  int32_t out_h, out_w;        /* output spatial size */
  int32_t out_c;               /* real output channels */
  int32_t out_cstride, out_coff;
  int32_t cc;                  /* channel chunk of the packed weight layout (climsr_conv_chunk) */
} ClimsrConvDesc;

/* Fused epilogue: v = acc + bias; v = act(v); v = v*alpha1 + res1; v = v*alpha2 + res2; store. */
typedef struct ClimsrEpilogue {
  int32_t act;                  /* 0 none, 1 leaky relu(slope), 2 relu */
  float slope;
  float alpha1;                 /* used when res1 != NULL */
  const void* res1;             /* bf16 NHWC, same pixels as the output */
  int32_t res1_cstride, res1_coff;
  float alpha2;
  const void* res2;
  int32_t res2_cstride, res2_coff;
  int32_t out_mode;             /* 0 bf16 store, 1 f32 store, 2 f32 accumulate (+=) */
  int32_t down2;                /* 1: sum 2x2 output pixels into out[y/2][x/2] (dgrad of a nearest x2 upsample) */
} ClimsrEpilogue;

const char* climsr_last_error(void);
int climsr_version(void);

/* Channel chunk used by the packed weight layout for a conv with `in_c` input channels. */
int climsr_conv_chunk(int in_c, int ks, int out_c);
/* Number of bf16 elements per output-channel row of the packed weight (nchunk * Kc_pad). */
int climsr_conv_packed_k(int in_c, int ks, int cc);

/* Rows (padded output channels) of the packed weight for a conv with out_c outputs. */
int climsr_conv_packed_rows(int out_c);
/* Pack fp32 OIHW weights [out_c][in_c_real][ks][ks] into the bf16 MFMA layout
 * [climsr_conv_packed_rows(out_c)][packed_k].  transpose_flip=1 packs the data-gradient weights
 * W'[ci][co][ks-1-ky][ks-1-kx] (then out_c/in_c name the TRANSPOSED conv).
 * Replaces the implicit weight handling of nn.Conv2d (esrgan.py:22-26). */
int climsr_pack_conv_weight(const float* w, int out_c, int in_c, int in_c_real, int out_c_real, int ks, int cc,
                            int transpose_flip, uint16_t* wpk, void* stream);

/* One pack job of climsr_pack_conv_weights_batched (fields as in climsr_pack_conv_weight). */
typedef struct ClimsrPackDesc {
  const float* w;
  uint16_t* out;
  int32_t out_c, in_c, in_c_real, out_c_real, ks, cc, tflip, reserved;
} ClimsrPackDesc;
/* Pack many convs in one launch; `descs` is a DEVICE array of ndesc descriptors, max_elems the
 * largest packed size (rows*packed_k) among them.  Used after every optimiser step. */
int climsr_pack_conv_weights_batched(const ClimsrPackDesc* descs, int ndesc, int64_t max_elems, void* stream);

/* Implicit-GEMM convolution on MFMA (bf16 in, fp32 accumulate), fused epilogue.
 * Forward of nn.Conv2d (esrgan.py:22-26,72-83; srcnn.py:9-11; rfb_esrgan.py:28-52) and, with
 * transpose_flip weights, its data gradient (stride 1). */
int climsr_conv2d_fwd(const ClimsrConvDesc* d, const uint16_t* x, const uint16_t* wpk, const float* bias,
                      const ClimsrEpilogue* ep, void* y, void* stream);

/* Weight (+ bias) gradient partials: partial[split][out_c_pad16][in_c*ks*ks] (OIHW order) and
 * bias_partial[split][out_c_pad16].  dz: bf16 NHWC [n][out_h][out_w][dz_cstride]. */
int climsr_conv2d_wgrad(const ClimsrConvDesc* d, const uint16_t* x, const uint16_t* dz, int dz_cstride,
                        float* partial, float* bias_partial, int nsplit, void* stream);
/* Sum the split partials into OIHW fp32 grads (accumulate=1: +=).  bias_grad may be NULL. */
int climsr_conv2d_wgrad_reduce(const float* partial, const float* bias_partial, int nsplit, int out_c, int in_c_real,
                               int in_c, int ks, float* wgrad, float* bias_grad, int accumulate, void* stream);
/* Split count and workspace floats climsr_conv2d_wgrad needs for this geometry. */
int climsr_conv2d_wgrad_splits(const ClimsrConvDesc* d);
size_t climsr_conv2d_wgrad_workspace(const ClimsrConvDesc* d, int nsplit);

/* dz[p][c] = bf16(scale * g[p][goff+c] * act'(y[p][yoff+c])) for c < c_real, 0 for c_real <= c < dz_cstride.
 * act: 0 none, 1 leaky relu(slope) (derivative taken from the sign of the OUTPUT y, valid since
 * LeakyReLU/ReLU preserve sign), 2 relu.  g is fp32.  Backward of nn.LeakyReLU / F.relu. */
int climsr_act_grad(int64_t npix, int c_real, const float* g, int g_cstride, int g_coff, const uint16_t* y,
                    int y_cstride, int y_coff, int act, float slope, float scale, uint16_t* dz, int dz_cstride,
                    void* stream);

/* NCHW fp32 -> NHWC bf16 (pad channels with 0): dst[n][h][w][coff+c] = src[n][c][h][w]. */
int climsr_nchw_to_nhwc_bf16(const float* src, int n, int c, int h, int w, uint16_t* dst, int cstride, int coff,
                             void* stream);
/* NHWC (bf16 or f32) -> NCHW fp32. */
int climsr_nhwc_to_nchw_f32(const void* src, int src_is_bf16, int n, int c, int h, int w, int cstride, int coff,
                            float* dst, void* stream);
/* y[p][c] (+)= x[p][c] elementwise fp32 over channel slices (init / residual gradient routing). */
int climsr_axpby_f32(int64_t npix, int c, float a, const float* x, int x_cstride, int x_coff, float b,
                     float* y, int y_cstride, int y_coff, void* stream);

/* Residual-dense-block backward prologue (esrgan.py:38,54) over npix pixels of [npix][dc] fp32
 * gradient buffers: save_skip: gskip = gx[:, :nf]; gy[:, :nf] = a_o*gx[:, :nf] (+ gskip if add_skip);
 * gy[:, nf:] = 0; dz[:, :nf] = bf16(0.2*a_o*gx[:, :nf]) (conv5's output gradient). */
int climsr_rdb_bwd_init(int64_t npix, int nf, int dc, const float* gx, float* gy, float* gskip, uint16_t* dz, float a_o,
                        int save_skip, int add_skip, void* stream);

/* L1Loss (mean) forward: out[0] = mean|a-b| (deterministic two-pass tree, fp64 partials).
 * workspace >= 1024 doubles.  torch.nn.L1Loss (task.py:141, pl_gan.py:20). */
int climsr_l1_loss(const float* a, const float* b, int64_t n, double* workspace, float* out, void* stream);
/* L1Loss backward: ga = gscale[0] * sign(a-b) / n. */
int climsr_l1_loss_grad(const float* a, const float* b, int64_t n, const float* gscale, float* ga, void* stream);

/* Device-side OneCycleLR(cos, beta1 cycling) + AdamW bias corrections (torch semantics),
 * state[0] = optimizer step count (as double) incremented here, state[1] = scheduler step.
 * hp out: {lr, beta1, beta2, eps, wd, step_size=lr/bc1, bc2_sqrt, 0}. */
int climsr_adamw_hparams(double* state, int total_steps, double max_lr, double pct_start, double div_factor,
                         double final_div_factor, double beta2, double eps, double wd, float* hp, void* stream);
/* Fused AdamW over flat fp32 buffers (conf/optimizers/adamw.yaml). */
int climsr_adamw_step(int64_t n, float* p, const float* g, float* m, float* v, const float* hp, void* stream);

#ifdef __cplusplus
}
#endif
#endif
