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
  int32_t up;                  /* 1; 2 = nearest x2 upsample on load (esrgan.py:94,97: src = dst >> 1);
                                  -2 = zero-insertion x2 (src = dst >> 1 for even dst, else 0): data gradient
                                  of a stride-2 conv (rfb_esrgan.py:30-50), forward kernel only */
  int32_t ks, stride, pad;     /* kernel size (1,3,5,9), stride (1,2), zero padding */
  int32_t out_h, out_w;        /* output spatial size */
  int32_t out_c;               /* real output channels */
  int32_t out_cstride, out_coff;
  int32_t cc;                  /* channel chunk of the packed weight layout (climsr_conv_chunk) */
} ClimsrConvDesc;

/* Fused epilogue: v = acc + bias; v = act(v); v = v*alpha1 + beta1*res1; v = v*alpha2 + beta2*res2; store v
 * (and, if aux != NULL, also aux = bf16(aux_scale * v)).
 * act 3 / 4 are activation BACKWARDS: v *= act'(res1) for a leaky relu / relu whose OUTPUT is res1 (the
 * derivative is read from its sign); res1 is then a mask source, not a residual. */
typedef struct ClimsrEpilogue {
  int32_t act;                  /* 0 none, 1 leaky relu(slope), 2 relu, 3 leaky relu backward, 4 relu backward */
  float slope;
  float alpha1;                 /* used when res1 != NULL */
  const void* res1;             /* bf16 (or fp32, res_f32 bit 0) NHWC, same pixels as the output */
  int32_t res1_cstride, res1_coff;
  float alpha2;
  const void* res2;             /* bf16 (or fp32, res_f32 bit 1) */
  int32_t res2_cstride, res2_coff;
  int32_t out_mode;             /* 0 bf16 store, 1 f32 store, 2 f32 accumulate (+=) */
  int32_t down2;                /* 1: sum 2x2 output pixels into out[y/2][x/2] (dgrad of a nearest x2 upsample); then no
                                   bias / forward act / residual, act 3/4 read res1 at the half-resolution pixel */
  int32_t res_f32;              /* bit 0: res1 is fp32, bit 1: res2 is fp32 */
  float beta1, beta2;           /* residual scales (1 for a plain residual add) */
  int32_t aux_cstride;
  void* aux;                    /* optional second output, bf16 NHWC, same pixels */
  int32_t aux_coff;
  float aux_scale;
  double* bn_part;              /* optional (plain bf16 output only): per-tile BatchNorm partials [tiles][2][out_c] (sum, sum of
                                   squares of the stored bf16 values) for climsr_bn_forward_parts; tiles and support from
                                   climsr_conv2d_fwd_bn_parts */
  /* BatchNorm-backward partials instead (bn_part and bn_z set; a data gradient whose output is dL/da of a BatchNorm +
     LeakyReLU(bn_slope) layer a = lrelu(BN(z))): bn_part[tile][0][c] = sum of d, [tile][1][c] = sum of d * xhat over the
     tile, d = out * lrelu'(z * gamma*rstd + (beta - mean*gamma*rstd)) with out bf16-rounded as stored, xhat = (z - mean) *
     rstd -- the statistics climsr_bn_backward's own pass would compute (rfb_esrgan.py:32-50's BatchNorm2d backward);
     finish with climsr_bn_backward_parts.  z: bf16 NHWC over the output's pixels, channel stride bn_z_cstride. */
  const uint16_t* bn_z;
  int32_t bn_z_cstride;
  float bn_slope;
  const float* bn_mean;
  const float* bn_rstd;
  const float* bn_gamma;
  const float* bn_beta;
  /* optional (the 64 -> 64 3x3 register-resident conv, climsr_conv2d_fwd_ch_parts > 0; fp32 or bf16 output): channel
     sums of the output values before any bf16 rounding, ch_part[row][out_c] fp32: one row per tile, the tiles of one
     image contiguous; with one image (n = 1) one row per workgroup of the launch instead (its tiles' sums, added in a
     fixed order) -- the global average pool of RCAN's channel attention (rcan.py:50-69) without re-reading the output; finish with climsr_channel_attention_parts */
  float* ch_part;
  /* 1: a 2x2 / stride-2 max pool of the (biased, activated) output is what gets stored: out[y/2][x/2] of the
     (out_h/2) x (out_w/2) image (even out_h / out_w; bf16 out, no residual / aux / BatchNorm / channel sums) -- VGG19's
     conv + ReLU + MaxPool2d (perceptual.py:16) without the full-size activation.  climsr_conv2d_fwd_pool_ok tells which
     convs have such a kernel. */
  int32_t pool2;
} ClimsrEpilogue;

/* rows of ClimsrEpilogue.ch_part for this conv and epilogue (tiles; workgroups when n = 1), 0 when its kernel cannot
 * emit them; the rows of one image are *tiles_per_image consecutive rows */
int64_t climsr_conv2d_fwd_ch_parts(const ClimsrConvDesc* d, const ClimsrEpilogue* ep, int32_t* tiles_per_image);
/* 1 when climsr_conv2d_fwd has a kernel for this conv with ep->pool2 = 1 (the 64 -> 64 register-resident conv, or the
 * LDS-DMA 3x3 conv with bias + activation), else 0 (store the full output and pool it with climsr_maxpool2_bf16). */
int climsr_conv2d_fwd_pool_ok(const ClimsrConvDesc* d, const ClimsrEpilogue* ep);

const char* climsr_last_error(void);
int climsr_version(void);

/* Channel chunk used by the packed weight layout for a conv with `in_c` input channels: stride 1 (and
 * every data gradient of a stride-1 conv); _ex takes the stride (a stride-2 conv and its data gradient,
 * which runs over the zero-inserted gradient, use stride 2). */
int climsr_conv_chunk(int in_c, int ks, int out_c);
int climsr_conv_chunk_ex(int in_c, int ks, int out_c, int stride);
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

/* "Pull" data-gradient weights of a residual dense block (esrgan.py:17-38).  The gradient of one
 * channel group of the dense concatenation (x, x1..x4) collects the transposed convs of EVERY later conv
 * that reads it; with the output gradients of those convs stored side by side (dZ1|dZ2|dZ3|dZ4|dZ5) the
 * sum is ONE conv over a contiguous channel suffix.  This packs its weights in the climsr_conv2d_fwd
 * layout: out row co (group channel ci_off+co), input channel c of segment s (the conv seg_w[s], seg_oc[s]
 * outputs, seg_ic[s] inputs): W_s[c - start_s][ci_off + co][ks-1-ky][ks-1-kx]. */
typedef struct ClimsrPullPackDesc {
  uint16_t* out;
  const float* seg_w[5];
  int32_t seg_oc[5];
  int32_t seg_ic[5];
  int32_t nseg, out_c, in_c, ks, cc, ci_off;
} ClimsrPullPackDesc;
int climsr_pack_pull_weights_batched(const ClimsrPullPackDesc* descs, int ndesc, int64_t max_elems, void* stream);

/* The four 16-output 3x3 convs of a residual dense block as one row-streaming launch (esrgan.py:22-37):
 * level L (1..4) reads [base (64 ch at boff) | outputs of levels 1..L-1] and writes 16 bf16 channels at
 * out[.., ooff[L-1]].  Forward: act 1 (leaky relu, bias[L-1]) = conv1..conv4 writing x1..x4 into the dense
 * buffer; pull backward: act 3 (leaky-relu derivative read from mask[.., moff[L-1]], no bias) = pull4..pull1
 * writing dZ4..dZ1.  wt[L-1]: bf16 [16][9*KP] with k = tap*KP + channel, KP = climsr_rdb_chain_kp(L), channel
 * order base | out1 | out2 | out3 (pack with climsr_pack_conv_weights_batched / _pull_weights_batched, cc = KP). */
typedef struct ClimsrChainDesc {
  const uint16_t* base;
  int32_t bcs, boff;
  uint16_t* out;
  int32_t ocs;
  int32_t ooff[4];
  const uint16_t* wt[4];
  const float* bias[4];
  const uint16_t* mask;
  int32_t mcs;
  int32_t moff[4];
  int32_t act;
  float slope;
  int32_t n, h, w;
} ClimsrChainDesc;
int climsr_rdb_chain(const ClimsrChainDesc* d, void* stream);
/* rocprof name of the kernel climsr_rdb_chain launches for d (nothing is launched; "" if invalid): widths 16 / 32 / 48 /
 * 64 run the level-per-wave kernel, any other width the column-windowed one */
const char* climsr_rdb_chain_kernel(const ClimsrChainDesc* d);
int climsr_rdb_chain_kp(int level);

/* Implicit-GEMM convolution on MFMA (bf16 in, fp32 accumulate), fused epilogue.
 * Forward of nn.Conv2d (esrgan.py:22-26,72-83; srcnn.py:9-11; rfb_esrgan.py:28-52) and, with
 * transpose_flip weights, its data gradient (stride 1). */
int climsr_conv2d_fwd(const ClimsrConvDesc* d, const uint16_t* x, const uint16_t* wpk, const float* bias,
                      const ClimsrEpilogue* ep, void* y, void* stream);
/* Number of BatchNorm partial rows (tiles) climsr_conv2d_fwd writes to ep->bn_part for this conv (no bias), or 0 when
 * its dispatch cannot produce them (then bn_part must be NULL). */
int64_t climsr_conv2d_fwd_bn_parts(const ClimsrConvDesc* d, const ClimsrEpilogue* ep);
/* Name of the kernel climsr_conv2d_fwd launches for these arguments (as rocprof reports it; "" if invalid).
 * Launches nothing; used to label per-kernel timings and PMC traffic. */
const char* climsr_conv2d_fwd_kernel(const ClimsrConvDesc* d, const float* bias, const ClimsrEpilogue* ep);
/* Dry-run kernel-name queries (profiler labels straight from the dispatch; nothing is launched): the weight-gradient
 * kernel climsr_conv2d_wgrad would launch for d (with climsr_conv2d_wgrad_splits(d) splits), and the data-gradient
 * stencil climsr_dgrad_single_output would launch for (ks, c, act).  "" if the arguments are unsupported. */
const char* climsr_conv2d_wgrad_kernel(const ClimsrConvDesc* d);
const char* climsr_dgrad_single_output_kernel(int ks, int c, int act);

/* Weight (+ bias) gradient partials (d->in_c may be 4 = "at most 4 real input channels", which packs
 * 4 taps x 4 channels per MFMA fragment; the input buffer still has a multiple-of-8 channel stride): partial[split][out_c_pad16][in_c*ks*ks] (OIHW order) and
 * bias_partial[split][out_c_pad16].  dz: bf16 NHWC [n][out_h][out_w][dz_cstride]. */
/* Data gradient of a stride-1 'same' conv with ONE output channel (conv_last esrgan.py:99, srcnn.conv3
 * srcnn.py:17), replacing their nn.Conv2d backward: out[q][c] = act'(res1[q][c]) * sum_{ky,kx} w[c][ky][kx] *
 * dz[q - (ky, kx) + pad], bf16 NHWC in / out (channel stride / offset), fp32 OIHW weight [1][c][ks][ks],
 * ks 3 or 5, c 32 or 64, act 0 (none), 3 (leaky-relu derivative, slope) or 4 (relu derivative)
 * taken from the bf16 activation res1.  Async on `stream`. */
int climsr_dgrad_single_output(int n, int h, int w, int ks, int pad, const uint16_t* dz, int dz_cstride, int dz_coff,
                               const float* weight, int c, int act, float slope, const uint16_t* res1, int res1_cstride,
                               int res1_coff, uint16_t* out, int out_cstride, int out_coff, void* stream);
/* Forward of a stride-1 'same' conv with ONE input channel (the RFB discriminator's features.0, rfb_esrgan.py:28:
 * 1 -> 64, 3x3), replacing its nn.Conv2d forward: out[q][c] = act(sum_{ky,kx} w[c][0][ky][kx] * x[q + (ky,kx) - pad]
 * + bias[c]); x = channel x_coff of a bf16 NHWC buffer, out bf16 NHWC; fp32 OIHW weight [c][1][ks][ks], bias
 * optional; ks 3 or 5, c 32 or 64, act 0 / 1 (leaky relu, slope) / 2 (relu). */
int climsr_conv_single_input(int n, int h, int w, int ks, int pad, const uint16_t* x, int x_cstride, int x_coff,
                             const float* weight, const float* bias, int c, int act, float slope, uint16_t* out,
                             int out_cstride, int out_coff, void* stream);
int climsr_conv2d_wgrad(const ClimsrConvDesc* d, const uint16_t* x, const uint16_t* dz, int dz_cstride,
                        float* partial, float* bias_partial, int nsplit, void* stream);
/* Sum the split partials into OIHW fp32 grads (accumulate=1: +=).  bias_grad may be NULL. */
int climsr_conv2d_wgrad_reduce(const float* partial, const float* bias_partial, int nsplit, int out_c, int in_c_real,
                               int in_c, int ks, float* wgrad, float* bias_grad, int accumulate, void* stream);
/* One conv of a row-sliced wgrad reduction: output channels = partial rows [row0, row0+out_c), inputs =
 * the first in_c_real*ks*ks columns of each row; wgrad OIHW fp32, bias_grad may be NULL. */
typedef struct ClimsrReduceDesc {
  float* wgrad;
  float* bias_grad;
  int32_t row0, out_c, in_c_real, reserved;
} ClimsrReduceDesc;
/* Sum the split partials of ONE climsr_conv2d_wgrad call (partial [nsplit][co_rows][kw]) into several
 * convs at once (descs: DEVICE array; max_elems = largest out_c*in_c_real*ks*ks + out_c).  Used for the
 * residual dense block, whose five weight gradients are one GEMM over the side-by-side conv output
 * gradients (esrgan.py:22-26). */
int climsr_conv2d_wgrad_reduce_rows(const float* partial, const float* bias_partial, int nsplit, int co_rows, int kw, int ks,
                                    const ClimsrReduceDesc* descs, int ndesc, int64_t max_elems, int accumulate, void* stream);
/* Split count and workspace floats climsr_conv2d_wgrad needs for this geometry. */
int climsr_conv2d_wgrad_splits(const ClimsrConvDesc* d);
size_t climsr_conv2d_wgrad_workspace(const ClimsrConvDesc* d, int nsplit);

/* dz[p][c] = bf16(scale * g[p][goff+c] * act'(y[p][yoff+c])) for c < c_real, 0 for c_real <= c < dz_cstride.
 * act: 0 none, 1 leaky relu(slope) (derivative taken from the sign of the OUTPUT y, valid since
 * LeakyReLU/ReLU preserve sign), 2 relu.  g is fp32.  Backward of nn.LeakyReLU / F.relu. */
int climsr_act_grad(int64_t npix, int c_real, const float* g, int g_cstride, int g_coff, const uint16_t* y,
                    int y_cstride, int y_coff, int act, float slope, float scale, uint16_t* dz, int dz_cstride,
                    void* stream);

/* Up to 8 fp32 image planes -> a bf16 NHWC buffer of exactly 8 channels per pixel (channel k = plane k, zeros where
 * p[k] is NULL), one 16 B store per pixel: the padded inputs of the networks (esrgan.py:89 lr + srcnn.py:13 elevation /
 * mask concatenation, rfb_esrgan.py:28 input, perceptual.py:26-31 torch.cat([x, x, x])).  Plane k of image b is
 * p[k] + b * img_stride[k] (elements), h*w contiguous fp32 values. */
typedef struct ClimsrPlanes8 {
  const float* p[8];
  int64_t img_stride[8];
} ClimsrPlanes8;
int climsr_pack_planes_nhwc8_bf16(const ClimsrPlanes8* planes, int n, int h, int w, uint16_t* dst, void* stream);
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
/* The same update, also writing bf16(p[mirror_lo + i]) to mirror[i] for i < mirror_n (the bf16 MFMA copy of a
 * weight inside the flat buffer: the RFB discriminator's fc.0, rfb_esrgan.py:56-61). */
int climsr_adamw_step_mirror(int64_t n, float* p, const float* g, float* m, float* v, const float* hp, int64_t mirror_lo,
                             int64_t mirror_n, uint16_t* mirror, void* stream);
/* ---------------- discriminator / perceptual loss / GAN loss (disc.hip) ---------------- */

/* nn.BatchNorm2d in train mode over z [npix][c] (bf16 NHWC; c % 8 == 0, c <= 2048, npix*c < 2^31), fused with
 * the following activation: y = act(gamma*(z-mean)*rstd + beta).  Saves mean/rstd for the backward, updates
 * run_mean/run_var (momentum, unbiased var) and increments *num_batches_tracked when non-NULL
 * (rfb_esrgan.py:32-50 BN + LeakyReLU).  workspace >= climsr_bn_workspace_doubles(npix, c) doubles
 * (per-block fp64 partial sums; the reduction order is fixed, so results are deterministic). */
int64_t climsr_bn_workspace_doubles(int64_t npix, int c);
int climsr_bn_forward(const uint16_t* z, int64_t npix, int c, const float* gamma, const float* beta, int act, float slope,
                      float eps, float momentum, double* workspace, float* mean, float* rstd, float* run_mean, float* run_var,
                      int64_t* num_batches_tracked, uint16_t* y, void* stream);
/* climsr_bn_forward with the batch statistics taken from the producing conv's epilogue partials (ClimsrEpilogue.bn_part,
 * nparts = climsr_conv2d_fwd_bn_parts) instead of a pass over z. */
int climsr_bn_forward_parts(const double* parts, int64_t nparts, const uint16_t* z, int64_t npix, int c, const float* gamma,
                            const float* beta, int act, float slope, float eps, float momentum, float* mean, float* rstd,
                            float* run_mean, float* run_var, int64_t* num_batches_tracked, uint16_t* y, void* stream);

/* climsr_bn_backward_z (bf16 da) with the statistics pass replaced by the producing data gradient's epilogue partials
 * (ClimsrEpilogue.bn_z + bn_part, nparts = climsr_conv2d_fwd_bn_parts with bn_z set): dgamma / dbeta and
 * dz = gamma*rstd * (d - mean(d) - xhat * mean(d*xhat)).  Replaces the BatchNorm2d backward of rfb_esrgan.py:32-50. */
int climsr_bn_backward_parts(const double* parts, int64_t nparts, const uint16_t* da, const uint16_t* z, int64_t npix, int c,
                             const float* mean, const float* rstd, const float* gamma, const float* beta, float slope, float* coef,
                             float* dgamma, float* dbeta, int accumulate, uint16_t* dz, void* stream);
/* Eval-mode BN (running statistics) + activation (nn.BatchNorm2d.eval()). */
int climsr_bn_inference(const uint16_t* z, int64_t npix, int c, const float* run_mean, const float* run_var, float eps,
                        const float* gamma, const float* beta, int act, float slope, uint16_t* y, void* stream);
/* *p += 1 on the device (BatchNorm num_batches_tracked). */
int climsr_increment_i64(int64_t* p, void* stream);
/* Backward of act(BN(z)): da = dL/d(act output) fp32, a = act output (bf16, sign gives lrelu'; slope 1 =
 * no activation), dz (bf16) = BN input gradient; dgamma/dbeta (+)= .  coef >= 3*c floats scratch;
 * workspace as for climsr_bn_forward.
 * out_slope != 1: z itself is a LeakyReLU output (plain discriminator, discriminator.py:17-18) and dz is
 * carried through its derivative (z <= 0 -> * out_slope). */
int climsr_bn_backward(const float* da, const uint16_t* a, const uint16_t* z, int64_t npix, int c, const float* mean,
                       const float* rstd, const float* gamma, float slope, float out_slope, double* workspace, float* coef,
                       float* dgamma, float* dbeta, int accumulate, uint16_t* dz, void* stream);
/* Backward of LeakyReLU(BN(z)) without the activation tensor (rfb_esrgan.py:32-50): lrelu' is taken from the sign
 * of gamma*(z-mean)*rstd + beta recomputed exactly as climsr_bn_forward applied it.  da = dL/d(act output), bf16
 * (da_bf16 = 1, as the next conv's data gradient writes it) or fp32; other arguments as climsr_bn_backward. */
int climsr_bn_backward_z(const void* da, int da_bf16, const uint16_t* z, int64_t npix, int c, const float* mean,
                         const float* rstd, const float* gamma, const float* beta, float slope, double* workspace, float* coef,
                         float* dgamma, float* dbeta, int accumulate, uint16_t* dz, void* stream);

/* nn.AdaptiveAvgPool2d((oh,ow)) (rfb_esrgan.py:54) on NHWC bf16 x [n][h][w][c]; out = torch.flatten
 * order [n][c*oh*ow] bf16; out_t (optional) = its transpose [c*oh*ow][n_pad] for the fc.0 weight grad. */
int climsr_adaptive_pool_fwd(const uint16_t* x, int n, int h, int w, int c, int oh, int ow, uint16_t* out, uint16_t* out_t,
                             int n_pad, void* stream);
/* Backward: dx [n][h][w][c] fp32 (overwritten) from dp [n][c*oh*ow] fp32. */
int climsr_adaptive_pool_bwd(const float* dp, int n, int h, int w, int c, int oh, int ow, float* dx, void* stream);

/* nn.Linear forward on MFMA: y[n][o] = act(x[n][k] . w[o][k] + b[o]) (fp32 out); n <= 64, k % 32 == 0,
 * o % 16 == 0; split-K partials in workspace (ws_floats >= nsplit*n*o, nsplit <= 3072/ceil(o/64) + 1). */
int climsr_linear_fwd(const uint16_t* x, const uint16_t* w, const float* bias, int n, int k, int o, int act, float slope,
                      float* workspace, int64_t ws_floats, float* y, void* stream);
/* dx[n][k] (+)= dy[n][o] . w[o][k] (bf16 in, fp32 out); k % 64 == 0, o % 32 == 0. */
int climsr_linear_dgrad(const uint16_t* dy, const uint16_t* w, int n, int k, int o, float* dx, int accumulate, void* stream);
/* dw[o][k] (+)= sum_n dy_t[o][n] x_t[k][n] (K = n_pad, multiple of 32; k % 64 == 0, o % 64 == 0). */
int climsr_linear_wgrad(const uint16_t* dy_t, const uint16_t* x_t, int n_pad, int k, int o, float* dw, int accumulate,
                        void* stream);
/* climsr_linear_wgrad continued over a second batch in the same launch: dw (+)= dy_t . x_t + dy_t2 . x_t2 (n_pad2 % 32 == 0);
 * the RFB discriminator's real and fake backward calls (pl_gan.py:51-61) write fc.0's gradient once. */
int climsr_linear_wgrad2(const uint16_t* dy_t, const uint16_t* x_t, int n_pad, const uint16_t* dy_t2, const uint16_t* x_t2,
                         int n_pad2, int k, int o, float* dw, int accumulate, void* stream);
/* The RFB discriminator's stem in one launch (rfb_esrgan.py:28-31): features.0 (1 -> 64, 3x3, pad 1, LeakyReLU slope)
 * recomputed where features.2 (64 -> 64, 3x3, stride 2, pad 1, no bias) needs it, z2 = features.2's pre-BatchNorm
 * output (bf16 [n][h/2][w/2][64]) with the BatchNorm partial sums of each 16x16 output tile in bn_part ([tiles][2][64],
 * climsr_d_stem_s2_bn_parts rows, the layout climsr_bn_forward_parts reads; NULL: none).  a0 (bf16 [n][h][w][64]) gets
 * features.0's output for the backward when non-NULL.  x: bf16 NHWC with the image in channel 0 (channel stride x_cs);
 * w0: features.0's fp32 OIHW weight [64][1][3][3]; w2: features.2's packed bf16 weight (climsr_pack_conv_weight,
 * cc 32: kpk2 = 576).  Replaces the features.0 stencil + the stride-2 conv launch (climsr_conv2d_fwd x 2). */
typedef struct ClimsrStemDesc {
  const uint16_t* x;
  int32_t x_cs;
  const float* w0;
  const uint16_t* w2;
  int32_t kpk2;
  uint16_t* a0;
  uint16_t* z2;
  double* bn_part;
  float slope;
  int32_t n, h, w;
} ClimsrStemDesc;
int climsr_d_stem_s2(const ClimsrStemDesc* d, void* stream);
int64_t climsr_d_stem_s2_bn_parts(int32_t n, int32_t h, int32_t w);
/* VGG19 conv1_1 (+ bias + ReLU) of the perceptual loss on torch.cat([x, x, x], 1) (perceptual.py:16,26-31) as ONE
 * 1-channel conv with the summed weight W0 + W1 + W2: images 0..n_half-1 from xa, n_half..2 n_half-1 from xb (fp32
 * [n_half][h][w] planes, rounded to bf16), weight fp32 [64][3][3][3], bias [64]; y bf16 NHWC [2 n_half][h][w][64]. */
int climsr_vgg_conv1_1(const float* xa, const float* xb, int n_half, int h, int w, const float* weight, const float* bias,
                       uint16_t* y, void* stream);

/* Discriminator head after fc.0 (+LeakyReLU) (h [n][o] fp32): s[n] = sigmoid(h.w2 + b2) (rfb_esrgan.py:59-60),
 * or h.w2 + b2 with sigmoid = 0 (plain discriminator's classification.1, discriminator.py:40). */
int climsr_d_head_fwd(const float* h, const float* w2, const float* b2, int n, int o, int sigmoid, float* s, void* stream);
/* Head backward from ds[n]: dw2/db2/db0 (+)=; du0 = d(fc.0 pre-activation) as bf16 [n][o] and [o][n_pad]
 * (slope = the LeakyReLU between fc.0 and the head; 1 = none). */
int climsr_d_head_bwd(const float* h, const float* s, const float* ds, const float* w2, int n, int o, int n_pad, float slope,
                      int sigmoid, float* dw2, float* db2, float* db0, int accumulate, uint16_t* du0, uint16_t* du0_t,
                      void* stream);
/* nn.ReflectionPad2d(1) (discriminator.py:15,21): y [n][h+2][w+2][cstride] bf16 from x [n][h][w][cstride]. */
int climsr_reflect_pad1_bf16(const uint16_t* x, int n, int h, int w, int cstride, uint16_t* y, void* stream);
/* Its backward: g [n][h][w][c] fp32 = sum of the padded gradient gp [n][h+2][w+2][c] over the mirrored reads. */
int climsr_reflect_pad1_bwd_f32(const float* gp, int n, int h, int w, int c, float* g, void* stream);
/* Relativistic-average BCEWithLogits (pl_gan.py:33-38, 54-59): loss = (BCE(s_f-mean(s_r), t_fr) +
 * BCE(s_r-mean(s_f), t_rf))/2; with gscale (device scalar) also the gradients w.r.t. s_real/s_fake. */
int climsr_relativistic_bce(const float* s_real, const float* s_fake, int n, float t_rf, float t_fr, float* loss,
                            const float* gscale, float* g_real, float* g_fake, void* stream);
/* VGG19 MaxPool2d(2,2) on NHWC bf16 (perceptual.py:16). */
int climsr_maxpool2_bf16(const uint16_t* x, int n, int h, int w, int c, uint16_t* y, void* stream);
/* mean |a-b| over n bf16 elements (n % 8 == 0); workspace >= 512 doubles (perceptual.py:31-34). */
int climsr_l1_loss_bf16(const uint16_t* a, const uint16_t* b, int64_t n, double* workspace, float* out, void* stream);
/* y = bf16(x) elementwise (MFMA copy of fp32 master weights). */
int climsr_f32_to_bf16(const float* x, int64_t n, uint16_t* y, void* stream);

/* ---------------------------------------------------------------------------------------------
 * On-device tile pipeline.  Replaces the per-sample CPU work of
 * ClimateDataset.__getitem__ (climsr/data/sr/climate_dataset.py:220-275), _get_training_sample
 * (:144-189), _get_val_test_sample (:191-218), _common_to_tensor / _concat_if_needed (:95-142) and
 * MinMaxScaler / StandardScaler._normalize (climsr/data/normalization.py:37-61, 99-113) for a batch
 * of raw tiles already in HBM.  All tensors are contiguous fp32 NCHW ([n][1][h][w] per plane).
 * --------------------------------------------------------------------------------------------- */
typedef struct {
  const float* hr_raw;       /* [n][h][w] raw tile (NaN = no data / sea) */
  const float* elev_raw;     /* [n][h][w] raw elevation (== elev_missing -> NaN); NULL if !use_elev */
  const double* hr_min;      /* [n] per-tile (or global) min / max, float64 as in the stats tables (method 0) */
  const double* hr_max;
  const float* elev_minmax;  /* [n][2] nanmin / nanmax of the elevation tile (climsr_tile_minmax_f32; method 0) */
  const int32_t* xform;      /* [n] bit0 np.flipud, bit1 np.fliplr, bits2-3 np.rot90 factor (applied in that order);
                                NULL = identity (val / test) */
  float* lr;                 /* [n][lr_c][h/scale][w/scale]; SRCNN: [n][lr_c][h][w] */
  float* hr;                 /* [n][1][h][w] normalised HR */
  float* elev;               /* [n][1][h][w] normalised elevation, or NULL */
  float* mask;               /* [n][1][h][w] land mask 1/0 (~isnan(original)), or NULL */
  float* nearest;            /* [n][1][h][w] nearest upscale of the LR temperature (val/test `nearest`), or NULL */
  float* elev_lr;            /* [n][1][h/scale][w/scale] (val/test `elevation_lr`), or NULL */
  float* hr_lr;              /* [n][1][h/scale][w/scale] LR temperature plane (input of the `cubic` upscale), or NULL */
  double range_a, range_b;   /* MinMaxScaler feature_range (normalize_range, default (-1, 1)) */
  double eps;                /* 1e-8 (both scalers) */
  double nan_sub;            /* MinMaxScaler nan_substitution (0.0) */
  double zs_hr_mean, zs_hr_std, zs_hr_nan_sub;      /* StandardScaler (method 1); nan_sub applied only if != 0 */
  double zs_elev_mean, zs_elev_std, zs_elev_nan_sub;
  float elev_missing;        /* consts.world_clim.elevation_missing_indicator = -32768 */
  int32_t method;            /* 0 minmax, 1 zscore, 2 none */
  int32_t n, h, w, scale;    /* h, w multiples of scale; h == w when xform is given */
  int32_t lr_c;              /* 1 + use_elev + use_mask */
  int32_t srcnn, use_elev, use_mask;
} ClimsrTileDesc;

/* out[2t], out[2t+1] = np.nanmin / np.nanmax of tile t (count floats each), treating value == missing as NaN
 * when use_missing (MinMaxScaler._normalize without min/max, normalization.py:45-50).  All-NaN -> NaN. */
int climsr_tile_minmax_f32(const float* x, int n, int64_t count, float missing, int use_missing, float* out, void* stream);
/* The fused flip / rot90 / normalise / mask / decimate / concat pass.  One launch per batch. */
int climsr_tile_prepare(const ClimsrTileDesc* d, void* stream);
/* cv2.resize(..., INTER_CUBIC) of fp32 planes [n][sh][sw] -> [n][dh][dw] (the val/test `cubic` item,
 * climate_dataset.py:195): A = -0.75, replicate border, horizontal then vertical pass. */
int climsr_resize_cubic_f32(const float* src, int n, int sh, int sw, float* dst, int dh, int dw, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Validation / test metrics on device: TaskSuperResolutionModule.
 * common_val_test_step + compute_metrics (climsr/core/task.py:262-294, 336-372) with the torchmetrics
 * definitions the reference instantiates (task.py:296-323) and RegressionAccuracy
 * (climsr/metrics/regression_accuracy.py:6-22).  Deterministic: fixed-order fp64 block partials.
 * out[CLIMSR_SR_METRICS] = acc@{eps[0..7]}, psnr, ssim, mae, mse, rmse, mape, smape, r2, l1(normalised).
 * --------------------------------------------------------------------------------------------- */
#define CLIMSR_SR_METRICS 17
typedef struct {
  const float* sr;         /* [n][1][h][w] normalised generator output */
  const float* hr;         /* [n][1][h][w] normalised HR */
  const float* original;   /* [n][1][h][w] raw HR (NaN at sea; zeroed by the mask like task.py:291) */
  const float* mask;       /* [n][1][h][w] land mask (0 = sea) */
  const double* min;       /* [n] per-sample min / max of the batch (method 0 denormalisation) */
  const double* max;
  double* workspace;       /* climsr_sr_metrics_workspace() bytes */
  double* out;             /* [CLIMSR_SR_METRICS] */
  double range_a, range_b, eps;
  double zs_mean, zs_std;  /* method 1: StandardScaler._denormalize */
  float acc_eps[8];        /* RegressionAccuracy eps list (task.py:297-304) */
  int32_t n, h, w;         /* h, w >= 11 (SSIM window) */
  int32_t method;          /* 0 minmax, 1 zscore, 2 identity */
} ClimsrMetricsDesc;

size_t climsr_sr_metrics_workspace(void);
int climsr_sr_metrics(const ClimsrMetricsDesc* d, void* stream);
/* RegressionAccuracy.update: counts[0] += #(|p - t| <= eps) (float32), counts[1] += n.  int64 device counters. */
int climsr_regression_accuracy_update(const float* preds, const float* target, int64_t n, float eps, int64_t* counts,
                                      void* stream);

/* Inference output (inference.py:73-80): out = MinMaxScaler.denormalize(sr, min[t], max[t]) per sample t
 * (float64 arithmetic, normalization.py:63-84) and NaN where mask == 0 (mask may be NULL).  [n][hw] fp32. */
int climsr_denormalize_mask(const float* sr, const float* mask, const double* min, const double* max, double range_a,
                            double range_b, int n, int64_t hw, float* out, void* stream);

/* ---------------------------------------------------------------------------------------------
 * RCAN (climsr/models/rcan.py).
 * --------------------------------------------------------------------------------------------- */
/* CALayer (rcan.py:50-69): s[n][c] = sigmoid(w2 . relu(w1 . mean_p u[n][p][:] + b1) + b2), u fp32 NHWC
 * [n][hw][u_cstride]; w1 [cr][c], w2 [c][cr] (the 1x1 conv_du weights); workspace
 * climsr_channel_attention_workspace(n, c) bytes.  Deterministic (fixed-order fp64 pooling). */
size_t climsr_channel_attention_workspace(int n, int c);
int climsr_channel_attention(const float* u, int n, int64_t hw, int c, int u_cstride, const float* w1, const float* b1,
                             const float* w2, const float* b2, int cr, double* workspace, float* s, void* stream);
/* The same from channel-sum rows already pooled by the conv that produced u (ClimsrEpilogue.ch_part):
 * part[n][tiles_per_image][c] fp32, summed over the rows in a fixed order in fp64 (at most 1024 rows of c = 64: by the
 * MLP kernel itself, else folded into fp64 slices first); hw = pixels per image;
 * workspace = climsr_channel_attention_workspace(n, c) bytes. */
int climsr_channel_attention_parts(const float* part, int n, int tiles_per_image, int64_t hw, int c, const float* w1,
                                   const float* b1, const float* w2, const float* b2, int cr, double* workspace, float* s,
                                   void* stream);
/* climsr_channel_attention / climsr_channel_attention_parts that also keep the pooled mean (mean_out fp32 [n][c]) for
 * the training backward (climsr_ca_backward). */
int climsr_channel_attention_mean(const float* u, int n, int64_t hw, int c, int u_cstride, const float* w1, const float* b1,
                                  const float* w2, const float* b2, int cr, double* workspace, float* s, float* mean_out, void* stream);
int climsr_channel_attention_parts_mean(const float* part, int n, int tiles_per_image, int64_t hw, int c, const float* w1,
                                        const float* b1, const float* w2, const float* b2, int cr, double* workspace, float* s,
                                        float* mean_out, void* stream);
/* Backward of the RCAB's channel attention + residual (CALayer / RCAB.forward, rcan.py:50-69,98-101; replaces the autograd
 * of AdaptiveAvgPool2d -> 1x1 -> ReLU -> 1x1 -> Sigmoid -> x * y under the reference's RCAN pre-training,
 * conf/experiment/rcan_pre_training.yaml).  y = u * s + x, s = sigmoid(w2 relu(w1 mean + b1) + b2): given gy = dL/dy
 * (fp32 [n][hw][gy_cstride]), u (fp32, or bf16 with u_bf16 = 1), s and mean (fp32 [n][c], the forward's; mean from
 * climsr_channel_attention*_mean), writes gu = dL/du = gy * s + (w1^T g_a1) / hw (bf16 [n][hw][gu_cstride]) and the
 * conv_du gradients gw1 [cr][c], gb1 [cr], gw2 [c][cr], gb2 [c] (fp32, '=' or '+=' with accumulate; gb1 / gb2 null
 * exactly when b1 / b2 are).  dL/dx = gy is left to the caller.  Deterministic (fixed-order fp64 slices, images summed
 * in order).  workspace = climsr_ca_backward_workspace(n, hw, c, cr) bytes; c a multiple of 8 (<= 1024). */
size_t climsr_ca_backward_workspace(int n, int64_t hw, int c, int cr);
int climsr_ca_backward(const float* gy, int gy_cstride, const void* u, int u_bf16, int u_cstride, const float* s, const float* mean, int n,
                       int64_t hw, int c, const float* w1, const float* b1, const float* w2, int cr, float* gw1, float* gb1, float* gw2,
                       float* gb2, int accumulate, void* workspace, uint16_t* gu, int gu_cstride, void* stream);
/* RCAB residual with the attention scale (rcan.py:104-107): xres = u * s + xres (fp32 [n][hw][c]) and
 * xb = bf16(xres) ([n][hw][xb_cstride], the next conv's input); u = the RCAB body's output, fp32 or (u_bf16 = 1)
 * bf16, channel stride u_cstride.  c, strides multiples of 4. */
int climsr_ca_scale_add(const void* u, int u_bf16, int u_cstride, const float* s, float* xres, uint16_t* xb, int xb_cstride,
                        int n, int64_t hw, int c, void* stream);
/* The SRCNN tail of the ESRGAN generator as ONE launch, replacing srcnn.conv1 -> ReLU -> conv2 -> ReLU -> conv3
 * (srcnn.py:9-18) on torch.cat([out, elev, mask], 1) (esrgan.py:99-100): x = bf16 NHWC, channels x_co .. x_co+3 (the
 * in_c <= 4 real ones + zeros); out = fp32 [n][1][h][w]; the 64- and 32-channel intermediates stay on chip (the
 * backward, climsr_srcnn_bwd, recomputes them).  wpk = climsr_srcnn_packed_elems() bf16 from climsr_srcnn_pack;
 * b1/b2/b3 = the fp32 biases (64 / 32 / 1). */
typedef struct ClimsrSrcnnDesc {
  const uint16_t* x;
  int32_t x_cs, x_co;
  const uint16_t* wpk;
  const float* b1;
  const float* b2;
  const float* b3;
  float* out;
  int32_t n, h, w;
} ClimsrSrcnnDesc;
int climsr_srcnn_fwd(const ClimsrSrcnnDesc* d, void* stream);
/* Backward of the fused SRCNN tail below conv1, recomputing relu(conv1) / relu(conv2) from x instead of storing them:
 * gout = dL/d(out) fp32 [n][1][h][w]; writes dz1 = dL/d(conv1 output) bf16 [n][h][w][64] (ReLU' applied: what conv1's
 * weight / data gradients read) and the conv2 / conv3 weight and bias gradients (fp32, OIHW; accumulate = 1: +=),
 * summed over climsr_srcnn_bwd_workspace(n, h, w) bytes of per-workgroup partials in a fixed order. */
typedef struct ClimsrSrcnnBwdDesc {
  const uint16_t* x;
  int32_t x_cs, x_co;
  const float* gout;
  const uint16_t* wpk;
  const float* b1;
  const float* b2;
  uint16_t* dz1;
  float* part;
  float* gw2;
  float* gb2;
  float* gw3;
  float* gb3;
  int32_t accumulate;
  int32_t n, h, w;
} ClimsrSrcnnBwdDesc;
int climsr_srcnn_bwd(const ClimsrSrcnnBwdDesc* d, void* stream);
int64_t climsr_srcnn_bwd_workspace(int n, int h, int w);
/* Pack the three SRCNN weights (fp32 OIHW: w1 [64][in_c][9][9], w2 [32][64][1][1], w3 [1][32][5][5]) into the MFMA
 * fragment order climsr_srcnn_fwd reads (async on stream; run after every weight update). */
int climsr_srcnn_pack(const float* w1, const float* w2, const float* w3, int in_c, uint16_t* out, void* stream);
int64_t climsr_srcnn_packed_elems(void);
/* nn.PixelShuffle(r) (Upsampler, rcan.py:17-47) on NHWC bf16: y[n][y*r+i][x*r+j][co] = x[n][y][x][co*r*r+i*r+j].
 * Bit-exact index map; c_out and out_cstride multiples of 8. */
int climsr_pixel_shuffle_bf16(const uint16_t* x, int n, int h, int w, int c_out, int r, int in_cstride, uint16_t* y,
                              int out_cstride, void* stream);

/* Backward of nn.PixelShuffle(r) (rcan.py:32; replaces its autograd under RCAN training): the inverse index map,
 * gx[n][y][x][co*r*r+i*r+j] = gy[n][y*r+i][x*r+j][co], NHWC bf16, bit-exact.  c_out*r*r and gx_cstride multiples of 8. */
int climsr_pixel_unshuffle_bf16(const uint16_t* gy, int n, int h, int w, int c_out, int r, int gy_cstride, uint16_t* gx,
                                int gx_cstride, void* stream);

#ifdef __cplusplus
}
#endif
#endif
