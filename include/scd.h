/*
 * scd.h — C-ABI of the MI355X (gfx950) Siamese change-detection kernel library (libscd.so).
 *
 * The reference (SebastianHafner/multimodal_siamese_cd) has no native code and no FFI: its hot path
 * is the torch module stack in utils/networks.py (DoubleConv 386-402, InConv 405-412, Down 415-426,
 * Up 429-451, OutConv 454-461, SiameseUNet.forward 139-154) and power_jaccard_loss
 * (utils/loss_functions.py:141-150).  Every aten op those modules call is replaced by one entry
 * point below; the "replaces" line of each cites the reference call site.  The Python host layer
 * (multimodal_siamese_cd_amd/hip.py, ctypes) binds exactly these symbols.
 *
 * Conventions
 *  - Every function returns int: 0 = ok, negative = error; scd_last_error() (thread-local) has text.
 *  - Activations are NHWC.  An scd_nhwc_t is a *channel slice* view: element (n,y,x,c) lives at
 *    data[((n*h + y)*w + x)*ldc + c].  c and ldc are multiples of 4; data is 16-byte aligned (fp32) or 8-byte
 *    aligned (bf16).
 *  - Element type (ABI 6): a view is fp32 (dtype 0, the value of a zero-initialised view) or bf16 (the activation
 *    and gradient storage of the bf16 configs).  A bf16 element is loaded exactly, every kernel computes in fp32,
 *    and a bf16 result is rounded to nearest-even once, when it is stored.  The NHWC views of one call share one
 *    type (scd_pack_nchw's NCHW fp32 source and the fp32 heads/losses aside); a bf16 conv view needs
 *    SCD_MATH_BF16 and a shape the bf16 kernels take (the query functions report 0 / negative otherwise).
 *    Statistics (BatchNorm records, weight-grad slabs, bounds) stay fp32.
 *  - The library never allocates, frees or synchronises.  Workspaces are caller-owned (torch caching
 *    allocator); size them with the *_workspace_bytes() queries.  All launches are asynchronous on the
 *    caller's stream (a hipStream_t passed as void*; NULL = legacy default stream).
 *  - Stateless and re-entrant: no process-wide modes and no environment switches; the arithmetic and kernel
 *    variant of a conv are fields of its descriptor.  One GPU per process.
 */
#ifndef SCD_H_
#define SCD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *scd_stream_t; /* hipStream_t */

enum scd_status {
    SCD_OK = 0,
    SCD_ERR_ARG = -1,         /* bad shape / null pointer / unsupported combination   */
    SCD_ERR_ALIGN = -2,       /* pointer or channel stride not 16-byte aligned          */
    SCD_ERR_LAUNCH = -3,      /* hipGetLastError() after launch                         */
    SCD_ERR_DEVICE = -4,      /* device is not gfx950                                   */
    SCD_ERR_WORKSPACE = -5,   /* workspace too small                                    */
};

/* Element type of a view (scd_nhwc_t.dtype). */
enum scd_dtype {
    SCD_DT_F32 = 0,
    SCD_DT_BF16 = 1
};

/* NHWC channel-slice view. */
typedef struct scd_nhwc {
    void *data;
    int32_t n, h, w, c, ldc;
    int32_t dtype; /* enum scd_dtype (ABI 6; fills the struct's former tail padding: size and offsets unchanged) */
} scd_nhwc_t;

/* ---------------------------------------------------------------------------------------------
 * Info
 * ------------------------------------------------------------------------------------------- */
const char *scd_version(void);
const char *scd_last_error(void);
/* 0 if `device` is a gfx950 (MI355X); SCD_ERR_DEVICE otherwise. */
int scd_device_check(int device);

/* ---------------------------------------------------------------------------------------------
 * Layout / weight packing
 * ------------------------------------------------------------------------------------------- */
/* dst[n, y, x, 0:c_count] = src[n, c_begin:c_begin+c_count, y, x]  (NCHW -> NHWC slice);
 * dst[n, y, x, c_count:dst.c] = 0 (channel padding to the MFMA K granule).
 * `bound` (nullable, a device float): raised to max |value| written -- the SCD_MATH_H2 operand bound of the packed
 * input (scd_igemm_t.src_bound of the input layer), at no extra pass.
 * replaces: the .to(device) input hand-off + implicit NCHW layout (train_supervised.py:68-69) and
 * the channel slicing/concats of DualStreamUNet/WhateverNet (networks.py:105-106,113-114,236,247). */
int scd_pack_nchw(const float *src, int32_t n, int32_t c, int32_t h, int32_t w, int32_t c_begin,
                  int32_t c_count, scd_nhwc_t dst, float *bound, scd_stream_t stream);

/* Conv2d 3x3 weight OIHW [co][ci][3][3] ->
 *   mode 0 (forward):   [co][9][ci_pad]           (zero for ci >= ci)
 *   mode 1 (data grad): [ci][9][co], taps flipped (W[co][ci][2-ky][2-kx])
 * replaces: nn.Conv2d(in,out,3,padding=1) parameter layout (networks.py:392,395). */
/* Batched form for one training step's weights: per job the packed layout above into `out` and, when
 * `split` != NULL, its fragment-major bf16x3 split (the scd_split_bf16x3_frag layout of `out`; its K, 9*ci_pad or
 * 9*co, a multiple of 16) -- or, for job.math == SCD_MATH_H2 and K / 9 a multiple of 32, the scd_split_h2_frag format.
 * Any number of jobs; one launch per 48. */
typedef struct scd_pack_job {
    const float *w;
    float *out;
    uint16_t *split;
    int32_t co, ci, ci_pad, mode;
    int32_t math; /* arithmetic of the convs reading `split`: SCD_MATH_H2 writes the h2 format where it applies */
} scd_pack_job_t;
int scd_pack_conv3x3_multi(const scd_pack_job_t *jobs, int32_t n, scd_stream_t stream);
int scd_pack_conv3x3(const float *w, int32_t co, int32_t ci, int32_t ci_pad, int32_t mode, float *out,
                     scd_stream_t stream);

/* ConvTranspose2d weight [ci][co][2][2] ->
 *   mode 0 (forward):   [(i*2+j)*co + o][ci]
 *   mode 1 (data grad): [ci][(i*2+j)*co + o]
 * replaces: nn.ConvTranspose2d(C,C,2,stride=2) parameter layout (networks.py:433). */
int scd_pack_convT2x2(const float *w, int32_t ci, int32_t co, int32_t mode, float *out, scd_stream_t stream);
/* Several ConvTranspose2d weights in three launches: per job (scd_pack_job_t: w [ci][co][2][2], out as
 * scd_pack_convT2x2 mode 0 / 1, ci_pad ignored) the packed layout and, with `split`, its fragment-order split in the
 * format the conv reading it expects under job.math (scd_split_h2_frag where h2_weight_format applies -- 1 tap over ci
 * channels (mode 0) or 4 taps over co (mode 1), a multiple of 32 -- else scd_split_bf16x3_frag; K % 16 == 0).
 * Results equal the one-weight calls. */
int scd_pack_convT2x2_multi(const scd_pack_job_t *jobs, int32_t n, scd_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Conv arithmetic, chosen per launch by scd_igemm_t.math / scd_wgrad_t.math (and scd_pack_job_t.math for the
 * weight split it feeds).  The library keeps no arithmetic state: two models with different arithmetic can run
 * in one process, on one stream or several.  Every mode computes an fp32 GEMM with fp32 accumulation:
 *   SCD_MATH_F32  v_mfma_f32_32x32x2_f32: exact fp32 products (a k-ordered fmaf chain per MFMA).  The value of a
 *                 zero-initialised descriptor.
 *   SCD_MATH_X3   v_mfma_f32_32x32x16_bf16 on an exact 3-way bf16 split of each fp32 operand
 *                 (x = h + m + l, each term rounded to nearest), accumulating the six terms
 *                 hh+hm+mh+mm+hl+lh.  The dropped terms are <= ~2^-26 relative, so the rounding error is
 *                 of fp32 order, at 6/16 of the matrix-core cycles.  Used when src.c % 16 == 0; other shapes
 *                 fall back to the fp32 MFMA kernel.
 *   SCD_MATH_BF16 bf16 operands (each fp32 operand rounded to nearest bf16, the h term of the split), one
 *                 v_mfma_f32_16x16x32_bf16 product per k step, fp32 accumulation: the arithmetic of a bf16
 *                 autocast conv (BASELINE configs baseline_dualstream / siamese_mmcr, dtype bf16).  Applies to
 *                 the 16x16x32 halo kernels (3x3 stride-1 fwd / data-grad / weight-grad, >= 98% of the
 *                 U-Net's conv FLOPs); every other conv shape keeps the SCD_MATH_X3 kernels.  Activations and
 *                 BatchNorm stay fp32.
 *   SCD_MATH_X5   SCD_MATH_X3 less one of its three second-order products (w_l*x_h in the fwd/data-grad halo
 *                 kernel, x_l*dy_h in the halo weight grad; each <= 2^-18 relative, below fp32 accumulation noise
 *                 over the contraction lengths here): five products, two weight / X planes.  Halo kernels only.
 *   SCD_MATH_H2   two-term fp16 split with power-of-two operand scaling (see scd_igemm_t.src_bound): three
 *                 v_mfma_f32_16x16x32_f16 products per fp32 product, 22 significant bits per operand.  Convs
 *                 without operand bounds, and shapes the h2 kernels do not take, run SCD_MATH_X3.
 * ------------------------------------------------------------------------------------------- */
enum scd_conv_math {
    SCD_MATH_F32 = 0,
    SCD_MATH_X3 = 1,
    SCD_MATH_BF16 = 2,
    SCD_MATH_X5 = 3,
    SCD_MATH_H2 = 4
};
/* ABI revision of this header (struct layouts and signatures); a binding checks it at load time.
 *   3: scd_igemm_t / scd_wgrad_t / scd_pack_job_t carry `math` (and `tune`); the process-wide mode setters
 *      (scd_set_conv_math, scd_set_halo16, scd_set_wgrad16) and every launch-time environment switch are gone.
 *   4: scd_pack_nchw takes a nullable `bound` (the input layer's h2 operand bound).
 *   5: scd_bn_relu_backward_coef takes `da_bound` / `dy_bound` (the h2 bound of the dy a weight grad forms itself);
 *      the 16-channel-source weight grad runs h2 when both scd_wgrad_t bounds are set.
 *   6: scd_nhwc_t.dtype: bf16 activation / gradient storage (the bf16 configs), every NHWC kernel.
 *   7: scd_bn_relu_pool_out (plain and dual-task encoder levels written into the decoders' concat buffers),
 *      scd_bn_relu_backward_pooled2 (a second, swapped skip gradient), scd_conv1x1_fwd_bn2 (two-source heads).
 *   8: scd_wgrad_t.rows_out / rows_out_bound appended (the halo weight grad forms and stores a plain BatchNorm
 *      backward's dY).
 *   9: scd_igemm_t.dst_bound_seed appended (a bound seeded with another buffer's bound inside the conv launch). */
#define SCD_ABI_VERSION 9
int scd_abi_version(void);
/* The arithmetic scd_conv_igemm / scd_conv_wgrad will use for a descriptor (its `math`, or SCD_MATH_X3 / F32 where
 * the shape or the missing operand bounds keep the conv off the requested kernels); negative = invalid descriptor.
 * (Declared with the descriptors below.) */
/* Kernel-variant selection, scd_igemm_t.tune / scd_wgrad_t.tune.  0 = the library's measured defaults; the other
 * values select variants kept for bit-identity tests and A/B measurements.  Every variant computes the same
 * outputs (bit-identical where the tests say so, else equal up to fp32 summation order). */
#define SCD_TUNE_HALO16_CFG(id)   ((uint32_t)((id) + 1))  /* force 16x16x32 halo tile id 0..5 (3-5: h2 only;
                                                             id 3 under bf16 storage: the 128x128 1x4 tile, never the
                                                             automatic 128x256 one)                              */
#define SCD_TUNE_HALO16_OFF       0xFu                    /* the 32x32x16 halo kernel instead                     */
#define SCD_TUNE_HALO16_MASK      0xFu
#define SCD_TUNE_HALO16_WRING     0x8u                    /* automatic tiles; h2 1xN tiles' weights via an LDS ring */
#define SCD_TUNE_H2_TILE_2X2      (1u << 4)   /* h2, >= 128 outputs: 2x2 waves instead of 1x4                     */
#define SCD_TUNE_H2_TILE64_2X2    (1u << 5)   /* h2, 64..127 outputs: 2x2 waves instead of 1x2                    */
#define SCD_TUNE_H2_NO_PRESCALE   (1u << 6)   /* h2 without the 2^11 pre-scaled low term (narrower range)         */
#define SCD_TUNE_NO_XCD_REMAP     (1u << 7)   /* plain block order instead of the XCD swizzle                     */
#define SCD_TUNE_HALO_ORDER_M     (1u << 8)   /* halo kernels: N-fastest block order                              */
#define SCD_TUNE_W16_LAYOUT_2X2   (1u << 9)   /* halo weight grad (h2 / bf16): 2x2 waves instead of along c       */
#define SCD_TUNE_WGRAD_R64        (1u << 10)  /* halo weight grad: 64-row blocks instead of 128                   */
#define SCD_TUNE_BF16_1XN         (1u << 11)  /* flips the bf16 arithmetic's 3x3 tile layout: 1 x N wave tiles (as h2;
                                                 the default with bf16 storage) <-> 2 x 2 (the default with fp32)     */
#define SCD_TUNE_X3_TILE(t)       ((uint32_t)(t) << 12)   /* per-tap x3 igemm tile 1..5 (0 = automatic); on the ConvT
                                                            gather kernel tile 1..3 (128x128, 128x64, 64x128):
                                                            the same bits, so a scope forcing an x3 tile also
                                                            forces the ConvT tiles -- never time ConvT launches
                                                            under an x3 tile study                              */
#define SCD_TUNE_X3_TILE_MASK     (0xFu << 12)
#define SCD_TUNE_C16_TILES(k)     ((uint32_t)(k) << 16)   /* input-layer forward: tiles per block (0 = 4; 15 =
                                                             one resident round)                                 */
#define SCD_TUNE_C16_TILES_MASK   (0xFu << 16)
#define SCD_TUNE_HALO16_DB_OFF    (1u << 20)  /* halo16 forward: single-buffered halo                             */
#define SCD_TUNE_HALO16_DB_ON     (1u << 21)  /* halo16 forward: double-buffered halo where it fits (h2 too)     */
#define SCD_TUNE_NO_GATHER16      (1u << 22)  /* ConvTranspose fwd / data grad on the x3 per-tap kernel           */
#define SCD_TUNE_NO_WGRAD_C16     (1u << 23)  /* input-layer weight grad on the generic x3 kernel                 */
#define SCD_TUNE_NO_WGRAD_H2      (1u << 24)  /* ConvTranspose weight grad on x3 instead of h2                    */
#define SCD_TUNE_NO_HALO16_C16    (1u << 25)  /* input-layer forward on the per-tap x3 kernel                     */
#define SCD_TUNE_NO_HALO          (1u << 26)  /* no halo kernels at all (per-tap kernels)                         */
#define SCD_TUNE_HALO16_LATE_LOAD (1u << 27)  /* single-buffered halo16: next chunk's halo loaded at the last tap  */
#define SCD_TUNE_H2_TILE64_128    (1u << 28)  /* 64..127 outputs of 64-channel sources (h2, bf16 storage): 128 x 64
                                                 tiles instead of 256 x 64 (2x2 waves of 128 px x 32 ch)             */
#define SCD_TUNE_HALO16_WS        (1u << 29)  /* h2 1 x N tiles as warp-specialized blocks: one producer wave stages
                                                 the halo, the compute waves load only weights (128 px tiles)        */
#define SCD_TUNE_WGRAD16_REGSTAGE (1u << 30)  /* bf16-storage halo weight grad staged through registers, one patch in
                                                 flight, instead of the LDS-DMA ring (A/B; until ABI 8 this bit chose
                                                 persistent ConvT gather blocks, removed: measured slower)           */
#define SCD_TUNE_WGRAD16_DB       (1u << 31)  /* h2 halo weight grad with two patch buffers, one barrier per patch and
                                                 (128-row blocks) the two wave groups staggered                      */
/* dst[p*n + i] = bf16 bits of term p (h, m, l) of src[i]: the exact 3-way split used by SCD_MATH_X3.
 * n % 8 == 0, src and dst 16-byte aligned. */
int scd_split_bf16x3(const float *src, int64_t n, uint16_t *dst, scd_stream_t stream);
/* The same split of a packed weight matrix w [n_out][K] (K % 16 == 0) in MFMA-fragment order, the layout
 * scd_igemm_t.wsplit expects: dst[p][nb][ks][lane][8] holds rows n = 32nb + (lane & 31) and
 * k = 16ks + 8(lane >> 5) + j (zero for n >= n_out), so one wave's B fragment is one 1 KB load. */
size_t scd_split_frag_bytes(int32_t n_out, int32_t K);
int scd_split_bf16x3_frag(const float *w, int32_t n_out, int32_t K, uint16_t *dst, scd_stream_t stream);
/* SCD_MATH_H2 weight split of a packed [n_out][K] matrix into a buffer of scd_split_frag_bytes(n_out, K): per
 * row r the power-of-two scale s_r that brings max_k |w[r][k]| below 2^15, the fp16 h and m planes of w * s_r in
 * the fragment order above (planes 0 and 1), then float inv[NB * 32] = 1 / s_r after the planes (1 for padding
 * rows).  scd_pack_conv3x3_multi writes this format instead of the bf16x3 split for 3x3 jobs whose K / 9 is a
 * multiple of 32 and whose math is SCD_MATH_H2 (including the per-row scales of the data-grad layout). */
int scd_split_h2_frag(const float *w, int32_t n_out, int32_t K, uint16_t *dst, scd_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Implicit-GEMM convolution on MFMA (arithmetic: scd_igemm_t.math).
 *   out[m, o] = bias[o] + sum_{t<ntaps, c<src.c} src[img, oy*stride+dy[t], ox*stride+dx[t], c] * wpk[o][t*src.c + c]
 *   m = (img, oy, ox) over src.n x out_h x out_w; out-of-range source pixels read as 0 (zero padding).
 * store_mode 0: dst[img, oy, ox, o]                            (dst.h == out_h, dst.w == out_w)
 * store_mode 1: 2x2 pixel shuffle, o = (i*2+j)*co + oc -> dst[img, 2oy+i, 2ox+j, oc], bias[oc]
 * Used for: Conv2d 3x3 forward (taps -1..1, stride 1), Conv2d 3x3 data-grad (flipped weights),
 *           ConvTranspose2d forward (1 tap, store_mode 1) and its data-grad (4 taps 0..1, stride 2).
 * replaces: aten::convolution / mkldnn_convolution (networks.py:392,395,433) and the data-grad half
 *           of aten::convolution_backward.  `cat([x2, x1], 1)` (networks.py:449) is zero-copy: dst may
 *           be a channel slice of the concat buffer.
 * ------------------------------------------------------------------------------------------- */
/* Fused BatchNorm + ReLU backward partial sums in the conv epilogue (for a data-grad conv whose output g
 * is dL/da of the layer a = relu(BN(y))): per output tile and channel c
 *   {sum dz, sum dz * xhat},  dz = g if fma(y, scale, shift) > 0 else 0,  xhat = (y - save_mean) * save_invstd
 * (coefficients of the tile's segment g = img / (n / nseg)) -> rec[c][tile][2], the records
 * scd_bn_relu_backward_tiles() consumes in place of its own partial pass over (y, g).
 * replaces: the reductions of native_batch_norm_backward (networks.py:393,396). */
typedef struct scd_bn_bwd_tiles {
    scd_nhwc_t y;  /* the BatchNorm input; same n, h, w as the conv output, c = n_out */
    int32_t nseg;
    const float *save_mean, *save_invstd, *scale, *shift;  /* [nseg][c] from the forward */
    float *rec;                                             /* [c][tiles][2] */
} scd_bn_bwd_tiles_t;

typedef struct scd_igemm {
    scd_nhwc_t src;
    int32_t out_h, out_w;
    int32_t stride;
    int32_t ntaps;
    int8_t dy[9], dx[9];
    const float *wpk;   /* [n_out][ntaps*src.c] */
    int32_t n_out;
    const float *bias;  /* [n_out] (store_mode 0) or [n_out/4] (store_mode 1) or NULL */
    scd_nhwc_t dst;
    int32_t store_mode;
    /* Optional (split arithmetics): wpk pre-split by scd_split_bf16x3_frag / scd_split_h2_frag (fragment order).
     * The weights are then staged by copy instead of being split in every workgroup.  NULL = split on
     * the fly.  Must describe the same values as wpk. */
    const uint16_t *wsplit;
    /* Optional fused BatchNorm statistics of the stored output (bias included): per output tile of
     * `tile_pixels` pixels (one image's rows) and channel, {mean, M2} -> stat_rec[tile][n_out][2], tiles in
     * image-major order.  Only when scd_igemm_stat_tiles() reports > 0 tiles for this descriptor; NULL = off.
     * replaces: the batch-statistics pass of aten::native_batch_norm (networks.py:393,396). */
    float *stat_rec;
    /* Optional fused input transform: the BatchNorm-apply + ReLU of the layer that produced src
     * (networks.py:393-394,396-397), so its activation never goes to memory.  Every in-range source
     * element of image img, channel c is read as max(s * in_scale[g*src.c + c] + in_shift[g*src.c + c], 0),
     * g = img / (src.n / in_nseg); the zero padding stays zero.  NULL = off.  Only for descriptors where
     * scd_igemm_input_bn_supported() returns 1 (16-byte aligned coefficient arrays). */
    const float *in_scale;
    const float *in_shift;
    int32_t in_nseg;
    /* Optional fused BatchNorm backward partial sums of the stored output (see scd_bn_bwd_tiles_t); only
     * where scd_igemm_bn_bwd_tiles() reports > 0 tiles.  NULL = off. */
    const scd_bn_bwd_tiles_t *bn_bwd;
    /* math == SCD_MATH_H2 only: device float holding an upper bound U >= |every src element as read| (after the input
     * transform).  A 3x3 conv with src.c % 32 == 0 (halo16 kernel), or a 1- / 4-tap conv with src.c % 32 == 0 and
     * n_out % 64 == 0 (the ConvTranspose forward and data grad: gather16 kernel), then runs the two-term fp16 split:
     * src scaled by the power of two that brings U below 2^15, weights from the h2 split of wsplit
     * (scd_pack_conv3x3_multi / scd_split_h2_frag), both scales undone exactly in the epilogue.  A bound below the true maximum overflows
     * fp16 (inf / NaN outputs); a loose one only lowers the absolute floor (2^-39 U).  NULL = the x3 kernels
     * (per-tap, fp32 weights split on the fly). */
    const float *src_bound;
    /* Optional: device float raised to max |stored output| as the epilogue writes it (atomic integer max;
     * caller-zeroed or holding an earlier bound) -- the SCD_MATH_H2 bound of the buffer the output lands in,
     * without a pass over it: the ConvTranspose forward (store_mode 1) on every split-bf16 kernel, store_mode 0
     * convs where scd_igemm_arith reports the halo16 / gather16 h2 path (the decoder's concat-gradient data grad).
     * NULL = off. */
    float *dst_bound;
    int32_t math;  /* enum scd_conv_math: the arithmetic of this launch */
    uint32_t tune; /* SCD_TUNE_* kernel-variant bits, 0 = defaults */
    /* ABI 9, optional (needs dst_bound): a device float whose value also enters dst_bound, folded in by the launch
     * itself -- seeds the bound of a buffer that holds another operand too (the decoder's concat: the skip's bound
     * and the ConvTranspose output's max) without a copy launch.  NULL = off. */
    const float *dst_bound_seed;
} scd_igemm_t;

int scd_conv_igemm(const scd_igemm_t *d, scd_stream_t stream);
int scd_igemm_arith(const scd_igemm_t *d); /* see enum scd_conv_math */
/* Tiles (and *tile_pixels) of the fused BatchNorm-backward partial sums for `d`, 0 if not available. */
int scd_igemm_bn_bwd_tiles(const scd_igemm_t *d, int32_t *tile_pixels);
/* 1 if the kernel scd_conv_igemm would run for `d` applies the in_scale/in_shift input transform, else 0. */
int scd_igemm_input_bn_supported(const scd_igemm_t *d);
/* Number of statistic tiles scd_conv_igemm would write for `d` (0: no fused statistics for this shape or
 * arithmetic, use scd_bn_train_stats); *tile_pixels receives the pixels per tile. */
int scd_igemm_stat_tiles(const scd_igemm_t *d, int32_t *tile_pixels);

/* ---------------------------------------------------------------------------------------------
 * Weight gradient (split-K implicit GEMM on MFMA), deterministic two-stage reduction.
 *   slab[s][r][t*src.c + c] = sum_{m in split s} rows[m, r] * src[img, oy*stride+dy[t], ox*stride+dx[t], c]
 *   m = (img, oy, ox) over rows.n x rows.h x rows.w.
 * Conv2d 3x3: rows = dY, src = X (taps -1..1).  ConvTranspose2d: rows = X, src = dOut (stride 2, taps 0..1).
 * The Siamese shared encoder runs both branches as one 2B batch, so the two-branch weight-grad
 * accumulation (networks.py:141-145 shared inc/encoder) is the K-sum itself.
 * replaces: the weight-grad half of aten::convolution_backward.
 * ------------------------------------------------------------------------------------------- */
typedef struct scd_wgrad {
    scd_nhwc_t rows;
    scd_nhwc_t src;
    int32_t stride;
    int32_t ntaps;
    int8_t dy[9], dx[9];
    /* Optional fused transform of src (as scd_igemm_t.in_scale): src elements of image img, channel c
     * are read as max(s * src_scale[g*src.c + c] + src_shift[g*src.c + c], 0), g = img / (src.n / src_nseg).
     * NULL = off.  Only where scd_wgrad_src_bn_supported() returns 1. */
    const float *src_scale;
    const float *src_shift;
    int32_t src_nseg;
    /* math == SCD_MATH_H2 only: device floats bounding |rows| and |src| (as read, after the src transform), as
     * scd_igemm_t.src_bound; with rows_y set (below), rows_bound bounds the dY formed from the rows
     * (scd_bn_relu_backward_coef's dy_bound).  With both set the 16x16x32 halo weight grads (64-channel multiples
     * and the 16-channel source) run the fp16 two-term split; else x3. */
    const float *rows_bound;
    const float *src_bound;
    /* Optional fused BatchNorm + ReLU backward of the rows (the input layer's: its dy is read by this weight grad
     * only): `rows` then holds dL/da of a = relu(BN(y)) and every dY element is formed while staging exactly as
     * scd_bn_relu_backward would write it, dy = gamma*invstd*(dz - k1 - xhat*k2), dz = da*[y*scale+shift > 0],
     * xhat = (y-mean)*invstd, so that dy is never written.  rows_y = y (same n, h, w, c as rows); rows_nseg
     * segments of images; save_mean / save_invstd / scale / shift [nseg][c] from the forward; gamma [c] (NULL = 1);
     * coef [nseg][c][2] = {k1, k2} from scd_bn_relu_backward_coef.  rows_y.data NULL = off.  Only where
     * scd_wgrad_rows_bn_supported() returns 1. */
    scd_nhwc_t rows_y;
    int32_t rows_nseg;
    const float *rows_mean, *rows_invstd, *rows_gamma, *rows_scale, *rows_shift, *rows_coef;
    int32_t math;  /* enum scd_conv_math: the arithmetic of this launch */
    uint32_t tune; /* SCD_TUNE_* kernel-variant bits, 0 = defaults */
    /* Optional [nsplit][ntaps * src.c] (nsplit from scd_wgrad_plan): per K-split, the sum over its pixels of every
     * gathered src column (tap t, channel c), summed as staged.  For a ConvTranspose2d weight grad (src = dOut,
     * every output pixel gathered by exactly one tap) scd_wgrad_colsum_finalize turns it into the bias grad, so dOut
     * is not read again for it.  NULL = off.  Only where scd_wgrad_colsum_supported() returns 1. */
    float *src_colsum;
    /* ABI 8, with rows_y set on the 64-channel-multiple halo weight grad: the formed dY is also stored here (same n,
     * h, w, c and dtype as rows), every element once, exactly as scd_bn_relu_backward would write it, and
     * rows_out_bound (device float, may be NULL) is raised to max |dY| stored -- the data grad that reads dY next
     * then needs no BatchNorm-backward apply pass (networks.py:392-397 backward).  rows_out.data NULL = off. */
    scd_nhwc_t rows_out;
    float *rows_out_bound;
} scd_wgrad_t;

/* Number of K-splits the library will use and the slab bytes it needs. */
int scd_wgrad_plan(const scd_wgrad_t *d, int32_t *nsplit, size_t *slab_bytes);
int scd_wgrad_arith(const scd_wgrad_t *d); /* see enum scd_conv_math */
/* Rows of dY (output channels) per workgroup of the halo weight-grad kernel scd_conv_wgrad would run for `d`:
 * 64 or 128 (SCD_TUNE_WGRAD_R64 keeps 64); 0 when `d` takes another weight-grad kernel.  Diagnostic. */
int scd_wgrad_rows_per_block(const scd_wgrad_t *d);
int scd_conv_wgrad(const scd_wgrad_t *d, float *slabs, size_t slab_bytes, scd_stream_t stream);
/* 1 if the weight-grad kernel scd_conv_wgrad would run for `d` applies the src_scale/src_shift transform. */
int scd_wgrad_src_bn_supported(const scd_wgrad_t *d);
/* 1 if it forms the rows through the fused BatchNorm backward (scd_wgrad_t.rows_y): the 16-channel-source kernel,
 * and (ABI 8) the 64-channel-multiple halo weight grad in bf16 or in h2 with 128-row blocks (both bounds set in `d`),
 * at most 2 rows segments per launch; those also store dY (rows_out). */
int scd_wgrad_rows_bn_supported(const scd_wgrad_t *d);
/* Sum the slabs (deterministic fixed-order two-level reduction; the slabs are scratch and are
 * overwritten) and unpack to the parameter layout.
 * mode 0: out OIHW [R][c_valid][3][3]  (slab cols (ky*3+kx)*C + c)
 * mode 1: out ConvT [R][C][2][2]       (slab cols (i*2+j)*C + c)                                  */
int scd_wgrad_finalize(float *slabs, int32_t nsplit, int32_t R, int32_t ntaps, int32_t C, int32_t mode,
                       int32_t c_valid, float *out, scd_stream_t stream);
/* 1 if the weight-grad kernel for `d` writes src_colsum (the generic split-arithmetic kernel), else 0. */
int scd_wgrad_colsum_supported(const scd_wgrad_t *d);
/* out[c] = sum over splits s and taps t of colsum[s][t*C + c], in a fixed order (the ConvTranspose bias grad from
 * scd_wgrad_t.src_colsum; colsum is scratch and is overwritten; ntaps <= 9).  replaces: the bias-grad reduction of
 * convolution_backward for ConvTranspose2d. */
int scd_wgrad_colsum_finalize(float *colsum, int32_t nsplit, int32_t ntaps, int32_t C, float *out,
                              scd_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * BatchNorm2d (train: batch statistics per segment; eval: running statistics) + ReLU.
 * A "segment" is a contiguous range of images normalised as one BN batch: the Siamese encoder runs
 * t1 and t2 as one 2B buffer with nseg = 2, matching the reference's two separate module calls
 * (networks.py:141-145) — per-branch batch statistics and two running-stat updates, t1 first.
 * replaces: aten::native_batch_norm (networks.py:393,396), aten::relu_ (394,397).
 * ------------------------------------------------------------------------------------------- */
size_t scd_bn_workspace_bytes(int32_t n, int32_t h, int32_t w, int32_t c, int32_t nseg);

/* Batch statistics of y per segment -> save_mean/save_invstd [nseg][C], scale/shift [nseg][C]
 * (scale = gamma*invstd, shift = beta - mean*scale).  If update_running != 0 the running buffers are
 * updated once per segment in segment order: r = (1-momentum)*r + momentum*stat (unbiased var). */
/* act_bound (optional, device float, caller-zeroed or holding an earlier bound): raised to an upper bound of
 * |relu(y * scale + shift)| over every segment -- |gamma| sqrt(n - 1) + |beta| per channel and segment of n values
 * (a value lies within sqrt(n - 1) standard deviations of its mean), plus rounding slack.  No pass over y.
 * The operand bound of the SCD_MATH_H2 convs reading this activation (scd_igemm_t.src_bound). */
int scd_bn_train_stats(scd_nhwc_t y, int32_t nseg, const float *gamma, const float *beta, float eps,
                       float momentum, int32_t update_running, float *running_mean, float *running_var,
                       float *save_mean, float *save_invstd, float *scale, float *shift, float *act_bound, void *ws,
                       size_t ws_bytes, scd_stream_t stream);
/* Same outputs as scd_bn_train_stats, from the conv-fused tile records of scd_conv_igemm (stat_rec):
 * ntiles tiles of tile_pixels pixels each, image-major, split evenly into nseg segments. */
size_t scd_bn_tile_stats_workspace_bytes(int32_t ntiles, int32_t c, int32_t nseg);
int scd_bn_stats_from_tiles(const float *tile_rec, int32_t ntiles, int32_t tile_pixels, int32_t c, int32_t nseg,
                            const float *gamma, const float *beta, float eps, float momentum, int32_t update_running,
                            float *running_mean, float *running_var, float *save_mean, float *save_invstd,
                            float *scale, float *shift, float *act_bound, void *ws, size_t ws_bytes,
                            scd_stream_t stream);
/* Eval: scale/shift [C] from running statistics. */
int scd_bn_eval_coeffs(int32_t c, const float *gamma, const float *beta, const float *running_mean,
                       const float *running_var, float eps, float *scale, float *shift, scd_stream_t stream);
/* *bound = max(*bound, max |v|) over the view (atomic integer max on the float bits: order-independent), v = x, or
 * relu(x * scale[g][c] + shift[g][c]) per segment g when scale/shift are given.  The caller zeroes *bound first.
 * The SCD_MATH_H2 operand bound where no producer supplies one (eval-mode BatchNorm, the decoder's upsampled half). */
int scd_absmax_bound(scd_nhwc_t x, int32_t nseg, const float *scale, const float *shift, float *bound,
                     scd_stream_t stream);
/* a = max(y*scale[seg] + shift[seg], 0); nseg = 1 with [C] coefficients in eval mode. */
int scd_bn_relu_apply(scd_nhwc_t y, int32_t nseg, const float *scale, const float *shift, scd_nhwc_t a,
                      scd_stream_t stream);
/* Backward of a = relu(bn(y)) given da:
 *   dz = da * [y*scale+shift > 0]; xhat = (y-mean)*invstd
 *   dgamma = sum dz*xhat, dbeta = sum dz (summed over segments); dy = gamma*invstd*(dz - mean(dz) - xhat*mean(dz*xhat))
 * dbias_prev (optional, [C]) receives sum(dy): the bias grad of the conv that produced y.
 * replaces: native_batch_norm_backward + threshold_backward (+ the conv bias-grad reduction). */
int scd_bn_relu_backward(scd_nhwc_t y, scd_nhwc_t da, int32_t nseg, const float *save_mean,
                         const float *save_invstd, const float *gamma, const float *scale, const float *shift,
                         float *dgamma, float *dbeta, float *dbias_prev, scd_nhwc_t dy, float *dy_bound, void *ws,
                         size_t ws_bytes, scd_stream_t stream);
/* dy_bound (optional, all three backward forms): *dy_bound = max(*dy_bound, max |dy|) as dy is written (the
 * SCD_MATH_H2 bound of the data-grad / weight-grad convs reading dy; caller-zeroed). */

/* scd_bn_relu_backward with the incoming gradient formed on the fly instead of read from a tensor:
 *   da[img] = maxpool_bwd(gy, idx)[img] (if gy.data)  -/+ gskip[img % gskip.n] (skip_mode 1: t1 images
 *   subtract; 0: add) (if gskip.data)
 * -- the operand scd_feature_grad would materialise (same expressions, bit-identical results).  Used by the
 * Siamese encoder's backward (networks.py:147-150, 420): one read of the pooled and difference gradients per
 * pass instead of writing and twice re-reading the level's full-resolution gradient. */
int scd_bn_relu_backward_pooled(scd_nhwc_t y, scd_nhwc_t gy, const uint8_t *idx, scd_nhwc_t gskip,
                                int32_t skip_mode, int32_t nseg, const float *save_mean, const float *save_invstd,
                                const float *gamma, const float *scale, const float *shift, float *dgamma,
                                float *dbeta, float *dbias_prev, scd_nhwc_t dy, float *dy_bound, void *ws,
                                size_t ws_bytes, scd_stream_t stream);
/* scd_bn_relu_backward_pooled with a second skip gradient (the dual-task encoder, networks.py:176-197, whose level
 * activations feed both the difference of decoder_change and, as [a_t2; a_t1], the 2B-image skip batch of
 * decoder_sem):  skip_mode 2 (y.n = 2 * gskip.n, nseg 2):
 *   da[img] = maxpool_bwd(gy, idx)[img] + (sgn(img) * gskip[img % gskip.n] + gskip2[img < n ? img + n : img - n])
 * with sgn as skip_mode 1 and n = gskip.n: bit-identical to the autograd sum of the difference gradient and the two
 * semantic skip slices fed to scd_bn_relu_backward_pooled as one plain skip.  skip_mode 0 / 1 with gskip2 null are
 * scd_bn_relu_backward_pooled. */
int scd_bn_relu_backward_pooled2(scd_nhwc_t y, scd_nhwc_t gy, const uint8_t *idx, scd_nhwc_t gskip,
                                 int32_t skip_mode, scd_nhwc_t gskip2, int32_t nseg, const float *save_mean,
                                 const float *save_invstd, const float *gamma, const float *scale, const float *shift,
                                 float *dgamma, float *dbeta, float *dbias_prev, scd_nhwc_t dy, float *dy_bound,
                                 void *ws, size_t ws_bytes, scd_stream_t stream);
/* scd_bn_relu_backward whose incoming gradient is the 1x1 head's input gradient, formed on the fly:
 *   da[p][c] = sum_o gout[img][o][pix] * w_head[o][c]   (gout NCHW [n][n_out][h][w], n_out <= 4)
 * -- what scd_conv1x1_bwd would write into gx (same fma chain, bit-identical results); y.n * y.h * y.w < 2^31.
 * w_grad (optional, [n_out][C]): also the head's weight grad, sum_p gout[o](p) * relu(fma(y, scale, shift)), from
 * the same partial pass over y (scd_conv1x1_bwd_bn then needs no gw); workspace scd_bn_head_workspace_bytes, else
 * scd_bn_workspace_bytes. */
size_t scd_bn_head_workspace_bytes(int32_t n, int32_t h, int32_t w, int32_t c, int32_t nseg, int32_t n_out);
int scd_bn_relu_backward_head(scd_nhwc_t y, const float *gout, const float *w_head, int32_t n_out, int32_t nseg,
                              const float *save_mean, const float *save_invstd, const float *gamma,
                              const float *scale, const float *shift, float *dgamma, float *dbeta,
                              float *dbias_prev, scd_nhwc_t dy, float *dy_bound, float *w_grad, void *ws,
                              size_t ws_bytes, scd_stream_t stream);
/* scd_bn_relu_backward with the partial sums taken from conv-epilogue tile records (scd_bn_bwd_tiles_t.rec,
 * ntiles tiles, image-major, split evenly into nseg segments) instead of a pass over (y, da). */
int scd_bn_relu_backward_tiles(scd_nhwc_t y, scd_nhwc_t da, int32_t nseg, const float *save_mean,
                               const float *save_invstd, const float *gamma, const float *scale, const float *shift,
                               const float *tile_rec, int32_t ntiles, float *dgamma, float *dbeta,
                               float *dbias_prev, scd_nhwc_t dy, float *dy_bound, void *ws, size_t ws_bytes,
                               scd_stream_t stream);

/* The statistics half of scd_bn_relu_backward(_tiles), for a consumer that forms dy itself (scd_wgrad_t.rows_y):
 * coef[nseg][c][2] = {mean(dz), mean(dz*xhat)} per segment, dgamma, dbeta, and dbias_prev = sum(dy) formed from the
 * sums (zero up to rounding: the BatchNorm removes the mean).  tile_rec = conv-epilogue records as in
 * scd_bn_relu_backward_tiles (da may then be null), or NULL for a partial pass over (y, da).
 * dy_bound (optional, needs da_bound = a device bound of |da|): raised to an upper bound of |dy| over every segment from
 * the statistics alone, |gamma*invstd| (da_bound + |k1| + sqrt(n - 1) |k2|) plus rounding slack -- the SCD_MATH_H2
 * rows bound (scd_wgrad_t.rows_bound) of the weight grad that forms this dy. */
int scd_bn_relu_backward_coef(scd_nhwc_t y, scd_nhwc_t da, int32_t nseg, const float *save_mean,
                              const float *save_invstd, const float *gamma, const float *scale, const float *shift,
                              const float *tile_rec, int32_t ntiles, float *coef, float *dgamma, float *dbeta,
                              float *dbias_prev, const float *da_bound, float *dy_bound, void *ws, size_t ws_bytes,
                              scd_stream_t stream);

/* out[c] = sum over all pixels of x[., c] (ConvTranspose2d bias grad, networks.py:433); workspace as
 * scd_bn_workspace_bytes(n, h, w, c, 1).  replaces: the bias-grad reduction of convolution_backward. */
int scd_channel_sum(scd_nhwc_t x, float *out, void *ws, size_t ws_bytes, scd_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * MaxPool2d(2) (kernel 2, stride 2, floor) with 2-bit argmax per output element (first max wins,
 * NaN propagates, as aten::max_pool2d_with_indices).  replaces: nn.MaxPool2d(2) (networks.py:420).
 * ------------------------------------------------------------------------------------------- */
int scd_maxpool2_fwd(scd_nhwc_t x, scd_nhwc_t y, uint8_t *idx, scd_stream_t stream);
/* The same on max(fma(x, scale[g][c], shift[g][c]), 0), g = img / (n / nseg): the encoder level's
 * BatchNorm-apply + ReLU (networks.py:396-397) fused into the next level's MaxPool2d (networks.py:420), so the
 * activation is not materialised.  Bit-identical to pooling the output of scd_bn_relu_apply. */
int scd_bn_relu_maxpool2_fwd(scd_nhwc_t x, int32_t nseg, const float *scale, const float *shift, scd_nhwc_t y,
                             uint8_t *idx, scd_stream_t stream);

/* Gradient into an encoder feature map (both Siamese branches):
 *   gx[img] = maxpool_bwd(gy, idx)[img]   (if gy.data != NULL)
 *           + sgn(img) * gskip[img % gskip.n]   (if gskip.data != NULL)
 * skip_mode 0: sgn = +1 (plain skip), 1: Siamese difference, sgn = -1 for img < gskip.n (t1), +1 (t2).
 * replaces: max_pool2d_with_indices_backward + the autograd of torch.sub(f_t2, f_t1)
 * (networks.py:147-150) + the skip-half of cat backward (networks.py:449). */
int scd_feature_grad(scd_nhwc_t gy, const uint8_t *idx, scd_nhwc_t gskip, int32_t skip_mode, scd_nhwc_t gx,
                     int32_t accumulate, scd_stream_t stream);

/* d[b] = a[half + b] - a[b], half = d.n (a.n == 2*d.n): f_t2 - f_t1 (networks.py:147-150).  d may be the
 * skip slice [0:C) of the decoder concat buffer (networks.py:449). */
int scd_siamese_diff(scd_nhwc_t a, scd_nhwc_t d, scd_stream_t stream);
/* d = relu(bn_t2(a[n + b])) - relu(bn_t1(a[b])), coefficients [2][c] (t1 segment 0, t2 segment 1): the
 * feature difference (networks.py:147-150) of the encoder's BatchNorm + ReLU outputs without materialising
 * them.  d may be a channel slice of the decoder's concat buffer (networks.py:449). */
int scd_bn_relu_siamese_diff(scd_nhwc_t a, const float *scale, const float *shift, scd_nhwc_t d,
                             scd_stream_t stream);
/* One level's two consumers of relu(BN1(a)) in one pass (even h, w): d as scd_bn_relu_siamese_diff and
 * y, idx = MaxPool2d(2) of both branches as scd_bn_relu_maxpool2_fwd with nseg 2 (networks.py:147-150, 420).
 * Bit-identical to the two calls. */
int scd_bn_relu_pool_diff(scd_nhwc_t a, const float *scale, const float *shift, scd_nhwc_t d, scd_nhwc_t y,
                          uint8_t *idx, scd_stream_t stream);
/* An encoder level's consumers of relu(BN1(a)) in one pass over 2x2 cells (even h, w), coefficients [nseg][c]:
 *   mode 0 (Siamese, nseg 2): scd_bn_relu_pool_diff (o unused);
 *   mode 1 (plain encoder, networks.py:334-343, 449): o = relu(bn(a)) (n images; o may be the skip slice of the
 *          decoder's concat buffer: zero-copy cat), images in nseg segments of n / nseg;
 *   mode 2 (dual-task Siamese, nseg 2, networks.py:176-197): d (n/2 images) as mode 0 and o (n images) =
 *          [relu(bn_t2(a_t2)); relu(bn_t1(a_t1))], the semantic decoder's skip batch (t2 first);
 * plus, when y.data != NULL, y / idx = MaxPool2d(2) of every image of a (networks.py:420).  Modes 1 and 2 derive every
 * output from the stored activation (rounded to the view's type), so they are bit-identical to scd_bn_relu_apply
 * followed by scd_maxpool2_fwd / scd_siamese_diff / copies of the materialised activation. */
int scd_bn_relu_pool_out(scd_nhwc_t a, int32_t nseg, const float *scale, const float *shift, int32_t mode,
                         scd_nhwc_t d, scd_nhwc_t o, scd_nhwc_t y, uint8_t *idx, scd_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * OutConv 1x1 head (networks.py:454-461): out NCHW [n][n_out][h][w] = b + x . w   (n_out <= 4)
 * ------------------------------------------------------------------------------------------- */
int scd_conv1x1_fwd(scd_nhwc_t x, const float *w, const float *b, int32_t n_out, float *out,
                    scd_stream_t stream);
size_t scd_conv1x1_workspace_bytes(scd_nhwc_t x, int32_t n_out);
/* gx (+)= gout . w ; gw = sum gout*x ; gb = sum gout. */
int scd_conv1x1_bwd(scd_nhwc_t x, const float *w, const float *gout, int32_t n_out, scd_nhwc_t gx,
                    int32_t accumulate, float *gw, float *gb, void *ws, size_t ws_bytes, scd_stream_t stream);
/* The head fused with the decoder's last BatchNorm + ReLU (networks.py:380-381 then 457): the head's input
 * x = relu(fma(y, scale[seg], shift[seg])) (per-segment coefficients of scd_bn_train_stats / scd_bn_eval_coeffs,
 * nseg | y.n; bn_relu_apply's expression, bit-identical) is read from the conv output y and never written.
 * _fwd_bn: the forward; _bwd_bn: gw = sum gout*x, gb = sum gout (the input gradient goes through
 * scd_bn_relu_backward_head instead).  Workspace: scd_conv1x1_workspace_bytes(y, n_out). */
int scd_conv1x1_fwd_bn(scd_nhwc_t y, const float *scale, const float *shift, int32_t nseg, const float *w,
                       const float *b, int32_t n_out, float *out, scd_stream_t stream);
int scd_conv1x1_bwd_bn(scd_nhwc_t y, const float *scale, const float *shift, int32_t nseg, const float *w,
                       const float *gout, int32_t n_out, float *gw, float *gb, void *ws, size_t ws_bytes,
                       scd_stream_t stream);
/* The heads over two decoder outputs (the fusion heads, networks.py:119, 258, and WhateverNet's per-stream heads in
 * the same launch): out = b + cat([xa, xb], channel) . w, w [n_out][ya.c + yb.c] (zeros where a head does not read a
 * source), each source read through its own coefficients (both given, or neither: plain activations).  yb.data NULL:
 * scd_conv1x1_fwd_bn.  Bit-identical to the single-source call on the concatenated activation. */
int scd_conv1x1_fwd_bn2(scd_nhwc_t ya, const float *scale_a, const float *shift_a, scd_nhwc_t yb,
                        const float *scale_b, const float *shift_b, int32_t nseg, const float *w, const float *b,
                        int32_t n_out, float *out, scd_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * power_jaccard_loss (utils/loss_functions.py:141-150): p = sigmoid(logit); I = sum p*t;
 * D = sum(p^2 + t^2) - I + 1e-6; loss = 1 - I/D, reduced over the whole batch.
 * sums_out = {I, sum(p^2+t^2), D} (device, float[3]); loss_out device float[1].
 * ------------------------------------------------------------------------------------------- */
/* Fused multi-term form (dual-task and MMCR trainers: train_supervised_dualtask.py:73-85,
 * train_semisupervised.py:78-113).  Tensors are [n_samples][pixels] (B,1,H,W).  Term t is
 * power_jaccard_loss(logits[sel], target[sel]) over the samples sel selects; a term selecting no sample is left
 * out (the reference's `if is_labeled.any()` branches, decided on the device: no host sync, no gathers).
 *   loss = sum_t coef_t * [|sel_t| > 0] * (1 - I_t / D_t)
 * sums (device float[n_terms][4]) = {I, sum(p^2 + t^2), D, |sel|}.  Backward writes dL/dlogits into glogits and,
 * for a soft target (target = sigmoid(target logits), not detached: train_semisupervised.py:107), dL/d(target
 * logits) into gtarget, for the selected samples; zero_unselected bit 0 / bit 1 also writes 0 into glogits /
 * gtarget for the other samples (set it where no other term covers them). */
typedef struct scd_jaccard_term {
    const float *logits;
    const float *target;
    float *glogits;
    float *gtarget;
    float coef;
    int32_t select;          /* 0: all samples, 1: labeled[s] != 0, 2: labeled[s] == 0 */
    int32_t soft_target;
    int32_t zero_unselected; /* bit 0: glogits, bit 1: gtarget */
} scd_jaccard_term_t;
size_t scd_jaccard_multi_workspace_bytes(int32_t n_terms);
int scd_jaccard_multi_fwd(const scd_jaccard_term_t *terms, int32_t n_terms, const uint8_t *labeled, int32_t n_samples,
                          int64_t pixels, float *sums, float *loss, void *ws, size_t ws_bytes, scd_stream_t stream);
int scd_jaccard_multi_bwd(const scd_jaccard_term_t *terms, int32_t n_terms, const uint8_t *labeled, int32_t n_samples,
                          int64_t pixels, const float *sums, const float *gloss, scd_stream_t stream);
/* Exact-DataParallel form (one loss over the batch of all ranks, as nn.DataParallel's gathered-batch loss,
 * utils/networks.py:27 + train_supervised.py:75): after the fwd call every rank all-reduces `sums` (SUM over ranks,
 * caller's collective), then these re-form D = sum(p^2 + t^2) - I + 1e-6 and the loss from the global sums in place
 * of the local ones; the bwd call then takes the global sums.  sums layout as the fwd call writes it. */
int scd_jaccard_multi_loss_from_sums(const scd_jaccard_term_t *terms, int32_t n_terms, float *sums, float *loss,
                                     scd_stream_t stream);
size_t scd_pjaccard_workspace_bytes(int64_t n);
int scd_pjaccard_fwd(const float *logits, const float *target, int64_t n, float *sums_out, float *loss_out,
                     void *ws, size_t ws_bytes, scd_stream_t stream);
int scd_pjaccard_loss_from_sums(float *sums, float *loss, scd_stream_t stream);
/* glogits = gloss * dL/dlogit; if gtarget != NULL also the soft-target grad (MMCR consistency loss,
 * train_semisupervised.py:107, where the target sigma(logits_s2) is not detached). */
int scd_pjaccard_bwd(const float *logits, const float *target, int64_t n, const float *sums,
                     const float *gloss, float *glogits, float *gtarget, scd_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Eval path
 * ------------------------------------------------------------------------------------------- */
/* dst[n, y, x, :] = src[n, y + oy, x + ox, :] where that source pixel exists, else 0 (same n and c).
 * replaces: F.pad(x1, (dX//2, dX - dX//2, dY//2, dY - dY//2)) of Up.forward (networks.py:437-443) when the skip
 * is larger than the upsampled map (oy = -dY//2, ox = -dX//2, dst = the concat buffer's up slice), and the
 * crop of its backward (oy = +dY//2, ox = +dX//2, dst = the ConvT output gradient). */
int scd_window_copy(scd_nhwc_t src, scd_nhwc_t dst, int32_t oy, int32_t ox, scd_stream_t stream);

/* Confusion counts of MultiThresholdMetric.add_sample (utils/metrics.py:22-31) over n flat elements, for
 * n_thr <= 16 thresholds:
 *   p = from_logits ? 1 / (1 + exp(-pred)) : pred      (utils/evaluation.py:25 folded in)
 *   positive(k) = round(p - thr[k] + 0.5) != 0          (fp32, round half to even; NaN counts as positive)
 *   label = truth != 0
 * counts (device int64[1 + 2*n_thr]) = {#label, then per k: #(label & positive(k)), #positive(k)}.  The
 * reference's TP/TN/FP/FN follow exactly from these and n.  Workspace from the query (0 = bad arguments). */
size_t scd_threshold_counts_workspace_bytes(int64_t n, int32_t n_thr);
int scd_threshold_counts(const float *pred, const float *truth, int64_t n, const float *thresholds, int32_t n_thr,
                         int32_t from_logits, int64_t *counts, void *ws, size_t ws_bytes, scd_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Data pipeline: batched on-device augmentations (utils/augmentations.py:6-142).  Tiles are HWC fp32, one per
 * sample and of any size (hw = int32[batch][2] = {H, W}); pointer tables and parameters live on the device.
 * ------------------------------------------------------------------------------------------- */
/* sums[b][k] = sum of labels[b][y : y + crop, x : x + crop] (one-channel HW tiles), yx = int32[batch][ncand][2]:
 * the candidate weights of ImportanceRandomCrop (augmentations.py:129-142). */
int scd_window_label_sums(const float *const *labels, const int32_t *hw, const int32_t *yx, int32_t batch,
                          int32_t ncand, int32_t crop, float *sums, scd_stream_t stream);
/* out[b][c][i][j] (NCHW, crop x crop) = the reference chain on tile src[b] (HWC, `channels` channels):
 * UniformCrop at params[b] = {y0, x0, flip_h, flip_v, rot_k} -> RandomFlip (axis 1, then axis 0) -> RandomRotate
 * (np.rot90 k times, axes (0, 1)) -> ColorShift (clip(x * scale[b][c], 0, 1), in double; scale NULL = off) ->
 * GammaCorrection (clip(x ** gamma[b][c], 0, 1), in double; gamma NULL = off) -> Numpy2Torch (CHW). */
int scd_augment_apply(const float *const *src, const int32_t *hw, int32_t batch, int32_t channels, int32_t crop,
                      const int32_t *params, const double *scale, const double *gamma, float *out,
                      scd_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SCD_H_ */
