// Shared pieces of the implicit-GEMM conv kernels (fp32 MFMA: conv_f32.hip, split-bf16 MFMA: conv_x3.hip).
#pragma once

#include "common.h"

namespace scd {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Loads/stores through the global address space (kernel-arg structs otherwise yield flat_* ops).
__device__ __forceinline__ f32x4 gload4(const float *p) {
    return *(const __attribute__((address_space(1))) f32x4 *)(p);
}
__device__ __forceinline__ void gstore1(float *p, float v) { *(__attribute__((address_space(1))) float *)(p) = v; }
__device__ __forceinline__ f32x4 lload4(const float *p) { return *reinterpret_cast<const f32x4 *>(p); }
__device__ __forceinline__ void lstore4(float *p, f32x4 v) { *reinterpret_cast<f32x4 *>(p) = v; }

// 9 taps packed as signed 4-bit fields.
__device__ __forceinline__ int tap_at(uint64_t packed, int t) {
    int v = int((packed >> (4 * t)) & 15ull);
    return v >= 8 ? v - 16 : v;
}

// XCD-aware block order (guide T1, bijective form): the dispatcher deals consecutive workgroup ids round-robin
// to the 8 XCDs, so id b runs beside ids b+8, b+16, ... under one L2.  Renumbering so that each XCD receives
// a contiguous range of logical tiles keeps neighbouring pixel tiles (which share halo rows through the
// 3x3 taps) and the N-tiles of one pixel tile (which share the gathered A rows) under the same L2.
// Placement only changes speed, never results.
__device__ __forceinline__ uint32_t xcd_swizzle(uint32_t bid, uint32_t nwg) {
    const uint32_t x = bid & 7u, slot = bid >> 3, q = nwg >> 3, r = nwg & 7u;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + slot;
}

// Kernel-variant bits of a launch (scd_igemm_t.tune / scd_wgrad_t.tune, SCD_TUNE_* in scd.h; 0 = defaults).
inline int xcd_remap_enabled(uint32_t tune) { return (tune & SCD_TUNE_NO_XCD_REMAP) ? 0 : 1; }
// Halo-tiled kernels for 3x3 convs (split arithmetics); SCD_TUNE_NO_HALO keeps the per-tap kernels.
inline int halo_enabled(uint32_t tune) { return (tune & SCD_TUNE_NO_HALO) ? 0 : 1; }
// Block order of the halo kernels: N-slowest XCD order (2) unless SCD_TUNE_HALO_ORDER_M / SCD_TUNE_NO_XCD_REMAP.
inline int halo_remap(uint32_t tune) {
    return !xcd_remap_enabled(tune) ? 0 : (tune & SCD_TUNE_HALO_ORDER_M) ? 1 : 2;
}

inline uint64_t pack_taps(const int8_t *v, int n) {
    uint64_t p = 0;
    for (int i = 0; i < n; ++i) p |= uint64_t(uint8_t(v[i]) & 15u) << (4 * i);
    return p;
}

// ------------------------------------------------------------------------------------------------
// igemm
// ------------------------------------------------------------------------------------------------
struct IgemmArgs {
    const float *src;
    int n_img, hs, ws, c, ldc_s;
    int ho, wo, stride, ntaps;
    uint64_t tdy, tdx;
    const float *w;
    int n_out, K;
    const float *bias;
    float *dst;
    int ldc_d, dst_h, dst_w, store_mode, cout;
    int M;
    int grid_m, grid_n, remap;
    const uint16_t *wsplit;  // optional pre-split weight planes [3][n_out*K] (x3 math)
    int64_t wplane;
    float *stat_rec;  // optional fused BN statistics [tile][n_out][2] (halo path)
    uint32_t src_bytes;  // byte extent of src for buffer loads (0 = above 2 GiB: no halo path)
    FastDiv div_hw, div_w;
    const float *in_scale, *in_shift;  // optional fused input BN-apply + ReLU (halo16 path only)
    int in_seg_imgs;                   // images per coefficient segment
    // optional fused BatchNorm-backward partial sums of the output (halo16 path only)
    const float *bb_y;
    int bb_ldy, bb_seg_imgs, bb_ntiles;
    const float *bb_mean, *bb_inv, *bb_scale, *bb_shift;
    float *bb_rec;
    // SCD_MATH_H2: device pointer to an upper bound of |src| as the kernel reads it (after the input transform);
    // the weight planes in wsplit are then the fp16 two-term split with per-row inverse scales (h2_wsplit_bytes)
    const float *src_bound;
    float *dst_bound;  // optional: raised to max |stored output| (x3 / halo16 / gather16 kernels; scd_igemm_t.dst_bound)
    const float *dst_bound_seed;  // optional (ABI 9): a value folded into dst_bound once per launch (bound_seed)
    int math;          // SCD_MATH_* of this launch (scd_igemm_t.math)
    uint32_t tune;     // SCD_TUNE_* bits (scd_igemm_t.tune)
    int sb;            // 1: src, dst and bb_y are bf16 views (ABI 6); the pointers above then address bf16 elements
};

// scd_igemm_t.dst_bound_seed: the first wave of block 0 folds the seed into its max |stored value| before
// wave_max_bound, so dst_bound ends at max(seed, max |output|) with no separate copy or pass.
__device__ __forceinline__ float bound_seed(const IgemmArgs &a) {
    return (a.dst_bound_seed && blockIdx.x == 0 && threadIdx.x < 64) ? fabsf(*a.dst_bound_seed) : 0.f;
}

struct WgradArgs {
    const float *rows;
    int ho, wo, R, ldc_r;
    const float *src;
    int hs, ws, C, ldc_s;
    int stride, ntaps;
    uint64_t tdy, tdx;
    int Ng, M, kchunk;
    int grid_r, grid_j, remap;
    uint32_t rows_bytes, src_bytes;  // extents of rows/src for the buffer-load range check (< 2 GiB)
    int n_img_w;                     // images (halo wgrad: split-K over 2x16 patches of all images)
    float *slabs;
    FastDiv div_hw, div_w, div_c;
    const float *src_scale, *src_shift;  // optional fused src BN-apply + ReLU (halo16 weight grad only)
    int src_seg_imgs;
    const float *rows_bound, *src_bound;  // SCD_MATH_H2: upper bounds of |rows| and |src| (as read), both or neither
    // optional fused BatchNorm + ReLU backward of the rows (the 16-channel-source weight grad, and the halo weight
    // grad in its h2 / bf16 along-c layouts): rows hold dL/da, the kernel forms dy = bn_bwd_dy4(y, da, ...) while
    // staging; coefficients per segment of rows_seg_imgs images
    const float *rows_y;
    int ldc_y;
    uint32_t y_bytes;
    const float *rbn_mean, *rbn_inv, *rbn_gamma, *rbn_scale, *rbn_shift, *rbn_coef;
    int rows_seg_imgs;
    // optional (halo weight grad with rows_y): the formed dy also written here (ldc_o), once, by the blocks of channel
    // tile 0, and rows_out_bound raised to max |dy| stored (the data grad's h2 operand bound)
    void *rows_out;
    int ldc_o;
    float *rows_out_bound;
    int math;       // SCD_MATH_* of this launch (scd_wgrad_t.math)
    uint32_t tune;  // SCD_TUNE_* bits (scd_wgrad_t.tune)
    int sb;         // 1: rows, src and rows_y are bf16 views (ABI 6)
    // optional [split][Ng] column sums of the staged src (generic weight grad: the ConvTranspose bias grad), written
    // by the blocks of row tile 0
    float *colsum;
};

// Split-bf16 ("x3") launchers, conv_x3.hip.  Return false when the shape is not supported by the x3 kernels
// (the caller then runs the fp32-MFMA kernel).
bool launch_igemm_x3(const IgemmArgs &a, hipStream_t s);
// Tiles (and pixels per tile) of the halo path for `a`, or 0 when `a` does not take it.
int halo_stat_tiles(const IgemmArgs &a, int *tile_pixels);
// 16x16x32-MFMA halo igemm (conv_halo16.hip): 0 when `a` does not take it, else its config; launcher.
int halo16_pick(const IgemmArgs &a, bool eligible, int *bm, int *tw);
// 16-channel-source forward (the input layer), conv_halo16.hip.
int halo16_c16_pick(const IgemmArgs &a, bool eligible, int *bm, int *tw);
void launch_halo16_c16(const IgemmArgs &a, int tw, hipStream_t s);
// Whether launch_igemm_x3 would run the halo16 kernel for `a` (the only one with the input transform).
bool igemm_takes_halo16(const IgemmArgs &a);
bool igemm_takes_c16(const IgemmArgs &a);  // igemm_halo16_c16 (16-channel source)
bool igemm_takes_gather16(const IgemmArgs &a);  // igemm_gather16, h2 or bf16 (ConvTranspose forward / data grad)
void launch_halo16(const IgemmArgs &a, int cfg, int tw, hipStream_t s);
// 16x16x32-MFMA halo weight grad (conv_halo16.hip).
const void *wgrad_halo16_fn(int math, uint32_t tune, bool bounded, int rblock);  // bounded: h2 under SCD_MATH_H2
void launch_wgrad_halo16_x3(const WgradArgs &a, dim3 grid, hipStream_t s);
// Whether the halo weight grad forms its rows through the BatchNorm backward (WgradArgs.rows_y) for this arithmetic.
bool wgrad16_rows_bn_ok(int math, uint32_t tune, bool bounded);
// dY rows per block of the halo weight grad (64 or 128; threads = 4 * rows): plan and launch use the same value.
int wgrad16_rblock(int math, uint32_t tune, int R, bool bounded);
// 16-channel-source variant (the input layer), same eligibility otherwise (conv_halo16.hip).
const void *wgrad_halo16_c16_fn(int math, uint32_t tune, bool bounded);
int wgrad_c16_planes(int math, uint32_t tune, bool bounded);  // 4 = h2 (both operands bounded), else as the x3 kernels
void launch_wgrad_halo16_c16(const WgradArgs &a, dim3 grid, hipStream_t s);
// Halo weight grad (3x3 / stride 1 / same size, R and C multiples of 64, maps in 2x16 patches).
inline const void *wgrad_halo_fn(int math, uint32_t tune, bool bounded, int rblock) {
    return wgrad_halo16_fn(math, tune, bounded, rblock);
}
inline int wgrad_halo_rblock(int math, uint32_t tune, int R, bool bounded) {
    return wgrad16_rblock(math, tune, R, bounded);
}
// x3 weight-grad instantiations, indexed like kWgradTiles (conv_f32.hip).
const void *wgrad_x3_fn(int tile_id);
void launch_wgrad_x3(const WgradArgs &a, int tile_id, dim3 grid, dim3 block, hipStream_t s);
// h2 variants of the generic weight grad (both operand bounds; tiles wgrad_x3_h2_tile accepts), conv_x3.hip.
bool wgrad_x3_h2_tile(int tile_id);
void launch_wgrad_x3_h2(const WgradArgs &a, int tile_id, dim3 grid, dim3 block, hipStream_t s);
// bf16 variants of the generic weight grad (the ConvTranspose weight grad under SCD_MATH_BF16), conv_x3.hip.
void launch_wgrad_x3_bf16(const WgradArgs &a, int tile_id, dim3 grid, dim3 block, hipStream_t s);
// bf16 storage (a.sb): the kernels that take bf16 views are the bf16-arithmetic instances of the halo16, c16, gather16
// and generic (ConvTranspose) weight-grad kernels.
inline int elem_size(int sb) { return sb ? 2 : 4; }
// Conv arithmetic of a launch (scd_igemm_t.math / scd_wgrad_t.math; enum scd_conv_math in scd.h).
inline bool math_valid(int m) { return m >= SCD_MATH_F32 && m <= SCD_MATH_H2; }
inline int math_split(int m) { return m != SCD_MATH_F32; }  // split-weight (x3, x5, bf16 or h2) pipeline
// halo16 kernel arithmetic: 3 (x3), 5 (x5: x3 less one product), 1 (bf16), 2 (h2: two-term fp16 split)
inline int math_planes(int m) { return m == SCD_MATH_BF16 ? 1 : m == SCD_MATH_X5 ? 5 : m == SCD_MATH_H2 ? 2 : 3; }
inline int h2_prescale(uint32_t tune) { return (tune & SCD_TUNE_H2_NO_PRESCALE) ? 0 : 1; }
// SCD_MATH_H2 weight splits exist for 3x3 convs (the halo16 kernels) and 1- / 4-tap convs (the ConvTranspose forward
// and data grad, the gather16 kernel) whose source channels are a multiple of 32, and for the 16-channel input layer
// (3x3, the igemm_halo16_c16 kernel); every other conv keeps the x3 split.  wsplit of such a conv is in the h2
// format.
inline bool h2_weight_format(int math, int ntaps, int c) {
    return math == SCD_MATH_H2 && (((ntaps == 9 || ntaps == 1 || ntaps == 4) && c % 32 == 0) || (ntaps == 9 && c == 16));
}
// gather igemm (conv_gather16.hip; h2 or bf16): 0 when `a` does not take it, else 1 + tile id; launcher.
int gather16_pick(const IgemmArgs &a);
void launch_gather16(const IgemmArgs &a, int cfg, hipStream_t s);

}  // namespace scd
