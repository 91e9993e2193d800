// Memory-bound kernels of the Siamese U-Net path (fp32 NHWC) + library info / error handling.
//
// Reference call sites: input hand-off (train_supervised.py:68-69), nn.MaxPool2d(2) (networks.py:420),
// torch.sub(f_t2, f_t1) (networks.py:149), OutConv 1x1 (networks.py:454-461), power_jaccard_loss
// (utils/loss_functions.py:141-150), the parameter layouts of Conv2d / ConvTranspose2d.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>

#include "common.h"

namespace scd {

static thread_local std::string g_err;

void set_error(const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}
void clear_error() { g_err.clear(); }

// bn_f32.hip: sum_p w(p) x[p][c] over all pixels (w = 1 or gout[img][o][pix]).
int weighted_channel_sum(const scd_nhwc_t &x, const float *wgt, int n_out, int o, float *out, void *ws,
                         size_t ws_bytes, hipStream_t s, const float *scale = nullptr, const float *shift = nullptr,
                         int nseg = 1);
size_t weighted_channel_sum_bytes(const scd_nhwc_t &x);

// Row-decomposed grid: x covers the quads of one row (256 per block), y walks rows (grid-stride past 65535).
static dim3 row_grid(int row_quads, int64_t rows) {
    return dim3(unsigned((row_quads + 255) / 256), unsigned(rows < 65535 ? rows : 65535));
}

static int grid_for(int64_t total, int cap = 4096) {
    int64_t b = (total + 255) / 256;
    if (b > cap) b = cap;
    if (b < 1) b = 1;
    return int(b);
}

// ------------------------------------------------------------------------------------------------
// One image per blockIdx.y, 32-bit index math only.  VEC (dc, ldc multiples of 4, 16-byte aligned destination):
// one thread per float4 of the destination, so a wave's stores cover consecutive 16-byte groups of whole pixels;
// the source planes are read 16 pixels x 4 channels per load.  Otherwise one thread per pixel with scalar stores,
// so any channel offset works (the early-fusion t2 bands).
// `bound`: raised to max |value| (one atomic per wave, after the loop every lane reaches).
template <bool VEC, class T>
__global__ void pack_nchw_kernel(const float *__restrict__ src, int c, int hw, int c_begin, int c_count,
                                 T *__restrict__ dst, int dc, int ldc, float *bound) {
    const int img = blockIdx.y;
    const float *s = src + (size_t(img) * c + c_begin) * hw;
    T *d = dst + size_t(img) * hw * ldc;
    float vmax = 0.f;
    if (VEC) {
        const int q4 = dc >> 2;  // float4 groups per pixel
        const int total = hw * q4;
        for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
            const int pix = e / q4, c0 = (e - pix * q4) * 4;
            bnf4 v;
            v.x = c0 + 0 < c_count ? s[size_t(c0 + 0) * hw + pix] : 0.f;
            v.y = c0 + 1 < c_count ? s[size_t(c0 + 1) * hw + pix] : 0.f;
            v.z = c0 + 2 < c_count ? s[size_t(c0 + 2) * hw + pix] : 0.f;
            v.w = c0 + 3 < c_count ? s[size_t(c0 + 3) * hw + pix] : 0.f;
            st4(d + size_t(pix) * ldc + c0, v);
            vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
        }
    } else {
        for (int pix = blockIdx.x * blockDim.x + threadIdx.x; pix < hw; pix += gridDim.x * blockDim.x)
            for (int cc = 0; cc < dc; ++cc) {
                const float v = cc < c_count ? s[size_t(cc) * hw + pix] : 0.f;
                st1(d + size_t(pix) * ldc + cc, v);
                vmax = fmaxf(vmax, fabsf(v));
            }
    }
    if (bound) {  // one atomic per block (the launch caps the blocks under a bound: one hot address)
        __shared__ float wmax[8];
        vmax = fabsf(vmax);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, off));
        if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = vmax;
        __syncthreads();
        if (threadIdx.x == 0) {
            float m = wmax[0];
            for (int k = 1; k < int(blockDim.x >> 6); ++k) m = fmaxf(m, wmax[k]);
            atomic_max_bound(bound, m);
        }
    }
}

__global__ void pack_conv3x3_kernel(const float *__restrict__ w, int co, int ci, int ci_pad, int mode,
                                    float *__restrict__ out) {
    const int64_t total = mode == 0 ? int64_t(co) * 9 * ci_pad : int64_t(ci) * 9 * co;
    for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < total; e += int64_t(gridDim.x) * blockDim.x) {
        if (mode == 0) {  // out[o][t][c]
            const int c = int(e % ci_pad);
            const int t = int((e / ci_pad) % 9);
            const int o = int(e / (int64_t(9) * ci_pad));
            out[e] = c < ci ? w[(int64_t(o) * ci + c) * 9 + t] : 0.f;
        } else {  // out[c][t'][o] = w[o][c][8-t']
            const int o = int(e % co);
            const int t = int((e / co) % 9);
            const int c = int(e / (int64_t(9) * co));
            out[e] = w[(int64_t(o) * ci + c) * 9 + (8 - t)];
        }
    }
}

__global__ void pack_convT_kernel(const float *__restrict__ w, int ci, int co, int mode, float *__restrict__ out) {
    const int64_t total = int64_t(ci) * co * 4;
    for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < total; e += int64_t(gridDim.x) * blockDim.x) {
        if (mode == 0) {  // out[(t*co + o)][c]
            const int c = int(e % ci);
            const int r = int(e / ci);
            const int t = r / co, o = r % co;
            out[e] = w[(int64_t(c) * co + o) * 4 + t];
        } else {  // out[c][t*co + o]
            const int col = int(e % (4 * co));
            const int c = int(e / (4 * co));
            const int t = col / co, o = col % co;
            out[e] = w[(int64_t(c) * co + o) * 4 + t];
        }
    }
}

// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void pool_pick(float v, int k, float &mx, int &idx) {
    if (v > mx || isnan(v)) {
        mx = v;
        idx = k;
    }
}

// Row-decomposed elementwise grids: grid.y walks image rows (img, y), grid.x the channel quads of a row,
// so the per-element index math is 32-bit (one FastDiv by the quads per pixel) instead of 64-bit div/mod.
// BN: the input is a conv output read through its BatchNorm-apply + ReLU, max(fma(x, sc, sh), 0) with the
// coefficients of the image's segment (the expression of bn_relu_apply_kernel, so results are bit-identical
// to pooling the materialised activation).
__device__ __forceinline__ bnf4 bn_relu_f4(bnf4 v, bnf4 sc, bnf4 sh) {
    return bnf4{fmaxf(fmaf(v.x, sc.x, sh.x), 0.f), fmaxf(fmaf(v.y, sc.y, sh.y), 0.f),
                fmaxf(fmaf(v.z, sc.z, sh.z), 0.f), fmaxf(fmaf(v.w, sc.w, sh.w), 0.f)};
}

template <bool BN, class T>
__global__ void maxpool2_fwd_kernel(const T *__restrict__ x, int hx, int wx, int ldx, T *__restrict__ y,
                                   int hy, int wy, int ldy, uint8_t *__restrict__ idx, int C, int rows,
                                   FastDiv div_cq, const float *__restrict__ bsc, const float *__restrict__ bsh,
                                   int seg_imgs) {
    const int cq = C / 4;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= wy * cq) return;
    const int ox = int(fdiv(uint32_t(e), div_cq));
    const int c = (e - ox * cq) * 4;
    for (int row = blockIdx.y; row < rows; row += gridDim.y) {
        const int img = row / hy, oy = row - img * hy;
        const int64_t p = int64_t(row) * wy + ox;  // output pixel
        const T *base = x + ((int64_t(img) * hx + 2 * oy) * wx + 2 * ox) * ldx + c;
        bnf4 v0 = ld4(base);
        bnf4 v1 = ld4(base + ldx);
        bnf4 v2 = ld4(base + int64_t(wx) * ldx);
        bnf4 v3 = ld4(base + int64_t(wx) * ldx + ldx);
        if constexpr (BN) {
            const int o = (img / seg_imgs) * C + c;
            const bnf4 sc = ld4(bsc + o), sh = ld4(bsh + o);
            v0 = bn_relu_f4(v0, sc, sh);
            v1 = bn_relu_f4(v1, sc, sh);
            v2 = bn_relu_f4(v2, sc, sh);
            v3 = bn_relu_f4(v3, sc, sh);
        }
        const float a0[4] = {v0.x, v0.y, v0.z, v0.w}, a1[4] = {v1.x, v1.y, v1.z, v1.w};
        const float a2[4] = {v2.x, v2.y, v2.z, v2.w}, a3[4] = {v3.x, v3.y, v3.z, v3.w};
        float o[4];
        uint32_t packed = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float mx = -INFINITY;
            int id = 0;
            pool_pick(a0[k], 0, mx, id);
            pool_pick(a1[k], 1, mx, id);
            pool_pick(a2[k], 2, mx, id);
            pool_pick(a3[k], 3, mx, id);
            o[k] = mx;
            packed |= uint32_t(id) << (8 * k);
        }
        st4(y + p * ldy + c, bnf4{o[0], o[1], o[2], o[3]});
        *reinterpret_cast<uint32_t *>(idx + p * C + c) = packed;
    }
}

template <class T>
__global__ void feature_grad_kernel(const T *__restrict__ gy, int hy, int wy, int ldgy,
                                    const uint8_t *__restrict__ idx, const T *__restrict__ gs, int gsn, int ldgs,
                                    int skip_mode, T *__restrict__ gx, int hx, int wx, int ldgx, int C,
                                    int accumulate, int rows, FastDiv div_cq) {
    const int cq = C / 4;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= wx * cq) return;
    const int x = int(fdiv(uint32_t(e), div_cq));
    const int c = (e - x * cq) * 4;
    for (int row = blockIdx.y; row < rows; row += gridDim.y) {
        const int img = row / hx, yy = row - img * hx;
        const int64_t p = int64_t(row) * wx + x;
        bnf4 r = {0.f, 0.f, 0.f, 0.f};
        if (gy) {
            const int oy = yy >> 1, ox = x >> 1;
            if (oy < hy && ox < wy) {
                const int64_t q = (int64_t(img) * hy + oy) * wy + ox;
                const uint32_t pk = *reinterpret_cast<const uint32_t *>(idx + q * C + c);
                const bnf4 g = ld4(gy + q * ldgy + c);
                const uint32_t want = uint32_t((yy & 1) * 2 + (x & 1));
                r.x = ((pk >> 0) & 0xff) == want ? g.x : 0.f;
                r.y = ((pk >> 8) & 0xff) == want ? g.y : 0.f;
                r.z = ((pk >> 16) & 0xff) == want ? g.z : 0.f;
                r.w = ((pk >> 24) & 0xff) == want ? g.w : 0.f;
            }
        }
        if (gs) {
            const int simg = img % gsn;
            const float sg = (skip_mode == 1 && img < gsn) ? -1.f : 1.f;
            const bnf4 s = ld4(gs + ((int64_t(simg) * hx + yy) * wx + x) * ldgs + c);
            r.x += sg * s.x;
            r.y += sg * s.y;
            r.z += sg * s.z;
            r.w += sg * s.w;
        }
        T *dst = gx + p * ldgx + c;
        if (accumulate) r += ld4(dst);
        st4(dst, r);
    }
}

template <bool BN, class T>
__global__ void siamese_diff_kernel(const T *__restrict__ a, int lda, T *__restrict__ d, int ldd, int C,
                                    int w, int64_t half_pixels, int rows, FastDiv div_cq,
                                    const float *__restrict__ bsc, const float *__restrict__ bsh) {
    const int cq = C / 4;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= w * cq) return;
    const int x = int(fdiv(uint32_t(e), div_cq));
    const int c = (e - x * cq) * 4;
    for (int row = blockIdx.y; row < rows; row += gridDim.y) {
        const int64_t p = int64_t(row) * w + x;
        bnf4 v1 = ld4(a + p * lda + c);
        bnf4 v2 = ld4(a + (p + half_pixels) * lda + c);
        if constexpr (BN) {  // branch t1 = coefficient segment 0, t2 = segment 1
            v1 = bn_relu_f4(v1, ld4(bsc + c), ld4(bsh + c));
            v2 = bn_relu_f4(v2, ld4(bsc + C + c), ld4(bsh + C + c));
        }
        st4(d + p * ldd + c, v2 - v1);
    }
}

// One encoder level's consumers of relu(BN1(y1)) in one read of y1 (even h, w), per 2x2 cell of the map:
//  MODE 0 (Siamese pairs): the feature difference d[b] = a_t2 - a_t1 at full resolution (into the decoder's concat
//          buffer) -- the expressions of siamese_diff_kernel<true> and maxpool2_fwd_kernel<true>, bit-identical to the
//          two-kernel path;
//  MODE 1 (plain images, `nseg` coefficient segments of seg_imgs images): the activation itself written into o (the
//          decoder's concat buffer slice: the skip of a plain encoder, zero-copy cat);
//  MODE 2 (Siamese pairs, dual-task): d as MODE 0 and o = [a_t2; a_t1] (the semantic decoder's 2B-image skip batch,
//          t2 first as the reference calls decoder_sem(features_t2) first).
// MODEs 1 and 2 form every output from the STORED activation (bf16-rounded under bf16 storage; identity in fp32), so
// they are bit-identical to materialising a with bn_relu_apply and running maxpool2_fwd / siamese_diff / copies on it.
// y / idx null: no pooling (the deepest level).  One thread = one cell quad of one unit (pair or image); rows = units * hy.
template <int MODE, class T>
__global__ void bn_relu_pool_out_kernel(const T *__restrict__ x, int hx, int wx, int ldx, T *__restrict__ y, int hy,
                                        int wy, int ldy, uint8_t *__restrict__ idx, T *__restrict__ d, int ldd,
                                        T *__restrict__ o, int ldo, int C, int units, int seg_imgs, int rows,
                                        FastDiv div_cq, const float *__restrict__ bsc, const float *__restrict__ bsh) {
    constexpr bool PAIR = MODE != 1;
    const int cq = C / 4;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= wy * cq) return;
    const int ox = int(fdiv(uint32_t(e), div_cq));
    const int c = (e - ox * cq) * 4;
    bnf4 sc1 = ld4(bsc + c), sh1 = ld4(bsh + c), sc2 = sc1, sh2 = sh1;
    if constexpr (PAIR) {
        sc2 = ld4(bsc + C + c);
        sh2 = ld4(bsh + C + c);
    }
    const int64_t half = int64_t(units) * hx * wx;  // pixels of one branch (pairs)
    for (int row = blockIdx.y; row < rows; row += gridDim.y) {
        const int b = row / hy, oy = row - b * hy;
        if constexpr (!PAIR) {
            const int so = (b / seg_imgs) * C + c;
            sc1 = ld4(bsc + so);
            sh1 = ld4(bsh + so);
        }
        const int64_t q[4] = {(int64_t(b) * hx + 2 * oy) * wx + 2 * ox, (int64_t(b) * hx + 2 * oy) * wx + 2 * ox + 1,
                              (int64_t(b) * hx + 2 * oy + 1) * wx + 2 * ox,
                              (int64_t(b) * hx + 2 * oy + 1) * wx + 2 * ox + 1};
        bnf4 v1[4], v2[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v1[k] = bn_relu_f4(ld4(x + q[k] * ldx + c), sc1, sh1);
            if constexpr (MODE != 0) v1[k] = stored4(o, v1[k]);
            if constexpr (PAIR) {
                v2[k] = bn_relu_f4(ld4(x + (q[k] + half) * ldx + c), sc2, sh2);
                if constexpr (MODE != 0) v2[k] = stored4(o, v2[k]);
            }
        }
        if constexpr (PAIR) {
#pragma unroll
            for (int k = 0; k < 4; ++k) st4(d + q[k] * ldd + c, v2[k] - v1[k]);
        }
        if constexpr (MODE == 1) {
#pragma unroll
            for (int k = 0; k < 4; ++k) st4(o + q[k] * ldo + c, v1[k]);
        }
        if constexpr (MODE == 2) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                st4(o + q[k] * ldo + c, v2[k]);
                st4(o + (q[k] + half) * ldo + c, v1[k]);
            }
        }
        if (!y) continue;  // uniform
#pragma unroll
        for (int br = 0; br < (PAIR ? 2 : 1); ++br) {
            const bnf4 *v = br ? v2 : v1;
            const float a0[4] = {v[0].x, v[0].y, v[0].z, v[0].w}, a1[4] = {v[1].x, v[1].y, v[1].z, v[1].w};
            const float a2[4] = {v[2].x, v[2].y, v[2].z, v[2].w}, a3[4] = {v[3].x, v[3].y, v[3].z, v[3].w};
            float om[4];
            uint32_t packed = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float mx = -INFINITY;
                int id = 0;
                pool_pick(a0[k], 0, mx, id);
                pool_pick(a1[k], 1, mx, id);
                pool_pick(a2[k], 2, mx, id);
                pool_pick(a3[k], 3, mx, id);
                om[k] = mx;
                packed |= uint32_t(id) << (8 * k);
            }
            const int64_t p = (int64_t(b + br * units) * hy + oy) * wy + ox;
            st4(y + p * ldy + c, bnf4{om[0], om[1], om[2], om[3]});
            *reinterpret_cast<uint32_t *>(idx + p * C + c) = packed;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Wave-cooperative 1x1 conv (the OutConv heads): G = pow2 >= P lanes share a pixel, each a 16-byte piece of CP
// channels (CP = 4 fp32 / 8 bf16 channels: a bf16 lane loads 16 bytes, not 8), partial dots combined with a fixed
// xor-shuffle tree.  Grid-stride over groups of U pixel sets per wave, whose loads are all issued before the arithmetic.
// Two sources (a: pieces [0, pa), b: pieces [pa, P)) read as ONE concatenated input: the fusion heads' cat([x_a, x_b])
// (networks.py:119, 258) without the cat, each source through its own BatchNorm + ReLU coefficients.  The piece order,
// per-lane chains and tree are those of the single-source kernel over the concatenated tensor, so the two-source launch
// is bit-identical to cat + conv.  Several heads over the same sources are one launch: the n_out <= 4 rows of w
// ([n_out][C], zeros where a head does not read a source) -- each source is read once for all heads.
// scale / shift (optional, per source): relu(fma(x, scale, shift)) per segment of pseg pixels
// (bn_relu_apply_kernel's expression), so the decoders' last activations are never written.
template <class T, int CP>
struct HeadPiece;
template <class T>
struct HeadPiece<T, 4> {
    bnf4 v[1];
    __device__ __forceinline__ void load(const T *p) { v[0] = ld4(p); }
};
template <>
struct HeadPiece<bf16_t, 8> {
    bnf4 v[2];
    __device__ __forceinline__ void load(const bf16_t *p) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 r = *reinterpret_cast<const u32x4 *>(p);
        v[0] = unpk_bf16x4(scd_u32x2{r[0], r[1]});
        v[1] = unpk_bf16x4(scd_u32x2{r[2], r[3]});
    }
};

struct HeadSrc {
    const void *x;
    int ld, C;  // row stride and channels of the source
    const float *scale, *shift;
};

// Sum over groups of G lanes (G a power of two <= 64, groups aligned), every lane of a group receiving the total:
// DPP quad permutes and row mirrors inside a row of 16 (VALU ops, no LDS traffic), then cross-row shuffles.  The tree
// adds the nearest lanes first, so a sum over G lanes whose upper G/2 lanes hold +0 equals the sum over the lower G/2.
template <int CTRL>
__device__ __forceinline__ float head_dpp(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float group_sum(float x, int G) {
    if (G >= 2) x += head_dpp<0xB1>(x);   // quad_perm [1,0,3,2]
    if (G >= 4) x += head_dpp<0x4E>(x);   // quad_perm [2,3,0,1]
    if (G >= 8) x += head_dpp<0x141>(x);  // row_half_mirror: i <-> 7 - i within each half row
    if (G >= 16) x += head_dpp<0x140>(x); // row_mirror: i <-> 15 - i
    if (G >= 32) x += __shfl_xor(x, 16, 64);
    if (G >= 64) x += __shfl_xor(x, 32, 64);
    return x;
}

// ONE: every piece has its own lane (P <= G): the lane's coefficients and weights are loaded once per kernel, pixel
// loads are unconditional (clamped to the last pixel; lanes past P read a valid piece and contribute +0).
template <int U, class T, int CP, bool ONE, int NO>
__global__ __launch_bounds__(256) void conv1x1_fwd_kernel(HeadSrc sa, HeadSrc sb, int pa, int P, int C, int hw,
                                                          int64_t npix, const float *__restrict__ w,
                                                          const float *__restrict__ b, int G,
                                                          int64_t pseg, FastDiv fseg, FastDiv fhw,
                                                          float *__restrict__ out) {
    constexpr int NQ = CP / 4;  // channel quads per piece
    constexpr int n_out = NO;   // output channels (heads) of the launch
    const int lane = threadIdx.x & 63;
    const int q = lane % G, pp = lane / G, ppw = 64 / G;
    const int64_t wave = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = (int64_t(gridDim.x) * blockDim.x) >> 6;
    const bool bn = sa.scale != nullptr;  // uniform: both sources or neither
    const bool segs = bn && pseg < npix;  // uniform: more than one coefficient segment
    auto seg_of = [&](int64_t p) -> int64_t {
        return npix < (int64_t(1) << 31) ? int64_t(fdiv(uint32_t(p), fseg)) : p / pseg;
    };
    if constexpr (ONE) {
        const bool act = q < P;
        const int qq = act ? q : P - 1;
        const bool in_a = qq < pa;
        const T *xs = static_cast<const T *>(in_a ? sa.x : sb.x);
        const int ld = in_a ? sa.ld : sb.ld, cs = in_a ? sa.C : sb.C;
        const int ch = (in_a ? qq : qq - pa) * CP;
        const float *scl = in_a ? sa.scale : sb.scale, *shf = in_a ? sa.shift : sb.shift;
        bnf4 wv[4][NQ];
#pragma unroll
        for (int o = 0; o < 4; ++o)
#pragma unroll
            for (int k = 0; k < NQ; ++k)
                wv[o][k] = o < n_out ? ld4(w + int64_t(o) * C + qq * CP + 4 * k) : bnf4{0.f, 0.f, 0.f, 0.f};
        bnf4 sc[NQ], sf[NQ];
        int64_t cur = 0;
        if (bn) {
#pragma unroll
            for (int k = 0; k < NQ; ++k) {
                sc[k] = ld4(scl + ch + 4 * k);
                sf[k] = ld4(shf + ch + 4 * k);
            }
        }
        for (int64_t p0 = wave * ppw * U; p0 < npix; p0 += nwaves * ppw * U) {
            HeadPiece<T, CP> v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                int64_t p = p0 + u * ppw + pp;
                p = p < npix ? p : npix - 1;
                v[u].load(xs + p * ld + ch);
            }
            float s[U][4];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (bn) {
                    if (segs) {  // the lane's coefficients follow its pixel's segment (rarely changes within a wave)
                        int64_t p = p0 + u * ppw + pp;
                        const int64_t sg = seg_of(p < npix ? p : npix - 1);
                        if (sg != cur) {
                            cur = sg;
#pragma unroll
                            for (int k = 0; k < NQ; ++k) {
                                sc[k] = ld4(scl + sg * cs + ch + 4 * k);
                                sf[k] = ld4(shf + sg * cs + ch + 4 * k);
                            }
                        }
                    }
#pragma unroll
                    for (int k = 0; k < NQ; ++k) v[u].v[k] = bn_relu_f4(v[u].v[k], sc[k], sf[k]);
                }
                if (!act) {
#pragma unroll
                    for (int k = 0; k < NQ; ++k) v[u].v[k] = bnf4{0.f, 0.f, 0.f, 0.f};
                }
                // one chain per channel quad, the quads' partial sums added: a 16-byte bf16 piece (two quads) forms
                // exactly what two fp32 lanes and the first step of their tree form, so bf16 storage of
                // bf16-representable values gives the fp32 path's bits
#pragma unroll
                for (int o = 0; o < 4; ++o) {
                    float acc = 0.f;
                    if (o < n_out) {
#pragma unroll
                        for (int k = 0; k < NQ; ++k) {
                            const bnf4 x4 = v[u].v[k], w4 = wv[o][k];
                            const float c4 = fmaf(x4.x, w4.x, fmaf(x4.y, w4.y, fmaf(x4.z, w4.z, fmaf(x4.w, w4.w, 0.f))));
                            acc = k == 0 ? c4 : acc + c4;
                        }
                    }
                    s[u][o] = acc;
                }
            }
#pragma unroll
            for (int o = 0; o < 4; ++o)
                if (o < n_out)
#pragma unroll
                    for (int u = 0; u < U; ++u) s[u][o] = group_sum(s[u][o], G);
            if (q == 0) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int64_t p = p0 + u * ppw + pp;
                    if (p < npix) {
                        const int64_t img = npix < (int64_t(1) << 31) ? int64_t(fdiv(uint32_t(p), fhw)) : p / hw;
                        const int64_t pix = p - img * hw;
#pragma unroll
                        for (int o = 0; o < 4; ++o)
                            if (o < n_out) out[(img * n_out + o) * hw + pix] = s[u][o] + (b ? b[o] : 0.f);
                    }
                }
            }
        }
        return;
    }
    // P > G: each lane walks pieces q, q + G, ...
    for (int64_t p0 = wave * ppw * U; p0 < npix; p0 += nwaves * ppw * U) {
        float s[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int o = 0; o < 4; ++o) s[u][o] = 0.f;
        for (int qq = q; qq < P; qq += G) {
            const bool in_a = qq < pa;  // a select, not a branch: lanes of one pixel may read different sources
            const T *xs = static_cast<const T *>(in_a ? sa.x : sb.x);
            const int ld = in_a ? sa.ld : sb.ld, cs = in_a ? sa.C : sb.C;
            const int ch = (in_a ? qq : qq - pa) * CP;
            HeadPiece<T, CP> v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                int64_t p = p0 + u * ppw + pp;
                p = p < npix ? p : npix - 1;
                v[u].load(xs + p * ld + ch);
            }
            if (bn) {
                const float *scl = in_a ? sa.scale : sb.scale, *shf = in_a ? sa.shift : sb.shift;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    int64_t p = p0 + u * ppw + pp;
                    const int64_t so = (segs ? seg_of(p < npix ? p : npix - 1) : 0) * cs + ch;
#pragma unroll
                    for (int k = 0; k < NQ; ++k)
                        v[u].v[k] = bn_relu_f4(v[u].v[k], ld4(scl + so + 4 * k), ld4(shf + so + 4 * k));
                }
            }
#pragma unroll
            for (int o = 0; o < 4; ++o) {
                if (o < n_out) {
#pragma unroll
                    for (int k = 0; k < NQ; ++k) {
                        const bnf4 wv = ld4(w + int64_t(o) * C + qq * CP + 4 * k);
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            const bnf4 x4 = v[u].v[k];
                            s[u][o] = fmaf(x4.x, wv.x, fmaf(x4.y, wv.y, fmaf(x4.z, wv.z, fmaf(x4.w, wv.w, s[u][o]))));
                        }
                    }
                }
            }
        }
#pragma unroll
        for (int o = 0; o < 4; ++o)
            if (o < n_out)
#pragma unroll
                for (int u = 0; u < U; ++u) s[u][o] = group_sum(s[u][o], G);
        if (q == 0) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t p = p0 + u * ppw + pp;
                if (p < npix) {
                    const int64_t img = npix < (int64_t(1) << 31) ? int64_t(fdiv(uint32_t(p), fhw)) : p / hw;
                    const int64_t pix = p - img * hw;
#pragma unroll
                    for (int o = 0; o < 4; ++o)
                        if (o < n_out) out[(img * n_out + o) * hw + pix] = s[u][o] + (b ? b[o] : 0.f);
                }
            }
        }
    }
}

template <class T>
__global__ void conv1x1_bwd_dx_kernel(const float *__restrict__ gout, int n_out, int hw, const float *__restrict__ w,
                                      T *__restrict__ gx, int ldgx, int C, int accumulate, int64_t total, FastDiv fcq,
                                      FastDiv fhw) {
    const int cq = C / 4;
    // below 2^31 elements the (pixel, quad) and (image, pixel) splits are multiply-shifts: four int64 divisions per
    // element made this pass VALU-bound (~1.5 TB/s)
    const bool small = total < (int64_t(1) << 31);
    for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < total; e += int64_t(gridDim.x) * blockDim.x) {
        int c;
        int64_t p, img, pix;
        if (small) {
            const uint32_t pe = fdiv(uint32_t(e), fcq), ie = fdiv(pe, fhw);
            c = int(uint32_t(e) - pe * uint32_t(cq)) * 4;
            p = pe;
            img = ie;
            pix = int64_t(pe - ie * uint32_t(hw));
        } else {
            c = int(e % cq) * 4;
            p = e / cq;
            img = p / hw;
            pix = p % hw;
        }
        bnf4 r = {0.f, 0.f, 0.f, 0.f};
        for (int o = 0; o < n_out; ++o) {
            const float g = gout[(img * n_out + o) * hw + pix];
            const float *wr = w + int64_t(o) * C + c;
            r.x = fmaf(g, wr[0], r.x);
            r.y = fmaf(g, wr[1], r.y);
            r.z = fmaf(g, wr[2], r.z);
            r.w = fmaf(g, wr[3], r.w);
        }
        T *dst = gx + p * ldgx + c;
        if (accumulate) r += ld4(dst);
        st4(dst, r);
    }
}

// partial sums of gout per output channel: rec[o][block]
__global__ __launch_bounds__(256) void conv1x1_bwd_db_partial(const float *__restrict__ gout, int n_out, int hw,
                                                              int64_t npix, float *__restrict__ rec) {
    __shared__ float sh[256];
    const int o = blockIdx.y;
    float s = 0.f;
    for (int64_t p = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; p < npix; p += int64_t(gridDim.x) * blockDim.x) {
        const int64_t img = p / hw, pix = p - img * hw;
        s += gout[(img * n_out + o) * hw + pix];
    }
    sh[threadIdx.x] = s;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (threadIdx.x < off) sh[threadIdx.x] += sh[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) rec[size_t(o) * gridDim.x + blockIdx.x] = sh[0];
}

// out[i] = sum_k rec[i][k] in double with a fixed tree; one workgroup per output
__global__ __launch_bounds__(256) void sum_rows_block(const float *__restrict__ rec, int n, float *__restrict__ out) {
    __shared__ double sh[256];
    const int t = threadIdx.x;
    double s = 0;
    for (int k = t; k < n; k += 256) s += rec[size_t(blockIdx.x) * n + k];
    sh[t] = s;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (t < off) sh[t] += sh[t + off];
        __syncthreads();
    }
    if (t == 0) out[blockIdx.x] = float(sh[0]);
}

// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

// rec[0][block] = sum p*t, rec[1][block] = sum p^2 + t^2
__global__ __launch_bounds__(256) void pjaccard_partial(const float *__restrict__ logits, const float *__restrict__ t,
                                                        int64_t n, float *__restrict__ rec) {
    __shared__ float s1[256], s2[256];
    float a = 0.f, b = 0.f;
    for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
        const float p = sigmoidf_(logits[i]);
        const float tt = t[i];
        a = fmaf(p, tt, a);
        b += p * p + tt * tt;
    }
    s1[threadIdx.x] = a;
    s2[threadIdx.x] = b;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (threadIdx.x < off) {
            s1[threadIdx.x] += s1[threadIdx.x + off];
            s2[threadIdx.x] += s2[threadIdx.x + off];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        rec[blockIdx.x] = s1[0];
        rec[gridDim.x + blockIdx.x] = s2[0];
    }
}

__global__ __launch_bounds__(256) void pjaccard_finalize(const float *__restrict__ rec, int nrec, float *sums,
                                                         float *loss) {
    __shared__ double sI[256], sA[256];
    const int t = threadIdx.x;
    double I = 0, A = 0;
    for (int k = t; k < nrec; k += 256) {
        I += rec[k];
        A += rec[nrec + k];
    }
    sI[t] = I;
    sA[t] = A;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (t < off) {
            sI[t] += sI[t + off];
            sA[t] += sA[t + off];
        }
        __syncthreads();
    }
    if (t == 0) {
        const float If = float(sI[0]);
        const float Df = float(sA[0]) - If + 1e-6f;
        sums[0] = If;
        sums[1] = float(sA[0]);
        sums[2] = Df;
        loss[0] = 1.f - If / Df;
    }
}

__global__ void pjaccard_bwd_kernel(const float *__restrict__ logits, const float *__restrict__ t, int64_t n,
                                    const float *__restrict__ sums, const float *__restrict__ gloss,
                                    float *__restrict__ gl, float *__restrict__ gt) {
    const float I = sums[0], D = sums[2];
    const float g = gloss ? gloss[0] : 1.f;
    const float invD2 = 1.f / (D * D);
    for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
        const float p = sigmoidf_(logits[i]);
        const float tt = t[i];
        const float dLdp = -(tt * D - I * (2.f * p - tt)) * invD2;
        gl[i] = g * dLdp * (p * (1.f - p));
        if (gt) gt[i] = g * (-(p * D - I * (2.f * tt - p)) * invD2);
    }
}

}  // namespace scd

using namespace scd;

// ------------------------------------------------------------------------------------------------
extern "C" const char *scd_version(void) { return "libscd 0.9.0 (gfx950, ABI 9: conv launches seed a bound with another buffer's bound)"; }
extern "C" const char *scd_last_error(void) { return g_err.c_str(); }

extern "C" int scd_device_check(int device) {
    clear_error();
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) {
        set_error("hipGetDeviceProperties(%d): %s", device, hipGetErrorString(e));
        return SCD_ERR_DEVICE;
    }
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_error("device %d is %s, libscd is built for gfx950 only", device, prop.gcnArchName);
        return SCD_ERR_DEVICE;
    }
    return SCD_OK;
}

extern "C" int scd_pack_nchw(const float *src, int32_t n, int32_t c, int32_t h, int32_t w, int32_t c_begin,
                             int32_t c_count, scd_nhwc_t dst, float *bound, scd_stream_t stream) {
    clear_error();
    // dst may start at any channel offset (scalar stores): only shape checks here.
    if (!src || !dst.data || n != dst.n || h != dst.h || w != dst.w || dst.c < 1 || dst.ldc < dst.c || c_begin < 0 ||
        c_count < 0 || c_begin + c_count > c || c_count > dst.c) {
        set_error("pack_nchw: bad arguments");
        return SCD_ERR_ARG;
    }
    const int hw = h * w;
    if (n > 65535 || int64_t(h) * w > (int64_t(1) << 30)) {
        set_error("pack_nchw: n must be <= 65535 and h*w <= 2^30");
        return SCD_ERR_ARG;
    }
    if (n == 0 || hw == 0) return SCD_OK;
    const bool vec = dst.c % 4 == 0 && dst.ldc % 4 == 0 &&
                     (reinterpret_cast<uintptr_t>(dst.data) & (is_bf16(dst) ? 7 : 15)) == 0;
    const int64_t per_img = vec ? int64_t(hw) * (dst.c / 4) : hw;
    if (per_img >= (int64_t(1) << 31)) {
        set_error("pack_nchw: image too large");
        return SCD_ERR_ARG;
    }
    // under a bound at most 64 blocks per image (each block's maximum goes to one address by atomic)
    const dim3 grid(unsigned(std::min<int64_t>((per_img + 255) / 256, bound ? 64 : 4096)), unsigned(n));
    SCD_WITH_T(dst.dtype, T, {
        T *d = view_ptr<T>(dst);
        if (vec)
            hipLaunchKernelGGL((pack_nchw_kernel<true, T>), grid, dim3(256), 0, as_stream(stream), src, c, hw, c_begin,
                               c_count, d, dst.c, dst.ldc, bound);
        else
            hipLaunchKernelGGL((pack_nchw_kernel<false, T>), grid, dim3(256), 0, as_stream(stream), src, c, hw, c_begin,
                               c_count, d, dst.c, dst.ldc, bound);
    });
    return launch_status("scd_pack_nchw");
}

extern "C" int scd_pack_conv3x3(const float *w, int32_t co, int32_t ci, int32_t ci_pad, int32_t mode, float *out,
                                scd_stream_t stream) {
    clear_error();
    if (!w || !out || co < 1 || ci < 1 || ci_pad < ci || (mode != 0 && mode != 1)) {
        set_error("pack_conv3x3: bad arguments");
        return SCD_ERR_ARG;
    }
    const int64_t total = mode == 0 ? int64_t(co) * 9 * ci_pad : int64_t(ci) * 9 * co;
    hipLaunchKernelGGL(pack_conv3x3_kernel, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), w, co, ci, ci_pad,
                       mode, out);
    return launch_status("scd_pack_conv3x3");
}

extern "C" int scd_pack_convT2x2(const float *w, int32_t ci, int32_t co, int32_t mode, float *out,
                                 scd_stream_t stream) {
    clear_error();
    if (!w || !out || co < 1 || ci < 1 || (mode != 0 && mode != 1)) {
        set_error("pack_convT2x2: bad arguments");
        return SCD_ERR_ARG;
    }
    hipLaunchKernelGGL(pack_convT_kernel, dim3(grid_for(int64_t(ci) * co * 4)), dim3(256), 0, as_stream(stream), w, ci,
                       co, mode, out);
    return launch_status("scd_pack_convT2x2");
}

extern "C" int scd_maxpool2_fwd(scd_nhwc_t x, scd_nhwc_t y, uint8_t *idx, scd_stream_t stream) {
    clear_error();
    SCD_TRY(check_view(x, "maxpool.x"));
    SCD_TRY(check_view(y, "maxpool.y"));
    if (!idx || y.n != x.n || y.c != x.c || y.h != x.h / 2 || y.w != x.w / 2 || (reinterpret_cast<uintptr_t>(idx) & 3)) {
        set_error("maxpool2_fwd: y must be (n, h/2, w/2, c); idx 4-byte aligned");
        return SCD_ERR_ARG;
    }
    const int64_t rows = int64_t(y.n) * y.h;
    const int dt = common_dtype("maxpool2_fwd", {&x, &y});
    if (dt < 0) return SCD_ERR_ARG;
    SCD_WITH_T(dt, T,
               hipLaunchKernelGGL((maxpool2_fwd_kernel<false, T>), row_grid(y.w * (y.c / 4), rows), dim3(256), 0,
                                  as_stream(stream), view_ptr<const T>(x), x.h, x.w, x.ldc, view_ptr<T>(y), y.h, y.w,
                                  y.ldc, idx, y.c, int(rows), make_fastdiv(uint32_t(y.c / 4)), nullptr, nullptr, 1));
    return launch_status("scd_maxpool2_fwd");
}

extern "C" int scd_bn_relu_maxpool2_fwd(scd_nhwc_t x, int32_t nseg, const float *scale, const float *shift,
                                        scd_nhwc_t y, uint8_t *idx, scd_stream_t stream) {
    clear_error();
    SCD_TRY(check_view(x, "bn_relu_maxpool.x"));
    SCD_TRY(check_view(y, "bn_relu_maxpool.y"));
    if (!idx || !scale || !shift || nseg < 1 || x.n % nseg || y.n != x.n || y.c != x.c || y.h != x.h / 2 ||
        y.w != x.w / 2 || y.h < 1 || y.w < 1 || !aligned16(scale) || !aligned16(shift)) {
        set_error("bn_relu_maxpool2_fwd: y must be (n, h/2, w/2, c) with idx, nseg | n, aligned coefficients");
        return SCD_ERR_ARG;
    }
    const int64_t rows = int64_t(y.n) * y.h;
    const int dt = common_dtype("bn_relu_maxpool2_fwd", {&x, &y});
    if (dt < 0) return SCD_ERR_ARG;
    SCD_WITH_T(dt, T,
               hipLaunchKernelGGL((maxpool2_fwd_kernel<true, T>), row_grid(y.w * (y.c / 4), rows), dim3(256), 0,
                                  as_stream(stream), view_ptr<const T>(x), x.h, x.w, x.ldc, view_ptr<T>(y), y.h, y.w,
                                  y.ldc, idx, y.c, int(rows), make_fastdiv(uint32_t(y.c / 4)), scale, shift,
                                  x.n / nseg));
    return launch_status("scd_bn_relu_maxpool2_fwd");
}

extern "C" int scd_feature_grad(scd_nhwc_t gy, const uint8_t *idx, scd_nhwc_t gskip, int32_t skip_mode,
                                scd_nhwc_t gx, int32_t accumulate, scd_stream_t stream) {
    clear_error();
    SCD_TRY(check_view(gx, "feature_grad.gx"));
    SCD_TRY(check_view(gy, "feature_grad.gy", true));
    SCD_TRY(check_view(gskip, "feature_grad.gskip", true));
    if (gy.data) {
        if (!idx || gy.n != gx.n || gy.c != gx.c || gy.h != gx.h / 2 || gy.w != gx.w / 2) {
            set_error("feature_grad: gy must be (n, h/2, w/2, c) with idx");
            return SCD_ERR_ARG;
        }
    }
    if (gskip.data) {
        if (gskip.c != gx.c || gskip.h != gx.h || gskip.w != gx.w || gx.n % gskip.n ||
            (skip_mode == 1 && gx.n != 2 * gskip.n) || (skip_mode != 0 && skip_mode != 1)) {
            set_error("feature_grad: gskip shape/mode mismatch");
            return SCD_ERR_ARG;
        }
    }
    const int64_t rows = int64_t(gx.n) * gx.h;
    const int dt = common_dtype("feature_grad", {&gy, &gskip, &gx});
    if (dt < 0) return SCD_ERR_ARG;
    SCD_WITH_T(dt, T,
               hipLaunchKernelGGL(feature_grad_kernel<T>, row_grid(gx.w * (gx.c / 4), rows), dim3(256), 0,
                                  as_stream(stream), view_ptr<const T>(gy), gy.h, gy.w, gy.ldc, idx,
                                  view_ptr<const T>(gskip), gskip.n > 0 ? gskip.n : 1, gskip.ldc, skip_mode,
                                  view_ptr<T>(gx), gx.h, gx.w, gx.ldc, gx.c, accumulate, int(rows),
                                  make_fastdiv(uint32_t(gx.c / 4))));
    return launch_status("scd_feature_grad");
}

extern "C" int scd_siamese_diff(scd_nhwc_t a, scd_nhwc_t d, scd_stream_t stream) {
    clear_error();
    SCD_TRY(check_view(a, "diff.a"));
    SCD_TRY(check_view(d, "diff.d"));
    if (a.n != 2 * d.n || a.h != d.h || a.w != d.w || a.c != d.c) {
        set_error("siamese_diff: a must be (2n, h, w, c) of d");
        return SCD_ERR_ARG;
    }
    const int64_t rows = int64_t(d.n) * d.h;
    const int dt = common_dtype("siamese_diff", {&a, &d});
    if (dt < 0) return SCD_ERR_ARG;
    SCD_WITH_T(dt, T,
               hipLaunchKernelGGL((siamese_diff_kernel<false, T>), row_grid(d.w * (d.c / 4), rows), dim3(256), 0,
                                  as_stream(stream), view_ptr<const T>(a), a.ldc, view_ptr<T>(d), d.ldc, d.c, d.w,
                                  pixels(d), int(rows), make_fastdiv(uint32_t(d.c / 4)), nullptr, nullptr));
    return launch_status("scd_siamese_diff");
}

extern "C" int scd_bn_relu_siamese_diff(scd_nhwc_t a, const float *scale, const float *shift, scd_nhwc_t d,
                                        scd_stream_t stream) {
    clear_error();
    SCD_TRY(check_view(a, "bn_relu_diff.a"));
    SCD_TRY(check_view(d, "bn_relu_diff.d"));
    if (a.n != 2 * d.n || a.h != d.h || a.w != d.w || a.c != d.c || !scale || !shift || !aligned16(scale) ||
        !aligned16(shift)) {
        set_error("bn_relu_siamese_diff: a must be (2n, h, w, c) of d, aligned coefficients [2][c]");
        return SCD_ERR_ARG;
    }
    const int64_t rows = int64_t(d.n) * d.h;
    const int dt = common_dtype("bn_relu_siamese_diff", {&a, &d});
    if (dt < 0) return SCD_ERR_ARG;
    SCD_WITH_T(dt, T,
               hipLaunchKernelGGL((siamese_diff_kernel<true, T>), row_grid(d.w * (d.c / 4), rows), dim3(256), 0,
                                  as_stream(stream), view_ptr<const T>(a), a.ldc, view_ptr<T>(d), d.ldc, d.c, d.w,
                                  pixels(d), int(rows), make_fastdiv(uint32_t(d.c / 4)), scale, shift));
    return launch_status("scd_bn_relu_siamese_diff");
}

namespace scd {
// One launch of the head kernel over one or two sources (b.data null: one).  16-byte bf16 pieces when every source
// allows them (channels and row stride multiples of 8, 16-byte aligned data), else channel quads.
static int conv1x1_fwd_run(const scd_nhwc_t &a, const float *sca, const float *sha, const scd_nhwc_t &b,
                           const float *scb, const float *shb, int nseg, const float *w, const float *bias, int n_out,
                           float *out, hipStream_t s) {
    const int64_t npix = pixels(a);
    const bool two = b.data != nullptr;
    const int C = a.c + (two ? b.c : 0);
    auto wide_ok = [](const scd_nhwc_t &v) { return is_bf16(v) && v.c % 8 == 0 && v.ldc % 8 == 0 && aligned16(v.data); };
    const bool wide = wide_ok(a) && (!two || wide_ok(b));
    const int CP = wide ? 8 : 4;
    const int P = C / CP, pa = a.c / CP;
    int G = 1;
    while (G < P && G < 64) G *= 2;
    constexpr int U = 4;
    const int64_t waves = (npix + (64 / G) * U - 1) / ((64 / G) * U);
    int blocks = int((waves + 3) / 4);
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    const HeadSrc A{a.data, a.ldc, a.c, sca, sha};
    const HeadSrc B{two ? b.data : a.data, two ? b.ldc : a.ldc, two ? b.c : a.c, two ? scb : sca, two ? shb : sha};
    const FastDiv fseg = make_fastdiv(uint32_t(npix / nseg > 0 ? npix / nseg : 1));
    const FastDiv fhw = make_fastdiv(uint32_t(a.h * a.w > 0 ? a.h * a.w : 1));
    const bool one = P <= G;
#define SCD_HEAD_LAUNCH(T_, CP_, ONE_, NO_)                                                                              \
    hipLaunchKernelGGL((conv1x1_fwd_kernel<U, T_, CP_, ONE_, NO_>), dim3(blocks), dim3(256), 0, s, A, B, pa, P, C,       \
                       a.h * a.w, npix, w, bias, G, npix / nseg, fseg, fhw, out)
#define SCD_HEAD_NO(T_, CP_, ONE_)                  \
    switch (n_out) {                                \
        case 1: SCD_HEAD_LAUNCH(T_, CP_, ONE_, 1); break; \
        case 2: SCD_HEAD_LAUNCH(T_, CP_, ONE_, 2); break; \
        case 3: SCD_HEAD_LAUNCH(T_, CP_, ONE_, 3); break; \
        default: SCD_HEAD_LAUNCH(T_, CP_, ONE_, 4); break; \
    }
    if (wide) {
        if (one) {
            SCD_HEAD_NO(bf16_t, 8, true);
        } else {
            SCD_HEAD_NO(bf16_t, 8, false);
        }
    } else {
        SCD_WITH_T(a.dtype, T, {
            if (one) {
                SCD_HEAD_NO(T, 4, true);
            } else {
                SCD_HEAD_NO(T, 4, false);
            }
        });
    }
#undef SCD_HEAD_NO
#undef SCD_HEAD_LAUNCH
    return launch_status("scd_conv1x1_fwd");
}

template <int MODE>
static int pool_out_run(const scd_nhwc_t &a, const float *scale, const float *shift, int nseg, const scd_nhwc_t &d,
                        const scd_nhwc_t &o, const scd_nhwc_t &y, uint8_t *idx, int dt, hipStream_t s) {
    const int units = MODE == 1 ? a.n : a.n / 2;
    const int hy = a.h / 2, wy = a.w / 2;
    const int64_t rows = int64_t(units) * hy;
    SCD_WITH_T(dt, T,
               hipLaunchKernelGGL((bn_relu_pool_out_kernel<MODE, T>), row_grid(wy * (a.c / 4), rows), dim3(256), 0, s,
                                  view_ptr<const T>(a), a.h, a.w, a.ldc, view_ptr<T>(y), hy, wy, y.ldc, idx,
                                  view_ptr<T>(d), d.ldc, view_ptr<T>(o), o.ldc, a.c, units, a.n / nseg, int(rows),
                                  make_fastdiv(uint32_t(a.c / 4)), scale, shift));
    return launch_status("scd_bn_relu_pool_out");
}
}  // namespace scd

extern "C" int scd_conv1x1_fwd(scd_nhwc_t x, const float *w, const float *b, int32_t n_out, float *out,
                               scd_stream_t stream) {
    clear_error();
    SCD_TRY(check_view(x, "conv1x1.x"));
    if (!w || !out || n_out < 1 || n_out > 4) {
        set_error("conv1x1_fwd: bad arguments (n_out in [1,4])");
        return SCD_ERR_ARG;
    }
    return conv1x1_fwd_run(x, nullptr, nullptr, scd_nhwc_t{}, nullptr, nullptr, 1, w, b, n_out, out,
                           as_stream(stream));
}

extern "C" int scd_conv1x1_fwd_bn(scd_nhwc_t y, const float *scale, const float *shift, int32_t nseg, const float *w,
                                  const float *b, int32_t n_out, float *out, scd_stream_t stream) {
    clear_error();
    SCD_TRY(check_view(y, "conv1x1_bn.y"));
    if (!w || !out || !scale || !shift || n_out < 1 || n_out > 4 || nseg < 1 || y.n % nseg ||
        !aligned16(scale) || !aligned16(shift)) {
        set_error("conv1x1_fwd_bn: bad arguments (n_out in [1,4], 16-byte aligned scale/shift, nseg | n)");
        return SCD_ERR_ARG;
    }
    return conv1x1_fwd_run(y, scale, shift, scd_nhwc_t{}, nullptr, nullptr, nseg, w, b, n_out, out,
                           as_stream(stream));
}

extern "C" int scd_conv1x1_fwd_bn2(scd_nhwc_t ya, const float *scale_a, const float *shift_a, scd_nhwc_t yb,
                                   const float *scale_b, const float *shift_b, int32_t nseg, const float *w,
                                   const float *b, int32_t n_out, float *out, scd_stream_t stream) {
    clear_error();
    SCD_TRY(check_view(ya, "conv1x1_bn2.ya"));
    SCD_TRY(check_view(yb, "conv1x1_bn2.yb", true));
    const bool bn = scale_a != nullptr;
    if (!w || !out || n_out < 1 || n_out > 4 || nseg < 1 || ya.n % nseg ||
        (bn && (!shift_a || !aligned16(scale_a) || !aligned16(shift_a))) ||
        (yb.data && (yb.n != ya.n || yb.h != ya.h || yb.w != ya.w ||
                     (bn != (scale_b != nullptr)) || (bn && (!shift_b || !aligned16(scale_b) || !aligned16(shift_b)))))) {
        set_error("conv1x1_fwd_bn2: bad arguments (n_out in [1,4]; ya, yb of one (n, h, w); coefficients for both "
                  "sources or neither, 16-byte aligned; nseg | n)");
        return SCD_ERR_ARG;
    }
    if (common_dtype("conv1x1_fwd_bn2", {&ya, &yb}) < 0) return SCD_ERR_ARG;
    return conv1x1_fwd_run(ya, scale_a, shift_a, yb, scale_b, shift_b, nseg, w, b, n_out, out, as_stream(stream));
}

extern "C" size_t scd_conv1x1_workspace_bytes(scd_nhwc_t x, int32_t n_out) {
    return weighted_channel_sum_bytes(x) + size_t(1024) * n_out * sizeof(float) + 256;
}

extern "C" int scd_conv1x1_bwd(scd_nhwc_t x, const float *w, const float *gout, int32_t n_out, scd_nhwc_t gx,
                               int32_t accumulate, float *gw, float *gb, void *ws, size_t ws_bytes,
                               scd_stream_t stream) {
    clear_error();
    SCD_TRY(check_view(x, "conv1x1_bwd.x"));
    SCD_TRY(check_view(gx, "conv1x1_bwd.gx", true));
    if (!w || !gout || n_out < 1 || n_out > 4) {
        set_error("conv1x1_bwd: bad arguments");
        return SCD_ERR_ARG;
    }
    if (gx.data && (gx.n != x.n || gx.h != x.h || gx.w != x.w || gx.c != x.c)) {
        set_error("conv1x1_bwd: gx shape mismatch");
        return SCD_ERR_ARG;
    }
    if (common_dtype("conv1x1_bwd", {&x, &gx}) < 0) return SCD_ERR_ARG;
    if ((gw || gb) && (!ws || ws_bytes < scd_conv1x1_workspace_bytes(x, n_out))) {
        set_error("conv1x1_bwd: workspace too small");
        return SCD_ERR_WORKSPACE;
    }
    hipStream_t s = as_stream(stream);
    const int64_t npix = pixels(x);
    const int hw = x.h * x.w;
    if (gx.data) {
        const int64_t total = npix * (x.c / 4);
        SCD_WITH_T(gx.dtype, T,
                   hipLaunchKernelGGL(conv1x1_bwd_dx_kernel<T>, dim3(grid_for(total)), dim3(256), 0, s, gout, n_out,
                                      hw, w, view_ptr<T>(gx), gx.ldc, x.c, accumulate, total,
                                      make_fastdiv(uint32_t(x.c / 4 > 0 ? x.c / 4 : 1)), make_fastdiv(uint32_t(hw > 0 ? hw : 1))));
    }
    float *rec = static_cast<float *>(ws);
    const size_t wbytes = weighted_channel_sum_bytes(x);
    if (gw)
        for (int o = 0; o < n_out; ++o)  // stream-ordered reuse of the record buffer
            SCD_TRY(weighted_channel_sum(x, gout, n_out, o, gw + size_t(o) * x.c, ws, wbytes, s));
    if (gb) {
        float *brec = rec + wbytes / sizeof(float);
        const int nb = 1024;
        hipLaunchKernelGGL(conv1x1_bwd_db_partial, dim3(nb, n_out), dim3(256), 0, s, gout, n_out, hw, npix, brec);
        hipLaunchKernelGGL(sum_rows_block, dim3(n_out), dim3(256), 0, s, brec, nb, gb);
    }
    return launch_status("scd_conv1x1_bwd");
}

extern "C" int scd_conv1x1_bwd_bn(scd_nhwc_t y, const float *scale, const float *shift, int32_t nseg, const float *w,
                                  const float *gout, int32_t n_out, float *gw, float *gb, void *ws, size_t ws_bytes,
                                  scd_stream_t stream) {
    clear_error();
    SCD_TRY(check_view(y, "conv1x1_bwd_bn.y"));
    if (!w || !gout || !scale || !shift || n_out < 1 || n_out > 4 || nseg < 1 || y.n % nseg || !aligned16(scale) ||
        !aligned16(shift)) {
        set_error("conv1x1_bwd_bn: bad arguments");
        return SCD_ERR_ARG;
    }
    if ((gw || gb) && (!ws || ws_bytes < scd_conv1x1_workspace_bytes(y, n_out))) {
        set_error("conv1x1_bwd_bn: workspace too small");
        return SCD_ERR_WORKSPACE;
    }
    hipStream_t s = as_stream(stream);
    const int64_t npix = pixels(y);
    const int hw = y.h * y.w;
    float *rec = static_cast<float *>(ws);
    const size_t wbytes = weighted_channel_sum_bytes(y);
    if (gw)
        for (int o = 0; o < n_out; ++o)
            SCD_TRY(weighted_channel_sum(y, gout, n_out, o, gw + size_t(o) * y.c, ws, wbytes, s, scale, shift, nseg));
    if (gb) {
        float *brec = rec + wbytes / sizeof(float);
        const int nb = 1024;
        hipLaunchKernelGGL(conv1x1_bwd_db_partial, dim3(nb, n_out), dim3(256), 0, s, gout, n_out, hw, npix, brec);
        hipLaunchKernelGGL(sum_rows_block, dim3(n_out), dim3(256), 0, s, brec, nb, gb);
    }
    return launch_status("scd_conv1x1_bwd_bn");
}

static constexpr int PJ_BLOCKS = 1024;

extern "C" size_t scd_pjaccard_workspace_bytes(int64_t n) {
    (void)n;
    return size_t(PJ_BLOCKS) * 2 * sizeof(float) + 256;
}

extern "C" int scd_pjaccard_fwd(const float *logits, const float *target, int64_t n, float *sums_out,
                                float *loss_out, void *ws, size_t ws_bytes, scd_stream_t stream) {
    clear_error();
    if (!logits || !target || n < 1 || !sums_out || !loss_out) {
        set_error("pjaccard_fwd: bad arguments");
        return SCD_ERR_ARG;
    }
    if (!ws || ws_bytes < scd_pjaccard_workspace_bytes(n)) {
        set_error("pjaccard_fwd: workspace too small");
        return SCD_ERR_WORKSPACE;
    }
    hipStream_t s = as_stream(stream);
    float *rec = static_cast<float *>(ws);
    hipLaunchKernelGGL(pjaccard_partial, dim3(PJ_BLOCKS), dim3(256), 0, s, logits, target, n, rec);
    hipLaunchKernelGGL(pjaccard_finalize, dim3(1), dim3(256), 0, s, rec, PJ_BLOCKS, sums_out, loss_out);
    return launch_status("scd_pjaccard_fwd");
}

extern "C" int scd_pjaccard_bwd(const float *logits, const float *target, int64_t n, const float *sums,
                                const float *gloss, float *glogits, float *gtarget, scd_stream_t stream) {
    clear_error();
    if (!logits || !target || n < 1 || !sums || !glogits) {
        set_error("pjaccard_bwd: bad arguments");
        return SCD_ERR_ARG;
    }
    hipLaunchKernelGGL(pjaccard_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), logits, target, n, sums,
                       gloss, glogits, gtarget);
    return launch_status("scd_pjaccard_bwd");
}

extern "C" int scd_bn_relu_pool_diff(scd_nhwc_t a, const float *scale, const float *shift, scd_nhwc_t d,
                                     scd_nhwc_t y, uint8_t *idx, scd_stream_t stream) {
    clear_error();
    SCD_TRY(check_view(y, "pool_diff.y"));
    return scd_bn_relu_pool_out(a, 2, scale, shift, 0, d, scd_nhwc_t{}, y, idx, stream);
}

extern "C" int scd_bn_relu_pool_out(scd_nhwc_t a, int32_t nseg, const float *scale, const float *shift, int32_t mode,
                                    scd_nhwc_t d, scd_nhwc_t o, scd_nhwc_t y, uint8_t *idx, scd_stream_t stream) {
    clear_error();
    SCD_TRY(check_view(a, "pool_out.a"));
    SCD_TRY(check_view(d, "pool_out.d", mode == 1));
    SCD_TRY(check_view(o, "pool_out.o", mode == 0));
    SCD_TRY(check_view(y, "pool_out.y", true));
    const bool pair = mode != 1;
    const int units = pair ? a.n / 2 : a.n;
    bool ok = mode >= 0 && mode <= 2 && (a.h & 1) == 0 && (a.w & 1) == 0 && a.h >= 2 && a.w >= 2 && scale && shift &&
              aligned16(scale) && aligned16(shift) && nseg >= 1 && a.n % nseg == 0 && (!pair || (nseg == 2 && a.n % 2 == 0));
    if (ok && pair) ok = d.n == units && d.h == a.h && d.w == a.w && d.c == a.c;
    if (ok && mode != 0) ok = o.n == a.n && o.h == a.h && o.w == a.w && o.c == a.c;
    if (ok && y.data)
        ok = y.n == a.n && y.c == a.c && y.h == a.h / 2 && y.w == a.w / 2 && idx && !(reinterpret_cast<uintptr_t>(idx) & 3);
    if (!ok) {
        set_error("bn_relu_pool_out: mode %d: a (n, h, w, c) with even h, w (pairs: 2 segments of n/2 images); d "
                  "(n/2, h, w, c) for modes 0, 2; o (n, h, w, c) for modes 1, 2; y (n, h/2, w/2, c) with 4-byte aligned "
                  "idx or null; aligned coefficients [nseg][c]", mode);
        return SCD_ERR_ARG;
    }
    const int dt = common_dtype("bn_relu_pool_out", {&a, &d, &o, &y});
    if (dt < 0) return SCD_ERR_ARG;
    hipStream_t s = as_stream(stream);
    if (mode == 0) return pool_out_run<0>(a, scale, shift, nseg, d, o, y, idx, dt, s);
    if (mode == 1) return pool_out_run<1>(a, scale, shift, nseg, d, o, y, idx, dt, s);
    return pool_out_run<2>(a, scale, shift, nseg, d, o, y, idx, dt, s);
}
