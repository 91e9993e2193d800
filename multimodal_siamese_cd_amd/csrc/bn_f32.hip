// BatchNorm2d (+ fused ReLU) kernels over NHWC fp32, per-segment batch statistics.
//
// Replaces aten::native_batch_norm / native_batch_norm_backward / relu_ / threshold_backward for the
// reference's `Conv2d -> BatchNorm2d -> ReLU(inplace)` pairs (utils/networks.py:392-397).
//
// Reductions are two-stage and deterministic:
//   partial  : one workgroup per (segment, pixel chunk, channel group); every thread owns one channel
//              quad (float4) and walks pixels with 4 independent 16-byte loads in flight; forward stats use
//              shifted sums (shift = the chunk's first value of the channel) turned into (n, mean, M2) and
//              Chan-merged in LDS, so there is no E[x^2]-E[x]^2 cancellation.  Records are written
//              channel-major, rec[c][chunk][field].
//   finalize : one workgroup per channel merges its chunk records in double with a fixed-shape tree.
#include "common.h"

namespace scd {

constexpr int BN_THREADS = 256;
constexpr int BN_CHUNK_MAX = 4096;  // pixels per reduction chunk (large maps)
constexpr int BN_CHUNK_MIN = 64;
constexpr int BN_TARGET_BLOCKS = 2048;  // 8 workgroups per CU

struct BnGeom {
    int64_t pseg;  // pixels per segment
    int chunk;     // pixels per chunk
    int ncps;      // chunks per segment
    int nrec;      // nseg * ncps
    int qpb;       // channel quads per block (power of two)
    int cgroups;   // channel groups (grid.y)
};

// The chunk shrinks (power of two, >= 64 px) until the grid fills the chip: deep 16x16..64x64 maps
// otherwise launch a few dozen workgroups that each walk thousands of pixels serially.
static BnGeom bn_geom(const scd_nhwc_t &y, int nseg) {
    BnGeom g;
    g.pseg = pixels(y) / nseg;
    const int cq = y.c / 4;
    int q = 1;
    while (q * 2 <= cq && q * 2 <= 64) q *= 2;
    g.qpb = q;
    g.cgroups = (cq + q - 1) / q;
    int chunk = BN_CHUNK_MAX;
    while (chunk > BN_CHUNK_MIN && int64_t(nseg) * ((g.pseg + chunk - 1) / chunk) * g.cgroups < BN_TARGET_BLOCKS)
        chunk /= 2;
    g.chunk = chunk;
    g.ncps = int((g.pseg + chunk - 1) / chunk);
    g.nrec = nseg * g.ncps;
    return g;
}

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 fabs4(f4 v) { return f4{fabsf(v.x), fabsf(v.y), fabsf(v.z), fabsf(v.w)}; }
__device__ __forceinline__ f4 fmax4(f4 a, f4 b) {
    return f4{fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z), fmaxf(a.w, b.w)};
}
// Keep a batch of loads in flight: an opaque use of the loaded registers right after issuing them stops
// hipcc from sinking each load next to its consumer (which serialised the loop at vmcnt(0) per load).
#define PIN4(a, b, c, d) asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d))

struct Welford4 {
    float n;
    f4 mean, m2;
};

__device__ __forceinline__ void chan_merge(Welford4 &a, const Welford4 &b) {
    if (b.n == 0.f) return;
    if (a.n == 0.f) {
        a = b;
        return;
    }
    const float n = a.n + b.n;
    const float fb = b.n / n;
    const float fab = a.n * b.n / n;
    const f4 d = b.mean - a.mean;
    a.mean += d * fb;
    a.m2 += b.m2 + d * d * fab;
    a.n = n;
}

// Chunk bounds of this block.
struct Chunk {
    int64_t beg, end;
    int seg;
};
__device__ __forceinline__ Chunk chunk_of(int64_t pseg, int ncps, int chunk) {
    Chunk c;
    c.seg = blockIdx.x / ncps;
    const int k = blockIdx.x % ncps;
    c.beg = c.seg * pseg + int64_t(k) * chunk;
    c.end = min(c.beg + chunk, (c.seg + 1) * pseg);
    return c;
}

// ------------------------------------------------------------------------------------------------
// forward statistics
// ------------------------------------------------------------------------------------------------
template <class T>
__global__ __launch_bounds__(BN_THREADS) void bn_stats_partial(const T *__restrict__ y, int ldc, int C,
                                                               int64_t pseg, int ncps, int chunk, int nrec, int qpb,
                                                               float *__restrict__ rec) {
    __shared__ Welford4 sh[BN_THREADS];
    const int tid = threadIdx.x;
    const int q = tid % qpb, pl = tid / qpb, npl = BN_THREADS / qpb;
    const int c = (blockIdx.y * qpb + q) * 4;
    const Chunk ch = chunk_of(pseg, ncps, chunk);
    Welford4 w;
    w.n = 0.f;
    w.mean = f4{0.f, 0.f, 0.f, 0.f};
    w.m2 = w.mean;
    if (c < C) {
        const f4 K = ld4(y + ch.beg * ldc + c);
        f4 s1 = {0.f, 0.f, 0.f, 0.f}, s2 = s1;
        int n = 0;
        int64_t p = ch.beg + pl;
        for (; p + 3 * npl < ch.end; p += 4 * npl) {
            f4 a = ld4(y + p * ldc + c), b = ld4(y + (p + npl) * ldc + c);
            f4 d = ld4(y + (p + 2 * npl) * ldc + c), e = ld4(y + (p + 3 * npl) * ldc + c);
            PIN4(a, b, d, e);
            a -= K;
            b -= K;
            d -= K;
            e -= K;
            s1 += (a + b) + (d + e);
            s2 += (a * a + b * b) + (d * d + e * e);
            n += 4;
        }
        for (; p < ch.end; p += npl) {
            const f4 a = ld4(y + p * ldc + c) - K;
            s1 += a;
            s2 += a * a;
            n += 1;
        }
        if (n > 0) {
            const float fn = float(n);
            w.n = fn;
            const f4 m = s1 / fn;
            w.mean = K + m;
            f4 m2 = s2 - s1 * m;
            m2.x = fmaxf(m2.x, 0.f);
            m2.y = fmaxf(m2.y, 0.f);
            m2.z = fmaxf(m2.z, 0.f);
            m2.w = fmaxf(m2.w, 0.f);
            w.m2 = m2;
        }
    }
    sh[tid] = w;
    __syncthreads();
    for (int off = npl / 2; off > 0; off >>= 1) {
        if (pl < off) {
            Welford4 a = sh[tid];
            chan_merge(a, sh[tid + off * qpb]);
            sh[tid] = a;
        }
        __syncthreads();
    }
    if (pl == 0 && c < C) {
        const Welford4 a = sh[tid];
        const float mv[4] = {a.mean.x, a.mean.y, a.mean.z, a.mean.w};
        const float qv[4] = {a.m2.x, a.m2.y, a.m2.z, a.m2.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float *r = rec + (size_t(c + k) * nrec + blockIdx.x) * 3;
            r[0] = a.n;
            r[1] = mv[k];
            r[2] = qv[k];
        }
    }
}

struct DWelford {
    double n, mean, m2;
};
__device__ __forceinline__ void dmerge(DWelford &a, const DWelford &b) {
    if (b.n == 0) return;
    if (a.n == 0) {
        a = b;
        return;
    }
    const double n = a.n + b.n;
    const double d = b.mean - a.mean;
    a.mean += d * b.n / n;
    a.m2 += b.m2 + d * d * a.n * b.n / n;
    a.n = n;
}

// Block merge of per-thread Welford states in a fixed order: xor-shuffle tree within each wave, then the waves'
// results in wave order by thread 0 (one barrier instead of a log2(BN_THREADS)-level LDS tree).  Valid in thread 0.
__device__ __forceinline__ DWelford block_dmerge(DWelford w, DWelford *sh) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const DWelford o{__shfl_xor(w.n, off), __shfl_xor(w.mean, off), __shfl_xor(w.m2, off)};
        dmerge(w, o);
    }
    const int t = threadIdx.x;
    if ((t & 63) == 0) sh[t >> 6] = w;
    __syncthreads();
    DWelford a = sh[0];
    if (t == 0)
        for (int k = 1; k < BN_THREADS / 64; ++k) dmerge(a, sh[k]);
    __syncthreads();  // sh is reused by the next call
    return a;
}

// Upper bound of |relu(fma(y, scale, shift))| over the n values of one segment and channel, from the statistics
// alone (SCD_MATH_H2 operand scaling): every value lies within sqrt(n - 1) population standard deviations of the
// mean, and scale = gamma * invstd with invstd <= 1 / std, so |scale * (y - mean)| <= |gamma| sqrt(n - 1).  The
// slack terms cover the rounding of the statistics and of the fma (relative 2^-20 of each addend).
__device__ __forceinline__ float bn_act_bound(double n, double gamma, double beta, double shift) {
    const double dev = fabs(gamma) * sqrt(n > 1 ? n - 1 : 0.0);
    return float((dev + fabs(beta)) * (1.0 + 0x1p-10) + (fabs(shift) + fabs(beta)) * 0x1p-16);
}

// one workgroup per channel; segments in order (t1 first), running stats updated once per segment
__global__ __launch_bounds__(BN_THREADS) void bn_stats_finalize(const float *__restrict__ rec, int C, int nseg,
                                                                int ncps, int nrec, const float *gamma,
                                                                const float *beta, float eps, float momentum,
                                                                int update, float *rmean, float *rvar, float *smean,
                                                                float *sinv, float *scale, float *shift,
                                                                float *act_bound) {
    __shared__ DWelford sh[BN_THREADS / 64];
    const int c = blockIdx.x;
    const int t = threadIdx.x;
    const float *rc = rec + size_t(c) * nrec * 3;
    for (int s = 0; s < nseg; ++s) {
        DWelford w{0, 0, 0};
        for (int k = t; k < ncps; k += BN_THREADS) {
            const float *r = rc + size_t(s * ncps + k) * 3;
            dmerge(w, DWelford{r[0], r[1], r[2]});
        }
        const DWelford a = block_dmerge(w, sh);
        if (t == 0) {
            const double g = gamma ? gamma[c] : 1.0, b = beta ? beta[c] : 0.0;
            const double var = a.n > 0 ? a.m2 / a.n : 0.0;
            const double inv = 1.0 / sqrt(var + double(eps));
            smean[s * C + c] = float(a.mean);
            sinv[s * C + c] = float(inv);
            const float sc = float(g * inv);
            scale[s * C + c] = sc;
            shift[s * C + c] = float(b - a.mean * double(sc));
            if (act_bound) atomic_max_bound(act_bound, bn_act_bound(a.n, g, b, double(shift[s * C + c])));
            if (update) {
                const double uvar = a.n > 1 ? a.m2 / (a.n - 1) : var;
                rmean[c] = float((1.0 - momentum) * rmean[c] + momentum * a.mean);
                rvar[c] = float((1.0 - momentum) * rvar[c] + momentum * uvar);
            }
        }
    }
}

// Conv-fused statistics: tile records trec[tile][C] = {mean, M2} of tile_px pixels each (scd_conv_igemm
// stat_rec) are Chan-merged in fixed order over groups of `group` consecutive tiles of one segment into the
// chunk records rec[c][g] = {n, mean, M2} that bn_stats_finalize merges in double.
__global__ __launch_bounds__(BN_THREADS) void bn_tile_merge(const float *__restrict__ trec, int C, int tiles_per_seg,
                                                            int group, int ncps, int nrec, float tile_px,
                                                            float *__restrict__ rec) {
    const int c = blockIdx.y * BN_THREADS + threadIdx.x;
    if (c >= C) return;
    const int g = blockIdx.x;
    const int seg = g / ncps, k = g - (g / ncps) * ncps;
    const int t0 = seg * tiles_per_seg + k * group;
    const int t1 = min(t0 + group, (seg + 1) * tiles_per_seg);
    float n = 0.f, mean = 0.f, m2 = 0.f;
    auto merge = [&](float2 r) {
        const float nn = n + tile_px;
        const float d = r.x - mean;
        mean += d * (tile_px / nn);
        m2 += r.y + d * d * (n * tile_px / nn);
        n = nn;
    };
    int t = t0;
    for (; t + 8 <= t1; t += 8) {  // 8 records loaded together, merged in tile order (latency, not the merge, bound)
        float2 r[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) r[u] = *reinterpret_cast<const float2 *>(trec + (size_t(t + u) * C + c) * 2);
#pragma unroll
        for (int u = 0; u < 8; ++u) merge(r[u]);
    }
    for (; t < t1; ++t) merge(*reinterpret_cast<const float2 *>(trec + (size_t(t) * C + c) * 2));
    float *o = rec + (size_t(c) * nrec + g) * 3;
    o[0] = n;
    o[1] = mean;
    o[2] = m2;
}

__global__ void bn_eval_coeffs_kernel(int C, const float *gamma, const float *beta, const float *rm, const float *rv,
                                      float eps, float *scale, float *shift) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const double inv = 1.0 / sqrt(double(rv[c]) + double(eps));
    const float sc = float((gamma ? gamma[c] : 1.0f) * inv);
    scale[c] = sc;
    shift[c] = float((beta ? beta[c] : 0.0f) - double(rm[c]) * sc);
}

__device__ __forceinline__ float bn_relu(float y, float sc, float sh) { return fmaxf(fmaf(y, sc, sh), 0.f); }
__device__ __forceinline__ f4 bn_relu4(f4 y, f4 sc, f4 sh) {
    return f4{bn_relu(y.x, sc.x, sh.x), bn_relu(y.y, sc.y, sh.y), bn_relu(y.z, sc.z, sh.z), bn_relu(y.w, sc.w, sh.w)};
}

// grid: (chunks, segments); each thread walks quads of its segment's pixels.
template <class T>
__global__ __launch_bounds__(256) void bn_relu_apply_kernel(const T *__restrict__ y, int ldy, T *__restrict__ a,
                                                            int lda, int C, int64_t pseg, const float *__restrict__ scale,
                                                            const float *__restrict__ shift) {
    const int seg = blockIdx.y;
    const int cq = C / 4;
    const int64_t total = pseg * cq;
    const float *sc = scale + seg * C;
    const float *sh = shift + seg * C;
    for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < total; e += int64_t(gridDim.x) * blockDim.x) {
        const int64_t p = seg * pseg + e / cq;
        const int c = int(e % cq) * 4;
        st4(a + p * lda + c, bn_relu4(ld4(y + p * ldy + c), ld4(sc + c), ld4(sh + c)));
    }
}

// ------------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------------
// relu_mask / bn_bwd_dy4: common.h (shared with the weight grad's fused dY staging)

// Incoming gradient dL/da of the BatchNorm + ReLU backward, read at (pixel p, channel quad c).
template <class T>
struct DaPlain {  // a materialised tensor
    const T *da;
    int ldda;
    __device__ __forceinline__ void bind(int) {}
    __device__ __forceinline__ f4 operator()(int64_t p, int c) const { return ld4(da + p * ldda + c); }
};
// The encoder level's gradient, formed on the fly with the expressions of feature_grad_kernel (misc_f32.hip):
// MaxPool2d backward of the next level's input gradient gy through the argmax bytes, plus -/+ the gradient of
// the Siamese feature difference (skip_mode 1: t1 images subtract) or a plain skip gradient (skip_mode 0).
// skip_mode 2 (the dual-task encoder): also the semantic decoder's skip gradient gs2, a [t2; t1] batch of 2 gsn images
// (image img of the [t1; t2] level reads gs2 image img + gsn for t1, img - gsn for t2), added to the difference term
// first: (sg * gs + gs2) is the one rounding autograd's sum of the two skip gradients makes.
template <class T>
struct DaPooled {
    const T *gy;  // (n, h/2, w/2, C) or null
    const uint8_t *idx;
    int hy, wy, ldgy;
    const T *gs;  // (gsn, h, w, C) or null
    int gsn, ldgs, skip_mode;
    const T *gs2;  // skip_mode 2: (2 gsn, h, w, C), else null
    int ldgs2;
    int hx, wx, C;
    FastDiv div_hw, div_w, div_gsn;
    __device__ __forceinline__ void bind(int) {}
    __device__ __forceinline__ f4 operator()(int64_t p, int c) const {
        const uint32_t img = fdiv(uint32_t(p), div_hw);
        const uint32_t rr = uint32_t(p) - img * uint32_t(hx * wx);
        const int yy = int(fdiv(rr, div_w)), x = int(rr) - yy * wx;
        f4 r = {0.f, 0.f, 0.f, 0.f};
        if (gy) {
            const int oy = yy >> 1, ox = x >> 1;
            if (oy < hy && ox < wy) {
                const int64_t q = (int64_t(img) * hy + oy) * wy + ox;
                const uint32_t pk = *reinterpret_cast<const uint32_t *>(idx + q * C + c);
                const f4 g = ld4(gy + q * ldgy + c);
                const uint32_t want = uint32_t((yy & 1) * 2 + (x & 1));
                r.x = ((pk >> 0) & 0xff) == want ? g.x : 0.f;
                r.y = ((pk >> 8) & 0xff) == want ? g.y : 0.f;
                r.z = ((pk >> 16) & 0xff) == want ? g.z : 0.f;
                r.w = ((pk >> 24) & 0xff) == want ? g.w : 0.f;
            }
        }
        if (gs) {
            const int simg = int(img - fdiv(img, div_gsn) * uint32_t(gsn));
            const float sg = (skip_mode != 0 && int(img) < gsn) ? -1.f : 1.f;
            const f4 sv = ld4(gs + ((int64_t(simg) * hx + yy) * wx + x) * ldgs + c);
            if (gs2) {
                const int img2 = int(img) < gsn ? int(img) + gsn : int(img) - gsn;
                const f4 s2 = ld4(gs2 + ((int64_t(img2) * hx + yy) * wx + x) * ldgs2 + c);
                r.x += sg * sv.x + s2.x;
                r.y += sg * sv.y + s2.y;
                r.z += sg * sv.z + s2.z;
                r.w += sg * sv.w + s2.w;
            } else {
                r.x += sg * sv.x;
                r.y += sg * sv.y;
                r.z += sg * sv.z;
                r.w += sg * sv.w;
            }
        }
        return r;
    }
};

// The decoder's last gradient when the 1x1 head reads its output: dL/da = sum_o gout[img][o][pix] * w[o][c], formed on
// the fly with conv1x1_bwd_dx_kernel's fma chain (misc_f32.hip; bit-identical), so the full-resolution gradient of
// the head's input is never written or read.
struct DaHead {
    const float *g;  // NCHW [n][n_out][hw]
    const float *w;  // [n_out][C]
    int n_out, C, hw;
    FastDiv div_hw;
    __device__ __forceinline__ void bind(int) {}
    __device__ __forceinline__ f4 operator()(int64_t p, int c) const {
        const uint32_t img = fdiv(uint32_t(p), div_hw);
        const int pix = int(uint32_t(p) - img * uint32_t(hw));
        f4 r = {0.f, 0.f, 0.f, 0.f};
        for (int o = 0; o < n_out; ++o) {
            const float gv = g[(int64_t(img) * n_out + o) * hw + pix];
            const float *wr = w + int64_t(o) * C + c;
            r.x = fmaf(gv, wr[0], r.x);
            r.y = fmaf(gv, wr[1], r.y);
            r.z = fmaf(gv, wr[2], r.z);
            r.w = fmaf(gv, wr[3], r.w);
        }
        return r;
    }
};

// DaHead with the head count a compile-time constant and the thread's weight quads held in registers (bind, once per
// thread): the per-pixel loop is branch-free and a pixel's NO gradient loads issue together.  With a runtime count
// the loop branched per head and re-loaded the weights per pixel (the stores to dy may alias them), which held the
// 3- and 4-head bf16 passes of the dual-stream / WhateverNet heads at 1.3-2.2 TB/s.  Same fma chain (bit-identical).
template <int NO>
struct DaHeadN {
    DaHead d;
    f4 w[NO];
    __device__ __forceinline__ void bind(int c) {
#pragma unroll
        for (int o = 0; o < NO; ++o) w[o] = c < d.C ? ld4(d.w + int64_t(o) * d.C + c) : f4{0.f, 0.f, 0.f, 0.f};
    }
    __device__ __forceinline__ f4 operator()(int64_t p, int c) const {
        (void)c;
        const uint32_t img = fdiv(uint32_t(p), d.div_hw);
        const int pix = int(uint32_t(p) - img * uint32_t(d.hw));
        float gv[NO];
#pragma unroll
        for (int o = 0; o < NO; ++o) gv[o] = d.g[(int64_t(img) * NO + o) * d.hw + pix];
        f4 r = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int o = 0; o < NO; ++o) {
            r.x = fmaf(gv[o], w[o].x, r.x);
            r.y = fmaf(gv[o], w[o].y, r.y);
            r.z = fmaf(gv[o], w[o].z, r.z);
            r.w = fmaf(gv[o], w[o].w, r.w);
        }
        return r;
    }
};

// The DaPooled gradient over 2x2 cells: cell (img, cy, cx) covers the full-resolution pixels (2cy + i, 2cx + j) that
// exist (ceil(h/2) x ceil(w/2) cells per image), so the pooled gradient and its argmax bytes are read and decoded once
// per cell instead of once per pixel, with the cell's four pixels' loads in flight together.
template <class T>
struct PooledCells {
    DaPooled<T> da;
    int ch, cw;                 // cells per image column / row
    FastDiv div_cimg, div_cw;   // ch * cw, cw
};

// dL/da of the four pixels of `cell` (flat cell index over images) at channel quad c; ok[k]: pixel k exists.
// S2: the dual-task second skip gradient (DaPooled.gs2, with gs present).
template <class T, bool S2>
__device__ __forceinline__ void cell_grads(const PooledCells<T> &P, uint32_t cell, int c, f4 (&g)[4], int64_t (&pix)[4],
                                           bool (&ok)[4], const T *fallback) {
    const DaPooled<T> &d = P.da;
    const uint32_t img = fdiv(cell, P.div_cimg);
    const uint32_t r = cell - img * uint32_t(P.ch * P.cw);
    const int cy = int(fdiv(r, P.div_cw)), cx = int(r) - cy * P.cw;
    // Every load is unconditional (addresses clamped into the maps, the values selected afterwards), so a cell's
    // loads issue together: guarded loads had each waited for the previous one (one memory latency per pixel).
    // No branches around the loads either: a missing operand (no pooled gradient, no skip) reads `fallback` (valid
    // memory: the BatchNorm input) and is discarded, so the loads need no wait before the block joins.
    const bool has_gy = d.gy && d.hy > 0 && d.wy > 0;  // uniform
    const bool in = has_gy && cy < d.hy && cx < d.wy;
    const int64_t q = has_gy ? (int64_t(img) * d.hy + min(cy, d.hy - 1)) * d.wy + min(cx, d.wy - 1) : 0;
    uint32_t pk = *reinterpret_cast<const uint32_t *>(
        (has_gy ? d.idx : reinterpret_cast<const uint8_t *>(fallback)) + q * d.C + c);
    f4 gp = ld4((has_gy ? d.gy : fallback) + q * d.ldgy + c);
    const int simg = d.gs ? int(img - fdiv(img, d.div_gsn) * uint32_t(d.gsn)) : 0;
    const float sg = (d.gs && d.skip_mode != 0 && int(img) < d.gsn) ? -1.f : 1.f;
    f4 sv[4], s2v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int yy = min(2 * cy + (k >> 1), d.hx - 1), xx = min(2 * cx + (k & 1), d.wx - 1);
        sv[k] = ld4((d.gs ? d.gs : fallback) + (d.gs ? ((int64_t(simg) * d.hx + yy) * d.wx + xx) * d.ldgs : 0) + c);
        if constexpr (S2) {
            const int img2 = int(img) < d.gsn ? int(img) + d.gsn : int(img) - d.gsn;
            s2v[k] = ld4(d.gs2 + ((int64_t(img2) * d.hx + yy) * d.wx + xx) * d.ldgs2 + c);
        }
    }
    if (!in) {  // no pooled gradient: no byte matches a sub-pixel
        pk = 0xffffffffu;
        gp = f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int yy = 2 * cy + (k >> 1), xx = 2 * cx + (k & 1);
        ok[k] = yy < d.hx && xx < d.wx;
        pix[k] = (int64_t(img) * d.hx + yy) * d.wx + xx;
        const uint32_t want = uint32_t(k);
        f4 v = {((pk >> 0) & 0xff) == want ? gp.x : 0.f, ((pk >> 8) & 0xff) == want ? gp.y : 0.f,
                ((pk >> 16) & 0xff) == want ? gp.z : 0.f, ((pk >> 24) & 0xff) == want ? gp.w : 0.f};
        // the skip term of a missing pixel (ok[k] false) reads a clamped neighbour: its g is never used; a select,
        // not a branch, so the caller's loads can be scheduled above
        if constexpr (S2) {
            const f4 u = {sg * sv[k].x + s2v[k].x, sg * sv[k].y + s2v[k].y, sg * sv[k].z + s2v[k].z,
                          sg * sv[k].w + s2v[k].w};
            g[k] = v + u;
        } else {
            const f4 t = {v.x + sg * sv[k].x, v.y + sg * sv[k].y, v.z + sg * sv[k].z, v.w + sg * sv[k].w};
            g[k] = d.gs ? t : v;
        }
    }
}

// The address a cell's pixel k is loaded from: itself, or (a pixel past the map edge, whose value is discarded) the
// cell's first pixel, which always exists.
__device__ __forceinline__ int64_t cell_load_pix(const int64_t (&pix)[4], const bool (&ok)[4], int k) {
    return ok[k] ? pix[k] : pix[0];
}

// cell_grads for a Siamese pair (skip_mode 1, two segments of gsn images): `cell` lies in a t1 image, its partner
// cell (same place) in image img + gsn.  The difference gradient is read once for both (t1 subtracts it, t2 adds
// it, with cell_grads' expressions: bit-identical).  pix[k] is the t1 pixel; its t2 partner is pix[k] + gsn*hx*wx.
template <class T, bool S2>
__device__ __forceinline__ void cell_grads_pair(const PooledCells<T> &P, uint32_t cell, int c, f4 (&g0)[4], f4 (&g1)[4],
                                                int64_t (&pix)[4], bool (&ok)[4]) {
    const DaPooled<T> &d = P.da;
    const uint32_t img = fdiv(cell, P.div_cimg);
    const uint32_t r = cell - img * uint32_t(P.ch * P.cw);
    const int cy = int(fdiv(r, P.div_cw)), cx = int(r) - cy * P.cw;
    // unconditional loads (clamped addresses, values selected afterwards): see cell_grads
    // a missing pooled gradient reads the skip gradient's memory (valid; discarded): no branch around the loads
    const bool has_gy = d.gy && d.hy > 0 && d.wy > 0;  // uniform
    const bool in = has_gy && cy < d.hy && cx < d.wy;
    const int64_t q0 = has_gy ? (int64_t(img) * d.hy + min(cy, d.hy - 1)) * d.wy + min(cx, d.wy - 1) : 0;
    const int64_t q1 = has_gy ? q0 + int64_t(d.gsn) * d.hy * d.wy : 0;
    const uint8_t *ib = has_gy ? d.idx : reinterpret_cast<const uint8_t *>(d.gs);
    const T *gb = has_gy ? d.gy : d.gs;
    uint32_t pk0 = *reinterpret_cast<const uint32_t *>(ib + q0 * d.C + c);
    uint32_t pk1 = *reinterpret_cast<const uint32_t *>(ib + q1 * d.C + c);
    f4 gp0 = ld4(gb + q0 * d.ldgy + c), gp1 = ld4(gb + q1 * d.ldgy + c);
    f4 svs[4], s2a[4], s2b[4];  // S2: the semantic skip gradient of the t1 (image img + gsn) and t2 (img) pixel
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int yy = min(2 * cy + (k >> 1), d.hx - 1), xx = min(2 * cx + (k & 1), d.wx - 1);
        svs[k] = ld4(d.gs + ((int64_t(img) * d.hx + yy) * d.wx + xx) * d.ldgs + c);
        if constexpr (S2) {
            s2a[k] = ld4(d.gs2 + ((int64_t(img + d.gsn) * d.hx + yy) * d.wx + xx) * d.ldgs2 + c);
            s2b[k] = ld4(d.gs2 + ((int64_t(img) * d.hx + yy) * d.wx + xx) * d.ldgs2 + c);
        }
    }
    if (!in) {
        pk0 = pk1 = 0xffffffffu;
        gp0 = gp1 = f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int yy = 2 * cy + (k >> 1), xx = 2 * cx + (k & 1);
        ok[k] = yy < d.hx && xx < d.wx;
        pix[k] = (int64_t(img) * d.hx + yy) * d.wx + xx;
        const uint32_t want = uint32_t(k);
        f4 v0 = {((pk0 >> 0) & 0xff) == want ? gp0.x : 0.f, ((pk0 >> 8) & 0xff) == want ? gp0.y : 0.f,
                 ((pk0 >> 16) & 0xff) == want ? gp0.z : 0.f, ((pk0 >> 24) & 0xff) == want ? gp0.w : 0.f};
        f4 v1 = {((pk1 >> 0) & 0xff) == want ? gp1.x : 0.f, ((pk1 >> 8) & 0xff) == want ? gp1.y : 0.f,
                 ((pk1 >> 16) & 0xff) == want ? gp1.z : 0.f, ((pk1 >> 24) & 0xff) == want ? gp1.w : 0.f};
        if constexpr (S2) {  // (sg * gs + gs2) first: see DaPooled
            const f4 sv = svs[k];
            const float m = -1.f, p1 = 1.f;
            v0 += f4{m * sv.x + s2a[k].x, m * sv.y + s2a[k].y, m * sv.z + s2a[k].z, m * sv.w + s2a[k].w};
            v1 += f4{p1 * sv.x + s2b[k].x, p1 * sv.y + s2b[k].y, p1 * sv.z + s2b[k].z, p1 * sv.w + s2b[k].w};
        } else {  // unconditional: a missing pixel's (ok[k] false) gradient is never used (see cell_grads)
            const f4 sv = svs[k];
            const float m = -1.f, p1 = 1.f;
            v0.x += m * sv.x;
            v0.y += m * sv.y;
            v0.z += m * sv.z;
            v0.w += m * sv.w;
            v1.x += p1 * sv.x;
            v1.y += p1 * sv.y;
            v1.z += p1 * sv.z;
            v1.w += p1 * sv.w;
        }
        g0[k] = v0;
        g1[k] = v1;
    }
}

// Block-wide tree sum of (a, b) per channel quad into rec[c][rec_idx][2] (bn_bwd_pooled_partial's tree and layout).
__device__ __forceinline__ void pooled_rec2(f4 (&sh1)[BN_THREADS], f4 (&sh2)[BN_THREADS], f4 a, f4 b, int tid, int pl,
                                            int npl, int qpb, int c, int C, int nrec, int rec_idx,
                                            float *__restrict__ rec) {
    sh1[tid] = a;
    sh2[tid] = b;
    __syncthreads();
    for (int off = npl / 2; off > 0; off >>= 1) {
        if (pl < off) {
            sh1[tid] += sh1[tid + off * qpb];
            sh2[tid] += sh2[tid + off * qpb];
        }
        __syncthreads();
    }
    if (pl == 0 && c < C) {
        const f4 x = sh1[tid], y = sh2[tid];
        const float xv[4] = {x.x, x.y, x.z, x.w}, yv[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float *r = rec + (size_t(c + k) * nrec + rec_idx) * 2;
            r[0] = xv[k];
            r[1] = yv[k];
        }
    }
    __syncthreads();
}

// bn_bwd_pooled_partial for a Siamese pair: block k covers chunk k of the t1 segment and chunk k of the t2 segment
// (same cells), reading the shared difference gradient once; same per-chunk records, bit-identical.
template <class T, bool S2>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_pooled_partial_pair(const T *__restrict__ y, int ldy,
                                                                         PooledCells<T> P, int C, int64_t cseg, int ncps,
                                                                         int chunk, int nrec, int qpb,
                                                                         const float *smean, const float *sinv,
                                                                         const float *scale, const float *shift,
                                                                         float *__restrict__ rec) {
    __shared__ f4 sh1[BN_THREADS], sh2[BN_THREADS];
    const int tid = threadIdx.x;
    const int q = tid % qpb, pl = tid / qpb, npl = BN_THREADS / qpb;
    const int c = (blockIdx.y * qpb + q) * 4;
    const Chunk ch = chunk_of(cseg, ncps, chunk);  // blockIdx.x < ncps: the t1 segment's chunk
    const int64_t poff = int64_t(P.da.gsn) * P.da.hx * P.da.wx;
    f4 a1 = {0.f, 0.f, 0.f, 0.f}, a2 = a1, b1 = a1, b2 = a1;
    if (c < C) {
        const f4 mu0 = ld4(smean + c), iv0 = ld4(sinv + c), sc0 = ld4(scale + c), sf0 = ld4(shift + c);
        const f4 mu1 = ld4(smean + C + c), iv1 = ld4(sinv + C + c), sc1 = ld4(scale + C + c), sf1 = ld4(shift + C + c);
        for (int64_t cell = ch.beg + pl; cell < ch.end; cell += npl) {
            f4 g0[4], g1[4];
            int64_t pix[4];
            bool ok[4];
            cell_grads_pair<T, S2>(P, uint32_t(cell), c, g0, g1, pix, ok);
            f4 y0[4], y1[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {  // unconditional (a missing pixel reads the cell's first; not used)
                y0[k] = ld4(y + cell_load_pix(pix, ok, k) * ldy + c);
                y1[k] = ld4(y + (cell_load_pix(pix, ok, k) + poff) * ldy + c);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (ok[k]) {
                    const f4 z0 = relu_mask(y0[k], sc0, sf0, g0[k]);
                    a1 += z0;
                    a2 += z0 * ((y0[k] - mu0) * iv0);
                    const f4 z1 = relu_mask(y1[k], sc1, sf1, g1[k]);
                    b1 += z1;
                    b2 += z1 * ((y1[k] - mu1) * iv1);
                }
        }
    }
    pooled_rec2(sh1, sh2, a1, a2, tid, pl, npl, qpb, c, C, nrec, blockIdx.x, rec);
    pooled_rec2(sh1, sh2, b1, b2, tid, pl, npl, qpb, c, C, nrec, ncps + blockIdx.x, rec);
}

// bn_bwd_partial over cells: rec[c][chunk][2] = {sum dz, sum dz*xhat} of the chunk's cells' pixels.
template <class T, bool S2>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_pooled_partial(const T *__restrict__ y, int ldy, PooledCells<T> P,
                                                                    int C, int64_t cseg, int ncps, int chunk, int nrec,
                                                                    int qpb, const float *smean, const float *sinv,
                                                                    const float *scale, const float *shift,
                                                                    float *__restrict__ rec) {
    __shared__ f4 sh1[BN_THREADS], sh2[BN_THREADS];
    const int tid = threadIdx.x;
    const int q = tid % qpb, pl = tid / qpb, npl = BN_THREADS / qpb;
    const int c = (blockIdx.y * qpb + q) * 4;
    const Chunk ch = chunk_of(cseg, ncps, chunk);
    f4 s1 = {0.f, 0.f, 0.f, 0.f}, s2 = s1;
    if (c < C) {
        const int o = ch.seg * C + c;
        const f4 mu = ld4(smean + o), iv = ld4(sinv + o), sc = ld4(scale + o), sf = ld4(shift + o);
        for (int64_t cell = ch.beg + pl; cell < ch.end; cell += npl) {
            f4 g[4];
            int64_t pix[4];
            bool ok[4];
            cell_grads<T, S2>(P, uint32_t(cell), c, g, pix, ok, y);
            f4 yv[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) yv[k] = ld4(y + cell_load_pix(pix, ok, k) * ldy + c);  // see above
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (ok[k]) {
                    const f4 z = relu_mask(yv[k], sc, sf, g[k]);
                    s1 += z;
                    s2 += z * ((yv[k] - mu) * iv);
                }
        }
    }
    sh1[tid] = s1;
    sh2[tid] = s2;
    __syncthreads();
    for (int off = npl / 2; off > 0; off >>= 1) {
        if (pl < off) {
            sh1[tid] += sh1[tid + off * qpb];
            sh2[tid] += sh2[tid + off * qpb];
        }
        __syncthreads();
    }
    if (pl == 0 && c < C) {
        const f4 a = sh1[tid], b = sh2[tid];
        const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float *r = rec + (size_t(c + k) * nrec + blockIdx.x) * 2;
            r[0] = av[k];
            r[1] = bv[k];
        }
    }
}

// bn_bwd_apply over cells (see bn_bwd_pooled_partial); brec[c][chunk] (conv bias grad) and dy_bound optional.
template <class T, bool S2>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_pooled_apply(const T *__restrict__ y, int ldy, PooledCells<T> P,
                                                                  T *__restrict__ dy, int lddy, int C, int64_t cseg,
                                                                  int ncps, int chunk, int nrec, int qpb,
                                                                  const float *smean, const float *sinv,
                                                                  const float *gamma, const float *scale,
                                                                  const float *shift, const float *coef,
                                                                  float *__restrict__ brec, float *dy_bound) {
    __shared__ f4 sh[BN_THREADS];
    const int tid = threadIdx.x;
    const int q = tid % qpb, pl = tid / qpb, npl = BN_THREADS / qpb;
    const int c = (blockIdx.y * qpb + q) * 4;
    const Chunk ch = chunk_of(cseg, ncps, chunk);
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    f4 amax = acc;
    if (c < C) {
        const int o = ch.seg * C + c;
        const f4 mu = ld4(smean + o), iv = ld4(sinv + o), sc = ld4(scale + o), sf = ld4(shift + o);
        const float *cf = coef + size_t(o) * 2;
        const f4 k1 = {cf[0], cf[2], cf[4], cf[6]};
        const f4 k2 = {cf[1], cf[3], cf[5], cf[7]};
        const f4 gm = gamma ? ld4(gamma + c) : f4{1.f, 1.f, 1.f, 1.f};
        const f4 mul = gm * iv;
        for (int64_t cell = ch.beg + pl; cell < ch.end; cell += npl) {
            f4 g[4];
            int64_t pix[4];
            bool ok[4];
            cell_grads<T, S2>(P, uint32_t(cell), c, g, pix, ok, y);
            f4 yv[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) yv[k] = ld4(y + cell_load_pix(pix, ok, k) * ldy + c);  // see above
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (ok[k]) {
                    const f4 ov = stored4(dy, bn_bwd_dy4(yv[k], g[k], mu, iv, sc, sf, k1, k2, mul));
                    st4(dy + pix[k] * lddy + c, ov);
                    acc += ov;
                    amax = fmax4(amax, fabs4(ov));
                }
        }
    }
    if (dy_bound) wave_max_bound(dy_bound, fmaxf(fmaxf(amax.x, amax.y), fmaxf(amax.z, amax.w)));
    if (!brec) return;  // uniform
    sh[tid] = acc;
    __syncthreads();
    for (int off = npl / 2; off > 0; off >>= 1) {
        if (pl < off) sh[tid] += sh[tid + off * qpb];
        __syncthreads();
    }
    if (pl == 0 && c < C) {
        const f4 a = sh[tid];
        const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) brec[size_t(c + k) * nrec + blockIdx.x] = av[k];
    }
}

// bn_bwd_pooled_apply for a Siamese pair (see bn_bwd_pooled_partial_pair): both segments' dy per cell, the conv-bias
// records of chunk k of each segment, bit-identical.
template <class T, bool S2>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_pooled_apply_pair(
    const T *__restrict__ y, int ldy, PooledCells<T> P, T *__restrict__ dy, int lddy, int C, int64_t cseg, int ncps,
    int chunk, int nrec, int qpb, const float *smean, const float *sinv, const float *gamma, const float *scale,
    const float *shift, const float *coef, float *__restrict__ brec, float *dy_bound) {
    __shared__ f4 sh[BN_THREADS];
    const int tid = threadIdx.x;
    const int q = tid % qpb, pl = tid / qpb, npl = BN_THREADS / qpb;
    const int c = (blockIdx.y * qpb + q) * 4;
    const Chunk ch = chunk_of(cseg, ncps, chunk);
    const int64_t poff = int64_t(P.da.gsn) * P.da.hx * P.da.wx;
    f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    f4 amax = acc0;
    if (c < C) {
        const f4 gm = gamma ? ld4(gamma + c) : f4{1.f, 1.f, 1.f, 1.f};
        const f4 mu0 = ld4(smean + c), iv0 = ld4(sinv + c), sc0 = ld4(scale + c), sf0 = ld4(shift + c);
        const f4 mu1 = ld4(smean + C + c), iv1 = ld4(sinv + C + c), sc1 = ld4(scale + C + c), sf1 = ld4(shift + C + c);
        const float *cf0 = coef + size_t(c) * 2, *cf1 = coef + size_t(C + c) * 2;
        const f4 k10 = {cf0[0], cf0[2], cf0[4], cf0[6]}, k20 = {cf0[1], cf0[3], cf0[5], cf0[7]};
        const f4 k11 = {cf1[0], cf1[2], cf1[4], cf1[6]}, k21 = {cf1[1], cf1[3], cf1[5], cf1[7]};
        const f4 mul0 = gm * iv0, mul1 = gm * iv1;
        for (int64_t cell = ch.beg + pl; cell < ch.end; cell += npl) {
            f4 g0[4], g1[4];
            int64_t pix[4];
            bool ok[4];
            cell_grads_pair<T, S2>(P, uint32_t(cell), c, g0, g1, pix, ok);
            f4 y0[4], y1[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {  // unconditional (a missing pixel reads the cell's first; not used)
                y0[k] = ld4(y + cell_load_pix(pix, ok, k) * ldy + c);
                y1[k] = ld4(y + (cell_load_pix(pix, ok, k) + poff) * ldy + c);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (ok[k]) {
                    const f4 o0 = stored4(dy, bn_bwd_dy4(y0[k], g0[k], mu0, iv0, sc0, sf0, k10, k20, mul0));
                    const f4 o1 = stored4(dy, bn_bwd_dy4(y1[k], g1[k], mu1, iv1, sc1, sf1, k11, k21, mul1));
                    st4(dy + pix[k] * lddy + c, o0);
                    st4(dy + (pix[k] + poff) * lddy + c, o1);
                    acc0 += o0;
                    acc1 += o1;
                    amax = fmax4(amax, fmax4(fabs4(o0), fabs4(o1)));
                }
        }
    }
    if (dy_bound) wave_max_bound(dy_bound, fmaxf(fmaxf(amax.x, amax.y), fmaxf(amax.z, amax.w)));
    if (!brec) return;  // uniform
#pragma unroll
    for (int sgm = 0; sgm < 2; ++sgm) {
        sh[tid] = sgm ? acc1 : acc0;
        __syncthreads();
        for (int off = npl / 2; off > 0; off >>= 1) {
            if (pl < off) sh[tid] += sh[tid + off * qpb];
            __syncthreads();
        }
        if (pl == 0 && c < C) {
            const f4 a = sh[tid];
            const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) brec[size_t(c + k) * nrec + sgm * ncps + blockIdx.x] = av[k];
        }
        __syncthreads();
    }
}

// per (chunk) record {sum dz, sum dz*xhat}, rec[c][chunk][2]
template <class T, class DA>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_partial(const T *__restrict__ y, int ldy, DA da, int C,
                                                             int64_t pseg, int ncps, int chunk, int nrec, int qpb,
                                                             const float *smean, const float *sinv, const float *scale,
                                                             const float *shift, float *__restrict__ rec) {
    __shared__ f4 sh1[BN_THREADS], sh2[BN_THREADS];
    const int tid = threadIdx.x;
    const int q = tid % qpb, pl = tid / qpb, npl = BN_THREADS / qpb;
    const int c = (blockIdx.y * qpb + q) * 4;
    const Chunk ch = chunk_of(pseg, ncps, chunk);
    f4 s1 = {0.f, 0.f, 0.f, 0.f}, s2 = s1;
    da.bind(c);
    if (c < C) {
        const int o = ch.seg * C + c;
        const f4 mu = ld4(smean + o), iv = ld4(sinv + o), sc = ld4(scale + o), sf = ld4(shift + o);
        int64_t p = ch.beg + pl;
        for (; p + 3 * npl < ch.end; p += 4 * npl) {
            f4 y0 = ld4(y + p * ldy + c), y1 = ld4(y + (p + npl) * ldy + c);
            f4 y2 = ld4(y + (p + 2 * npl) * ldy + c), y3 = ld4(y + (p + 3 * npl) * ldy + c);
            f4 g0 = da(p, c), g1 = da(p + npl, c);
            f4 g2 = da(p + 2 * npl, c), g3 = da(p + 3 * npl, c);
            PIN4(y0, y1, y2, y3);
            PIN4(g0, g1, g2, g3);
            const f4 z0 = relu_mask(y0, sc, sf, g0), z1 = relu_mask(y1, sc, sf, g1);
            const f4 z2 = relu_mask(y2, sc, sf, g2), z3 = relu_mask(y3, sc, sf, g3);
            s1 += (z0 + z1) + (z2 + z3);
            s2 += (z0 * ((y0 - mu) * iv) + z1 * ((y1 - mu) * iv)) + (z2 * ((y2 - mu) * iv) + z3 * ((y3 - mu) * iv));
        }
        for (; p < ch.end; p += npl) {
            const f4 y0 = ld4(y + p * ldy + c);
            const f4 z0 = relu_mask(y0, sc, sf, da(p, c));
            s1 += z0;
            s2 += z0 * ((y0 - mu) * iv);
        }
    }
    sh1[tid] = s1;
    sh2[tid] = s2;
    __syncthreads();
    for (int off = npl / 2; off > 0; off >>= 1) {
        if (pl < off) {
            sh1[tid] += sh1[tid + off * qpb];
            sh2[tid] += sh2[tid + off * qpb];
        }
        __syncthreads();
    }
    if (pl == 0 && c < C) {
        const f4 a = sh1[tid], b = sh2[tid];
        const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float *r = rec + (size_t(c + k) * nrec + blockIdx.x) * 2;
            r[0] = av[k];
            r[1] = bv[k];
        }
    }
}

// bn_bwd_partial for the head's BatchNorm (DaHead) that also takes the 1x1 head's weight grad from the same pass:
//   hrec[o][c][chunk] = sum_p gout[o](p) * relu(fma(y, scale, shift))(p, c)
// (what weighted_channel_sum's chan_sum_partial summed in a pass of its own over y; same chunks, per-thread order and
// tree).  The gradient values g_o(p) are loaded once per pixel for both the head's dL/da and the weight grad.
template <class T, int NO>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_partial_head(const T *__restrict__ y, int ldy, DaHead da, int C,
                                                                  int64_t pseg, int ncps, int chunk, int nrec, int qpb,
                                                                  const float *smean, const float *sinv,
                                                                  const float *scale, const float *shift,
                                                                  float *__restrict__ rec, float *__restrict__ hrec) {
    __shared__ f4 sh1[BN_THREADS], sh2[BN_THREADS], shh[NO][BN_THREADS];
    const int tid = threadIdx.x;
    const int q = tid % qpb, pl = tid / qpb, npl = BN_THREADS / qpb;
    const int c = (blockIdx.y * qpb + q) * 4;
    const Chunk ch = chunk_of(pseg, ncps, chunk);
    const f4 zero = {0.f, 0.f, 0.f, 0.f};
    f4 s1 = zero, s2 = zero, hw[NO];
#pragma unroll
    for (int k = 0; k < NO; ++k) hw[k] = zero;
    if (c < C) {
        const int o = ch.seg * C + c;
        const f4 mu = ld4(smean + o), iv = ld4(sinv + o), sc = ld4(scale + o), sf = ld4(shift + o);
        f4 w4[NO];
#pragma unroll
        for (int k = 0; k < NO; ++k) w4[k] = ld4(da.w + int64_t(k) * C + c);
        // one pixel: its n_out gradient values, dL/da (DaHead's fma chain) and the activation
        auto px = [&](int64_t p, f4 yv, f4 (&gk)[NO]) {
            const uint32_t img = fdiv(uint32_t(p), da.div_hw);
            const int pix = int(uint32_t(p) - img * uint32_t(da.hw));
            float gv[NO];
#pragma unroll
            for (int k = 0; k < NO; ++k) gv[k] = da.g[(int64_t(img) * NO + k) * da.hw + pix];
            f4 r = zero;
#pragma unroll
            for (int k = 0; k < NO; ++k) {
                gk[k] = f4{gv[k], gv[k], gv[k], gv[k]};
                r.x = fmaf(gv[k], w4[k].x, r.x);
                r.y = fmaf(gv[k], w4[k].y, r.y);
                r.z = fmaf(gv[k], w4[k].z, r.z);
                r.w = fmaf(gv[k], w4[k].w, r.w);
            }
            return r;
        };
        int64_t p = ch.beg + pl;
        for (; p + 3 * npl < ch.end; p += 4 * npl) {
            f4 y0 = ld4(y + p * ldy + c), y1 = ld4(y + (p + npl) * ldy + c);
            f4 y2 = ld4(y + (p + 2 * npl) * ldy + c), y3 = ld4(y + (p + 3 * npl) * ldy + c);
            f4 k0[NO], k1[NO], k2[NO], k3[NO];
            f4 g0 = px(p, y0, k0), g1 = px(p + npl, y1, k1);
            f4 g2 = px(p + 2 * npl, y2, k2), g3 = px(p + 3 * npl, y3, k3);
            PIN4(y0, y1, y2, y3);
            PIN4(g0, g1, g2, g3);
            const f4 z0 = relu_mask(y0, sc, sf, g0), z1 = relu_mask(y1, sc, sf, g1);
            const f4 z2 = relu_mask(y2, sc, sf, g2), z3 = relu_mask(y3, sc, sf, g3);
            s1 += (z0 + z1) + (z2 + z3);
            s2 += (z0 * ((y0 - mu) * iv) + z1 * ((y1 - mu) * iv)) + (z2 * ((y2 - mu) * iv) + z3 * ((y3 - mu) * iv));
            const f4 a0 = bn_relu4(y0, sc, sf), a1 = bn_relu4(y1, sc, sf);
            const f4 a2 = bn_relu4(y2, sc, sf), a3 = bn_relu4(y3, sc, sf);
#pragma unroll
            for (int k = 0; k < NO; ++k) hw[k] += (a0 * k0[k] + a1 * k1[k]) + (a2 * k2[k] + a3 * k3[k]);
        }
        for (; p < ch.end; p += npl) {
            const f4 y0 = ld4(y + p * ldy + c);
            f4 k0[NO];
            const f4 z0 = relu_mask(y0, sc, sf, px(p, y0, k0));
            s1 += z0;
            s2 += z0 * ((y0 - mu) * iv);
            const f4 a0 = bn_relu4(y0, sc, sf);
#pragma unroll
            for (int k = 0; k < NO; ++k) hw[k] += a0 * k0[k];
        }
    }
    sh1[tid] = s1;
    sh2[tid] = s2;
#pragma unroll
    for (int k = 0; k < NO; ++k) shh[k][tid] = hw[k];
    __syncthreads();
    for (int off = npl / 2; off > 0; off >>= 1) {
        if (pl < off) {
            sh1[tid] += sh1[tid + off * qpb];
            sh2[tid] += sh2[tid + off * qpb];
#pragma unroll
            for (int k = 0; k < NO; ++k) shh[k][tid] += shh[k][tid + off * qpb];
        }
        __syncthreads();
    }
    if (pl == 0 && c < C) {
        const f4 a = sh1[tid], b = sh2[tid];
        const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float *r = rec + (size_t(c + k) * nrec + blockIdx.x) * 2;
            r[0] = av[k];
            r[1] = bv[k];
        }
#pragma unroll
        for (int o = 0; o < NO; ++o) {
            const f4 h = shh[o][tid];
            const float hv[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) hrec[(size_t(o) * C + c + k) * nrec + blockIdx.x] = hv[k];
        }
    }
}

// Upper bound of |dy| = |gamma*invstd*(dz - k1 - xhat*k2)| over one segment and channel of n values from the statistics
// alone (the SCD_MATH_H2 operand bound of a weight grad that forms dy itself, scd_wgrad_t.rows_y): |dz| <= the bound
// of the incoming gradient, |xhat| <= sqrt(n - 1) (as bn_act_bound) plus the rounding of (y - mean) * invstd in fp32;
// a relative 2^-10 covers the rounding of the expression.
__device__ __forceinline__ float bn_dy_bound(double da_bound, double n, double gamma, double mean, double inv, double k1,
                                             double k2) {
    const double xhat = sqrt(n > 1 ? n - 1 : 0.0) * (1.0 + 0x1p-10) + fabs(mean) * inv * 0x1p-20 + 1.0;
    return float(fabs(gamma * inv) * (da_bound + fabs(k1) + xhat * fabs(k2)) * (1.0 + 0x1p-10));
}

// one workgroup per channel: coef[seg][C][2] = {mean(dz), mean(dz*xhat)}; dgamma/dbeta summed over segments.
// dbias (optional; the deferred form, whose dy is formed by its consumer and never summed): sum(dy) from the sums,
// sum_seg gamma*invstd * (S1 - pseg * k1) -- zero but for the rounding of k1, as BatchNorm removes the mean.
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_finalize(const float *__restrict__ rec, int C, int nseg,
                                                              int ncps, int nrec, int64_t pseg, float *coef,
                                                              float *dgamma, float *dbeta, const float *gamma = nullptr,
                                                              const float *sinv = nullptr, float *dbias = nullptr,
                                                              const float *smean = nullptr,
                                                              const float *da_bound = nullptr,
                                                              float *dy_bound = nullptr) {
    __shared__ double a1[BN_THREADS], a2[BN_THREADS];
    const int c = blockIdx.x;
    const int t = threadIdx.x;
    const float *rc = rec + size_t(c) * nrec * 2;
    double tg = 0, tb = 0, db = 0;
    for (int s = 0; s < nseg; ++s) {
        // 4 records per thread and trip, loads issued together (long tile-record lists are latency-bound otherwise);
        // fixed order: record k goes to accumulator (k / BN_THREADS) % 4
        double s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
        const float2 *rs = reinterpret_cast<const float2 *>(rc) + size_t(s) * ncps;
        int k = t;
        for (; k + 3 * BN_THREADS < ncps; k += 4 * BN_THREADS) {
            float2 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = rs[k + u * BN_THREADS];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                s1[u] += v[u].x;
                s2[u] += v[u].y;
            }
        }
        for (int u = 0; k < ncps; k += BN_THREADS, ++u) {
            const float2 v = rs[k];
            s1[u] += v.x;
            s2[u] += v.y;
        }
        double v1 = (s1[0] + s1[1]) + (s1[2] + s1[3]), v2 = (s2[0] + s2[1]) + (s2[2] + s2[3]);
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {  // fixed-order xor tree in the wave, then the waves in order
            v1 += __shfl_xor(v1, off);
            v2 += __shfl_xor(v2, off);
        }
        if ((t & 63) == 0) {
            a1[t >> 6] = v1;
            a2[t >> 6] = v2;
        }
        __syncthreads();
        if (t == 0) {
            for (int k = 1; k < BN_THREADS / 64; ++k) {
                a1[0] += a1[k];
                a2[0] += a2[k];
            }
            const float k1 = float(a1[0] / double(pseg));
            const float k2 = float(a2[0] / double(pseg));
            coef[(s * C + c) * 2 + 0] = k1;
            coef[(s * C + c) * 2 + 1] = k2;
            if (dy_bound) atomic_max_bound(dy_bound, bn_dy_bound(double(*da_bound), double(pseg), gamma ? gamma[c] : 1.0,
                                                                 smean[s * C + c], sinv[s * C + c], k1, k2));
            tb += a1[0];
            tg += a2[0];
            if (dbias) {
                const float mul = (gamma ? gamma[c] : 1.f) * sinv[s * C + c];
                db += double(mul) * (a1[0] - double(pseg) * double(k1));
            }
        }
        __syncthreads();
    }
    if (t == 0) {
        if (dgamma) dgamma[c] = float(tg);
        if (dbeta) dbeta[c] = float(tb);
        if (dbias) dbias[c] = float(db);
    }
}

// dy = gamma*invstd*(dz - k1 - xhat*k2); optional per-chunk sums of dy (conv bias grad), brec[c][chunk]
template <class T, class DA>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_apply(const T *__restrict__ y, int ldy, DA da,
                                                           T *__restrict__ dy, int lddy, int C, int64_t pseg,
                                                           int ncps, int chunk, int nrec, int qpb, const float *smean,
                                                           const float *sinv, const float *gamma, const float *scale,
                                                           const float *shift, const float *coef,
                                                           float *__restrict__ brec, float *dy_bound) {
    __shared__ f4 sh[BN_THREADS];
    const int tid = threadIdx.x;
    const int q = tid % qpb, pl = tid / qpb, npl = BN_THREADS / qpb;
    const int c = (blockIdx.y * qpb + q) * 4;
    const Chunk ch = chunk_of(pseg, ncps, chunk);
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    f4 amax = acc;  // max |dy| of this thread (dy_bound)
    da.bind(c);
    if (c < C) {
        const int o = ch.seg * C + c;
        const f4 mu = ld4(smean + o), iv = ld4(sinv + o), sc = ld4(scale + o), sf = ld4(shift + o);
        const float *cf = coef + size_t(o) * 2;
        const f4 k1 = {cf[0], cf[2], cf[4], cf[6]};
        const f4 k2 = {cf[1], cf[3], cf[5], cf[7]};
        const f4 gm = gamma ? ld4(gamma + c) : f4{1.f, 1.f, 1.f, 1.f};
        const f4 mul = gm * iv;
        int64_t p = ch.beg + pl;
        for (; p + 3 * npl < ch.end; p += 4 * npl) {
            f4 y0 = ld4(y + p * ldy + c), y1 = ld4(y + (p + npl) * ldy + c);
            f4 y2 = ld4(y + (p + 2 * npl) * ldy + c), y3 = ld4(y + (p + 3 * npl) * ldy + c);
            f4 g0 = da(p, c), g1 = da(p + npl, c);
            f4 g2 = da(p + 2 * npl, c), g3 = da(p + 3 * npl, c);
            PIN4(y0, y1, y2, y3);
            PIN4(g0, g1, g2, g3);
            const f4 o0 = stored4(dy, bn_bwd_dy4(y0, g0, mu, iv, sc, sf, k1, k2, mul));
            const f4 o1 = stored4(dy, bn_bwd_dy4(y1, g1, mu, iv, sc, sf, k1, k2, mul));
            const f4 o2 = stored4(dy, bn_bwd_dy4(y2, g2, mu, iv, sc, sf, k1, k2, mul));
            const f4 o3 = stored4(dy, bn_bwd_dy4(y3, g3, mu, iv, sc, sf, k1, k2, mul));
            st4(dy + p * lddy + c, o0);
            st4(dy + (p + npl) * lddy + c, o1);
            st4(dy + (p + 2 * npl) * lddy + c, o2);
            st4(dy + (p + 3 * npl) * lddy + c, o3);
            acc += (o0 + o1) + (o2 + o3);
            if (dy_bound) amax = fmax4(amax, fmax4(fmax4(fabs4(o0), fabs4(o1)), fmax4(fabs4(o2), fabs4(o3))));
        }
        for (; p < ch.end; p += npl) {
            const f4 y0 = ld4(y + p * ldy + c);
            const f4 o0 = stored4(dy, bn_bwd_dy4(y0, da(p, c), mu, iv, sc, sf, k1, k2, mul));
            st4(dy + p * lddy + c, o0);
            acc += o0;
            if (dy_bound) amax = fmax4(amax, fabs4(o0));
        }
    }
    if (dy_bound) wave_max_bound(dy_bound, fmaxf(fmaxf(amax.x, amax.y), fmaxf(amax.z, amax.w)));
    if (!brec) return;  // uniform
    sh[tid] = acc;
    __syncthreads();
    for (int off = npl / 2; off > 0; off >>= 1) {
        if (pl < off) sh[tid] += sh[tid + off * qpb];
        __syncthreads();
    }
    if (pl == 0 && c < C) {
        const f4 a = sh[tid];
        const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) brec[size_t(c + k) * nrec + blockIdx.x] = av[k];
    }
}

// out[c] = sum_r rec[c][r] (double, fixed tree); one workgroup per channel
__global__ __launch_bounds__(BN_THREADS) void sum_records(const float *__restrict__ rec, int nrec, float *out) {
    __shared__ double sh[BN_THREADS];
    const int c = blockIdx.x;
    const int t = threadIdx.x;
    double s = 0;
    for (int k = t; k < nrec; k += BN_THREADS) s += rec[size_t(c) * nrec + k];
    sh[t] = s;
    __syncthreads();
    for (int off = BN_THREADS / 2; off > 0; off >>= 1) {
        if (t < off) sh[t] += sh[t + off];
        __syncthreads();
    }
    if (t == 0) out[c] = float(sh[0]);
}

// Per-chunk channel sums (ConvTranspose2d bias grad) and weighted sums (1x1 head weight grad):
//   rec[c][chunk] = sum_p w(p) * v(p, c),  w(p) = 1 or gout[img][o][pix],
//   v = x, or (scale given) relu(fma(x, scale[seg][c], shift[seg][c])) -- the head's input read through the last
//   BatchNorm + ReLU with bn_relu_apply_kernel's expression (pseg pixels per segment).
// Four pixels' loads in flight per thread on both paths.
template <class T>
__global__ __launch_bounds__(BN_THREADS) void chan_sum_partial(const T *__restrict__ x, int ldx, int C,
                                                               int64_t npix, int chunk, int nrec, int qpb,
                                                               const float *__restrict__ wgt, int hw, int n_out,
                                                               int o, const float *__restrict__ scale,
                                                               const float *__restrict__ shift, int64_t pseg,
                                                               float *__restrict__ rec) {
    __shared__ f4 sh[BN_THREADS];
    const int tid = threadIdx.x;
    const int q = tid % qpb, pl = tid / qpb, npl = BN_THREADS / qpb;
    const int c = (blockIdx.y * qpb + q) * 4;
    const int64_t pbeg = int64_t(blockIdx.x) * chunk;
    const int64_t pend = min(pbeg + chunk, npix);
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    // The weighted path's per-pixel operands (the head gradient, the segment's coefficients) are loaded together
    // with the pixels, before any use; 32-bit index math where the map allows (npix < 2^31: the head's 256^2 maps)
    const bool small = npix < (int64_t(1) << 31);
    auto img_of = [&](int64_t p) { return small ? int64_t(uint32_t(p) / uint32_t(hw)) : p / hw; };
    auto seg_of = [&](int64_t p) { return small ? int64_t(uint32_t(p) / uint32_t(pseg)) : p / pseg; };
    auto wgt_at = [&](int64_t p) {
        const int64_t img = img_of(p), pix = p - img * hw;
        return wgt[(img * n_out + o) * hw + pix];
    };
    auto value = [&](int64_t p, f4 v, float wv) {
        if (scale) {
            const int64_t sc_off = seg_of(p) * C + c;
            v = bn_relu4(v, ld4(scale + sc_off), ld4(shift + sc_off));
        }
        if (wgt) v *= wv;
        return v;
    };
    if (c < C) {
        int64_t p = pbeg + pl;
        for (; p + 3 * npl < pend; p += 4 * npl) {
            f4 v0 = ld4(x + p * ldx + c), v1 = ld4(x + (p + npl) * ldx + c);
            f4 v2 = ld4(x + (p + 2 * npl) * ldx + c), v3 = ld4(x + (p + 3 * npl) * ldx + c);
            float w0 = 1.f, w1 = 1.f, w2 = 1.f, w3 = 1.f;
            if (wgt) {  // uniform
                w0 = wgt_at(p);
                w1 = wgt_at(p + npl);
                w2 = wgt_at(p + 2 * npl);
                w3 = wgt_at(p + 3 * npl);
            }
            PIN4(v0, v1, v2, v3);
            if (wgt || scale) {
                v0 = value(p, v0, w0);
                v1 = value(p + npl, v1, w1);
                v2 = value(p + 2 * npl, v2, w2);
                v3 = value(p + 3 * npl, v3, w3);
            }
            acc += (v0 + v1) + (v2 + v3);
        }
        for (; p < pend; p += npl) acc += value(p, ld4(x + p * ldx + c), wgt ? wgt_at(p) : 1.f);
    }
    sh[tid] = acc;
    __syncthreads();
    for (int off = npl / 2; off > 0; off >>= 1) {
        if (pl < off) sh[tid] += sh[tid + off * qpb];
        __syncthreads();
    }
    if (pl == 0 && c < C) {
        const f4 a = sh[tid];
        const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) rec[size_t(c + k) * nrec + blockIdx.x] = av[k];
    }
}

static int bn_check(const scd_nhwc_t &y, int nseg) {
    SCD_TRY(check_view(y, "bn.y"));
    if (nseg < 1 || y.n % nseg) {
        set_error("bn: nseg=%d must divide n=%d", nseg, y.n);
        return SCD_ERR_ARG;
    }
    return SCD_OK;
}

// Shared with misc_f32.hip (1x1 head weight grad).
size_t weighted_channel_sum_bytes(const scd_nhwc_t &x) {
    const BnGeom g = bn_geom(x, 1);
    return size_t(g.nrec) * x.c * sizeof(float);
}

int weighted_channel_sum(const scd_nhwc_t &x, const float *wgt, int n_out, int o, float *out, void *ws,
                         size_t ws_bytes, hipStream_t s, const float *scale = nullptr, const float *shift = nullptr,
                         int nseg = 1);

// scale / shift (optional, per segment of nseg): sum relu(fma(x, scale, shift)) instead of x.
int weighted_channel_sum(const scd_nhwc_t &x, const float *wgt, int n_out, int o, float *out, void *ws,
                         size_t ws_bytes, hipStream_t s, const float *scale, const float *shift, int nseg) {
    const BnGeom g = bn_geom(x, 1);
    if (!ws || ws_bytes < size_t(g.nrec) * x.c * sizeof(float)) {
        set_error("channel_sum: workspace too small");
        return SCD_ERR_WORKSPACE;
    }
    if ((scale != nullptr) != (shift != nullptr) || nseg < 1 || x.n % nseg) {
        set_error("channel_sum: scale and shift go together, nseg must divide n");
        return SCD_ERR_ARG;
    }
    float *rec = static_cast<float *>(ws);
    SCD_WITH_T(x.dtype, T,
               hipLaunchKernelGGL(chan_sum_partial<T>, dim3(g.nrec, g.cgroups), dim3(BN_THREADS), 0, s,
                                  view_ptr<const T>(x), x.ldc, x.c, pixels(x), g.chunk, g.nrec, g.qpb, wgt, x.h * x.w,
                                  n_out, o, scale, shift, pixels(x) / nseg, rec));
    hipLaunchKernelGGL(sum_records, dim3(x.c), dim3(BN_THREADS), 0, s, rec, g.nrec, out);
    return SCD_OK;
}

}  // namespace scd

using namespace scd;

extern "C" size_t scd_bn_workspace_bytes(int32_t n, int32_t h, int32_t w, int32_t c, int32_t nseg) {
    if (nseg < 1) nseg = 1;
    scd_nhwc_t v{nullptr, n, h, w, c, c};
    const BnGeom g = bn_geom(v, nseg);
    // stats: 3 floats/rec/channel; backward: 2 (+1 bias) floats/rec/channel + coef 2/seg/channel.
    const size_t a = size_t(g.nrec) * c * 3;
    const size_t b = size_t(g.nrec) * c * 3 + size_t(nseg) * c * 2;
    return (a > b ? a : b) * sizeof(float) + 256;
}

extern "C" int scd_bn_train_stats(scd_nhwc_t y, int32_t nseg, const float *gamma, const float *beta, float eps,
                                  float momentum, int32_t update_running, float *running_mean, float *running_var,
                                  float *save_mean, float *save_invstd, float *scale, float *shift, float *act_bound,
                                  void *ws, size_t ws_bytes, scd_stream_t stream) {
    clear_error();
    SCD_TRY(bn_check(y, nseg));
    if (!save_mean || !save_invstd || !scale || !shift || (update_running && (!running_mean || !running_var))) {
        set_error("bn_train_stats: null output");
        return SCD_ERR_ARG;
    }
    if (!ws || ws_bytes < scd_bn_workspace_bytes(y.n, y.h, y.w, y.c, nseg)) {
        set_error("bn_train_stats: workspace too small");
        return SCD_ERR_WORKSPACE;
    }
    const BnGeom g = bn_geom(y, nseg);
    hipStream_t s = as_stream(stream);
    float *rec = static_cast<float *>(ws);
    SCD_WITH_T(y.dtype, T,
               hipLaunchKernelGGL(bn_stats_partial<T>, dim3(g.nrec, g.cgroups), dim3(BN_THREADS), 0, s,
                                  view_ptr<const T>(y), y.ldc, y.c, g.pseg, g.ncps, g.chunk, g.nrec, g.qpb, rec));
    hipLaunchKernelGGL(bn_stats_finalize, dim3(y.c), dim3(BN_THREADS), 0, s, rec, y.c, nseg, g.ncps, g.nrec, gamma,
                       beta, eps, momentum, update_running, running_mean, running_var, save_mean, save_invstd, scale,
                       shift, act_bound);
    return launch_status("scd_bn_train_stats");
}

static void tile_groups(int ntiles, int nseg, int *tiles_per_seg, int *group, int *ncps) {
    *tiles_per_seg = ntiles / nseg;
    *group = *tiles_per_seg / 256 > 1 ? *tiles_per_seg / 256 : 1;
    *ncps = (*tiles_per_seg + *group - 1) / *group;
}

extern "C" size_t scd_bn_tile_stats_workspace_bytes(int32_t ntiles, int32_t c, int32_t nseg) {
    if (nseg < 1 || ntiles < 1 || c < 1) return 0;
    int tps, group, ncps;
    tile_groups(ntiles, nseg, &tps, &group, &ncps);
    return size_t(nseg) * ncps * c * 3 * sizeof(float) + 256;
}

extern "C" int scd_bn_stats_from_tiles(const float *tile_rec, int32_t ntiles, int32_t tile_pixels, int32_t c,
                                       int32_t nseg, const float *gamma, const float *beta, float eps, float momentum,
                                       int32_t update_running, float *running_mean, float *running_var,
                                       float *save_mean, float *save_invstd, float *scale, float *shift,
                                       float *act_bound, void *ws, size_t ws_bytes, scd_stream_t stream) {
    clear_error();
    if (!tile_rec || ntiles < 1 || tile_pixels < 1 || c < 1 || nseg < 1 || ntiles % nseg || !save_mean ||
        !save_invstd || !scale || !shift || (update_running && (!running_mean || !running_var))) {
        set_error("bn_stats_from_tiles: bad arguments");
        return SCD_ERR_ARG;
    }
    if (!ws || ws_bytes < scd_bn_tile_stats_workspace_bytes(ntiles, c, nseg)) {
        set_error("bn_stats_from_tiles: workspace too small");
        return SCD_ERR_WORKSPACE;
    }
    int tps, group, ncps;
    tile_groups(ntiles, nseg, &tps, &group, &ncps);
    const int nrec = nseg * ncps;
    float *rec = static_cast<float *>(ws);
    hipStream_t s = as_stream(stream);
    hipLaunchKernelGGL(bn_tile_merge, dim3(nrec, (c + BN_THREADS - 1) / BN_THREADS), dim3(BN_THREADS), 0, s, tile_rec,
                       c, tps, group, ncps, nrec, float(tile_pixels), rec);
    hipLaunchKernelGGL(bn_stats_finalize, dim3(c), dim3(BN_THREADS), 0, s, rec, c, nseg, ncps, nrec, gamma, beta, eps,
                       momentum, update_running, running_mean, running_var, save_mean, save_invstd, scale, shift,
                       act_bound);
    return launch_status("scd_bn_stats_from_tiles");
}

extern "C" int scd_bn_eval_coeffs(int32_t c, const float *gamma, const float *beta, const float *running_mean,
                                  const float *running_var, float eps, float *scale, float *shift,
                                  scd_stream_t stream) {
    clear_error();
    if (c < 1 || !running_mean || !running_var || !scale || !shift) {
        set_error("bn_eval_coeffs: bad arguments");
        return SCD_ERR_ARG;
    }
    hipLaunchKernelGGL(bn_eval_coeffs_kernel, dim3((c + 127) / 128), dim3(128), 0, as_stream(stream), c, gamma, beta,
                       running_mean, running_var, eps, scale, shift);
    return launch_status("scd_bn_eval_coeffs");
}

extern "C" int scd_bn_relu_apply(scd_nhwc_t y, int32_t nseg, const float *scale, const float *shift, scd_nhwc_t a,
                                 scd_stream_t stream) {
    clear_error();
    SCD_TRY(bn_check(y, nseg));
    SCD_TRY(check_view(a, "bn_relu_apply.a"));
    if (a.n != y.n || a.h != y.h || a.w != y.w || a.c != y.c || !scale || !shift) {
        set_error("bn_relu_apply: shape mismatch");
        return SCD_ERR_ARG;
    }
    const int dt = common_dtype("bn_relu_apply", {&y, &a});
    if (dt < 0) return SCD_ERR_ARG;
    const int64_t pseg = pixels(y) / nseg;
    const int64_t total = pseg * (y.c / 4);
    int blocks = int((total + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    SCD_WITH_T(dt, T,
               hipLaunchKernelGGL(bn_relu_apply_kernel<T>, dim3(blocks, nseg), dim3(256), 0, as_stream(stream),
                                  view_ptr<const T>(y), y.ldc, view_ptr<T>(a), a.ldc, y.c, pseg, scale, shift));
    return launch_status("scd_bn_relu_apply");
}

namespace scd {
// partial -> finalize -> apply (+ conv-bias sums) over a gradient source DA
template <class T, class DA>
static void bn_backward_run(const scd_nhwc_t &y, DA da, int nseg, const float *save_mean, const float *save_invstd,
                            const float *gamma, const float *scale, const float *shift, float *dgamma, float *dbeta,
                            float *dbias_prev, const scd_nhwc_t &dy, float *dy_bound, void *ws, hipStream_t s) {
    const BnGeom g = bn_geom(y, nseg);
    float *rec = static_cast<float *>(ws);
    float *brec = rec + size_t(g.nrec) * y.c * 2;
    float *coef = brec + size_t(g.nrec) * y.c;
    hipLaunchKernelGGL((bn_bwd_partial<T, DA>), dim3(g.nrec, g.cgroups), dim3(BN_THREADS), 0, s,
                       view_ptr<const T>(y), y.ldc, da, y.c, g.pseg, g.ncps, g.chunk, g.nrec, g.qpb,
                       save_mean, save_invstd, scale, shift, rec);
    hipLaunchKernelGGL(bn_bwd_finalize, dim3(y.c), dim3(BN_THREADS), 0, s, rec, y.c, nseg, g.ncps, g.nrec, g.pseg,
                       coef, dgamma, dbeta);
    hipLaunchKernelGGL((bn_bwd_apply<T, DA>), dim3(g.nrec, g.cgroups), dim3(BN_THREADS), 0, s,
                       view_ptr<const T>(y), y.ldc, da, view_ptr<T>(dy), dy.ldc, y.c,
                       g.pseg, g.ncps, g.chunk, g.nrec, g.qpb, save_mean, save_invstd, gamma, scale, shift, coef,
                       dbias_prev ? brec : nullptr, dy_bound);
    if (dbias_prev) hipLaunchKernelGGL(sum_records, dim3(y.c), dim3(BN_THREADS), 0, s, brec, g.nrec, dbias_prev);
}
// The head's BatchNorm backward (DaHead) with the head's weight grad from the same partial pass (w_grad non-null):
// hrec after the usual records (scd_bn_head_workspace_bytes).
template <class T, int NO>
static void bn_backward_run_head(const scd_nhwc_t &y, const DaHead &da, int nseg, const float *save_mean,
                                 const float *save_invstd, const float *gamma, const float *scale, const float *shift,
                                 float *dgamma, float *dbeta, float *dbias_prev, const scd_nhwc_t &dy, float *dy_bound,
                                 float *w_grad, void *ws, hipStream_t s) {
    const BnGeom g = bn_geom(y, nseg);
    float *rec = static_cast<float *>(ws);
    float *brec = rec + size_t(g.nrec) * y.c * 2;
    float *coef = brec + size_t(g.nrec) * y.c;
    float *hrec = reinterpret_cast<float *>(static_cast<unsigned char *>(ws) +
                                            scd_bn_workspace_bytes(y.n, y.h, y.w, y.c, nseg));
    hipLaunchKernelGGL((bn_bwd_partial_head<T, NO>), dim3(g.nrec, g.cgroups), dim3(BN_THREADS), 0, s,
                       view_ptr<const T>(y), y.ldc, da, y.c, g.pseg, g.ncps, g.chunk, g.nrec, g.qpb,
                       save_mean, save_invstd, scale, shift, rec, hrec);
    hipLaunchKernelGGL(bn_bwd_finalize, dim3(y.c), dim3(BN_THREADS), 0, s, rec, y.c, nseg, g.ncps, g.nrec, g.pseg,
                       coef, dgamma, dbeta);
    hipLaunchKernelGGL((bn_bwd_apply<T, DaHeadN<NO>>), dim3(g.nrec, g.cgroups), dim3(BN_THREADS), 0, s,
                       view_ptr<const T>(y), y.ldc, DaHeadN<NO>{da, {}}, view_ptr<T>(dy), dy.ldc, y.c,
                       g.pseg, g.ncps, g.chunk, g.nrec, g.qpb, save_mean, save_invstd, gamma, scale, shift, coef,
                       dbias_prev ? brec : nullptr, dy_bound);
    if (dbias_prev) hipLaunchKernelGGL(sum_records, dim3(y.c), dim3(BN_THREADS), 0, s, brec, g.nrec, dbias_prev);
    hipLaunchKernelGGL(sum_records, dim3(da.n_out * y.c), dim3(BN_THREADS), 0, s, hrec, g.nrec, w_grad);
}
// The encoder levels' BatchNorm backward with the pooled gradient (DaPooled) over 2x2 cells.  The chunks partition
// each segment's cells into at most bn_geom's chunk count, so the records fit the same workspace.
// Building with -DSCD_BN_POOLED_CELLS=0 runs the per-pixel kernels instead (A/B experiments; bit-identical).
#ifndef SCD_BN_POOLED_CELLS
#define SCD_BN_POOLED_CELLS 1
#endif
#ifndef SCD_BN_POOLED_PAIR
#define SCD_BN_POOLED_PAIR 1
#endif
template <class T, bool S2>
static void bn_backward_pooled_cells(const scd_nhwc_t &y, const PooledCells<T> &P, int nseg, const BnGeom &g,
                                     int64_t cseg, int chunk, int ncps, int nrec, const float *save_mean,
                                     const float *save_invstd, const float *gamma, const float *scale,
                                     const float *shift, float *dgamma, float *dbeta, float *dbias_prev,
                                     const scd_nhwc_t &dy, float *dy_bound, float *rec, float *brec, float *coef,
                                     hipStream_t s);
template <class T>
static void bn_backward_run_pooled(const scd_nhwc_t &y, const DaPooled<T> &da, int nseg, const float *save_mean,
                                   const float *save_invstd, const float *gamma, const float *scale, const float *shift,
                                   float *dgamma, float *dbeta, float *dbias_prev, const scd_nhwc_t &dy,
                                   float *dy_bound, void *ws, hipStream_t s) {
    if (!SCD_BN_POOLED_CELLS) {
        bn_backward_run<T>(y, da, nseg, save_mean, save_invstd, gamma, scale, shift, dgamma, dbeta, dbias_prev, dy,
                           dy_bound, ws, s);
        return;
    }
    const BnGeom g = bn_geom(y, nseg);
    PooledCells<T> P;
    P.da = da;
    P.ch = (y.h + 1) / 2;
    P.cw = (y.w + 1) / 2;
    P.div_cimg = make_fastdiv(uint32_t(P.ch * P.cw));
    P.div_cw = make_fastdiv(uint32_t(P.cw));
    const int64_t cseg = int64_t(y.n / nseg) * P.ch * P.cw;
    const int chunk = int((cseg + g.ncps - 1) / g.ncps);
    const int ncps = int((cseg + chunk - 1) / chunk);
    const int nrec = nseg * ncps;
    float *rec = static_cast<float *>(ws);
    float *brec = rec + size_t(g.nrec) * y.c * 2;
    float *coef = brec + size_t(g.nrec) * y.c;
    // Siamese pairs (-DSCD_BN_POOLED_PAIR=0: one image per cell walk): the t1 and t2 cells at one place in one block,
    // the shared difference gradient read once instead of once per branch
    if (da.gs2) {
        bn_backward_pooled_cells<T, true>(y, P, nseg, g, cseg, chunk, ncps, nrec, save_mean, save_invstd, gamma, scale,
                                          shift, dgamma, dbeta, dbias_prev, dy, dy_bound, rec, brec, coef, s);
    } else {
        bn_backward_pooled_cells<T, false>(y, P, nseg, g, cseg, chunk, ncps, nrec, save_mean, save_invstd, gamma, scale,
                                           shift, dgamma, dbeta, dbias_prev, dy, dy_bound, rec, brec, coef, s);
    }
}

template <class T, bool S2>
static void bn_backward_pooled_cells(const scd_nhwc_t &y, const PooledCells<T> &P, int nseg, const BnGeom &g,
                                     int64_t cseg, int chunk, int ncps, int nrec, const float *save_mean,
                                     const float *save_invstd, const float *gamma, const float *scale,
                                     const float *shift, float *dgamma, float *dbeta, float *dbias_prev,
                                     const scd_nhwc_t &dy, float *dy_bound, float *rec, float *brec, float *coef,
                                     hipStream_t s) {
    const DaPooled<T> &da = P.da;
    if (SCD_BN_POOLED_PAIR && nseg == 2 && da.gs && (da.skip_mode == 1 || da.skip_mode == 2) && 2 * da.gsn == y.n) {
        hipLaunchKernelGGL((bn_bwd_pooled_partial_pair<T, S2>), dim3(ncps, g.cgroups), dim3(BN_THREADS), 0, s,
                           view_ptr<const T>(y), y.ldc, P, y.c, cseg, ncps, chunk, nrec, g.qpb, save_mean,
                           save_invstd, scale, shift, rec);
        hipLaunchKernelGGL(bn_bwd_finalize, dim3(y.c), dim3(BN_THREADS), 0, s, rec, y.c, nseg, ncps, nrec, g.pseg,
                           coef, dgamma, dbeta);
        hipLaunchKernelGGL((bn_bwd_pooled_apply_pair<T, S2>), dim3(ncps, g.cgroups), dim3(BN_THREADS), 0, s,
                           view_ptr<const T>(y), y.ldc, P, view_ptr<T>(dy), dy.ldc, y.c,
                           cseg, ncps, chunk, nrec, g.qpb, save_mean, save_invstd, gamma, scale, shift, coef,
                           dbias_prev ? brec : nullptr, dy_bound);
        if (dbias_prev) hipLaunchKernelGGL(sum_records, dim3(y.c), dim3(BN_THREADS), 0, s, brec, nrec, dbias_prev);
        return;
    }
    hipLaunchKernelGGL((bn_bwd_pooled_partial<T, S2>), dim3(nrec, g.cgroups), dim3(BN_THREADS), 0, s,
                       view_ptr<const T>(y), y.ldc, P, y.c, cseg, ncps, chunk, nrec, g.qpb, save_mean,
                       save_invstd, scale, shift, rec);
    hipLaunchKernelGGL(bn_bwd_finalize, dim3(y.c), dim3(BN_THREADS), 0, s, rec, y.c, nseg, ncps, nrec, g.pseg, coef,
                       dgamma, dbeta);
    hipLaunchKernelGGL((bn_bwd_pooled_apply<T, S2>), dim3(nrec, g.cgroups), dim3(BN_THREADS), 0, s,
                       view_ptr<const T>(y), y.ldc, P, view_ptr<T>(dy), dy.ldc, y.c, cseg,
                       ncps, chunk, nrec, g.qpb, save_mean, save_invstd, gamma, scale, shift, coef,
                       dbias_prev ? brec : nullptr, dy_bound);
    if (dbias_prev) hipLaunchKernelGGL(sum_records, dim3(y.c), dim3(BN_THREADS), 0, s, brec, nrec, dbias_prev);
}
}  // namespace scd

extern "C" int scd_bn_relu_backward(scd_nhwc_t y, scd_nhwc_t da, int32_t nseg, const float *save_mean,
                                    const float *save_invstd, const float *gamma, const float *scale,
                                    const float *shift, float *dgamma, float *dbeta, float *dbias_prev,
                                    scd_nhwc_t dy, float *dy_bound, void *ws, size_t ws_bytes, scd_stream_t stream) {
    clear_error();
    SCD_TRY(bn_check(y, nseg));
    SCD_TRY(check_view(da, "bn_bwd.da"));
    SCD_TRY(check_view(dy, "bn_bwd.dy"));
    if (da.n != y.n || da.h != y.h || da.w != y.w || da.c != y.c || dy.n != y.n || dy.h != y.h || dy.w != y.w ||
        dy.c != y.c || !save_mean || !save_invstd || !scale || !shift) {
        set_error("bn_relu_backward: shape mismatch / null");
        return SCD_ERR_ARG;
    }
    if (!ws || ws_bytes < scd_bn_workspace_bytes(y.n, y.h, y.w, y.c, nseg)) {
        set_error("bn_relu_backward: workspace too small");
        return SCD_ERR_WORKSPACE;
    }
    const int dt = common_dtype("bn_relu_backward", {&y, &da, &dy});
    if (dt < 0) return SCD_ERR_ARG;
    SCD_WITH_T(dt, T,
               bn_backward_run<T>(y, DaPlain<T>{view_ptr<const T>(da), da.ldc}, nseg, save_mean, save_invstd, gamma,
                                  scale, shift, dgamma, dbeta, dbias_prev, dy, dy_bound, ws, as_stream(stream)));
    return launch_status("scd_bn_relu_backward");
}

extern "C" size_t scd_bn_head_workspace_bytes(int32_t n, int32_t h, int32_t w, int32_t c, int32_t nseg,
                                              int32_t n_out) {
    if (nseg < 1) nseg = 1;
    scd_nhwc_t v{nullptr, n, h, w, c, c};
    const BnGeom g = bn_geom(v, nseg);
    return scd_bn_workspace_bytes(n, h, w, c, nseg) + size_t(n_out > 0 ? n_out : 1) * c * g.nrec * sizeof(float);
}

extern "C" int scd_bn_relu_backward_head(scd_nhwc_t y, const float *gout, const float *w_head, int32_t n_out,
                                         int32_t nseg, const float *save_mean, const float *save_invstd,
                                         const float *gamma, const float *scale, const float *shift, float *dgamma,
                                         float *dbeta, float *dbias_prev, scd_nhwc_t dy, float *dy_bound,
                                         float *w_grad, void *ws, size_t ws_bytes, scd_stream_t stream) {
    clear_error();
    SCD_TRY(bn_check(y, nseg));
    SCD_TRY(check_view(dy, "bn_bwd_head.dy"));
    if (!gout || !w_head || n_out < 1 || n_out > 4 || dy.n != y.n || dy.h != y.h || dy.w != y.w || dy.c != y.c ||
        !save_mean || !save_invstd || !scale || !shift || pixels(y) >= (int64_t(1) << 31)) {
        set_error("bn_relu_backward_head: shape mismatch / null / n_out not in [1,4] / 2^31 pixels or more");
        return SCD_ERR_ARG;
    }
    const size_t need = w_grad ? scd_bn_head_workspace_bytes(y.n, y.h, y.w, y.c, nseg, n_out)
                               : scd_bn_workspace_bytes(y.n, y.h, y.w, y.c, nseg);
    if (!ws || ws_bytes < need) {
        set_error("bn_relu_backward_head: workspace %zu < %zu bytes", ws_bytes, need);
        return SCD_ERR_WORKSPACE;
    }
    const DaHead da{gout, w_head, n_out, y.c, y.h * y.w, make_fastdiv(uint32_t(y.h * y.w))};
    const int dt = common_dtype("bn_relu_backward_head", {&y, &dy});
    if (dt < 0) return SCD_ERR_ARG;
    auto run = [&](auto no) {
        constexpr int NO = decltype(no)::value;
        if (w_grad) {
            SCD_WITH_T(dt, T,
                       (bn_backward_run_head<T, NO>(y, da, nseg, save_mean, save_invstd, gamma, scale, shift, dgamma,
                                                    dbeta, dbias_prev, dy, dy_bound, w_grad, ws, as_stream(stream))));
        } else {
            SCD_WITH_T(dt, T,
                       bn_backward_run<T>(y, DaHeadN<NO>{da, {}}, nseg, save_mean, save_invstd, gamma, scale, shift,
                                          dgamma, dbeta, dbias_prev, dy, dy_bound, ws, as_stream(stream)));
        }
    };
    switch (n_out) {
        case 1: run(std::integral_constant<int, 1>{}); break;
        case 2: run(std::integral_constant<int, 2>{}); break;
        case 3: run(std::integral_constant<int, 3>{}); break;
        default: run(std::integral_constant<int, 4>{}); break;
    }
    return launch_status("scd_bn_relu_backward_head");
}

extern "C" int scd_bn_relu_backward_pooled(scd_nhwc_t y, scd_nhwc_t gy, const uint8_t *idx, scd_nhwc_t gskip,
                                           int32_t skip_mode, int32_t nseg, const float *save_mean,
                                           const float *save_invstd, const float *gamma, const float *scale,
                                           const float *shift, float *dgamma, float *dbeta, float *dbias_prev,
                                           scd_nhwc_t dy, float *dy_bound, void *ws, size_t ws_bytes, scd_stream_t stream) {
    if (skip_mode == 2) {
        clear_error();
        set_error("bn_relu_backward_pooled: skip_mode 2 takes a second skip gradient (scd_bn_relu_backward_pooled2)");
        return SCD_ERR_ARG;
    }
    return scd_bn_relu_backward_pooled2(y, gy, idx, gskip, skip_mode, scd_nhwc_t{}, nseg, save_mean, save_invstd, gamma,
                                        scale, shift, dgamma, dbeta, dbias_prev, dy, dy_bound, ws, ws_bytes, stream);
}

extern "C" int scd_bn_relu_backward_pooled2(scd_nhwc_t y, scd_nhwc_t gy, const uint8_t *idx, scd_nhwc_t gskip,
                                            int32_t skip_mode, scd_nhwc_t gskip2, int32_t nseg,
                                            const float *save_mean, const float *save_invstd, const float *gamma,
                                            const float *scale, const float *shift, float *dgamma, float *dbeta,
                                            float *dbias_prev, scd_nhwc_t dy, float *dy_bound, void *ws,
                                            size_t ws_bytes, scd_stream_t stream) {
    clear_error();
    SCD_TRY(bn_check(y, nseg));
    SCD_TRY(check_view(gy, "bn_bwd_pooled.gy", true));
    SCD_TRY(check_view(gskip, "bn_bwd_pooled.gskip", true));
    SCD_TRY(check_view(gskip2, "bn_bwd_pooled.gskip2", true));
    SCD_TRY(check_view(dy, "bn_bwd_pooled.dy"));
    if (dy.n != y.n || dy.h != y.h || dy.w != y.w || dy.c != y.c || !save_mean || !save_invstd || !scale || !shift ||
        (!gy.data && !gskip.data) || pixels(y) >= (int64_t(1) << 31)) {
        set_error("bn_relu_backward_pooled: shape mismatch / null");
        return SCD_ERR_ARG;
    }
    if (gy.data && (!idx || gy.n != y.n || gy.c != y.c || gy.h != y.h / 2 || gy.w != y.w / 2 ||
                    (reinterpret_cast<uintptr_t>(idx) & 3))) {
        set_error("bn_relu_backward_pooled: gy must be (n, h/2, w/2, c) with 4-byte aligned idx");
        return SCD_ERR_ARG;
    }
    if (gskip.data && (gskip.c != y.c || gskip.h != y.h || gskip.w != y.w || y.n % gskip.n ||
                       (skip_mode != 0 && y.n != 2 * gskip.n) || skip_mode < 0 || skip_mode > 2)) {
        set_error("bn_relu_backward_pooled: gskip shape/mode mismatch");
        return SCD_ERR_ARG;
    }
    if ((skip_mode == 2) != (gskip2.data != nullptr) ||
        (gskip2.data && (!gskip.data || nseg != 2 || gskip2.n != y.n || gskip2.h != y.h || gskip2.w != y.w ||
                         gskip2.c != y.c))) {
        set_error("bn_relu_backward_pooled: skip_mode 2 needs gskip (n/2 images), gskip2 (n images) and nseg 2; "
                  "gskip2 only with skip_mode 2");
        return SCD_ERR_ARG;
    }
    if (!ws || ws_bytes < scd_bn_workspace_bytes(y.n, y.h, y.w, y.c, nseg)) {
        set_error("bn_relu_backward_pooled: workspace too small");
        return SCD_ERR_WORKSPACE;
    }
    const int dt = common_dtype("bn_relu_backward_pooled", {&y, &gy, &gskip, &gskip2, &dy});
    if (dt < 0) return SCD_ERR_ARG;
    SCD_WITH_T(dt, T, {
        DaPooled<T> da;
        da.gy = view_ptr<const T>(gy);
        da.idx = idx;
        da.hy = gy.h;
        da.wy = gy.w;
        da.ldgy = gy.ldc;
        da.gs = view_ptr<const T>(gskip);
        da.gsn = gskip.n > 0 ? gskip.n : 1;
        da.ldgs = gskip.ldc;
        da.skip_mode = skip_mode;
        da.gs2 = view_ptr<const T>(gskip2);
        da.ldgs2 = gskip2.ldc;
        da.hx = y.h;
        da.wx = y.w;
        da.C = y.c;
        da.div_hw = make_fastdiv(uint32_t(y.h * y.w));
        da.div_w = make_fastdiv(uint32_t(y.w));
        da.div_gsn = make_fastdiv(uint32_t(da.gsn));
        bn_backward_run_pooled<T>(y, da, nseg, save_mean, save_invstd, gamma, scale, shift, dgamma, dbeta, dbias_prev,
                                  dy, dy_bound, ws, as_stream(stream));
    });
    return launch_status("scd_bn_relu_backward_pooled");
}

extern "C" int scd_bn_relu_backward_tiles(scd_nhwc_t y, scd_nhwc_t da, int32_t nseg, const float *save_mean,
                                          const float *save_invstd, const float *gamma, const float *scale,
                                          const float *shift, const float *tile_rec, int32_t ntiles, float *dgamma,
                                          float *dbeta, float *dbias_prev, scd_nhwc_t dy, float *dy_bound, void *ws, size_t ws_bytes,
                                          scd_stream_t stream) {
    clear_error();
    SCD_TRY(bn_check(y, nseg));
    SCD_TRY(check_view(da, "bn_bwd.da"));
    SCD_TRY(check_view(dy, "bn_bwd.dy"));
    if (da.n != y.n || da.h != y.h || da.w != y.w || da.c != y.c || dy.n != y.n || dy.h != y.h || dy.w != y.w ||
        dy.c != y.c || !save_mean || !save_invstd || !scale || !shift || !tile_rec || ntiles < nseg ||
        ntiles % nseg || pixels(y) % ntiles) {
        set_error("bn_relu_backward_tiles: shape mismatch / null / %d tiles not divisible into %d segments", ntiles,
                  nseg);
        return SCD_ERR_ARG;
    }
    if (!ws || ws_bytes < scd_bn_workspace_bytes(y.n, y.h, y.w, y.c, nseg)) {
        set_error("bn_relu_backward_tiles: workspace too small");
        return SCD_ERR_WORKSPACE;
    }
    const BnGeom g = bn_geom(y, nseg);
    float *brec = static_cast<float *>(ws);
    float *coef = brec + size_t(g.nrec) * y.c;
    hipStream_t s = as_stream(stream);
    hipLaunchKernelGGL(bn_bwd_finalize, dim3(y.c), dim3(BN_THREADS), 0, s, tile_rec, y.c, nseg, ntiles / nseg, ntiles,
                       g.pseg, coef, dgamma, dbeta);
    const int dt = common_dtype("bn_relu_backward_tiles", {&y, &da, &dy});
    if (dt < 0) return SCD_ERR_ARG;
    SCD_WITH_T(dt, T,
               hipLaunchKernelGGL((bn_bwd_apply<T, DaPlain<T>>), dim3(g.nrec, g.cgroups), dim3(BN_THREADS), 0, s,
                                  view_ptr<const T>(y), y.ldc, DaPlain<T>{view_ptr<const T>(da), da.ldc},
                                  view_ptr<T>(dy), dy.ldc, y.c, g.pseg, g.ncps, g.chunk, g.nrec, g.qpb, save_mean,
                                  save_invstd, gamma, scale, shift, coef, dbias_prev ? brec : nullptr, dy_bound));
    if (dbias_prev) hipLaunchKernelGGL(sum_records, dim3(y.c), dim3(BN_THREADS), 0, s, brec, g.nrec, dbias_prev);
    return launch_status("scd_bn_relu_backward_tiles");
}

extern "C" int scd_bn_relu_backward_coef(scd_nhwc_t y, scd_nhwc_t da, int32_t nseg, const float *save_mean,
                                         const float *save_invstd, const float *gamma, const float *scale,
                                         const float *shift, const float *tile_rec, int32_t ntiles, float *coef,
                                         float *dgamma, float *dbeta, float *dbias_prev, const float *da_bound,
                                         float *dy_bound, void *ws, size_t ws_bytes, scd_stream_t stream) {
    clear_error();
    SCD_TRY(bn_check(y, nseg));
    SCD_TRY(check_view(da, "bn_bwd_coef.da", tile_rec != nullptr));
    if ((!tile_rec && (da.n != y.n || da.h != y.h || da.w != y.w || da.c != y.c)) || !save_mean || !save_invstd ||
        !scale || !shift || !coef || (tile_rec && (ntiles < nseg || ntiles % nseg || pixels(y) % ntiles)) ||
        (dy_bound && !da_bound)) {
        set_error("bn_relu_backward_coef: shape mismatch / null / %d tiles not divisible into %d segments / dy_bound "
                  "without da_bound", ntiles, nseg);
        return SCD_ERR_ARG;
    }
    if (!ws || ws_bytes < scd_bn_workspace_bytes(y.n, y.h, y.w, y.c, nseg)) {
        set_error("bn_relu_backward_coef: workspace too small");
        return SCD_ERR_WORKSPACE;
    }
    const BnGeom g = bn_geom(y, nseg);
    hipStream_t s = as_stream(stream);
    if (tile_rec) {
        hipLaunchKernelGGL(bn_bwd_finalize, dim3(y.c), dim3(BN_THREADS), 0, s, tile_rec, y.c, nseg, ntiles / nseg,
                           ntiles, g.pseg, coef, dgamma, dbeta, gamma, save_invstd, dbias_prev, save_mean, da_bound,
                           dy_bound);
    } else {
        float *rec = static_cast<float *>(ws);
        const int dt = common_dtype("bn_relu_backward_coef", {&y, &da});
        if (dt < 0) return SCD_ERR_ARG;
        SCD_WITH_T(dt, T,
                   hipLaunchKernelGGL((bn_bwd_partial<T, DaPlain<T>>), dim3(g.nrec, g.cgroups), dim3(BN_THREADS), 0, s,
                                      view_ptr<const T>(y), y.ldc, DaPlain<T>{view_ptr<const T>(da), da.ldc}, y.c,
                                      g.pseg, g.ncps, g.chunk, g.nrec, g.qpb, save_mean, save_invstd, scale, shift,
                                      rec));
        hipLaunchKernelGGL(bn_bwd_finalize, dim3(y.c), dim3(BN_THREADS), 0, s, rec, y.c, nseg, g.ncps, g.nrec, g.pseg,
                           coef, dgamma, dbeta, gamma, save_invstd, dbias_prev, save_mean, da_bound, dy_bound);
    }
    return launch_status("scd_bn_relu_backward_coef");
}

extern "C" int scd_channel_sum(scd_nhwc_t x, float *out, void *ws, size_t ws_bytes, scd_stream_t stream) {
    clear_error();
    SCD_TRY(check_view(x, "channel_sum.x"));
    if (!out) {
        set_error("channel_sum: null output");
        return SCD_ERR_ARG;
    }
    SCD_TRY(weighted_channel_sum(x, nullptr, 1, 0, out, ws, ws_bytes, as_stream(stream)));
    return launch_status("scd_channel_sum");
}

namespace scd {
// bound = max(bound, max |v|) over an NHWC view, v = x or relu(fma(x, scale[g][c], shift[g][c])) (g = segment).
__global__ __launch_bounds__(256) void absmax_bound_kernel(const float *__restrict__ x, int ldx, int C, int64_t pseg,
                                                           const float *__restrict__ scale,
                                                           const float *__restrict__ shift, float *bound) {
    const int seg = blockIdx.y;
    const int cq = C / 4;
    const int64_t total = pseg * cq;
    f4 m = {0.f, 0.f, 0.f, 0.f};
    for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < total; e += int64_t(gridDim.x) * blockDim.x) {
        const int64_t p = seg * pseg + e / cq;
        const int c = int(e % cq) * 4;
        f4 v = ld4(x + p * ldx + c);
        if (scale) v = bn_relu4(v, ld4(scale + seg * C + c), ld4(shift + seg * C + c));
        m = fmax4(m, fabs4(v));
    }
    wave_max_bound(bound, fmaxf(fmaxf(m.x, m.y), fmaxf(m.z, m.w)));
}
}  // namespace scd

extern "C" int scd_absmax_bound(scd_nhwc_t x, int32_t nseg, const float *scale, const float *shift, float *bound,
                                scd_stream_t stream) {
    clear_error();
    SCD_TRY(bn_check(x, nseg));
    if (!bound || (!scale) != (!shift) || (scale && (!aligned16(scale) || !aligned16(shift))) || is_bf16(x)) {
        set_error("absmax_bound: null bound, unpaired / unaligned coefficients or a bf16 view (h2 bounds are fp32-only)");
        return SCD_ERR_ARG;
    }
    const int64_t pseg = pixels(x) / nseg;
    const int64_t total = pseg * (x.c / 4);
    int blocks = int((total + 255) / 256);
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(absmax_bound_kernel, dim3(blocks, nseg), dim3(256), 0, as_stream(stream),
                       static_cast<const float *>(x.data), x.ldc, x.c, pseg, scale, shift, bound);
    return launch_status("scd_absmax_bound");
}
