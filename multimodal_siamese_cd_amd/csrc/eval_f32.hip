// Eval-path kernels: the Up zero-pad window copy (networks.py:437-443) and the fused multi-threshold
// confusion counts of MultiThresholdMetric.add_sample (utils/metrics.py:22-31) with the sigmoid of
// utils/evaluation.py:25 folded in.  Both are HBM-bound streaming passes.
#include "common.h"

namespace scd {

// dst[n, y, x, :] = src[n, y + oy, x + ox, :] where that pixel exists, else 0.  One row of dst per grid.y
// step, channel quads of the row across grid.x (the row-decomposed grid of misc_f32.hip).
template <class T>
__global__ void window_copy_kernel(const T *__restrict__ src, int hs, int ws, int lds, T *__restrict__ dst,
                                   int hd, int wd, int ldd, int C, int oy, int ox, int rows, FastDiv div_cq) {
    const int cq = C / 4;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= wd * cq) return;
    const int x = int(fdiv(uint32_t(e), div_cq));
    const int c = (e - x * cq) * 4;
    const int sx = x + ox;
    for (int row = blockIdx.y; row < rows; row += gridDim.y) {
        const int img = row / hd, y = row - img * hd;
        const int sy = y + oy;
        bnf4 v = {0.f, 0.f, 0.f, 0.f};
        if (sy >= 0 && sy < hs && sx >= 0 && sx < ws) v = ld4(src + ((int64_t(img) * hs + sy) * ws + sx) * lds + c);
        st4(dst + (int64_t(row) * wd + x) * ldd + c, v);
    }
}

// ------------------------------------------------------------------------------------------------
// Confusion counts.  metrics.py:26 decides y_pred_offset = round(p - t + 0.5).bool() in fp32: the value
// v = (p - t) + 0.5 (two roundings, no fma) is "true" unless round-half-even(v) == 0, i.e. unless
// -0.5 <= v <= 0.5; NaN is true.  y_true.bool() is y != 0 (NaN true).
// Counters per launch: [0] = #true labels, then per threshold k: [1 + 2k] = TP(k), [2 + 2k] = #pred(k).
// TN/FP/FN follow exactly on the host (integers).
constexpr int MT_MAX = 16;      // thresholds per launch (registers)
constexpr int MT_BLOCKS = 512;  // partial-record blocks

__device__ __forceinline__ float mt_sigmoid(float x) { return 1.f / (1.f + expf(-x)); }

template <int T>
__device__ __forceinline__ void mt_count(float p, float y, const float *thr, uint32_t &nt, uint32_t (&tp)[T],
                                         uint32_t (&pp)[T]) {
    const bool t = y != 0.f;
    nt += t;
#pragma unroll
    for (int k = 0; k < T; ++k) {
        const float d = __fsub_rn(p, thr[k]);
        const float v = __fadd_rn(d, 0.5f);
        const bool pr = !(v >= -0.5f && v <= 0.5f);
        pp[k] += pr;
        tp[k] += pr & t;
    }
}

template <int T>
__global__ __launch_bounds__(256) void threshold_counts_partial(const float *__restrict__ pred,
                                                                const float *__restrict__ truth, int64_t n,
                                                                const float *__restrict__ thr_g, int from_logits,
                                                                unsigned long long *__restrict__ rec) {
    float thr[T];
#pragma unroll
    for (int k = 0; k < T; ++k) thr[k] = thr_g[k];
    uint32_t nt = 0, tp[T], pp[T];
#pragma unroll
    for (int k = 0; k < T; ++k) tp[k] = pp[k] = 0;
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    const int64_t n4 = n / 4;
    for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n4; i += stride) {
        float4 p = reinterpret_cast<const float4 *>(pred)[i];
        const float4 y = reinterpret_cast<const float4 *>(truth)[i];
        if (from_logits) p = make_float4(mt_sigmoid(p.x), mt_sigmoid(p.y), mt_sigmoid(p.z), mt_sigmoid(p.w));
        mt_count<T>(p.x, y.x, thr, nt, tp, pp);
        mt_count<T>(p.y, y.y, thr, nt, tp, pp);
        mt_count<T>(p.z, y.z, thr, nt, tp, pp);
        mt_count<T>(p.w, y.w, thr, nt, tp, pp);
    }
    for (int64_t i = n4 * 4 + blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += stride) {
        const float p = from_logits ? mt_sigmoid(pred[i]) : pred[i];
        mt_count<T>(p, truth[i], thr, nt, tp, pp);
    }
    // 64-bit wave sums (DPP/permute shuffles), then the block's 4 waves through LDS
    constexpr int NC = 1 + 2 * T;
    __shared__ unsigned long long part[4][NC];
    uint32_t v[NC];
    v[0] = nt;
#pragma unroll
    for (int k = 0; k < T; ++k) {
        v[1 + 2 * k] = tp[k];
        v[2 + 2 * k] = pp[k];
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        unsigned long long s = v[j];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
        if (lane == 0) part[wave][j] = s;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < NC; j += blockDim.x)
        rec[int64_t(blockIdx.x) * NC + j] = part[0][j] + part[1][j] + part[2][j] + part[3][j];
}

// counts[j] = sum over blocks of rec[block][j] (fixed order per column; integers, so exact anyway).
__global__ __launch_bounds__(256) void threshold_counts_finalize(const unsigned long long *__restrict__ rec,
                                                                 int nblocks, int nc, int64_t *__restrict__ counts) {
    __shared__ unsigned long long s[256];
    for (int j = 0; j < nc; ++j) {
        unsigned long long a = 0;
        for (int b = threadIdx.x; b < nblocks; b += 256) a += rec[int64_t(b) * nc + j];
        s[threadIdx.x] = a;
        __syncthreads();
        for (int off = 128; off > 0; off >>= 1) {
            if (threadIdx.x < off) s[threadIdx.x] += s[threadIdx.x + off];
            __syncthreads();
        }
        if (threadIdx.x == 0) counts[j] = int64_t(s[0]);
        __syncthreads();
    }
}

template <int T>
static void launch_counts(const float *pred, const float *truth, int64_t n, const float *thr, int from_logits,
                          unsigned long long *rec, int blocks, int64_t *counts, hipStream_t s) {
    hipLaunchKernelGGL(threshold_counts_partial<T>, dim3(blocks), dim3(256), 0, s, pred, truth, n, thr, from_logits,
                       rec);
    hipLaunchKernelGGL(threshold_counts_finalize, dim3(1), dim3(256), 0, s, rec, blocks, 1 + 2 * T, counts);
}

static int mt_blocks(int64_t n) {
    int64_t b = (n / 4 + 255) / 256;
    if (b > MT_BLOCKS) b = MT_BLOCKS;
    return int(b < 1 ? 1 : b);
}

}  // namespace scd

using namespace scd;

extern "C" int scd_window_copy(scd_nhwc_t src, scd_nhwc_t dst, int32_t oy, int32_t ox, scd_stream_t stream) {
    clear_error();
    SCD_TRY(check_view(src, "window_copy.src"));
    SCD_TRY(check_view(dst, "window_copy.dst"));
    if (src.n != dst.n || src.c != dst.c) {
        set_error("window_copy: src and dst must have the same n and c");
        return SCD_ERR_ARG;
    }
    const int64_t rows = int64_t(dst.n) * dst.h;
    if (rows > INT32_MAX || int64_t(dst.w) * (dst.c / 4) > INT32_MAX) {
        set_error("window_copy: view too large");
        return SCD_ERR_ARG;
    }
    const int quads = dst.w * (dst.c / 4);
    const int dt = common_dtype("window_copy", {&src, &dst});
    if (dt < 0) return SCD_ERR_ARG;
    SCD_WITH_T(dt, T,
               hipLaunchKernelGGL(window_copy_kernel<T>,
                                  dim3(unsigned((quads + 255) / 256), unsigned(rows < 65535 ? rows : 65535)), dim3(256),
                                  0, as_stream(stream), view_ptr<const T>(src), src.h, src.w, src.ldc, view_ptr<T>(dst),
                                  dst.h, dst.w, dst.ldc, dst.c, oy, ox, int(rows), make_fastdiv(uint32_t(dst.c / 4))));
    return launch_status("scd_window_copy");
}

extern "C" size_t scd_threshold_counts_workspace_bytes(int64_t n, int32_t n_thr) {
    if (n < 1 || n_thr < 1 || n_thr > MT_MAX) return 0;
    return size_t(mt_blocks(n)) * size_t(1 + 2 * n_thr) * sizeof(unsigned long long);
}

extern "C" int scd_threshold_counts(const float *pred, const float *truth, int64_t n, const float *thresholds,
                                    int32_t n_thr, int32_t from_logits, int64_t *counts, void *ws, size_t ws_bytes,
                                    scd_stream_t stream) {
    clear_error();
    if (!pred || !truth || !thresholds || !counts || n < 1 || n_thr < 1 || n_thr > MT_MAX) {
        set_error("threshold_counts: bad arguments (1 <= n_thr <= %d)", MT_MAX);
        return SCD_ERR_ARG;
    }
    if (!aligned16(pred) || !aligned16(truth)) {
        set_error("threshold_counts: pred and truth must be 16-byte aligned");
        return SCD_ERR_ALIGN;
    }
    if (!ws || ws_bytes < scd_threshold_counts_workspace_bytes(n, n_thr)) {
        set_error("threshold_counts: workspace too small");
        return SCD_ERR_WORKSPACE;
    }
    const int blocks = mt_blocks(n);
    auto *rec = static_cast<unsigned long long *>(ws);
    hipStream_t s = as_stream(stream);
    switch (n_thr) {
#define SCD_MT_CASE(T) \
    case T: launch_counts<T>(pred, truth, n, thresholds, from_logits, rec, blocks, counts, s); break;
        SCD_MT_CASE(1) SCD_MT_CASE(2) SCD_MT_CASE(3) SCD_MT_CASE(4) SCD_MT_CASE(5) SCD_MT_CASE(6) SCD_MT_CASE(7)
        SCD_MT_CASE(8) SCD_MT_CASE(9) SCD_MT_CASE(10) SCD_MT_CASE(11) SCD_MT_CASE(12) SCD_MT_CASE(13)
        SCD_MT_CASE(14) SCD_MT_CASE(15) SCD_MT_CASE(16)
#undef SCD_MT_CASE
    }
    return launch_status("scd_threshold_counts");
}
