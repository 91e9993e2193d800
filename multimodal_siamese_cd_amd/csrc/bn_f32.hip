// BatchNorm2d (+ fused ReLU) kernels over NHWC fp32, per-segment batch statistics.
//
// Replaces aten::native_batch_norm / native_batch_norm_backward / relu_ / threshold_backward for the
// reference's `Conv2d -> BatchNorm2d -> ReLU(inplace)` pairs (utils/networks.py:392-397).
// Reductions are chunked: each workgroup reduces one (segment, pixel-chunk, channel-group) tile
// (Welford in registers, Chan merges in LDS), then one thread per channel merges the chunk records in
// double, in chunk order — deterministic and free of E[x^2]-E[x]^2 cancellation.
#include "common.h"

namespace scd {

constexpr int BN_THREADS = 256;
constexpr int BN_CHUNK = 4096;  // pixels per reduction chunk

struct BnGeom {
    int64_t pseg;   // pixels per segment
    int ncps;       // chunks per segment
    int qpb;        // channel quads per block (power of two)
    int cgroups;    // channel groups (grid.y)
};

static BnGeom bn_geom(const scd_nhwc_t &y, int nseg) {
    BnGeom g;
    g.pseg = pixels(y) / nseg;
    g.ncps = int((g.pseg + BN_CHUNK - 1) / BN_CHUNK);
    const int cq = y.c / 4;
    int q = 1;
    while (q * 2 <= cq && q * 2 <= 64) q *= 2;
    g.qpb = q;
    g.cgroups = (cq + q - 1) / q;
    return g;
}

struct Welford4 {
    float n;
    float mean[4], m2[4];
};

__device__ __forceinline__ void chan_merge(Welford4 &a, const Welford4 &b) {
    const float n = a.n + b.n;
    if (b.n == 0.f) return;
    if (a.n == 0.f) {
        a = b;
        return;
    }
    const float fb = b.n / n;
    const float fab = a.n * b.n / n;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float d = b.mean[k] - a.mean[k];
        a.mean[k] += d * fb;
        a.m2[k] += b.m2[k] + d * d * fab;
    }
    a.n = n;
}

// records: [nseg*ncps][C][3] = {count, mean, m2}
__global__ __launch_bounds__(BN_THREADS) void bn_stats_partial(const float *__restrict__ y, int ldc, int C,
                                                               int64_t pseg, int ncps, int qpb,
                                                               float *__restrict__ rec) {
    __shared__ Welford4 sh[BN_THREADS];
    const int tid = threadIdx.x;
    const int q = tid % qpb, pl = tid / qpb, npl = BN_THREADS / qpb;
    const int cq = blockIdx.y * qpb + q;
    const int seg = blockIdx.x / ncps, chunk = blockIdx.x % ncps;
    const int64_t pbeg = seg * pseg + int64_t(chunk) * BN_CHUNK;
    const int64_t pend = min(pbeg + BN_CHUNK, (seg + 1) * pseg);
    Welford4 w;
    w.n = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) w.mean[k] = w.m2[k] = 0.f;
    if (cq * 4 < C) {
        for (int64_t p = pbeg + pl; p < pend; p += npl) {
            const float4 v = *reinterpret_cast<const float4 *>(y + p * ldc + cq * 4);
            w.n += 1.f;
            const float inv = 1.f / w.n;
            const float x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float d = x[k] - w.mean[k];
                w.mean[k] += d * inv;
                w.m2[k] += d * (x[k] - w.mean[k]);
            }
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
    if (pl == 0 && cq * 4 < C) {
        const Welford4 a = sh[tid];
        float *r = rec + (size_t(blockIdx.x) * C + cq * 4) * 3;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            r[3 * k + 0] = a.n;
            r[3 * k + 1] = a.mean[k];
            r[3 * k + 2] = a.m2[k];
        }
    }
}

__global__ void bn_stats_finalize(const float *__restrict__ rec, int C, int nseg, int ncps, const float *gamma,
                                  const float *beta, float eps, float momentum, int update, float *rmean,
                                  float *rvar, float *smean, float *sinv, float *scale, float *shift) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const double g = gamma ? gamma[c] : 1.0, b = beta ? beta[c] : 0.0;
    for (int s = 0; s < nseg; ++s) {
        double n = 0, mean = 0, m2 = 0;
        for (int k = 0; k < ncps; ++k) {
            const float *r = rec + (size_t(s * ncps + k) * C + c) * 3;
            const double nb = r[0];
            if (nb == 0) continue;
            const double d = r[1] - mean;
            const double nn = n + nb;
            mean += d * nb / nn;
            m2 += r[2] + d * d * n * nb / nn;
            n = nn;
        }
        const double var = n > 0 ? m2 / n : 0.0;
        const double inv = 1.0 / sqrt(var + double(eps));
        smean[s * C + c] = float(mean);
        sinv[s * C + c] = float(inv);
        const float sc = float(g * inv);
        scale[s * C + c] = sc;
        shift[s * C + c] = float(b - mean * double(sc));
        if (update) {
            const double uvar = n > 1 ? m2 / (n - 1) : var;
            rmean[c] = float((1.0 - momentum) * rmean[c] + momentum * mean);
            rvar[c] = float((1.0 - momentum) * rvar[c] + momentum * uvar);
        }
    }
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

// grid: (chunks, segments); each thread walks quads of its segment's pixels.
__global__ __launch_bounds__(256) void bn_relu_apply_kernel(const float *__restrict__ y, int ldy, float *__restrict__ a,
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
        const float4 v = *reinterpret_cast<const float4 *>(y + p * ldy + c);
        const float4 s4 = *reinterpret_cast<const float4 *>(sc + c);
        const float4 h4 = *reinterpret_cast<const float4 *>(sh + c);
        float4 o;
        o.x = bn_relu(v.x, s4.x, h4.x);
        o.y = bn_relu(v.y, s4.y, h4.y);
        o.z = bn_relu(v.z, s4.z, h4.z);
        o.w = bn_relu(v.w, s4.w, h4.w);
        *reinterpret_cast<float4 *>(a + p * lda + c) = o;
    }
}

// Backward reduce: per (chunk, C) record {sum dz, sum dz*xhat}.
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_partial(const float *__restrict__ y, int ldy,
                                                             const float *__restrict__ da, int ldda, int C,
                                                             int64_t pseg, int ncps, int qpb, const float *smean,
                                                             const float *sinv, const float *scale, const float *shift,
                                                             float *__restrict__ rec) {
    __shared__ float4 sh1[BN_THREADS], sh2[BN_THREADS];
    const int tid = threadIdx.x;
    const int q = tid % qpb, pl = tid / qpb, npl = BN_THREADS / qpb;
    const int cq = blockIdx.y * qpb + q;
    const int seg = blockIdx.x / ncps, chunk = blockIdx.x % ncps;
    const int64_t pbeg = seg * pseg + int64_t(chunk) * BN_CHUNK;
    const int64_t pend = min(pbeg + BN_CHUNK, (seg + 1) * pseg);
    float4 s1 = make_float4(0, 0, 0, 0), s2 = make_float4(0, 0, 0, 0);
    if (cq * 4 < C) {
        const int c = cq * 4;
        const float4 mu = *reinterpret_cast<const float4 *>(smean + seg * C + c);
        const float4 iv = *reinterpret_cast<const float4 *>(sinv + seg * C + c);
        const float4 sc = *reinterpret_cast<const float4 *>(scale + seg * C + c);
        const float4 sf = *reinterpret_cast<const float4 *>(shift + seg * C + c);
        for (int64_t p = pbeg + pl; p < pend; p += npl) {
            const float4 v = *reinterpret_cast<const float4 *>(y + p * ldy + c);
            const float4 g = *reinterpret_cast<const float4 *>(da + p * ldda + c);
            float dz;
            dz = fmaf(v.x, sc.x, sf.x) > 0.f ? g.x : 0.f;
            s1.x += dz;
            s2.x += dz * ((v.x - mu.x) * iv.x);
            dz = fmaf(v.y, sc.y, sf.y) > 0.f ? g.y : 0.f;
            s1.y += dz;
            s2.y += dz * ((v.y - mu.y) * iv.y);
            dz = fmaf(v.z, sc.z, sf.z) > 0.f ? g.z : 0.f;
            s1.z += dz;
            s2.z += dz * ((v.z - mu.z) * iv.z);
            dz = fmaf(v.w, sc.w, sf.w) > 0.f ? g.w : 0.f;
            s1.w += dz;
            s2.w += dz * ((v.w - mu.w) * iv.w);
        }
    }
    sh1[tid] = s1;
    sh2[tid] = s2;
    __syncthreads();
    for (int off = npl / 2; off > 0; off >>= 1) {
        if (pl < off) {
            float4 a = sh1[tid], b = sh1[tid + off * qpb];
            sh1[tid] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
            a = sh2[tid];
            b = sh2[tid + off * qpb];
            sh2[tid] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
        }
        __syncthreads();
    }
    if (pl == 0 && cq * 4 < C) {
        float *r = rec + (size_t(blockIdx.x) * C + cq * 4) * 2;
        const float4 a = sh1[tid], b = sh2[tid];
        r[0] = a.x; r[1] = b.x;
        r[2] = a.y; r[3] = b.y;
        r[4] = a.z; r[5] = b.z;
        r[6] = a.w; r[7] = b.w;
    }
}

// coef[seg][C][2] = {mean(dz), mean(dz*xhat)}; dgamma/dbeta summed over segments.
__global__ void bn_bwd_finalize(const float *__restrict__ rec, int C, int nseg, int ncps, int64_t pseg,
                                float *coef, float *dgamma, float *dbeta) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    double tg = 0, tb = 0;
    for (int s = 0; s < nseg; ++s) {
        double s1 = 0, s2 = 0;
        for (int k = 0; k < ncps; ++k) {
            const float *r = rec + (size_t(s * ncps + k) * C + c) * 2;
            s1 += r[0];
            s2 += r[1];
        }
        coef[(s * C + c) * 2 + 0] = float(s1 / double(pseg));
        coef[(s * C + c) * 2 + 1] = float(s2 / double(pseg));
        tg += s2;
        tb += s1;
    }
    if (dgamma) dgamma[c] = float(tg);
    if (dbeta) dbeta[c] = float(tb);
}

// dy = gamma*invstd*(dz - k1 - xhat*k2); optional per-chunk sums of dy (conv bias grad).
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_apply(const float *__restrict__ y, int ldy,
                                                           const float *__restrict__ da, int ldda,
                                                           float *__restrict__ dy, int lddy, int C, int64_t pseg,
                                                           int ncps, int qpb, const float *smean, const float *sinv,
                                                           const float *gamma, const float *scale, const float *shift,
                                                           const float *coef, float *__restrict__ brec) {
    __shared__ float4 sh[BN_THREADS];
    const int tid = threadIdx.x;
    const int q = tid % qpb, pl = tid / qpb, npl = BN_THREADS / qpb;
    const int cq = blockIdx.y * qpb + q;
    const int seg = blockIdx.x / ncps, chunk = blockIdx.x % ncps;
    const int64_t pbeg = seg * pseg + int64_t(chunk) * BN_CHUNK;
    const int64_t pend = min(pbeg + BN_CHUNK, (seg + 1) * pseg);
    float4 acc = make_float4(0, 0, 0, 0);
    if (cq * 4 < C) {
        const int c = cq * 4;
        const float4 mu = *reinterpret_cast<const float4 *>(smean + seg * C + c);
        const float4 iv = *reinterpret_cast<const float4 *>(sinv + seg * C + c);
        const float4 sc = *reinterpret_cast<const float4 *>(scale + seg * C + c);
        const float4 sf = *reinterpret_cast<const float4 *>(shift + seg * C + c);
        const float *cf = coef + (seg * C + c) * 2;
        const float k1[4] = {cf[0], cf[2], cf[4], cf[6]};
        const float k2[4] = {cf[1], cf[3], cf[5], cf[7]};
        const float gm[4] = {gamma ? gamma[c] : 1.f, gamma ? gamma[c + 1] : 1.f, gamma ? gamma[c + 2] : 1.f,
                             gamma ? gamma[c + 3] : 1.f};
        const float mul[4] = {gm[0] * iv.x, gm[1] * iv.y, gm[2] * iv.z, gm[3] * iv.w};
        const float mus[4] = {mu.x, mu.y, mu.z, mu.w};
        const float ivs[4] = {iv.x, iv.y, iv.z, iv.w};
        const float scs[4] = {sc.x, sc.y, sc.z, sc.w};
        const float sfs[4] = {sf.x, sf.y, sf.z, sf.w};
        for (int64_t p = pbeg + pl; p < pend; p += npl) {
            const float4 v4 = *reinterpret_cast<const float4 *>(y + p * ldy + c);
            const float4 g4 = *reinterpret_cast<const float4 *>(da + p * ldda + c);
            const float v[4] = {v4.x, v4.y, v4.z, v4.w};
            const float g[4] = {g4.x, g4.y, g4.z, g4.w};
            float o[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float dz = fmaf(v[k], scs[k], sfs[k]) > 0.f ? g[k] : 0.f;
                const float xh = (v[k] - mus[k]) * ivs[k];
                o[k] = mul[k] * (dz - k1[k] - xh * k2[k]);
            }
            *reinterpret_cast<float4 *>(dy + p * lddy + c) = make_float4(o[0], o[1], o[2], o[3]);
            acc.x += o[0];
            acc.y += o[1];
            acc.z += o[2];
            acc.w += o[3];
        }
    }
    if (!brec) return;  // uniform
    sh[tid] = acc;
    __syncthreads();
    for (int off = npl / 2; off > 0; off >>= 1) {
        if (pl < off) {
            const float4 a = sh[tid], b = sh[tid + off * qpb];
            sh[tid] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
        }
        __syncthreads();
    }
    if (pl == 0 && cq * 4 < C) {
        const float4 a = sh[tid];
        float *r = brec + size_t(blockIdx.x) * C + cq * 4;
        r[0] = a.x;
        r[1] = a.y;
        r[2] = a.z;
        r[3] = a.w;
    }
}

__global__ void sum_records(const float *__restrict__ rec, int nrec, int C, float *out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    double s = 0;
    for (int k = 0; k < nrec; ++k) s += rec[size_t(k) * C + c];
    out[c] = float(s);
}

// Per-chunk channel sums (ConvTranspose2d bias grad): rec[chunk][C].
__global__ __launch_bounds__(BN_THREADS) void chan_sum_partial(const float *__restrict__ x, int ldx, int C,
                                                               int64_t npix, int qpb, float *__restrict__ rec) {
    __shared__ float4 sh[BN_THREADS];
    const int tid = threadIdx.x;
    const int q = tid % qpb, pl = tid / qpb, npl = BN_THREADS / qpb;
    const int cq = blockIdx.y * qpb + q;
    const int64_t pbeg = int64_t(blockIdx.x) * BN_CHUNK;
    const int64_t pend = min(pbeg + BN_CHUNK, npix);
    float4 acc = make_float4(0, 0, 0, 0);
    if (cq * 4 < C) {
        for (int64_t p = pbeg + pl; p < pend; p += npl) {
            const float4 v = *reinterpret_cast<const float4 *>(x + p * ldx + cq * 4);
            acc.x += v.x;
            acc.y += v.y;
            acc.z += v.z;
            acc.w += v.w;
        }
    }
    sh[tid] = acc;
    __syncthreads();
    for (int off = npl / 2; off > 0; off >>= 1) {
        if (pl < off) {
            const float4 a = sh[tid], b = sh[tid + off * qpb];
            sh[tid] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
        }
        __syncthreads();
    }
    if (pl == 0 && cq * 4 < C) *reinterpret_cast<float4 *>(rec + size_t(blockIdx.x) * C + cq * 4) = sh[tid];
}

static int bn_check(const scd_nhwc_t &y, int nseg) {
    SCD_TRY(check_view(y, "bn.y"));
    if (nseg < 1 || y.n % nseg) {
        set_error("bn: nseg=%d must divide n=%d", nseg, y.n);
        return SCD_ERR_ARG;
    }
    return SCD_OK;
}

}  // namespace scd

using namespace scd;

extern "C" size_t scd_bn_workspace_bytes(int32_t n, int32_t h, int32_t w, int32_t c, int32_t nseg) {
    if (nseg < 1) nseg = 1;
    scd_nhwc_t v{nullptr, n, h, w, c, c};
    const BnGeom g = bn_geom(v, nseg);
    const size_t nrec = size_t(nseg) * g.ncps;
    // stats: 3 floats/rec/channel; backward: 2 (+1 bias) floats/rec/channel + coef 2/seg/channel.
    const size_t a = nrec * c * 3;
    const size_t b = nrec * c * 3 + size_t(nseg) * c * 2;
    return (a > b ? a : b) * sizeof(float) + 256;
}

extern "C" int scd_bn_train_stats(scd_nhwc_t y, int32_t nseg, const float *gamma, const float *beta, float eps,
                                  float momentum, int32_t update_running, float *running_mean, float *running_var,
                                  float *save_mean, float *save_invstd, float *scale, float *shift, void *ws,
                                  size_t ws_bytes, scd_stream_t stream) {
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
    hipLaunchKernelGGL(bn_stats_partial, dim3(nseg * g.ncps, g.cgroups), dim3(BN_THREADS), 0, s,
                       static_cast<const float *>(y.data), y.ldc, y.c, g.pseg, g.ncps, g.qpb, rec);
    hipLaunchKernelGGL(bn_stats_finalize, dim3((y.c + 127) / 128), dim3(128), 0, s, rec, y.c, nseg, g.ncps, gamma,
                       beta, eps, momentum, update_running, running_mean, running_var, save_mean, save_invstd,
                       scale, shift);
    return launch_status("scd_bn_train_stats");
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
    const int64_t pseg = pixels(y) / nseg;
    const int64_t total = pseg * (y.c / 4);
    int blocks = int((total + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(bn_relu_apply_kernel, dim3(blocks, nseg), dim3(256), 0, as_stream(stream),
                       static_cast<const float *>(y.data), y.ldc, static_cast<float *>(a.data), a.ldc, y.c, pseg,
                       scale, shift);
    return launch_status("scd_bn_relu_apply");
}

extern "C" int scd_bn_relu_backward(scd_nhwc_t y, scd_nhwc_t da, int32_t nseg, const float *save_mean,
                                    const float *save_invstd, const float *gamma, const float *scale,
                                    const float *shift, float *dgamma, float *dbeta, float *dbias_prev,
                                    scd_nhwc_t dy, void *ws, size_t ws_bytes, scd_stream_t stream) {
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
    const BnGeom g = bn_geom(y, nseg);
    const int nrec = nseg * g.ncps;
    float *rec = static_cast<float *>(ws);
    float *brec = rec + size_t(nrec) * y.c * 2;
    float *coef = brec + size_t(nrec) * y.c;
    hipStream_t s = as_stream(stream);
    hipLaunchKernelGGL(bn_bwd_partial, dim3(nrec, g.cgroups), dim3(BN_THREADS), 0, s,
                       static_cast<const float *>(y.data), y.ldc, static_cast<const float *>(da.data), da.ldc, y.c,
                       g.pseg, g.ncps, g.qpb, save_mean, save_invstd, scale, shift, rec);
    hipLaunchKernelGGL(bn_bwd_finalize, dim3((y.c + 127) / 128), dim3(128), 0, s, rec, y.c, nseg, g.ncps, g.pseg, coef,
                       dgamma, dbeta);
    hipLaunchKernelGGL(bn_bwd_apply, dim3(nrec, g.cgroups), dim3(BN_THREADS), 0, s,
                       static_cast<const float *>(y.data), y.ldc, static_cast<const float *>(da.data), da.ldc,
                       static_cast<float *>(dy.data), dy.ldc, y.c, g.pseg, g.ncps, g.qpb, save_mean, save_invstd, gamma,
                       scale, shift, coef, dbias_prev ? brec : nullptr);
    if (dbias_prev)
        hipLaunchKernelGGL(sum_records, dim3((y.c + 127) / 128), dim3(128), 0, s, brec, nrec, y.c, dbias_prev);
    return launch_status("scd_bn_relu_backward");
}

extern "C" int scd_channel_sum(scd_nhwc_t x, float *out, void *ws, size_t ws_bytes, scd_stream_t stream) {
    clear_error();
    SCD_TRY(check_view(x, "channel_sum.x"));
    if (!out) {
        set_error("channel_sum: null output");
        return SCD_ERR_ARG;
    }
    if (!ws || ws_bytes < scd_bn_workspace_bytes(x.n, x.h, x.w, x.c, 1)) {
        set_error("channel_sum: workspace too small");
        return SCD_ERR_WORKSPACE;
    }
    const BnGeom g = bn_geom(x, 1);
    float *rec = static_cast<float *>(ws);
    hipStream_t s = as_stream(stream);
    hipLaunchKernelGGL(chan_sum_partial, dim3(g.ncps, g.cgroups), dim3(BN_THREADS), 0, s,
                       static_cast<const float *>(x.data), x.ldc, x.c, pixels(x), g.qpb, rec);
    hipLaunchKernelGGL(sum_records, dim3((x.c + 127) / 128), dim3(128), 0, s, rec, g.ncps, x.c, out);
    return launch_status("scd_channel_sum");
}
