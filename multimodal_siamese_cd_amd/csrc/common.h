// Internal helpers shared by the libscd translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../../include/scd.h"

namespace scd {

void set_error(const char *fmt, ...);
void clear_error();

inline hipStream_t as_stream(scd_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Validate an NHWC view used with 16-byte vector accesses.
inline int check_view(const scd_nhwc_t &v, const char *name, bool allow_null = false) {
    if (v.data == nullptr) {
        if (allow_null) return SCD_OK;
        set_error("%s: null data", name);
        return SCD_ERR_ARG;
    }
    if (v.n <= 0 || v.h <= 0 || v.w <= 0 || v.c <= 0 || v.ldc < v.c) {
        set_error("%s: bad shape n=%d h=%d w=%d c=%d ldc=%d", name, v.n, v.h, v.w, v.c, v.ldc);
        return SCD_ERR_ARG;
    }
    if ((v.c & 3) || (v.ldc & 3) || !aligned16(v.data)) {
        set_error("%s: c=%d / ldc=%d must be multiples of 4 and data 16-byte aligned", name, v.c, v.ldc);
        return SCD_ERR_ALIGN;
    }
    return SCD_OK;
}

inline int64_t pixels(const scd_nhwc_t &v) { return int64_t(v.n) * v.h * v.w; }

inline int launch_status(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return SCD_ERR_LAUNCH;
    }
    return SCD_OK;
}

#define SCD_TRY(expr)                 \
    do {                              \
        int _rc = (expr);             \
        if (_rc != SCD_OK) return _rc; \
    } while (0)

// Division by a runtime constant: n / d = (umulhi(n, mul) + n) >> shr, valid for n < 2^31.
struct FastDiv {
    uint32_t d, mul, shr;
};

inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f;
    f.d = d;
    uint32_t s = 0;
    while ((1ull << s) < d) ++s;
    f.shr = s;
    f.mul = uint32_t(((1ull << 32) * ((1ull << s) - d)) / d + 1);
    return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv &f) {
    return (__umulhi(n, f.mul) + n) >> f.shr;
}

// Magnitude bounds (SCD_MATH_H2 operand scaling): a non-negative float's bits order as unsigned integers, so an
// integer atomic max keeps max(*bound, v) whatever the arrival order (deterministic).  NaN compares above +inf.
// A bound only grows, so the atomic is skipped when a plain read (possibly stale: then smaller) already covers v --
// the same final value with far fewer same-address atomics, which serialise in one L2 channel (a ConvTranspose
// forward issuing one per wave ran 2x slower).
__device__ __forceinline__ void atomic_max_bound(float *bound, float v) {
    unsigned int *const p = reinterpret_cast<unsigned int *>(bound);
    const unsigned int u = __float_as_uint(fabsf(v));
    if (u > __atomic_load_n(p, __ATOMIC_RELAXED)) atomicMax(p, u);
}
// Max of v over the wave, then one atomic from lane 0.
__device__ __forceinline__ void wave_max_bound(float *bound, float v) {
    v = fabsf(v);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    if ((threadIdx.x & 63) == 0) atomic_max_bound(bound, v);
}

// BatchNorm + ReLU backward of one channel quad, shared by bn_bwd_apply and the weight grad's fused dY staging so
// both form the same bits:  dz = g where fma(y, sc, sf) > 0 (the forward's exact ReLU test), else 0;
//   dy = mul * (dz - k1 - ((y - mu) * iv) * k2),  mul = gamma * invstd, k1 = mean(dz), k2 = mean(dz * xhat).
typedef float bnf4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ bnf4 relu_mask(bnf4 y, bnf4 sc, bnf4 sf, bnf4 g) {
    return bnf4{fmaf(y.x, sc.x, sf.x) > 0.f ? g.x : 0.f, fmaf(y.y, sc.y, sf.y) > 0.f ? g.y : 0.f,
                fmaf(y.z, sc.z, sf.z) > 0.f ? g.z : 0.f, fmaf(y.w, sc.w, sf.w) > 0.f ? g.w : 0.f};
}
__device__ __forceinline__ bnf4 bn_bwd_dy4(bnf4 y, bnf4 g, bnf4 mu, bnf4 iv, bnf4 sc, bnf4 sf, bnf4 k1, bnf4 k2,
                                           bnf4 mul) {
#pragma clang fp contract(off)  // no fma formation that could differ between the two call sites
    return mul * (relu_mask(y, sc, sf, g) - k1 - ((y - mu) * iv) * k2);
}

// Device-side NHWC element pointer helpers.
struct View {
    float *p;
    int n, h, w, c, ldc;
};

inline View make_view(const scd_nhwc_t &v) {
    return View{static_cast<float *>(v.data), v.n, v.h, v.w, v.c, v.ldc};
}

}  // namespace scd
