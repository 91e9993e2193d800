// Internal helpers shared by the libscd translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <initializer_list>

#include "../../include/scd.h"

namespace scd {

void set_error(const char *fmt, ...);
void clear_error();

inline hipStream_t as_stream(scd_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline bool aligned8(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 7u) == 0; }

// Element type of a view (scd_nhwc_t.dtype).  A channel quad is 16 bytes (fp32) or 8 bytes (bf16).
inline bool is_bf16(const scd_nhwc_t &v) { return v.dtype == SCD_DT_BF16; }
inline int elem_bytes(const scd_nhwc_t &v) { return is_bf16(v) ? 2 : 4; }

// Validate an NHWC view used with channel-quad vector accesses.
inline int check_view(const scd_nhwc_t &v, const char *name, bool allow_null = false) {
    if (v.data == nullptr) {
        if (allow_null) return SCD_OK;
        set_error("%s: null data", name);
        return SCD_ERR_ARG;
    }
    if (v.dtype != SCD_DT_F32 && v.dtype != SCD_DT_BF16) {
        set_error("%s: unknown dtype %d", name, v.dtype);
        return SCD_ERR_ARG;
    }
    if (v.n <= 0 || v.h <= 0 || v.w <= 0 || v.c <= 0 || v.ldc < v.c) {
        set_error("%s: bad shape n=%d h=%d w=%d c=%d ldc=%d", name, v.n, v.h, v.w, v.c, v.ldc);
        return SCD_ERR_ARG;
    }
    if ((v.c & 3) || (v.ldc & 3) || !(is_bf16(v) ? aligned8(v.data) : aligned16(v.data))) {
        set_error("%s: c=%d / ldc=%d must be multiples of 4 and data %d-byte aligned", name, v.c, v.ldc,
                  is_bf16(v) ? 8 : 16);
        return SCD_ERR_ALIGN;
    }
    return SCD_OK;
}

// All given (non-null) views of one call share one element type; returns it, or -1 (error set) if they do not.
inline int common_dtype(const char *what, std::initializer_list<const scd_nhwc_t *> views) {
    int dt = -1;
    for (const scd_nhwc_t *v : views) {
        if (v == nullptr || v->data == nullptr) continue;
        if (dt < 0) {
            dt = v->dtype;
        } else if (v->dtype != dt) {
            set_error("%s: views of different element types (fp32 and bf16) in one call", what);
            return -1;
        }
    }
    return dt < 0 ? SCD_DT_F32 : dt;
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

// ------------------------------------------------------------------------------------------------
// Storage element types of the NHWC kernels: float, or bf16 (the bf16 configs' activations and gradients).
// ld4 / st4 move one channel quad (4 consecutive channels) between memory and fp32 registers: a bf16 load is
// exact (the bits are the top half of the float), a bf16 store rounds to nearest-even (v_cvt_pk_bf16_f32).  The
// kernels templated on the element type T compute in fp32 either way.
// ------------------------------------------------------------------------------------------------
struct bf16_t {
    uint16_t u;
};
typedef unsigned int scd_u32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 scd_bf16x2 __attribute__((ext_vector_type(2)));
typedef float scd_f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
    const scd_f32x2 v = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, scd_bf16x2));  // RNE
}
__device__ __forceinline__ bnf4 unpk_bf16x4(scd_u32x2 p) {
    return bnf4{__builtin_bit_cast(float, p[0] << 16), __builtin_bit_cast(float, p[0] & 0xffff0000u),
                __builtin_bit_cast(float, p[1] << 16), __builtin_bit_cast(float, p[1] & 0xffff0000u)};
}
__device__ __forceinline__ scd_u32x2 pk_bf16x4(bnf4 v) { return scd_u32x2{pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3])}; }
// v rounded to bf16 and back (the value a bf16 store keeps)
__device__ __forceinline__ bnf4 round_bf16x4(bnf4 v) { return unpk_bf16x4(pk_bf16x4(v)); }

__device__ __forceinline__ bnf4 ld4(const float *p) { return *reinterpret_cast<const bnf4 *>(p); }
__device__ __forceinline__ bnf4 ld4(const bf16_t *p) { return unpk_bf16x4(*reinterpret_cast<const scd_u32x2 *>(p)); }
__device__ __forceinline__ void st4(float *p, bnf4 v) { *reinterpret_cast<bnf4 *>(p) = v; }
__device__ __forceinline__ void st4(bf16_t *p, bnf4 v) { *reinterpret_cast<scd_u32x2 *>(p) = pk_bf16x4(v); }
__device__ __forceinline__ float ld1(const float *p) { return *p; }
__device__ __forceinline__ float ld1(const bf16_t *p) { return __builtin_bit_cast(float, uint32_t(p->u) << 16); }
__device__ __forceinline__ void st1(float *p, float v) { *p = v; }
__device__ __forceinline__ void st1(bf16_t *p, float v) { p->u = uint16_t(pk_bf16(v, 0.f) & 0xffffu); }
// the storage value of v (identity for fp32)
__device__ __forceinline__ bnf4 stored4(const float *, bnf4 v) { return v; }
__device__ __forceinline__ bnf4 stored4(const bf16_t *, bnf4 v) { return round_bf16x4(v); }

template <class T>
inline T *view_ptr(const scd_nhwc_t &v) { return static_cast<T *>(v.data); }

// Run `body` with T = the element type of dtype `dt` (float or bf16_t).
#define SCD_WITH_T(dt, T, ...)          \
    do {                                \
        if ((dt) == SCD_DT_BF16) {      \
            using T = ::scd::bf16_t;    \
            __VA_ARGS__;                \
        } else {                        \
            using T = float;            \
            __VA_ARGS__;                \
        }                               \
    } while (0)

// Device-side NHWC element pointer helpers.
struct View {
    float *p;
    int n, h, w, c, ldc;
};

inline View make_view(const scd_nhwc_t &v) {
    return View{static_cast<float *>(v.data), v.n, v.h, v.w, v.c, v.ldc};
}

}  // namespace scd
