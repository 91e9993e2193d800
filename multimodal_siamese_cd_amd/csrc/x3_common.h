// Shared pieces of the split-bf16 ("x3") conv kernels (conv_x3.hip, conv_halo16.hip): operand types, the
// exact three-way bf16 split and raw buffer loads.
#pragma once

#include <type_traits>

#include "conv_common.h"

namespace scd {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
    const f32x2 v = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));  // v_cvt_pk_bf16_f32 (RNE)
}
__device__ __forceinline__ float bf16_lo(uint32_t p) { return __builtin_bit_cast(float, p << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t p) { return __builtin_bit_cast(float, p & 0xffff0000u); }

// Split four consecutive fp32 values into their h, m, l bf16 terms (4 bf16 = 8 bytes each).
__device__ __forceinline__ void split3(const f32x4 v, u32x2 &h, u32x2 &m, u32x2 &l) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const float x0 = v[2 * p], x1 = v[2 * p + 1];
        const uint32_t ph = cvt_pk_bf16(x0, x1);
        const float r0 = x0 - bf16_lo(ph), r1 = x1 - bf16_hi(ph);
        const uint32_t pm = cvt_pk_bf16(r0, r1);
        const float s0 = r0 - bf16_lo(pm), s1 = r1 - bf16_hi(pm);
        h[p] = ph;
        m[p] = pm;
        l[p] = cvt_pk_bf16(s0, s1);
    }
}

// ------------------------------------------------------------------------------------------------
// Two-term fp16 split ("h2", SCD_MATH_H2).  A power-of-two scale s brings an operand's magnitude bound U
// to U * s < 2^15 (< fp16 max 65504); x * s = h + m with h = fp16(x * s) and m = fp16(x * s - h), both rounded
// to nearest.  The subtraction is exact, h and m carry 11 significant bits each, so h + m represents x * s to
// 2^-22 relative while m stays in the fp16 normal range (x * s >= 2^-3), with a floor of 2^-25 absolute
// below.  A product keeps hh + hm + mh (the dropped mm is <= 2^-24 relative): three MFMAs against x3's six.
//
// Activations and gradients can span far more than the 2^17 binades above that floor (a few large gradient
// values over a bulk 2^20 below them), so their low term is kept pre-scaled: m' = fp16((x * s - h) * 2^11),
// normal down to x * s = 2^-14, floor 2^-36 absolute.  The product against the other operand's h then takes
// that operand's h * 2^-11 (formed in registers, exact while it is an fp16 normal): one MFMA accumulator.
// ------------------------------------------------------------------------------------------------
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t cvt_pk_f16(float a, float b) {
    const f32x2 v = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2));  // RNE
}
__device__ __forceinline__ float f16_lo(uint32_t p) { return float(__builtin_bit_cast(f16x2, p)[0]); }
__device__ __forceinline__ float f16_hi(uint32_t p) { return float(__builtin_bit_cast(f16x2, p)[1]); }

// Split four consecutive (already scaled) fp32 values into their h, m fp16 terms (4 fp16 = 8 bytes each).
__device__ __forceinline__ void split2h(const f32x4 v, u32x2 &h, u32x2 &m) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const float x0 = v[2 * p], x1 = v[2 * p + 1];
        const uint32_t ph = cvt_pk_f16(x0, x1);
        h[p] = ph;
        m[p] = cvt_pk_f16(x0 - f16_lo(ph), x1 - f16_hi(ph));
    }
}

// The same with the low term pre-scaled by 2^11 (activation / gradient operands, see above).
__device__ __forceinline__ void split2h_pre(const f32x4 v, u32x2 &h, u32x2 &m) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const float x0 = v[2 * p], x1 = v[2 * p + 1];
        const uint32_t ph = cvt_pk_f16(x0, x1);
        h[p] = ph;
        m[p] = cvt_pk_f16((x0 - f16_lo(ph)) * 2048.f, (x1 - f16_hi(ph)) * 2048.f);
    }
}
// h * 2^-11 of an fp16 fragment (v_pk_mul_f16): the partner of a pre-scaled low term.
__device__ __forceinline__ u32x4 f16_down11(const u32x4 v) {
    const f16x8 r = __builtin_bit_cast(f16x8, v) * (_Float16)0x1p-11f;
    return __builtin_bit_cast(u32x4, r);
}

// Power-of-two scale for a magnitude bound ub: s = 2^k with ub * s < 2^15, k clamped to [-126, 126] so s and 1/s
// are normal floats (0 -> 1; a non-finite bound gives a finite scale and the garbage it describes).
__device__ __forceinline__ void h2_scale(float ub, float &s, float &inv) {
    const uint32_t b = __builtin_bit_cast(uint32_t, ub) & 0x7fffffffu;
    int k = b ? 14 - (int(b >> 23) - 127) : 0;
    k = k < -126 ? -126 : (k > 126 ? 126 : k);
    s = __builtin_bit_cast(float, uint32_t(127 + k) << 23);
    inv = __builtin_bit_cast(float, uint32_t(127 - k) << 23);
}

__device__ __forceinline__ f32x4 mfma16_f16(const u32x4 a, const u32x4 b, const f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

// Raw buffer loads: 32-bit byte offsets with the hardware range check, so an out-of-range offset
// (kOOB) returns zeros with no branch, no exec-mask juggling and no zero-fill moves.
constexpr uint32_t kOOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, int(bytes), 0x00020000);
}
__device__ __forceinline__ f32x4 bload4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ u32x4 bload4u(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
// 8 bytes: one bf16 channel quad (SB: bf16 activation storage)
__device__ __forceinline__ u32x2 bload2u(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
__device__ __forceinline__ void gstore2u(void *p, u32x2 v) { *(__attribute__((address_space(1))) u32x2 *)(p) = v; }

// Kernel storage of the activation operands and outputs: fp32 (SB false) or bf16 (SB true: ABI 6 bf16 views, the bf16
// configs).  A bf16 channel quad is staged as its bits (it is already the bf16 operand), or unpacked for an input
// transform and rounded back; outputs are rounded once (RNE) and the fused statistics are taken of the stored values.
template <bool SB>
using StageT = typename std::conditional<SB, u32x2, f32x4>::type;
template <bool SB>
__device__ __forceinline__ StageT<SB> bload_q(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    if constexpr (SB)
        return bload2u(r, off);
    else
        return bload4(r, off);
}
// bf16 bits of a staged quad (SB: as loaded; fp32: rounded to nearest)
template <bool SB>
__device__ __forceinline__ u32x2 stage_bits(const StageT<SB> &v) {
    if constexpr (SB)
        return v;
    else
        return u32x2{cvt_pk_bf16(v[0], v[1]), cvt_pk_bf16(v[2], v[3])};
}
template <bool SB>
__device__ __forceinline__ f32x4 stage_f32(const StageT<SB> &v) {
    if constexpr (SB)
        return unpk_bf16x4(v);
    else
        return v;
}
// Store one output channel quad at element offset e of `dst` (fp32 or bf16); returns the stored value.
template <bool SB>
__device__ __forceinline__ f32x4 store_q(float *dst, size_t e, f32x4 v) {
    if constexpr (SB) {
        const u32x2 pk = pk_bf16x4(v);
        gstore2u(reinterpret_cast<bf16_t *>(dst) + e, pk);
        return unpk_bf16x4(pk);
    } else {
        *(__attribute__((address_space(1))) f32x4 *)(dst + e) = v;
        return v;
    }
}
// store_q / load_q at a byte address (the epilogues' incrementally formed row addresses)
template <bool SB>
__device__ __forceinline__ f32x4 store_qb(unsigned char *p, f32x4 v) {
    if constexpr (SB) {
        const u32x2 pk = pk_bf16x4(v);
        gstore2u(p, pk);
        return unpk_bf16x4(pk);
    } else {
        *(__attribute__((address_space(1))) f32x4 *)(p) = v;
        return v;
    }
}
template <bool SB>
__device__ __forceinline__ f32x4 load_qb(const unsigned char *p) {
    if constexpr (SB)
        return unpk_bf16x4(*(const __attribute__((address_space(1))) u32x2 *)(p));
    else
        return *(const __attribute__((address_space(1))) f32x4 *)(p);
}
template <bool SB>
__device__ __forceinline__ f32x4 load_q(const float *src, size_t e) {
    if constexpr (SB)
        return ld4(reinterpret_cast<const bf16_t *>(src) + e);
    else
        return *(const __attribute__((address_space(1))) f32x4 *)(src + e);
}


typedef short s16x4 __attribute__((ext_vector_type(4)));


__device__ __forceinline__ s16x4 lds_tr16(const unsigned char *p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4 *)(reinterpret_cast<const __attribute__((address_space(3))) unsigned char *>(
            reinterpret_cast<uintptr_t>(p))));
}

constexpr int tr_stride(int w) { return (2 * w) % 128 == 0 ? 2 * w + 64 : 2 * w; }

// ds_read_b64_tr_b16 with an immediate offset (hipcc does not fold offsets into the builtin, which then
// needs one address VGPR per distinct read).  Inline asm is invisible to the compiler's LDS counters: every
// use is preceded by lds_wait<N>() on the fragments it consumes.
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return uint32_t(uintptr_t((const __attribute__((address_space(3))) unsigned char *)(p)));
}
template <int OFF>
__device__ __forceinline__ void tr_read(s16x4 &dst, uint32_t vaddr) {
    static_assert(OFF >= 0 && OFF < 65536, "ds offset is 16 bits");
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(dst) : "v"(vaddr), "i"(OFF) : "memory");
}
template <int N>
__device__ __forceinline__ void lds_wait(bf16x8 &a, bf16x8 &b, bf16x8 &c) {
    asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(a), "+v"(b), "+v"(c) : "n"(N));
}
template <int N>
__device__ __forceinline__ void lds_wait(bf16x8 &a, bf16x8 &b) {
    asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N));
}
template <int N>
__device__ __forceinline__ void lds_wait(bf16x8 &a) {
    asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "n"(N));
}

__device__ __forceinline__ bf16x8 cat8(s16x4 lo, s16x4 hi) {
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

}  // namespace scd
