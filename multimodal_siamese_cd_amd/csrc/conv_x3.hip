// Implicit-GEMM convolution on gfx950 bf16 MFMA with exact three-way operand splitting ("x3").
//
// Every fp32 operand x is split into three bf16 terms, each rounded to nearest:
//   h = bf16(x), m = bf16(x - h), l = bf16(x - h - m).
// The subtractions are exact in fp32, so h + m + l reproduces x to within 2^-27 |x|.
//
// A product of two split operands is accumulated from the six terms whose magnitudes reach fp32's
// precision: hh + hm + mh + mm + hl + lh.  The dropped terms ml, lm, ll are at most ~2^-26 relative.
// Each bf16 x bf16 product is exact in the fp32 accumulator.  The result is therefore an fp32 GEMM with
// a rounding error of the same order as the fp32-MFMA kernel (conv_f32.hip); it differs only in
// summation order.
//
// Cost: 6 x v_mfma_f32_32x32x16_bf16 (32 cycles each) per 16-deep k step of a 32x32 tile, against
// 8 x v_mfma_f32_32x32x2_f32 (64 cycles each), i.e. 2.67x less matrix-core time per FLOP.
//
// Same GEMM view as igemm_f32: out[m, o] = bias + sum_k A[m, k] * Wpk[o, k], where A is gathered on the
// fly from an NHWC source and k = (tap, c).  This kernel requires c % 16 == 0, so a 16-deep k step never
// straddles two taps.
//
// LDS image: per stage and per operand, three planes (h, m, l) of [row][16 bf16] with 32-byte rows.  The
// 16-byte half of a row is XOR-swizzled with row bit 3, which makes the ds_read_b128 operand reads
// conflict-free; see the bank analysis in DESIGN.md.
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

template <int WAVES_M, int WAVES_N, int TM, int TN>
__global__ __launch_bounds__(64 * WAVES_M *WAVES_N) void igemm_x3(IgemmArgs a) {
    constexpr int BK = 16;
    constexpr int NT = 64 * WAVES_M * WAVES_N;
    constexpr int BM = WAVES_M * TM * 32;
    constexpr int BN = WAVES_N * TN * 32;
    constexpr int ROWS = BM + BN;
    constexpr int KC = BK / 4;            // 4-float chunks per row and stage
    constexpr int A_CH = BM * KC;
    constexpr int B_CH = BN * KC;
    constexpr int A_PER = (A_CH + NT - 1) / NT;
    constexpr int B_PER = (B_CH + NT - 1) / NT;
    constexpr int PLANE = ROWS * 32;      // bytes of one plane: ROWS x 16 bf16
    constexpr int STAGE = 3 * PLANE;
    __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wm = wid % WAVES_M;
    const int wn = wid / WAVES_M;
    int mt, nt;
    if (a.remap) {
        const uint32_t L = xcd_swizzle(blockIdx.x, uint32_t(a.grid_m * a.grid_n));
        mt = int(L / uint32_t(a.grid_n));
        nt = int(L - uint32_t(mt) * uint32_t(a.grid_n));
    } else {
        mt = int(blockIdx.x % uint32_t(a.grid_m));
        nt = int(blockIdx.x / uint32_t(a.grid_m));
    }
    const int m0 = mt * BM;
    const int n0 = nt * BN;

    // byte offset of (row, 4-float chunk col) inside a plane: 32-byte rows, 16-byte half swizzled by row bit 3
    auto soff = [](int row, int col) { return row * 32 + ((((col >> 1) ^ (row >> 3)) & 1) << 4) + ((col & 1) << 3); };

    const float *a_base[A_PER];
    int a_sy[A_PER], a_sx[A_PER], a_off[A_PER];
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
        const int ch = tid + i * NT;
        const int row = ch / KC, col = ch % KC;
        const int m = m0 + row;
        const bool ok = (ch < A_CH) && (m < a.M);
        const uint32_t mm = ok ? uint32_t(m) : 0u;
        const uint32_t img = fdiv(mm, a.div_hw);
        const uint32_t r = mm - img * uint32_t(a.ho * a.wo);
        const uint32_t oy = fdiv(r, a.div_w);
        const uint32_t ox = r - oy * uint32_t(a.wo);
        a_sy[i] = ok ? int(oy) * a.stride : -(1 << 20);
        a_sx[i] = int(ox) * a.stride;
        a_base[i] = a.src + (size_t(int(img) * a.hs + a_sy[i] * ok) * a.ws + a_sx[i]) * a.ldc_s + col * 4;
        a_off[i] = soff(row, col);
    }
    int b_row[B_PER], b_off[B_PER];
    bool b_ok[B_PER], b_in[B_PER];
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
        const int ch = tid + i * NT;
        const int row = ch / KC, col = ch % KC;
        b_in[i] = ch < B_CH;
        b_ok[i] = b_in[i] && (n0 + row < a.n_out);
        b_row[i] = (n0 + row) * a.K + col * 4;
        b_off[i] = soff(BM + row, col);
    }

    f32x4 ra[A_PER], rb[B_PER];
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};

    auto load_stage = [&](int t, int c0) {
        const int dyt = tap_at(a.tdy, t), dxt = tap_at(a.tdx, t);
        const long toff = long(dyt * a.ws + dxt) * a.ldc_s + c0;
#pragma unroll
        for (int i = 0; i < A_PER; ++i) {
            const bool v = unsigned(a_sy[i] + dyt) < unsigned(a.hs) && unsigned(a_sx[i] + dxt) < unsigned(a.ws);
            ra[i] = v ? gload4(a_base[i] + toff) : zero4;
        }
        const int k0 = t * a.c + c0;
#pragma unroll
        for (int i = 0; i < B_PER; ++i) rb[i] = b_ok[i] ? gload4(a.w + size_t(b_row[i]) + k0) : zero4;
    };
    auto store_stage = [&](int buf) {
        unsigned char *S = smem + buf * STAGE;
#pragma unroll
        for (int i = 0; i < A_PER; ++i)
            if (tid + i * NT < A_CH) {
                u32x2 h, m, l;
                split3(ra[i], h, m, l);
                *reinterpret_cast<u32x2 *>(S + a_off[i]) = h;
                *reinterpret_cast<u32x2 *>(S + PLANE + a_off[i]) = m;
                *reinterpret_cast<u32x2 *>(S + 2 * PLANE + a_off[i]) = l;
            }
#pragma unroll
        for (int i = 0; i < B_PER; ++i)
            if (b_in[i]) {
                u32x2 h, m, l;
                split3(rb[i], h, m, l);
                *reinterpret_cast<u32x2 *>(S + b_off[i]) = h;
                *reinterpret_cast<u32x2 *>(S + PLANE + b_off[i]) = m;
                *reinterpret_cast<u32x2 *>(S + 2 * PLANE + b_off[i]) = l;
            }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // operand reads: lane (r = lane&31, h = lane>>5) takes row r, k = 8h..8h+7 -> 16-byte half h of the row
    const int h = lane >> 5;
    int a_rd[TM], b_rd[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int row = wm * TM * 32 + i * 32 + (lane & 31);
        a_rd[i] = row * 32 + (((h ^ (row >> 3)) & 1) << 4);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int row = BM + wn * TN * 32 + j * 32 + (lane & 31);
        b_rd[j] = row * 32 + (((h ^ (row >> 3)) & 1) << 4);
    }

    const int csteps = a.c / BK;
    const int nsteps = a.ntaps * csteps;
    int t = 0, cs = 0;
    load_stage(0, 0);
    store_stage(0);
    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
        const bool more = s + 1 < nsteps;
        if (more) {
            if (++cs == csteps) {
                cs = 0;
                ++t;
            }
            load_stage(t, cs * BK);
        }
        const unsigned char *S = smem + (s & 1) * STAGE;
        bf16x8 av[3][TM], bv[3][TN];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
                av[p][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4 *>(S + p * PLANE + a_rd[i]));
#pragma unroll
            for (int j = 0; j < TN; ++j)
                bv[p][j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4 *>(S + p * PLANE + b_rd[j]));
        }
        // small terms first: mm, hl, lh, hm, mh, hh
        constexpr int PA[6] = {1, 0, 2, 0, 1, 0};
        constexpr int PB[6] = {1, 2, 0, 1, 0, 0};
#pragma unroll
        for (int q = 0; q < 6; ++q)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[PA[q]][i], bv[PB[q]][j], acc[i][j], 0, 0, 0);
        if (more) store_stage((s + 1) & 1);
        __syncthreads();
    }

#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * TN * 32 + j * 32 + (lane & 31);
        if (n >= a.n_out) continue;
        if (a.store_mode == 0) {
            const float bias = a.bias ? a.bias[n] : 0.f;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    if (m < a.M) gstore1(a.dst + size_t(m) * a.ldc_d + n, acc[i][j][r] + bias);
                }
        } else {
            const int ij = n / a.cout, oc = n - ij * a.cout;
            const int di = ij >> 1, dj = ij & 1;
            const float bias = a.bias ? a.bias[oc] : 0.f;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    if (m < a.M) {
                        const uint32_t img = fdiv(uint32_t(m), a.div_hw);
                        const uint32_t rr = uint32_t(m) - img * uint32_t(a.ho * a.wo);
                        const uint32_t oy = fdiv(rr, a.div_w);
                        const uint32_t ox = rr - oy * uint32_t(a.wo);
                        const size_t pix = size_t(int(img) * a.dst_h + 2 * int(oy) + di) * a.dst_w + 2 * int(ox) + dj;
                        gstore1(a.dst + pix * a.ldc_d + oc, acc[i][j][r] + bias);
                    }
                }
        }
    }
}

template <int WM, int WN, int TM, int TN>
static void launch_x3(const IgemmArgs &a, hipStream_t s) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    IgemmArgs b = a;
    b.grid_m = (a.M + BM - 1) / BM;
    b.grid_n = (a.n_out + BN - 1) / BN;
    b.remap = xcd_remap_enabled();
    hipLaunchKernelGGL((igemm_x3<WM, WN, TM, TN>), dim3(b.grid_m * b.grid_n), dim3(64 * WM * WN), 0, s, b);
}

bool launch_igemm_x3(const IgemmArgs &a, hipStream_t s) {
    if (a.c % 16) return false;
    if (a.n_out >= 128)
        launch_x3<2, 2, 2, 2>(a, s);  // 128 x 128
    else if (a.n_out >= 64)
        launch_x3<4, 1, 2, 2>(a, s);  // 256 x 64
    else
        launch_x3<4, 1, 2, 1>(a, s);  // 256 x 32
    return true;
}

}  // namespace scd
