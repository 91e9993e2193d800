// Microbenchmark: does the x3 conv inner loop run faster (wall time, random data) on
// v_mfma_f32_16x16x32_bf16 than on v_mfma_f32_32x32x16_bf16 at the same output tile per wave?
// (MI355X_MICROARCH.md 'DVFS give-back' item 7; cdna_hip_programming.md rule 28.)
//
// Both variants: 4 waves/block, 3 blocks/CU, wave tile 64 x 64, per 32-deep k step 12 ds_read_b128 of A
// (3 planes), 12 x 1 KB loads of B fragments from an L2-resident buffer (3 planes), 6 split products.
//   S32: 2 substeps x 6 products x (2 x 2) 32x32x16 MFMAs = 48 MFMAs
//   S16: 6 products x (4 x 4) 16x16x32 MFMAs            = 96 MFMAs   (same FLOPs)
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/mfma_shape_bench tools/mfma_shape_bench.hip && tools/mfma_shape_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

constexpr int NBFRAG = 256;  // B buffer: 256 KB of fragments (L2-resident)
constexpr int LDS_FRAGS = 24;  // A image in LDS: 24 x 1 KB per plane

__device__ __forceinline__ u32x4 bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

template <bool S16>
__global__ __launch_bounds__(256, 3) void kern(const uint16_t *__restrict__ bsrc, const uint16_t *__restrict__ asrc,
                                                float *out, int nsteps) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[3 * LDS_FRAGS * 1024];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (int e = tid; e < 3 * LDS_FRAGS * 64; e += 256)
        *reinterpret_cast<u32x4 *>(smem + e * 16) = *reinterpret_cast<const u32x4 *>(asrc + (size_t(e) * 8) % (1 << 20));
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(bsrc), 0, NBFRAG * 1024, 0x00020000);
    constexpr int PL = LDS_FRAGS * 1024;
    constexpr int QA[6] = {0, 0, 1, 1, 0, 2};
    constexpr int QB[6] = {0, 1, 0, 1, 2, 0};
    uint32_t boff = uint32_t((blockIdx.x * 5 + wid * 3) % NBFRAG);
    if constexpr (S16) {
        f32x4 acc[4][4];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int s = 0; s < nsteps; ++s) {
            const int sh = (s * 7) % (LDS_FRAGS - 4);
            u32x4 bq[3][4];
#pragma unroll
            for (int p = 0; p < 3; ++p)
#pragma unroll
                for (int j = 0; j < 4; ++j) bq[p][j] = bload(rb, ((boff + p * 4 + j) % NBFRAG) * 1024u + lane * 16u);
            boff += 12;
            bf16x8 av[3][4];
#pragma unroll
            for (int p = 0; p < 3; ++p)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    av[p][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4 *>(smem + p * PL + (sh + i) * 1024 + lane * 16));
#pragma unroll
            for (int q = 0; q < 6; ++q)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[QA[q]][i], __builtin_bit_cast(bf16x8, bq[QB[q]][j]),
                                                                            acc[i][j], 0, 0, 0);
        }
        float t = 0.f;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j)
                for (int r = 0; r < 4; ++r) t += acc[i][j][r];
        out[blockIdx.x * 256 + tid] = t;
    } else {
        f32x16 acc[2][2];
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 2; ++j)
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
        for (int s = 0; s < 2 * nsteps; ++s) {
            const int sh = (s * 7) % (LDS_FRAGS - 2);
            u32x4 bq[3][2];
#pragma unroll
            for (int p = 0; p < 3; ++p)
#pragma unroll
                for (int j = 0; j < 2; ++j) bq[p][j] = bload(rb, ((boff + p * 2 + j) % NBFRAG) * 1024u + lane * 16u);
            boff += 6;
            bf16x8 av[3][2];
#pragma unroll
            for (int p = 0; p < 3; ++p)
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    av[p][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4 *>(smem + p * PL + (sh + i) * 1024 + lane * 16));
#pragma unroll
            for (int q = 0; q < 6; ++q)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[QA[q]][i], __builtin_bit_cast(bf16x8, bq[QB[q]][j]),
                                                                            acc[i][j], 0, 0, 0);
        }
        float t = 0.f;
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 2; ++j)
                for (int r = 0; r < 16; ++r) t += acc[i][j][r];
        out[blockIdx.x * 256 + tid] = t;
    }
}

static uint16_t bf16_bits(float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    return uint16_t((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}

int main(int argc, char **argv) {
    const int nsteps = argc > 1 ? atoi(argv[1]) : 2000;
    const int grid = 256 * 3 * 4;
    std::vector<uint16_t> hb(NBFRAG * 512), ha(1 << 20);
    uint64_t st = 0x9e3779b97f4a7c15ull;
    auto rnd = [&]() {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;
        return float(int64_t(st >> 11) % 2000001 - 1000000) * 1e-6f;
    };
    // random h/m/l-like magnitudes: plane index by position is irrelevant for timing, all operands random
    for (auto &v : hb) v = bf16_bits(rnd());
    for (auto &v : ha) v = bf16_bits(rnd());
    uint16_t *db, *da;
    float *dout;
    CHECK(hipMalloc(&db, hb.size() * 2));
    CHECK(hipMalloc(&da, ha.size() * 2));
    CHECK(hipMalloc(&dout, size_t(grid) * 256 * 4));
    CHECK(hipMemcpy(db, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(da, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const double flops = double(grid) * 4 * nsteps * (6.0 * 16 * 2 * 16 * 16 * 32);
    // warm the clock for ~2 s
    for (int r = 0; r < 150; ++r) {
        hipLaunchKernelGGL(kern<true>, dim3(grid), dim3(256), 0, 0, db, da, dout, nsteps);
        hipLaunchKernelGGL(kern<false>, dim3(grid), dim3(256), 0, 0, db, da, dout, nsteps);
    }
    CHECK(hipDeviceSynchronize());
    for (int round = 0; round < 5; ++round) {
        for (int v = 0; v < 2; ++v) {
            CHECK(hipEventRecord(e0));
            for (int r = 0; r < 5; ++r) {
                if (v)
                    hipLaunchKernelGGL(kern<true>, dim3(grid), dim3(256), 0, 0, db, da, dout, nsteps);
                else
                    hipLaunchKernelGGL(kern<false>, dim3(grid), dim3(256), 0, 0, db, da, dout, nsteps);
            }
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            printf("round %d %s: %.3f ms/launch  %.1f TFLOP/s (bf16 MFMA)\n", round, v ? "16x16x32" : "32x32x16", ms / 5,
                   flops / (ms / 5 * 1e-3) / 1e12);
        }
    }
    return 0;
}
