// Microbenchmark: the MFMA rate the chip SUSTAINS (its held clock under load) per MFMA shape,
// on random operands, every CU busy for about two seconds.  The Winograd tile runs fp32
// `v_mfma_f32_32x32x2_f32` and holds 2.05-2.35 GHz; MI355X_MICROARCH.md (7) reports that for
// bf16 the 16x16 shape holds a higher clock than the 32x32 one at equal cycles per FLOP.  This
// measures whether the same holds for fp32 (16x16x4 vs 32x32x2) before any tile is rebuilt on it.
//
// One workgroup of 4 waves per CU (one wave per SIMD), 192 accumulator registers per lane in
// independent accumulators, operands from 8 random register sets rotated per MFMA.  Wave 0 of
// every workgroup stamps s_memtime / s_memrealtime around its loop: the in-kernel clock is
// d(memtime) / d(memrealtime) x 100 MHz (median over workgroups); stamps go to their own buffer.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_power.hip -o /tmp/mfma_power && /tmp/mfma_power
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned uvec4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned hash(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
__device__ __forceinline__ float rnd(unsigned s) {  // uniform in [-1, 1)
    return __uint_as_float(0x3f800000u | (hash(s) >> 9)) * 2.f - 3.f;
}

// SHAPE 0: f32 32x32x2 (12 accumulators of 16), 1: f32 16x16x4 (48 of 4),
//       2: bf16 32x32x16 (12 of 16),          3: bf16 16x16x32 (48 of 4)
// (iters: a multiple of 8; the operand rotation is unrolled so every index is static)
template <int SHAPE>
__global__ __launch_bounds__(256, 1) void kpow(int iters, float* out, unsigned long long* stamps) {
    const unsigned seed = (blockIdx.x * 256 + threadIdx.x) * 16;
    float fa[8], fb[8];
    uvec4 ba[8], bb[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        fa[i] = rnd(seed + i);
        fb[i] = rnd(seed + 8 + i);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            ba[i][q] = (hash(seed * 7 + i * 4 + q) & 0x3fff3fffu) | 0x3c003c00u;  // bf16 pairs in [1, 2)-ish
            bb[i][q] = (hash(seed * 13 + i * 4 + q) & 0x3fff3fffu) | 0x3c003c00u;
        }
    }
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    float sink = 0.f;
    if constexpr (SHAPE == 0 || SHAPE == 2) {
        f32x16 acc[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) acc[i] = f32x16{};
        for (int it8 = 0; it8 < iters; it8 += 8) {
#pragma unroll
            for (int it = 0; it < 8; ++it)
#pragma unroll
            for (int i = 0; i < 12; ++i) {
                if constexpr (SHAPE == 0)
                    acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[(i + it) & 7], fb[(i * 3 + it) & 7], acc[i], 0, 0, 0);
                else
                    acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, ba[(i + it) & 7]),
                                                                     __builtin_bit_cast(bf16x8, bb[(i * 3 + it) & 7]),
                                                                     acc[i], 0, 0, 0);
            }
        }
#pragma unroll
        for (int i = 0; i < 12; ++i)
#pragma unroll
            for (int q = 0; q < 16; ++q) sink += acc[i][q];
    } else {
        f32x4 acc[48];
#pragma unroll
        for (int i = 0; i < 48; ++i) acc[i] = f32x4{};
        for (int it8 = 0; it8 < iters; it8 += 8) {
#pragma unroll
            for (int it = 0; it < 8; ++it)
#pragma unroll
            for (int i = 0; i < 48; ++i) {
                if constexpr (SHAPE == 1)
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[(i + it) & 7], fb[(i * 3 + it) & 7], acc[i], 0, 0, 0);
                else
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ba[(i + it) & 7]),
                                                                     __builtin_bit_cast(bf16x8, bb[(i * 3 + it) & 7]),
                                                                     acc[i], 0, 0, 0);
            }
        }
#pragma unroll
        for (int i = 0; i < 48; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q) sink += acc[i][q];
    }
    if (threadIdx.x == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
    out[blockIdx.x * 256 + threadIdx.x] = sink;
}

template <int SHAPE>
void run(const char* name, double macs_per_mfma, int mfma_per_iter, int iters, float* out,
         unsigned long long* stamps, int nblk) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    kpow<SHAPE><<<nblk, 256>>>(iters / 64 * 8, out, stamps);  // warm (short)
    hipDeviceSynchronize();
    // about two seconds of back-to-back launches so the held clock settles, then timed launches
    for (int w = 0; w < 2; ++w) {
        kpow<SHAPE><<<nblk, 256>>>(iters, out, stamps);
    }
    const int reps = 3;
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) kpow<SHAPE><<<nblk, 256>>>(iters, out, stamps);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> st(2 * nblk);
    hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> ghz;
    for (int b = 0; b < nblk; ++b)
        if (st[2 * b + 1]) ghz.push_back(double(st[2 * b]) / double(st[2 * b + 1]) * 0.1);
    std::sort(ghz.begin(), ghz.end());
    const double flops = 2.0 * macs_per_mfma * mfma_per_iter * double(iters) * 4.0 * nblk * reps;
    const double tf = flops / (ms * 1e-3) / 1e12;
    const double cyc_per_mfma = (ms * 1e-3 / reps) * ghz[ghz.size() / 2] * 1e9 / (double(iters) * mfma_per_iter);
    printf("{\"shape\": \"%s\", \"tflops\": %.1f, \"ms_per_launch\": %.1f, \"clock_ghz_median\": %.3f, "
           "\"clock_ghz_min\": %.3f, \"clock_ghz_max\": %.3f, \"cycles_per_mfma_at_held_clock\": %.1f}\n",
           name, tf, ms / reps, ghz[ghz.size() / 2], ghz.front(), ghz.back(), cyc_per_mfma);
    fflush(stdout);
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const int nblk = ncu;
    float* out;
    unsigned long long* stamps;
    hipMalloc(&out, nblk * 256 * 4);
    hipMalloc(&stamps, nblk * 16);
    // iteration counts sized for ~0.7 s per launch at the nominal rate
    run<0>("f32_32x32x2", 32 * 32 * 2, 12, 700000, out, stamps, nblk);
    run<1>("f32_16x16x4", 16 * 16 * 4, 48, 350000, out, stamps, nblk);
    run<2>("bf16_32x32x16", 32 * 32 * 16, 12, 1400000, out, stamps, nblk);
    run<3>("bf16_16x16x32", 16 * 16 * 32, 48, 700000, out, stamps, nblk);
    run<0>("f32_32x32x2_again", 32 * 32 * 2, 12, 700000, out, stamps, nblk);
    hipFree(out);
    hipFree(stamps);
    return 0;
}
