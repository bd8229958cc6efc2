// Microbenchmark: how much independent f32 VALU work hides beside fp32 MFMAs on gfx950.
// One persistent workgroup of 4 waves per CU; each wave runs ITERS rounds of NM MFMAs on
// independent accumulators with GAP scalar v_fma_f32 (independent chains) after each MFMA.
// Prints achieved MFMA TFLOP/s and cycles per MFMA for each (shape, GAP).
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_gap.hip -o /tmp/mfma_gap && /tmp/mfma_gap
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int GAP>
__device__ __forceinline__ void fillers(float (&f)[8], float b) {
#pragma unroll
    for (int i = 0; i < GAP; ++i) asm volatile("v_fma_f32 %0, %1, %1, %0" : "+v"(f[i & 7]) : "v"(b));
}

// 16x16x4: NM = 36 MFMAs per round (the F(4x4,3x3) k-step)
template <int GAP>
__global__ __launch_bounds__(256, 1) void k16(int iters, float* out) {
    f32x4 acc[36];
#pragma unroll
    for (int i = 0; i < 36; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float a = threadIdx.x * 1e-3f, b = 1.0001f;
    float f[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = a + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 36; ++i) {
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            fillers<GAP>(f, b);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 36; ++i) s += acc[i][0] + acc[i][3];
#pragma unroll
    for (int i = 0; i < 8; ++i) s += f[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

// 32x32x2: NM = 16 MFMAs per round (the F(2x2,3x3) k-step)
template <int GAP>
__global__ __launch_bounds__(256, 1) void k32(int iters, float* out) {
    f32x16 acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = f32x16{};
    float a = threadIdx.x * 1e-3f, b = 1.0001f;
    float f[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = a + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            fillers<GAP>(f, b);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][15];
#pragma unroll
    for (int i = 0; i < 8; ++i) s += f[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <class K>
static void run(const char* name, K kern, int nm, int gap, double flops_per_mfma, float* out, int cus) {
    const int iters = 2000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    kern<<<cus, 256>>>(10, out);
    hipEventRecord(e0);
    kern<<<cus, 256>>>(iters, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double mfmas = (double)cus * 4 * iters * nm;  // per SIMD: 1 wave
    const double tf = mfmas * flops_per_mfma / (ms * 1e-3) / 1e12;
    // cycles per MFMA at 2.4 GHz nominal (the chip may run slower under load)
    const double cyc = (ms * 1e-3) * 2.4e9 / ((double)iters * nm);
    printf("{\"shape\": \"%s\", \"gap_fma\": %d, \"tflops\": %.1f, \"cycles_per_mfma_at_2.4GHz\": %.1f}\n",
           name, gap, tf, cyc);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    hipMalloc(&out, (size_t)cus * 256 * 4);
    run("16x16x4", k16<0>, 36, 0, 2048, out, cus);
    run("16x16x4", k16<2>, 36, 2, 2048, out, cus);
    run("16x16x4", k16<4>, 36, 4, 2048, out, cus);
    run("16x16x4", k16<5>, 36, 5, 2048, out, cus);
    run("16x16x4", k16<6>, 36, 6, 2048, out, cus);
    run("16x16x4", k16<8>, 36, 8, 2048, out, cus);
    run("16x16x4", k16<12>, 36, 12, 2048, out, cus);
    run("32x32x2", k32<0>, 16, 0, 4096, out, cus);
    run("32x32x2", k32<4>, 16, 4, 4096, out, cus);
    run("32x32x2", k32<8>, 16, 8, 4096, out, cus);
    run("32x32x2", k32<12>, 16, 12, 4096, out, cus);
    run("32x32x2", k32<16>, 16, 16, 4096, out, cus);
    run("32x32x2", k32<24>, 16, 24, 4096, out, cus);
    hipFree(out);
    return 0;
}
