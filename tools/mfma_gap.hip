// Microbenchmark: how much independent f32 VALU work hides beside fp32 MFMAs on gfx950.
// One persistent workgroup of 4 waves per CU; each wave runs ITERS rounds of NM MFMAs on
// independent accumulators with GAP scalar v_fma_f32 (independent chains) after each MFMA.
// Prints achieved MFMA TFLOP/s and cycles per MFMA for each (shape, GAP).
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_gap.hip -o /tmp/mfma_gap && /tmp/mfma_gap
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// filler kinds: 0 v_fma_f32, 1 v_pk_add_f32, 2 v_mov_b32, 3 v_add_u32, 4 ds_read_b128,
// 5 ds_write_b64, 6 v_exp_f32, 7 v_cvt_pk_bf16_f32
template <int GAP, int KIND = 0>
__device__ __forceinline__ void fillers(float (&f)[8], float b) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef float f4 __attribute__((ext_vector_type(4)));
    __shared__ float lds[4096];
#pragma unroll
    for (int i = 0; i < GAP; ++i) {
        if constexpr (KIND == 0) asm volatile("v_fma_f32 %0, %1, %1, %0" : "+v"(f[i & 7]) : "v"(b));
        if constexpr (KIND == 1) {
            f2 x{f[i & 7], f[(i + 1) & 7]};
            asm volatile("v_pk_add_f32 %0, %0, %0" : "+v"(x));
            f[i & 7] = x[0];
        }
        if constexpr (KIND == 2) asm volatile("v_mov_b32 %0, %1" : "=v"(f[i & 7]) : "v"(b));
        if constexpr (KIND == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(f[i & 7]) : "v"(b));
        if constexpr (KIND == 4) {
            f4 x;
            asm volatile("ds_read_b128 %0, %1" : "=v"(x) : "v"((threadIdx.x & 63) * 16 + (i & 7) * 1024));
            asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
            f[i & 7] += 0.f * x[0];
        }
        if constexpr (KIND == 5) {
            f2 x{f[i & 7], b};
            asm volatile("ds_write_b64 %0, %1" : : "v"((threadIdx.x & 63) * 8 + (i & 7) * 512), "v"(x) : "memory");
        }
        if constexpr (KIND == 6) asm volatile("v_exp_f32 %0, %1" : "=v"(f[i & 7]) : "v"(b));
        if constexpr (KIND == 7)
            asm volatile("v_cvt_pk_bf16_f32 %0, %0, %1" : "+v"(f[i & 7]) : "v"(b));
    }
    if (b < -1e30f) lds[threadIdx.x] = f[0];
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
template <int GAP, int KIND = 0>
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
            fillers<GAP, KIND>(f, b);
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

// bursts: GAP fillers after every EVERY-th MFMA (the same total as GAP / EVERY per gap)
template <int GAP, int EVERY, int KIND = 0>
__global__ __launch_bounds__(256, 1) void k32b(int iters, float* out) {
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
            if (i % EVERY == EVERY - 1) fillers<GAP, KIND>(f, b);
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

// k-step models: F(4x4,3x3) = 36 x 16x16x4 MFMAs + NPK packed adds in NB bursts;
// F(2x2,3x3) = 16 x 32x32x2 MFMAs + 16 packed adds in one burst (the current tile)
template <int NPK, int NB>
__global__ __launch_bounds__(256, 1) void kf43(int iters, float* out) {
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
            if ((i + 1) % (36 / NB) == 0) fillers<NPK / NB, 1>(f, b);
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

// bf16 MFMA (v_mfma_f32_32x32x16_bf16, 16x the fp32 MFMA's MACs per cycle): 16 per round,
// GAP fillers after every EVERY-th — is VALU work beside bf16 MFMAs hidden, unlike fp32?
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
template <int GAP, int EVERY, int KIND>
__global__ __launch_bounds__(256, 1) void kbf(int iters, float* out) {
    f32x16 acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = f32x16{};
    float a = threadIdx.x * 1e-3f, b = 1.0001f;
    bf16x8 av, bv;
#pragma unroll
    for (int i = 0; i < 8; ++i) av[i] = (__bf16)(a + i), bv[i] = (__bf16)(b - i);
    float f[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = a + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc[i], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (i % EVERY == EVERY - 1) fillers<GAP, KIND>(f, b);
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
static void run(const char* name, K kern, int nm, int gap, double flops_per_mfma, float* out, int cus,
                const char* kind = "v_fma_f32") {
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
    printf("{\"shape\": \"%s\", \"filler\": \"%s\", \"per_gap\": %d, \"tflops\": %.1f, "
           "\"cycles_per_mfma_at_2.4GHz\": %.1f}\n", name, kind, gap, tf, cyc);
}


// Two waves per SIMD (512 threads) vs one (256): 16x16x4 f32 MFMAs on 32 independent
// accumulators (128 registers) with GAP fillers after every EVERY-th MFMA.  If one wave's
// VALU work co-executes with the other wave's MFMAs, the fillers' cost disappears at 2 waves.
template <int GAP, int EVERY, int KIND>
__global__ __launch_bounds__(512, 1) void k16w(int iters, float* out) {
    f32x4 acc[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float a = threadIdx.x * 1e-3f, b = 1.0001f;
    float f[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = a + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (i % EVERY == EVERY - 1) fillers<GAP, KIND>(f, b);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) s += acc[i][0] + acc[i][3];
#pragma unroll
    for (int i = 0; i < 8; ++i) s += f[i];
    out[blockIdx.x * 512 + threadIdx.x] = s;
}

template <class K>
static void run_w(const char* name, K kern, int threads, int nm, int gap, double flops_per_mfma, float* out,
                  int cus, const char* kind) {
    const int iters = 1000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    kern<<<cus, threads>>>(10, out);
    hipEventRecord(e0);
    kern<<<cus, threads>>>(iters, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double mfmas = (double)cus * (threads / 64) * iters * nm;
    const double tf = mfmas * flops_per_mfma / (ms * 1e-3) / 1e12;
    printf("{\"shape\": \"%s\", \"waves_per_simd\": %d, \"filler\": \"%s\", \"per_burst\": %d, \"tflops\": %.1f}\n",
           name, threads / 256, kind, gap, tf);
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
    const char* kinds[] = {"v_fma_f32", "v_pk_add_f32", "v_mov_b32", "v_add_u32", "ds_read_b128",
                           "ds_write_b64", "v_exp_f32", "v_cvt_pk_bf16_f32"};
    run("32x32x2", k32<4, 1>, 16, 4, 4096, out, cus, kinds[1]);
    run("32x32x2", k32<4, 2>, 16, 4, 4096, out, cus, kinds[2]);
    run("32x32x2", k32<4, 3>, 16, 4, 4096, out, cus, kinds[3]);
    run("32x32x2", k32<2, 4>, 16, 2, 4096, out, cus, kinds[4]);
    run("32x32x2", k32<4, 4>, 16, 4, 4096, out, cus, kinds[4]);
    run("32x32x2", k32<2, 5>, 16, 2, 4096, out, cus, kinds[5]);
    run("32x32x2", k32<4, 5>, 16, 4, 4096, out, cus, kinds[5]);
    run("32x32x2", k32<4, 6>, 16, 4, 4096, out, cus, kinds[6]);
    run("32x32x2", k32<1, 0>, 16, 1, 4096, out, cus, kinds[0]);
    run("32x32x2", k32<2, 0>, 16, 2, 4096, out, cus, kinds[0]);
    run("32x32x2", k32<1, 1>, 16, 1, 4096, out, cus, kinds[1]);
    run("32x32x2", k32<2, 1>, 16, 2, 4096, out, cus, kinds[1]);
    run("32x32x2 burst/2", k32b<4, 2>, 16, 4, 4096, out, cus, kinds[0]);
    run("32x32x2 burst/4", k32b<8, 4>, 16, 8, 4096, out, cus, kinds[0]);
    run("32x32x2 burst/8", k32b<16, 8>, 16, 16, 4096, out, cus, kinds[0]);
    run("32x32x2 burst/16", k32b<32, 16>, 16, 32, 4096, out, cus, kinds[0]);
    run("32x32x2 burst/4", k32b<4, 4>, 16, 4, 4096, out, cus, kinds[1]);
    run("32x32x2 burst/8", k32b<8, 8>, 16, 8, 4096, out, cus, kinds[1]);
    run("32x32x2 burst/16 (F23 k-step: 16 pk)", k32b<16, 16>, 16, 16, 4096, out, cus, kinds[1]);
    run("16x16x4 F43 k-step: 96 pk in 4 bursts", kf43<96, 4>, 36, 96, 2048, out, cus, kinds[1]);
    run("16x16x4 F43 k-step: 96 pk in 2 bursts", kf43<96, 2>, 36, 96, 2048, out, cus, kinds[1]);
    run("16x16x4 F43 k-step: 72 pk in 4 bursts", kf43<72, 4>, 36, 72, 2048, out, cus, kinds[1]);
    run("16x16x4 F43 k-step: 0 pk", kf43<0, 4>, 36, 0, 2048, out, cus, kinds[1]);
    run("bf16 32x32x16", kbf<0, 1, 0>, 16, 0, 32768, out, cus, kinds[0]);
    run("bf16 32x32x16", kbf<1, 1, 0>, 16, 1, 32768, out, cus, kinds[0]);
    run("bf16 32x32x16", kbf<2, 1, 0>, 16, 2, 32768, out, cus, kinds[0]);
    run("bf16 32x32x16", kbf<4, 1, 0>, 16, 4, 32768, out, cus, kinds[0]);
    run("bf16 32x32x16", kbf<8, 1, 0>, 16, 8, 32768, out, cus, kinds[0]);
    run("bf16 32x32x16", kbf<2, 1, 1>, 16, 2, 32768, out, cus, kinds[1]);
    run("bf16 32x32x16", kbf<4, 1, 1>, 16, 4, 32768, out, cus, kinds[1]);
    run("bf16 32x32x16", kbf<8, 1, 1>, 16, 8, 32768, out, cus, kinds[1]);
    run("bf16 32x32x16", kbf<2, 1, 7>, 16, 2, 32768, out, cus, kinds[7]);
    run("bf16 32x32x16", kbf<4, 1, 7>, 16, 4, 32768, out, cus, kinds[7]);
    run("bf16 32x32x16", kbf<8, 1, 7>, 16, 8, 32768, out, cus, kinds[7]);
    run("bf16 32x32x16", kbf<2, 1, 4>, 16, 2, 32768, out, cus, kinds[4]);
    run("bf16 32x32x16 burst/4", kbf<16, 4, 1>, 16, 16, 32768, out, cus, kinds[1]);
    run("bf16 32x32x16 burst/16", kbf<64, 16, 1>, 16, 64, 32768, out, cus, kinds[1]);
    for (int thr : {256, 512}) {
        run_w("16x16x4 f32", k16w<0, 1, 0>, thr, 32, 0, 2048, out, cus, kinds[0]);
        run_w("16x16x4 f32", k16w<16, 4, 1>, thr, 32, 16, 2048, out, cus, kinds[1]);
        run_w("16x16x4 f32", k16w<16, 16, 1>, thr, 32, 16, 2048, out, cus, kinds[1]);
        run_w("16x16x4 f32", k16w<8, 4, 0>, thr, 32, 8, 2048, out, cus, kinds[0]);
        run_w("16x16x4 f32", k16w<32, 16, 0>, thr, 32, 32, 2048, out, cus, kinds[0]);
    }
    hipFree(out);
    return 0;
}
