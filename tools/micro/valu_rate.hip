// valu_rate.hip -- issue rate of v_fma_f32 vs v_pk_fma_f32 vs v_pk_mul_f32 on
// the local GPU (microbenchmark behind the packed-fp32 choice in
// lbm_stream2.hip).  8 independent chains per lane, enough waves to fill
// every SIMD; prints wave-instructions per SIMD-cycle for each form.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 1 << 14;

__global__ void k_fma(float *out, float a, float b) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3f + i;
    for (int it = 0; it < ITERS; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_fmaf(x[i], a, b);
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_pkfma(float *out, float a, float b) {
    f2 x[8];
    for (int i = 0; i < 8; ++i) x[i] = f2{threadIdx.x * 1e-3f + i, (float)i};
    const f2 A = f2{a, a}, B = f2{b, b};
    for (int it = 0; it < ITERS; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_elementwise_fma(x[i], A, B);
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_pkmul(float *out, float a, float b) {
    f2 x[8];
    for (int i = 0; i < 8; ++i) x[i] = f2{threadIdx.x * 1e-3f + i, (float)i};
    const f2 A = f2{a, a};
    for (int it = 0; it < ITERS; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = x[i] * A;
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul(float *out, float a, float b) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3f + i;
    for (int it = 0; it < ITERS; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = x[i] * a;
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    const int blocks = cus * 4 * 8;  // 8 waves per SIMD
    float *out;
    hipMalloc(&out, sizeof(float) * blocks * 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int clk_khz = 0;
    hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
    struct { const char *name; void (*k)(float *, float, float); } ks[] = {
        {"v_fma_f32", k_fma}, {"v_pk_fma_f32", k_pkfma}, {"v_mul_f32", k_mul}, {"v_pk_mul_f32", k_pkmul}};
    for (auto &k : ks) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(64), 0, 0, out, 0.999f, 1e-3f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double instr = (double)blocks * ITERS * 8;  // wave-instructions
            const double simd_cycles = ms * 1e-3 * clk_khz * 1e3 * cus * 4;
            if (rep)
                printf("%-14s %.3f ms  %.3f wave-instr per SIMD-cycle (clock %d MHz, %d CUs)\n", k.name, ms,
                       instr / simd_cycles, clk_khz / 1000, cus);
        }
    }
    return 0;
}
