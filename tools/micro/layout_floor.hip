// layout_floor.hip -- the HBM rate of the stream kernel's access pattern (no
// arithmetic) under two lattice layouts, to tell whether the ~1.2 ms per pass
// floor at 8192^2 comes from the pattern itself (DRAM / TLB locality of nine
// 512-B plane chunks per row, 300 KB apart) or from the kernel:
//   L0: row-interleaved f[y][k][x] (the engine's layout)
//   L3: block-major f[xb][y][k][128]: one strip's rows are contiguous, so a
//       wave streams 4.6 KB per row through consecutive addresses.
// Strips are 128 columns without overlap here (the floor of the pattern, not
// the kernel's geometry); segments of HS rows re-stream 2S rows as the kernel.
//   hipcc --offload-arch=gfx950 -O3 -o layout_floor layout_floor.hip && ./layout_floor
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int NX = 8192, NY = 8192, S = 5, Q = 9, BW = 128;
constexpr int RF = NX + 256;                    // L0 plane row (floats), with a ghost pad
constexpr long long P0 = (long long)Q * RF;     // L0 row pitch
constexpr long long P3 = (long long)Q * BW;     // L3 row pitch inside a block
constexpr long long B3 = P3 * (NY + 16);        // L3 block stride
constexpr int NB = NX / BW;

__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int xcd = b & 7;
    const int q = nb >> 3, r = nb & 7;
    const int start = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return start + (b >> 3);
}

template <int LAYOUT, int W, bool NT, int PD>
__global__ __launch_bounds__(64 * W) void pattern(const float *__restrict__ fin, float *__restrict__ fout, int hs,
                                                  int total, float *sink) {
    const int t = xcd_remap(blockIdx.x, gridDim.x) * W + (int)(threadIdx.x >> 6);
    if (t >= total) return;
    const int lane = threadIdx.x & 63;
    const int seg = t / NB, strip = t - seg * NB;
    const int yo0 = seg * hs, yo1 = min(yo0 + hs, NY);
    const long long ps = LAYOUT == 0 ? P0 : P3, ks = LAYOUT == 0 ? RF : BW;
    const long long col = LAYOUT == 0 ? (long long)strip * BW + 2 * lane : (long long)strip * B3 + 2 * lane;
    const float *src = fin + 8 * ps + col;
    float *dst = fout + 8 * ps + col;
    extern __shared__ float occupancy_limiter[];
    if (hs < 0) occupancy_limiter[threadIdx.x] = 0.f;
    f2 v[PD + 1][Q];
    int j = yo0 - S;
    const int jl = yo1 + S - 1;
#pragma unroll
    for (int d = 0; d < PD; ++d)
#pragma unroll
        for (int k = 0; k < Q; ++k) v[d][k] = *reinterpret_cast<const f2 *>(src + (long long)min(j + d, jl) * ps + k * ks);
    f2 acc = {0.f, 0.f};
    for (; j <= jl; ++j) {
#pragma unroll
        for (int k = 0; k < Q; ++k) v[PD][k] = *reinterpret_cast<const f2 *>(src + (long long)min(j + PD, jl) * ps + k * ks);
        const int y = j - S;
        if (y >= yo0) {
#pragma unroll
            for (int k = 0; k < Q; ++k) {
                f2 *pd = reinterpret_cast<f2 *>(dst + (long long)y * ps + k * ks);
                if (NT)
                    __builtin_nontemporal_store(v[0][k], pd);
                else
                    *pd = v[0][k];
            }
        }
        acc += v[0][0];
#pragma unroll
        for (int d = 0; d < PD; ++d)
#pragma unroll
            for (int k = 0; k < Q; ++k) v[d][k] = v[d + 1][k];
    }
    if (acc[0] == 12345.f) sink[0] = acc[1];
}

template <int LAYOUT, int W, bool NT, int PD>
void run(const char *name, float *a, float *b, int hs, float *sink, int waves_per_simd) {
    const size_t lds = waves_per_simd > 0 ? (size_t)(160 * 1024) / (4 * waves_per_simd) * W - 256 : 0;
    const int nseg = (NY + hs - 1) / hs, total = NB * nseg;
    const int blocks = (total + W - 1) / W;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 20; ++i)
        hipLaunchKernelGGL((pattern<LAYOUT, W, NT, PD>), dim3(blocks), dim3(64 * W), lds, 0, a, b, hs, total, sink);
    const int reps = 40;
    (void)hipEventRecord(e0);
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((pattern<LAYOUT, W, NT, PD>), dim3(blocks), dim3(64 * W), lds, 0, (i & 1) ? b : a,
                           (i & 1) ? a : b, hs, total, sink);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    const double lattice = 72.0 * NX * NY;
    const double moved = 36.0 * NX * NY * ((double)(hs + 2 * S) / hs) + 36.0 * NX * NY;
    printf("{\"variant\": \"%s\", \"hs\": %d, \"waves_per_simd\": %d, \"ms\": %.4f, \"lattice_TBps\": %.3f, "
           "\"moved_TBps\": %.3f, \"err\": \"%s\"}\n",
           name, hs, waves_per_simd, ms, lattice / ms / 1e9, moved / ms / 1e9, hipGetErrorString(hipPeekAtLastError()));
    fflush(stdout);
    if (hipGetLastError() != hipSuccess || ms <= 0.f) exit(3);  // stop at the first fault
}

__global__ __launch_bounds__(256) void copy4(const f4 *__restrict__ a, f4 *__restrict__ b, long long n4) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) b[i] = a[i];
}

int main() {
    // L0 rows 8 + j for j in [-S, NY + S - 1]: (NY + 16) rows of P0; L3: NB blocks of B3
    const size_t n = std::max((size_t)(NY + 16) * P0, (size_t)NB * B3) + 4096;
    float *a = nullptr, *b = nullptr, *sink = nullptr;
    if (hipMalloc(&a, n * 4) != hipSuccess || hipMalloc(&b, n * 4) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) {
        fprintf(stderr, "alloc failed\n");
        return 1;
    }
    (void)hipMemset(a, 0, n * 4);
    (void)hipMemset(b, 0, n * 4);
    {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        const long long n4 = (long long)(72LL * NX * NY / 8 / 16);  // one lattice worth of floats / 4
        for (int r = 0; r < 25; ++r) {
            if (r == 5) (void)hipEventRecord(e0);
            hipLaunchKernelGGL(copy4, dim3(256 * 32), dim3(256), 0, 0, (const f4 *)a, (f4 *)b, n4);
        }
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ms /= 20;
        printf("{\"variant\": \"copy4\", \"ms\": %.4f, \"moved_TBps\": %.3f}\n", ms, 32.0 * n4 / ms / 1e9);
    }
    run<0, 1, false, 1>("L0_o2", a, b, 96, sink, 2);
    run<3, 1, false, 1>("L3_o2", a, b, 96, sink, 2);
    run<0, 1, true, 1>("L0_nt_o2", a, b, 96, sink, 2);
    run<3, 1, true, 1>("L3_nt_o2", a, b, 96, sink, 2);
    run<0, 4, true, 1>("L0_w4_nt_o2", a, b, 96, sink, 2);
    run<3, 4, true, 1>("L3_w4_nt_o2", a, b, 96, sink, 2);
    run<0, 1, false, 2>("L0_pd2_o2", a, b, 96, sink, 2);
    run<3, 1, false, 2>("L3_pd2_o2", a, b, 96, sink, 2);
    run<0, 1, false, 1>("L0_o4", a, b, 96, sink, 4);
    run<3, 1, false, 1>("L3_o4", a, b, 96, sink, 4);
    run<0, 1, false, 1>("L0_hs400_o2", a, b, 400, sink, 2);
    run<3, 1, false, 1>("L3_hs400_o2", a, b, 400, sink, 2);
    return 0;
}
