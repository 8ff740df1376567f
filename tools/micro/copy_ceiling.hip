// Copy-rate ceiling on this box: what a float4 streaming copy / read reaches
// at the stream kernel's lattice size (2 x 2.4 GB), with 1 or 4 loads in
// flight per lane and plain or non-temporal accesses.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/copy_ceiling tools/micro/copy_ceiling.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copyk(const f4 *__restrict__ a, f4 *__restrict__ b, long long n4) {
    const long long stride = (long long)gridDim.x * 256 * U;
    for (long long i = blockIdx.x * 256LL * U + threadIdx.x; i < n4; i += stride) {
        f4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long k = i + u * 256LL;
            v[u] = k < n4 ? (NT ? __builtin_nontemporal_load(a + k) : a[k]) : f4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long k = i + u * 256LL;
            if (k < n4) {
                if (NT) __builtin_nontemporal_store(v[u], b + k);
                else b[k] = v[u];
            }
        }
    }
}

template <int U>
__global__ __launch_bounds__(256) void readk(const f4 *__restrict__ a, long long n4, float *sink) {
    const long long stride = (long long)gridDim.x * 256 * U;
    f4 acc = {0, 0, 0, 0};
    for (long long i = blockIdx.x * 256LL * U + threadIdx.x; i < n4; i += stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long k = i + u * 256LL;
            if (k < n4) acc += a[k];
        }
    }
    if (acc.x + acc.y + acc.z + acc.w == 1234.5f) sink[0] = acc.x;
}

template <class K, class... A>
static void timeit(const char *name, double bytes, int blocks, K k, A... args) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, args...);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, args...);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("{\"variant\": \"%s\", \"blocks\": %d, \"ms\": %.4f, \"TBps\": %.3f, \"err\": \"%s\"}\n", name, blocks, ms,
           bytes / ms / 1e9, hipGetErrorString(hipGetLastError()));
}

int main() {
    const long long n4 = 2416LL * 1000 * 1000 / 16;  // 2.416 GB per buffer (one 8192^2 lattice)
    f4 *a = nullptr, *b = nullptr;
    float *sink = nullptr;
    if (hipMalloc(&a, n4 * 16) != hipSuccess || hipMalloc(&b, n4 * 16) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess)
        return 1;
    (void)hipMemset(a, 0, n4 * 16);
    (void)hipMemset(b, 0, n4 * 16);
    const double cb = 32.0 * n4, rb = 16.0 * n4;
    for (int blocks : {2048, 8192, 32768}) {
        timeit("copy_u1", cb, blocks, copyk<1, false>, (const f4 *)a, b, n4);
        timeit("copy_u4", cb, blocks, copyk<4, false>, (const f4 *)a, b, n4);
        timeit("copy_u4_nt", cb, blocks, copyk<4, true>, (const f4 *)a, b, n4);
        timeit("read_u1", rb, blocks, readk<1>, (const f4 *)a, n4, sink);
        timeit("read_u4", rb, blocks, readk<4>, (const f4 *)a, n4, sink);
    }
    return 0;
}
