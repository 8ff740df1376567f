// stream_pattern.hip -- HBM rate of the register-streaming kernels' memory
// pattern with the arithmetic removed (or replaced by a tunable amount of
// independent packed-fp32 work), to separate "the access pattern's own
// bandwidth ceiling" from "compute / memory overlap" for lbm_stream2.hip.
//
// Lattice: row-interleaved SoA like the engine, f[y][k][x] (9 planes of a row
// adjacent), 8192^2 cells, plane row = RF floats.  One wave walks a strip of
// 64*V columns (V floats per lane: 2 = the stream kernel's float2, 4 =
// float4) over a segment of HS rows plus 2*S re-streamed rows, loading the
// nine plane chunks of every row (prefetched one row ahead) and storing the
// owned columns of row j-S to the second lattice.  Strips overlap by 2*S
// columns, as in the kernel.  WORK = packed-fp32 FMAs per lane per row (the
// real kernel issues ~430 packed ops per row at S = 4).
//
//   hipcc --offload-arch=gfx950 -O3 -o stream_pattern stream_pattern.hip && ./stream_pattern
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int NX = 8192, NY = 8192, S = 4, Q = 9;
constexpr int XOFF = 64, GR = 8;  // GR ghost rows each side: >= every SS used below
constexpr int RF = ((NX + XOFF + GR + 2 + 63) / 64) * 64;  // floats per plane row
constexpr long long PITCH = (long long)Q * RF;             // floats per lattice row

__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int xcd = b & 7;
    const int q = nb >> 3, r = nb & 7;
    const int start = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return start + (b >> 3);
}

template <int V>
struct Vec;
template <>
struct Vec<2> { typedef f2 T; };
template <>
struct Vec<4> { typedef f4 T; };

// LAYOUT 0: f[y][k][x] (row-interleaved, the engine's); 1: f[k][y][x] (planar);
// 2: f[y][x/128][k][x%128] (row-interleaved blocks of 128 columns: one row of a
// 128-column block = 9 x 512 B contiguous).
// W waves per workgroup take W adjacent strips (co-scheduled on one CU).
// NT: non-temporal stores.  SS: steps (re-streamed rows and overlap columns).
// ALT: units of odd segments walk their rows top-down, so two neighbouring
// segments read their shared 2*SS boundary rows at about the same time (both
// at the start or both at the end of the unit) instead of a unit apart.
template <int V, int WORK, int LAYOUT = 0, int W = 1, bool NT = false, int PD = 1, bool STORE = true, int SS = S,
          bool ALT = false>
__global__ __launch_bounds__(64 * W) void pattern(const float *__restrict__ fin, float *__restrict__ fout, int hs,
                                                  int nstrip, int total, float *sink) {
    typedef typename Vec<V>::T T;
    const long long PS = LAYOUT == 1 ? RF : PITCH;                                            // row stride
    const long long KS = LAYOUT == 0 ? RF : LAYOUT == 2 ? 128 : (long long)(NY + 2 * GR) * RF;  // plane stride
    const int t = xcd_remap(blockIdx.x, gridDim.x) * W + (int)(threadIdx.x >> 6);
    if (t >= total) return;
    const int lane = threadIdx.x & 63;
    const int ow = 64 * V - 2 * SS;
    const int seg = t / nstrip, strip = t - seg * nstrip;
    const int xo0 = strip * ow, xo1 = min(xo0 + ow, NX);
    const int base = ((xo0 - SS) & ~(V - 1));
    const int xa = base + V * lane;
    const bool own = xa >= xo0 && xa + V - 1 < xo1;
    const int yo0 = seg * hs, yo1 = min(yo0 + hs, NY);
    const int xg = XOFF + xa;
    const long long xo = LAYOUT == 2 ? (long long)(xg >> 7) * (Q * 128) + (xg & 127) : xg;
    const float *src = fin + (long long)GR * PS + xo;
    float *dst = fout + (long long)GR * PS + xo;
    extern __shared__ float occupancy_limiter[];
    if (hs < 0) occupancy_limiter[threadIdx.x] = 0.f;  // never: keeps the dynamic LDS request
    T v[Q], nv[Q], nv2[Q];
    const bool down = ALT && (seg & 1);
    const int d = down ? -1 : 1;
    const int jf = down ? yo1 + SS - 1 : yo0 - SS;  // first and last row of the walk
    const int jl = down ? yo0 - SS : yo1 + SS - 1;
    auto clampj = [&](int jj) { return down ? max(jj, jl) : min(jj, jl); };
    int j = jf;
#pragma unroll
    for (int k = 0; k < Q; ++k) v[k] = *reinterpret_cast<const T *>(src + (long long)j * PS + (long long)k * KS);
    if (PD == 2) {
#pragma unroll
        for (int k = 0; k < Q; ++k) nv2[k] = *reinterpret_cast<const T *>(src + (long long)clampj(j + d) * PS + (long long)k * KS);
    }
    f2 acc[4] = {f2{0.f, 0.f}, f2{1.f, 1.f}, f2{2.f, 2.f}, f2{3.f, 3.f}};
    const int nrows = yo1 - yo0 + 2 * SS;
    for (int i = 0; i < nrows; ++i, j += d) {
        const int jn = clampj(j + PD * d);
        if (PD == 2) {
#pragma unroll
            for (int k = 0; k < Q; ++k) nv[k] = nv2[k];
        }
#pragma unroll
        for (int k = 0; k < Q; ++k) (PD == 2 ? nv2[k] : nv[k]) = *reinterpret_cast<const T *>(src + (long long)jn * PS + (long long)k * KS);
        // stand-in arithmetic: WORK independent packed FMAs per lane
#pragma unroll
        for (int w = 0; w < WORK; ++w) acc[w & 3] = __builtin_elementwise_fma(acc[w & 3], f2{1.0001f, 0.9999f}, f2{v[w % Q][0], v[(w + 1) % Q][1]});
        const int y = j - SS * d;
        if (STORE && y >= yo0 && y < yo1 && own) {
#pragma unroll
            for (int k = 0; k < Q; ++k) {
                T o = v[k];
                o[0] += acc[k & 3][0] * 0.0f;
                T *pd = reinterpret_cast<T *>(dst + (long long)y * PS + (long long)k * KS);
                if (NT)
                    __builtin_nontemporal_store(o, pd);
                else
                    *pd = o;
            }
        }
#pragma unroll
        for (int k = 0; k < Q; ++k) v[k] = nv[k];
    }
    if (acc[0][0] == 12345.f) sink[0] = acc[1][1] + acc[2][0] + acc[3][1];
}

template <int V, int WORK, int LAYOUT = 0, int W = 1, bool NT = false, int PD = 1, bool STORE = true, int SS = S,
          bool ALT = false>
void run(const char *name, float *a, float *b, int hs, float *sink, int waves_per_simd = 0) {
    // waves_per_simd > 0: dynamic LDS so that only that many waves fit per SIMD
    const size_t lds = waves_per_simd > 0 ? (size_t)(160 * 1024) / (4 * waves_per_simd) * W - 256 : 0;
    const int ow = 64 * V - 2 * SS;
    const int nstrip = (NX + ow - 1) / ow, nseg = (NY + hs - 1) / hs, total = nstrip * nseg;
    const int blocks = (total + W - 1) / W;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 20; ++i)
        hipLaunchKernelGGL((pattern<V, WORK, LAYOUT, W, NT, PD, STORE, SS, ALT>), dim3(blocks), dim3(64 * W), lds, 0, a, b, hs, nstrip, total,
                           sink);
    const int reps = 40;
    (void)hipEventRecord(e0);
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((pattern<V, WORK, LAYOUT, W, NT, PD, STORE, SS, ALT>), dim3(blocks), dim3(64 * W), lds, 0, (i & 1) ? b : a,
                           (i & 1) ? a : b, hs, nstrip, total, sink);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    const double lattice = 72.0 * NX * NY;                                      // algorithmic bytes per pass
    const double moved = 36.0 * NX * NY * ((double)(hs + 2 * SS) / hs) * (64.0 * V / ow) + 36.0 * NX * NY;
    printf("{\"variant\": \"%s\", \"V\": %d, \"hs\": %d, \"work\": %d, \"waves\": %d, \"waves_per_simd\": %d, "
           "\"ms\": %.4f, \"lattice_TBps\": %.3f, \"moved_TBps\": %.3f, \"err\": \"%s\"}\n",
           name, V, hs, WORK, total, waves_per_simd, ms, lattice / ms / 1e9, moved / ms / 1e9,
           hipGetErrorString(hipGetLastError()));
}

// plain float4 copy of n floats (grid-stride), the HBM ceiling for comparison
__global__ __launch_bounds__(256) void copy4(const f4 *__restrict__ a, f4 *__restrict__ b, long long n4) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) b[i] = a[i];
}
__global__ __launch_bounds__(256) void read4(const f4 *__restrict__ a, float *sink, long long n4) {
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) acc += a[i];
    if (acc[0] == 12345.f) sink[0] = acc[1] + acc[2] + acc[3];
}
static void run_copy(const char *name, float *a, float *b, size_t n, float *sink, bool read_only) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const long long n4 = (long long)(n / 4);
    const int blocks = 256 * 32;
    for (int r = 0; r < 25; ++r) {
        if (r == 5) (void)hipEventRecord(e0);
        if (read_only)
            hipLaunchKernelGGL(read4, dim3(blocks), dim3(256), 0, 0, (const f4 *)a, sink, n4);
        else
            hipLaunchKernelGGL(copy4, dim3(blocks), dim3(256), 0, 0, (const f4 *)a, (f4 *)b, n4);
    }
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 20;
    const double bytes = (read_only ? 4.0 : 8.0) * (double)n;
    printf("{\"variant\": \"%s\", \"ms\": %.4f, \"moved_TBps\": %.3f, \"err\": \"%s\"}\n", name, ms, bytes / ms / 1e9,
           hipGetErrorString(hipGetLastError()));
}

int main(int argc, char **argv) {
    const size_t n = (size_t)(NY + 2 * GR) * PITCH;
    float *a = nullptr, *b = nullptr, *sink = nullptr;
    if (hipMalloc(&a, n * 4) != hipSuccess || hipMalloc(&b, n * 4) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) {
        fprintf(stderr, "alloc failed\n");
        return 1;
    }
    (void)hipMemset(a, 0, n * 4);
    (void)hipMemset(b, 0, n * 4);
    // occupancy-matched to the stream kernel (2 waves per SIMD)
    const int which = argc > 1 ? atoi(argv[1]) : 0;
    if (which == 0) {
        run<2, 0>("f2_hs35_o2", a, b, 35, sink, 2);
        run<2, 0, 0, 4>("f2_hs35_w4_o2", a, b, 35, sink, 2);
        run<2, 0, 0, 4, true>("f2_hs35_w4_nt_o2", a, b, 35, sink, 2);
        run<2, 0, 0, 1, false, 2>("f2_hs35_pd2_o2", a, b, 35, sink, 2);
        run<2, 0, 0, 4, true, 2>("f2_hs35_w4_nt_pd2_o2", a, b, 35, sink, 2);
        run<2, 0, 0, 4, true>("f2_hs35_w4_nt_o3", a, b, 35, sink, 3);
        run<2, 0, 0, 4, true>("f2_hs35_w4_nt_o4", a, b, 35, sink, 4);
        run<2, 0>("f2_hs35_o8", a, b, 35, sink, 0);
        run<2, 0, 0, 4, true>("f2_hs35_w4_nt_o8", a, b, 35, sink, 0);
        run<2, 384, 0, 4, true>("f2_hs35_w4_nt_work384_o2", a, b, 35, sink, 2);
        run<2, 384>("f2_hs35_work384_o2", a, b, 35, sink, 2);
    } else if (which == 2) {
        run_copy("copy4_lattice", a, b, n, sink, false);
        run_copy("read4_lattice", a, b, n, sink, true);
        run<2, 0, 0, 1, false, 1, false>("L0_hs96_o2_noStore", a, b, 96, sink, 2);
        run<2, 0, 0, 1, false, 1, false>("L0_hs96_o8_noStore", a, b, 96, sink, 0);
        run<2, 0, 0, 4, true>("L0_hs96_w4nt_o2", a, b, 96, sink, 2);
        run<2, 0, 0, 4, true>("L0_hs96_w4nt_o8", a, b, 96, sink, 0);
        run<4, 0, 0>("V4_hs96_o2", a, b, 96, sink, 2);
        run<4, 0, 0>("V4_hs96_o8", a, b, 96, sink, 0);
        run<2, 0, 0>("L0_hs400_o8", a, b, 400, sink, 0);
        run<2, 0, 0>("L0_hs20_o8", a, b, 20, sink, 0);
    } else if (which == 3) {
        // S = 7, 144-row segments (the tolerance default): odd segments walking
        // down (ALT) against all up; with and without stand-in arithmetic
        for (int rep = 0; rep < 2; ++rep) {
            run<2, 0, 0, 1, false, 1, true, 7, false>("s7_hs144_up", a, b, 144, sink, 2);
            run<2, 0, 0, 1, false, 1, true, 7, true>("s7_hs144_alt", a, b, 144, sink, 2);
            run<2, 0, 0, 1, false, 1, true, 7, false>("s7_hs48_up", a, b, 48, sink, 2);
            run<2, 0, 0, 1, false, 1, true, 7, true>("s7_hs48_alt", a, b, 48, sink, 2);
            run<2, 384, 0, 1, false, 1, true, 7, false>("s7_hs144_up_work384", a, b, 144, sink, 2);
            run<2, 384, 0, 1, false, 1, true, 7, true>("s7_hs144_alt_work384", a, b, 144, sink, 2);
        }
    } else {
        // layouts: row-interleaved (0), planar (1), 128-column blocks (2); hs 35 and 96
        run<2, 0, 0>("L0_hs35_o2", a, b, 35, sink, 2);
        run<2, 0, 1>("L1_hs35_o2", a, b, 35, sink, 2);
        run<2, 0, 2>("L2_hs35_o2", a, b, 35, sink, 2);
        run<2, 0, 0>("L0_hs96_o2", a, b, 96, sink, 2);
        run<2, 0, 1>("L1_hs96_o2", a, b, 96, sink, 2);
        run<2, 0, 2>("L2_hs96_o2", a, b, 96, sink, 2);
        run<2, 0, 2, 4, true>("L2_hs96_w4_nt_o2", a, b, 96, sink, 2);
        run<2, 0, 0>("L0_hs96_o4", a, b, 96, sink, 4);
        run<2, 0, 2>("L2_hs96_o4", a, b, 96, sink, 4);
        run<2, 0, 0>("L0_hs96_o8", a, b, 96, sink, 0);
        run<2, 0, 2>("L2_hs96_o8", a, b, 96, sink, 0);
        run<2, 384, 2>("L2_hs96_work384_o2", a, b, 96, sink, 2);
        run<2, 384, 0>("L0_hs96_work384_o2", a, b, 96, sink, 2);
    }
    return 0;
}
