// lbm_pipeline.hip -- the UNFUSED step pipeline: one
// kernel per stage of the reference's Poplibs program
// (main/LbmPoplibs.cpp:225-233 timestep = accelerate_flow -> propagate ->
// collision, :23-95 averageVelocity), for per-stage profiles and as an A/B
// check of the fused kernels:
//
//   accelerate_flow  conditional accelerate of row ny-2, EVERY step
//                    (lbm_kernels.hip accelerate_row; LastChance.cpp:161-183,
//                    D2Q9CodeletsOld.cpp:52-80)
//   (halo refresh)   the populations a propagate pulls across a sub-domain
//                    edge (W1 halo, the engine's pack / exchange / unpack)
//   pipe_propagate   tmp_k(x, y) = cells_k(x - cx_k, y - cy_k)
//                    (LbmPoplibs.cpp:134-175 PropagateVertex)
//   pipe_rebound     obstacle cells: cells_k = tmp_opp(k)
//   pipe_collision   fluid cells: textbook BGK with the equilibrium written
//                    w * rho * (1 + u/c^2 + u^2/(2c^4) - |u|^2/(2c^2)),
//                    every expression in the order of CollisionVertex
//                    (D2Q9CodeletsOptimised.cpp:102-212); per-block partial
//                    sums of |u| (pre-collision)
//   pipe_av          fixed-order fold of the block partials into av_local[t]
//                    (reduceWithOutput + AppendReducedSum, D2Q9Codelets.cpp:18-38;
//                    the engine divides by the fluid-cell count on store)
//
// Each stage reads and writes the SoA lattices through HBM: 72 B per cell for
// propagate, 72 B (fluid) or 64 B (obstacle) for collision / rebound -- the
// memory-traffic cost the fused kernels avoid.  Results are bitwise equal to
// oracle/lbm_oracle.c oracle_pipe_run (IEEE fp32, -ffp-contract=off,
// correctly rounded / and sqrt).

#include "lbm_device.hpp"

namespace lbm {

// grid (ceil(w / BLOCK), h): one cell per thread, rows contiguous
__global__ __launch_bounds__(BLOCK) void pipe_propagate(const float *f, float *t, long long P, int pitch, int w) {
    const int x = blockIdx.x * BLOCK + threadIdx.x, y = blockIdx.y;
    if (x >= w) return;
    const float *c = f + (long long)y * pitch + x;
    float *o = t + (long long)y * pitch + x;
    o[0] = c[0];
    o[1 * P] = c[1 * P - 1];
    o[2 * P] = c[2 * P - pitch];
    o[3 * P] = c[3 * P + 1];
    o[4 * P] = c[4 * P + pitch];
    o[5 * P] = c[5 * P - pitch - 1];
    o[6 * P] = c[6 * P - pitch + 1];
    o[7 * P] = c[7 * P + pitch + 1];
    o[8 * P] = c[8 * P + pitch - 1];
}

__global__ __launch_bounds__(BLOCK) void pipe_rebound(const float *t, float *f, const uint8_t *obst, long long P,
                                                     int pitch, int w) {
    const int x = blockIdx.x * BLOCK + threadIdx.x, y = blockIdx.y;
    if (x >= w || !obst[(long long)y * w + x]) return;
    const float *s = t + (long long)y * pitch + x;
    float *o = f + (long long)y * pitch + x;
    o[0] = s[0];
    o[1 * P] = s[3 * P];
    o[2 * P] = s[4 * P];
    o[3 * P] = s[1 * P];
    o[4 * P] = s[2 * P];
    o[5 * P] = s[7 * P];
    o[6 * P] = s[8 * P];
    o[7 * P] = s[5 * P];
    o[8 * P] = s[6 * P];
}

__global__ __launch_bounds__(BLOCK) void pipe_collision(const float *t, float *f, const uint8_t *obst, long long P,
                                                       int pitch, int w, float omega, float *partials) {
    __shared__ float lds[BLOCK / 64];
    const int x = blockIdx.x * BLOCK + threadIdx.x, y = blockIdx.y;
    float usum = 0.f;
    if (x < w && !obst[(long long)y * w + x]) {
        const float *in = t + (long long)y * pitch + x;
        float *out = f + (long long)y * pitch + x;
        const float c_sq = 1.f / 3.f;
        const float cc2 = (2.f * c_sq * c_sq);
        const float w0 = 4.f / 9.f, w1 = 1.f / 9.f, w2 = 1.f / 36.f;
        float s[Q];
#pragma unroll
        for (int k = 0; k < Q; ++k) s[k] = in[k * P];
        float local_density = 0.f;
#pragma unroll
        for (int kk = 0; kk < Q; ++kk) local_density += s[kk];
        const float u_x = ((s[1] + s[5] + s[8]) - (s[3] + s[6] + s[7])) / local_density;
        const float u_y = ((s[2] + s[5] + s[6]) - (s[4] + s[7] + s[8])) / local_density;
        const float u_sq = u_x * u_x + u_y * u_y;
        usum = sqrtf(u_sq);
        const float u[Q] = {0, u_x, u_y, -u_x, -u_y, u_x + u_y, -u_x + u_y, -u_x - u_y, u_x - u_y};
        const float u_over_2csq = u_sq / (2.f * c_sq);
        float d[Q];
        d[0] = w0 * local_density * (1.f - u_over_2csq);
#pragma unroll
        for (int k = 1; k < Q; ++k) {
            const float wk = k < 5 ? w1 : w2;
            d[k] = wk * local_density * (1.f + u[k] / c_sq + (u[k] * u[k]) / cc2 - u_over_2csq);
        }
#pragma unroll
        for (int kk = 0; kk < Q; ++kk) out[kk * P] = s[kk] + omega * (d[kk] - s[kk]);
    }
    const float b = block_sum(usum, lds);
    if (threadIdx.x == 0) partials[blockIdx.y * gridDim.x + blockIdx.x] = b;
}

__global__ __launch_bounds__(BLOCK) void pipe_av(const float *partials, int n, float *av_local, int t) {
    __shared__ float lds[BLOCK / 64];
    const float v = sum_partials_n<BLOCK>(partials, n, lds);
    if (threadIdx.x == 0) av_local[t] = v;
}

// ---- host side ---------------------------------------------------------------

int pipe_blocks(int w, int h) { return ((w + BLOCK - 1) / BLOCK) * h; }

hipError_t launch_pipe_propagate(const float *f, float *t, long long P, int pitch, int w, int h, hipStream_t s) {
    hipLaunchKernelGGL(pipe_propagate, dim3((w + BLOCK - 1) / BLOCK, h), dim3(BLOCK), 0, s, f, t, P, pitch, w);
    return hipGetLastError();
}

hipError_t launch_pipe_rebound(const float *t, float *f, const uint8_t *obst, long long P, int pitch, int w, int h,
                               hipStream_t s) {
    hipLaunchKernelGGL(pipe_rebound, dim3((w + BLOCK - 1) / BLOCK, h), dim3(BLOCK), 0, s, t, f, obst, P, pitch, w);
    return hipGetLastError();
}

hipError_t launch_pipe_collision(const float *t, float *f, const uint8_t *obst, long long P, int pitch, int w, int h,
                                 float omega, float *partials, hipStream_t s) {
    hipLaunchKernelGGL(pipe_collision, dim3((w + BLOCK - 1) / BLOCK, h), dim3(BLOCK), 0, s, t, f, obst, P, pitch, w,
                       omega, partials);
    return hipGetLastError();
}

hipError_t launch_pipe_av(const float *partials, int n, float *av_local, int t, hipStream_t s) {
    hipLaunchKernelGGL(pipe_av, dim3(1), dim3(BLOCK), 0, s, partials, n, av_local, t);
    return hipGetLastError();
}

}  // namespace lbm
