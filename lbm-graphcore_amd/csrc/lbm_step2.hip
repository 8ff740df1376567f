// lbm_step2.hip -- fused TWO-step kernel (temporal blocking through LDS).
//
// Each workgroup owns a T2W x T2H tile of output cells.  Phase 1 computes
// step t+1 on the tile plus a one-cell halo ((T2W+2) x (T2H+2) cells) from
// the HBM lattice at step t (pulling from up to two cells out: ghost ring
// width 2) and keeps it in LDS; phase 2 computes step t+2 on the tile from
// LDS and writes it back.  The lattice crosses HBM once per two time steps
// (72 B per cell per launch instead of per step); the halo recompute costs
// (T2W+2)(T2H+2)/(T2W*T2H) - 1 = 16 % extra arithmetic and L2/MALL re-reads.
//
// The per-cell arithmetic is the same as the one-step kernels
// (lbm_device.hpp, LastChance.cpp:226-262), evaluated in the same order, so
// the result is bitwise identical to two one-step launches and to the CPU
// oracle.  Halo cells outside the sub-domain are the periodic images (or the
// neighbour sub-domain's cells) -- their populations come from the width-2
// ghost ring and their obstacle flags from a ghosted obstacle map, so they
// are computed exactly as their owner computes them.
//
// Both steps' |u| sums (step t+1 over the tile interior only, so each cell is
// counted once) are reduced per block; the next reducing launch folds them.
// Edge cells write all nine populations of the two outermost rows/columns to
// the W2 halo destinations (own ghost ring or send buffers).

#include "lbm_device.hpp"

namespace lbm {

__device__ __forceinline__ float accel_flag(const Step2Args &a, int y) {
    int g = a.gy0 + y;
    g = g < 0 ? g + a.ny : (g >= a.ny ? g - a.ny : g);
    return (g == a.accel_g) ? 1.00f : 0.00f;
}

__device__ __forceinline__ void store2(const Dst2 &d, int sa, int sb, const float (&o)[Q]) {
    float *p = d.base + (long long)sa * d.s1 + (long long)sb * d.s2;
#pragma unroll
    for (int k = 0; k < Q; ++k) p[k * d.ks] = o[k];
}

template <bool kReduce>
__global__ __launch_bounds__(BLOCK) void step2(Step2Args a) {
    constexpr int MW = T2W + 2, MH = T2H + 2;
    __shared__ float mid[Q][MH][MW];
    __shared__ float lds[4];
    if (kReduce && blockIdx.x == 0) reduce_pending(a.ctl, a.partials_prev, a.av_local, lds);

    const int tid = threadIdx.x;
    const long long P = a.plane;
    const int pitch = a.pitch;
    const int nb = gridDim.x;
    const int t = xcd_remap(blockIdx.x, nb);
    float tot1 = 0.f, tot2 = 0.f;

    if (t < a.total) {
        const int r = rect_of(a.rect_begin, t);
        const Rect R = a.rect[r];
        const int lt = t - a.rect_begin[r];
        const int ty = R.y0 + lt / R.wc;
        const int tx = R.x0 + (lt - (lt / R.wc) * R.wc);
        const int X0 = tx * T2W, Y0 = ty * T2H;

        // ---- phase 1: step t+1 on tile + 1-cell halo, into LDS ----
        for (int i = tid; i < MW * MH; i += BLOCK) {
            const int ly = i / MW, lx = i - ly * MW;
            const int x = X0 + lx - 1, y = Y0 + ly - 1;
            if (x > a.w || y > a.h) continue;  // beyond what the tile's outputs pull
            const float *c = a.fin + (long long)y * pitch + x;
            const float s[Q] = {c[0],
                                c[1 * P - 1],
                                c[2 * P - pitch],
                                c[3 * P + 1],
                                c[4 * P + pitch],
                                c[5 * P - pitch - 1],
                                c[6 * P - pitch + 1],
                                c[7 * P + pitch + 1],
                                c[8 * P + pitch - 1]};
            const bool ob = a.obst_g[(long long)(y + 1) * a.ogp + (x + 1)] != 0;
            float o[Q];
            const float u = collide(s, o, ob, accel_flag(a, y), a.omega, a.omo, a.w1, a.w2);
#pragma unroll
            for (int k = 0; k < Q; ++k) mid[k][ly][lx] = o[k];
            if (lx >= 1 && lx <= T2W && ly >= 1 && ly <= T2H && x < a.w && y < a.h) tot1 += u;
        }
        __syncthreads();

        // ---- phase 2: step t+2 on the tile, from LDS, to HBM ----
        for (int i = tid; i < T2W * T2H; i += BLOCK) {
            const int ly = i / T2W, lx = i - ly * T2W;
            const int x = X0 + lx, y = Y0 + ly;
            if (x >= a.w || y >= a.h) continue;
            const int mx = lx + 1, my = ly + 1;
            const float s[Q] = {mid[0][my][mx],         mid[1][my][mx - 1],     mid[2][my - 1][mx],
                                mid[3][my][mx + 1],     mid[4][my + 1][mx],     mid[5][my - 1][mx - 1],
                                mid[6][my - 1][mx + 1], mid[7][my + 1][mx + 1], mid[8][my + 1][mx - 1]};
            const bool ob = a.obst_g[(long long)(y + 1) * a.ogp + (x + 1)] != 0;
            float o[Q];
            tot2 += collide(s, o, ob, accel_flag(a, y), a.omega, a.omo, a.w1, a.w2);
            float *w0 = a.fout + (long long)y * pitch + x;
#pragma unroll
            for (int k = 0; k < Q; ++k) w0[k * P] = o[k];

            // W2 halo: all nine populations of the two outermost rows/columns
            const bool east = x >= a.w - 2, west = x < 2, north = y >= a.h - 2, south = y < 2;
            if (east) store2(a.dst[DE], x - (a.w - 2), y, o);
            if (west) store2(a.dst[DW], x, y, o);
            if (north) {
                store2(a.dst[DN], y - (a.h - 2), x, o);
                if (east) store2(a.dst[DNE], y - (a.h - 2), x - (a.w - 2), o);
                if (west) store2(a.dst[DNW], y - (a.h - 2), x, o);
            }
            if (south) {
                store2(a.dst[DS], y, x, o);
                if (west) store2(a.dst[DSW], y, x, o);
                if (east) store2(a.dst[DSE], y, x - (a.w - 2), o);
            }
        }
    }

    const float s1 = block_sum(tot1, lds);
    const float s2 = block_sum(tot2, lds);
    if (threadIdx.x == 0) {
        a.partials_out[blockIdx.x] = s1;
        a.partials_out[(long long)a.stride + blockIdx.x] = s2;
        if (kReduce && blockIdx.x == 0) publish_pending(a.ctl, 2, a.n_total, a.stride);
    }
}

hipError_t launch_step2(const Step2Args &a, int blocks, bool reduce, hipStream_t s) {
    if (reduce)
        hipLaunchKernelGGL(step2<true>, dim3(blocks), dim3(BLOCK), 0, s, a);
    else
        hipLaunchKernelGGL(step2<false>, dim3(blocks), dim3(BLOCK), 0, s, a);
    return hipGetLastError();
}

}  // namespace lbm
