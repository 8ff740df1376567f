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

template <int T2W, int T2H, bool kReduce>
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

// --------------------------------------------------------------------------
// v2: one wave per tile row (TW = 64 = wave width), WR waves per workgroup,
// TH rows per tile.  Phase 1 computes the tile's own cells with the same
// lane -> column mapping phase 2 uses, so the rest population (plane 0) and
// the x-only planes 1 and 3 stay in registers and reach their phase-2
// consumer by a cross-lane shuffle; only planes 2,4,5,6,7,8 (and the halo
// column's planes 1/3) go through LDS.  The halo ring is a separate pass.
// LDS per block = 6 x (TH+2) x 66 floats: 28.5 KB at TH = 16.
// --------------------------------------------------------------------------
template <int TH, int WR, bool kReduce>
__global__ __launch_bounds__(64 * WR) void step2w(Step2Args a) {
    constexpr int TW = 64, MW = TW + 2, MH = TH + 2, NT = 64 * WR, RPW = TH / WR;
    static_assert(TH % WR == 0, "rows per wave");
    // LDS slots for planes 2,4,5,6,7,8
    __shared__ float mid[6][MH][MW];
    __shared__ float e1[TH], e3[TH];  // plane 1 of the left / plane 3 of the right halo column
    __shared__ float lds[WR];
    if (kReduce && blockIdx.x == 0) reduce_pending_n<NT>(a.ctl, a.partials_prev, a.av_local, lds);

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
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
        const int X0 = tx * TW, Y0 = ty * TH;
        const int x = X0 + lane;

        // ---- phase 1a: step t+1 on the tile's own cells ----
        float k0[RPW], k1[RPW], k3[RPW];
#pragma unroll
        for (int q = 0; q < RPW; ++q) {
            const int ly = wv + q * WR;
            const int y = Y0 + ly;
            k0[q] = k1[q] = k3[q] = 0.f;
            if (x <= a.w && y <= a.h) {
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
                k0[q] = o[0];
                k1[q] = o[1];
                k3[q] = o[3];
                mid[0][ly + 1][lane + 1] = o[2];
                mid[1][ly + 1][lane + 1] = o[4];
                mid[2][ly + 1][lane + 1] = o[5];
                mid[3][ly + 1][lane + 1] = o[6];
                mid[4][ly + 1][lane + 1] = o[7];
                mid[5][ly + 1][lane + 1] = o[8];
                if (x < a.w && y < a.h) tot1 += u;
            }
        }
        // ---- phase 1b: the one-cell halo ring around the tile ----
        constexpr int RING = 2 * MH + 2 * TW;
        for (int i = tid; i < RING; i += NT) {
            int lx, ly;
            if (i < MH) { lx = 0; ly = i; }
            else if (i < 2 * MH) { lx = MW - 1; ly = i - MH; }
            else if (i < 2 * MH + TW) { lx = i - 2 * MH + 1; ly = 0; }
            else { lx = i - 2 * MH - TW + 1; ly = MH - 1; }
            const int hx = X0 + lx - 1, hy = Y0 + ly - 1;
            if (hx > a.w || hy > a.h) continue;
            const float *c = a.fin + (long long)hy * pitch + hx;
            const float s[Q] = {c[0],
                                c[1 * P - 1],
                                c[2 * P - pitch],
                                c[3 * P + 1],
                                c[4 * P + pitch],
                                c[5 * P - pitch - 1],
                                c[6 * P - pitch + 1],
                                c[7 * P + pitch + 1],
                                c[8 * P + pitch - 1]};
            const bool ob = a.obst_g[(long long)(hy + 1) * a.ogp + (hx + 1)] != 0;
            float o[Q];
            (void)collide(s, o, ob, accel_flag(a, hy), a.omega, a.omo, a.w1, a.w2);
            mid[0][ly][lx] = o[2];
            mid[1][ly][lx] = o[4];
            mid[2][ly][lx] = o[5];
            mid[3][ly][lx] = o[6];
            mid[4][ly][lx] = o[7];
            mid[5][ly][lx] = o[8];
            if (ly >= 1 && ly <= TH) {
                if (lx == 0) e1[ly - 1] = o[1];
                if (lx == MW - 1) e3[ly - 1] = o[3];
            }
        }
        __syncthreads();

        // ---- phase 2: step t+2 on the tile ----
#pragma unroll
        for (int q = 0; q < RPW; ++q) {
            const int ly = wv + q * WR;
            const int y = Y0 + ly;
            const int my = ly + 1, mx = lane + 1;
            float s1 = __shfl_up(k1[q], 1, 64);    // plane 1 from x-1
            float s3 = __shfl_down(k3[q], 1, 64);  // plane 3 from x+1
            if (lane == 0) s1 = e1[ly];
            if (lane == 63) s3 = e3[ly];
            if (x >= a.w || y >= a.h) continue;
            const float s[Q] = {k0[q],
                                s1,
                                mid[0][my - 1][mx],
                                s3,
                                mid[1][my + 1][mx],
                                mid[2][my - 1][mx - 1],
                                mid[3][my - 1][mx + 1],
                                mid[4][my + 1][mx + 1],
                                mid[5][my + 1][mx - 1]};
            const bool ob = a.obst_g[(long long)(y + 1) * a.ogp + (x + 1)] != 0;
            float o[Q];
            tot2 += collide(s, o, ob, accel_flag(a, y), a.omega, a.omo, a.w1, a.w2);
            float *w0 = a.fout + (long long)y * pitch + x;
#pragma unroll
            for (int k = 0; k < Q; ++k) w0[k * P] = o[k];

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

    const float s1 = block_sum_n<WR>(tot1, lds);
    const float s2 = block_sum_n<WR>(tot2, lds);
    if (threadIdx.x == 0) {
        a.partials_out[blockIdx.x] = s1;
        a.partials_out[(long long)a.stride + blockIdx.x] = s2;
        if (kReduce && blockIdx.x == 0) publish_pending(a.ctl, 2, a.n_total, a.stride);
    }
}

template <int TW, int TH>
static void launch_tile(const Step2Args &a, int blocks, bool reduce, hipStream_t s) {
    if (reduce)
        hipLaunchKernelGGL((step2<TW, TH, true>), dim3(blocks), dim3(BLOCK), 0, s, a);
    else
        hipLaunchKernelGGL((step2<TW, TH, false>), dim3(blocks), dim3(BLOCK), 0, s, a);
}

template <int TH, int WR>
static void launch_w(const Step2Args &a, int blocks, bool reduce, hipStream_t s) {
    if (reduce)
        hipLaunchKernelGGL((step2w<TH, WR, true>), dim3(blocks), dim3(64 * WR), 0, s, a);
    else
        hipLaunchKernelGGL((step2w<TH, WR, false>), dim3(blocks), dim3(64 * WR), 0, s, a);
}

// Tile shapes offered (Tile2 in lbm_layout.hpp); the engine picks one at create.
hipError_t launch_step2(const Step2Args &a, int blocks, bool reduce, hipStream_t s) {
    switch (a.tile) {
        case T2V_64x8_W8: launch_w<8, 8>(a, blocks, reduce, s); break;
        case T2_64x8: launch_tile<64, 8>(a, blocks, reduce, s); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace lbm
