// lbm_stream.hip -- S-step register-streaming kernel (temporal blocking in
// registers, no LDS).
//
// One wave owns a strip of 64 consecutive columns (one cell per lane) and
// walks it row by row.  Each row of the input lattice is read from HBM once;
// as row j arrives, level 1 (step t+1) computes row j-1, level 2 computes
// row j-2 from level 1's rows, ..., level S writes row j-S of step t+S back
// to HBM.  The pull stencil needs, for level L at row y, level L-1's
//   row y+1: planes 4, 7 (from x+1), 8 (from x-1)   -- just produced
//   row y  : planes 0, 1 (from x-1), 3 (from x+1)   -- held one iteration
//   row y-1: planes 2, 5 (from x-1), 6 (from x+1)   -- held two iterations
// so between consecutive levels only nine registers per lane are live; the
// x-1 / x+1 neighbours come from the adjacent lane with a DPP wave shift
// (v_mov_b32_dpp wave_shr:1 / wave_shl:1), once per produced value.
//
// Every level loses one valid column at each wave edge, so a strip writes its
// middle 64 - 2S columns and neighbouring strips overlap by 2S columns
// (recomputed).  A strip is cut into segments of hs output rows; a segment
// streams hs + 2S input rows.  The lattice crosses HBM once per S steps: 72 B
// per cell per launch (+ the overlap re-reads) instead of per step.
//
// The per-cell arithmetic is collide() (lbm_device.hpp, LastChance.cpp:
// 226-262 in the same order), so the lattice is bitwise identical to S
// one-step launches and to the CPU oracle.  Cells outside the sub-domain are
// computed from the S-wide ghost ring and the ghosted obstacle map exactly as
// their owner computes them; values that are not needed (early iterations,
// lanes past the edges) may be garbage and never reach an owned cell.
//
// |u| of every level is summed over the cells the wave owns (each cell of
// each step counted once) and reduced per wave; the next reducing launch
// folds the S partials per wave in a fixed order (ctl protocol, lbm_layout.hpp).

#include "lbm_device.hpp"

namespace lbm {

__device__ __forceinline__ float from_left(float v) {  // lane - 1  (x - 1)
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138 /* wave_shr:1 */, 0xf, 0xf, false));
}
__device__ __forceinline__ float from_right(float v) {  // lane + 1  (x + 1)
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130 /* wave_shl:1 */, 0xf, 0xf, false));
}

__device__ __forceinline__ float stream_accel(const StreamArgs &a, int y) {
    int g = a.gy0 + y;
    g = g < 0 ? g + a.ny : (g >= a.ny ? g - a.ny : g);
    return (g == a.accel_g) ? 1.00f : 0.00f;
}

template <int S, bool kReduce>
__global__ __launch_bounds__(64) void stream_steps(StreamArgs a) {
    __shared__ float lds[1];
    if (kReduce && blockIdx.x == 0) reduce_pending_n<64>(a.ctl, a.partials_prev, a.av_local, lds);

    const int lane = threadIdx.x;
    const int t = xcd_remap(blockIdx.x, gridDim.x);
    float tot[S];
#pragma unroll
    for (int l = 0; l < S; ++l) tot[l] = 0.f;

    if (t < a.total) {
        const int r = rect_of(a.rect_begin, t);
        const SRect R = a.rect[r];
        const int lt = t - a.rect_begin[r];
        const int seg = lt / R.nstrip, strip = lt - seg * R.nstrip;
        const int x = R.x0 + strip * R.ow - S + lane;
        const bool own = lane >= S && lane < 64 - S && x < R.x0 + R.w;
        const int yo0 = R.y0 + seg * R.hs;
        const int yo1 = min(yo0 + R.hs, R.y0 + R.h);
        const int xc = min(x, a.xmax);
        const long long P = a.plane;
        const int pitch = a.pitch;
        const float *src = a.fin + xc;
        const uint8_t *obp = a.obst_g + (xc + a.og);
        const int jlast = yo1 + S - 1;

        // boundary b = values produced by level b for level b+1
        float c0[S], c1[S], c3[S];     // row r-1: planes 0, 1 (x-1), 3 (x+1)
        float a2[S], a5[S], a6[S];     // row r-1: planes 2, 5 (x-1), 6 (x+1)
        float b2[S], b5[S], b6[S];     // row r-2: same planes
#pragma unroll
        for (int b = 0; b < S; ++b) c0[b] = c1[b] = c3[b] = a2[b] = a5[b] = a6[b] = b2[b] = b5[b] = b6[b] = 0.f;
        unsigned obits = 0;  // bit L: obstacle at (x, j - L)

        int j = yo0 - S;
        float v[Q];
        unsigned vo;
        {
            const float *c = src + (long long)j * pitch;
#pragma unroll
            for (int k = 0; k < Q; ++k) v[k] = c[k * P];
            vo = obp[(long long)(j + a.og) * a.ogp];
        }
        for (; j <= jlast; ++j) {
            // prefetch row j+1 (clamped: the last iteration re-reads its own row)
            const int jn = min(j + 1, jlast);
            float nv[Q];
            const float *cn = src + (long long)jn * pitch;
#pragma unroll
            for (int k = 0; k < Q; ++k) nv[k] = cn[k * P];
            const unsigned nvo = obp[(long long)(jn + a.og) * a.ogp];

            obits = (obits << 1) | (vo != 0 ? 1u : 0u);
            float cur[Q];
#pragma unroll
            for (int k = 0; k < Q; ++k) cur[k] = v[k];
#pragma unroll
            for (int L = 1; L <= S; ++L) {
                const int b = L - 1;
                const int y = j - L;
                const float s[Q] = {c0[b],          c1[b], b2[b], c3[b], cur[4],
                                    b5[b],          b6[b], from_right(cur[7]), from_left(cur[8])};
                // rotate boundary b: rows r-1 -> r-2, r -> r-1
                b2[b] = a2[b];
                b5[b] = a5[b];
                b6[b] = a6[b];
                a2[b] = cur[2];
                a5[b] = from_left(cur[5]);
                a6[b] = from_right(cur[6]);
                c0[b] = cur[0];
                c1[b] = from_left(cur[1]);
                c3[b] = from_right(cur[3]);

                const bool ob = (obits >> L) & 1u;
                float o[Q];
                const float u = collide(s, o, ob, stream_accel(a, y), a.omega, a.omo, a.w1, a.w2);
                const bool live = own && y >= yo0 && y < yo1;
                if (live) tot[b] += u;
                if (L == S) {
                    if (live) {
                        float *w0 = a.fout + (long long)y * pitch + x;
#pragma unroll
                        for (int k = 0; k < Q; ++k) w0[k * P] = o[k];
                        // WG halo (g = S): all nine populations of the S outermost rows/columns
                        const bool east = x >= a.w - S, west = x < S, north = y >= a.h - S, south = y < S;
                        if (east) store2(a.dst[DE], x - (a.w - S), y, o);
                        if (west) store2(a.dst[DW], x, y, o);
                        if (north) {
                            store2(a.dst[DN], y - (a.h - S), x, o);
                            if (east) store2(a.dst[DNE], y - (a.h - S), x - (a.w - S), o);
                            if (west) store2(a.dst[DNW], y - (a.h - S), x, o);
                        }
                        if (south) {
                            store2(a.dst[DS], y, x, o);
                            if (west) store2(a.dst[DSW], y, x, o);
                            if (east) store2(a.dst[DSE], y, x - (a.w - S), o);
                        }
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < Q; ++k) cur[k] = o[k];
                }
            }
#pragma unroll
            for (int k = 0; k < Q; ++k) v[k] = nv[k];
            vo = nvo;
        }
    }

    // per-wave |u| sums, fixed tree order
#pragma unroll
    for (int l = 0; l < S; ++l) {
        float sum = tot[l];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) sum += __shfl_down(sum, off, 64);
        if (lane == 0) a.partials_out[(long long)l * a.stride + blockIdx.x] = sum;
    }
    if (kReduce && blockIdx.x == 0 && lane == 0) publish_pending(a.ctl, S, a.n_total, a.stride);
}

template <int S>
static void launch_s(const StreamArgs &a, int blocks, bool reduce, hipStream_t s) {
    if (reduce)
        hipLaunchKernelGGL((stream_steps<S, true>), dim3(blocks), dim3(64), 0, s, a);
    else
        hipLaunchKernelGGL((stream_steps<S, false>), dim3(blocks), dim3(64), 0, s, a);
}

hipError_t launch_stream(const StreamArgs &a, int blocks, int steps, bool reduce, hipStream_t s) {
    switch (steps) {
        case 2: launch_s<2>(a, blocks, reduce, s); break;
        case 3: launch_s<3>(a, blocks, reduce, s); break;
        case 4: launch_s<4>(a, blocks, reduce, s); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace lbm
