// lbm_resident2.hip -- the lattice-resident persistent kernel with a ghost
// ring TWO cells wide (v5): one neighbour hand-off per TWO time steps.
//
// v2 (lbm_resident.hip) exchanges a one-cell ring every step; at 1024^2 a
// step costs ~4.0 us (tolerance), ~1.5 us of it waiting for the neighbours'
// granules (their skew plus the hop).  Here each tile keeps a
// two-cell ring: step A advances the tile AND its inner ring (ring 1) from
// t to t+1, pulling from the outer ring (ring 2); step B advances the tile
// alone from t+1 to t+2, pulling from the ring-1 values step A produced;
// then the tiles hand off the two-deep bands their neighbours need and wait
// for theirs.  The wait is paid once per two steps, for ~6 % more collision
// work (ring 1) and three times the granules per hand-off.
//
// Geometry: 128 x 32 tiles (a column pair per work item, packed fp32
// collide2 / collide2t), 16 waves, two tile pairs per thread (2048); in
// step A threads 0..195 also advance one ring-1 item (2 x 64 row pairs,
// 2 x 34 column / corner cells; waves 0..3, one per SIMD), pulled with the
// tile pairs before the first barrier.  (A form that ran the ring as a third
// phase, after the tile, from a side buffer of the tile's edge values, held
// fewer registers but cost a barrier: 4.7 vs 4.4 us per step at 1024^2.)
// The step loop launders the item coordinates every step so the compiler
// does not hoist ~100 loop-invariant addresses (they spilled 80-90 VGPRs at
// the 128-VGPR cap of 16 waves).  LDS: populations 1..8 of the tile plus the
// two-cell ring (36 x 132 per plane, 152 KB), population 0 of the ring-1
// cells; population 0 of the tile in registers.
//
// Measured (profiles/r04/res5/): at 1024^2 v5 LOSES to v2 -- tolerance
// 4.4 vs 4.0 us per step, bitwise 5.3 vs 4.7; breakdown of the 4.4 us:
// ~3.0 us the collisions (17 wave-collisions per SIMD per two steps against
// v2's 16, plus the third barrier-free ring item), ~0.5 us publishing the
// 2 916 granules of a two-deep hand-off (global stores, agent scope), ~0.9 us
// waiting -- the wait per hand-off (~1.8 us) is not shorter than v2's, so
// halving the hand-offs saves less than the ring and the larger hand-off
// cost.  v5 stays an opt-in variant (LBM_RES_V=5, whole 128 x 32 tiles).
//
// What a tile needs from a neighbour (its ring cells r whose populations k
// move into the extended region [-1, tw] x [-1, th]: r + e_k inside it):
//   side ring, depth 1: six speeds (e.g. north row ly = th: cy <= 0 ->
//   0, 1, 3, 4, 7, 8); depth 2: three (north ly = th + 1: cy = -1 -> 4, 7, 8);
//   corner 2 x 2 blocks: 4 + 2 + 2 + 1 speeds.
// Each tile publishes those values from its own two-deep bands after step B
// as 8-byte {value, step-tag} granules (as v2: self-validating, no flags),
// double-buffered by hand-off parity: halo[2][ntiles][8 dirs][9][RES_GW].
// Semantics per cell are exactly the one-step kernels' (LastChance.cpp:
// 192-266 pull, rebound, collision, folded acceleration): bitwise equal to
// the oracle in bitwise mode, to the v2 tiles in tolerance mode.

#include "lbm_packed.hpp"

namespace lbm {

#ifndef R5_DBG
#define R5_DBG 0  // A/B breakdown builds (tools/build_variant.sh): 8 no poll, 32 no publish (timing only:
                  // the results are wrong); 2, 4 extra barriers
#endif
constexpr int R5_NW = 16;
constexpr int R5_NT = 64 * R5_NW;
constexpr int R5_TH = 32;
constexpr int R5_LS = RES2_TW + 4;          // columns -2 .. 129
constexpr int R5_PS = (R5_TH + 4) * R5_LS;  // rows -2 .. 33
constexpr int R5_MAXIT = 2;                 // tile pairs per thread: 64 x 32 / 1024
constexpr int R5_NRING = 2 * (RES2_TW / 2) + 2 * (R5_TH + 2);  // ring-1 items (196)
static_assert(R5_NRING <= R5_NT, "one ring-1 item per thread");

// speeds a tile needs from the neighbour across side d (its ring there),
// depth 1 (six) then depth 2 (three)
__device__ constexpr int R5_SIDE_K[4][9] = {
    {0, 2, 3, 4, 6, 7, 3, 6, 7},  // DE: lx = tw, tw + 1 (cx <= 0, cx = -1)
    {0, 1, 3, 4, 7, 8, 4, 7, 8},  // DN: ly = th, th + 1
    {0, 1, 2, 4, 5, 8, 1, 5, 8},  // DW: lx = -1, -2
    {0, 1, 2, 3, 5, 6, 2, 5, 6},  // DS: ly = -1, -2
};
// corner blocks, by the corner's direction (DNE, DNW, DSW, DSE): {ex, ey, k},
// ring cell at depth (ex, ey) from the tile's corner
__device__ constexpr int R5_CORNER[4][9][3] = {
    {{1, 1, 0}, {1, 1, 3}, {1, 1, 4}, {1, 1, 7}, {2, 1, 3}, {2, 1, 7}, {1, 2, 4}, {1, 2, 7}, {2, 2, 7}},
    {{1, 1, 0}, {1, 1, 1}, {1, 1, 4}, {1, 1, 8}, {2, 1, 1}, {2, 1, 8}, {1, 2, 4}, {1, 2, 8}, {2, 2, 8}},
    {{1, 1, 0}, {1, 1, 1}, {1, 1, 2}, {1, 1, 5}, {2, 1, 1}, {2, 1, 5}, {1, 2, 2}, {1, 2, 5}, {2, 2, 5}},
    {{1, 1, 0}, {1, 1, 2}, {1, 1, 3}, {1, 1, 6}, {2, 1, 3}, {2, 1, 6}, {1, 2, 2}, {1, 2, 6}, {2, 2, 6}},
};

__device__ __forceinline__ void r5_publish(unsigned long long *g, float v, unsigned tag) {
    const unsigned long long word = ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(v);
    // (a global-address-space store, not a flat one: the granule buffer is device memory)
    __hip_atomic_store((__attribute__((address_space(1))) unsigned long long *)g, word, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long r5_load(const unsigned long long *g) {
    return __hip_atomic_load((const __attribute__((address_space(1))) unsigned long long *)g, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
}

// a band row pair's entries J0 .. J0 + NJ - 1 of the receiver side KD's list
// (positions lx, lx + 1 of each entry's row of RES_GW granules)
template <int KD, int J0, int NJ>
__device__ __forceinline__ void r5_pub_row(unsigned long long *g, const f2 (&o)[Q], unsigned tag) {
#pragma unroll
    for (int j = J0; j < J0 + NJ; ++j) {
        r5_publish(g + j * RES_GW, o[R5_SIDE_K[KD][j]].x, tag);
        r5_publish(g + j * RES_GW + 1, o[R5_SIDE_K[KD][j]].y, tag);
    }
}
// a band column pair (one row): depth-1 entries from the edge column (the
// pair's right cell when RIGHT1), depth-2 entries from the other
template <int KD, bool RIGHT1>
__device__ __forceinline__ void r5_pub_col(unsigned long long *g, const f2 (&o)[Q], unsigned tag) {
#pragma unroll
    for (int j = 0; j < 9; ++j) {
        const f2 v = o[R5_SIDE_K[KD][j]];
        r5_publish(g + j * RES_GW, (j < 6) == RIGHT1 ? v.y : v.x, tag);
    }
}
// the receiver corner C's entries at depth EY from this pair's row; the
// pair's right cell holds depth ex == RX
template <int C, int EY, int RX>
__device__ __forceinline__ void r5_pub_corner(unsigned long long *g, const f2 (&o)[Q], unsigned tag) {
#pragma unroll
    for (int j = 0; j < 9; ++j)
        if (R5_CORNER[C][j][1] == EY) {
            const f2 v = o[R5_CORNER[C][j][2]];
            r5_publish(g + j, R5_CORNER[C][j][0] == RX ? v.y : v.x, tag);
        }
}

template <bool TOL>
__global__ __launch_bounds__(R5_NT) void resident_steps_r2(ResidentArgs a) {
    __shared__ __attribute__((aligned(16))) float L[8 * R5_PS];
    __shared__ float F0R[2][RES2_TW + 2];  // ring-1 rows, population 0: [0] ly = -1, [1] ly = th; index lx + 1
    __shared__ float F0C[2][R5_TH];        // ring-1 columns: [0] lx = -1, [1] lx = tw; index ly
    __shared__ float wsum[R5_NW];
    __shared__ int abort_flag;

    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int ntiles = a.tiles_x * a.tiles_y;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int tx = tile % a.tiles_x, ty = tile / a.tiles_x;
    const int gx0 = tx * RES2_TW, gy0 = ty * R5_TH;
    constexpr int tw = RES2_TW, th = R5_TH, npx = tw / 2;  // whole tiles only (the engine checks)
    const long long P = a.plane;
    const int pitch = a.pitch;
#define LK(k, ly, lx) (((k) - 1) * R5_PS + ((ly) + 2) * R5_LS + ((lx) + 2))
    if (threadIdx.x == 0) abort_flag = 0;

    // ---- work items -----------------------------------------------------------
    // tile pairs: the two-deep bands first (rows 0, 1, th-2, th-1; then the
    // pairs px = 0, npx-1 of the middle rows), so the populations a hand-off
    // carries are computed and published early in step B; then the interior
    constexpr int nband_rows = 4 * npx, mid = th - 4, nband_cols = 2 * mid;
    static_assert(nband_rows + nband_cols + (npx - 2) * mid == R5_MAXIT * R5_NT, "two tile pairs per thread");
    int ilx[R5_MAXIT], ily[R5_MAXIT];
    unsigned oa = 0, ob = 0, anyo = 0;
    f2 f0[R5_MAXIT];
    auto gobst = [&](int lx, int ly) -> bool {  // periodic obstacle lookup
        const int gx = ((gx0 + lx) % a.nx + a.nx) % a.nx, gy = ((gy0 + ly) % a.ny + a.ny) % a.ny;
        return a.obst[(long long)gy * a.nx + gx] != 0;
    };
#pragma unroll
    for (int it = 0; it < R5_MAXIT; ++it) {
        const int i = threadIdx.x + it * R5_NT;
        int lx, ly;
        if (i < nband_rows) {
            const int r = i / npx;
            lx = 2 * (i - r * npx);
            ly = r < 2 ? r : th - 4 + r;
        } else if (i < nband_rows + nband_cols) {
            const int j = i - nband_rows;
            lx = j < mid ? 0 : tw - 2;
            ly = 2 + (j < mid ? j : j - mid);
        } else {
            const int j = i - nband_rows - nband_cols;
            const int q = j / (npx - 2);
            lx = 2 * (1 + (j - q * (npx - 2)));
            ly = 2 + q;
        }
        ilx[it] = lx;
        ily[it] = ly;
        const float *src = a.fin + (long long)(gy0 + ly) * pitch + gx0 + lx;
        f0[it] = *reinterpret_cast<const f2 *>(src);
#pragma unroll
        for (int k = 1; k < Q; ++k)
            *reinterpret_cast<f2 *>(&L[LK(k, ly, lx)]) = *reinterpret_cast<const f2 *>(src + k * P);
        const bool o0 = gobst(lx, ly), o1 = gobst(lx + 1, ly);
        oa |= (unsigned)o0 << it;
        ob |= (unsigned)o1 << it;
        if (__ballot(o0 || o1) != 0) anyo |= 1u << it;  // wave-uniform
    }
    // ring-1 item of threads 0..195: row pairs (ly = -1, th), then column /
    // corner cells (lx = -1, tw; ly = -1 .. th)
    const bool has_ring0 = threadIdx.x < R5_NRING;
    int rlx = 0, rly = 0;
    if (threadIdx.x < 2 * npx) {
        rlx = 2 * (threadIdx.x % npx);
        rly = threadIdx.x < npx ? -1 : th;
    } else if (has_ring0) {
        const int j = threadIdx.x - 2 * npx;
        rlx = j < th + 2 ? -1 : tw;
        rly = (j < th + 2 ? j : j - (th + 2)) - 1;
    }
    const bool ro0 = has_ring0 && gobst(rlx, rly);
    const bool ro1 = has_ring0 && (threadIdx.x < 2 * npx ? gobst(rlx + 1, rly) : ro0);
    const bool anyr = __ballot(ro0 || ro1) != 0;
    // the two-cell ring: periodic images from the global lattice (planes
    // 1..8 everywhere in it, population 0 of ring 1)
    for (int i = threadIdx.x; i < 4 * (tw + 4) + 4 * th; i += R5_NT) {
        int lx, ly;
        if (i < 4 * (tw + 4)) {
            const int r = i / (tw + 4);
            lx = i - r * (tw + 4) - 2;
            ly = r < 2 ? r - 2 : th + r - 2;  // -2, -1, th, th + 1
        } else {
            const int j = i - 4 * (tw + 4), c = j / th;
            ly = j - c * th;
            lx = c < 2 ? c - 2 : tw + c - 2;  // -2, -1, tw, tw + 1
        }
        const int gx = ((gx0 + lx) % a.nx + a.nx) % a.nx;
        const int gy = ((gy0 + ly) % a.ny + a.ny) % a.ny;
        const float *src = a.fin + (long long)gy * pitch + gx;
#pragma unroll
        for (int k = 1; k < Q; ++k) L[LK(k, ly, lx)] = src[k * P];
        if (ly == -1 || ly == th) {
            if (lx >= -1 && lx <= tw) F0R[ly < 0 ? 0 : 1][lx + 1] = src[0];
        } else if ((lx == -1 || lx == tw) && ly >= 0 && ly < th) {  // (not the ring-2 rows' corners)
            F0C[lx < 0 ? 0 : 1][ly] = src[0];
        }
    }
    __syncthreads();

    // the step loop recomputes item addresses every step (opaque copies of
    // the coordinates and of the halo base): hoisted, the ~100 loop-invariant
    // LDS / global addresses of the pulls, the ring phase and the hand-off
    // spill (measured: 80-90 VGPRs spilled at the 128-VGPR cap of 16 waves)
    unsigned long long *halo_base = a.halo;
    int tid = threadIdx.x, tl = tile;
    auto launder = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int it = 0; it < R5_MAXIT; ++it) asm volatile("" : "+v"(ilx[it]), "+v"(ily[it]));
        asm volatile("" : "+v"(rlx), "+v"(rly), "+v"(tid));
        asm volatile("" : "+s"(halo_base), "+s"(tl));
    };
    auto gbase = [&](int slot, int tl, int d) -> unsigned long long * {
        return halo_base + (((long long)slot * ntiles + tl) * 8 + d) * (9 * RES_GW);
    };
    const TolK tk{a.omo, a.tc0, a.tc1, a.tc2};
    auto collide_pair = [&](const f2 (&s)[Q], f2 (&o)[Q], bool o_a, bool o_b, bool any, int gy) -> f2 {
        const bool accrow = gy == a.accel_row;
        if constexpr (TOL) {
            const f2 usq = collide2t(s, o, o_a, o_b, any, accrow, tk, a.w1, a.w2);
            return f2{o_a ? 0.f : sqrt_av(usq.x), o_b ? 0.f : sqrt_av(usq.y)} * mk2(TOL_USQ_ROOT);
        } else {
            return collide2(s, o, o_a, o_b, any, accrow ? 1.00f : 0.00f, a.omega, a.omo, a.w1, a.w2);
        }
    };
    auto pull_pair = [&](f2 (&s)[Q], int lx, int ly) {
        s[1] = f2{L[LK(1, ly, lx - 1)], L[LK(1, ly, lx)]};
        s[2] = *reinterpret_cast<const f2 *>(&L[LK(2, ly - 1, lx)]);
        s[3] = f2{L[LK(3, ly, lx + 1)], L[LK(3, ly, lx + 2)]};
        s[4] = *reinterpret_cast<const f2 *>(&L[LK(4, ly + 1, lx)]);
        s[5] = f2{L[LK(5, ly - 1, lx - 1)], L[LK(5, ly - 1, lx)]};
        s[6] = f2{L[LK(6, ly - 1, lx + 1)], L[LK(6, ly - 1, lx + 2)]};
        s[7] = f2{L[LK(7, ly + 1, lx + 1)], L[LK(7, ly + 1, lx + 2)]};
        s[8] = f2{L[LK(8, ly + 1, lx - 1)], L[LK(8, ly + 1, lx)]};
    };
    auto pull_single = [&](f2 (&r)[Q], int lx, int ly) {
        r[1] = mk2(L[LK(1, ly, lx - 1)]);
        r[2] = mk2(L[LK(2, ly - 1, lx)]);
        r[3] = mk2(L[LK(3, ly, lx + 1)]);
        r[4] = mk2(L[LK(4, ly + 1, lx)]);
        r[5] = mk2(L[LK(5, ly - 1, lx - 1)]);
        r[6] = mk2(L[LK(6, ly - 1, lx + 1)]);
        r[7] = mk2(L[LK(7, ly + 1, lx + 1)]);
        r[8] = mk2(L[LK(8, ly + 1, lx - 1)]);
    };
    const long long deadline_span = a.timeout_ticks;
    int t = 0;
    auto flush_partial = [&]() {  // step t - 1's tile sum (complete after the previous barrier)
        if (t > 0 && threadIdx.x == 0) {
            float sw = wsum[0];
#pragma unroll
            for (int i = 1; i < R5_NW; ++i) sw += wsum[i];
            a.partials[(long long)(t - 1) * ntiles + tile] = sw;
        }
    };
    auto finish_step = [&](float tot) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) tot += __shfl_down(tot, off, 64);
        if (lane == 0) wsum[wv] = tot;
    };

    // ---- step A: tile + ring 1, t -> t + 1 (no hand-off) ----------------------
    auto stepA = [&]() __attribute__((always_inline)) {
        launder();
        if (R5_DBG & 4) __syncthreads();
        flush_partial();
        f2 s[R5_MAXIT][Q];
#pragma unroll
        for (int it = 0; it < R5_MAXIT; ++it) {
            s[it][0] = f0[it];
            pull_pair(s[it], ilx[it], ily[it]);
        }
        // ring 1 (threads 0..195): the same pulls, from the ring and the tile's edges
        f2 r[Q];
        const bool ring_row = tid < 2 * npx, has_ring = tid < R5_NRING;
        if (ring_row) {
            const int yi = rly < 0 ? 0 : 1;
            r[0] = f2{F0R[yi][rlx + 1], F0R[yi][rlx + 2]};
            pull_pair(r, rlx, rly);
        } else if (has_ring) {
            r[0] = mk2((rly == -1 || rly == th) ? F0R[rly < 0 ? 0 : 1][rlx + 1] : F0C[rlx < 0 ? 0 : 1][rly]);
            pull_single(r, rlx, rly);
        }
        __syncthreads();
        float tot = 0.f;
#pragma unroll
        for (int it = 0; it < R5_MAXIT; ++it) {
            const int lx = ilx[it], ly = ily[it];
            f2 o[Q];
            const f2 u = collide_pair(s[it], o, (oa >> it) & 1u, (ob >> it) & 1u, (anyo >> it) & 1u, gy0 + ly);
            tot += u.x + u.y;
            f0[it] = o[0];
#pragma unroll
            for (int k = 1; k < Q; ++k) *reinterpret_cast<f2 *>(&L[LK(k, ly, lx)]) = o[k];
        }
        finish_step(tot);
        if (has_ring) {
            f2 o[Q];
            (void)collide_pair(r, o, ro0, ro1, anyr, ((gy0 + rly) % a.ny + a.ny) % a.ny);
            if (ring_row) {
                const int yi = rly < 0 ? 0 : 1;
                F0R[yi][rlx + 1] = o[0].x;
                F0R[yi][rlx + 2] = o[0].y;
#pragma unroll
                for (int k = 1; k < Q; ++k) *reinterpret_cast<f2 *>(&L[LK(k, rly, rlx)]) = o[k];
            } else {
                if (rly == -1 || rly == th)
                    F0R[rly < 0 ? 0 : 1][rlx + 1] = o[0].x;
                else
                    F0C[rlx < 0 ? 0 : 1][rly] = o[0].x;
#pragma unroll
                for (int k = 1; k < Q; ++k) L[LK(k, rly, rlx)] = o[k].x;
            }
        }
        __syncthreads();
        ++t;
    };

    // ---- step B: the tile, t + 1 -> t + 2; publish the bands; poll the ring ----
    auto stepB = [&]() __attribute__((always_inline)) -> bool {
        launder();
        if (R5_DBG & 4) __syncthreads();
        flush_partial();
        f2 s[R5_MAXIT][Q];
#pragma unroll
        for (int it = 0; it < R5_MAXIT; ++it) {
            s[it][0] = f0[it];
            pull_pair(s[it], ilx[it], ily[it]);
        }
        __syncthreads();
        const unsigned tag = a.tag0 + (unsigned)t + 1u;
        const int slot = (t >> 1) & 1;
        float tot = 0.f;
#pragma unroll
        for (int it = 0; it < R5_MAXIT; ++it) {
            const int lx = ilx[it], ly = ily[it];
            f2 o[Q];
            const f2 u = collide_pair(s[it], o, (oa >> it) & 1u, (ob >> it) & 1u, (anyo >> it) & 1u, gy0 + ly);
            tot += u.x + u.y;
            f0[it] = o[0];
#pragma unroll
            for (int k = 1; k < Q; ++k) *reinterpret_cast<f2 *>(&L[LK(k, ly, lx)]) = o[k];
            // the values of this pair's cells on the neighbours' rings (every
            // speed index a compile-time constant: a runtime index puts o[] in
            // scratch -- measured 3x slower steps)
            if (R5_DBG & 32) continue;
            if (ly == 0) r5_pub_row<DN, 0, 6>(gbase(slot, tl, DS) + lx, o, tag);  // -> the south neighbour's north ring
            if (ly == 1) r5_pub_row<DN, 6, 3>(gbase(slot, tl, DS) + lx, o, tag);
            if (ly == th - 1) r5_pub_row<DS, 0, 6>(gbase(slot, tl, DN) + lx, o, tag);  // -> the north neighbour's south ring
            if (ly == th - 2) r5_pub_row<DS, 6, 3>(gbase(slot, tl, DN) + lx, o, tag);
            if (lx == 0) {  // columns 0 (depth 1), 1 (depth 2) -> the west neighbour's east ring
                r5_pub_col<DE, false>(gbase(slot, tl, DW) + ly, o, tag);
                if (ly == 0) r5_pub_corner<0, 1, 2>(gbase(slot, tl, DSW), o, tag);  // -> the SW neighbour's NE corner
                if (ly == 1) r5_pub_corner<0, 2, 2>(gbase(slot, tl, DSW), o, tag);
                if (ly == th - 1) r5_pub_corner<3, 1, 2>(gbase(slot, tl, DNW), o, tag);  // -> the NW neighbour's SE corner
                if (ly == th - 2) r5_pub_corner<3, 2, 2>(gbase(slot, tl, DNW), o, tag);
            }
            if (lx == tw - 2) {  // columns tw-1 (depth 1), tw-2 (depth 2) -> the east neighbour's west ring
                r5_pub_col<DW, true>(gbase(slot, tl, DE) + ly, o, tag);
                if (ly == 0) r5_pub_corner<1, 1, 1>(gbase(slot, tl, DSE), o, tag);  // -> the SE neighbour's NW corner
                if (ly == 1) r5_pub_corner<1, 2, 1>(gbase(slot, tl, DSE), o, tag);
                if (ly == th - 1) r5_pub_corner<2, 1, 1>(gbase(slot, tl, DNE), o, tag);  // -> the NE neighbour's SW corner
                if (ly == th - 2) r5_pub_corner<2, 2, 1>(gbase(slot, tl, DNE), o, tag);
            }
        }
        // poll: waves 0..3 the sides, waves 4..7 the corners (the ring slots
        // are read only by the next step A, after the barrier below)
        if (R5_DBG & 2) __syncthreads();
        bool ok = true;
        const long long deadline = (long long)wall_clock64() + deadline_span;
        const int lane = tid & 63, wv = (R5_DBG & 8) ? 99 : __builtin_amdgcn_readfirstlane(tid >> 6);
        const int tx = tl % a.tiles_x, ty = tl / a.tiles_x;
        const int txe = tx + 1 == a.tiles_x ? 0 : tx + 1, txw = tx == 0 ? a.tiles_x - 1 : tx - 1;
        const int tyn = ty + 1 == a.tiles_y ? 0 : ty + 1, tys = ty == 0 ? a.tiles_y - 1 : ty - 1;
        if (wv < 4) {
            const int d = wv;  // DE, DN, DW, DS: this tile's ring side
            const int src = d == DE ? ty * a.tiles_x + txe : d == DN ? tyn * a.tiles_x + tx
                          : d == DW ? ty * a.tiles_x + txw : tys * a.tiles_x + tx;
            const unsigned long long *g = gbase(slot, src, OPP_DIR[d]);
            const int len = (d == DN || d == DS) ? tw : th;
            unsigned pending = 0;  // bit (q * 9 + j): position lane + 64 q, entry j
#pragma unroll
            for (int q = 0; q < 2; ++q)
                if (lane + 64 * q < len) pending |= 0x1ffu << (9 * q);
            float v[18];
            for (;;) {
                unsigned long long w[18];
#pragma unroll
                for (int q = 0; q < 2; ++q)
#pragma unroll
                    for (int j = 0; j < 9; ++j)
                        w[9 * q + j] = r5_load(g + j * RES_GW + min(lane + 64 * q, RES_GW - 1));
#pragma unroll
                for (int e = 0; e < 18; ++e)
                    if (((pending >> e) & 1u) && (unsigned)(w[e] >> 32) == tag) {
                        v[e] = __uint_as_float((unsigned)w[e]);
                        pending &= ~(1u << e);
                    }
                if (!pending) break;
                if ((long long)wall_clock64() > deadline) {
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (ok) {
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int p = lane + 64 * q;
                    if (p >= len) continue;
#pragma unroll
                    for (int j = 0; j < 9; ++j) {
                        const int k = R5_SIDE_K[d][j], e = j < 6 ? 1 : 2;
                        const int lx = d == DE ? tw - 1 + e : d == DW ? -e : p;
                        const int ly = d == DN ? th - 1 + e : d == DS ? -e : p;
                        if (k == 0) {
                            if (d == DN || d == DS) F0R[d == DS ? 0 : 1][lx + 1] = v[9 * q + j];
                            else F0C[d == DW ? 0 : 1][ly] = v[9 * q + j];
                        } else {
                            L[LK(k, ly, lx)] = v[9 * q + j];
                        }
                    }
                }
            }
        } else if (wv < 8 && lane < 9) {
            const int c = wv - 4;  // 0 DNE, 1 DNW, 2 DSW, 3 DSE: this tile's ring corner
            const int dx = (c == 0 || c == 3) ? 1 : -1, dy = c < 2 ? 1 : -1;
            const int src = (dy > 0 ? tyn : tys) * a.tiles_x + (dx > 0 ? txe : txw);
            const int cd = c == 0 ? DNE : c == 1 ? DNW : c == 2 ? DSW : DSE;
            const unsigned long long *g = gbase(slot, src, OPP_DIR[cd]) + lane;
            float v = 0.f;
            for (;;) {
                const unsigned long long w = r5_load(g);
                if ((unsigned)(w >> 32) == tag) {
                    v = __uint_as_float((unsigned)w);
                    break;
                }
                if ((long long)wall_clock64() > deadline) {
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (ok) {
                int ex = 1, ey = 1, k = 0;
#pragma unroll
                for (int j = 0; j < 9; ++j)
                    if (lane == j) {
                        ex = R5_CORNER[c][j][0];
                        ey = R5_CORNER[c][j][1];
                        k = R5_CORNER[c][j][2];
                    }
                const int lx = dx > 0 ? tw - 1 + ex : -ex, ly = dy > 0 ? th - 1 + ey : -ey;
                if (k == 0)
                    F0R[dy < 0 ? 0 : 1][lx + 1] = v;
                else
                    L[LK(k, ly, lx)] = v;
            }
        }
        finish_step(tot);
        if (!ok) {
            abort_flag = 1;
            __hip_atomic_store(a.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        ++t;
        return !abort_flag;
    };

    while (t < a.steps) {
        stepA();
        if (t >= a.steps) break;  // odd step count: the last step is an A step
        if (!stepB()) break;
    }
    if (t == a.steps && a.steps > 0 && threadIdx.x == 0) {
        float sw = wsum[0];
#pragma unroll
        for (int i = 1; i < R5_NW; ++i) sw += wsum[i];
        a.partials[(long long)(a.steps - 1) * ntiles + tile] = sw;
    }
#pragma unroll
    for (int it = 0; it < R5_MAXIT; ++it) {
        float *dst = a.fout + (long long)(gy0 + ily[it]) * pitch + gx0 + ilx[it];
        *reinterpret_cast<f2 *>(dst) = f0[it];
#pragma unroll
        for (int k = 1; k < Q; ++k)
            *reinterpret_cast<f2 *>(dst + k * P) = *reinterpret_cast<const f2 *>(&L[LK(k, ily[it], ilx[it])]);
    }
#undef LK
}

const void *resident_kernel_r2(bool tol, int &threads) {
    threads = R5_NT;
    return tol ? reinterpret_cast<const void *>(&resident_steps_r2<true>)
               : reinterpret_cast<const void *>(&resident_steps_r2<false>);
}

}  // namespace lbm
