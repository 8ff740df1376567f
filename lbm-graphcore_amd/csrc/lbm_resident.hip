// lbm_resident.hip -- lattice-resident persistent kernel: every time step of a
// run in ONE launch, the lattice held on chip (LDS + registers) throughout.
//
// Why: the reference's 1024x1024 problem (BASELINE config 2) has 1 M cells --
// 37.7 MB of populations, which fits in the 256 CUs' 40 MB of LDS.  A
// per-step (or per-2-step) launch pays a kernel boundary (~1.5-2 us) and a
// trip of the lattice through L2/MALL every launch; here each CU keeps its
// tile resident and only the populations that cross a tile edge move,
// through L2, between neighbouring workgroups.  This replaces the IPU design
// where each tile keeps its cells in its own SRAM and exchanges halos every
// step (main/LbmAoS.cpp:135-372, BSP exchange of stitched halo views).
//
// Geometry: one workgroup per tile of 64 columns x TH = NW*R rows (NW waves,
// one column per lane, R consecutive rows per lane), tiles in row-major
// order over the grid (ragged last tiles allowed).  All tiles must be
// co-resident: the engine launches cooperatively and only when the occupancy
// query admits the whole grid.
//
// Per tile, per step t (pull streaming, LastChance.cpp:192-266 semantics):
//   LDS holds populations 1..8 of the tile plus a one-cell ring, population 0
//   and the obstacle bits stay in registers.
//   1. pull: each lane reads its cells' nine pulled populations from LDS;
//   2. barrier;
//   3. collide (lbm_device.hpp collide(): the exact reference expression
//      order -> bitwise equal to the CPU oracle), write the outputs back to
//      the cell's own LDS slots; populations leaving the tile are also
//      published to global memory as 8-byte {value, tag} granules (one sc1
//      store each; the tag is the step number, so a granule validates itself
//      and needs no flag, fence or barrier -- MI355X_MICROARCH.md
//      "handoff-1to1");
//   4. four waves poll the granules of the eight neighbour tiles for step t
//      and write them into the LDS ring;
//   5. barrier.
// Granules are double-buffered by step parity: a tile can only publish step
// t+2 after receiving its neighbours' step t+1, which they publish after
// reading its step t -- so a slot is never overwritten before it is read.
// Every poll is bounded by a wall-clock deadline: on timeout the tile sets a
// status word and all tiles drain out (neighbours then time out in turn), so
// a residency failure ends the launch instead of hanging the GPU.
//
// |u| per step: per-wave tree sums -> per-tile partial (fixed order) ->
// partials[t][tile]; resident_reduce folds the tiles in a fixed order into
// av_local[t] after the launch.

#include "lbm_packed.hpp"

namespace lbm {

constexpr int RES_LS = RES_TW + 2;  // LDS row stride (ring column on both sides)

__device__ __forceinline__ void publish(unsigned long long *g, float v, unsigned tag) {
    const unsigned long long word = ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(v);
    __hip_atomic_store(g, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ float rdlane(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// Fetch one ring side of step `tag`: positions p = lane + 64 j (j < NPOS,
// p < len) x the three planes at g[i * RES_GW + p], plus one corner granule
// cg on lanes that pass one.  Every round issues all outstanding loads back
// to back (one memory round trip per round, not one per granule) and
// re-polls only the granules whose tag is not there yet.  v[j * 3 + i] /
// v[3 * NPOS] receive the values; false on deadline, or as soon as another tile
// has reported a timeout in *status (the whole grid then drains within one
// poll round instead of one deadline per ring of neighbours).

template <int NPOS>
__device__ __forceinline__ bool fetch_ring(const unsigned long long *g, int len, const unsigned long long *cg,
                                           unsigned tag, long long deadline, const int *status,
                                           float (&v)[3 * NPOS + 1]) {
    constexpr int N = 3 * NPOS + 1;
    const int lane = threadIdx.x & 63;
    unsigned pending = 0;
#pragma unroll
    for (int j = 0; j < NPOS; ++j)
        if (lane + 64 * j < len) pending |= 7u << (3 * j);
    if (cg) pending |= 1u << (N - 1);
    const unsigned long long *c = cg ? cg : g;
    for (;;) {
        unsigned long long w[N];
#pragma unroll
        for (int j = 0; j < NPOS; ++j)
#pragma unroll
            for (int i = 0; i < 3; ++i)
                w[3 * j + i] = __hip_atomic_load(g + i * RES_GW + lane + 64 * j, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
        w[N - 1] = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int q = 0; q < N; ++q)
            if (((pending >> q) & 1u) && (unsigned)(w[q] >> 32) == tag) {
                v[q] = __uint_as_float((unsigned)w[q]);
                pending &= ~(1u << q);
            }
        if (!pending) return true;
        if ((long long)wall_clock64() > deadline) return false;
        if (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
        __builtin_amdgcn_s_sleep(1);
    }
}

template <int NW, int R>
__global__ __launch_bounds__(64 * NW) void resident_steps(ResidentArgs a) {
    constexpr int TH = NW * R;
    constexpr int LS = RES_LS;
    constexpr int PS = (TH + 2) * LS;  // LDS plane stride (planes 1..8)
    __shared__ float L[8 * PS];
    __shared__ float wsum[NW];
    __shared__ int abort_flag;

    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int ntiles = a.tiles_x * a.tiles_y;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);  // row-major neighbours share an XCD's L2
    const int tx = tile % a.tiles_x, ty = tile / a.tiles_x;
    const int gx0 = tx * RES_TW, gy0 = ty * TH;
    const int tw = min(RES_TW, a.nx - gx0), th = min(TH, a.ny - gy0);
    const int txe = tx + 1 == a.tiles_x ? 0 : tx + 1, txw = tx == 0 ? a.tiles_x - 1 : tx - 1;
    const int tyn = ty + 1 == a.tiles_y ? 0 : ty + 1, tys = ty == 0 ? a.tiles_y - 1 : ty - 1;
    const long long P = a.plane;
    const int pitch = a.pitch;
    // LDS slot of speed k (1..8) at local cell (lx, ly), -1 <= lx <= tw, -1 <= ly <= th
#define LI(k, ly, lx) (((k) - 1) * PS + ((ly) + 1) * LS + ((lx) + 1))

    if (threadIdx.x == 0) abort_flag = 0;

    // ---- load the tile and its ring from the global lattice ----------------
    float f0[R];
    unsigned obits = 0, active = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int ly = wv * R + r;
        f0[r] = 0.f;
        if (lane < tw && ly < th) {
            active |= 1u << r;
            const int gx = gx0 + lane, gy = gy0 + ly;
            const float *src = a.fin + (long long)gy * pitch + gx;
            f0[r] = src[0];
#pragma unroll
            for (int k = 1; k < Q; ++k) L[LI(k, ly, lane)] = src[k * P];
            if (a.obst[(long long)gy * a.nx + gx]) obits |= 1u << r;
        }
    }
    // ring cells: periodic images straight from the global lattice
    for (int side = wv; side < 4; side += NW) {
        const int len = side < 2 ? tw : th;
        for (int i = lane; i < len + 2; i += 64) {
            const int p = i - 1;  // -1 .. len
            int lx, ly;
            if (side == 0) { lx = p; ly = -1; }
            else if (side == 1) { lx = p; ly = th; }
            else if (side == 2) { lx = -1; ly = p; }
            else { lx = tw; ly = p; }
            if (side >= 2 && (p < 0 || p >= len)) continue;  // corners done by the row sides
            const int gx = ((gx0 + lx) % a.nx + a.nx) % a.nx;
            const int gy = ((gy0 + ly) % a.ny + a.ny) % a.ny;
            const float *src = a.fin + (long long)gy * pitch + gx;
#pragma unroll
            for (int k = 1; k < Q; ++k) L[LI(k, ly, lx)] = src[k * P];
        }
    }
    __syncthreads();

    // granule base of (slot, tile, direction): [2][ntiles][8][3][RES_GW]
    auto gbase = [&](int slot, int tl, int d) -> unsigned long long * {
        return a.halo + (((long long)slot * ntiles + tl) * 8 + d) * (3 * RES_GW);
    };
    const long long deadline_span = a.timeout_ticks;
    int t = 0;
    for (; t < a.steps; ++t) {
        if (tile == a.stall_tile && t == a.stall_step) break;  // debug: a tile that stops publishing
        const bool tr = a.trace && tile == 0 && threadIdx.x == 0 && t < a.trace_steps;
        if (tr) a.trace[t * 5 + 0] = (long long)wall_clock64();
        if (t > 0 && threadIdx.x == 0) {
            float s = wsum[0];
#pragma unroll
            for (int i = 1; i < NW; ++i) s += wsum[i];
            a.partials[(long long)(t - 1) * ntiles + tile] = s;
        }
        // 1. pull
        float s[R][Q];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int ly = wv * R + r, lx = lane;
            if ((active >> r) & 1u) {
                s[r][0] = f0[r];
                s[r][1] = L[LI(1, ly, lx - 1)];
                s[r][2] = L[LI(2, ly - 1, lx)];
                s[r][3] = L[LI(3, ly, lx + 1)];
                s[r][4] = L[LI(4, ly + 1, lx)];
                s[r][5] = L[LI(5, ly - 1, lx - 1)];
                s[r][6] = L[LI(6, ly - 1, lx + 1)];
                s[r][7] = L[LI(7, ly + 1, lx + 1)];
                s[r][8] = L[LI(8, ly + 1, lx - 1)];
            } else {
#pragma unroll
                for (int k = 0; k < Q; ++k) s[r][k] = 0.f;
            }
        }
        __syncthreads();
        if (tr) a.trace[t * 5 + 1] = (long long)wall_clock64();
        // 2. collide, write back, publish the leaving populations
        const unsigned tag = a.tag0 + (unsigned)t + 1u;
        const int slot = t & 1;
        float tot = 0.f;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (!((active >> r) & 1u)) continue;
            const int ly = wv * R + r, lx = lane;
            const int gy = gy0 + ly;
            float o[Q];
            const float accf = (gy == a.accel_row) ? 1.00f : 0.00f;
            tot += collide(s[r], o, (obits >> r) & 1u, accf, a.omega, a.omo, a.w1, a.w2);
            f0[r] = o[0];
#pragma unroll
            for (int k = 1; k < Q; ++k) L[LI(k, ly, lx)] = o[k];
            if (ly == th - 1) {  // leaving north: 2, 5, 6
                unsigned long long *g = gbase(slot, tile, DN);
                publish(g + lx, o[2], tag);
                publish(g + RES_GW + lx, o[5], tag);
                publish(g + 2 * RES_GW + lx, o[6], tag);
                if (lx == tw - 1) publish(gbase(slot, tile, DNE), o[5], tag);
                if (lx == 0) publish(gbase(slot, tile, DNW), o[6], tag);
            }
            if (ly == 0) {       // leaving south: 4, 7, 8
                unsigned long long *g = gbase(slot, tile, DS);
                publish(g + lx, o[4], tag);
                publish(g + RES_GW + lx, o[7], tag);
                publish(g + 2 * RES_GW + lx, o[8], tag);
                if (lx == 0) publish(gbase(slot, tile, DSW), o[7], tag);
                if (lx == tw - 1) publish(gbase(slot, tile, DSE), o[8], tag);
            }
            if (lx == tw - 1) {  // leaving east: 1, 5, 8
                unsigned long long *g = gbase(slot, tile, DE);
                publish(g + ly, o[1], tag);
                publish(g + RES_GW + ly, o[5], tag);
                publish(g + 2 * RES_GW + ly, o[8], tag);
            }
            if (lx == 0) {       // leaving west: 3, 6, 7
                unsigned long long *g = gbase(slot, tile, DW);
                publish(g + ly, o[3], tag);
                publish(g + RES_GW + ly, o[6], tag);
                publish(g + 2 * RES_GW + ly, o[7], tag);
            }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) tot += __shfl_down(tot, off, 64);
        if (lane == 0) wsum[wv] = tot;
        if (tr) a.trace[t * 5 + 2] = (long long)wall_clock64();
        // 3. the neighbours' step-t populations into the ring
        //    side 0: south ring row <- tile below, its north edge (2, 5, 6)
        //    side 1: north ring row <- tile above, its south edge (4, 7, 8)
        //    side 2: west ring column <- tile left, its east edge (1, 5, 8)
        //    side 3: east ring column <- tile right, its west edge (3, 6, 7)
        //    corners (one population each) ride with the row sides: below-left
        //    sends NE (5), below-right NW (6), above-left SE (8), above-right SW (7)
        bool ok = true;
        const long long deadline = (long long)wall_clock64() + deadline_span;
        for (int side = wv; side < 4; side += NW) {
            const int len = side < 2 ? tw : th;
            const int src_tile = side == 0 ? tys * a.tiles_x + tx
                               : side == 1 ? tyn * a.tiles_x + tx
                               : side == 2 ? ty * a.tiles_x + txw
                                           : ty * a.tiles_x + txe;
            const int d = side == 0 ? DN : side == 1 ? DS : side == 2 ? DE : DW;
            const bool corner = side < 2 && lane < 2, left = lane == 0;
            const int cd = side == 0 ? (left ? DNE : DNW) : (left ? DSE : DSW);
            const unsigned long long *cg =
                corner ? gbase(slot, (side == 0 ? tys : tyn) * a.tiles_x + (left ? txw : txe), cd) : nullptr;
            float v[4];
            ok = ok && fetch_ring<1>(gbase(slot, src_tile, d), len, cg, tag, deadline, a.status, v);
            const int p = lane;
            if (p < len) {
                const int lx = side < 2 ? p : (side == 2 ? -1 : tw);
                const int ly = side >= 2 ? p : (side == 0 ? -1 : th);
#pragma unroll
                for (int i = 0; i < 3; ++i) L[LI(PLANES[d][i], ly, lx)] = v[i];
            }
            if (corner) L[LI(PLANES[cd][0], side == 0 ? -1 : th, left ? -1 : tw)] = v[3];
        }
        if (tr) a.trace[t * 5 + 3] = (long long)wall_clock64();
        if (!ok) {
            abort_flag = 1;
            __hip_atomic_store(a.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (tr) a.trace[t * 5 + 4] = (long long)wall_clock64();
        if (abort_flag) break;
    }
    if (t == a.steps && a.steps > 0 && threadIdx.x == 0) {
        float s = wsum[0];
#pragma unroll
        for (int i = 1; i < NW; ++i) s += wsum[i];
        a.partials[(long long)(a.steps - 1) * ntiles + tile] = s;
    }

    // ---- final state back to the global lattice ----------------------------
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (!((active >> r) & 1u)) continue;
        const int ly = wv * R + r, lx = lane;
        float *dst = a.fout + (long long)(gy0 + ly) * pitch + gx0 + lx;
        dst[0] = f0[r];
#pragma unroll
        for (int k = 1; k < Q; ++k) dst[k * P] = L[LI(k, ly, lx)];
    }
#undef LI
}

// ---------------------------------------------------------------------------
// v2: packed fp32, one column PAIR per work item (collide2, lbm_packed.hpp),
// 128-column tiles (even nx).  Work items are listed boundary first -- the
// tile's bottom and top rows, then its left and right column pairs, then the
// interior -- and dealt round-robin to the threads, so the populations that
// leave the tile are computed and published in the first half of the
// collision phase and the hop to the neighbours overlaps the interior work.
// LDS rows hold 132 floats (ring column at x = -1 and x = tw, pairs 8-byte
// aligned): the unshifted pulls (N, S) are one ds_read_b64, the shifted ones
// one ds_read2_b32, every write-back one ds_write_b64.
// ---------------------------------------------------------------------------
// TOL: the LBM_FLAG_TOLERANCE collision (collide2t, lbm_packed.hpp) instead
// of the bitwise one -- same tiles, granules and schedule.
template <int NW, int TH, int MINW = 1, bool TOL = false>
__global__ __launch_bounds__(64 * NW, MINW) void resident_steps2(ResidentArgs a) {
    constexpr int NT = 64 * NW;
    constexpr int LS = RES2_TW + 4;
    constexpr int PS = (TH + 2) * LS;
    constexpr int MAXIT = (64 * TH + NT - 1) / NT;
    __shared__ __attribute__((aligned(16))) float L[8 * PS];
    __shared__ float wsum[NW];
    __shared__ int abort_flag;

    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int ntiles = a.tiles_x * a.tiles_y;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int tx = tile % a.tiles_x, ty = tile / a.tiles_x;
    const int gx0 = tx * RES2_TW, gy0 = ty * TH;
    const int tw = min(RES2_TW, a.nx - gx0), th = min(TH, a.ny - gy0);  // tw even
    const int npx = tw >> 1;
    const int txe = tx + 1 == a.tiles_x ? 0 : tx + 1, txw = tx == 0 ? a.tiles_x - 1 : tx - 1;
    const int tyn = ty + 1 == a.tiles_y ? 0 : ty + 1, tys = ty == 0 ? a.tiles_y - 1 : ty - 1;
    const long long P = a.plane;
    const int pitch = a.pitch;
#define LJ(k, ly, lx) (((k) - 1) * PS + ((ly) + 1) * LS + ((lx) + 2))
    // pair at (ly, lx .. lx + 1) of plane k; al: lx even (one 8-byte access)
#define LD2(k, ly, lx, al) \
    ((al) ? *reinterpret_cast<const f2 *>(&L[LJ(k, ly, lx)]) : f2{L[LJ(k, ly, lx)], L[LJ(k, ly, (lx) + 1)]})
#define ST2(k, ly, lx, al, v)                                    \
    do {                                                         \
        if (al) {                                                \
            *reinterpret_cast<f2 *>(&L[LJ(k, ly, lx)]) = (v);    \
        } else {                                                 \
            L[LJ(k, ly, lx)] = (v).x;                            \
            L[LJ(k, ly, (lx) + 1)] = (v).y;                      \
        }                                                        \
    } while (0)
    if (threadIdx.x == 0) abort_flag = 0;

    // ---- work items: boundary first ----------------------------------------
    const int nrow = th > 1 ? 2 * npx : npx;
    const int m = th > 2 ? th - 2 : 0;
    const int ncol = npx >= 2 ? 2 * m : m;
    const int nin = npx >= 3 ? (npx - 2) * m : 0;
    const int total = nrow + ncol + nin;
    int lxs[MAXIT], lys[MAXIT];
    unsigned valid = 0, oa = 0, ob = 0, anyo = 0;
    f2 f0[MAXIT];
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) {
        const int i = threadIdx.x + it * NT;
        int px = 0, ly = 0;
        if (i < total) {
            valid |= 1u << it;
            if (i < nrow) {
                px = i < npx ? i : i - npx;
                ly = i < npx ? 0 : th - 1;
            } else if (i < nrow + ncol) {
                const int j = i - nrow;
                px = j < m ? 0 : npx - 1;
                ly = 1 + (j < m ? j : j - m);
            } else {
                const int j = i - nrow - ncol;
                const int q = j / (npx - 2);
                px = 1 + (j - q * (npx - 2));
                ly = 1 + q;
            }
        }
        lxs[it] = 2 * px;
        lys[it] = ly;
        f0[it] = mk2(0.f);
        bool o0 = false, o1 = false;
        if ((valid >> it) & 1u) {
            const int gx = gx0 + 2 * px, gy = gy0 + ly;
            const float *src = a.fin + (long long)gy * pitch + gx;
            f0[it] = *reinterpret_cast<const f2 *>(src);
#pragma unroll
            for (int k = 1; k < Q; ++k)
                *reinterpret_cast<f2 *>(&L[LJ(k, ly, 2 * px)]) = *reinterpret_cast<const f2 *>(src + k * P);
            const uint8_t *ob8 = a.obst + (long long)gy * a.nx + gx;
            o0 = ob8[0] != 0;
            o1 = ob8[1] != 0;
        }
        oa |= (unsigned)o0 << it;
        ob |= (unsigned)o1 << it;
        if (__ballot(o0 || o1) != 0) anyo |= 1u << it;  // wave-uniform
    }
    // ring cells: periodic images from the global lattice
    for (int side = wv; side < 4; side += NW) {
        const int len = side < 2 ? tw : th;
        for (int i = lane; i < len + 2; i += 64) {
            const int p = i - 1;
            if (side >= 2 && (p < 0 || p >= len)) continue;
            const int lx = side == 0 || side == 1 ? p : (side == 2 ? -1 : tw);
            const int ly = side == 2 || side == 3 ? p : (side == 0 ? -1 : th);
            const int gx = ((gx0 + lx) % a.nx + a.nx) % a.nx;
            const int gy = ((gy0 + ly) % a.ny + a.ny) % a.ny;
            const float *src = a.fin + (long long)gy * pitch + gx;
#pragma unroll
            for (int k = 1; k < Q; ++k) L[LJ(k, ly, lx)] = src[k * P];
        }
    }
    __syncthreads();

    auto gbase = [&](int slot, int tl, int d) -> unsigned long long * {
        return a.halo + (((long long)slot * ntiles + tl) * 8 + d) * (3 * RES_GW);
    };
    const long long deadline_span = a.timeout_ticks;
    int t = 0;
    // one time step of the tile; returns false on abort
    auto step = [&]() __attribute__((always_inline)) -> bool {
        const bool tr = a.trace && tile == 0 && threadIdx.x == 0 && t < a.trace_steps;
        if (tr) a.trace[t * 5 + 0] = (long long)wall_clock64();
        if (t > 0 && threadIdx.x == 0) {
            float sw = wsum[0];
#pragma unroll
            for (int i = 1; i < NW; ++i) sw += wsum[i];
            a.partials[(long long)(t - 1) * ntiles + tile] = sw;
        }
        // 1. pull
        f2 s[MAXIT][Q];
#pragma unroll
        for (int it = 0; it < MAXIT; ++it) {
            if (!((valid >> it) & 1u)) {
#pragma unroll
                for (int k = 0; k < Q; ++k) s[it][k] = mk2(0.f);
                continue;
            }
            const int lx = lxs[it], ly = lys[it];
            s[it][0] = f0[it];
            s[it][1] = f2{L[LJ(1, ly, lx - 1)], L[LJ(1, ly, lx)]};
            s[it][2] = *reinterpret_cast<const f2 *>(&L[LJ(2, ly - 1, lx)]);
            s[it][3] = f2{L[LJ(3, ly, lx + 1)], L[LJ(3, ly, lx + 2)]};
            s[it][4] = *reinterpret_cast<const f2 *>(&L[LJ(4, ly + 1, lx)]);
            s[it][5] = f2{L[LJ(5, ly - 1, lx - 1)], L[LJ(5, ly - 1, lx)]};
            s[it][6] = f2{L[LJ(6, ly - 1, lx + 1)], L[LJ(6, ly - 1, lx + 2)]};
            s[it][7] = f2{L[LJ(7, ly + 1, lx + 1)], L[LJ(7, ly + 1, lx + 2)]};
            s[it][8] = f2{L[LJ(8, ly + 1, lx - 1)], L[LJ(8, ly + 1, lx)]};
        }
        __syncthreads();
        if (tr) a.trace[t * 5 + 1] = (long long)wall_clock64();
        // 2. collide, write back, publish; 3. the neighbours' step-t
        // populations into the ring (the ring slots are read only by the next
        // step's pull, so the poll may run while other waves still collide:
        // with early_poll the polling waves wait right after their first --
        // boundary -- item, hiding the hop behind the remaining items)
        const unsigned tag = a.tag0 + (unsigned)t + 1u;
        const int slot = t & 1;
        float tot = 0.f;
        bool ok = true;
        // neighbour's o_k for ring cell (ly, lx): into the ring slot
        auto ring_put = [&](int k, int ly, int lx, float v) { L[LJ(k, ly, lx)] = v; };
        auto poll_ring = [&]() {
            const long long deadline = (long long)wall_clock64() + deadline_span;
            for (int side = wv; side < 4; side += NW) {
                const int len = side < 2 ? tw : th;
                const int src_tile = side == 0 ? tys * a.tiles_x + tx
                                   : side == 1 ? tyn * a.tiles_x + tx
                                   : side == 2 ? ty * a.tiles_x + txw
                                               : ty * a.tiles_x + txe;
                const int d = side == 0 ? DN : side == 1 ? DS : side == 2 ? DE : DW;
                const bool corner = side < 2 && lane < 2, left = lane == 0;
                const int cd = side == 0 ? (left ? DNE : DNW) : (left ? DSE : DSW);
                const unsigned long long *cg =
                    corner ? gbase(slot, (side == 0 ? tys : tyn) * a.tiles_x + (left ? txw : txe), cd) : nullptr;
                float v[7];
                ok = ok && fetch_ring<2>(gbase(slot, src_tile, d), len, cg, tag, deadline, a.status, v);
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int p = lane + 64 * j;
                    if (p >= len) continue;
                    const int lx = side < 2 ? p : (side == 2 ? -1 : tw);
                    const int ly = side >= 2 ? p : (side == 0 ? -1 : th);
#pragma unroll
                    for (int i = 0; i < 3; ++i) ring_put(PLANES[d][i], ly, lx, v[3 * j + i]);
                }
                if (corner) ring_put(PLANES[cd][0], side == 0 ? -1 : th, left ? -1 : tw, v[6]);
            }
            if (a.htrace && t < a.trace_steps && wv < 4 && lane == 0)
                atomicMax(&a.htrace[((long long)t * ntiles + tile) * 2 + 1], (unsigned long long)wall_clock64());
        };
        const int poll_it = (a.early_poll && MAXIT >= 2) ? 0 : MAXIT - 1;
#pragma unroll
        for (int it = 0; it < MAXIT; ++it) {
            // the poll runs where the wave is converged: never while some of
            // its lanes still have to publish (a tile can be its own neighbour)
            if (it > 0 && it - 1 == poll_it) poll_ring();
            if (!((valid >> it) & 1u)) continue;
            const int lx = lxs[it], ly = lys[it];
            const float accf = (gy0 + ly == a.accel_row) ? 1.00f : 0.00f;
            f2 o[Q];
            f2 u;
            if constexpr (TOL) {
                const bool oab = (oa >> it) & 1u, obb = (ob >> it) & 1u;
                const f2 usq = collide2t<false>(s[it], o, oab, obb, (anyo >> it) & 1u, accf != 0.00f,
                                         TolK{a.omo, a.tc0, a.tc1, a.tc2}, a.w1, a.w2);
                u = f2{oab ? 0.f : sqrt_av(usq.x), obb ? 0.f : sqrt_av(usq.y)};
            } else {
                u = collide2(s[it], o, (oa >> it) & 1u, (ob >> it) & 1u, (anyo >> it) & 1u, accf, a.omega, a.omo,
                             a.w1, a.w2);
            }
            tot += u.x + u.y;
            f0[it] = o[0];
#pragma unroll
            for (int k = 1; k < Q; ++k) ST2(k, ly, lx, true, o[k]);
            const bool west = lx == 0, east = lx + 2 == tw;
            if (ly == th - 1) {  // leaving north: 2, 5, 6
                unsigned long long *g = gbase(slot, tile, DN) + lx;
                publish(g, o[2].x, tag);
                publish(g + 1, o[2].y, tag);
                publish(g + RES_GW, o[5].x, tag);
                publish(g + RES_GW + 1, o[5].y, tag);
                publish(g + 2 * RES_GW, o[6].x, tag);
                publish(g + 2 * RES_GW + 1, o[6].y, tag);
                if (east) publish(gbase(slot, tile, DNE), o[5].y, tag);
                if (west) publish(gbase(slot, tile, DNW), o[6].x, tag);
            }
            if (ly == 0) {       // leaving south: 4, 7, 8
                unsigned long long *g = gbase(slot, tile, DS) + lx;
                publish(g, o[4].x, tag);
                publish(g + 1, o[4].y, tag);
                publish(g + RES_GW, o[7].x, tag);
                publish(g + RES_GW + 1, o[7].y, tag);
                publish(g + 2 * RES_GW, o[8].x, tag);
                publish(g + 2 * RES_GW + 1, o[8].y, tag);
                if (west) publish(gbase(slot, tile, DSW), o[7].x, tag);
                if (east) publish(gbase(slot, tile, DSE), o[8].y, tag);
            }
            if (east) {          // leaving east: 1, 5, 8 of the pair's right cell
                unsigned long long *g = gbase(slot, tile, DE) + ly;
                publish(g, o[1].y, tag);
                publish(g + RES_GW, o[5].y, tag);
                publish(g + 2 * RES_GW, o[8].y, tag);
            }
            if (west) {          // leaving west: 3, 6, 7 of the pair's left cell
                unsigned long long *g = gbase(slot, tile, DW) + ly;
                publish(g, o[3].x, tag);
                publish(g + RES_GW, o[6].x, tag);
                publish(g + 2 * RES_GW, o[7].x, tag);
            }
        }
        if (a.htrace && t < a.trace_steps && lane == 0)
            atomicMax(&a.htrace[((long long)t * ntiles + tile) * 2], (unsigned long long)wall_clock64());
        if (poll_it == MAXIT - 1) poll_ring();
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) tot += __shfl_down(tot, off, 64);
        if (TOL) tot *= TOL_USQ_ROOT;  // collide2t returns 9 |u|^2
        if (lane == 0) wsum[wv] = tot;
        if (tr) a.trace[t * 5 + 2] = (long long)wall_clock64();
        if (tr) a.trace[t * 5 + 3] = (long long)wall_clock64();
        if (!ok) {
            abort_flag = 1;
            __hip_atomic_store(a.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (tr) a.trace[t * 5 + 4] = (long long)wall_clock64();
        return !abort_flag;
    };
    for (; t < a.steps; ++t) {
        if (tile == a.stall_tile && t == a.stall_step) break;  // debug: a tile that stops publishing
        if (!step()) break;
    }
    if (t == a.steps && a.steps > 0 && threadIdx.x == 0) {
        float sw = wsum[0];
#pragma unroll
        for (int i = 1; i < NW; ++i) sw += wsum[i];
        a.partials[(long long)(a.steps - 1) * ntiles + tile] = sw;
    }
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) {
        if (!((valid >> it) & 1u)) continue;
        const int lx = lxs[it], ly = lys[it];
        float *dst = a.fout + (long long)(gy0 + ly) * pitch + gx0 + lx;
        *reinterpret_cast<f2 *>(dst) = f0[it];
#pragma unroll
        for (int k = 1; k < Q; ++k) *reinterpret_cast<f2 *>(dst + k * P) = LD2(k, ly, lx, true);
    }
#undef ST2
#undef LD2
#undef LJ
}

// av_local[t] = sum over tiles of partials[t][tile], fixed order (one wave per step).
__global__ __launch_bounds__(256) void resident_reduce(const float *partials, float *av_local, int steps, int ntiles) {
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (t >= steps) return;
    const float *p = partials + (long long)t * ntiles;
    float v = 0.f;
    for (int i = lane; i < ntiles; i += 64) v += p[i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if (lane == 0) av_local[t] = v;
}

// ---- host side ---------------------------------------------------------------

namespace {
template <int NW, int R>
const void *resident_fn() {
    return reinterpret_cast<const void *>(&resident_steps<NW, R>);
}

template <int NW, int TH, int MINW = 1>
const void *resident_fn2(bool tol) {
    return tol ? reinterpret_cast<const void *>(&resident_steps2<NW, TH, MINW, true>)
               : reinterpret_cast<const void *>(&resident_steps2<NW, TH, MINW, false>);
}


// tol selects the LBM_FLAG_TOLERANCE collision of the packed (v2) tiles; the
// scalar v1 tiles have only the bitwise one
const void *resident_kernel(int variant, int &threads, bool tol) {
    switch (variant) {
        case RES_64: threads = 1024; return resident_fn<16, 4>();
        case RES_32: threads = 1024; return resident_fn<16, 2>();
        case RES_16: threads = 1024; return resident_fn<16, 1>();
        case RES_16x4: threads = 256; return resident_fn<4, 4>();
        case RES_8: threads = 512; return resident_fn<8, 1>();
        case RES_4: threads = 256; return resident_fn<4, 1>();
        case RES2_32: threads = 1024; return resident_fn2<16, 32>(tol);
        case RES2_16: threads = 1024; return resident_fn2<16, 16>(tol);
        case RES2_16x8: threads = 512; return resident_fn2<8, 16, 4>(tol);  // 2 blocks per CU: 4 waves per SIMD
        case RES2_8: threads = 512; return resident_fn2<8, 8>(tol);
        case RES2_4: threads = 256; return resident_fn2<4, 4>(tol);
        default: threads = 128; return resident_fn2<2, 2>(tol);  // RES2_2
    }
}
}  // namespace

// Blocks of `variant` the device keeps resident at once (occupancy query x CUs).
hipError_t resident_capacity(int variant, int device, bool tol, int &capacity) {
    int threads = 0;
    const void *fn = resident_kernel(variant, threads, tol);
    int per_cu = 0, cus = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, 0);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    if (e != hipSuccess) return e;
    capacity = per_cu * cus;
    return hipSuccess;
}

// coop (default): hipLaunchCooperativeKernel (the runtime rejects a grid that
// cannot be fully resident; HIP runs it on its own cooperative queue); else a
// plain launch of a grid the engine has already sized to the occupancy
// capacity (resident_capacity).  Neither makes the tiles co-resident when
// another kernel holds CUs: then the poll deadline drains the grid, the
// engine finds the status word set and repeats the run on the STEP2 kernel
// from the untouched input lattice (lbm_engine.hip run_steps).
hipError_t launch_resident(const ResidentArgs &a, int variant, bool tol, bool coop, hipStream_t s) {
    int threads = 0;
    const void *fn = resident_kernel(variant, threads, tol);
    ResidentArgs arg = a;
    void *params[] = {&arg};
    if (coop) return hipLaunchCooperativeKernel(fn, dim3(a.tiles_x * a.tiles_y), dim3(threads), params, 0, s);
    return hipLaunchKernel(fn, dim3(a.tiles_x * a.tiles_y), dim3(threads), params, 0, s);
}

hipError_t launch_resident_reduce(const float *partials, float *av_local, int steps, int ntiles, hipStream_t s) {
    if (steps <= 0) return hipSuccess;
    hipLaunchKernelGGL(resident_reduce, dim3((steps + 3) / 4), dim3(256), 0, s, partials, av_local, steps, ntiles);
    return hipGetLastError();
}

}  // namespace lbm
