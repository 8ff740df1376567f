// lbm_stream2.hip -- the S-step register-streaming kernel (stream_steps2d),
// two columns per lane, packed fp32 arithmetic: the default fused kernel
// for sub-domains of 4 M cells and more.
//
// One wave walks a strip of 128 columns row by row; as input row j arrives,
// level L computes row j-L of time step t+L, so the lattice crosses HBM once
// per S steps.  Each lane owns TWO adjacent columns (xa = base + 2l, xb = xa + 1):
//   * loads and stores are float2 (512 B per wave and plane row);
//   * the x-1 / x+1 neighbours are half in-lane (B's left is A, A's right is
//     B) and half one DPP wave shift away, so a shift costs one v_mov_dpp per
//     two cells;
//   * the two cells' arithmetic runs as packed fp32 (v_pk_add_f32 /
//     v_pk_mul_f32 / v_pk_fma_f32 on ext_vector_type(2) float);
//   * a 128-column strip recomputes 2S (+2 when its first column has the
//     wrong parity for float2 alignment) of every 128 columns.
//
// Bitwise parity with the one-step kernels and the CPU oracle: the packed
// collision and its exact short division / sqrt sequences live in
// lbm_packed.hpp (shared with the packed resident kernel); the
// LBM_FLAG_TOLERANCE form (collide2t) is checked against a stated tolerance
// instead (tests/test_gpu_tolerance.py).

#include "lbm_packed.hpp"

// The x-shifted planes the levels keep (rows of planes 1, 3, 5, 6, 7, 8) are
// held swapped, shifted in place (lbm_packed.hpp left2x); 0 builds the
// in-order form (tools/build_variant.sh, A/B only).
#ifndef LBM_SWAP_SHIFT
#define LBM_SWAP_SHIFT 1
#endif
namespace lbm {

__device__ __forceinline__ f2 shl_kept(f2 v) { return LBM_SWAP_SHIFT ? left2x(v) : left2(v); }
__device__ __forceinline__ f2 shr_kept(f2 v) { return LBM_SWAP_SHIFT ? right2x(v) : right2(v); }
__device__ __forceinline__ f2 kept(f2 u) { return LBM_SWAP_SHIFT ? unswap(u) : u; }

// halo_out with the destinations read from device memory inside the (rare)
// branch that stores them, so they hold no scalar registers across the loop
typedef const __attribute__((address_space(4))) Dst2 CDst2;
__device__ __forceinline__ Dst2 ld_dst(CDst2 *p) {
    Dst2 d;
    d.base = p->base;
    d.ks = p->ks;
    d.s1 = p->s1;
    d.s2 = p->s2;
    return d;
}

// S: the launch's steps (cells x < S or >= w - S are halo cells); the tables
// are laid out for the engine's ring width a.hw >= S, so east / north
// positions count from w - hw (h - hw): a remainder launch of fewer steps
// writes the innermost S of the hw ghost columns (rows), where the periodic /
// neighbour images of its cells belong.
__device__ __forceinline__ void halo_out_g(const StreamArgs &a, int S, int x, int y, const float (&o)[Q]) {
    const bool east = x >= a.w - S, west = x < S, north = y >= a.h - S, south = y < S;
    const int ex = x - (a.w - a.hw), ny = y - (a.h - a.hw);
    // The table is launch-invariant: read through the constant address space
    // under wave-uniform branches it becomes scalar loads, which never make
    // the wave wait for its row prefetch (a vector load here would need a
    // full vmcnt drain before its use).
    CDst2 *dg = (CDst2 *)a.dstg;
    const bool any_e = __builtin_amdgcn_ballot_w64(east) != 0, any_w = __builtin_amdgcn_ballot_w64(west) != 0;
    if (any_e) {
        const Dst2 d = ld_dst(dg + DE);
        if (east) store2(d, ex, y, o);
    }
    if (any_w) {
        const Dst2 d = ld_dst(dg + DW);
        if (west) store2(d, x, y, o);
    }
    if (north) {
        const Dst2 d = ld_dst(dg + DN);
        store2(d, ny, x, o);
        if (any_e) {
            const Dst2 e = ld_dst(dg + DNE);
            if (east) store2(e, ny, ex, o);
        }
        if (any_w) {
            const Dst2 w = ld_dst(dg + DNW);
            if (west) store2(w, ny, x, o);
        }
    }
    if (south) {
        const Dst2 d = ld_dst(dg + DS);
        store2(d, y, x, o);
        if (any_w) {
            const Dst2 w = ld_dst(dg + DSW);
            if (west) store2(w, y, x, o);
        }
        if (any_e) {
            const Dst2 e = ld_dst(dg + DSE);
            if (east) store2(e, y, ex, o);
        }
    }
}

// ---------------------------------------------------------------------------
// stream_steps2d: the work the streaming order makes redundant is removed
// (round 2 against its predecessor, every lattice value and every |u| partial
// bitwise unchanged):
//   * level L's first 2L row iterations of a segment would compute rows whose
//     own inputs were never loaded (their results are never used): they are
//     skipped (a warm-up loop of 2S iterations with wave-uniform guards, then
//     a guard-free main loop);
//   * the row loop is unrolled by two with the rows y-1 / y of planes 2, 5, 6
//     in parity-alternating registers, so the row rotation costs no moves;
//   * the folded acceleration is applied on the accelerated row only (a
//     wave-uniform branch, as LastChance.cpp:253-261) instead of adding zero
//     everywhere else;
//   * |u| (a v_sqrt per cell) only for rows that count towards av_vels;
//   * one ballot per loaded row (not per level) tells whether any obstacle
//     cell is in it.
template <int S>
struct Stream2State {
    f2 c0[S], c1[S], c3[S];          // planes 0, 1, 3 of row y (level L input; 1, 3 shifted, held swapped)
    f2 p2[2][S], p5[2][S], p6[2][S]; // [parity]: planes 2, 5, 6 of rows y-1 / y (5, 6 shifted, held swapped)
    float tot[S];                    // per level: running sum of |u| over the wave's owned cells
    f2 tot2[S];                      // OBST = false units: the same per column, all lanes (masked at the end)
    f2 v[2][Q];                      // [parity]: input row j (parity of j) / prefetched row j+1
    unsigned ob[2][2];               // [parity][A/B]: obstacle bytes of those rows
    unsigned oba, obb;               // per-lane obstacle bits of the last rows (bit L = row j-L)
    unsigned long long rob;          // wave-uniform: bit L = row j-L has an obstacle cell
};

struct Stream2Geo {
    const float *src;
    const uint8_t *obp;
    long long P;
    int pitch, xa, xb, yo0, yo1, j0, jlast;
    bool owna, ownb;
};

// Prefetch distance PD: the loads of row j+PD (clamped to the segment) are
// issued while row j is computed -- PD = 2 keeps two rows of every wave in
// flight (the kernel is bound by the memory-level parallelism of two waves
// per SIMD, not by VALU: tools/pmc_summary.py SQ_WAIT_ANY), at 18 more VGPRs.
template <int PD, bool OBST>
__device__ __forceinline__ void stream2d_load(const StreamArgs &a, const Stream2Geo &g, int j, f2 (&v)[Q],
                                              unsigned (&ob)[2]) {
    const int jn = min(j, g.jlast);
    const float *cn = g.src + (long long)jn * g.pitch;
#pragma unroll
    for (int k = 0; k < Q; ++k) v[k] = *reinterpret_cast<const f2 *>(cn + k * g.P);
    if (OBST) {
        const uint8_t *ocn = g.obp + (long long)(jn + a.og) * a.ogp;
        ob[0] = ocn[0];
        ob[1] = ocn[1];
    }
}

// OBST = false: the work unit reads no obstacle cell (stream2d_flags), so the
// obstacle bytes are neither loaded nor tracked and no level carries the
// rebound selects (their merge cost ~18 register copies per cell pair).
// LP (LDS planes): the older of the two rows of planes 2, 5, 6 a level keeps
// (row y-1, read two row iterations after it was stored) lives in LDS
// instead of registers -- lpl points at this lane's slot of a per-wave
// [S][3][64] f2 array; each level reads row y-1 from it and writes row y
// back (the same lane, the same address: no barrier, LDS keeps a wave's
// order) -- 6 VGPRs fewer per level.  (Rounds 3-4 kept the per-level |u|
// sums there too, S VGPRs fewer; once the in-place shifts freed 32 VGPRs,
// registers ran the S = 10 launch 2.5 % faster, profiles/r05/swap/us2_*.)
template <int S, int PAR, bool GUARD, int PD, bool NT, bool OBST, bool TOL, bool LP>
__device__ __forceinline__ void stream2d_row(const StreamArgs &a, const Stream2Geo &g, Stream2State<S> &st, int j,
                                             const TolK &tk, f2 *lpl) {
    // PD = 1: row j+1 into the other parity's buffer; PD = 2: row j+2 into this one once it is read
    // (LP forms issue row j+1's loads later, at level 2: see below)
    if (PD == 1 && !LP) stream2d_load<PD, OBST>(a, g, j + 1, st.v[1 - PAR], st.ob[1 - PAR]);
    if (OBST) {
        const unsigned voa = st.ob[PAR][0] != 0 ? 1u : 0u, vob = st.ob[PAR][1] != 0 ? 1u : 0u;
        st.oba = (st.oba << 1) | voa;
        st.obb = (st.obb << 1) | vob;
        st.rob = (st.rob << 1) | (__builtin_amdgcn_ballot_w64((voa | vob) != 0) != 0 ? 1ull : 0ull);
    }

    // keep the row's arithmetic between its own prefetch and the next row's:
    // the scheduler would otherwise hoist the next row's first uses of its
    // just-issued loads into this row (a full vmcnt wait one row early)
    __builtin_amdgcn_sched_barrier(0);
    f2 cur[Q];
#pragma unroll
    for (int k = 0; k < Q; ++k) cur[k] = st.v[PAR][k];
    if (PD == 2) stream2d_load<PD, OBST>(a, g, j + 2, st.v[PAR], st.ob[PAR]);
#pragma unroll
    for (int L = 1; L <= S; ++L) {
        const int b = L - 1;
        const int y = j - L;
        if constexpr (LP && PD == 1) {
            // LP forms: row j+1 is loaded once level 1 has consumed row j, into
            // the row buffer itself (cur holds row j by then) -- one 18-VGPR
            // row buffer; levels 2..S (>= 5 levels) cover the latency
            if (L == 2) {
                stream2d_load<PD, OBST>(a, g, j + 1, st.v[0], st.ob[0]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // pulled populations of row y (level L-1 values; x +- 1 by DPP)
        f2 s[Q];
        if constexpr (LP) {
            // LP: the registers hold row y-1 of planes 2, 5, 6 (the older row),
            // the LDS slot row y; both move on after the collision (below)
            s[2] = st.p2[0][b];
            s[5] = kept(st.p5[0][b]);
            s[6] = kept(st.p6[0][b]);
        } else {
            s[2] = st.p2[PAR][b];
            s[5] = kept(st.p5[PAR][b]);
            s[6] = kept(st.p6[PAR][b]);
            st.p2[PAR][b] = cur[2];
            st.p5[PAR][b] = shl_kept(cur[5]);
            st.p6[PAR][b] = shr_kept(cur[6]);
        }
        s[0] = st.c0[b];
        s[1] = kept(st.c1[b]);
        s[3] = kept(st.c3[b]);
        s[4] = cur[4];
        s[7] = kept(shr_kept(cur[7]));
        s[8] = kept(shl_kept(cur[8]));
        if constexpr (!LP) {
            st.c0[b] = cur[0];
            st.c1[b] = shl_kept(cur[1]);
            st.c3[b] = shr_kept(cur[3]);
        }
        // inputs of this row were never loaded: the result is unused.  The LP
        // forms skip only the collision (the level's inputs still pass
        // through, never reaching a store or a sum: rowlive) -- skipping the
        // whole level makes the compiler hold a second copy of the level state
        // in the tolerance forms (S = 7: 234 vs 202 VGPRs, S = 10: 35 spilled
        // vs 254)
        const bool cold = GUARD && j < g.j0 + 2 * L;
        if (!LP && cold) continue;

        f2 o[Q];
        const bool oa = OBST && ((st.oba >> L) & 1u), ob = OBST && ((st.obb >> L) & 1u);
        const bool any_obst = OBST && ((st.rob >> L) & 1ull);
        int gy = a.gy0 + y;
        gy = gy < 0 ? gy + a.ny : (gy >= a.ny ? gy - a.ny : gy);
        f2 usq;
        if (LP && cold) {
#pragma unroll
            for (int k = 0; k < Q; ++k) o[k] = s[k];
            usq = s[0];
        } else if constexpr (TOL) {
            usq = collide2t(s, o, oa, ob, any_obst, gy == a.accel_g, tk, a.w1, a.w2);
        } else {
            usq = collide2u(s, o, oa, ob, any_obst, gy == a.accel_g, a.omega, a.omo, a.w1, a.w2);
        }
        if constexpr (LP) {
            // the level state moves on once the collision has consumed the old
            // rows, so the new values can take the old ones' registers (updated
            // before the collision they needed a register each plus a copy:
            // ~5 v_mov_b64 per level and row): planes 2, 5, 6 of row y from the
            // LDS slot into the registers, row y+1 into the slot (read before
            // write: one wave's LDS operations stay in order), planes 0, 1, 3
            // of row y+1
            f2 *slot = lpl + b * 3 * 64;
            st.p2[0][b] = slot[0];
            st.p5[0][b] = slot[64];
            st.p6[0][b] = slot[128];
            slot[0] = cur[2];
            slot[64] = shl_kept(cur[5]);
            slot[128] = shr_kept(cur[6]);
            st.c0[b] = cur[0];
            st.c1[b] = shl_kept(cur[1]);
            st.c3[b] = shr_kept(cur[3]);
        }
        const bool rowlive = (!GUARD || y >= g.yo0) && (L == S || y < g.yo1);
        if (rowlive) {
            if constexpr (OBST) {
                const float ua = (oa || !g.owna) ? 0.f : sqrt_av(usq.x);
                const float ub = (ob || !g.ownb) ? 0.f : sqrt_av(usq.y);
                st.tot[b] += ua + ub;
            } else {
                // no obstacle cell in the unit: the lane's column ownership is
                // the unit's, applied once at its end (stream2d_unit) -- one
                // packed add per level instead of two selects and two adds
                // (the empty asm keeps `rowlive` a branch: if-converted, the
                // sums would cost two selects per level again)
                asm volatile("");
                st.tot2[b] += f2{sqrt_av(usq.x), sqrt_av(usq.y)};
            }
        }
        if (L == S) {
            if (rowlive && (g.owna || g.ownb)) {
                float *w0 = a.fout + (long long)y * g.pitch + g.xa;
                if (g.owna && g.ownb) {
#pragma unroll
                    for (int k = 0; k < Q; ++k) {
                        f2 *pd = reinterpret_cast<f2 *>(w0 + k * g.P);
                        if (NT)
                            __builtin_nontemporal_store(o[k], pd);
                        else
                            *pd = o[k];
                    }
                } else if (g.owna) {
#pragma unroll
                    for (int k = 0; k < Q; ++k) w0[k * g.P] = o[k].x;
                } else {
#pragma unroll
                    for (int k = 0; k < Q; ++k) w0[k * g.P + 1] = o[k].y;
                }
                if (g.xa < S || g.xb >= a.w - S || y < S || y >= a.h - S) {
                    float oa_[Q], ob_[Q];
#pragma unroll
                    for (int k = 0; k < Q; ++k) {
                        oa_[k] = o[k].x;
                        ob_[k] = o[k].y;
                    }
                    if (g.owna) halo_out_g(a, S, g.xa, y, oa_);
                    if (g.ownb) halo_out_g(a, S, g.xb, y, ob_);
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < Q; ++k) cur[k] = o[k];
        }
        // LP forms: one level at a time (the scheduler would otherwise start
        // the next level's LDS reads and shifts early and spill at S >= 6)
        if constexpr (LP) __builtin_amdgcn_sched_barrier(0);
    }
}

// Geometry of work unit t (strip x segment) for this lane.
template <int S>
__device__ __forceinline__ Stream2Geo stream2d_geo(const StreamArgs &a, int t, int lane) {
    const int r = rect_of(a.rect_begin, t);
    const SRect R = a.rect[r];
    const int lt = t - a.rect_begin[r];
    const int seg = lt / R.nstrip, strip = lt - seg * R.nstrip;
    const int xo0 = R.x0 + strip * R.ow;             // first owned column
    const int xo1 = min(xo0 + R.ow, R.x0 + R.w);     // past the last owned column
    const int base = (xo0 - S) & ~1;                 // even: float2-aligned
    Stream2Geo g;
    g.xa = base + 2 * lane;
    g.xb = g.xa + 1;
    g.owna = g.xa >= xo0 && g.xa < xo1;
    g.ownb = g.xb >= xo0 && g.xb < xo1;
    g.yo0 = R.y0 + seg * R.hs;
    g.yo1 = min(g.yo0 + R.hs, R.y0 + R.h);
    const int xca = min(g.xa, (a.xmax - 1) & ~1);
    g.P = a.plane;
    g.pitch = a.pitch;
    g.src = a.fin + xca;
    g.obp = a.obst_g + (xca + a.og);
    g.j0 = g.yo0 - S;
    g.jlast = g.yo1 + S - 1;
    return g;
}

// One work unit (strip x segment t) of the launch; accumulates |u| per level into st.tot.
// LP forms walk the rows one per iteration (the non-LP forms two, with the
// rows y-1 / y of planes 2, 5, 6 in parity-alternating registers): unrolling
// by two lets the compiler give every level-state value a register per
// parity instead of one register and a copy, which costs 6-8 VGPRs per level
// (S = 10: 253 VGPRs without spills one row per iteration; 256 + 221 spilled
// two rows per iteration).
template <int S, int PD, bool NT, bool OBST, bool TOL, bool LP>
__device__ __forceinline__ void stream2d_unit(const StreamArgs &a, int t, int lane, Stream2State<S> &st,
                                              f2 *lpl) {
    const Stream2Geo g = stream2d_geo<S>(a, t, lane);
    const TolK tk{a.omo, a.tc0, a.tc1, a.tc2};
    if constexpr (LP) {
#pragma unroll
        for (int i = 0; i < 3 * S; ++i) lpl[i * 64] = mk2(0.f);
    }

#pragma unroll
    for (int b = 0; b < S; ++b) {
        st.c0[b] = st.c1[b] = st.c3[b] = mk2(0.f);
        st.p2[0][b] = st.p5[0][b] = st.p6[0][b] = st.p2[1][b] = st.p5[1][b] = st.p6[1][b] = mk2(0.f);
    }
    st.oba = st.obb = 0;
    st.rob = 0;
    if constexpr (!OBST) {
#pragma unroll
        for (int b = 0; b < S; ++b) st.tot2[b] = mk2(0.f);
    }
    stream2d_load<PD, OBST>(a, g, g.j0, st.v[0], st.ob[0]);
    if (PD == 2) stream2d_load<PD, OBST>(a, g, g.j0 + 1, st.v[1], st.ob[1]);
    // warm-up: rows j0 .. j0+2S-1 (level L valid from j0+2L); jlast >= j0+2S
    int j = g.j0;
    if constexpr (LP) {
#pragma unroll 1
        for (int i = 0; i < 2 * S; ++i, ++j) stream2d_row<S, 0, true, PD, NT, OBST, TOL, LP>(a, g, st, j, tk, lpl);
#pragma unroll 1
        for (; j <= g.jlast; ++j) stream2d_row<S, 0, false, PD, NT, OBST, TOL, LP>(a, g, st, j, tk, lpl);
    } else {
#pragma unroll 1
        for (int i = 0; i < S; ++i, j += 2) {
            stream2d_row<S, 0, true, PD, NT, OBST, TOL, LP>(a, g, st, j, tk, lpl);
            stream2d_row<S, 1, true, PD, NT, OBST, TOL, LP>(a, g, st, j + 1, tk, lpl);
        }
#pragma unroll 1
        for (; j + 1 <= g.jlast; j += 2) {
            stream2d_row<S, 0, false, PD, NT, OBST, TOL, LP>(a, g, st, j, tk, lpl);
            stream2d_row<S, 1, false, PD, NT, OBST, TOL, LP>(a, g, st, j + 1, tk, lpl);
        }
        if (j <= g.jlast) stream2d_row<S, 0, false, PD, NT, OBST, TOL, LP>(a, g, st, j, tk, lpl);
    }
    if constexpr (!OBST) {
#pragma unroll
        for (int b = 0; b < S; ++b) st.tot[b] += (g.owna ? st.tot2[b].x : 0.f) + (g.ownb ? st.tot2[b].y : 0.f);
    }
}

// |u| partials of one work unit, one per level (= time step of the launch)
// (TOL: the sums are of sqrt(9 |u|^2), collide2t; scaled by 1/3 here, once)
template <int S, bool TOL>
__device__ __forceinline__ void stream2d_partials(const StreamArgs &a, int idx, int lane, Stream2State<S> &st) {
#pragma unroll
    for (int l = 0; l < S; ++l) {
        float sum = st.tot[l];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) sum += __shfl_down(sum, off, 64);
        if (TOL) sum *= TOL_USQ_ROOT;
        if (lane == 0) a.partials_out[(long long)l * a.stride + idx] = sum;
        st.tot[l] = 0.f;
    }
}

// Work units: W waves per workgroup take W consecutive units (adjacent strips
// of one segment row, so they run side by side on one CU and read their
// shared overlap columns through its L1 / L2); t = xcd_remap(blockIdx) * W +
// wave, and blocks b and b+8 share an XCD and take neighbouring units.  NT:
// non-temporal lattice stores (the output is not read again by this launch).
// tools/micro/stream_pattern.hip, the kernel's memory pattern alone at
// 8192^2: 1.245 ms per pass with one wave per workgroup and plain stores,
// 1.172 with four waves, 1.187 with nt stores, 1.121 with both.
// (A persistent grid taking units from a device-scope counter balanced the
// waves better but read 1.30x the algorithmic bytes instead of 1.18x:
// neighbouring strips landed on different XCDs.)
// Two waves per SIMD (256 VGPRs each).  Deeper LP forms were measured and
// removed: at two waves per SIMD S >= 7 spills (41-63 VGPRs), at one wave per
// SIMD (AGPRs as spill space, no scratch) S = 7..12 ran 175-214 GLUPS
// bitwise and 263-314 tolerance against 290 / 333 for S = 6
// (profiles/r03/ab_lp_depth.log).
template <int S, bool kReduce, int W, bool NT, bool TOL = false, bool LP = false>
__global__ __launch_bounds__(64 * W, 2) void stream_steps2d(StreamArgs a) {
    __shared__ float lds[W];
    __shared__ f2 lds_p[LP ? W * 3 * S * 64 : 1];   // LP: [wave][S][3][64] older rows of planes 2, 5, 6
    // (S = 10: 15 KB per one-wave workgroup, so eight fit a CU's 160 KB)
    if (kReduce && blockIdx.x == 0) reduce_pending_n<64 * W>(a.ctl, a.partials_prev, a.av_local, lds);

    const int lane = threadIdx.x & 63;
    Stream2State<S> st;
#pragma unroll
    for (int l = 0; l < S; ++l) st.tot[l] = 0.f;
    f2 *const lpl = lds_p + (LP ? (threadIdx.x >> 6) * 3 * S * 64 : 0) + lane;
    // wave-uniform: keeps the unit geometry and the row loop in scalar registers
    const int slot = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * W + (int)(threadIdx.x >> 6));
    // dispatch order -> work unit (a.uperm: per XCD range, obstacle-bearing
    // units first, so the slower units never start last); partials and flags
    // are indexed by unit, so the |u| sums do not depend on the order
    typedef const __attribute__((address_space(4))) int CI32;
    const int t = (a.uperm != nullptr && slot < a.total) ? ((CI32 *)a.uperm)[slot] : slot;
    const unsigned long long t_start = a.trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
    if (t < a.total) {
        // per-unit obstacle flag (launch-invariant; scalar load): units that
        // read no obstacle cell run the select-free copy of the unit loop
        typedef const __attribute__((address_space(4))) uint8_t CU8;
        if (a.uobst == nullptr || ((CU8 *)a.uobst)[t] != 0)
            stream2d_unit<S, 1, NT, true, TOL, LP>(a, t, lane, st, lpl);
        else
            stream2d_unit<S, 1, NT, false, TOL, LP>(a, t, lane, st, lpl);
    }
    if (t < max(a.total, 1)) stream2d_partials<S, TOL>(a, t, lane, st);
    if (a.trace && lane == 0 && t < a.total) {
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        a.trace[2 * (long long)t] = t_start;
        a.trace[2 * (long long)t + 1] = t_end;
    }
    if (kReduce && blockIdx.x == 0 && threadIdx.x == 0) publish_pending(a.ctl, S, a.n_total, a.stride);
}

// uobst[t] = 1 when work unit t loads any obstacle cell (rows j0 .. jlast of
// its strip, the same bytes stream2d_load reads), else 0.  One wave per unit;
// run once per launch plan (obstacles are fixed for the engine's lifetime).
template <int S>
__global__ __launch_bounds__(64) void stream2d_flags(StreamArgs a, uint8_t *uobst) {
    const int t = __builtin_amdgcn_readfirstlane((int)blockIdx.x);
    if (t >= a.total) return;
    const Stream2Geo g = stream2d_geo<S>(a, t, (int)threadIdx.x);
    unsigned any = 0;
    for (int j = g.j0; j <= g.jlast; ++j) {
        const uint8_t *ocn = g.obp + (long long)(j + a.og) * a.ogp;
        any |= (unsigned)ocn[0] | (unsigned)ocn[1];
    }
    const bool hit = __builtin_amdgcn_ballot_w64(any != 0) != 0;
    if (threadIdx.x == 0) uobst[t] = hit ? 1 : 0;
}

hipError_t stream2d_unit_flags(const StreamArgs &a, int steps, uint8_t *uobst, hipStream_t s) {
    if (a.total <= 0) return hipSuccess;
    switch (steps) {
        case 2: hipLaunchKernelGGL(stream2d_flags<2>, dim3(a.total), dim3(64), 0, s, a, uobst); break;
        case 3: hipLaunchKernelGGL(stream2d_flags<3>, dim3(a.total), dim3(64), 0, s, a, uobst); break;
        case 4: hipLaunchKernelGGL(stream2d_flags<4>, dim3(a.total), dim3(64), 0, s, a, uobst); break;
        case 5: hipLaunchKernelGGL(stream2d_flags<5>, dim3(a.total), dim3(64), 0, s, a, uobst); break;
        case 6: hipLaunchKernelGGL(stream2d_flags<6>, dim3(a.total), dim3(64), 0, s, a, uobst); break;
        case 7: hipLaunchKernelGGL(stream2d_flags<7>, dim3(a.total), dim3(64), 0, s, a, uobst); break;
        case 8: hipLaunchKernelGGL(stream2d_flags<8>, dim3(a.total), dim3(64), 0, s, a, uobst); break;
        case 9: hipLaunchKernelGGL(stream2d_flags<9>, dim3(a.total), dim3(64), 0, s, a, uobst); break;
        case 10: hipLaunchKernelGGL(stream2d_flags<10>, dim3(a.total), dim3(64), 0, s, a, uobst); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int S, bool NT, bool TOL = false, bool LP = false>
static void launch_s2d(const StreamArgs &a, int units, bool reduce, hipStream_t s) {
    if (reduce)
        hipLaunchKernelGGL((stream_steps2d<S, true, 1, NT, TOL, LP>), dim3(units), dim3(64), 0, s, a);
    else
        hipLaunchKernelGGL((stream_steps2d<S, false, 1, NT, TOL, LP>), dim3(units), dim3(64), 0, s, a);
}

template <int S, bool TOL, bool LP>
static const void *s2d_fn() {
    return (const void *)&stream_steps2d<S, false, 1, false, TOL, LP>;
}

// Launch forms (cfg; one wave per workgroup in all of them -- four-wave
// workgroups on adjacent strips lost their A/B, profiles/r02/ab_cfg_s5.log):
//   0 plain stores, 3 non-temporal lattice stores, 4 LP (older rows of
//   planes 2, 5, 6 and the |u| sums in LDS; bitwise S = 6, the default form
//   at S = 6, where the plain form runs out of registers -- at S = 5 the two
//   forms measure equal, profiles/r03/ab_forms_s5_s6.log; tolerance S = 6..8).
// tol: the LBM_FLAG_TOLERANCE collision (collide2t) in forms 0 and 4.
bool s2d_form_ok(int steps, int cfg, bool tol) {
    if (cfg == 4) return steps == 6 || (tol && steps >= 7 && steps <= 10);
    if (cfg == 0) return steps >= 2 && steps <= 6;
    if (cfg == 3) return !tol && steps >= 2 && steps <= 6;
    return false;
}

// resident one-wave workgroups per CU of the instantiation a launch with
// these parameters uses (the engine sizes segments to whole rounds of them)
hipError_t stream2d_blocks_per_cu(int steps, int cfg, bool tol, int &n) {
    if (!s2d_form_ok(steps, cfg, tol)) return hipErrorInvalidValue;
    const void *fn = nullptr;
    if (cfg == 4) {
        switch (steps) {
            case 7: fn = s2d_fn<7, true, true>(); break;
            case 8: fn = s2d_fn<8, true, true>(); break;
            case 9: fn = s2d_fn<9, true, true>(); break;
            case 10: fn = s2d_fn<10, true, true>(); break;
            default: fn = tol ? s2d_fn<6, true, true>() : s2d_fn<6, false, true>(); break;
        }
    } else {  // cfg 3 has the registers of cfg 0
        switch (steps) {
            case 2: fn = tol ? s2d_fn<2, true, false>() : s2d_fn<2, false, false>(); break;
            case 3: fn = tol ? s2d_fn<3, true, false>() : s2d_fn<3, false, false>(); break;
            case 4: fn = tol ? s2d_fn<4, true, false>() : s2d_fn<4, false, false>(); break;
            case 5: fn = tol ? s2d_fn<5, true, false>() : s2d_fn<5, false, false>(); break;
            default: fn = tol ? s2d_fn<6, true, false>() : s2d_fn<6, false, false>(); break;
        }
    }
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, 64, 0);
}

hipError_t launch_stream2d(const StreamArgs &a, int units, int steps, bool reduce, int cfg, bool tol, hipStream_t s) {
    if (!s2d_form_ok(steps, cfg, tol)) return hipErrorInvalidValue;
    if (cfg == 4) {
        switch (steps * 2 + (tol ? 1 : 0)) {
            case 12: launch_s2d<6, false, false, true>(a, units, reduce, s); break;
            case 13: launch_s2d<6, false, true, true>(a, units, reduce, s); break;
            case 15: launch_s2d<7, false, true, true>(a, units, reduce, s); break;
            case 17: launch_s2d<8, false, true, true>(a, units, reduce, s); break;
            case 19: launch_s2d<9, false, true, true>(a, units, reduce, s); break;
            case 21: launch_s2d<10, false, true, true>(a, units, reduce, s); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    if (tol) {
        switch (steps) {
            case 2: launch_s2d<2, false, true>(a, units, reduce, s); break;
            case 3: launch_s2d<3, false, true>(a, units, reduce, s); break;
            case 4: launch_s2d<4, false, true>(a, units, reduce, s); break;
            case 5: launch_s2d<5, false, true>(a, units, reduce, s); break;
            case 6: launch_s2d<6, false, true>(a, units, reduce, s); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    switch (steps * 10 + cfg) {
        case 20: launch_s2d<2, false>(a, units, reduce, s); break;
        case 30: launch_s2d<3, false>(a, units, reduce, s); break;
        case 40: launch_s2d<4, false>(a, units, reduce, s); break;
        case 50: launch_s2d<5, false>(a, units, reduce, s); break;
        case 60: launch_s2d<6, false>(a, units, reduce, s); break;
        case 23: launch_s2d<2, true>(a, units, reduce, s); break;
        case 33: launch_s2d<3, true>(a, units, reduce, s); break;
        case 43: launch_s2d<4, true>(a, units, reduce, s); break;
        case 53: launch_s2d<5, true>(a, units, reduce, s); break;
        case 63: launch_s2d<6, true>(a, units, reduce, s); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace lbm
