// lbm_engine.hip -- the C ABI (include/lbm_hip.h) over the gfx950 kernels.
//
// Replaces what the reference delegates to Poplar: graph build and tile
// mapping (main/LbmAoS.cpp:135-372, main/include/StructuredGridUtils.hpp),
// the BSP halo exchange of stitched views (LbmAoS.cpp:151-189,
// GraphcoreUtils.hpp:119-127) and the Engine run/stream API
// (main/LbmRunner.cpp:81-144).
//
// Structure
//   * The domain is split into R x C sub-domains with the reference's
//     partitionForIpus rule (StructuredGridUtils.hpp:472-561).
//   * Each sub-domain owns a ghosted SoA lattice pair, a compute stream and a
//     comm stream.  Periodic wrap inside a sub-domain is written by the step
//     kernel itself into its ghost ring ("self" directions); directions that
//     cross sub-domains go through send buffers the step kernel packs, a
//     transport (device copies, or grouped ncclSend/ncclRecv over xGMI), and
//     an unpack kernel.
//   * Multi-sub-domain step: boundary strip kernel -> exchange on the comm
//     stream, overlapped with the interior kernel on the compute stream.
//   * The per-step |u| sums stay on the device (block partials folded by the
//     next step's kernel); ranks combine them once, in rank order, on store.

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "lbm_hip.h"
#include "lbm_layout.hpp"

namespace lbm {
hipError_t launch_step(const StepArgs &a, int blocks, bool vec4, bool reduce, int flags, int min_waves,
                       hipStream_t s);
hipError_t launch_finalize(const float *partials, int n, float *av_local, int *ctl, hipStream_t s);
hipError_t launch_accelerate(float *f, const uint8_t *obst, long long P, int pitch, int w, int row, float w1,
                             float w2, hipStream_t s);
hipError_t launch_init_equilibrium(float *f, long long rows, int rf, int pitch, long long P, float c0, float c1,
                                   float c2, hipStream_t s);
hipError_t launch_aos_to_soa(const float *aos, float *f, long long P, int pitch, int w, int h, hipStream_t s);
hipError_t launch_soa_to_aos(const float *f, float *aos, long long P, int pitch, int w, int h, hipStream_t s);
hipError_t launch_halo_pack(const HaloArgs &a, hipStream_t s);
hipError_t launch_halo_unpack(const HaloArgs &a, hipStream_t s);
}  // namespace lbm

using namespace lbm;

namespace {

struct lbm_failure : std::runtime_error {
    int code;
    lbm_failure(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

#define HIP_CHECK(expr)                                                                                  \
    do {                                                                                                 \
        hipError_t e_ = (expr);                                                                          \
        if (e_ != hipSuccess)                                                                            \
            throw lbm_failure(LBM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));             \
    } while (0)

#define NCCL_CHECK(expr)                                                                                 \
    do {                                                                                                 \
        ncclResult_t r_ = (expr);                                                                        \
        if (r_ != ncclSuccess) throw lbm_failure(LBM_E_RCCL, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

inline long long round_up(long long v, long long m) { return (v + m - 1) / m * m; }

// Reference rule, StructuredGridUtils.hpp:472-527 (numIpus -> numRows x numCols).
bool choose_grid(int nx, int ny, int parts, int &rows, int &cols) {
    const float row_imb = (float)(ny % parts) / (float)ny;
    const float col_imb = (float)(nx % parts) / (float)nx;
    switch (parts) {
        case 1: rows = 1; cols = 1; return true;
        case 2: if (row_imb < col_imb) { rows = 2; cols = 1; } else { rows = 1; cols = 2; } return true;
        case 4: rows = 2; cols = 2; return true;
        case 8: if (row_imb < col_imb) { rows = 4; cols = 2; } else { rows = 2; cols = 4; } return true;
        case 16: rows = 4; cols = 4; return true;
        default: return false;
    }
}

// Round-robin allocation (StructuredGridUtils.hpp:161-165): the first n % k parts get one more.
std::vector<int> round_robin(int n, int k) {
    std::vector<int> v(k, n / k);
    for (int i = 0; i < n % k; ++i) v[i]++;
    return v;
}

int partition(int nx, int ny, int parts, int grid_rows, int grid_cols, int &R, int &C, std::vector<lbm_rect> &rects) {
    if (nx <= 0 || ny <= 0 || parts <= 0) return LBM_E_INVALID;
    if (grid_rows > 0 && grid_cols > 0) {
        R = grid_rows;
        C = grid_cols;
    } else if (!choose_grid(nx, ny, parts, R, C)) {
        return LBM_E_INVALID;
    }
    if (R * C != parts || R > ny || C > nx) return LBM_E_INVALID;
    const auto ra = round_robin(ny, R), ca = round_robin(nx, C);
    rects.assign(parts, lbm_rect{0, 0, 0, 0});
    int y0 = 0;
    for (int r = 0; r < R; ++r) {
        int x0 = 0;
        for (int c = 0; c < C; ++c) {
            rects[r * C + c] = lbm_rect{x0, y0, ca[c], ra[r]};  // rank = row * cols + col (:548)
            x0 += ca[c];
        }
        y0 += ra[r];
    }
    return LBM_OK;
}

struct Sub {
    int id = 0, row = 0, col = 0, dev = 0;
    lbm_rect rect{};
    int w = 0, h = 0, pitch = 0;
    long long plane = 0;
    long long lattice_floats = 0;
    float *f[2] = {nullptr, nullptr};
    uint8_t *obst = nullptr;
    float *halo_mem = nullptr;  // all send + recv buffers
    float *send[8] = {};
    float *recv[8] = {};
    int nb[8] = {};             // neighbour sub id / rank per direction
    bool remote[8] = {};
    float *partials[2] = {nullptr, nullptr};
    int n_int_blocks = 0, n_bnd_blocks = 0;
    float *av_local = nullptr;
    int av_cap = 0;
    int *ctl = nullptr;
    int accel_row = -1;
    hipStream_t s_comp = nullptr, s_comm = nullptr;
    hipEvent_t ev_b = nullptr, ev_u = nullptr, ev_end = nullptr;
    StepArgs args_int[2]{}, args_bnd[2]{};  // per parity
    HaloArgs unpack[2]{};                   // per parity (lattice written by that step)
    int cur = 0;                            // lattice holding the current state
    bool any_remote() const {
        for (bool r : remote)
            if (r) return true;
        return false;
    }
};

int edge_len(int d, int w, int h) { return d < 4 ? ((d & 1) ? w : h) : 1; }

}  // namespace

struct lbm_handle {
    lbm_params p{};
    int R = 1, C = 1, parts = 1;
    int transport = LBM_TRANSPORT_LOCAL;
    int rank = 0, world = 1;
    bool vec4 = true;
    int graph_steps = 8;  // default: replay 16-step graphs on the single-domain path
    // hipGraph of 2*graph_steps single-sub-domain steps, one per starting parity
    hipGraphExec_t graph_exec[2] = {nullptr, nullptr};
    // tuning knobs (environment, read at create): LBM_KFLAGS (bit0 nt stores,
    // bit1 nt loads), LBM_MIN_WAVES, LBM_MAX_BLOCKS, LBM_LAYOUT (planar|rows)
    // defaults chosen by tools/ab_bench.py on MI355X (profiles/r01/ab_*.log):
    // plane-ordered kernel, row-interleaved f[y][k][x], one tile per block
    int kflags = 4, kwaves = 1, max_blocks_cfg = 1 << 30;
    bool row_interleaved = true;
    std::vector<lbm_rect> all_rects;
    std::vector<Sub> subs;  // local sub-domains
    ncclComm_t comm = nullptr;
    int64_t free_cells = 0;
    bool loaded = false;
    int last_steps = 0;
    double last_seconds = 0.0;
    hipEvent_t t0 = nullptr, t1 = nullptr;
    std::string err;
    bool force_exchange = false;
    // any direction goes through the transport (several sub-domains, or forced)
    bool multi() const { return parts > 1 || force_exchange; }

    // ------------------------------------------------------------------
    void set_device(const Sub &s) const { HIP_CHECK(hipSetDevice(s.dev)); }

    EdgeDst make_dst(const Sub &s, float *lattice, int d) const {
        EdgeDst e{};
        if (s.remote[d]) {
            const int len = edge_len(d, s.w, s.h);
            for (int i = 0; i < NPLANES[d]; ++i) e.p[i] = s.send[d] + (long long)i * len;
            e.ps = 1;
            return e;
        }
        // own ghost ring on the opposite side
        const int g = OPP_DIR[d];
        int xg = 0, yg = 0;
        switch (g) {
            case DE: xg = s.w; break;
            case DW: xg = -1; break;
            case DN: yg = s.h; break;
            case DS: yg = -1; break;
            case DNE: xg = s.w; yg = s.h; break;
            case DNW: xg = -1; yg = s.h; break;
            case DSW: xg = -1; yg = -1; break;
            case DSE: xg = s.w; yg = -1; break;
        }
        long long base;
        if (g == DE || g == DW) {  // column, position = y
            base = 1LL * s.pitch + XOFF + xg;
            e.ps = s.pitch;
        } else if (g == DN || g == DS) {  // row, position = x
            base = (long long)(yg + 1) * s.pitch + XOFF;
            e.ps = 1;
        } else {
            base = (long long)(yg + 1) * s.pitch + XOFF + xg;
            e.ps = 1;
        }
        for (int i = 0; i < NPLANES[d]; ++i) e.p[i] = lattice + PLANES[d][i] * s.plane + base;
        return e;
    }

    int max_blocks() const { return max_blocks_cfg; }

    static int env_int(const char *name, int dflt) {
        const char *v = getenv(name);
        return (v && *v) ? atoi(v) : dflt;
    }

    void read_tuning() {
        kflags = env_int("LBM_KFLAGS", kflags);
        kwaves = env_int("LBM_MIN_WAVES", kwaves);
        max_blocks_cfg = std::max(1, env_int("LBM_MAX_BLOCKS", max_blocks_cfg));
        graph_steps = std::max(0, env_int("LBM_GRAPH_STEPS", graph_steps));
        const char *l = getenv("LBM_LAYOUT");
        if (l && *l) row_interleaved = std::string(l) != "planar";
    }

    // rects: x0, y0 in cells; widths in cells (converted to work items here)
    void fill_rects(StepArgs &a, const std::vector<Rect> &cells_rects, int &blocks) const {
        const int vw = vec4 ? 4 : 1;
        int tiles = 0;
        a.nrect = (int)cells_rects.size();
        for (int i = 0; i < MAX_RECTS; ++i) {
            if (i < a.nrect) {
                Rect r = cells_rects[i];
                r.wc = r.wc / vw;
                a.rect[i] = r;
                a.rect_begin[i] = tiles;
                const long long items = (long long)r.wc * r.hr;
                tiles += (int)((items + BLOCK - 1) / BLOCK);
            } else {
                a.rect[i] = Rect{0, 0, 1, 1};
                a.rect_begin[i] = INT_MAX;
            }
        }
        a.total = tiles;
        blocks = std::max(1, std::min(tiles, max_blocks()));
    }

    void build_args(Sub &s) {
        const float w1 = p.density * p.accel / 9.f;
        const float w2 = p.density * p.accel / 36.f;
        const bool xdec = s.remote[DE] || s.remote[DW];
        const bool ydec = s.remote[DN] || s.remote[DS];
        std::vector<Rect> interior, boundary;
        if (!xdec && !ydec) {
            interior.push_back(Rect{0, 0, s.w, s.h});
        } else {
            // boundary strips: rows 0 and h-1; with x decomposed also the
            // outermost column chunk on each side
            const int cw = vec4 ? 4 : 1;
            boundary.push_back(Rect{0, 0, s.w, 1});
            if (s.h > 1) boundary.push_back(Rect{0, s.h - 1, s.w, 1});
            const int ih = s.h - 2;
            if (xdec) {
                if (ih > 0) {
                    boundary.push_back(Rect{0, 1, cw, ih});
                    if (s.w > cw) boundary.push_back(Rect{s.w - cw, 1, cw, ih});
                    if (s.w > 2 * cw) interior.push_back(Rect{cw, 1, s.w - 2 * cw, ih});
                }
            } else if (ih > 0) {
                interior.push_back(Rect{0, 1, s.w, ih});
            }
            if (!ydec && !xdec) interior.clear();
        }
        int bi = 1, bb = 0;
        StepArgs base{};
        base.plane = s.plane;
        base.pitch = s.pitch;
        base.w = s.w;
        base.h = s.h;
        base.obst = s.obst;
        base.accel_row = s.accel_row;
        base.omega = p.omega;
        base.omo = 1 - p.omega;
        base.w1 = w1;
        base.w2 = w2;
        base.ctl = s.ctl;
        StepArgs ai = base, ab = base;
        fill_rects(ai, interior, bi);
        if (!boundary.empty()) fill_rects(ab, boundary, bb);
        s.n_int_blocks = bi;
        s.n_bnd_blocks = boundary.empty() ? 0 : bb;
        const int np = s.n_int_blocks + s.n_bnd_blocks;
        for (int k = 0; k < 2; ++k) {
            if (s.partials[k]) HIP_CHECK(hipFree(s.partials[k]));
            HIP_CHECK(hipMalloc(&s.partials[k], sizeof(float) * (size_t)round_up(np, 64)));
            HIP_CHECK(hipMemset(s.partials[k], 0, sizeof(float) * (size_t)round_up(np, 64)));
        }
        for (int par = 0; par < 2; ++par) {
            float *fin = s.f[par], *fout = s.f[1 - par];
            for (StepArgs *a : {&ai, &ab}) {
                a->fin = fin;
                a->fout = fout;
                for (int d = 0; d < 8; ++d) a->dst[d] = make_dst(s, fout, d);
                a->partials_prev = s.partials[1 - par];
                a->n_prev = np;
                a->av_local = s.av_local;
            }
            ai.partials_out = s.partials[par];
            ab.partials_out = s.partials[par] + s.n_int_blocks;
            s.args_int[par] = ai;
            s.args_bnd[par] = ab;
            HaloArgs u{};
            u.f = fout;
            u.plane = s.plane;
            u.pitch = s.pitch;
            u.w = s.w;
            u.h = s.h;
            for (int e = 0; e < 8; ++e) {
                if (s.remote[e]) u.mask |= 1u << e;
                u.recv[e] = s.recv[e];
            }
            s.unpack[par] = u;
        }
    }

    void ensure_av(int n) {
        for (auto &s : subs) {
            if (s.av_cap >= n) continue;
            drop_graphs();
            set_device(s);
            if (s.av_local) HIP_CHECK(hipFree(s.av_local));
            s.av_cap = std::max(n, 1);
            HIP_CHECK(hipMalloc(&s.av_local, sizeof(float) * (size_t)s.av_cap));
            HIP_CHECK(hipMemset(s.av_local, 0, sizeof(float) * (size_t)s.av_cap));
            for (int par = 0; par < 2; ++par) {
                s.args_int[par].av_local = s.av_local;
                s.args_bnd[par].av_local = s.av_local;
            }
        }
    }

    // ------------------------------------------------------------------
    void create(const lbm_params *prm, const uint8_t *obstacles, const lbm_config &cfg) {
        p = *prm;
        if (p.nx <= 0 || p.ny <= 0 || p.max_iters < 0) throw lbm_failure(LBM_E_INVALID, "nx, ny must be > 0 and max_iters >= 0");
        if (!obstacles) throw lbm_failure(LBM_E_INVALID, "obstacles must not be NULL");
        parts = cfg.parts > 0 ? cfg.parts : 1;
        transport = cfg.transport;
        read_tuning();  // environment knobs first; explicit config wins
        if (cfg.graph_steps > 0) graph_steps = cfg.graph_steps;
        if (cfg.graph_steps < 0) graph_steps = 0;
        force_exchange = (cfg.flags & LBM_FLAG_FORCE_EXCHANGE) != 0 || env_int("LBM_FORCE_EXCHANGE", 0) != 0;
        if (partition(p.nx, p.ny, parts, cfg.grid_rows, cfg.grid_cols, R, C, all_rects) != LBM_OK)
            throw lbm_failure(LBM_E_INVALID, "cannot partition " + std::to_string(p.nx) + "x" + std::to_string(p.ny) +
                                                 " into " + std::to_string(parts) + " parts");
        int ndev = 0;
        HIP_CHECK(hipGetDeviceCount(&ndev));
        if (ndev <= 0) throw lbm_failure(LBM_E_HIP, "no HIP device visible");

        free_cells = 0;
        for (long long i = 0; i < (long long)p.nx * p.ny; ++i) free_cells += obstacles[i] ? 0 : 1;

        // kernel choice
        bool can_vec = true;
        for (auto &r : all_rects) {
            if (r.w % 4 != 0) can_vec = false;
            if (C > 1 && r.w < 8) can_vec = false;
        }
        if (cfg.kernel == LBM_KERNEL_VEC4 && !can_vec)
            throw lbm_failure(LBM_E_INVALID, "vec4 kernel needs sub-domain widths that are multiples of 4 (>= 8 when split in x)");
        vec4 = (cfg.kernel == LBM_KERNEL_SCALAR) ? false : can_vec;

        std::vector<int> mine;
        if (transport == LBM_TRANSPORT_RCCL) {
            if (cfg.world != parts || cfg.rank < 0 || cfg.rank >= parts)
                throw lbm_failure(LBM_E_INVALID, "RCCL transport needs world == parts and 0 <= rank < world");
            if (!cfg.rccl_unique_id) throw lbm_failure(LBM_E_INVALID, "RCCL transport needs rccl_unique_id");
            rank = cfg.rank;
            world = cfg.world;
            mine.push_back(rank);
        } else if (transport == LBM_TRANSPORT_LOCAL) {
            for (int i = 0; i < parts; ++i) mine.push_back(i);
        } else {
            throw lbm_failure(LBM_E_INVALID, "unknown transport");
        }

        subs.resize(mine.size());
        for (size_t k = 0; k < mine.size(); ++k) {
            Sub &s = subs[k];
            s.id = mine[k];
            s.row = s.id / C;
            s.col = s.id % C;
            if (transport == LBM_TRANSPORT_RCCL)
                s.dev = (cfg.devices && cfg.num_devices > 0) ? cfg.devices[0] : rank % ndev;
            else
                s.dev = (cfg.devices && cfg.num_devices > 0) ? cfg.devices[s.id % cfg.num_devices] : s.id % ndev;
            if (s.dev < 0 || s.dev >= ndev) throw lbm_failure(LBM_E_INVALID, "device index out of range");
            s.rect = all_rects[s.id];
            s.w = s.rect.w;
            s.h = s.rect.h;
            for (int d = 0; d < 8; ++d) {
                const int r = ((s.row + DIR_Y[d]) % R + R) % R;
                const int c = ((s.col + DIR_X[d]) % C + C) % C;
                s.nb[d] = r * C + c;
                s.remote[d] = force_exchange || s.nb[d] != s.id;
            }
            const int gy = p.ny - 2;
            s.accel_row = (p.ny >= 2 && gy >= s.rect.y0 && gy < s.rect.y0 + s.h) ? gy - s.rect.y0 : -1;
            alloc_sub(s, obstacles);
        }
        if (transport == LBM_TRANSPORT_RCCL) {
            ncclUniqueId id;
            static_assert(sizeof(id) == 128, "unexpected ncclUniqueId size");
            memcpy(&id, cfg.rccl_unique_id, sizeof(id));
            set_device(subs[0]);
            NCCL_CHECK(ncclCommInitRank(&comm, world, id, rank));
        } else if (subs.size() > 1) {
            // peer access between the devices of this process (copies work without it, just slower)
            for (auto &a : subs)
                for (auto &b : subs)
                    if (a.dev != b.dev) {
                        int can = 0;
                        HIP_CHECK(hipDeviceCanAccessPeer(&can, a.dev, b.dev));
                        if (can) {
                            HIP_CHECK(hipSetDevice(a.dev));
                            hipError_t e = hipDeviceEnablePeerAccess(b.dev, 0);
                            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIP_CHECK(e);
                            (void)hipGetLastError();
                        }
                    }
        }
        for (auto &s : subs) {
            set_device(s);
            build_args(s);
        }
        ensure_av(std::max(p.max_iters, 1));
        set_device(subs[0]);
        HIP_CHECK(hipEventCreate(&t0));
        HIP_CHECK(hipEventCreate(&t1));
    }

    void alloc_sub(Sub &s, const uint8_t *obstacles) {
        set_device(s);
        const int row_floats = (int)round_up(s.w + XOFF + 1, 64);
        const long long rows = s.h + 2;
        long long total_floats;
        if (row_interleaved) {
            // f[y][k][x]: the nine populations of a row are adjacent
            s.plane = row_floats;
            s.pitch = Q * row_floats;
            total_floats = rows * s.pitch;
        } else {
            // f[k][y][x]: plane stride padded off a power of two so the nine
            // concurrent plane streams do not alias
            s.pitch = row_floats;
            s.plane = round_up(rows * s.pitch, 1024) + 320;
            total_floats = Q * s.plane;
        }
        s.lattice_floats = total_floats;
        for (int k = 0; k < 2; ++k) {
            HIP_CHECK(hipMalloc(&s.f[k], sizeof(float) * (size_t)total_floats));
            HIP_CHECK(hipMemset(s.f[k], 0, sizeof(float) * (size_t)total_floats));
        }
        HIP_CHECK(hipMalloc(&s.obst, (size_t)round_up((long long)s.w * s.h + 16, 256)));
        HIP_CHECK(hipMemcpy2D(s.obst, (size_t)s.w, obstacles + (size_t)s.rect.y0 * p.nx + s.rect.x0, (size_t)p.nx,
                              (size_t)s.w, (size_t)s.h, hipMemcpyHostToDevice));
        // halo buffers (only for directions that cross sub-domains)
        long long total = 0;
        long long off_send[8], off_recv[8];
        for (int d = 0; d < 8; ++d) {
            const long long n = s.remote[d] ? round_up((long long)NPLANES[d] * edge_len(d, s.w, s.h), 64) : 0;
            off_send[d] = total;
            total += n;
            off_recv[d] = total;
            total += n;
        }
        if (total > 0) {
            HIP_CHECK(hipMalloc(&s.halo_mem, sizeof(float) * (size_t)total));
            HIP_CHECK(hipMemset(s.halo_mem, 0, sizeof(float) * (size_t)total));
            for (int d = 0; d < 8; ++d) {
                s.send[d] = s.remote[d] ? s.halo_mem + off_send[d] : nullptr;
                s.recv[d] = s.remote[d] ? s.halo_mem + off_recv[d] : nullptr;
            }
        }
        HIP_CHECK(hipMalloc(&s.ctl, 64));
        HIP_CHECK(hipMemset(s.ctl, 0, 64));
        HIP_CHECK(hipStreamCreateWithFlags(&s.s_comp, hipStreamNonBlocking));
        HIP_CHECK(hipStreamCreateWithFlags(&s.s_comm, hipStreamNonBlocking));
        HIP_CHECK(hipEventCreateWithFlags(&s.ev_b, hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&s.ev_u, hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&s.ev_end, hipEventDisableTiming));
    }

    Sub *local_sub(int id) {
        for (auto &s : subs)
            if (s.id == id) return &s;
        return nullptr;
    }

    // ------------------------------------------------------------------
    // Exchange of the halo send buffers, after every sub-domain recorded
    // ev_b on its compute stream.  Ends with the unpack into `unpack_args`
    // and ev_u recorded on each comm stream.
    void exchange(const HaloArgs *unpack_args_per_sub) {
        if (transport == LBM_TRANSPORT_RCCL) {
            Sub &s = subs[0];
            set_device(s);
            HIP_CHECK(hipStreamWaitEvent(s.s_comm, s.ev_b, 0));
            NCCL_CHECK(ncclGroupStart());
            for (int d = 0; d < 8; ++d) {
                // send the populations leaving through d to the neighbour on
                // side d; receive into ghost side OPP(d) from the neighbour on
                // that side.  Both peers enumerate d in the same order, so
                // repeated peers (extent-2 dimensions) match in order.
                if (s.remote[d])
                    NCCL_CHECK(ncclSend(s.send[d], (size_t)NPLANES[d] * edge_len(d, s.w, s.h), ncclFloat, s.nb[d],
                                        comm, s.s_comm));
                const int e = OPP_DIR[d];
                if (s.remote[e])
                    NCCL_CHECK(ncclRecv(s.recv[e], (size_t)NPLANES[e] * edge_len(e, s.w, s.h), ncclFloat, s.nb[e],
                                        comm, s.s_comm));
            }
            NCCL_CHECK(ncclGroupEnd());
            HIP_CHECK(launch_halo_unpack(unpack_args_per_sub[0], s.s_comm));
            HIP_CHECK(hipEventRecord(s.ev_u, s.s_comm));
            return;
        }
        // LOCAL: receiver pulls each message with a device (peer) copy
        for (size_t k = 0; k < subs.size(); ++k) {
            Sub &s = subs[k];
            set_device(s);
            for (int e = 0; e < 8; ++e) {
                if (!s.remote[e]) continue;
                Sub *src = local_sub(s.nb[e]);
                if (!src) throw lbm_failure(LBM_E_INTERNAL, "missing local neighbour");
                HIP_CHECK(hipStreamWaitEvent(s.s_comm, src->ev_b, 0));
                const size_t bytes = sizeof(float) * (size_t)NPLANES[e] * edge_len(e, s.w, s.h);
                const float *from = src->send[OPP_DIR[e]];
                if (src->dev == s.dev)
                    HIP_CHECK(hipMemcpyAsync(s.recv[e], from, bytes, hipMemcpyDeviceToDevice, s.s_comm));
                else
                    HIP_CHECK(hipMemcpyPeerAsync(s.recv[e], s.dev, from, src->dev, bytes, s.s_comm));
            }
            HIP_CHECK(launch_halo_unpack(unpack_args_per_sub[k], s.s_comm));
            HIP_CHECK(hipEventRecord(s.ev_u, s.s_comm));
        }
    }

    // Compute streams wait for the exchange: own ghosts unpacked, and (LOCAL)
    // every neighbour done reading this sub-domain's send buffers.
    void wait_exchange() {
        for (auto &s : subs) {
            set_device(s);
            HIP_CHECK(hipStreamWaitEvent(s.s_comp, s.ev_u, 0));
            if (transport == LBM_TRANSPORT_LOCAL)
                for (int d = 0; d < 8; ++d)
                    if (s.remote[d]) HIP_CHECK(hipStreamWaitEvent(s.s_comp, local_sub(s.nb[d])->ev_u, 0));
        }
    }

    // Make every ghost cell of the current lattices consistent (after load,
    // init or accelerate).
    void refresh_halos() {
        std::vector<HaloArgs> unp(subs.size());
        for (size_t k = 0; k < subs.size(); ++k) {
            Sub &s = subs[k];
            set_device(s);
            HaloArgs a{};
            a.f = s.f[s.cur];
            a.plane = s.plane;
            a.pitch = s.pitch;
            a.w = s.w;
            a.h = s.h;
            a.mask = 0xffu;
            for (int d = 0; d < 8; ++d) a.dst[d] = make_dst(s, s.f[s.cur], d);
            HIP_CHECK(launch_halo_pack(a, s.s_comp));
            HIP_CHECK(hipEventRecord(s.ev_b, s.s_comp));
            unp[k] = s.unpack[1 - s.cur];  // unpack args of the step that produced lattice `cur`
            unp[k].f = s.f[s.cur];
        }
        if (multi()) {
            exchange(unp.data());
            wait_exchange();
        }
    }

    void step_once() {
        if (!multi()) {
            Sub &s = subs[0];
            HIP_CHECK(launch_step(s.args_int[s.cur], s.n_int_blocks, vec4, true, kflags, kwaves, s.s_comp));
            s.cur ^= 1;
            return;
        }
        std::vector<HaloArgs> unp(subs.size());
        for (size_t k = 0; k < subs.size(); ++k) {
            Sub &s = subs[k];
            set_device(s);
            if (s.n_bnd_blocks > 0)
                HIP_CHECK(launch_step(s.args_bnd[s.cur], s.n_bnd_blocks, vec4, false, kflags, kwaves, s.s_comp));
            HIP_CHECK(hipEventRecord(s.ev_b, s.s_comp));
            unp[k] = s.unpack[s.cur];
        }
        exchange(unp.data());
        for (auto &s : subs) {
            set_device(s);
            HIP_CHECK(launch_step(s.args_int[s.cur], s.n_int_blocks, vec4, true, kflags, kwaves, s.s_comp));
        }
        wait_exchange();
        for (auto &s : subs) s.cur ^= 1;
    }

    void drop_graphs() {
        for (auto &g : graph_exec)
            if (g) {
                (void)hipGraphExecDestroy(g);
                g = nullptr;
            }
    }

    // Capture 2*graph_steps steps starting at parity `par` (single sub-domain):
    // the launch-bound small grids replay them instead of paying a host
    // launch per step.  Kernel arguments are per parity and the av index is
    // device-side, so one graph serves every replay.
    hipGraphExec_t graph_for(int par) {
        if (graph_exec[par]) return graph_exec[par];
        Sub &s = subs[0];
        set_device(s);
        hipGraph_t g = nullptr;
        HIP_CHECK(hipStreamBeginCapture(s.s_comp, hipStreamCaptureModeThreadLocal));
        int cur = par;
        for (int i = 0; i < 2 * graph_steps; ++i) {
            const hipError_t e = launch_step(s.args_int[cur], s.n_int_blocks, vec4, true, kflags, kwaves, s.s_comp);
            if (e != hipSuccess) {
                hipGraph_t junk = nullptr;
                (void)hipStreamEndCapture(s.s_comp, &junk);
                if (junk) (void)hipGraphDestroy(junk);
                HIP_CHECK(e);
            }
            cur ^= 1;
        }
        HIP_CHECK(hipStreamEndCapture(s.s_comp, &g));
        hipGraphExec_t ge = nullptr;
        const hipError_t e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        HIP_CHECK(e);
        graph_exec[par] = ge;
        return ge;
    }

    void run_steps(int steps, bool accelerate_first) {
        if (!loaded) throw lbm_failure(LBM_E_STATE, "lattice not initialised (call lbm_load_cells or lbm_init_equilibrium)");
        if (steps < 0) throw lbm_failure(LBM_E_INVALID, "steps must be >= 0");
        ensure_av(std::max(steps, 1));
        for (auto &s : subs) {
            set_device(s);
            HIP_CHECK(hipMemsetAsync(s.ctl, 0, 64, s.s_comp));
            HIP_CHECK(hipStreamSynchronize(s.s_comp));
        }
        if (multi()) sync_all();
        const int chunk = 2 * graph_steps;
        const bool use_graph = !multi() && graph_steps > 0 && steps >= chunk;
        if (use_graph) (void)graph_for(subs[0].cur);  // capture + instantiate outside the timed region
        Sub &s0 = subs[0];
        set_device(s0);
        HIP_CHECK(hipEventRecord(t0, s0.s_comp));
        if (multi())
            for (size_t k = 1; k < subs.size(); ++k) {
                set_device(subs[k]);
                HIP_CHECK(hipStreamWaitEvent(subs[k].s_comp, t0, 0));
            }
        if (accelerate_first && p.ny >= 2) {
            const float w1 = p.density * p.accel / 9.f;
            const float w2 = p.density * p.accel / 36.f;
            for (auto &s : subs) {
                if (s.accel_row < 0) continue;
                set_device(s);
                HIP_CHECK(launch_accelerate(s.f[s.cur], s.obst, s.plane, s.pitch, s.w, s.accel_row, w1, w2, s.s_comp));
            }
            refresh_halos();
        }
        int t = 0;
        if (use_graph) {
            hipGraphExec_t ge = graph_for(s0.cur);  // even chunk: parity unchanged per replay
            for (; t + chunk <= steps; t += chunk) HIP_CHECK(hipGraphLaunch(ge, s0.s_comp));
        }
        for (; t < steps; ++t) step_once();
        for (auto &s : subs) {
            set_device(s);
            const int np = s.n_int_blocks + s.n_bnd_blocks;
            HIP_CHECK(launch_finalize(s.partials[1 - s.cur], np, s.av_local, s.ctl, s.s_comp));
            HIP_CHECK(hipEventRecord(s.ev_end, s.s_comp));
        }
        set_device(s0);
        for (size_t k = 1; k < subs.size(); ++k) HIP_CHECK(hipStreamWaitEvent(s0.s_comp, subs[k].ev_end, 0));
        HIP_CHECK(hipEventRecord(t1, s0.s_comp));
        HIP_CHECK(hipEventSynchronize(t1));
        float ms = 0.f;
        HIP_CHECK(hipEventElapsedTime(&ms, t0, t1));
        last_seconds = ms * 1e-3;
        last_steps = steps;
        sync_all();
    }

    void sync_all() {
        for (auto &s : subs) {
            set_device(s);
            HIP_CHECK(hipStreamSynchronize(s.s_comp));
            HIP_CHECK(hipStreamSynchronize(s.s_comm));
        }
    }

    void init_equilibrium() {
        const float c0 = p.density * 4.f / 9.f, c1 = p.density / 9.f, c2 = p.density / 36.f;
        for (auto &s : subs) {
            set_device(s);
            s.cur = 0;
            HIP_CHECK(launch_init_equilibrium(s.f[0], s.h + 2, (int)std::min<long long>(s.pitch, s.plane), s.pitch,
                                              s.plane, c0, c1, c2, s.s_comp));
        }
        sync_all();
        loaded = true;
    }

    void load_cells(const float *aos) {
        if (!aos) throw lbm_failure(LBM_E_INVALID, "cells must not be NULL");
        for (auto &s : subs) {
            set_device(s);
            float *stage = nullptr;
            const size_t row_bytes = sizeof(float) * Q * (size_t)s.w;
            HIP_CHECK(hipMalloc(&stage, row_bytes * (size_t)s.h));
            HIP_CHECK(hipMemcpy2D(stage, row_bytes, aos + ((size_t)s.rect.y0 * p.nx + s.rect.x0) * Q,
                                  sizeof(float) * Q * (size_t)p.nx, row_bytes, (size_t)s.h, hipMemcpyHostToDevice));
            s.cur = 0;
            HIP_CHECK(launch_aos_to_soa(stage, s.f[0], s.plane, s.pitch, s.w, s.h, s.s_comp));
            HIP_CHECK(hipStreamSynchronize(s.s_comp));
            HIP_CHECK(hipFree(stage));
        }
        refresh_halos();
        sync_all();
        loaded = true;
    }

    void store(float *aos, float *av, int n_av) {
        if (!loaded) throw lbm_failure(LBM_E_STATE, "nothing to store");
        sync_all();
        if (aos) {
            for (auto &s : subs) {
                set_device(s);
                float *stage = nullptr;
                const size_t row_bytes = sizeof(float) * Q * (size_t)s.w;
                HIP_CHECK(hipMalloc(&stage, row_bytes * (size_t)s.h));
                HIP_CHECK(launch_soa_to_aos(s.f[s.cur], stage, s.plane, s.pitch, s.w, s.h, s.s_comp));
                HIP_CHECK(hipStreamSynchronize(s.s_comp));
                HIP_CHECK(hipMemcpy2D(aos + ((size_t)s.rect.y0 * p.nx + s.rect.x0) * Q, sizeof(float) * Q * (size_t)p.nx,
                                      stage, row_bytes, row_bytes, (size_t)s.h, hipMemcpyDeviceToHost));
                HIP_CHECK(hipFree(stage));
            }
        }
        if (av && n_av > 0) {
            const int n = std::min(n_av, last_steps);
            std::vector<float> per((size_t)parts * std::max(n, 1), 0.f);
            if (n > 0) {
                if (transport == LBM_TRANSPORT_RCCL) {
                    Sub &s = subs[0];
                    set_device(s);
                    float *gath = nullptr;
                    HIP_CHECK(hipMalloc(&gath, sizeof(float) * (size_t)n * world));
                    NCCL_CHECK(ncclAllGather(s.av_local, gath, (size_t)n, ncclFloat, comm, s.s_comm));
                    HIP_CHECK(hipStreamSynchronize(s.s_comm));
                    HIP_CHECK(hipMemcpy(per.data(), gath, sizeof(float) * (size_t)n * world, hipMemcpyDeviceToHost));
                    HIP_CHECK(hipFree(gath));
                } else {
                    for (auto &s : subs) {
                        set_device(s);
                        HIP_CHECK(hipMemcpy(per.data() + (size_t)s.id * n, s.av_local, sizeof(float) * (size_t)n,
                                            hipMemcpyDeviceToHost));
                    }
                }
            }
            const float fc = (float)free_cells;
            for (int t = 0; t < n_av; ++t) {
                if (t >= n) {
                    av[t] = 0.f;
                    continue;
                }
                float tot = 0.f;
                for (int r = 0; r < parts; ++r) tot += per[(size_t)r * n + t];  // fixed rank order
                av[t] = tot / fc;
            }
        }
    }

    void destroy() {
        drop_graphs();
        for (auto &s : subs) {
            if (hipSetDevice(s.dev) != hipSuccess) continue;
            (void)hipDeviceSynchronize();
            for (int k = 0; k < 2; ++k) {
                if (s.f[k]) (void)hipFree(s.f[k]);
                if (s.partials[k]) (void)hipFree(s.partials[k]);
            }
            if (s.obst) (void)hipFree(s.obst);
            if (s.halo_mem) (void)hipFree(s.halo_mem);
            if (s.av_local) (void)hipFree(s.av_local);
            if (s.ctl) (void)hipFree(s.ctl);
            if (s.s_comp) (void)hipStreamDestroy(s.s_comp);
            if (s.s_comm) (void)hipStreamDestroy(s.s_comm);
            if (s.ev_b) (void)hipEventDestroy(s.ev_b);
            if (s.ev_u) (void)hipEventDestroy(s.ev_u);
            if (s.ev_end) (void)hipEventDestroy(s.ev_end);
        }
        if (comm) (void)ncclCommDestroy(comm);
        if (t0) (void)hipEventDestroy(t0);
        if (t1) (void)hipEventDestroy(t1);
    }
};

// --------------------------------------------------------------------------
// C ABI
// --------------------------------------------------------------------------
namespace {
thread_local std::string g_create_error;

template <class F>
int guarded(lbm_handle *h, F &&f) {
    try {
        f();
        return LBM_OK;
    } catch (const lbm_failure &e) {
        if (h) h->err = e.what();
        return e.code;
    } catch (const std::bad_alloc &) {
        if (h) h->err = "host allocation failed";
        return LBM_E_NOMEM;
    } catch (const std::exception &e) {
        if (h) h->err = e.what();
        return LBM_E_INTERNAL;
    } catch (...) {
        if (h) h->err = "unknown failure";
        return LBM_E_INTERNAL;
    }
}
}  // namespace

extern "C" {

int32_t lbm_abi_version(void) { return LBM_ABI_VERSION; }

int lbm_partition(int32_t nx, int32_t ny, int32_t parts, int32_t grid_rows, int32_t grid_cols, int32_t *rows_out,
                  int32_t *cols_out, lbm_rect *rects) {
    int R = 0, C = 0;
    std::vector<lbm_rect> v;
    const int rc = partition(nx, ny, parts, grid_rows, grid_cols, R, C, v);
    if (rc != LBM_OK) return rc;
    if (rows_out) *rows_out = R;
    if (cols_out) *cols_out = C;
    if (rects)
        for (int i = 0; i < parts; ++i) rects[i] = v[i];
    return LBM_OK;
}

int lbm_halo_plan(int32_t table[48]) {
    if (!table) return LBM_E_INVALID;
    for (int d = 0; d < 8; ++d) {
        int32_t *t = table + 6 * d;
        t[0] = DIR_X[d];
        t[1] = DIR_Y[d];
        t[2] = NPLANES[d];
        for (int i = 0; i < 3; ++i) t[3 + i] = PLANES[d][i];
    }
    return LBM_OK;
}

int32_t lbm_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

int lbm_rccl_unique_id(uint8_t out[128]) {
    if (!out) return LBM_E_INVALID;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return LBM_E_RCCL;
    memcpy(out, &id, sizeof(id));
    return LBM_OK;
}

int lbm_create_ex(const lbm_params *params, const uint8_t *obstacles, const lbm_config *config, lbm_handle **out) {
    if (!params || !config || !out) return LBM_E_INVALID;
    *out = nullptr;
    auto *h = new (std::nothrow) lbm_handle();
    if (!h) return LBM_E_NOMEM;
    const int rc = guarded(h, [&] { h->create(params, obstacles, *config); });
    if (rc != LBM_OK) {
        g_create_error = h->err;
        h->destroy();
        delete h;
        return rc;
    }
    *out = h;
    return LBM_OK;
}

int lbm_create(const lbm_params *params, const uint8_t *obstacles, int32_t num_gpus, lbm_handle **out) {
    lbm_config cfg{};
    cfg.parts = num_gpus > 0 ? num_gpus : 1;
    cfg.transport = LBM_TRANSPORT_LOCAL;
    return lbm_create_ex(params, obstacles, &cfg, out);
}

int lbm_load_cells(lbm_handle *h, const float *cells_aos) {
    if (!h) return LBM_E_INVALID;
    return guarded(h, [&] { h->load_cells(cells_aos); });
}

int lbm_init_equilibrium(lbm_handle *h) {
    if (!h) return LBM_E_INVALID;
    return guarded(h, [&] { h->init_equilibrium(); });
}

int lbm_run(lbm_handle *h) {
    if (!h) return LBM_E_INVALID;
    return guarded(h, [&] { h->run_steps(h->p.max_iters, true); });
}

int lbm_run_steps(lbm_handle *h, int32_t steps, int32_t accelerate_first) {
    if (!h) return LBM_E_INVALID;
    return guarded(h, [&] { h->run_steps(steps, accelerate_first != 0); });
}

int lbm_store(lbm_handle *h, float *cells_aos, float *av_vels, int32_t n_av) {
    if (!h) return LBM_E_INVALID;
    return guarded(h, [&] { h->store(cells_aos, av_vels, n_av); });
}

int lbm_last_run_seconds(lbm_handle *h, double *seconds) {
    if (!h || !seconds) return LBM_E_INVALID;
    *seconds = h->last_seconds;
    return LBM_OK;
}

int64_t lbm_total_free_cells(lbm_handle *h) { return h ? h->free_cells : -1; }

int lbm_local_rects(lbm_handle *h, lbm_rect *rects, int32_t max_rects, int32_t *n_out) {
    if (!h) return LBM_E_INVALID;
    const int n = (int)h->subs.size();
    if (n_out) *n_out = n;
    if (rects)
        for (int i = 0; i < n && i < max_rects; ++i) rects[i] = h->subs[i].rect;
    return LBM_OK;
}

int32_t lbm_kernel_in_use(lbm_handle *h) { return (h && h->vec4) ? LBM_KERNEL_VEC4 : LBM_KERNEL_SCALAR; }

const char *lbm_last_error(lbm_handle *h) { return h ? h->err.c_str() : g_create_error.c_str(); }

void lbm_destroy(lbm_handle *h) {
    if (!h) return;
    try {
        h->destroy();
    } catch (...) {
    }
    delete h;
}

}  // extern "C"
