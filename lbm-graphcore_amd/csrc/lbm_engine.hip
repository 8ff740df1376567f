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
//   * Fused mode (default): each launch advances spl time steps -- the
//     register-streaming kernel (lbm_stream.hip, spl = 2..4) or the LDS
//     two-step kernel (lbm_step2.hip, spl = 2) -- and the halo is spl cells
//     wide with all nine populations (WG); remaining steps (steps % spl) run
//     the one-step kernel (W1 halo) and then refresh the WG ring.
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
#include <array>
#include <vector>

#include "lbm_hip.h"
#include "lbm_layout.hpp"

namespace lbm {
hipError_t launch_step(const StepArgs &a, int blocks, bool vec4, bool reduce, hipStream_t s);
hipError_t launch_step2(const Step2Args &a, int blocks, bool reduce, hipStream_t s);
hipError_t launch_stream2d(const StreamArgs &a, int units, int steps, bool reduce, int cfg, bool tol, hipStream_t s);
hipError_t stream2d_blocks_per_cu(int steps, int cfg, bool tol, int &n);
bool s2d_form_ok(int steps, int cfg, bool tol);
hipError_t stream2d_unit_flags(const StreamArgs &a, int steps, uint8_t *uobst, hipStream_t s);
hipError_t launch_finalize(const float *partials, float *av_local, int *ctl, hipStream_t s);
hipError_t launch_accelerate(float *f, const uint8_t *obst, long long P, int pitch, int w, int row, float w1,
                             float w2, hipStream_t s);
hipError_t launch_init_equilibrium(float *base, long long rows, int rf, int pitch, long long P, float c0, float c1,
                                   float c2, hipStream_t s);
hipError_t launch_aos_to_soa(const float *aos, float *f, long long P, int pitch, int w, int h, hipStream_t s);
hipError_t launch_count_nonfinite(const float *f, long long P, int pitch, int w, int h, unsigned long long *out,
                                  hipStream_t s);
hipError_t launch_soa_to_aos(const float *f, float *aos, long long P, int pitch, int w, int h, hipStream_t s);
hipError_t launch_halo_pack(const HaloArgs &a, hipStream_t s);
hipError_t launch_halo_unpack(const HaloArgs &a, hipStream_t s);
hipError_t resident_capacity(int variant, int device, bool tol, int &capacity);
int pipe_blocks(int w, int h);
hipError_t launch_pipe_propagate(const float *f, float *t, long long P, int pitch, int w, int h, hipStream_t s);
hipError_t launch_pipe_rebound(const float *t, float *f, const uint8_t *obst, long long P, int pitch, int w, int h,
                               hipStream_t s);
hipError_t launch_pipe_collision(const float *t, float *f, const uint8_t *obst, long long P, int pitch, int w, int h,
                                 float omega, float *partials, hipStream_t s);
hipError_t launch_pipe_av(const float *partials, int n, float *av_local, int t, hipStream_t s);
hipError_t launch_resident(const ResidentArgs &a, int variant, bool tol, bool coop, hipStream_t s);
hipError_t launch_resident_reduce(const float *partials, float *av_local, int steps, int ntiles, hipStream_t s);
hipError_t launch_debug_spin(int microseconds, hipStream_t s);
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

// Neighbours of sub-domain `id` on the R x C periodic torus of the
// reference's partition (rank = row * C + col; the periodic halo slices of
// StructuredGridUtils.hpp:805-851): nb[d] = the sub-domain across side d;
// remote[d] = side d goes through the exchange (else the step kernel writes
// the periodic image straight into the ghost ring).
void torus_neighbours(int id, int R, int C, bool force_exchange, int nb[8], bool remote[8]) {
    const int row = id / C, col = id % C;
    for (int d = 0; d < 8; ++d) {
        const int r = ((row + DIR_Y[d]) % R + R) % R;
        const int c = ((col + DIR_X[d]) % C + C) % C;
        nb[d] = r * C + c;
        remote[d] = force_exchange || nb[d] != id;
    }
}

// The ordered transfers of one sub-domain's halo exchange (format `mode`,
// WG width `hw`): for d = E, N, W, S, NE, NW, SW, SE the send of the halo
// leaving through side d to nb[d] (or SELF: written in place by the step
// kernel), then the receive of ghost side OPP(d) from nb[OPP(d)].  RCCL
// pairs the messages between two ranks purely by this posting order (one
// ncclGroupStart/End), which is what lets extent-2 dimensions send several
// messages to one peer.  exchange() posts exactly this list;
// lbm_exchange_schedule exports it for host-side checking.
std::vector<lbm_xfer> exchange_posts(int id, const int nb[8], const bool remote[8], int w, int h, int mode, int hw) {
    std::vector<lbm_xfer> v;
    for (int d = 0; d < 8; ++d) {
        v.push_back(lbm_xfer{remote[d] ? LBM_XFER_SEND : LBM_XFER_SELF, d, remote[d] ? nb[d] : id, 0,
                             msg_floats(mode, d, w, h, hw)});
        const int e = OPP_DIR[d];
        if (remote[e]) v.push_back(lbm_xfer{LBM_XFER_RECV, e, nb[e], 0, msg_floats(mode, e, w, h, hw)});
    }
    return v;
}

struct Sub {
    int id = 0, row = 0, col = 0, dev = 0;
    lbm_rect rect{};
    int w = 0, h = 0, pitch = 0, rf = 0;
    long long plane = 0;
    long long lattice_floats = 0, origin_off = 0;
    float *f[2] = {nullptr, nullptr};   // allocations
    bool f_joint = false;                // f[1] lies in f[0]'s allocation (LBM_LATTICE_PAD)
    float *o[2] = {nullptr, nullptr};   // origins: cell (0,0), plane 0
    uint8_t *obst = nullptr;            // [h][w]
    uint8_t *obst_g = nullptr;          // [(h+2og)][(w+2og)], periodic / neighbour images in the ring
    float *halo_mem = nullptr;          // all send + recv buffers
    float *send[8] = {};
    float *recv[8] = {};
    int nb[8] = {};                     // neighbour sub id / rank per direction
    bool remote[8] = {};
    float *partials[2] = {nullptr, nullptr};
    int n1_int = 0, n1_bnd = 0;         // one-step launch block counts
    int n2_int = 0, n2_bnd = 0;         // two-step launch block counts
    float *av_local = nullptr;
    int av_cap = 0;
    int *ctl = nullptr;
    int accel_row = -1;
    // s_comp: interior launches and everything else; s_bnd (high priority):
    // boundary launches of multi-sub-domain runs; s_comm: halo exchange.
    hipStream_t s_comp = nullptr, s_comm = nullptr, s_bnd = nullptr;
    hipEvent_t ev_b = nullptr, ev_u = nullptr, ev_end = nullptr;
    hipEvent_t ev_i = nullptr;                  // interior launch done (s_comp)
    hipEvent_t ev_bp[2] = {nullptr, nullptr};   // boundary launch done, per parity (s_bnd)
    StepArgs a1_int[2]{}, a1_bnd[2]{};      // per parity (parity = lattice read)
    Step2Args a2_int[2]{}, a2_bnd[2]{};
    StreamArgs a3_int[2]{}, a3_bnd[2]{};
    int n3_int = 0, n3_bnd = 0;             // stream launch block counts
    int cur = 0;                            // lattice holding the current state
    float *pipe_partials = nullptr;         // PIPELINE: collision block partials
    Dst2 *dst2_dev = nullptr;               // [parity][8] stream-kernel halo destinations (StreamArgs::dstg)
    unsigned long long *trace = nullptr;    // LBM_STREAM_TRACE: per-wave timestamps of the last interior launch
    uint8_t *uobst = nullptr;               // v3 per-unit obstacle flags: [interior units | boundary units]
    int *uperm = nullptr;                   // v3 dispatch order: [interior | boundary]
};

}  // namespace

struct lbm_handle {
    lbm_params p{};
    int R = 1, C = 1, parts = 1;
    int transport = LBM_TRANSPORT_LOCAL;
    int rank = 0, world = 1;
    bool vec4 = true;
    bool fused = true;       // fused multi-step launches (WG halo)
    bool use_stream = false; // fused kernel: register-streaming (true) or LDS two-step
    int spl = 2;             // steps per fused launch
    int hw = 2;              // WG halo width (= spl)
    int gr = 2;              // ghost ring width
    int stream_s = 6;        // LBM_STREAM_S: steps per stream launch when not configured
    int stream_hs = 0;       // LBM_STREAM_HS: rows per stream segment (0 = by size)
    int og = 4;              // ghost width of the obstacle map
    std::vector<std::pair<int, float>> guide;  // LBM_STREAM_GUIDE tiers (height, fraction of a band's rows)
    bool guide_set = false;                    // guide given by LBM_STREAM_GUIDE (else by S at create)
    bool guide_auto = false;                   // the default tiers: only where they fit the rect (tiers_fit)
    int stream_cfg = 4;      // LBM_STREAM_CFG (launch form, one wave per workgroup): 0 plain stores;
                             // 3 non-temporal lattice stores; 4 LP (older rows of planes 2,5,6 in LDS, S <= 10)
    // LBM_TOL_S / LBM_TOL_CFG: steps per launch and form with LBM_FLAG_TOLERANCE
    // (S = 10, LP form, one row per iteration: 0.155 vs 0.183 ms per step for
    // S = 7 and 0.174 for S = 8 at 8192^2; profiles/r04/ab_lp10.log)
    int tol_s = 10, tol_cfg = 4;
    int env_kernel = -1;     // LBM_KERNEL: overrides an AUTO kernel request
    long long stream_min_cells = 4LL << 20;  // LBM_STREAM_MIN_CELLS: AUTO picks the stream kernel for sub-domains
                                             // at least this large (smaller ones lack waves for it: step2)
    bool pipeline = false;   // LBM_KERNEL_PIPELINE: unfused per-stage kernels (lbm_pipeline.hip)
    // lattice-resident persistent kernel (lbm_resident.hip): single sub-domain only
    bool resident = false;
    int res_variant = -1;    // ResVariant (LBM_RES_TH picks the tile height)
    int res_th_env = 0;
    int res_per_cu = 1;      // LBM_RES_PER_CU: tiles per CU the choice may plan for (1 or 2)
    int res_early_poll = 0;  // LBM_RES_EARLY: v2 polls the ring after its first work item
    int res_version = 0;     // LBM_RES_V: 1 scalar 64-col tiles, 2 packed 128-col; 0 = by grid
    // The resident kernel is launched with hipLaunchCooperativeKernel (the
    // runtime's admission check of the whole grid).  LBM_RES_COOP=0 (debug
    // knob) launches it plainly: a process that had made a cooperative launch
    // died in exit() under rocprofv3 (SIGSEGV in libhsa-runtime64 under
    // libamdhip64's exit-time teardown, after the profiler's finalisation; no
    // frame of this library: profiles/r05/exitseg/),
    // so the profiling scripts set it.  Either way a grid that does not
    // become co-resident is caught by the poll deadline and the run is
    // repeated on STEP2 (run_steps, res_failed).
    bool res_coop = true;
    bool res_failed = false;        // a resident run timed out: this handle runs STEP2 from then on
    int res_stall_tile = -1, res_stall_step = 1;  // LBM_DEBUG_RES_STALL_TILE / _STEP
    int res_timeout_ms = 2000;      // LBM_DEBUG_RES_TIMEOUT_MS: poll deadline
    bool res_oversubscribe = false; // LBM_DEBUG_RES_OVERSUBSCRIBE: skip the capacity check of the tile choice
    int res_tx = 0, res_ty = 0;
    unsigned long long *res_halo = nullptr;
    float *res_partials = nullptr;
    long long res_partials_cap = 0;
    int *res_status = nullptr;
    unsigned res_tag = 0;    // granule tags used so far (each run continues the sequence)
    long long res_timeout = 0;
    long long resident_max_cells = 1LL << 20;  // LBM_RES_MAX_CELLS: AUTO uses the resident kernel up to this size
    bool forked = false;     // boundary stream running ahead of s_comp (multi-sub-domain launches)
    bool force_exchange = false;
    int graph_steps = 8;     // replay graphs of 2*graph_steps launches on the single-domain path
    hipGraphExec_t graph_exec[2] = {nullptr, nullptr};
    std::vector<float> probe_ms;  // placement probe: ms per launch of each lattice pair tried
    int probe_kept = -1;          // the pair kept (-1: no probe)
    bool debug_knobs = false;     // LBM_DEBUG_KNOBS=1: the tuning knobs below are read from the environment
    bool poison = false;          // LBM_POISON=1: fresh allocations filled with NaN bytes (read-before-write check)
    bool nan_check = false;       // LBM_NAN_CHECK=1: every run ends with a scan of the lattice for NaN / Inf
    bool tolerance = false;       // LBM_FLAG_TOLERANCE: stream kernel with the reciprocal collision (not bitwise)
    // Ordering regression knobs (debug only, tests/test_gpu_ordering.py):
    // LBM_DEBUG_DELAY_SUB = id of the sub-domain whose streams are stalled by
    // LBM_DEBUG_DELAY_US before each of its compute launches;
    // LBM_DEBUG_NO_OWN_WAIT=1 drops the LOCAL unpack's wait on the receiving
    // sub-domain's own event (the round-4 race), so the test can show that the
    // stall exposes the race and that the wait removes it.
    int delay_sub = -1, delay_us = 0;
    bool no_own_wait = false;
    // LBM_FLAG_PROFILE: every launch bracketed by a pair of HIP events on its
    // own stream, folded per launch class after each run (lbm_profile_summary;
    // the counterpart of the reference's engine.printProfileSummary under -d,
    // LbmRunner.cpp:115-122).  Off: no event is recorded.
    bool profile = false;
    struct ProfRec { int cls, dev; hipEvent_t a, b; };
    struct ProfAcc { std::string name; long long launches = 0; double total_ms = 0, min_ms = 1e30, max_ms = 0; };
    std::vector<ProfRec> prof_open;
    std::vector<ProfAcc> prof_acc;
    std::vector<std::pair<int, hipEvent_t>> prof_pool;  // (device, event) free list

    int prof_class(const std::string &name) {
        for (size_t i = 0; i < prof_acc.size(); ++i)
            if (prof_acc[i].name == name) return (int)i;
        prof_acc.push_back(ProfAcc{name});
        return (int)prof_acc.size() - 1;
    }
    hipEvent_t prof_event(int dev) {
        for (size_t i = 0; i < prof_pool.size(); ++i)
            if (prof_pool[i].first == dev) {
                hipEvent_t e = prof_pool[i].second;
                prof_pool[i] = prof_pool.back();
                prof_pool.pop_back();
                return e;
            }
        hipEvent_t e = nullptr;
        HIP_CHECK(hipEventCreate(&e));
        return e;
    }
    // run `f` (which enqueues work on st of sub s) bracketed by profile events
    template <class F>
    void timed(const Sub &s, hipStream_t st, const std::string &cls, F &&f) {
        if (!profile) {
            f();
            return;
        }
        // the record is listed before anything can throw, so a failed launch
        // returns its two events to the pool (prof_drop at the next run)
        ProfRec r{prof_class(cls), s.dev, prof_event(s.dev), nullptr};
        try {
            r.b = prof_event(s.dev);
        } catch (...) {
            prof_pool.push_back({s.dev, r.a});
            throw;
        }
        prof_open.push_back(r);
        HIP_CHECK(hipEventRecord(r.a, st));
        f();
        HIP_CHECK(hipEventRecord(r.b, st));
    }
    // after a run's streams are synchronised: fold this run's records
    void prof_collect() {
        for (auto &r : prof_open) {
            float ms = 0.f;
            HIP_CHECK(hipEventElapsedTime(&ms, r.a, r.b));
            ProfAcc &a = prof_acc[r.cls];
            a.launches++;
            a.total_ms += ms;
            a.min_ms = std::min(a.min_ms, (double)ms);
            a.max_ms = std::max(a.max_ms, (double)ms);
            prof_pool.push_back({r.dev, r.a});
            prof_pool.push_back({r.dev, r.b});
        }
        prof_open.clear();
    }
    // records of a run that failed part-way are dropped (their events may never have been recorded)
    void prof_drop() {
        for (auto &r : prof_open) {
            prof_pool.push_back({r.dev, r.a});
            prof_pool.push_back({r.dev, r.b});
        }
        prof_open.clear();
    }
    void prof_release() {
        for (auto &r : prof_open) {
            prof_pool.push_back({r.dev, r.a});
            prof_pool.push_back({r.dev, r.b});
        }
        prof_open.clear();
        for (auto &e : prof_pool) (void)hipEventDestroy(e.second);
        prof_pool.clear();
    }
    std::string part_name(bool fused_launch, bool interior, int steps) const {
        const char *where = multi() ? (interior ? " interior" : " boundary") : "";
        if (fused_launch && use_stream)
            return std::string("stream_steps2d S=") + std::to_string(steps > 0 ? steps : spl) +
                   (tolerance ? " tolerance" : "") + where;
        if (fused_launch) return std::string("step2") + where;
        return std::string(vec4 ? "step_vec4" : "step_scalar") + where;
    }
    int run_fused = 0, run_single = 0;  // launches of the last run: fused (spl steps) / one-step
    // Tuning knobs (environment, read at create): LBM_TWO_STEP, LBM_MAX_BLOCKS,
    // LBM_LAYOUT (rows|planar), LBM_GRAPH_STEPS, LBM_FORCE_EXCHANGE.  Defaults
    // chosen with tools/ab_bench.py on MI355X (profiles/r01/ab_*.log).
    int max_blocks_cfg = 1 << 30;
    bool row_interleaved = true;
    int tile2 = -1;          // two-step tile shape (LBM_TILE2 = index into T2_W/T2_H); -1 = by size
    int xoff = 64;           // floats before interior column 0 in a plane row (LBM_XOFF): 256-B aligned rows
    std::vector<lbm_rect> all_rects;
    std::vector<Sub> subs;  // local sub-domains
    ncclComm_t comm = nullptr;
    int64_t free_cells = 0;
    bool loaded = false;
    bool ring_stale = false;  // the last run ended with a remainder: the ghost ring is rebuilt before the next run
    int last_steps = 0;
    double last_seconds = 0.0;
    hipEvent_t t0 = nullptr, t1 = nullptr;
    std::string err;

    // any direction goes through the transport (several sub-domains, or forced)
    bool multi() const { return parts > 1 || force_exchange; }
    int halo_mode() const { return fused ? HALO_WG : HALO_W1; }

    // ------------------------------------------------------------------
    void set_device(const Sub &s) const { HIP_CHECK(hipSetDevice(s.dev)); }

    // Initial fill of a fresh device allocation, ordered on `st` and waited
    // for (the engine's streams are non-blocking: a null-stream hipMemset is
    // not ordered with them).  Zero, or with LBM_POISON=1 all-ones bytes (a
    // NaN in every float), so that a value the engine reads without having
    // written it shows up as NaN in the lattice or in av_vels (SURVEY §5
    // sanitizer row; tests/test_poison.py).
    void fill_fresh(void *ptr, size_t bytes, hipStream_t st) const {
        HIP_CHECK(hipMemsetAsync(ptr, poison ? 0xFF : 0, bytes, st));
        HIP_CHECK(hipStreamSynchronize(st));
    }
    // Protocol words whose zero IS their initialisation (control block, status)
    static void fill_zero(void *ptr, size_t bytes, hipStream_t st) {
        HIP_CHECK(hipMemsetAsync(ptr, 0, bytes, st));
        HIP_CHECK(hipStreamSynchronize(st));
    }

    // LBM_STREAM_GUIDE tiers "h1:f1,h2:f2,...,hK" (see guided_rects); "0" = uniform
    void set_guide(const std::string &spec) {
        guide.clear();
        guide_set = true;
        if (spec == "0") return;
        size_t pos = 0;
        while (pos < spec.size()) {
            size_t end = spec.find(',', pos);
            if (end == std::string::npos) end = spec.size();
            const std::string item = spec.substr(pos, end - pos);
            const size_t c = item.find(':');
            const int ht = atoi(item.substr(0, c).c_str());
            const float fr = c == std::string::npos ? 1.f : (float)atof(item.substr(c + 1).c_str());
            if (ht > 0) guide.emplace_back(ht, fr);
            pos = end + 1;
        }
    }

    static int env_int(const char *name, int dflt) {
        const char *v = getenv(name);
        return (v && *v) ? atoi(v) : dflt;
    }
    // Tuning / A-B knobs are read only with LBM_DEBUG_KNOBS=1:
    // without it the library ignores the environment and runs its defaults
    // (LBM_POISON, a read-before-write check that changes no result of a
    // correct engine, is the one exception).
    int knob(const char *name, int dflt) const { return debug_knobs ? env_int(name, dflt) : dflt; }
    const char *knob_str(const char *name) const { return debug_knobs ? getenv(name) : nullptr; }

    void read_tuning() {
        debug_knobs = env_int("LBM_DEBUG_KNOBS", 0) != 0;
        poison = env_int("LBM_POISON", 0) != 0;
        nan_check = env_int("LBM_NAN_CHECK", 0) != 0;
        max_blocks_cfg = std::max(1, knob("LBM_MAX_BLOCKS", max_blocks_cfg));
        graph_steps = std::max(0, knob("LBM_GRAPH_STEPS", graph_steps));
        fused = knob("LBM_TWO_STEP", fused ? 1 : 0) != 0;
        tile2 = std::min(std::max(knob("LBM_TILE2", tile2), -1), NUM_TILE2 - 1);
        xoff = std::max(MIN_XOFF, (knob("LBM_XOFF", xoff) + 3) / 4 * 4);
        stream_s = std::min(std::max(knob("LBM_STREAM_S", stream_s), 2), 6);
        stream_hs = std::max(0, knob("LBM_STREAM_HS", stream_hs));
        auto form = [](int c, int dflt) { return (c == 0 || c == 3 || c == 4) ? c : dflt; };
        stream_cfg = form(knob("LBM_STREAM_CFG", stream_cfg), stream_cfg);
        tol_cfg = form(knob("LBM_TOL_CFG", tol_cfg), tol_cfg);
        tol_s = std::min(std::max(knob("LBM_TOL_S", tol_s), 2), 10);
        stream_min_cells = std::max(0, knob("LBM_STREAM_MIN_CELLS", (int)stream_min_cells));
        if (const char *g = knob_str("LBM_STREAM_GUIDE")) set_guide(g);
        res_th_env = std::max(0, knob("LBM_RES_TH", 0));
        res_version = knob("LBM_RES_V", 0);
        res_coop = knob("LBM_RES_COOP", res_coop ? 1 : 0) != 0;
        res_stall_tile = knob("LBM_DEBUG_RES_STALL_TILE", -1);
        res_stall_step = std::max(0, knob("LBM_DEBUG_RES_STALL_STEP", 1));
        res_timeout_ms = std::min(std::max(knob("LBM_DEBUG_RES_TIMEOUT_MS", res_timeout_ms), 1), 60000);
        res_oversubscribe = knob("LBM_DEBUG_RES_OVERSUBSCRIBE", 0) != 0;
        res_per_cu = std::min(std::max(knob("LBM_RES_PER_CU", res_per_cu), 1), 2);
        res_early_poll = knob("LBM_RES_EARLY", res_early_poll) != 0 ? 1 : 0;
        resident_max_cells = std::max(0, knob("LBM_RES_MAX_CELLS", (int)resident_max_cells));
        delay_sub = knob("LBM_DEBUG_DELAY_SUB", -1);
        delay_us = std::min(std::max(knob("LBM_DEBUG_DELAY_US", 0), 0), 100000);
        // only together with a stall, and never silently: it removes the
        // round-4 race fix so the ordering test can show the race
        no_own_wait = delay_sub >= 0 && knob("LBM_DEBUG_NO_OWN_WAIT", 0) != 0;
        if (no_own_wait)
            fprintf(stderr, "lbm: LBM_DEBUG_NO_OWN_WAIT=1 -- the loop-back unpack's own-event wait is OFF "
                            "(debug only: lattices may be wrong)\n");
        if (const char *k = knob_str("LBM_KERNEL")) {
            const std::string v(k);
            env_kernel = v == "pipeline" ? LBM_KERNEL_PIPELINE
                       : v == "resident" ? LBM_KERNEL_RESIDENT
                       : v == "stream" ? LBM_KERNEL_STREAM : v == "step2" ? LBM_KERNEL_STEP2
                       : v == "vec4" ? LBM_KERNEL_VEC4 : v == "scalar" ? LBM_KERNEL_SCALAR : -1;
        }
        const char *l = knob_str("LBM_LAYOUT");
        if (l && *l) row_interleaved = std::string(l) != "planar";
    }

    // ---- halo destinations --------------------------------------------
    // W1: populations leaving through d -> own ghost ring (opposite side) or send[d]
    EdgeDst make_dst1(const Sub &s, float *org, int d) const {
        EdgeDst e{};
        if (s.remote[d]) {
            const int len = edge_len(d, s.w, s.h);
            for (int i = 0; i < NPLANES[d]; ++i) e.p[i] = s.send[d] + (long long)i * len;
            e.ps = 1;
            return e;
        }
        long long base = 0;
        switch (OPP_DIR[d]) {  // ghost side that receives them
            case DE: base = s.w; e.ps = s.pitch; break;
            case DW: base = -1; e.ps = s.pitch; break;
            case DN: base = (long long)s.h * s.pitch; e.ps = 1; break;
            case DS: base = -(long long)s.pitch; e.ps = 1; break;
            case DNE: base = (long long)s.h * s.pitch + s.w; e.ps = 1; break;
            case DNW: base = (long long)s.h * s.pitch - 1; e.ps = 1; break;
            case DSW: base = -(long long)s.pitch - 1; e.ps = 1; break;
            case DSE: base = -(long long)s.pitch + s.w; e.ps = 1; break;
        }
        for (int i = 0; i < NPLANES[d]; ++i) e.p[i] = org + PLANES[d][i] * s.plane + base;
        return e;
    }

    // WG: the hw outermost rows/columns of side d, all nine speeds, placed
    // where the periodic image on the opposite side sits (strip coordinates
    // (a, b) as in lbm_layout.hpp).
    Dst2 self_dst2(const Sub &s, float *org, int d) const {
        const long long P = s.plane, pt = s.pitch, g_ = hw;
        Dst2 g{};
        g.ks = P;
        switch (d) {
            case DE: g.base = org - g_; g.s1 = 1; g.s2 = (int)pt; break;                // cols w-g.. -> -g..
            case DW: g.base = org + s.w; g.s1 = 1; g.s2 = (int)pt; break;               // cols 0..  -> w..
            case DN: g.base = org - g_ * pt; g.s1 = (int)pt; g.s2 = 1; break;           // rows h-g.. -> -g..
            case DS: g.base = org + (long long)s.h * pt; g.s1 = (int)pt; g.s2 = 1; break;  // rows 0.. -> h..
            case DNE: g.base = org - g_ * pt - g_; g.s1 = (int)pt; g.s2 = 1; break;
            case DNW: g.base = org - g_ * pt + s.w; g.s1 = (int)pt; g.s2 = 1; break;
            case DSW: g.base = org + (long long)s.h * pt + s.w; g.s1 = (int)pt; g.s2 = 1; break;
            case DSE: g.base = org + (long long)s.h * pt - g_; g.s1 = (int)pt; g.s2 = 1; break;
        }
        return g;
    }

    Dst2 make_dst2(const Sub &s, float *org, int d) const {
        if (!s.remote[d]) return self_dst2(s, org, d);
        Dst2 g{};
        g.base = s.send[d];
        if (d < 4) {  // [9][hw][len]
            const int len = edge_len(d, s.w, s.h);
            g.ks = (long long)hw * len;
            g.s1 = len;
            g.s2 = 1;
        } else {      // [9][hw][hw]
            g.ks = (long long)hw * hw;
            g.s1 = hw;
            g.s2 = 1;
        }
        return g;
    }

    HaloArgs halo_args(const Sub &s, float *org, int mode, bool for_unpack) const {
        HaloArgs a{};
        a.f = org;
        a.plane = s.plane;
        a.pitch = s.pitch;
        a.w = s.w;
        a.h = s.h;
        a.mode = mode;
        a.g = hw;
        for (int d = 0; d < 8; ++d) {
            if (for_unpack) {
                if (s.remote[d]) a.mask |= 1u << d;
                a.recv[d] = s.recv[d];
                // side d's ghost receives the neighbour's strip of direction OPP(d)
                a.ghost2[d] = self_dst2(s, org, OPP_DIR[d]);
            } else {
                a.mask |= 1u << d;
                a.dst[d] = make_dst1(s, org, d);
                a.dst2[d] = make_dst2(s, org, d);
            }
        }
        return a;
    }

    // ---- work decomposition ---------------------------------------------
    int fill_rects(Rect (&rect)[MAX_RECTS], int (&begin)[MAX_RECTS], int &nrect, const std::vector<Rect> &rs,
                   int unit_w, bool tiles_are_items) const {
        int tiles = 0;
        nrect = (int)rs.size();
        for (int i = 0; i < MAX_RECTS; ++i) {
            if (i < nrect) {
                Rect r = rs[i];
                r.wc = r.wc / unit_w;
                rect[i] = r;
                begin[i] = tiles;
                const long long items = (long long)r.wc * r.hr;
                tiles += tiles_are_items ? (int)items : (int)((items + BLOCK - 1) / BLOCK);
            } else {
                rect[i] = Rect{0, 0, 1, 1};
                begin[i] = INT_MAX;
            }
        }
        return tiles;
    }

    // Boundary / interior split of a sub-domain in units of `ux` x `uy`
    // cells (x units count columns, y units rows).  xs/ys: first unit index
    // that touches the outer strip on the high side.
    void split(const Sub &s, int nx_u, int ny_u, int xs_hi, int ys_hi, std::vector<Rect> &bnd,
               std::vector<Rect> &inr) const {
        const bool xdec = s.remote[DE] || s.remote[DW];
        const bool ydec = s.remote[DN] || s.remote[DS];
        bnd.clear();
        inr.clear();
        if (!xdec && !ydec) {
            inr.push_back(Rect{0, 0, nx_u, ny_u});
            return;
        }
        const int top = std::max(1, std::min(ys_hi, ny_u));
        bnd.push_back(Rect{0, 0, nx_u, 1});
        if (ny_u > top) bnd.push_back(Rect{0, top, nx_u, ny_u - top});
        const int mid_h = top - 1;
        if (mid_h <= 0) return;
        if (xdec) {
            const int right = std::max(1, std::min(xs_hi, nx_u));
            bnd.push_back(Rect{0, 1, 1, mid_h});
            if (nx_u > right) bnd.push_back(Rect{right, 1, nx_u - right, mid_h});
            if (right > 1) inr.push_back(Rect{1, 1, right - 1, mid_h});
        } else {
            inr.push_back(Rect{0, 1, nx_u, mid_h});
        }
    }

    void build_args(Sub &s) {
        const float w1 = p.density * p.accel / 9.f;
        const float w2 = p.density * p.accel / 36.f;
        std::vector<Rect> bnd, inr;

        // one-step launches: units = 4-cell chunks (vec4) or cells, by rows
        const int cw = vec4 ? 4 : 1;
        split(s, s.w / cw, s.h, (s.w - 1) / cw, s.h - 1, bnd, inr);
        for (auto &r : bnd) r = Rect{r.x0 * cw, r.y0, r.wc * cw, r.hr};
        for (auto &r : inr) r = Rect{r.x0 * cw, r.y0, r.wc * cw, r.hr};
        StepArgs b1{};
        b1.plane = s.plane;
        b1.pitch = s.pitch;
        b1.w = s.w;
        b1.h = s.h;
        b1.obst = s.obst;
        b1.accel_row = s.accel_row;
        b1.omega = p.omega;
        b1.omo = 1 - p.omega;
        b1.w1 = w1;
        b1.w2 = w2;
        b1.ctl = s.ctl;
        StepArgs ai = b1, ab = b1;
        const int ti = fill_rects(ai.rect, ai.rect_begin, ai.nrect, inr, cw, false);
        const int tb = fill_rects(ab.rect, ab.rect_begin, ab.nrect, bnd, cw, false);
        ai.total = ti;
        ab.total = tb;
        s.n1_int = std::max(1, std::min(ti, max_blocks_cfg));
        s.n1_bnd = bnd.empty() ? 0 : std::max(1, std::min(tb, max_blocks_cfg));

        // two-step launches: units = TW x TH tiles, one per workgroup.  Tile
        // by size (tools/ab_bench.py, profiles/r01/ab_step2_tiles.log): the
        // wave-per-row v2 kernel wins while the lattice pair lives in the
        // Infinity Cache, the 64x8 v1 kernel once it streams from HBM.
        if (tile2 < 0) tile2 = ((long long)s.w * s.h <= (2LL << 20)) ? T2V_64x8_W8 : T2_64x8;
        const int TW = T2_W[tile2], TH = T2_H[tile2];
        const int tx = (s.w + TW - 1) / TW, ty = (s.h + TH - 1) / TH;
        split(s, tx, ty, (s.w - 2) / TW, (s.h - 2) / TH, bnd, inr);
        Step2Args b2{};
        b2.tile = tile2;
        b2.ogp = s.w + 2 * og;
        b2.obst_g = s.obst_g + (long long)(og - 1) * b2.ogp + (og - 1);  // the kernel indexes (y+1)*ogp + (x+1)
        b2.plane = s.plane;
        b2.pitch = s.pitch;
        b2.w = s.w;
        b2.h = s.h;
        b2.gy0 = s.rect.y0;
        b2.ny = p.ny;
        b2.accel_g = p.ny >= 2 ? p.ny - 2 : -1;
        b2.omega = p.omega;
        b2.omo = 1 - p.omega;
        b2.w1 = w1;
        b2.w2 = w2;
        b2.ctl = s.ctl;
        Step2Args ci = b2, cb = b2;
        s.n2_int = std::max(1, fill_rects(ci.rect, ci.rect_begin, ci.nrect, inr, 1, true));
        ci.total = s.n2_int;
        const int t2b = fill_rects(cb.rect, cb.rect_begin, cb.nrect, bnd, 1, true);
        cb.total = t2b;
        s.n2_bnd = bnd.empty() ? 0 : t2b;
        if (inr.empty()) ci.total = 0;  // one idle block keeps the reduction / partials protocol

        // stream launches: rects in cells, units = strip x segment (one wave
        // each).  Decomposed dimensions get boundary bands spl cells deep so
        // the interior never reads the ghost ring.
        StreamArgs b3{};
        b3.obst_g = s.obst_g;
        b3.og = og;
        b3.ogp = s.w + 2 * og;
        b3.plane = s.plane;
        b3.pitch = s.pitch;
        b3.w = s.w;
        b3.h = s.h;
        b3.xmax = s.rf - xoff - 1;  // last column inside the row allocation (>= w + gr + 1)
        b3.hw = hw;
        b3.gy0 = s.rect.y0;
        b3.ny = p.ny;
        b3.accel_g = p.ny >= 2 ? p.ny - 2 : -1;
        b3.omega = p.omega;
        b3.omo = 1 - p.omega;
        b3.tc0 = p.omega * (4.f / 9.f);
        b3.tc1 = p.omega * (1.f / 9.f);
        b3.tc2 = p.omega * (1.f / 36.f);
        b3.w1 = w1;
        b3.w2 = w2;
        b3.ctl = s.ctl;
        StreamArgs si = b3, sb = b3;
        s.n3_int = s.n3_bnd = 0;
        if (use_stream) {
            std::vector<SRect> ri, rb;
            stream_split(s, ri, rb);
            si.total = fill_srects(si, ri);
            sb.total = fill_srects(sb, rb);
            s.n3_int = std::max(1, si.total);  // one idle block keeps the reduction / partials protocol
            s.n3_bnd = sb.total;
        }

        const int n1 = s.n1_int + s.n1_bnd, n2 = s.n2_int + s.n2_bnd, n3 = s.n3_int + s.n3_bnd;
        const int st1 = (int)round_up(n1, 4), st2 = (int)round_up(n2, 4), st3 = (int)round_up(n3, 4);
        const long long cap = std::max<long long>(std::max<long long>(st1, 2LL * st2), (long long)spl * st3) + 64;
        for (int k = 0; k < 2; ++k) {
            if (s.partials[k]) HIP_CHECK(hipFree(s.partials[k]));
            HIP_CHECK(hipMalloc(&s.partials[k], sizeof(float) * (size_t)cap));
            fill_fresh(s.partials[k], sizeof(float) * (size_t)cap, s.s_comp);
        }
        for (int par = 0; par < 2; ++par) {
            const float *fin = s.o[par];
            float *fout = s.o[1 - par];
            for (StepArgs *a : {&ai, &ab}) {
                a->fin = fin;
                a->fout = fout;
                for (int d = 0; d < 8; ++d) a->dst[d] = make_dst1(s, fout, d);
                a->partials_prev = s.partials[1 - par];
                a->av_local = s.av_local;
                a->n_total = n1;
                a->stride = st1;
            }
            ai.partials_out = s.partials[par];
            ab.partials_out = s.partials[par] + s.n1_int;
            s.a1_int[par] = ai;
            s.a1_bnd[par] = ab;
            for (Step2Args *a : {&ci, &cb}) {
                a->fin = fin;
                a->fout = fout;
                for (int d = 0; d < 8; ++d) a->dst[d] = make_dst2(s, fout, d);
                a->partials_prev = s.partials[1 - par];
                a->av_local = s.av_local;
                a->n_total = n2;
                a->stride = st2;
            }
            ci.partials_out = s.partials[par];
            cb.partials_out = s.partials[par] + s.n2_int;
            s.a2_int[par] = ci;
            s.a2_bnd[par] = cb;
            for (StreamArgs *a : {&si, &sb}) {
                a->fin = fin;
                a->fout = fout;
                for (int d = 0; d < 8; ++d) a->dst[d] = make_dst2(s, fout, d);
                a->partials_prev = s.partials[1 - par];
                a->av_local = s.av_local;
                a->n_total = n3;
                a->stride = st3;
            }
            if (!s.dst2_dev) HIP_CHECK(hipMalloc(&s.dst2_dev, sizeof(Dst2) * 16));
            HIP_CHECK(hipMemcpy(s.dst2_dev + 8 * par, si.dst, sizeof(Dst2) * 8, hipMemcpyHostToDevice));
            si.dstg = sb.dstg = s.dst2_dev + 8 * par;
            if (knob_str("LBM_STREAM_TRACE") && use_stream && s.n3_int > 0) {
                if (!s.trace) HIP_CHECK(hipMalloc(&s.trace, sizeof(unsigned long long) * 2 * (size_t)s.n3_int));
                si.trace = s.trace;
            }
            si.partials_out = s.partials[par];
            sb.partials_out = s.partials[par] + s.n3_int;
            s.a3_int[par] = si;
            s.a3_bnd[par] = sb;
        }
        // v3: which work units read an obstacle cell (the rest run without
        // rebound selects); obstacles and the work split are fixed from here on
        const char *uo = knob_str("LBM_STREAM_UOBST");
        if (use_stream && !(uo && atoi(uo) == 0)) {
            if (s.uobst) HIP_CHECK(hipFree(s.uobst));
            const int ni = std::max(0, s.a3_int[0].total), nb = std::max(0, s.a3_bnd[0].total);
            HIP_CHECK(hipMalloc(&s.uobst, (size_t)ni + nb + 1));
            HIP_CHECK(stream2d_unit_flags(s.a3_int[0], spl, s.uobst, s.s_comp));
            HIP_CHECK(stream2d_unit_flags(s.a3_bnd[0], spl, s.uobst + ni, s.s_comp));
            HIP_CHECK(hipStreamSynchronize(s.s_comp));
            for (int par = 0; par < 2; ++par) {
                s.a3_int[par].uobst = s.uobst;
                s.a3_bnd[par].uobst = s.uobst + ni;
            }
            // dispatch order: within each XCD's range of slots (xcd_remap),
            // the units that read obstacle cells (slower: rebound selects)
            // first, the rest after, each group in its original order
            const char *so = knob_str("LBM_STREAM_ORDER");
            if (!(so && atoi(so) == 0)) {
                std::vector<uint8_t> fl((size_t)ni + nb);
                HIP_CHECK(hipMemcpy(fl.data(), s.uobst, fl.size(), hipMemcpyDeviceToHost));
                const int W = 1;  // one wave per workgroup in every launch form
                std::vector<int> perm((size_t)ni + nb);
                auto order = [&](int off, int n) {
                    const int blocks = (n + W - 1) / W, q = blocks / 8, r = blocks % 8;
                    for (int x = 0; x < 8; ++x) {
                        const int b0 = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
                        const int nbx = q + (x < r ? 1 : 0);
                        const int t0 = std::min(n, b0 * W), t1 = std::min(n, (b0 + nbx) * W);
                        int k = t0;
                        for (int pass = 0; pass < 2; ++pass)
                            for (int t = t0; t < t1; ++t)
                                if ((fl[(size_t)off + t] != 0) == (pass == 0)) perm[(size_t)off + k++] = t;
                    }
                };
                order(0, ni);
                order(ni, nb);
                if (s.uperm) HIP_CHECK(hipFree(s.uperm));
                HIP_CHECK(hipMalloc(&s.uperm, sizeof(int) * (perm.size() + 1)));
                HIP_CHECK(hipMemcpy(s.uperm, perm.data(), sizeof(int) * perm.size(), hipMemcpyHostToDevice));
                for (int par = 0; par < 2; ++par) {
                    s.a3_int[par].uperm = s.uperm;
                    s.a3_bnd[par].uperm = s.uperm + ni;
                }
            }
        }
    }

    // Stream-kernel work split of a sub-domain (cells).  Segment height by
    // size: about 8192 waves over the interior (32 per CU; measured best at
    // 8192^2, profiles/r01/stream/ab_v2.log), at least 4*spl rows so the
    // 2*spl re-streamed rows per segment stay a modest overhead.
    void stream_split(const Sub &s, std::vector<SRect> &inr, std::vector<SRect> &bnd) const {
        const int S = spl, b = S;
        // owned columns per strip: 64 - 2S (one column per lane); 128 - 2S
        // (two per lane), 2 fewer when the strip's first cell minus S is odd
        // (float2 alignment shifts the wave one column left)
        // ow16: owned widths (and the x bands) rounded down to 16 columns, so
        // that with 64-B aligned interior rows every strip's stores start and
        // end on a 64-B sector -- partial-sector stores cost more than the
        // extra recomputed columns (8192^2: tolerance S = 4 / 6 +6 / +8 %,
        // bitwise S = 5 +6 %; bitwise S = 6, VALU-bound, -4 % and keeps the
        // natural width; profiles/r03/ab_ow16.log)
        // S = 9, 10 (tolerance): 128 - 2S rounds down to 96 -- a sixth more
        // recomputed columns cost more than the unaligned stores (S = 10:
        // 0.155 vs 0.169 ms per step, profiles/r04/ab_lp10.log)
        const bool ow16 = knob("LBM_STREAM_OW16", ((tolerance && S <= 8) || S <= 5) ? 1 : 0) != 0;
        auto ow_of = [&](int rx) {
            const int n = ((rx - S) & 1) ? 126 - 2 * S : 128 - 2 * S;
            return ow16 ? n / 16 * 16 : n;
        };
        const bool xdec = s.remote[DE] || s.remote[DW];
        const bool ydec = s.remote[DN] || s.remote[DS];
        // a decomposed x side's boundary band is one whole strip wide when the
        // sub-domain has room: an S-column band costs nearly a full strip per
        // segment for S useful columns (tools/ab_parts.py)
        const int ow_min = ow16 ? (126 - 2 * S) / 16 * 16 : 126 - 2 * S;
        const int xb = (xdec && s.w >= 4 * ow_min) ? ow_min : b;
        const int y0 = ydec ? b : 0, y1 = ydec ? s.h - b : s.h;
        const int x0 = xdec ? xb : 0, x1 = xdec ? s.w - xb : s.w;
        int hs = stream_hs;
        long long cap = 0;  // the device's concurrently resident waves of this launch form
        const long long strips_in = (std::max(x1 - x0, 1) + ow_of(x0) - 1) / ow_of(x0);
        if (hs <= 0) {
            const long long strips = (std::max(x1 - x0, 1) + ow_of(x0) - 1) / ow_of(x0);
            const long long rows = std::max(y1 - y0, 1);
            const long long target = 8192;
            hs = (int)std::max<long long>(4LL * S, (rows * strips + target - 1) / target);
            // whole rounds of the device's concurrently resident waves: 8211
            // waves at 2048 per round ran a fifth round of 19 waves (209 GLUPS
            // at 8192^2); 8142 waves (four rounds) 217-227, 16215 (eight) 222
            // (profiles/r01/stream/ab_hs_rounds.log).  Eight rounds where the
            // segments stay at least 4S rows high, fewer otherwise.
            int per_cu = 0, cus = 0;
            const hipError_t occ = stream2d_blocks_per_cu(S, stream_cfg, tolerance, per_cu);
            if (occ == hipSuccess &&
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s.dev) == hipSuccess &&
                per_cu > 0 && cus > 0) {
                cap = (long long)per_cu * cus;
                const long long nseg_max = std::max<long long>(1, rows / (4LL * S));
                const long long k_max = std::max<long long>(1, nseg_max * strips / cap);
                const long long k = std::min<long long>(8, k_max);
                const long long nseg = std::min(nseg_max, std::max<long long>(1, k * cap / strips));
                hs = (int)((rows + nseg - 1) / nseg);
            }
            if (knob_str("LBM_STREAM_DEBUG"))
                fprintf(stderr, "[stream split] %dx%d: strips %lld rows %lld waves/CU %d CUs %d -> hs %d\n", s.w, s.h,
                        strips, rows, per_cu, cus, hs);
        }
        auto mk = [&](int rx, int ry, int rw, int rh, int rhs) {
            const int ow = ow_of(rx);
            return SRect{rx, ry, rw, rh, (rw + ow - 1) / ow, std::max(1, std::min(rhs, rh)), ow};
        };
        inr.clear();
        bnd.clear();
        if (ydec) {
            bnd.push_back(mk(0, 0, s.w, b, b));
            bnd.push_back(mk(0, s.h - b, s.w, b, b));
        }
        if (xdec && y1 > y0) {
            bnd.push_back(mk(0, y0, xb, y1 - y0, hs));
            bnd.push_back(mk(s.w - xb, y0, xb, y1 - y0, hs));
        }
        if (x1 > x0 && y1 > y0) {
            if (!guided_rects(x0, y0, x1 - x0, y1 - y0, mk, inr, strips_in, cap))
                inr.push_back(mk(x0, y0, x1 - x0, y1 - y0, hs));
        }
    }

    // Guided segment heights for the interior of the stream launch (auto
    // heights only).  Waves of one launch differ in duration by +-10-15 %
    // (tools/stream_trace.py), so equal segments leave the device's slots
    // idling while the last ones finish; instead the rows are cut into one
    // band per XCD (blocks b and b+8 share an XCD and are dispatched in b
    // order, xcd_remap gives each XCD a contiguous range of work units), and
    // each band into tiers of decreasing segment height: tall segments
    // (little re-streamed overlap) first, short ones last to fill the tail.
    // LBM_STREAM_GUIDE = "h1:f1,h2:f2,...,hK" (tier heights, fractions of a
    // band's rows; the last tier takes the rest), "0" = uniform heights.
    // Whether the default tiers suit an h-row rect of `strips` strips: they
    // were tuned at 8192^2 (3.6 rounds of the device's wave slots at S = 10,
    // 5.3 at S = 6, the shortest tier taking 6 % of each band); on smaller
    // rects they cut too few work units to fill the device, or leave a large
    // share of each band to the shortest tier (4096^2: 34 % in 16-row
    // segments, each re-streaming 2S = 20 rows).  There the uniform heights
    // of stream_split's rounds rule serve better (profiles/r05/mid/: 4096^2
    // tolerance 0.065 -> 0.046 ms per step, 3072^2 0.061 -> 0.028, bitwise
    // 3072^2 0.081 -> 0.046; 4096 x 8192 and 6144^2 keep the tiers).  Fit:
    // at least 1.5 rounds (2.5 for the S <= 6 tiers) and at most a quarter of
    // the rows in the shortest tier.
    bool tiers_fit(long long strips, int h, long long cap) const {
        if (!guide_auto || cap <= 0 || guide.empty()) return true;
        long long segs = 0, last_rows = 0;
        for (const int rb : round_robin(h, 8)) {
            int rest = rb;
            for (size_t k = 0; k < guide.size() && rest > 0; ++k) {
                const int ht = std::max(1, guide[k].first);
                int r = rest;
                if (k + 1 < guide.size()) r = std::min(rest, std::max(ht, (int)(rb * guide[k].second) / ht * ht));
                segs += (r + ht - 1) / ht;
                if (k + 1 == guide.size()) last_rows += r;
                rest -= r;
            }
        }
        const double rounds_min = guide[0].first >= 144 ? 1.5 : 2.5;
        return (double)(segs * strips) >= rounds_min * (double)cap && 4 * last_rows <= h;
    }

    template <class MK>
    bool guided_rects(int x0, int y0, int w, int h, MK &&mk, std::vector<SRect> &out, long long strips,
                      long long cap) const {
        if (stream_hs > 0 || guide.empty()) return false;
        if (!tiers_fit(strips, h, cap)) return false;
        constexpr int NB = 8;
        const int hb = h / NB;
        if (hb < 2 * guide[0].first) return false;
        const auto rows = round_robin(h, NB);
        // built apart and appended only when every tier rect fits, so a guide
        // with too many tiers leaves `out` untouched and the caller falls back
        // to uniform heights
        std::vector<SRect> tiers;
        int y = y0;
        for (int band = 0; band < NB; ++band) {
            int rest = rows[band];
            for (size_t k = 0; k < guide.size() && rest > 0; ++k) {
                const int ht = std::max(1, guide[k].first);
                int r = rest;
                if (k + 1 < guide.size()) r = std::min(rest, std::max(ht, (int)(rows[band] * guide[k].second) / ht * ht));
                tiers.push_back(mk(x0, y, w, r, ht));
                y += r;
                rest -= r;
            }
        }
        if ((int)(out.size() + tiers.size()) > MAX_SRECTS) return false;
        out.insert(out.end(), tiers.begin(), tiers.end());
        return true;
    }

    int fill_srects(StreamArgs &a, const std::vector<SRect> &rs) const {
        int units = 0;
        a.nrect = (int)rs.size();
        if (a.nrect > MAX_SRECTS) throw lbm_failure(LBM_E_INTERNAL, "too many stream rects");
        for (int i = 0; i < MAX_SRECTS; ++i) {
            if (i < a.nrect) {
                a.rect[i] = rs[i];
                a.rect_begin[i] = units;
                units += rs[i].nstrip * ((rs[i].h + rs[i].hs - 1) / rs[i].hs);
            } else {
                a.rect[i] = SRect{0, 0, 1, 1, 1, 1, 1};
                a.rect_begin[i] = INT_MAX;
            }
        }
        return units;
    }

    void ensure_av(int n) {
        for (auto &s : subs) {
            if (s.av_cap >= n) continue;
            drop_graphs();
            set_device(s);
            if (s.av_local) HIP_CHECK(hipFree(s.av_local));
            s.av_cap = std::max(n, 1);
            HIP_CHECK(hipMalloc(&s.av_local, sizeof(float) * (size_t)s.av_cap));
            fill_fresh(s.av_local, sizeof(float) * (size_t)s.av_cap, s.s_comp);
            for (int par = 0; par < 2; ++par) {
                s.a1_int[par].av_local = s.av_local;
                s.a1_bnd[par].av_local = s.av_local;
                s.a2_int[par].av_local = s.av_local;
                s.a2_bnd[par].av_local = s.av_local;
                s.a3_int[par].av_local = s.av_local;
                s.a3_bnd[par].av_local = s.av_local;
            }
        }
    }

    // ------------------------------------------------------------------
    void create(const lbm_params *prm, const uint8_t *obstacles, const lbm_config &cfg) {
        p = *prm;
        if (p.nx <= 0 || p.ny <= 0 || p.max_iters < 0)
            throw lbm_failure(LBM_E_INVALID, "nx, ny must be > 0 and max_iters >= 0");
        if (!obstacles) throw lbm_failure(LBM_E_INVALID, "obstacles must not be NULL");
        parts = cfg.parts > 0 ? cfg.parts : 1;
        transport = cfg.transport;
        read_tuning();  // environment knobs first; explicit config wins
        if (cfg.graph_steps > 0) graph_steps = cfg.graph_steps;
        if (cfg.graph_steps < 0) graph_steps = 0;
        if (cfg.flags & LBM_FLAG_ONE_STEP) fused = false;
        force_exchange = (cfg.flags & LBM_FLAG_FORCE_EXCHANGE) != 0 || knob("LBM_FORCE_EXCHANGE", 0) != 0;
        tolerance = (cfg.flags & LBM_FLAG_TOLERANCE) != 0;
        profile = (cfg.flags & LBM_FLAG_PROFILE) != 0;
        if (partition(p.nx, p.ny, parts, cfg.grid_rows, cfg.grid_cols, R, C, all_rects) != LBM_OK)
            throw lbm_failure(LBM_E_INVALID, "cannot partition " + std::to_string(p.nx) + "x" + std::to_string(p.ny) +
                                                 " into " + std::to_string(parts) + " parts");
        int ndev = 0;
        HIP_CHECK(hipGetDeviceCount(&ndev));
        if (ndev <= 0) throw lbm_failure(LBM_E_HIP, "no HIP device visible");

        free_cells = 0;
        for (long long i = 0; i < (long long)p.nx * p.ny; ++i) free_cells += obstacles[i] ? 0 : 1;

        // kernel choice: vec4 needs widths that are multiples of 4 (>= 8 when split in x)
        bool can_vec = true;
        for (auto &r : all_rects) {
            if (r.w % 4 != 0) can_vec = false;
            if ((C > 1 || force_exchange) && r.w < 8) can_vec = false;
            if (r.w < 2 || r.h < 2) fused = false;  // the two-step halo strips need two rows/columns
        }
        const int kernel = (cfg.kernel == LBM_KERNEL_AUTO && env_kernel >= 0) ? env_kernel : cfg.kernel;
        if (kernel == LBM_KERNEL_VEC4 && !can_vec)
            throw lbm_failure(LBM_E_INVALID,
                              "vec4 kernel needs sub-domain widths that are multiples of 4 (>= 8 when split in x)");
        vec4 = (kernel == LBM_KERNEL_SCALAR) ? false : can_vec;
        if (kernel == LBM_KERNEL_PIPELINE) {  // per-stage kernels, W1 halo of the pre-propagate lattice
            pipeline = true;
            fused = false;
        }
        if (kernel == LBM_KERNEL_VEC4 || kernel == LBM_KERNEL_SCALAR) {
            if (env_kernel >= 0 && cfg.kernel == LBM_KERNEL_AUTO) fused = false;  // LBM_KERNEL=vec4|scalar: one step per launch
        }
        // register-streaming kernel: S steps per launch, S-wide ghost ring;
        // every sub-domain at least S cells (2S across a decomposed dimension)
        // launch form: the tolerance collision has forms 0 and 4 only
        if (tolerance) stream_cfg = tol_cfg == 3 ? 0 : tol_cfg;
        // the v3 kernel takes up to 6 steps per launch, 10 in the tolerance LP form
        const int s_max = tolerance ? 10 : 6;
        int S = cfg.steps_per_launch > 0 ? cfg.steps_per_launch : std::min(tolerance ? tol_s : stream_s, s_max);
        if (cfg.steps_per_launch <= 0) {
            // library default: the deepest S <= the default that every
            // sub-domain allows (S cells, 2S across a decomposed dimension)
            // instead of refusing small sub-domains an explicit request would fit
            for (auto &r : all_rects) {
                const int lw = (C > 1 || force_exchange) ? r.w / 2 : r.w, lh = (R > 1 || force_exchange) ? r.h / 2 : r.h;
                S = std::min(S, std::max(2, std::min(lw, lh)));
            }
        }
        if (kernel == LBM_KERNEL_STREAM && (S < 2 || S > s_max))
            throw lbm_failure(LBM_E_INVALID, "steps_per_launch must be 2.." + std::to_string(s_max) +
                                                 (tolerance ? "" : " (up to 10 with LBM_FLAG_TOLERANCE)"));
        // the LP form exists for S = 6 (bitwise) and 6..10 (tolerance); S > 6 have only it
        if (S > 6) stream_cfg = 4;
        if (!s2d_form_ok(S, stream_cfg, tolerance)) stream_cfg = 0;
        bool can_stream = fused && S >= 2 && S <= s_max, big = true;
        for (auto &r : all_rects) {
            const int mw = (C > 1 || force_exchange) ? 2 * S : S, mh = (R > 1 || force_exchange) ? 2 * S : S;
            if (r.w < mw || r.h < mh) can_stream = false;
            if ((long long)r.w * r.h < stream_min_cells) big = false;
        }
        if (kernel == LBM_KERNEL_STREAM && !can_stream)
            throw lbm_failure(LBM_E_INVALID, "stream kernel needs fused launches and sub-domains of at least "
                                             "steps_per_launch cells (twice that across a decomposed dimension)");
        use_stream = kernel == LBM_KERNEL_STREAM || (kernel == LBM_KERNEL_AUTO && can_stream && big);
        spl = use_stream ? S : 2;
        hw = spl;
        // default segment tiers by S (2S rows re-streamed per segment): S <= 6
        // 96/32/10 (profiles/r02/ab_guide_tiers.log), S >= 7 144/48/16
        // (profiles/r03/guide7/: 400 vs 390 GLUPS at 98 steps, 385 vs 377 at 20)
        if (!guide_set) {
            set_guide(spl >= 7 ? "144:0.85,48:0.1,16" : "96:0.85,32:0.1,10");
            guide_auto = true;
        }
        gr = std::max(2, hw);
        og = gr + 2;  // the two-column stream kernel's strips start up to S+1 columns left of their first cell

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
            torus_neighbours(s.id, R, C, force_exchange, s.nb, s.remote);
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
        placement_probe(subs[0]);
        if (pipeline)
            for (auto &s : subs) {
                set_device(s);
                HIP_CHECK(hipMalloc(&s.pipe_partials, sizeof(float) * (size_t)round_up(pipe_blocks(s.w, s.h), 4)));
                fill_fresh(s.pipe_partials, sizeof(float) * (size_t)round_up(pipe_blocks(s.w, s.h), 4), s.s_comp);
            }
        // lattice-resident kernel: one sub-domain whose 64-column tiles can all be co-resident
        const bool res_ok = parts == 1 && !force_exchange && subs.size() == 1 && !pipeline;
        if (kernel == LBM_KERNEL_RESIDENT && !res_ok)
            throw lbm_failure(LBM_E_INVALID, "resident kernel needs a single sub-domain without forced exchange");
        if (res_ok && (kernel == LBM_KERNEL_RESIDENT ||
                       (kernel == LBM_KERNEL_AUTO && (long long)p.nx * p.ny <= resident_max_cells))) {
            resident = setup_resident(subs[0]);
            if (kernel == LBM_KERNEL_RESIDENT && !resident)
                throw lbm_failure(LBM_E_INVALID, "resident kernel: the grid's tiles cannot all be co-resident on the device");
        }
        ensure_av(std::max(p.max_iters, 1));
        set_device(subs[0]);
        HIP_CHECK(hipEventCreate(&t0));
        HIP_CHECK(hipEventCreate(&t1));
        if (!resident && !multi() && graph_steps > 0) {  // capture both parities now, not inside a timed run
            (void)graph_for(0);
            (void)graph_for(1);
        }
    }

    // Pick the resident tile height (smallest with at most one tile per CU,
    // or LBM_RES_TH) and allocate the granule buffer.  false: does not fit.
    bool setup_resident(const Sub &s) {
        set_device(s);
        int cus = 0;
        HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s.dev));
        // v2 (packed pairs, 128-column tiles) needs an even width; v1 takes any grid
        std::vector<int> order;
        // (smallest tile height with one tile per CU first, except that 2-row
        // tiles are slower than 4-row ones on every grid measured:
        // profiles/r01/resident/)
        if (p.nx % 2 == 0 && (res_version == 0 || res_version == 2))
            order.insert(order.end(), {RES2_4, RES2_8, RES2_16, RES2_32, RES2_2, RES2_16x8});
        if (res_version == 0 || res_version == 1) order.insert(order.end(), {RES_4, RES_8, RES_16, RES_32, RES_64, RES_16x4});
        res_variant = -1;
        for (int v : order) {
            if (res_th_env > 0 && RES_TH[v] != res_th_env) continue;
            const int tx = (p.nx + RES_TWV[v] - 1) / RES_TWV[v];
            const int ty = (p.ny + RES_TH[v] - 1) / RES_TH[v];
            int cap = 0;
            HIP_CHECK(resident_capacity(v, s.dev, tolerance && RES_VER[v] >= 2, cap));
            const long long n = (long long)tx * ty;
            // LBM_DEBUG_RES_OVERSUBSCRIBE=1: take the first tile shape whatever
            // the capacity -- a grid that cannot be co-resident (tests)
            if ((n <= cap && n <= (long long)res_per_cu * cus) || res_oversubscribe) {
                res_variant = v;
                res_tx = tx;
                res_ty = ty;
                break;
            }
        }
        if (res_variant < 0) return false;
        const size_t granules = 2ull * res_tx * res_ty * 8 * RES_GV[res_variant] * RES_GW;
        // granules validate by their step tag (== the expected step, never 0 or
        // all-ones in a run): the poison pattern reads as "not there yet"
        HIP_CHECK(hipMalloc(&res_halo, granules * sizeof(unsigned long long)));
        fill_fresh(res_halo, granules * sizeof(unsigned long long), s.s_comp);
        HIP_CHECK(hipMalloc(&res_status, 64));
        fill_zero(res_status, 64, s.s_comp);
        int khz = 0;
        HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, s.dev));
        res_timeout = (long long)std::max(khz, 1000) * res_timeout_ms;  // 2 s of wall clock per poll phase
        return true;
    }

    // Every step of the run in one cooperative launch (lbm_resident.hip),
    // then the fixed-order |u| fold.  The ghost ring of the result is not
    // maintained (the resident kernel reads the periodic images itself; a
    // STEP2 fallback rebuilds it).  Returns false when a neighbour hand-off
    // timed out (the tiles were not all co-resident): the kernel only reads
    // s.o[s.cur] and writes the other lattice, so the input lattice -- with
    // the first accelerate applied -- is intact, and s.cur, res_tag and
    // last_steps are left as they were.
    bool run_resident(int steps, bool accelerate_first) {
        Sub &s = subs[0];
        set_device(s);
        const int ntiles = res_tx * res_ty;
        if ((long long)steps * ntiles > res_partials_cap) {
            if (res_partials) HIP_CHECK(hipFree(res_partials));
            res_partials = nullptr;
            res_partials_cap = (long long)std::max(steps, 1) * ntiles;
            HIP_CHECK(hipMalloc(&res_partials, sizeof(float) * (size_t)res_partials_cap));
        }
        HIP_CHECK(hipMemsetAsync(res_status, 0, 64, s.s_comp));
        HIP_CHECK(hipEventRecord(t0, s.s_comp));
        if (accelerate_first && s.accel_row >= 0) {
            const float w1 = p.density * p.accel / 9.f;
            const float w2 = p.density * p.accel / 36.f;
            timed(s, s.s_comp, "accelerate_row", [&] {
                HIP_CHECK(launch_accelerate(s.o[s.cur], s.obst, s.plane, s.pitch, s.w, s.accel_row, w1, w2, s.s_comp));
            });
        }
        if (steps > 0) {
            ResidentArgs a{};
            a.fin = s.o[s.cur];
            a.fout = s.o[1 - s.cur];
            a.obst = s.obst;
            a.plane = s.plane;
            a.pitch = s.pitch;
            a.nx = p.nx;
            a.ny = p.ny;
            a.tiles_x = res_tx;
            a.tiles_y = res_ty;
            a.steps = steps;
            a.tag0 = res_tag;
            a.accel_row = p.ny >= 2 ? p.ny - 2 : -1;
            a.omega = p.omega;
            a.omo = 1 - p.omega;
            a.w1 = p.density * p.accel / 9.f;
            a.w2 = p.density * p.accel / 36.f;
            a.tc0 = p.omega * (4.f / 9.f);
            a.tc1 = p.omega * (1.f / 9.f);
            a.tc2 = p.omega * (1.f / 36.f);
            a.halo = res_halo;
            a.partials = res_partials;
            a.status = res_status;
            a.timeout_ticks = res_timeout;
            a.early_poll = res_early_poll;
            a.stall_tile = res_stall_tile;
            a.stall_step = res_stall_step;
            long long *trace = nullptr;
            unsigned long long *htrace = nullptr;
            const int trace_steps = std::min(steps, 256);
            const int trace_mode = knob("LBM_RES_TRACE", 0);
            if (trace_mode) {
                HIP_CHECK(hipMalloc(&trace, sizeof(long long) * 5 * trace_steps));
                HIP_CHECK(hipMemsetAsync(trace, 0, sizeof(long long) * 5 * trace_steps, s.s_comp));
                a.trace = trace;
                a.trace_steps = trace_steps;
            }
            if (trace_mode >= 2) {
                const size_t n = sizeof(unsigned long long) * 2 * trace_steps * ntiles;
                HIP_CHECK(hipMalloc(&htrace, n));
                HIP_CHECK(hipMemsetAsync(htrace, 0, n, s.s_comp));
                a.htrace = htrace;
            }
            bool rejected = false;  // the cooperative launch refused the grid: a residency failure too
            timed(s, s.s_comp, std::string("resident_steps (all steps, one launch)") + (tolerance && RES_VER[res_variant] >= 2 ? " tolerance" : ""),
                  [&] {
                      const hipError_t e = launch_resident(a, res_variant, tolerance && RES_VER[res_variant] >= 2,
                                                           res_coop, s.s_comp);
                      if (e == hipErrorCooperativeLaunchTooLarge) {
                          (void)hipGetLastError();
                          rejected = true;
                      } else {
                          HIP_CHECK(e);
                      }
                  });
            if (rejected) HIP_CHECK(hipMemsetAsync(res_status, 0xff, sizeof(int), s.s_comp));
            if (htrace) {  // per tile and step: wait for the slowest neighbour, then the hop itself
                std::vector<unsigned long long> hv((size_t)2 * trace_steps * ntiles);
                HIP_CHECK(hipMemcpyAsync(hv.data(), htrace, hv.size() * 8, hipMemcpyDeviceToHost, s.s_comp));
                HIP_CHECK(hipStreamSynchronize(s.s_comp));
                HIP_CHECK(hipFree(htrace));
                double wait = 0, hop = 0, step = 0, hop_max = 0;
                long long cnt = 0;
                for (int t = 2; t + 1 < trace_steps; ++t)
                    for (int tl = 0; tl < ntiles; ++tl) {
                        const int tx = tl % res_tx, ty = tl / res_tx;
                        unsigned long long nbmax = 0;
                        for (int dy = -1; dy <= 1; ++dy)
                            for (int dx = -1; dx <= 1; ++dx) {
                                if (!dx && !dy) continue;
                                const int nt = ((ty + dy + res_ty) % res_ty) * res_tx + (tx + dx + res_tx) % res_tx;
                                nbmax = std::max(nbmax, hv[((size_t)t * ntiles + nt) * 2]);
                            }
                        const unsigned long long own = hv[((size_t)t * ntiles + tl) * 2];
                        const unsigned long long ready = hv[((size_t)t * ntiles + tl) * 2 + 1];
                        wait += (double)nbmax - (double)own;
                        hop += (double)ready - (double)nbmax;
                        hop_max = std::max(hop_max, (double)ready - (double)nbmax);
                        step += (double)hv[((size_t)(t + 1) * ntiles + tl) * 2] - (double)own;
                        ++cnt;
                    }
                int khz = 1;
                HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, s.dev));
                const double us = 1e3 / khz;
                fprintf(stderr, "[resident hop] %dx%d tile-height %d early_poll %d: per tile-step (us) own collision end -> "
                        "slowest neighbour's %.3f, -> ring ready %.3f (max %.3f), collision end to next %.3f\n", p.nx,
                        p.ny, RES_TH[res_variant], res_early_poll, wait / cnt * us, hop / cnt * us, hop_max * us,
                        step / cnt * us);
            }
            if (trace) {  // mean phase durations over the traced steps (skipping the first)
                std::vector<long long> tv((size_t)5 * trace_steps);
                HIP_CHECK(hipMemcpyAsync(tv.data(), trace, tv.size() * sizeof(long long), hipMemcpyDeviceToHost, s.s_comp));
                HIP_CHECK(hipStreamSynchronize(s.s_comp));
                HIP_CHECK(hipFree(trace));
                double ph[5] = {0, 0, 0, 0, 0};
                int n = 0;
                for (int t = 1; t + 1 < trace_steps; ++t, ++n) {
                    const long long *r = &tv[(size_t)5 * t];
                    ph[0] += (double)(r[1] - r[0]);
                    ph[1] += (double)(r[2] - r[1]);
                    ph[2] += (double)(r[3] - r[2]);
                    ph[3] += (double)(r[4] - r[3]);
                    ph[4] += (double)(tv[(size_t)5 * (t + 1)] - r[0]);
                }
                int khz = 1;
                HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, s.dev));
                const double us = 1e3 / khz / std::max(n, 1);
                fprintf(stderr, "[resident trace] %dx%d tile-height %d: per step (us) pull+barrier %.3f collide+publish %.3f "
                        "poll %.3f barrier %.3f total %.3f\n", p.nx, p.ny, RES_TH[res_variant], ph[0] * us, ph[1] * us,
                        ph[2] * us, ph[3] * us, ph[4] * us);
            }
            timed(s, s.s_comp, "resident_reduce",
                  [&] { HIP_CHECK(launch_resident_reduce(res_partials, s.av_local, steps, ntiles, s.s_comp)); });
        }
        HIP_CHECK(hipEventRecord(t1, s.s_comp));
        HIP_CHECK(hipEventSynchronize(t1));
        float ms = 0.f;
        HIP_CHECK(hipEventElapsedTime(&ms, t0, t1));
        int status = 0;
        HIP_CHECK(hipMemcpy(&status, res_status, sizeof(int), hipMemcpyDeviceToHost));
        prof_collect();
        if (status != 0) return false;
        if (steps > 0) {
            res_tag += (unsigned)steps;
            s.cur ^= 1;
        }
        last_seconds = ms * 1e-3;
        last_steps = steps;
        return true;
    }

    // Unfused pipeline, one kernel per stage (lbm_pipeline.hip): every step
    // accelerates row ny-2 (conditionally), refreshes the W1 ghost ring of
    // the current lattice (exchanging across sub-domains), propagates into
    // the other lattice, rebounds / collides back, and folds the |u|
    // partials into av_local[t].  The current lattice never changes parity.
    void run_pipeline(int steps) {
        const float w1 = p.density * p.accel / 9.f;
        const float w2 = p.density * p.accel / 36.f;
        Sub &s0 = subs[0];
        set_device(s0);
        HIP_CHECK(hipEventRecord(t0, s0.s_comp));
        for (size_t k = 1; k < subs.size(); ++k) {
            set_device(subs[k]);
            HIP_CHECK(hipStreamWaitEvent(subs[k].s_comp, t0, 0));
        }
        for (int t = 0; t < steps; ++t) {
            for (auto &s : subs) {
                if (s.accel_row < 0 || p.ny < 2) continue;
                set_device(s);
                timed(s, s.s_comp, "accelerate_row", [&] {
                    HIP_CHECK(launch_accelerate(s.o[s.cur], s.obst, s.plane, s.pitch, s.w, s.accel_row, w1, w2, s.s_comp));
                });
            }
            refresh_halos();
            for (auto &s : subs) {
                set_device(s);
                float *cells = s.o[s.cur], *tmp = s.o[1 - s.cur];
                debug_delay(s, s.s_comp);
                timed(s, s.s_comp, "pipe_propagate",
                      [&] { HIP_CHECK(launch_pipe_propagate(cells, tmp, s.plane, s.pitch, s.w, s.h, s.s_comp)); });
                timed(s, s.s_comp, "pipe_rebound",
                      [&] { HIP_CHECK(launch_pipe_rebound(tmp, cells, s.obst, s.plane, s.pitch, s.w, s.h, s.s_comp)); });
                timed(s, s.s_comp, "pipe_collision", [&] {
                    HIP_CHECK(launch_pipe_collision(tmp, cells, s.obst, s.plane, s.pitch, s.w, s.h, p.omega,
                                                    s.pipe_partials, s.s_comp));
                });
                timed(s, s.s_comp, "pipe_av", [&] {
                    HIP_CHECK(launch_pipe_av(s.pipe_partials, pipe_blocks(s.w, s.h), s.av_local, t, s.s_comp));
                });
            }
        }
        for (auto &s : subs) {
            set_device(s);
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
        prof_collect();
    }

    void alloc_sub(Sub &s, const uint8_t *obstacles) {
        set_device(s);
        // streams first: every initial fill below is ordered on s_comp
        HIP_CHECK(hipStreamCreateWithFlags(&s.s_comp, hipStreamNonBlocking));
        HIP_CHECK(hipStreamCreateWithFlags(&s.s_comm, hipStreamNonBlocking));
        int prio_lo = 0, prio_hi = 0;
        HIP_CHECK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
        HIP_CHECK(hipStreamCreateWithPriority(&s.s_bnd, hipStreamNonBlocking, prio_hi));
        HIP_CHECK(hipEventCreateWithFlags(&s.ev_b, hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&s.ev_i, hipEventDisableTiming));
        for (auto &e : s.ev_bp) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&s.ev_u, hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&s.ev_end, hipEventDisableTiming));
        // two spare columns past the ring: a two-column stream lane reads its
        // pair unclamped up to column w + gr
        s.rf = (int)round_up(s.w + xoff + gr + 2, 64);
        const long long rows = s.h + 2LL * gr;
        if (row_interleaved) {
            // f[y][k][x]: the nine populations of a lattice row are adjacent
            s.plane = s.rf;
            s.pitch = Q * s.rf;
            s.lattice_floats = rows * s.pitch;
        } else {
            // f[k][y][x]: plane stride padded off a power of two so the nine
            // concurrent plane streams do not alias
            s.pitch = s.rf;
            s.plane = round_up(rows * s.pitch, 1024) + 320;
            s.lattice_floats = Q * s.plane;
        }
        s.origin_off = (long long)gr * s.pitch + xoff;
        const char *lp = knob_str("LBM_LATTICE_PAD");
        if (lp && *lp) {
            // both lattices in one allocation, the second pad bytes (rounded to
            // 256 B) after the end of the first
            const long long second = s.lattice_floats + (std::max(0LL, atoll(lp)) + 255) / 256 * 64;
            const size_t n = sizeof(float) * (size_t)(second + s.lattice_floats);
            HIP_CHECK(hipMalloc(&s.f[0], n));
            fill_fresh(s.f[0], n, s.s_comp);
            s.f[1] = s.f[0] + second;
            s.f_joint = true;
        } else {
            for (int k = 0; k < 2; ++k) {
                HIP_CHECK(hipMalloc(&s.f[k], sizeof(float) * (size_t)s.lattice_floats));
                fill_fresh(s.f[k], sizeof(float) * (size_t)s.lattice_floats, s.s_comp);
            }
        }
        for (int k = 0; k < 2; ++k) s.o[k] = s.f[k] + s.origin_off;
        HIP_CHECK(hipMalloc(&s.obst, (size_t)round_up((long long)s.w * s.h + 16, 256)));
        HIP_CHECK(hipMemcpy2D(s.obst, (size_t)s.w, obstacles + (size_t)s.rect.y0 * p.nx + s.rect.x0, (size_t)p.nx,
                              (size_t)s.w, (size_t)s.h, hipMemcpyHostToDevice));
        // ghosted obstacle map (ring of og cells) for the fused kernels' halo cells
        {
            const int gw = s.w + 2 * og, gh = s.h + 2 * og;
            std::vector<uint8_t> g((size_t)gw * gh);
            for (int y = -og; y < s.h + og; ++y) {
                const int gyy = ((s.rect.y0 + y) % p.ny + p.ny) % p.ny;
                for (int x = -og; x < s.w + og; ++x) {
                    const int gxx = ((s.rect.x0 + x) % p.nx + p.nx) % p.nx;
                    g[(size_t)(y + og) * gw + (x + og)] = obstacles[(size_t)gyy * p.nx + gxx] ? 1 : 0;
                }
            }
            HIP_CHECK(hipMalloc(&s.obst_g, g.size() + 256));
            HIP_CHECK(hipMemcpy(s.obst_g, g.data(), g.size(), hipMemcpyHostToDevice));
        }
        // halo buffers (only for directions that cross sub-domains), sized for
        // the larger of the two formats
        long long total = 0;
        long long off_send[8], off_recv[8];
        for (int d = 0; d < 8; ++d) {
            const long long n =
                s.remote[d] ? round_up(std::max(msg_floats(HALO_W1, d, s.w, s.h, hw), msg_floats(HALO_WG, d, s.w, s.h, hw)), 64)
                            : 0;
            off_send[d] = total;
            total += n;
            off_recv[d] = total;
            total += n;
        }
        if (total > 0) {
            HIP_CHECK(hipMalloc(&s.halo_mem, sizeof(float) * (size_t)total));
            fill_fresh(s.halo_mem, sizeof(float) * (size_t)total, s.s_comp);
            for (int d = 0; d < 8; ++d) {
                s.send[d] = s.remote[d] ? s.halo_mem + off_send[d] : nullptr;
                s.recv[d] = s.remote[d] ? s.halo_mem + off_recv[d] : nullptr;
            }
        }
        HIP_CHECK(hipMalloc(&s.ctl, 64));
        fill_zero(s.ctl, 64, s.s_comp);
    }

    Sub *local_sub(int id) {
        for (auto &s : subs)
            if (s.id == id) return &s;
        return nullptr;
    }

    // ------------------------------------------------------------------
    // Exchange of the halo send buffers (format `mode`), after every
    // sub-domain recorded ev_b on its compute stream.  `target[k]` is the
    // lattice origin of local sub k whose ghost ring receives.  Ends with the
    // unpack and ev_u recorded on each comm stream.
    void exchange(int mode, const std::vector<float *> &target) {
        if (transport == LBM_TRANSPORT_RCCL) {
            Sub &s = subs[0];
            set_device(s);
            HIP_CHECK(hipStreamWaitEvent(s.s_comm, s.ev_b, 0));
            timed(s, s.s_comm, mode == HALO_WG ? "halo exchange WG (RCCL) + unpack" : "halo exchange W1 (RCCL) + unpack",
                  [&] {
                NCCL_CHECK(ncclGroupStart());
                for (const lbm_xfer &x : exchange_posts(s.id, s.nb, s.remote, s.w, s.h, mode, hw)) {
                    if (x.op == LBM_XFER_SEND)
                        NCCL_CHECK(ncclSend(s.send[x.dir], (size_t)x.floats, ncclFloat, x.peer, comm, s.s_comm));
                    else if (x.op == LBM_XFER_RECV)
                        NCCL_CHECK(ncclRecv(s.recv[x.dir], (size_t)x.floats, ncclFloat, x.peer, comm, s.s_comm));
                }
                NCCL_CHECK(ncclGroupEnd());
                HIP_CHECK(launch_halo_unpack(halo_args(s, target[0], mode, true), s.s_comm));
            });
            HIP_CHECK(hipEventRecord(s.ev_u, s.s_comm));
            return;
        }
        // LOCAL: receiver pulls each message with a device (peer) copy.  The
        // unpack into s's own lattice also waits for s's own pack / boundary
        // event: without it, when the neighbours ran ahead, the pipeline's
        // unpack of step t rewrote s's ghost ring while s's propagate of step
        // t-1 was still reading it (intermittent, test_pipeline_decomposed_bitwise)
        for (size_t k = 0; k < subs.size(); ++k) {
            Sub &s = subs[k];
            set_device(s);
            if (!no_own_wait) HIP_CHECK(hipStreamWaitEvent(s.s_comm, s.ev_b, 0));
            for (int e = 0; e < 8; ++e) {
                if (!s.remote[e]) continue;
                const Sub *src = local_sub(s.nb[e]);
                if (!src) throw lbm_failure(LBM_E_INTERNAL, "missing local neighbour");
                HIP_CHECK(hipStreamWaitEvent(s.s_comm, src->ev_b, 0));
            }
            timed(s, s.s_comm, mode == HALO_WG ? "halo exchange WG (device copies) + unpack"
                                               : "halo exchange W1 (device copies) + unpack", [&] {
                for (int e = 0; e < 8; ++e) {
                    if (!s.remote[e]) continue;
                    const Sub *src = local_sub(s.nb[e]);
                    const size_t bytes = sizeof(float) * (size_t)msg_floats(mode, e, s.w, s.h, hw);
                    const float *from = src->send[OPP_DIR[e]];
                    if (src->dev == s.dev)
                        HIP_CHECK(hipMemcpyAsync(s.recv[e], from, bytes, hipMemcpyDeviceToDevice, s.s_comm));
                    else
                        HIP_CHECK(hipMemcpyPeerAsync(s.recv[e], s.dev, from, src->dev, bytes, s.s_comm));
                }
                HIP_CHECK(launch_halo_unpack(halo_args(s, target[k], mode, true), s.s_comm));
            });
            HIP_CHECK(hipEventRecord(s.ev_u, s.s_comm));
        }
    }

    // Point the v3 stream arguments of s at lattices f0 / f1 (placement probe).
    void set_stream_lattices(Sub &s, float *f0, float *f1) {
        s.f[0] = f0;
        s.f[1] = f1;
        for (int k = 0; k < 2; ++k) s.o[k] = s.f[k] + s.origin_off;
        for (int par = 0; par < 2; ++par) {
            for (StreamArgs *a : {&s.a3_int[par], &s.a3_bnd[par]}) {
                a->fin = s.o[par];
                a->fout = s.o[1 - par];
                for (int d = 0; d < 8; ++d) a->dst[d] = make_dst2(s, s.o[1 - par], d);
            }
            HIP_CHECK(hipMemcpy(s.dst2_dev + 8 * par, s.a3_int[par].dst, sizeof(Dst2) * 8, hipMemcpyHostToDevice));
        }
    }

    // Placement probe.  The stream kernel runs a large
    // sub-domain at one of two speed levels (about 7 % apart) set by the
    // physical pages under its lattices, fixed for the engine's life.  A single
    // sub-domain per process (one domain, or one RCCL rank's block: the probe
    // launches touch only its own lattices and send buffers) of at least 2^25 cells allocates LBM_PLACEMENT_TRIES (5; at most
    // 96 GB of them) lattice pairs, all held at once, times the interior launch on each
    // (non-reducing form: av_local and the reduction control block are not
    // touched; constant populations; two interleaved rounds after a clock
    // warm-up, minimum per pair), keeps the fastest pair and frees the others.  The kept
    // pair is zeroed and the launch arguments are rebuilt, so the engine state
    // is as if the probe had not run.  LBM_PLACEMENT_TRIES=1 turns it off.
    // Scope: the single-sub-domain 2-D stream engine only.  LOCAL multi-sub
    // engines are the one-GPU loop-back test mode (their sub-domains share one
    // device and a probe would time them against each other), the D3Q19 engine
    // showed no two-level spread worth a probe (38.9-42.0 GLUPS over seven
    // placements at 512^3, profiles/r02/placement/d3.log, inside its +-10 %
    // build-to-build noise).
    void placement_probe(Sub &s) {
        const size_t pair_bytes = 2 * sizeof(float) * (size_t)s.lattice_floats;
        // at most 96 GB of candidate pairs held at once (a third of HBM):
        // five at 8192^2 (4.9 GB per pair), four at 16384^2 (19.5 GB)
        const int cap = (int)std::max<size_t>(1, (96ull << 30) / pair_bytes);
        const int tries = std::min({std::max(knob("LBM_PLACEMENT_TRIES", 5), 1), 8, cap});
        if (tries <= 1 || !use_stream || subs.size() != 1 || s.f_joint ||
            (long long)s.w * s.h < (1LL << 25) || s.n3_int <= 0)
            return;
        const size_t n = (size_t)s.lattice_floats;
        std::vector<std::array<float *, 2>> cand{{s.f[0], s.f[1]}};
        size_t keep = 0;
        // on any failure inside the probe: free every extra candidate and put the
        // original pair back, so the handle owns exactly what it allocated
        auto unwind = [&]() {
            for (size_t c = 1; c < cand.size(); ++c)
                if (c != keep)
                    for (float *&p : cand[c])
                        if (p) {
                            (void)hipFree(p);
                            p = nullptr;
                        }
        };
        hipEvent_t e0 = nullptr, e1 = nullptr;  // outside the try: the catch destroys them too
        auto drop_events = [&]() {
            if (e0) (void)hipEventDestroy(e0);
            if (e1) (void)hipEventDestroy(e1);
            e0 = e1 = nullptr;
        };
        try {
            for (int c = 1; c < tries; ++c) {
                std::array<float *, 2> f{nullptr, nullptr};
                if (hipMalloc(&f[0], sizeof(float) * n) != hipSuccess) { (void)hipGetLastError(); break; }
                if (hipMalloc(&f[1], sizeof(float) * n) != hipSuccess) {
                    (void)hipGetLastError();
                    (void)hipFree(f[0]);
                    break;
                }
                cand.push_back(f);
            }
            const unsigned fill = 0x3dcccccdu;  // 0.1f: rho = 0.9 everywhere, no tiny-density path
            for (auto &f : cand)
                for (float *p : f)
                    HIP_CHECK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(p), (int)fill, n, s.s_comp));
            HIP_CHECK(hipEventCreate(&e0));
            HIP_CHECK(hipEventCreate(&e1));
            std::vector<float> best(cand.size(), 1e30f);
            const int warm = 8, timed = 4;
            for (int round = 0; round < 2; ++round)
                for (size_t c = 0; c < cand.size(); ++c) {
                    set_stream_lattices(s, cand[c][0], cand[c][1]);
                    for (int i = 0; i < (round == 0 && c == 0 ? warm : 1); ++i)
                        HIP_CHECK(launch_stream2d(s.a3_int[i & 1], s.n3_int, spl, false, stream_cfg, tolerance,
                                                  s.s_comp));
                    HIP_CHECK(hipEventRecord(e0, s.s_comp));
                    for (int i = 0; i < timed; ++i)
                        HIP_CHECK(launch_stream2d(s.a3_int[i & 1], s.n3_int, spl, false, stream_cfg, tolerance,
                                                  s.s_comp));
                    HIP_CHECK(hipEventRecord(e1, s.s_comp));
                    HIP_CHECK(hipEventSynchronize(e1));
                    float ms = 0.f;
                    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
                    best[c] = std::min(best[c], ms / timed);
                }
            drop_events();
            for (size_t c = 1; c < cand.size(); ++c)
                if (best[c] < best[keep]) keep = c;
            // LBM_PLACEMENT_KEEP=k (tests): keep candidate k whatever the timings,
            // so the swap path (k > 0) is exercised deterministically
            const int force = knob("LBM_PLACEMENT_KEEP", -1);
            if (force >= 0 && force < (int)cand.size()) keep = (size_t)force;
            probe_ms.assign(best.begin(), best.end());
            probe_kept = (int)keep;
            if (knob_str("LBM_PLACEMENT_LOG")) {
                fprintf(stderr, "lbm placement probe (%dx%d): ms per launch", s.w, s.h);
                for (float v : best) fprintf(stderr, " %.4f", v);
                fprintf(stderr, "; kept pair %d\n", probe_kept);
            }
            unwind();
            if (keep != 0)
                for (float *&p : cand[0]) {
                    float *q = p;
                    p = nullptr;
                    HIP_CHECK(hipFree(q));
                }
            set_stream_lattices(s, cand[keep][0], cand[keep][1]);
            for (float *p : cand[keep]) fill_fresh(p, sizeof(float) * n, s.s_comp);
            build_args(s);
        } catch (...) {
            drop_events();
            // keep == 0 here unless the failure came after the choice; either way
            // the handle ends up owning exactly one pair
            unwind();
            if (keep != 0 && cand[0][0]) {  // original pair not yet freed: fall back to it
                for (float *&p : cand[keep])
                    if (p) (void)hipFree(p);
                keep = 0;
            }
            s.f[0] = cand[keep][0];
            s.f[1] = cand[keep][1];
            for (int k = 0; k < 2; ++k) s.o[k] = s.f[k] + s.origin_off;
            throw;
        }
    }

    // `st` waits for the last exchange: own ghosts unpacked, and (LOCAL)
    // every neighbour done reading this sub-domain's send buffers.
    void wait_exchange_on(Sub &s, hipStream_t st) {
        HIP_CHECK(hipStreamWaitEvent(st, s.ev_u, 0));
        if (transport == LBM_TRANSPORT_LOCAL)
            for (int d = 0; d < 8; ++d)
                if (s.remote[d]) HIP_CHECK(hipStreamWaitEvent(st, local_sub(s.nb[d])->ev_u, 0));
    }

    void wait_exchange() {
        for (auto &s : subs) {
            set_device(s);
            wait_exchange_on(s, s.s_comp);
        }
    }

    // Make every ghost cell of the current lattices consistent in the
    // current mode's format (after load, init, accelerate, or a trailing
    // one-step launch in two-step mode).
    void refresh_halos() {
        const int mode = halo_mode();
        std::vector<float *> tgt(subs.size());
        for (size_t k = 0; k < subs.size(); ++k) {
            Sub &s = subs[k];
            set_device(s);
            timed(s, s.s_comp, "halo_pack",
                  [&] { HIP_CHECK(launch_halo_pack(halo_args(s, s.o[s.cur], mode, false), s.s_comp)); });
            HIP_CHECK(hipEventRecord(s.ev_b, s.s_comp));
            tgt[k] = s.o[s.cur];
        }
        if (multi()) {
            exchange(mode, tgt);
            wait_exchange();
        }
    }

    // debug stall of sub-domain s's stream st (LBM_DEBUG_DELAY_SUB / _US)
    void debug_delay(const Sub &s, hipStream_t st) const {
        if (delay_us > 0 && s.id == delay_sub) HIP_CHECK(launch_debug_spin(delay_us, st));
    }

    // launch form of a fused remainder launch of `steps` < spl steps: the
    // engine's form where it has that depth, else the shallowest that does
    int rem_form(int steps) const {
        if (s2d_form_ok(steps, stream_cfg, tolerance)) return stream_cfg;
        return steps > 6 ? 4 : 0;
    }

    // Interior (reducing) or boundary launch of sub-domain s reading parity
    // `cur`: one fused launch (spl steps, WG halo) or one step (W1 halo).
    // steps > 0 (single sub-domain stream engines): a remainder launch of that
    // many fused steps (< spl) on the same work split and halo tables.
    hipError_t launch_part(Sub &s, int cur, bool fused_launch, bool interior, hipStream_t st, int steps = 0) const {
        if (fused_launch && use_stream) {
            const int n = interior ? s.n3_int : s.n3_bnd;
            if (n <= 0) return hipSuccess;
            const StreamArgs &a = interior ? s.a3_int[cur] : s.a3_bnd[cur];
            if (steps > 0 && steps != spl) return launch_stream2d(a, n, steps, interior, rem_form(steps), tolerance, st);
            return launch_stream2d(a, n, spl, interior, stream_cfg, tolerance, st);
        }
        if (fused_launch) {
            const int n = interior ? s.n2_int : s.n2_bnd;
            return n > 0 ? launch_step2(interior ? s.a2_int[cur] : s.a2_bnd[cur], n, interior, st) : hipSuccess;
        }
        const int n = interior ? s.n1_int : s.n1_bnd;
        return n > 0 ? launch_step(interior ? s.a1_int[cur] : s.a1_bnd[cur], n, vec4, interior, st) : hipSuccess;
    }

    // One launch: one time step (W1 halo) or spl steps (fused, WG halo).
    //
    // Multi-sub-domain launch t (reads lattice c = cur, writes 1-c):
    //   B(t) boundary tiles on s_bnd, after I(t-1) (it overwrites the cells
    //        I(t-1) read, and the partials I(t-1) reduced) and after the
    //        exchange U(t-1) that filled c's ghost ring (LOCAL: and after
    //        every neighbour finished copying this sub-domain's send buffers);
    //   X(t) exchange + unpack on s_comm, after B(t) (exchange());
    //   I(t) interior tiles on s_comp, after B(t-1) only: interior tiles
    //        never read the ghost ring, so the exchange of launch t-1 runs
    //        under I(t) and B(t+1) overlaps I(t+1)'s tail.
    // join() re-serialises everything onto s_comp.
    // steps > 0: a fused remainder launch of that many steps (< spl).
    void launch_once(bool two, int steps = 0) {
        if (!multi()) {
            Sub &s = subs[0];
            timed(s, s.s_comp, part_name(two, true, steps),
                  [&] { HIP_CHECK(launch_part(s, s.cur, two, true, s.s_comp, steps)); });
            s.cur ^= 1;
            return;
        }
        if (!forked) {
            for (auto &s : subs) {
                set_device(s);
                HIP_CHECK(hipEventRecord(s.ev_i, s.s_comp));  // B(first) after all prior s_comp work
            }
            forked = true;
        }
        std::vector<float *> tgt(subs.size());
        for (size_t k = 0; k < subs.size(); ++k) {
            Sub &s = subs[k];
            set_device(s);
            HIP_CHECK(hipStreamWaitEvent(s.s_bnd, s.ev_i, 0));
            wait_exchange_on(s, s.s_bnd);
            debug_delay(s, s.s_bnd);
            timed(s, s.s_bnd, part_name(two, false, steps),
                  [&] { HIP_CHECK(launch_part(s, s.cur, two, false, s.s_bnd, steps)); });
            HIP_CHECK(hipEventRecord(s.ev_b, s.s_bnd));
            HIP_CHECK(hipEventRecord(s.ev_bp[s.cur], s.s_bnd));
            tgt[k] = s.o[1 - s.cur];
        }
        exchange(two ? HALO_WG : HALO_W1, tgt);
        for (auto &s : subs) {
            set_device(s);
            HIP_CHECK(hipStreamWaitEvent(s.s_comp, s.ev_bp[1 - s.cur], 0));  // B(t-1)
            debug_delay(s, s.s_comp);
            timed(s, s.s_comp, part_name(two, true, steps),
                  [&] { HIP_CHECK(launch_part(s, s.cur, two, true, s.s_comp, steps)); });
            HIP_CHECK(hipEventRecord(s.ev_i, s.s_comp));
        }
        for (auto &s : subs) s.cur ^= 1;
    }

    // After a run of launch_once: s_comp waits for the last boundary launch
    // and the last exchange, so later s_comp work sees a complete state.
    void join() {
        if (!forked) return;
        for (auto &s : subs) {
            set_device(s);
            HIP_CHECK(hipStreamWaitEvent(s.s_comp, s.ev_bp[1 - s.cur], 0));
        }
        wait_exchange();
        forked = false;
    }

    void drop_graphs() {
        for (auto &g : graph_exec)
            if (g) {
                (void)hipGraphExecDestroy(g);
                g = nullptr;
            }
    }

    // Capture 2*graph_steps launches starting at parity `par` (single
    // sub-domain, no exchange): the step loop replays them instead of paying
    // a host launch per step.  Kernel arguments are per parity and the av
    // index is device-side, so one graph serves every replay.
    hipGraphExec_t graph_for(int par) {
        if (graph_exec[par]) return graph_exec[par];
        Sub &s = subs[0];
        set_device(s);
        hipGraph_t g = nullptr;
        HIP_CHECK(hipStreamBeginCapture(s.s_comp, hipStreamCaptureModeThreadLocal));
        int cur = par;
        for (int i = 0; i < 2 * graph_steps; ++i) {
            const hipError_t e = launch_part(s, cur, fused, true, s.s_comp);
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
        run_fused = run_single = 0;
        prof_drop();
        if (resident) {
            if (run_resident(steps, accelerate_first)) {
                run_fused = steps > 0 ? 1 : 0;
                return;
            }
            // Residency failure (another kernel held CUs, so part of the grid
            // waited behind tiles that waited for it): repeat the run on the
            // STEP2 kernel from the intact input lattice, which already
            // carries the run's first accelerate, and stay on STEP2 -- the
            // blocking engine.run(1) contract of LbmRunner.cpp:102-104 holds
            // whatever else runs on the device.
            resident = false;
            res_failed = true;
            ring_stale = true;  // the resident kernel kept no ghost ring
            accelerate_first = false;
            fprintf(stderr, "lbm: resident kernel hand-off timed out (tiles not co-resident); "
                            "run repeated on the step2 kernel, which this handle keeps from now on\n");
            prof_drop();
        }
        if (pipeline) {
            run_pipeline(steps);
            run_single = steps;
            return;
        }
        for (auto &s : subs) {  // stream-ordered before this run's first launch
            set_device(s);
            HIP_CHECK(hipMemsetAsync(s.ctl, 0, 64, s.s_comp));
        }
        if (multi()) sync_all();
        const int per_launch = fused ? spl : 1;
        const int launches = steps / per_launch;
        const int chunk = 2 * graph_steps;  // launches per graph replay (even: parity unchanged)
        const bool use_graph = !multi() && !profile && graph_steps > 0 && launches >= chunk;
        if (use_graph) (void)graph_for(subs[0].cur);  // capture + instantiate outside the timed region
        Sub &s0 = subs[0];
        set_device(s0);
        HIP_CHECK(hipEventRecord(t0, s0.s_comp));
        if (multi())
            for (size_t k = 1; k < subs.size(); ++k) {
                set_device(subs[k]);
                HIP_CHECK(hipStreamWaitEvent(subs[k].s_comp, t0, 0));
            }
        // a ring left partial by the previous run's remainder launch is rebuilt
        // first, inside this run's device timer: every run that needs the
        // rebuild pays for it exactly once (lbm_last_run_seconds)
        if (ring_stale) {
            refresh_halos();
            ring_stale = false;
        }
        if (accelerate_first && p.ny >= 2) {
            const float w1 = p.density * p.accel / 9.f;
            const float w2 = p.density * p.accel / 36.f;
            for (auto &s : subs) {
                if (s.accel_row < 0) continue;
                set_device(s);
                timed(s, s.s_comp, "accelerate_row", [&] {
                    HIP_CHECK(launch_accelerate(s.o[s.cur], s.obst, s.plane, s.pitch, s.w, s.accel_row, w1, w2, s.s_comp));
                });
            }
            refresh_halos();
        }
        int l = 0;
        if (use_graph) {
            set_device(s0);
            hipGraphExec_t ge = graph_for(s0.cur);
            for (; l + chunk <= launches; l += chunk) HIP_CHECK(hipGraphLaunch(ge, s0.s_comp));
        }
        for (; l < launches; ++l) launch_once(fused);
        int rem = steps - launches * per_launch;
        // remainder of a stream engine (2 <= rem < spl): ONE fused launch of
        // rem steps on the same work split and boundary bands (the strips'
        // overlap and the ghost ring are sized for spl >= rem).  The halo
        // tables and send buffers are laid out for spl; halo_out_g puts a
        // shorter launch's halo cells in the innermost rem ghost columns / rows
        // (send-buffer positions), where the periodic / neighbour images of
        // its cells belong, so the exchange of this launch leaves the rem-deep
        // ring right; the next run starts by restoring the whole spl-deep ring
        // (ring_stale)
        const bool fused_rem = fused && use_stream && rem >= 2;
        if (fused_rem) launch_once(true, rem);
        for (int i = 0; i < (fused_rem ? 0 : rem); ++i) launch_once(false);  // remainder: one-step kernel (W1 halo) ...
        run_fused = fused ? launches + (fused_rem ? 1 : 0) : 0;
        run_single = fused ? (fused_rem ? 0 : rem) : launches;
        join();
        if (rem > 0) ring_stale = true;                    // ... the next run restores the WG ring first
        for (auto &s : subs) {
            set_device(s);
            timed(s, s.s_comp, "finalize_av",
                  [&] { HIP_CHECK(launch_finalize(s.partials[1 - s.cur], s.av_local, s.ctl, s.s_comp)); });
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
        prof_collect();
        dump_trace();
    }

    // LBM_STREAM_TRACE=<file>: raw {start, end} s_memrealtime (100 MHz) per
    // block of sub-domain 0's last interior stream launch (tools/stream_trace.py)
    void dump_trace() {
        const char *path = knob_str("LBM_STREAM_TRACE");
        if (!path || !*path || subs.empty() || !subs[0].trace) return;
        Sub &s = subs[0];
        set_device(s);
        std::vector<unsigned long long> v(2 * (size_t)s.n3_int);
        HIP_CHECK(hipMemcpy(v.data(), s.trace, v.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        if (FILE *f = fopen(path, "wb")) {
            fwrite(v.data(), sizeof(unsigned long long), v.size(), f);
            fclose(f);
        }
    }

    void sync_all() {
        for (auto &s : subs) {
            set_device(s);
            HIP_CHECK(hipStreamSynchronize(s.s_comp));
            HIP_CHECK(hipStreamSynchronize(s.s_comm));
            HIP_CHECK(hipStreamSynchronize(s.s_bnd));
        }
    }

    // NaN / Inf populations in the current lattices of every local sub-domain
    long long nonfinite_count() {
        if (!loaded) throw lbm_failure(LBM_E_STATE, "nothing to scan");
        sync_all();
        long long total = 0;
        for (auto &s : subs) {
            set_device(s);
            unsigned long long *d = nullptr, hcount = 0;
            HIP_CHECK(hipMalloc(&d, sizeof(unsigned long long)));
            HIP_CHECK(hipMemsetAsync(d, 0, sizeof(unsigned long long), s.s_comp));
            const hipError_t e = launch_count_nonfinite(s.o[s.cur], s.plane, s.pitch, s.w, s.h, d, s.s_comp);
            if (e == hipSuccess) (void)hipMemcpyAsync(&hcount, d, sizeof(hcount), hipMemcpyDeviceToHost, s.s_comp);
            const hipError_t e2 = hipStreamSynchronize(s.s_comp);
            (void)hipFree(d);
            HIP_CHECK(e);
            HIP_CHECK(e2);
            total += (long long)hcount;
        }
        return total;
    }

    void check_finite_after_run() {
        if (!nan_check) return;
        const long long bad = nonfinite_count();
        if (bad > 0)
            throw lbm_failure(LBM_E_INTERNAL, "LBM_NAN_CHECK: " + std::to_string(bad) +
                                                  " non-finite populations in the lattice after the run");
    }

    void init_equilibrium() {
        const float c0 = p.density * 4.f / 9.f, c1 = p.density / 9.f, c2 = p.density / 36.f;
        for (auto &s : subs) {
            set_device(s);
            s.cur = 0;
            HIP_CHECK(launch_init_equilibrium(s.f[0], s.h + 2LL * gr, s.rf, s.pitch, s.plane, c0, c1, c2, s.s_comp));
        }
        sync_all();
        loaded = true;
        ring_stale = false;  // every row and column, ghosts included, is written
    }

    // Host AoS source / destination of sub-domain k: the full-domain array
    // (row stride nx cells, the sub-domain at its global rectangle) or, for
    // the *_local calls, the local sub-domains packed one after another in
    // lbm_local_rects order (row stride w cells).
    const float *aos_of(const float *aos, size_t k, bool local) const {
        if (!local) return aos + ((size_t)subs[k].rect.y0 * p.nx + subs[k].rect.x0) * Q;
        size_t off = 0;
        for (size_t i = 0; i < k; ++i) off += (size_t)subs[i].w * subs[i].h * Q;
        return aos + off;
    }
    size_t aos_pitch(const Sub &s, bool local) const { return sizeof(float) * Q * (size_t)(local ? s.w : p.nx); }

    void load_cells(const float *aos, bool local = false) {
        if (!aos) throw lbm_failure(LBM_E_INVALID, "cells must not be NULL");
        for (size_t k = 0; k < subs.size(); ++k) {
            Sub &s = subs[k];
            set_device(s);
            float *stage = nullptr;
            const size_t row_bytes = sizeof(float) * Q * (size_t)s.w;
            HIP_CHECK(hipMalloc(&stage, row_bytes * (size_t)s.h));
            HIP_CHECK(hipMemcpy2D(stage, row_bytes, aos_of(aos, k, local), aos_pitch(s, local), row_bytes, (size_t)s.h,
                                  hipMemcpyHostToDevice));
            s.cur = 0;
            HIP_CHECK(launch_aos_to_soa(stage, s.o[0], s.plane, s.pitch, s.w, s.h, s.s_comp));
            HIP_CHECK(hipStreamSynchronize(s.s_comp));
            HIP_CHECK(hipFree(stage));
        }
        refresh_halos();
        sync_all();
        loaded = true;
        ring_stale = false;
    }

    void store(float *aos, float *av, int n_av, bool local = false) {
        if (!loaded) throw lbm_failure(LBM_E_STATE, "nothing to store");
        sync_all();
        if (aos) {
            for (size_t k = 0; k < subs.size(); ++k) {
                Sub &s = subs[k];
                set_device(s);
                float *stage = nullptr;
                const size_t row_bytes = sizeof(float) * Q * (size_t)s.w;
                HIP_CHECK(hipMalloc(&stage, row_bytes * (size_t)s.h));
                HIP_CHECK(launch_soa_to_aos(s.o[s.cur], stage, s.plane, s.pitch, s.w, s.h, s.s_comp));
                HIP_CHECK(hipStreamSynchronize(s.s_comp));
                HIP_CHECK(hipMemcpy2D(const_cast<float *>(aos_of(aos, k, local)), aos_pitch(s, local), stage, row_bytes,
                                      row_bytes, (size_t)s.h, hipMemcpyDeviceToHost));
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
        prof_release();
        for (auto &s : subs) {
            if (hipSetDevice(s.dev) != hipSuccess) continue;
            (void)hipDeviceSynchronize();
            for (int k = 0; k < 2; ++k) {
                if (s.f[k] && !(k == 1 && s.f_joint)) (void)hipFree(s.f[k]);
                if (s.partials[k]) (void)hipFree(s.partials[k]);
            }
            if (s.obst) (void)hipFree(s.obst);
            if (s.pipe_partials) (void)hipFree(s.pipe_partials);
            if (s.dst2_dev) (void)hipFree(s.dst2_dev);
            if (s.uobst) (void)hipFree(s.uobst);
            if (s.uperm) (void)hipFree(s.uperm);
            if (s.trace) (void)hipFree(s.trace);
            if (s.obst_g) (void)hipFree(s.obst_g);
            if (s.halo_mem) (void)hipFree(s.halo_mem);
            if (s.av_local) (void)hipFree(s.av_local);
            if (s.ctl) (void)hipFree(s.ctl);
            if (s.s_comp) (void)hipStreamDestroy(s.s_comp);
            if (s.s_comm) (void)hipStreamDestroy(s.s_comm);
            if (s.s_bnd) (void)hipStreamDestroy(s.s_bnd);
            if (s.ev_i) (void)hipEventDestroy(s.ev_i);
            for (auto e : s.ev_bp)
                if (e) (void)hipEventDestroy(e);
            if (s.ev_b) (void)hipEventDestroy(s.ev_b);
            if (s.ev_u) (void)hipEventDestroy(s.ev_u);
            if (s.ev_end) (void)hipEventDestroy(s.ev_end);
        }
        if (res_halo) (void)hipFree(res_halo);
        if (res_partials) (void)hipFree(res_partials);
        if (res_status) (void)hipFree(res_status);
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

int lbm_exchange_schedule(int32_t nx, int32_t ny, int32_t parts, int32_t grid_rows, int32_t grid_cols, int32_t rank,
                          int32_t halo_mode, int32_t halo_width, int32_t force_exchange, lbm_xfer *out,
                          int32_t max_out, int32_t *n_out) {
    if (!n_out || (halo_mode != LBM_HALO_W1 && halo_mode != LBM_HALO_WG) || rank < 0 || rank >= parts ||
        (halo_mode == LBM_HALO_WG && (halo_width < 1 || halo_width > MAX_GR)))
        return LBM_E_INVALID;
    int R = 0, C = 0;
    std::vector<lbm_rect> rects;
    const int rc = partition(nx, ny, parts, grid_rows, grid_cols, R, C, rects);
    if (rc != LBM_OK) return rc;
    int nb[8];
    bool remote[8];
    torus_neighbours(rank, R, C, force_exchange != 0, nb, remote);
    const auto v = exchange_posts(rank, nb, remote, rects[rank].w, rects[rank].h, halo_mode,
                                  halo_mode == LBM_HALO_WG ? halo_width : 1);
    *n_out = (int32_t)v.size();
    if (out) {
        if (max_out < (int32_t)v.size()) return LBM_E_INVALID;
        for (size_t i = 0; i < v.size(); ++i) out[i] = v[i];
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
    return guarded(h, [&] {
        h->run_steps(h->p.max_iters, true);
        h->check_finite_after_run();
    });
}

int lbm_run_steps(lbm_handle *h, int32_t steps, int32_t accelerate_first) {
    if (!h) return LBM_E_INVALID;
    return guarded(h, [&] {
        h->run_steps(steps, accelerate_first != 0);
        h->check_finite_after_run();
    });
}

int lbm_nonfinite_count(lbm_handle *h, int64_t *count) {
    if (!h || !count) return LBM_E_INVALID;
    return guarded(h, [&] { *count = h->nonfinite_count(); });
}

int lbm_store(lbm_handle *h, float *cells_aos, float *av_vels, int32_t n_av) {
    if (!h) return LBM_E_INVALID;
    return guarded(h, [&] { h->store(cells_aos, av_vels, n_av); });
}

int lbm_load_cells_local(lbm_handle *h, const float *cells_aos_local) {
    if (!h) return LBM_E_INVALID;
    return guarded(h, [&] { h->load_cells(cells_aos_local, true); });
}

int lbm_store_local(lbm_handle *h, float *cells_aos_local, float *av_vels, int32_t n_av) {
    if (!h) return LBM_E_INVALID;
    return guarded(h, [&] { h->store(cells_aos_local, av_vels, n_av, true); });
}

int64_t lbm_local_cells(lbm_handle *h) {
    if (!h) return -1;
    int64_t n = 0;
    for (const auto &s : h->subs) n += (int64_t)s.w * s.h;
    return n;
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

int32_t lbm_kernel_in_use(lbm_handle *h) {
    if (!h) return LBM_KERNEL_SCALAR;
    if (h->resident) return LBM_KERNEL_RESIDENT;
    if (h->pipeline) return LBM_KERNEL_PIPELINE;
    if (h->fused) return h->use_stream ? LBM_KERNEL_STREAM : LBM_KERNEL_STEP2;
    return h->vec4 ? LBM_KERNEL_VEC4 : LBM_KERNEL_SCALAR;
}

int lbm_run_stats(lbm_handle *h, int32_t *fused_launches, int32_t *one_step_launches) {
    if (!h) return LBM_E_INVALID;
    if (fused_launches) *fused_launches = h->run_fused;
    if (one_step_launches) *one_step_launches = h->run_single;
    return LBM_OK;
}

int lbm_profile_summary(lbm_handle *h, lbm_kernel_time *out, int32_t max_out, int32_t *n_out) {
    if (!h || !n_out) return LBM_E_INVALID;
    if (!h->profile) {
        h->err = "handle was not created with LBM_FLAG_PROFILE";
        return LBM_E_STATE;
    }
    *n_out = (int32_t)h->prof_acc.size();
    for (int i = 0; out && i < (int)h->prof_acc.size() && i < max_out; ++i) {
        const auto &a = h->prof_acc[i];
        lbm_kernel_time &k = out[i];
        memset(&k, 0, sizeof(k));
        snprintf(k.name, sizeof(k.name), "%s", a.name.c_str());
        k.launches = a.launches;
        k.total_ms = a.total_ms;
        k.min_ms = a.launches ? a.min_ms : 0.0;
        k.max_ms = a.max_ms;
    }
    return LBM_OK;
}

int lbm_profile_reset(lbm_handle *h) {
    if (!h) return LBM_E_INVALID;
    h->prof_acc.clear();
    return LBM_OK;
}

int lbm_placement_probe(lbm_handle *h, int32_t *kept, int32_t *tried, float *ms_per_launch, int32_t max_ms) {
    if (!h) return LBM_E_INVALID;
    if (kept) *kept = h->probe_kept;
    if (tried) *tried = (int32_t)h->probe_ms.size();
    if (ms_per_launch)
        for (int i = 0; i < (int)h->probe_ms.size() && i < max_ms; ++i) ms_per_launch[i] = h->probe_ms[i];
    return LBM_OK;
}

int32_t lbm_numerics(lbm_handle *h) {
    if (!h) return -1;
    if (!h->tolerance || h->pipeline) return 0;
    if (h->resident) return RES_VER[h->res_variant] >= 2 ? 1 : 0;
    return (h->use_stream && h->fused) ? 1 : 0;
}

const char *lbm_source_hash(void) { return LBM_SOURCE_HASH; }

int32_t lbm_steps_per_launch(lbm_handle *h) {
    if (!h) return 0;
    if (h->resident) return std::max(1, h->last_steps > 0 ? h->last_steps : h->p.max_iters);
    return h->fused ? h->spl : 1;
}

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
