// lbm_engine.hpp -- declaration of the engine behind the C ABI
// (include/lbm_hip.h), shared by its units:
//   lbm_engine.hip        create, allocation, placement probe, the step loop,
//                         load / store / destroy (the run path);
//   lbm_exchange.hip      partition rule, torus neighbours, halo destinations,
//                         the posted exchange (RCCL or device copies);
//   lbm_split.hip         work decomposition: boundary / interior split,
//                         stream segments and tiers, kernel argument tables;
//   lbm_resident_run.hip  host side of the lattice-resident kernel (tile
//                         choice, launch, residency-failure fallback);
//   lbm_pipeline_run.hip  step loop of the unfused per-stage pipeline;
//   lbm_abi.hip           the extern "C" functions.
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

#pragma once

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

namespace lbm {
namespace eng {

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
bool choose_grid(int nx, int ny, int parts, int &rows, int &cols);

// Round-robin allocation (StructuredGridUtils.hpp:161-165): the first n % k parts get one more.
std::vector<int> round_robin(int n, int k);
int partition(int nx, int ny, int parts, int grid_rows, int grid_cols, int &R, int &C, std::vector<lbm_rect> &rects);

// Neighbours of sub-domain `id` on the R x C periodic torus of the
// reference's partition (rank = row * C + col; the periodic halo slices of
// StructuredGridUtils.hpp:805-851): nb[d] = the sub-domain across side d;
// remote[d] = side d goes through the exchange (else the step kernel writes
// the periodic image straight into the ghost ring).
void torus_neighbours(int id, int R, int C, bool force_exchange, int nb[8], bool remote[8]);

// The ordered transfers of one sub-domain's halo exchange (format `mode`,
// WG width `hw`): for d = E, N, W, S, NE, NW, SW, SE the send of the halo
// leaving through side d to nb[d] (or SELF: written in place by the step
// kernel), then the receive of ghost side OPP(d) from nb[OPP(d)].  RCCL
// pairs the messages between two ranks purely by this posting order (one
// ncclGroupStart/End), which is what lets extent-2 dimensions send several
// messages to one peer.  exchange() posts exactly this list;
// lbm_exchange_schedule exports it for host-side checking.
std::vector<lbm_xfer> exchange_posts(int id, const int nb[8], const bool remote[8], int w, int h, int mode, int hw);

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
}  // namespace eng
}  // namespace lbm

using namespace lbm;
using namespace lbm::eng;

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
    std::vector<std::pair<int, hipEvent_t>> prof_pool;    int prof_class(const std::string &name);
    hipEvent_t prof_event(int dev);
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
    void prof_collect();
    void prof_drop();
    void prof_release();
    std::string part_name(bool fused_launch, bool interior, int steps) const;
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
    void fill_fresh(void *ptr, size_t bytes, hipStream_t st) const;
    static void fill_zero(void *ptr, size_t bytes, hipStream_t st);
    void set_guide(const std::string &spec);
    static int env_int(const char *name, int dflt);
    // Tuning / A-B knobs are read only with LBM_DEBUG_KNOBS=1:
    // without it the library ignores the environment and runs its defaults
    // (LBM_POISON, a read-before-write check that changes no result of a
    // correct engine, is the one exception).
    int knob(const char *name, int dflt) const { return debug_knobs ? env_int(name, dflt) : dflt; }
    const char *knob_str(const char *name) const { return debug_knobs ? getenv(name) : nullptr; }
    void read_tuning();
    EdgeDst make_dst1(const Sub &s, float *org, int d) const;
    Dst2 self_dst2(const Sub &s, float *org, int d) const;
    Dst2 make_dst2(const Sub &s, float *org, int d) const;
    HaloArgs halo_args(const Sub &s, float *org, int mode, bool for_unpack) const;
    int fill_rects(Rect (&rect)[MAX_RECTS], int (&begin)[MAX_RECTS], int &nrect, const std::vector<Rect> &rs,
                   int unit_w, bool tiles_are_items) const;
    void split(const Sub &s, int nx_u, int ny_u, int xs_hi, int ys_hi, std::vector<Rect> &bnd,
               std::vector<Rect> &inr) const;
    void build_args(Sub &s);
    void stream_split(const Sub &s, std::vector<SRect> &inr, std::vector<SRect> &bnd) const;
    bool tiers_fit(long long strips, int h, long long cap) const;

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
    int fill_srects(StreamArgs &a, const std::vector<SRect> &rs) const;
    void ensure_av(int n);
    void create(const lbm_params *prm, const uint8_t *obstacles, const lbm_config &cfg);
    bool setup_resident(const Sub &s);
    bool run_resident(int steps, bool accelerate_first);
    void run_pipeline(int steps);
    void alloc_sub(Sub &s, const uint8_t *obstacles);
    Sub *local_sub(int id);
    void exchange(int mode, const std::vector<float *> &target);
    void set_stream_lattices(Sub &s, float *f0, float *f1);
    void placement_probe(Sub &s);
    void wait_exchange_on(Sub &s, hipStream_t st);
    void wait_exchange();
    void refresh_halos();
    void debug_delay(const Sub &s, hipStream_t st) const;
    int rem_form(int steps) const;
    hipError_t launch_part(Sub &s, int cur, bool fused_launch, bool interior, hipStream_t st, int steps = 0) const;
    void launch_once(bool two, int steps = 0);
    void join();
    void drop_graphs();
    hipGraphExec_t graph_for(int par);
    void run_steps(int steps, bool accelerate_first);
    void dump_trace();
    void sync_all();
    long long nonfinite_count();
    void check_finite_after_run();
    void init_equilibrium();
    const float *aos_of(const float *aos, size_t k, bool local) const;
    size_t aos_pitch(const Sub &s, bool local) const { return sizeof(float) * Q * (size_t)(local ? s.w : p.nx); }
    void load_cells(const float *aos, bool local = false);
    void store(float *aos, float *av, int n_av, bool local = false);
    void destroy();
};
