// lbm_engine.hip -- the run path: create, allocation, placement probe, the step loop
// (launch_once / run_steps), load / store, destroy.

#include "lbm_engine.hpp"

  // (device, event) free list

int lbm_handle::prof_class(const std::string &name) {
    for (size_t i = 0; i < prof_acc.size(); ++i)
        if (prof_acc[i].name == name) return (int)i;
    prof_acc.push_back(ProfAcc{name});
    return (int)prof_acc.size() - 1;
}

hipEvent_t lbm_handle::prof_event(int dev) {
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

// after a run's streams are synchronised: fold this run's records
void lbm_handle::prof_collect() {
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
void lbm_handle::prof_drop() {
    for (auto &r : prof_open) {
        prof_pool.push_back({r.dev, r.a});
        prof_pool.push_back({r.dev, r.b});
    }
    prof_open.clear();
}

void lbm_handle::prof_release() {
    for (auto &r : prof_open) {
        prof_pool.push_back({r.dev, r.a});
        prof_pool.push_back({r.dev, r.b});
    }
    prof_open.clear();
    for (auto &e : prof_pool) (void)hipEventDestroy(e.second);
    prof_pool.clear();
}

std::string lbm_handle::part_name(bool fused_launch, bool interior, int steps) const {
    const char *where = multi() ? (interior ? " interior" : " boundary") : "";
    if (fused_launch && use_stream)
        return std::string("stream_steps2d S=") + std::to_string(steps > 0 ? steps : spl) +
               (tolerance ? " tolerance" : "") + where;
    if (fused_launch) return std::string("step2") + where;
    return std::string(vec4 ? "step_vec4" : "step_scalar") + where;
}

// Initial fill of a fresh device allocation, ordered on `st` and waited
// for (the engine's streams are non-blocking: a null-stream hipMemset is
// not ordered with them).  Zero, or with LBM_POISON=1 all-ones bytes (a
// NaN in every float), so that a value the engine reads without having
// written it shows up as NaN in the lattice or in av_vels (SURVEY §5
// sanitizer row; tests/test_poison.py).
void lbm_handle::fill_fresh(void *ptr, size_t bytes, hipStream_t st) const {
    HIP_CHECK(hipMemsetAsync(ptr, poison ? 0xFF : 0, bytes, st));
    HIP_CHECK(hipStreamSynchronize(st));
}

// Protocol words whose zero IS their initialisation (control block, status)
void lbm_handle::fill_zero(void *ptr, size_t bytes, hipStream_t st) {
    HIP_CHECK(hipMemsetAsync(ptr, 0, bytes, st));
    HIP_CHECK(hipStreamSynchronize(st));
}

int lbm_handle::env_int(const char *name, int dflt) {
    const char *v = getenv(name);
    return (v && *v) ? atoi(v) : dflt;
}

void lbm_handle::read_tuning() {
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

// ------------------------------------------------------------------
void lbm_handle::create(const lbm_params *prm, const uint8_t *obstacles, const lbm_config &cfg) {
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

void lbm_handle::alloc_sub(Sub &s, const uint8_t *obstacles) {
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

// Point the v3 stream arguments of s at lattices f0 / f1 (placement probe).
void lbm_handle::set_stream_lattices(Sub &s, float *f0, float *f1) {
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
void lbm_handle::placement_probe(Sub &s) {
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

// debug stall of sub-domain s's stream st (LBM_DEBUG_DELAY_SUB / _US)
void lbm_handle::debug_delay(const Sub &s, hipStream_t st) const {
    if (delay_us > 0 && s.id == delay_sub) HIP_CHECK(launch_debug_spin(delay_us, st));
}

// launch form of a fused remainder launch of `steps` < spl steps: the
// engine's form where it has that depth, else the shallowest that does
int lbm_handle::rem_form(int steps) const {
    if (s2d_form_ok(steps, stream_cfg, tolerance)) return stream_cfg;
    return steps > 6 ? 4 : 0;
}

// Interior (reducing) or boundary launch of sub-domain s reading parity
// `cur`: one fused launch (spl steps, WG halo) or one step (W1 halo).
// steps > 0 (single sub-domain stream engines): a remainder launch of that
// many fused steps (< spl) on the same work split and halo tables.
hipError_t lbm_handle::launch_part(Sub &s, int cur, bool fused_launch, bool interior, hipStream_t st, int steps) const {
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
void lbm_handle::launch_once(bool two, int steps) {
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
void lbm_handle::join() {
    if (!forked) return;
    for (auto &s : subs) {
        set_device(s);
        HIP_CHECK(hipStreamWaitEvent(s.s_comp, s.ev_bp[1 - s.cur], 0));
    }
    wait_exchange();
    forked = false;
}

void lbm_handle::drop_graphs() {
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
hipGraphExec_t lbm_handle::graph_for(int par) {
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

void lbm_handle::run_steps(int steps, bool accelerate_first) {
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
void lbm_handle::dump_trace() {
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

void lbm_handle::sync_all() {
    for (auto &s : subs) {
        set_device(s);
        HIP_CHECK(hipStreamSynchronize(s.s_comp));
        HIP_CHECK(hipStreamSynchronize(s.s_comm));
        HIP_CHECK(hipStreamSynchronize(s.s_bnd));
    }
}

// NaN / Inf populations in the current lattices of every local sub-domain
long long lbm_handle::nonfinite_count() {
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

void lbm_handle::check_finite_after_run() {
    if (!nan_check) return;
    const long long bad = nonfinite_count();
    if (bad > 0)
        throw lbm_failure(LBM_E_INTERNAL, "LBM_NAN_CHECK: " + std::to_string(bad) +
                                              " non-finite populations in the lattice after the run");
}

void lbm_handle::init_equilibrium() {
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
const float * lbm_handle::aos_of(const float *aos, size_t k, bool local) const {
    if (!local) return aos + ((size_t)subs[k].rect.y0 * p.nx + subs[k].rect.x0) * Q;
    size_t off = 0;
    for (size_t i = 0; i < k; ++i) off += (size_t)subs[i].w * subs[i].h * Q;
    return aos + off;
}

void lbm_handle::load_cells(const float *aos, bool local) {
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

void lbm_handle::store(float *aos, float *av, int n_av, bool local) {
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

void lbm_handle::destroy() {
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
