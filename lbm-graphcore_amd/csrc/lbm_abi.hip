// lbm_abi.hip -- the extern "C" functions of include/lbm_hip.h over the engine.

#include "lbm_engine.hpp"

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
