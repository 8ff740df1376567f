// lbm_exchange.hip -- partition rule (StructuredGridUtils.hpp:472-561), torus neighbours,
// halo destinations and the posted halo exchange (RCCL grouped send/recv or
// device copies; StructuredGridUtils.hpp:805-851, LbmAoS.cpp:151-160).

#include "lbm_engine.hpp"

namespace lbm {
namespace eng {

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

void torus_neighbours(int id, int R, int C, bool force_exchange, int nb[8], bool remote[8]) {
    const int row = id / C, col = id % C;
    for (int d = 0; d < 8; ++d) {
        const int r = ((row + DIR_Y[d]) % R + R) % R;
        const int c = ((col + DIR_X[d]) % C + C) % C;
        nb[d] = r * C + c;
        remote[d] = force_exchange || nb[d] != id;
    }
}

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

}  // namespace eng
}  // namespace lbm

// ---- halo destinations --------------------------------------------
// W1: populations leaving through d -> own ghost ring (opposite side) or send[d]
EdgeDst lbm_handle::make_dst1(const Sub &s, float *org, int d) const {
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
Dst2 lbm_handle::self_dst2(const Sub &s, float *org, int d) const {
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

Dst2 lbm_handle::make_dst2(const Sub &s, float *org, int d) const {
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

HaloArgs lbm_handle::halo_args(const Sub &s, float *org, int mode, bool for_unpack) const {
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

Sub * lbm_handle::local_sub(int id) {
    for (auto &s : subs)
        if (s.id == id) return &s;
    return nullptr;
}

// ------------------------------------------------------------------
// Exchange of the halo send buffers (format `mode`), after every
// sub-domain recorded ev_b on its compute stream.  `target[k]` is the
// lattice origin of local sub k whose ghost ring receives.  Ends with the
// unpack and ev_u recorded on each comm stream.
void lbm_handle::exchange(int mode, const std::vector<float *> &target) {
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

// `st` waits for the last exchange: own ghosts unpacked, and (LOCAL)
// every neighbour done reading this sub-domain's send buffers.
void lbm_handle::wait_exchange_on(Sub &s, hipStream_t st) {
    HIP_CHECK(hipStreamWaitEvent(st, s.ev_u, 0));
    if (transport == LBM_TRANSPORT_LOCAL)
        for (int d = 0; d < 8; ++d)
            if (s.remote[d]) HIP_CHECK(hipStreamWaitEvent(st, local_sub(s.nb[d])->ev_u, 0));
}

void lbm_handle::wait_exchange() {
    for (auto &s : subs) {
        set_device(s);
        wait_exchange_on(s, s.s_comp);
    }
}

// Make every ghost cell of the current lattices consistent in the
// current mode's format (after load, init, accelerate, or a trailing
// one-step launch in two-step mode).
void lbm_handle::refresh_halos() {
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
