// lbm_split.hip -- work decomposition: boundary / interior split, stream-kernel
// segments and tiers, per-parity kernel argument tables.

#include "lbm_engine.hpp"

// LBM_STREAM_GUIDE tiers "h1:f1,h2:f2,...,hK" (see guided_rects); "0" = uniform
void lbm_handle::set_guide(const std::string &spec) {
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

// ---- work decomposition ---------------------------------------------
int lbm_handle::fill_rects(Rect (&rect)[MAX_RECTS], int (&begin)[MAX_RECTS], int &nrect, const std::vector<Rect> &rs,
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
void lbm_handle::split(const Sub &s, int nx_u, int ny_u, int xs_hi, int ys_hi, std::vector<Rect> &bnd,
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

void lbm_handle::build_args(Sub &s) {
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
void lbm_handle::stream_split(const Sub &s, std::vector<SRect> &inr, std::vector<SRect> &bnd) const {
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
bool lbm_handle::tiers_fit(long long strips, int h, long long cap) const {
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

int lbm_handle::fill_srects(StreamArgs &a, const std::vector<SRect> &rs) const {
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

void lbm_handle::ensure_av(int n) {
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
