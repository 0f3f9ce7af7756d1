// api.cpp -- C ABI (include/mhnsw.h) over the HIP kernels: handle lifecycle,
// options, Add / BatchAdd (levels drawn like graph.go:388-417, the compat and
// batched build schedules), Delete, statistics.  Searches: search_host.cpp;
// export / import and string keys: io_host.cpp; the shared state: index.hpp.
// The graph lives in HBM; the host keeps only the key -> internal-id map,
// per-node levels and per-layer counts/entries.
#include "index.hpp"

#include <functional>
#include <unordered_set>

using namespace mhh;

namespace mhh {

thread_local std::string g_create_err;

int fail(mhnsw_index* h, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (h)
        h->err = buf;
    else
        g_create_err = buf;
    return code;
}

// graph.go:916-937
int validate(mhnsw_index* h) {
    if (h->M <= 0) return fail(h, MHNSW_EINVAL, "M must be greater than 0, got %d", h->M);
    if (h->ml <= 0 || h->ml >= 1) return fail(h, MHNSW_EINVAL, "Ml must be between 0 and 1 (exclusive), got %f", h->ml);
    if (h->ef <= 0) return fail(h, MHNSW_EINVAL, "EfSearch must be greater than 0, got %d", h->ef);
    if (h->metric != COSINE && h->metric != EUCLIDEAN) return fail(h, MHNSW_EINVAL, "Distance function must be set");
    return MHNSW_OK;
}

// graph.go:370-385
int max_level(double ml, int64_t num) {
    if (ml == 0) return -1;
    if (num == 0) return 1;
    double l = std::log((double)num);
    l /= std::log(1.0 / ml);
    return (int)std::round(l) + 1;
}

// SplitMix64 draw (same stream as oracle/oracle.c og_rng_next)
double rng_next(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z = z ^ (z >> 31);
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

// graph.go:388-417 randomLevel with the layer-0 size before this insert
int random_level(double ml, bool layers_exist, int64_t count, uint64_t* rng) {
    int max = 1;
    if (layers_exist) max = max_level(ml, count);
    for (int level = 0; level < max; ++level) {
        double r = rng_next(rng);
        if (r > ml) return level;
    }
    return max;
}

int m0_of(const mhnsw_index* h) {
    if (h->build_mode == MHNSW_BUILD_COMPAT) return h->M;
    return h->m0 > 0 ? h->m0 : 2 * h->M;
}
int cap_of(const mhnsw_index* h, int l) {
    const int m = l == 0 ? m0_of(h) : h->M;
    return m + 1;  // addNeighbor overflows by one before evicting (graph.go:50-53)
}



int ensure_layer(mhnsw_index* h, int l) {
    while ((int)h->layers.size() <= l) {
        if ((int)h->layers.size() >= MH_MAXL) return fail(h, MHNSW_EUNSUPPORTED, "more than %d layers", MH_MAXL);
        Layer L;
        L.cap = cap_of(h, (int)h->layers.size());
        const int64_t c = std::max<int64_t>(h->capn, 1);
        int r;
        if ((r = grow(h, L.deg, 0, c, -1, true, 0xFFFFFFFEu))) return r;
        if ((r = grow(h, L.adj, 0, c * L.cap, 0xFF))) return r;
        if ((r = grow(h, L.adjd, 0, c * L.cap, 0))) return r;
        h->layers.push_back(L);
    }
    return 0;
}

// re-stride adjacency when M (or M0) grew beyond the allocated row width
int ensure_caps(mhnsw_index* h) {
    for (int l = 0; l < (int)h->layers.size(); ++l) {
        Layer& L = h->layers[l];
        const int need = cap_of(h, l);
        if (need <= L.cap) continue;
        const int64_t c = std::max<int64_t>(h->capn, 1);
        int32_t* na = nullptr;
        float* nd = nullptr;
        if (hipMalloc(&na, (size_t)c * need * 4) != hipSuccess || hipMalloc(&nd, (size_t)c * need * 4) != hipSuccess)
            return fail(h, MHNSW_ENOMEM, "device allocation failed");
        HIPCHK(h, hipMemsetAsync(na, 0xFF, (size_t)c * need * 4, h->stream));
        HIPCHK(h, hipMemcpy2DAsync(na, need * 4, L.adj, L.cap * 4, L.cap * 4, c, hipMemcpyDeviceToDevice, h->stream));
        HIPCHK(h, hipMemcpy2DAsync(nd, need * 4, L.adjd, L.cap * 4, L.cap * 4, c, hipMemcpyDeviceToDevice, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        (void)hipFree(L.adj);
        (void)hipFree(L.adjd);
        L.adj = na;
        L.adjd = nd;
        L.cap = need;
    }
    return 0;
}

int ensure_capacity(mhnsw_index* h, int64_t need) {
    if (h->max_rows > 0 && need > h->max_rows)
        return fail(h, MHNSW_ENOMEM, "row capacity limit: %lld rows > max_rows %lld", (long long)need,
                    (long long)h->max_rows);
    if (need <= h->capn) return 0;
    int64_t nc = std::max<int64_t>(need, std::max<int64_t>(1024, h->capn * 2));
    if (h->capn > 0) nc = std::max<int64_t>(need, h->capn + h->capn / 2);
    const int64_t oc = h->capn;
    int r;
    if ((r = grow(h, h->vecs, oc * h->pitch, nc * h->pitch, 0))) return r;
    if ((r = grow(h, h->norms, oc, nc, 0))) return r;
    if (h->screen & 1) {
        if ((r = grow(h, h->h16, oc * h->pitch, nc * h->pitch, 0))) return r;
        if ((r = grow(h, h->h16aux, oc, nc, 0xFF))) return r;
    }
    if ((r = grow(h, h->keys, oc, nc, 0))) return r;
    if ((r = grow(h, h->levels, oc, nc, 0))) return r;
    if ((r = grow(h, h->dead, oc, nc, 0))) return r;
    if (h->aliased && ((r = grow(h, h->kid, oc, nc, 0xFF)) || (r = grow(h, h->kidlive, oc, nc, 0xFF)) ||
                       (r = grow(h, h->kprev, oc, nc, 0xFF))))
        return r;
    if ((r = grow(h, h->cur_entry, 0, nc, 0))) return r;
    if ((r = grow(h, h->inc_cnt, 0, nc, 0))) return r;
    if (h->build_mode == MHNSW_BUILD_BATCH || h->inc_src) {
        if ((r = grow(h, h->inc_src, 0, nc * h->inc_cap, 0))) return r;
        if ((r = grow(h, h->inc_dist, 0, nc * h->inc_cap, 0))) return r;
    }
    for (auto& L : h->layers) {
        if ((r = grow(h, L.deg, oc, nc, -1, true, 0xFFFFFFFEu))) return r;
        if ((r = grow(h, L.adj, oc * L.cap, nc * L.cap, 0xFF))) return r;
        if ((r = grow(h, L.adjd, oc * L.cap, nc * L.cap, 0))) return r;
    }
    h->capn = nc;
    return 0;
}

// mirror the per-layer pointers into the device table read by the kernels
int sync_layer_table(mhnsw_index* h) {
    LayerDev t[MH_MAXL];
    memset(t, 0, sizeof(t));
    for (int l = 0; l < (int)h->layers.size(); ++l) {
        t[l].deg = h->layers[l].deg;
        t[l].adj = h->layers[l].adj;
        t[l].adjd = h->layers[l].adjd;
        t[l].cap = h->layers[l].cap;
    }
    if (memcmp(t, h->layers_host, sizeof(t)) == 0) return 0;
    memcpy(h->layers_host, t, sizeof(t));
    HIPCHK(h, hipMemcpyAsync(h->d_layers, h->layers_host, sizeof(t), hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

GraphDev graph_view(const mhnsw_index* h) {
    GraphDev g;
    memset(&g, 0, sizeof(g));
    g.vecs = h->vecs;
    g.norms = h->norms;
    g.keys = h->keys;
    g.layers = h->d_layers;
    g.pitch = h->pitch;
    g.dim = h->dim;
    g.metric = h->metric;
    g.nlayers = (int)h->layers.size();
    g.capn = (uint32_t)std::max<int64_t>(h->capn, 1);
    g.err = h->d_err;
    g.dead = h->any_dead ? h->dead : nullptr;
    g.h16 = (h->screen & 1) ? h->h16 : nullptr;
    g.h16aux = h->h16aux;
    g.h16err = h->h16err;
    if (h->h16_metric != h->metric) g.h16 = nullptr;  // stale format: no screening
    g.kid = h->aliased ? h->kid : nullptr;
    g.kidlive = h->aliased ? h->kidlive : nullptr;
    g.kprev = h->aliased ? h->kprev : nullptr;
    return g;
}

int64_t live_count(const mhnsw_index* h) { return h->layers.empty() ? 0 : h->layers[0].count; }

// highest layer holding a live node (Search skips emptied top layers, graph.go:572-582)
int top_live_layer(const mhnsw_index* h) {
    int top = (int)h->layers.size() - 1;
    while (top > 0 && h->layers[top].count == 0) --top;
    return top;
}

bool in_layer(const mhnsw_index* h, int64_t id, int l) { return (h->hmask[id] >> l) & 1u; }

// lowest-id live member: the deterministic stand-in for entry() (graph.go:250-258)
void fix_entries(mhnsw_index* h) {
    for (int l = 0; l < (int)h->layers.size(); ++l) {
        Layer& L = h->layers[l];
        if (L.entry >= 0 && in_layer(h, L.entry, l) && !h->hdead[L.entry]) continue;
        L.entry = -1;
        if (L.count == 0) continue;
        for (int64_t i = 0; i < h->n; ++i)
            if (in_layer(h, i, l) && !h->hdead[i]) {
                L.entry = (int32_t)i;
                break;
            }
    }
}

int set_shape(mhnsw_index* h, int dim) {
    int lpr, vpl;
    if (!pick_cfg(dim, lpr, vpl)) return fail(h, MHNSW_EUNSUPPORTED, "dimension %d not supported (1..4096)", dim);
    h->dim = dim;
    h->lpr = lpr;
    h->vpl = vpl;
    h->pitch = pitch_of(lpr, vpl);
    return 0;
}

int set_deg(mhnsw_index* h, int l, int64_t id, int32_t v) {
    HIPCHK(h, hipMemcpyAsync(h->layers[l].deg + id, &v, 4, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int sync_layer_entries(mhnsw_index* h) {
    int32_t e[MH_MAXL];
    for (int l = 0; l < MH_MAXL; ++l)
        e[l] = l < (int)h->layers.size() && h->layers[l].count > 0 ? h->layers[l].entry : -1;
    HIPCHK(h, hipMemcpyAsync(h->d_layer_entry, e, sizeof(e), hipMemcpyHostToDevice, h->stream));
    return 0;
}

int zero_err(mhnsw_index* h) {
    HIPCHK(h, hipMemsetAsync(h->d_err, 0, sizeof(int), h->stream));
    return 0;
}

// ---------------------------------------------------------------------------
// build drivers
// ---------------------------------------------------------------------------
// BatchAdd of a present key (graph.go:1015-1024): the launch's last insert
struct CompatRep {
    int level = -1, i0 = -1;  // level -1: none
    int32_t a = -1, b = -1;   // rows above i0 / from i0 down
    const int32_t* entry = nullptr;  // [MH_MAXL] entry() at each layer's turn (the row itself: empty then)
    const int32_t* sweep = nullptr;  // [MH_MAXL] row deleted + isolated per layer (-1 none)
};

// fresh inserts [n0, n1) then cr's; entry: [MH_MAXL] layer entries the fresh
// inserts see.  On the reference's "no nodes found in neighborhood search"
// returns 0 with *fail_row / *fail_layer set (the caller unwinds).
int run_build_compat(mhnsw_index* h, int64_t n0, int64_t n1, int top0, const int32_t* entry, const CompatRep& cr,
                     int64_t* fail_row, int* fail_layer) {
    if (h->M + 1 > 64) return fail(h, MHNSW_EUNSUPPORTED, "compat build supports M <= 63");
    int r;
    int32_t e[3 * MH_MAXL];
    for (int l = 0; l < MH_MAXL; ++l) {
        e[l] = entry[l];
        e[MH_MAXL + l] = cr.entry ? cr.entry[l] : -1;
        e[2 * MH_MAXL + l] = cr.sweep ? cr.sweep[l] : -1;
    }
    HIPCHK(h, hipMemcpyAsync(h->d_layer_entry, e, sizeof(e), hipMemcpyHostToDevice, h->stream));
    if ((r = sync_layer_table(h))) return r;  // (e stays alive until the stream sync below)
    HIPCHK(h, hipMemsetAsync(h->d_err, 0, 4 * sizeof(int), h->stream));
    CompatBuildArgs a;
    a.g = graph_view(h);
    a.n0 = n0;
    a.n1 = n1;
    a.levels = h->levels;
    a.layer_entry = h->d_layer_entry;
    a.top0 = top0;
    a.M = h->M;
    a.ef = h->ef;
    a.stats = h->d_stats + 4;
    a.err = h->d_err;
    a.vis_log2 = h->vis_log2;
    a.rep_level = cr.level;
    a.rep_i0 = cr.i0;
    a.rep_a = cr.a >= 0 ? (uint32_t)cr.a : EMPTY_ID;
    a.rep_b = cr.b >= 0 ? (uint32_t)cr.b : EMPTY_ID;
    a.rep_entry = h->d_layer_entry + MH_MAXL;
    a.rep_sweep = h->d_layer_entry + 2 * MH_MAXL;
    int lr = launch_build_compat(a, h->lpr, h->vpl, h->compat_waves, h->stream);
    if (lr == -2) return fail(h, MHNSW_EUNSUPPORTED, "compat build LDS budget exceeded (ef=%d, M=%d)", h->ef, h->M);
    LCHK(h, lr);
    int err[4] = {0, 0, 0, 0};
    HIPCHK(h, hipMemcpyAsync(err, h->d_err, sizeof(err), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (err[0] & 1) return fail(h, MHNSW_EINTERNAL, "visited set overflow (raise vis_log2)");
    if (err[0] & 4) return fail(h, MHNSW_EINTERNAL, "out-of-range node id in adjacency (graph corrupt)");
    if (err[0] & 8) return fail(h, MHNSW_EINTERNAL, "replenish candidate heap overflow");
    if (err[0] & 2) {
        *fail_layer = err[2];
        *fail_row = err[3];
    }
    return 0;
}

// One batch of the batched insert.  fuse_descent (default): one launch walks
// every node's greedy descent through the layers above its level, then layer
// l's search launch covers only the nodes with level >= l (a prefix of the
// batch sorted by level); otherwise every layer's launch covers the whole
// batch and descends the others itself.  Both read each layer before its
// commit, so they build the same graph.
int run_batch_layers(mhnsw_index* h, int64_t a0, int64_t a1, int top, uint32_t entry) {
    if (a1 <= a0) return 0;
    HIPCHK(h, hipMemsetD32Async((hipDeviceptr_t)(h->cur_entry + a0), (int)entry, (size_t)(a1 - a0), h->stream));
    int maxlvl = 0;
    for (int64_t i = a0; i < a1; ++i) maxlvl = std::max(maxlvl, h->hlevels[i]);
    int r;
    if ((r = sync_layer_table(h))) return r;
    const int efc = h->efc > 0 ? h->efc : h->ef;
    const int64_t nb = a1 - a0;
    std::vector<int64_t> count(MH_MAXL + 1, 0);  // nodes with level >= l
    const bool fuse = h->fuse_descent != 0;
    if (fuse) {
        if (h->ord_cap < nb) {
            if (h->ord_pin) (void)hipHostFree(h->ord_pin);
            h->ord_pin = nullptr;
            h->ord_cap = 0;
            if (hipHostMalloc((void**)&h->ord_pin, (size_t)nb * 4, hipHostMallocDefault) != hipSuccess)
                return fail(h, MHNSW_ENOMEM, "pinned allocation failed");
            h->ord_cap = nb;
        }
        if ((r = ensure_buf(h, h->border, (size_t)nb))) return r;
        if (h->ord_pending) HIPCHK(h, hipEventSynchronize(h->ord_ev));  // the previous batch's copy has read ord_pin
        for (int64_t i = a0; i < a1; ++i) count[std::min(h->hlevels[i], MH_MAXL)]++;
        for (int l = MH_MAXL - 1; l >= 0; --l) count[l] += count[l + 1];
        std::vector<int64_t> pos(MH_MAXL + 1, 0);  // level-descending, stable within a level
        for (int l = 0; l <= MH_MAXL; ++l) pos[l] = l < MH_MAXL ? count[l + 1] : 0;
        for (int64_t i = a0; i < a1; ++i) h->ord_pin[pos[std::min(h->hlevels[i], MH_MAXL)]++] = (uint32_t)i;
        HIPCHK(h, hipMemcpyAsync(h->border.p, h->ord_pin, (size_t)nb * 4, hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, hipEventRecord(h->ord_ev, h->stream));
        h->ord_pending = true;
    }
    auto args = [&](int l) {
        const int mcap = l == 0 ? m0_of(h) : h->M;
        BatchBuildArgs a;
        a.order = nullptr;
        a.count = 0;
        a.g = graph_view(h);
        a.layer = l;
        a.n0 = a0;
        a.n1 = a1;
        a.levels = h->levels;
        a.cur_entry = h->cur_entry;
        // upper_efc: a narrower candidate list in the layers above 0 (their rows hold M,
        // their searches are the build's narrow, latency-bound launches)
        a.ef = std::max(l > 0 && h->upper_efc > 0 ? std::min(efc, h->upper_efc) : efc, mcap);
        a.mcap = mcap;
        a.heuristic = h->heuristic;
        a.keep_pruned = h->keep_pruned;
        a.expand = h->build_expand;
        a.alpha = (float)h->alpha_pct / 100.0f;
        a.inc_cnt = h->inc_cnt;
        a.inc_src = h->inc_src;
        a.inc_dist = h->inc_dist;
        a.inc_cap = h->inc_cap;
        a.touched = h->touched;
        a.touched_cnt = h->touched_cnt;
        a.stats = h->d_stats + 4;
        a.vis_log2 = h->vis_log2;
        a.mw_max = h->build_mw_max;
        // the compact visited set where it holds more than the 32-bit one in about the
        // same LDS, for searches wide enough to fill that (efConstruction > 128;
        // at efC 64 the plain set never fills and its probe is cheaper)
        // (only in place of the 2^12-entry set: the LDS batch_lds sizes is the same
        // 16 KiB; a larger vis_log2 keeps the larger 32-bit set the user asked for)
        a.vis16 = h->vis_compact && a.ef > 128 && h->capn <= (int64_t(1) << 24) && h->vis_log2 == 12;
        return a;
    };
    // time_build: HIP events around every insert kernel (descent, layer searches, commits)
    auto tmark = [&]() -> int {
        if (!h->time_build) return 0;
        if (h->tev_used == h->tev.size()) {
            hipEvent_t e;
            HIPCHK(h, hipEventCreate(&e));
            h->tev.push_back(e);
        }
        HIPCHK(h, hipEventRecord(h->tev[h->tev_used++], h->stream));
        return 0;
    };
    for (int l = top; l >= 0; --l) {
        BatchBuildArgs a = args(l);
        const int mcap = a.mcap;
        if (fuse) {
            if (l == top) {
                if ((r = tmark())) return r;
                LCHK(h, launch_build_batch_descend(a, h->lpr, h->vpl, h->stream));  // a.layer = top
                if ((r = tmark())) return r;
            }
            if (l > maxlvl) continue;
            a.order = h->border.p;
            a.count = count[std::min(l, MH_MAXL)];
        }
        HIPCHK(h, hipMemsetAsync(h->touched_cnt, 0, 4, h->stream));
        if ((r = tmark())) return r;
        LCHK(h, launch_build_batch_search(a, h->lpr, h->vpl, h->stream));
        if (maxlvl >= l) LCHK(h, launch_build_batch_commit(a, h->lpr, h->vpl, (a1 - a0) * mcap, h->stream));
        if ((r = tmark())) return r;
    }
    return 0;
}

// top / entry: the live top layer and its entry before this batch (-1: empty graph)
int run_build_batch(mhnsw_index* h, int64_t n0, int64_t n1, int top, uint32_t entry,
                    const std::function<void()>& while_gpu) {
    int r;
    if ((r = zero_err(h))) return r;
    if (!h->inc_src) {
        if ((r = grow(h, h->inc_src, 0, h->capn * h->inc_cap, 0))) return r;
        if ((r = grow(h, h->inc_dist, 0, h->capn * h->inc_cap, 0))) return r;
    }
    const size_t tneed = (size_t)h->batch_max * (size_t)std::max(m0_of(h), h->M) + 64;
    if (h->touched_cap < tneed) {
        if (h->touched) (void)hipFree(h->touched);
        if (hipMalloc(&h->touched, tneed * 4) != hipSuccess) return fail(h, MHNSW_ENOMEM, "device allocation failed");
        h->touched_cap = tneed;
    }
    int64_t i = n0;
    while (i < n1) {
        const int lv = h->hlevels[i];
        if (top < 0) {  // first node of the graph: alone in every layer
            for (int l = 0; l <= lv; ++l)
                if ((r = set_deg(h, l, i, 0))) return r;
            top = lv;
            entry = (uint32_t)i;
            ++i;
            continue;
        }
        if (lv > top) {  // new top layers: insert alone, then it becomes the entry
            for (int l = top + 1; l <= lv; ++l)
                if ((r = set_deg(h, l, i, 0))) return r;
            if ((r = run_batch_layers(h, i, i + 1, top, entry))) return r;
            top = lv;
            entry = (uint32_t)i;
            ++i;
            continue;
        }
        int64_t bsz = std::max<int64_t>(h->batch_min, (int64_t)((double)i * h->batch_ratio_pct / 100.0));
        bsz = std::min<int64_t>(bsz, h->batch_max);
        int64_t j = i;
        while (j < n1 && j - i < bsz && h->hlevels[j] <= top) ++j;
        if ((r = run_batch_layers(h, i, j, top, entry))) return r;
        i = j;
    }
    int err = 0;
    HIPCHK(h, hipMemcpyAsync(&err, h->d_err, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    if (while_gpu) while_gpu();  // host work that overlaps the last batches' kernels
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (err & 4) return fail(h, MHNSW_EINTERNAL, "out-of-range node id in adjacency (graph corrupt)");
    return 0;
}

// (re)write the fp16 screening copy of rows [r0, r1) for the current metric
int h16_rows(mhnsw_index* h, int64_t r0, int64_t r1) {
    if (!(h->screen & 1 && h->h16)) return 0;
    if (h->h16_metric != h->metric && r0 > 0) r0 = 0;  // format change: every row
    if (h->screen & 1 && h->h16)
    {
        if (r0 == 0) HIPCHK(h, hipMemsetAsync(h->h16err, 0, sizeof(float), h->stream));  // whole copy rewritten
        LCHK(h, launch_h16_rows(h->vecs, h->norms, r0, r1, h->pitch, h->metric, h->h16, h->h16aux, h->h16err,
                                h->stream));
    }
    h->h16_metric = h->metric;
    return 0;
}

// ---- key identity (compat semantics, GraphDev::kid) -------------------------
// The reference's layer and neighbour maps are keyed by K.  A replaced key
// (BatchAdd, graph.go:1015-1024) or a deleted key added again leaves several
// rows with one key, the old ones reachable through one-directional edges.
// From the first such row on, rows carry kid = the first row that held their
// key (kid[r] = r before), and kidlive[kid] = the key's live row.
const int32_t kNoRow = -1;  // source of kidlive resets (async copies read it later)
int32_t kid_of_row(const mhnsw_index* h, int64_t r) { return h->aliased ? h->hkid[r] : (int32_t)r; }

int set_kidlive(mhnsw_index* h, int32_t kid, int32_t row) {
    HIPCHK(h, hipMemcpyAsync(h->kidlive + kid, &row, 4, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));  // `row` is a stack value
    return 0;
}

int start_alias(mhnsw_index* h) {
    if (h->aliased) return 0;
    const int64_t c = std::max<int64_t>(h->capn, 1);
    int r;
    if ((r = grow(h, h->kid, 0, c, 0xFF)) || (r = grow(h, h->kidlive, 0, c, 0xFF)) || (r = grow(h, h->kprev, 0, c, 0xFF)))
        return r;
    h->hkid.resize((size_t)h->n);
    h->hprev.assign((size_t)h->n, -1);
    std::vector<int32_t> live((size_t)std::max<int64_t>(h->n, 1));
    for (int64_t i = 0; i < h->n; ++i) {
        h->hkid[i] = (int32_t)i;
        live[i] = h->hdead[i] ? -1 : (int32_t)i;
    }
    if (h->n > 0) {
        HIPCHK(h, hipMemcpyAsync(h->kid, h->hkid.data(), (size_t)h->n * 4, hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, hipMemcpyAsync(h->kidlive, live.data(), (size_t)h->n * 4, hipMemcpyHostToDevice, h->stream));
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));
    h->aliased = true;
    return 0;
}

// a row leaves the key map (Delete): remember its kid for a later re-add
void forget_key(mhnsw_index* h, int64_t key, int32_t row) { h->dead_kid[key] = kid_of_row(h, row); }

// every live row of the key, newest first (the key's nodes in disjoint layers: a
// failed insert leaves its node in the layers above the failing one, graph.go:1009,
// and a later insert of the key below them adds another)
std::vector<int32_t> key_rows(const mhnsw_index* h, int64_t key) {
    std::vector<int32_t> out;
    auto it = h->key2id.find(key);
    if (it == h->key2id.end()) return out;
    for (int32_t r = it->second; r >= 0 && (int)out.size() < MH_MAXL; r = h->aliased ? h->hprev[r] : -1)
        if (!h->hdead[r]) out.push_back(r);
    return out;
}
// layers[l].nodes[key]: the key's live row that is a member of layer l, -1 none
int32_t key_row_in(const mhnsw_index* h, int64_t key, int l) {
    for (int32_t r : key_rows(h, key))
        if (in_layer(h, r, l)) return r;
    return -1;
}

// One step of BatchAdd's walk (graph.go:950-1039) over nodes [0, n): *reached =
// the inserts it got to (levels consumed, graph.go:962), the replacing or
// failing one included; *cont > 0 when the walk goes on at node *cont (a key
// whose nodes sat only in upper layers was replaced and Len() grew).
int add_step(mhnsw_index* h, const int64_t* keys, const float* vecs, bool vecs_on_device, int64_t n, int dim,
             const int32_t* levels, int64_t* reached, int64_t* cont_out) {
    *reached = 0;
    *cont_out = -1;
    int r = validate(h);
    if (r) return r;
    if (n <= 0) return 0;
    ++h->mut_epoch;
    if (h->layers_exist && h->dim != dim)  // graph.go:955-960
        return fail(h, MHNSW_EDIM, "embedding dimension mismatch: %d != %d", h->dim, dim);
    if (!h->layers_exist && (r = set_shape(h, dim))) return r;
    const bool flat = h->build_mode == MHNSW_BUILD_FLAT;  // no graph: every row in layer 0, no links
    const bool compat = h->build_mode == MHNSW_BUILD_COMPAT;
    // A present key.  Compat: BatchAdd's replacement (graph.go:1015-1024) -- the
    // walk inserts every node up to the first present key (in the index or
    // earlier in this batch), replaces that one, and stops with "node not
    // added" (graph.go:1035-1037: Len() did not grow).  The batched and flat
    // builds have no reference semantics to follow: they reject it.
    if (!compat) {
        // (host time matters at 1.6 M inserts/s: strictly increasing keys cannot
        // repeat within the batch, and an empty index holds none of them)
        bool increasing = true;
        for (int64_t i = 1; i < n && increasing; ++i) increasing = keys[i] > keys[i - 1];
        std::unordered_set<int64_t> seen;
        if (!increasing) seen.reserve((size_t)n);
        for (int64_t i = 0; i < n; ++i) {
            if ((!h->key2id.empty() && h->key2id.count(keys[i])) || (!increasing && !seen.insert(keys[i]).second))
                return fail(h, MHNSW_EUNSUPPORTED, "duplicate key %lld: replacement needs the compat build mode",
                            (long long)keys[i]);
        }
    }
    if (compat && h->M + 1 > 64) return fail(h, MHNSW_EUNSUPPORTED, "compat build supports M <= 63");
    if (m0_of(h) + 1 > 64 || h->M + 1 > 64) return fail(h, MHNSW_EUNSUPPORTED, "degree caps above 63 unsupported");
    if ((r = ensure_caps(h))) return r;
    for (int64_t i = 0; i < n && levels && !flat; ++i) {
        if (levels[i] < 0) return fail(h, MHNSW_EINVAL, "invalid level: %d", levels[i]);
        if (levels[i] >= MH_MAXL) return fail(h, MHNSW_EUNSUPPORTED, "level %d >= %d", levels[i], MH_MAXL);
    }
    const int64_t n0 = h->n;
    const int64_t live0 = live_count(h);
    const uint64_t rng0 = h->rng;
    const bool le0 = h->layers_exist;
    // key identity: a key present (or repeated), or a deleted key coming back
    if (compat) {
        bool need_alias = false;
        std::unordered_map<int64_t, int> seen;
        for (int64_t i = 0; i < n && !need_alias; ++i)
            need_alias = h->key2id.count(keys[i]) || h->dead_kid.count(keys[i]) || !seen.emplace(keys[i], 1).second;
        if (need_alias && (r = start_alias(h))) return r;
    }
    const int top0 = (int)h->layers.size() - 1;  // len(g.layers) - 1 before this batch
    int top_live = -1;
    uint32_t entry_live = EMPTY_ID;
    if (h->layers_exist && live0 > 0) {
        top_live = top_live_layer(h);
        entry_live = (uint32_t)h->layers[top_live].entry;
    }
    // Host bookkeeping (layer membership, counts, entries, keys) in the walk's
    // order.  floor >= 0: an insert that failed at layer `floor` -- only the
    // layers above it were touched (graph.go:1005-1010 returns there).
    std::vector<int32_t> lv;      // level of each insert the walk reaches
    std::vector<int64_t> rowkey;  // key of every new row
    lv.reserve((size_t)n);
    rowkey.reserve((size_t)n + 2);
    h->hlevels.reserve((size_t)(h->n + n + 2));
    h->key2id.reserve(h->key2id.size() + (size_t)n);
    std::vector<int32_t> kidset;  // kidlive entries to publish: (kid, row) pairs
    std::vector<std::pair<int64_t, int32_t>> snap_layers;
    for (auto& L : h->layers) snap_layers.emplace_back(L.count, L.entry);
    const bool snap_any_dead = h->any_dead;
    std::unordered_map<int64_t, int32_t> snap_dead_kid;  // re-added keys' entries, restored on unwind
    std::unordered_map<int64_t, int32_t> snap_key2id;    // the batch's keys before it (-1 absent)
    for (int64_t i = 0; i < n && compat; ++i) {
        auto it = h->key2id.find(keys[i]);
        snap_key2id.emplace(keys[i], it == h->key2id.end() ? -1 : it->second);
    }
    const size_t hm0 = h->hmask.size(), hd0 = h->hdead.size(), hl0 = h->hlevels.size(), hk0 = h->hkid.size();
    const size_t hp0 = h->hprev.size();
    const size_t nlay0 = h->layers.size();
    // the batched and flat builds publish the new keys in the key map while the
    // device builds (no step of the build reads the map; 1M map inserts are tens
    // of ms of host time)
    const bool defer_keys = !compat && !h->aliased;
    h->hmask.resize(n0 + n + 1, 0u);
    h->hdead.resize(n0 + n + 1, 0);
    int nl = top0 + 1;
    auto book_fresh = [&](int64_t i, int floor) {
        const int32_t id = (int32_t)(n0 + i);
        rowkey.push_back(keys[i]);
        h->hlevels.push_back(lv[i]);
        if (h->aliased) {
            // kid: the key's live node (a node left in upper layers only by a failed
            // insert), else its deleted one, else this row
            auto kp = h->key2id.find(keys[i]);
            auto dk = h->dead_kid.find(keys[i]);
            int32_t kid = id;
            if (kp != h->key2id.end()) {
                kid = kid_of_row(h, kp->second);
            } else if (dk != h->dead_kid.end()) {
                kid = dk->second;
                snap_dead_kid[keys[i]] = dk->second;
                h->dead_kid.erase(dk);
            }
            h->hkid.push_back(kid);
            h->hprev.push_back(-1);
            kidset.push_back(kid);
            kidset.push_back(id);
        } else if (!h->dead_kid.empty()) {
            h->dead_kid.erase(keys[i]);
        }
        nl = std::max(nl, lv[i] + 1);  // graph.go:967-969
        uint32_t mask = 0;
        for (int l = nl - 1; l > floor; --l) {
            Layer& L = h->layers[l];
            // graph.go:990-993: an empty layer takes the node whatever its level
            if (!(l <= lv[i] || (compat && L.count == 0))) continue;
            if (L.count == 0) L.entry = id;
            L.count++;
            mask |= 1u << l;
        }
        h->hmask[id] = mask;
        if (mask) {
            // the key's newest live row; older ones (in higher layers) stay reachable per layer
            if (h->aliased) {
                auto kp = h->key2id.find(keys[i]);
                h->hprev[id] = kp != h->key2id.end() ? kp->second : -1;
            }
            if (!defer_keys) h->key2id[keys[i]] = id;
        } else if (snap_dead_kid.count(keys[i])) {  // failed before touching a layer: still a deleted key
            h->dead_kid[keys[i]] = snap_dead_kid[keys[i]];
        }
    };
    // The walk (graph.go:950-1039): levels drawn insert by insert (graph.go:962,
    // the layer-0 size growing by one per insert; nothing is drawn for inserts
    // never reached).  A present key whose node holds a layer at or below the
    // new level is replaced there and ends the walk; one whose node sits only in
    // higher layers (left by a failed insert) is inserted like a new key.
    int64_t rep = -1, nfresh = 0, cont = -1;
    int rep_i0 = -1;
    int32_t old = -1;               // the key's newest live row
    std::vector<int32_t> old_rows;  // all its live rows (the sweep deletes every one)
    bool rep_in0 = false;           // one of them in layer 0: Len() stays put, "node not added"
    // A host-detected failure after the bookkeeping began (a drawn level past
    // MH_MAXL, a layer, capacity or staging allocation) leaves the index as it
    // was: records, key maps, layers created by this call and the Rng back to
    // their state before it (the reference has no such failure: Go panics on OOM).
    // Nothing has reached the device yet when these can fail.
    auto abort_add = [&](int rc) -> int {
        for (size_t l = nlay0; l < h->layers.size(); ++l) {
            Layer& L = h->layers[l];
            (void)hipFree(L.deg);
            (void)hipFree(L.adj);
            (void)hipFree(L.adjd);
        }
        h->layers.resize(nlay0);
        for (size_t l = 0; l < nlay0; ++l) {
            h->layers[l].count = l < snap_layers.size() ? snap_layers[l].first : 0;
            h->layers[l].entry = l < snap_layers.size() ? snap_layers[l].second : -1;
        }
        h->any_dead = snap_any_dead;
        if (compat) {
            for (auto& kv : snap_key2id) {
                if (kv.second < 0)
                    h->key2id.erase(kv.first);
                else
                    h->key2id[kv.first] = kv.second;
            }
        } else {
            for (int64_t i = 0; i < nfresh; ++i) h->key2id.erase(keys[i]);  // all new (duplicates rejected above)
        }
        for (int32_t r : old_rows)
            if ((size_t)r < hd0) h->hdead[r] = 0;  // live until the sweep
        for (auto& kv : snap_dead_kid) h->dead_kid[kv.first] = kv.second;
        h->hlevels.resize(hl0);
        h->hkid.resize(hk0);
        h->hprev.resize(hp0);
        h->hmask.resize(hm0);
        h->hdead.resize(hd0);
        h->rng = rng0;
        return rc;
    };
    {
        bool le = h->layers_exist;
        for (int64_t i = 0; i < n; ++i) {
            int32_t l_i;
            if (flat) {
                l_i = 0;
            } else if (levels) {
                l_i = levels[i];
                if (l_i < 0) return fail(h, MHNSW_EINVAL, "invalid level: %d", l_i);
            } else {
                l_i = random_level(h->ml, le, live0 + i, &h->rng);
            }
            if (l_i >= MH_MAXL) return abort_add(fail(h, MHNSW_EUNSUPPORTED, "level %d >= %d", l_i, MH_MAXL));
            le = true;
            lv.push_back(l_i);
            if ((r = ensure_layer(h, l_i))) return abort_add(r);
            if (compat) {
                auto it = h->key2id.find(keys[i]);
                if (it != h->key2id.end()) {
                    for (int l = l_i; l >= 0 && rep_i0 < 0; --l)
                        if (key_row_in(h, keys[i], l) >= 0) rep_i0 = l;
                    if (rep_i0 >= 0) {
                        rep = i;
                        old = it->second;
                        old_rows = key_rows(h, keys[i]);
                        rep_in0 = key_row_in(h, keys[i], 0) >= 0;
                        break;
                    }
                }
            }
            book_fresh(i, -1);
            ++nfresh;
        }
    }
    int32_t fresh_entry[MH_MAXL];  // the entries the fresh inserts' walk sees
    for (int l = 0; l < MH_MAXL; ++l)
        fresh_entry[l] = l < (int)h->layers.size() && h->layers[l].count > 0 ? h->layers[l].entry : -1;
    // the replacing insert: old row, the layer i0 of the sweep, the new rows
    int rep_level = -1;
    int32_t ida = -1, idb = -1;
    int32_t rep_entry[MH_MAXL], rep_sweep[MH_MAXL];
    for (int l = 0; l < MH_MAXL; ++l) rep_entry[l] = rep_sweep[l] = -1;
    int64_t nrows = nfresh;
    uint32_t amask = 0;
    auto book_rep = [&](int floor) {
        const int32_t kid = kid_of_row(h, old);
        for (int32_t id : {ida, idb}) {
            if (id < 0) continue;
            rowkey.push_back(keys[rep]);
            h->hlevels.push_back(rep_level);
            h->hkid.push_back(kid);
            h->hprev.push_back(-1);
        }
        // graph.go:980-1032 top-down, as the walk sees the layers
        for (int l = nl - 1; l > floor; --l) {
            Layer& L = h->layers[l];
            const int32_t id = l > rep_i0 && ida >= 0 ? ida : idb;
            if (l == rep_i0) {  // the sweep, after this layer's search
                rep_entry[l] = L.entry;
                // layers[l2].nodes[key] of every layer: one of the key's old rows, or A
                for (int l2 = 0; l2 < (int)h->layers.size(); ++l2) {
                    int32_t x = -1;
                    for (int32_t o : old_rows)
                        if (in_layer(h, o, l2)) x = o;
                    if (x < 0 && ida >= 0 && ((amask >> l2) & 1u)) x = ida;
                    rep_sweep[l2] = x;
                    if (x >= 0) h->layers[l2].count--;
                }
                for (int32_t o : old_rows) h->hdead[o] = 1;
                if (ida >= 0) h->hdead[ida] = 1;
                h->any_dead = true;
                h->key2id[keys[rep]] = idb;
                L.count++;
                h->hmask[idb] |= 1u << l;
                continue;
            }
            const bool empty = L.count == 0;
            if (!(l <= rep_level || (compat && empty))) {
                rep_entry[l] = L.entry;
                continue;
            }
            if (empty) L.entry = id;
            rep_entry[l] = empty ? id : L.entry;
            L.count++;
            h->hmask[id] |= 1u << l;
        }
    };
    if (rep >= 0) {
        rep_level = lv[rep];
        nl = std::max(nl, rep_level + 1);
        for (int l = nl - 1; l > rep_i0; --l)
            if (h->layers[l].count == 0 || l <= rep_level) amask |= 1u << l;
        if (amask) ida = (int32_t)(n0 + nrows++);
        idb = (int32_t)(n0 + nrows++);
        book_rep(-1);
    }
    const int64_t nproc = (int64_t)lv.size();
    // a failed insert (graph.go:1009 "no nodes found in neighborhood search"):
    // back to the snapshot, then the inserts the walk did make, the failing one
    // only above its failing layer; later rows never existed
    auto unwind = [&](int64_t fail_row, int fail_layer) -> int {
        const bool rep_failed = rep >= 0 && (fail_row == ida || fail_row == idb);
        const int64_t i_f = rep_failed ? rep : fail_row - n0;
        *reached = i_f + 1;
        for (size_t l = 0; l < h->layers.size(); ++l) {
            h->layers[l].count = l < snap_layers.size() ? snap_layers[l].first : 0;
            h->layers[l].entry = l < snap_layers.size() ? snap_layers[l].second : -1;
        }
        h->any_dead = snap_any_dead;
        for (auto& kv : snap_key2id) {  // the batch's keys as they were
            if (kv.second < 0)
                h->key2id.erase(kv.first);
            else
                h->key2id[kv.first] = kv.second;
        }
        for (int32_t o : old_rows) h->hdead[o] = 0;  // live until the sweep
        for (auto& kv : snap_dead_kid) h->dead_kid[kv.first] = kv.second;
        for (size_t t = 0; t + 1 < kidset.size() && h->aliased; t += 2)  // unpublish; the replay republishes
            HIPCHK(h, hipMemcpyAsync(h->kidlive + kidset[t], &kNoRow, 4, hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        rowkey.clear();
        kidset.clear();
        snap_dead_kid.clear();
        h->hlevels.resize(n0);
        if (h->aliased) {
            h->hkid.resize(n0);
            h->hprev.resize(n0);
        }
        std::fill(h->hmask.begin() + n0, h->hmask.end(), 0u);
        std::fill(h->hdead.begin() + n0, h->hdead.end(), (uint8_t)0);
        nl = top0 + 1;
        for (int64_t i = 0; i < i_f && i < nfresh; ++i) book_fresh(i, -1);
        int64_t rows = i_f + 1;
        if (!rep_failed) {
            book_fresh(i_f, fail_layer);
        } else {
            nl = std::max(nl, rep_level + 1);
            book_rep(fail_layer);
            rows = nfresh + (ida >= 0 ? 2 : 1);
            if (fail_layer >= rep_i0) {  // failed before the sweep: the old nodes stay ...
                h->key2id[keys[rep]] = old;
                for (int32_t o : old_rows) h->hdead[o] = 0;
                if (ida >= 0) h->hdead[ida] = 0;
                h->any_dead = snap_any_dead;
                // ... and the new node, in the layers above the failing one, is the key's node there
                const int32_t placed = ida >= 0 && h->hmask[ida] ? ida : h->hmask[idb] ? idb : -1;
                if (placed >= 0) {
                    h->hprev[placed] = old;
                    h->key2id[keys[rep]] = placed;
                }
            }
        }
        std::vector<int32_t> live;  // (kid, row): the batch's keys' live rows after the replay
        for (auto& kv : snap_key2id) {
            auto it = h->key2id.find(kv.first);
            if (it == h->key2id.end()) continue;
            live.push_back(kid_of_row(h, it->second));
            live.push_back(it->second);
        }
        for (size_t t = 0; t + 1 < live.size() && h->aliased; t += 2)
            HIPCHK(h, hipMemcpyAsync(h->kidlive + live[t], &live[t + 1], 4, hipMemcpyHostToDevice, h->stream));
        if (h->aliased)
            HIPCHK(h, hipMemcpyAsync(h->kprev + n0, h->hprev.data() + n0, (size_t)rows * 4, hipMemcpyHostToDevice,
                                     h->stream));
        HIPCHK(h, hipMemcpyAsync(h->dead, h->hdead.data(), (size_t)(n0 + rows), hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        h->n = n0 + rows;
        h->hmask.resize(h->n);
        h->hdead.resize(h->n);
        if (!levels && !flat) {  // the draws of the inserts the walk never reached are not made
            h->rng = rng0;
            bool le2 = le0;
            for (int64_t i = 0; i <= i_f; ++i) {
                (void)random_level(h->ml, le2, live0 + i, &h->rng);
                le2 = true;
            }
        }
        fix_entries(h);
        h->partial_rows = 0;
        for (int64_t i = 0; i < h->n; ++i) h->partial_rows += !h->hdead[i] && !in_layer(h, i, 0);
        return 0;
    };
    const int64_t n1 = n0 + nrows;
    if ((r = ensure_capacity(h, n1))) return abort_add(r);
    if (!vecs_on_device && (r = ensure_buf(h, h->tmp, (size_t)nproc * dim))) return abort_add(r);
    h->hmask.resize(n1);
    h->hdead.resize(n1);
    // upload keys, levels, vectors (padded), norms
    HIPCHK(h, hipMemcpyAsync(h->keys + n0, rowkey.data(), nrows * sizeof(int64_t), hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipMemcpyAsync(h->levels + n0, h->hlevels.data() + n0, nrows * sizeof(int32_t), hipMemcpyHostToDevice,
                             h->stream));
    if (h->aliased) {
        HIPCHK(h, hipMemcpyAsync(h->kid + n0, h->hkid.data() + n0, nrows * sizeof(int32_t), hipMemcpyHostToDevice,
                                 h->stream));
        HIPCHK(h, hipMemcpyAsync(h->kprev + n0, h->hprev.data() + n0, nrows * sizeof(int32_t), hipMemcpyHostToDevice,
                                 h->stream));
        for (size_t t = 0; t + 1 < kidset.size(); t += 2)
            HIPCHK(h, hipMemcpyAsync(h->kidlive + kidset[t], &kidset[t + 1], 4, hipMemcpyHostToDevice, h->stream));
    }
    const float* src = vecs;
    if (!vecs_on_device) {
        HIPCHK(h, hipMemcpyAsync(h->tmp.p, vecs, (size_t)nproc * dim * 4, hipMemcpyHostToDevice, h->stream));
        src = h->tmp.p;
    }
    if (nfresh > 0) LCHK(h, launch_pad_rows(src, nfresh, dim, h->vecs + (size_t)n0 * h->pitch, h->pitch, h->stream));
    for (int32_t id : {ida, idb})  // the replacing node's rows hold its vector
        if (rep >= 0 && id >= 0)
            LCHK(h, launch_pad_rows(src + (size_t)rep * dim, 1, dim, h->vecs + (size_t)id * h->pitch, h->pitch,
                                    h->stream));
    LCHK(h, launch_norms(h->vecs, n0, n1, h->pitch, h->lpr, h->vpl, h->norms, h->stream));
    if ((r = h16_rows(h, n0, n1))) return r;
    h->layers_exist = true;
    h->n = n1;
    bool published = !defer_keys;
    auto publish_keys = [&]() {
        if (published) return;
        for (int64_t i = 0; i < nfresh; ++i) h->key2id[keys[i]] = (int32_t)(n0 + i);
        published = true;
    };
    if (flat) {  // members of layer 0 without links (an empty neighbour map, not an absent node)
        r = hipMemsetD32Async((hipDeviceptr_t)(h->layers[0].deg + n0), 0, (size_t)n, h->stream) == hipSuccess
                ? 0
                : fail(h, MHNSW_EDEVICE, "device memset failed");
        publish_keys();
    } else if (compat) {
        CompatRep cr;
        if (rep >= 0) cr = CompatRep{rep_level, rep_i0, ida >= 0 ? ida : idb, idb, rep_entry, rep_sweep};
        int64_t fail_row = -1;
        int fail_layer = -1;
        r = run_build_compat(h, n0, n0 + nfresh, top0, fresh_entry, cr, &fail_row, &fail_layer);
        if (r == 0 && fail_row >= 0) {
            if ((r = unwind(fail_row, fail_layer)) == 0)
                r = fail(h, MHNSW_EINTERNAL, "no nodes found in neighborhood search");
        } else if (r == 0 && rep >= 0) {
            HIPCHK(h, hipMemcpyAsync(h->dead, h->hdead.data(), (size_t)h->n, hipMemcpyHostToDevice, h->stream));
            fix_entries(h);
            // graph.go:1035-1037: a replacement of a key that layer 0 held leaves Len()
            // unchanged -- "node not added" ends the walk; one whose nodes sat only in
            // upper layers (left by a failed insert) grows it, and the walk goes on
            *reached = nproc;  // up to the replacing insert
            if (rep_in0)
                r = fail(h, MHNSW_EINTERNAL, "node not added");
            else
                cont = rep + 1;
        }
    } else {
        r = run_build_batch(h, n0, n1, top_live, entry_live, publish_keys);
        publish_keys();  // (an early device error: the rows exist, so do their keys)
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));
    for (size_t i = 0; i + 1 < h->tev_used; i += 2) {
        float ms = 0.f;
        HIPCHK(h, hipEventElapsedTime(&ms, h->tev[i], h->tev[i + 1]));
        h->build_search_us += ms * 1e3;
    }
    h->tev_used = 0;
    if (r == 0) *reached = nproc;
    *cont_out = cont;
    return r;
}

int add_impl(mhnsw_index* h, const int64_t* keys, const float* vecs, bool vecs_on_device, int64_t n, int dim,
             const int32_t* levels) {
    h->add_reached = 0;
    for (;;) {
        int64_t reached = 0, cont = -1;
        const int r = add_step(h, keys, vecs, vecs_on_device, n, dim, levels, &reached, &cont);
        h->add_reached += reached;
        if (r || cont <= 0 || cont >= n) return r;
        // the rest of the walk (graph.go:950: the next node)
        keys += cont;
        vecs += (size_t)cont * dim;
        n -= cont;
        if (levels) levels += cont;
    }
}

}  // namespace mhh

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int mhnsw_create(int metric, int M, double ml, int ef_search, uint64_t seed, mhnsw_index** out) {
    if (!out) return MHNSW_EINVAL;
    *out = nullptr;
    mhnsw_index* h = new (std::nothrow) mhnsw_index();
    if (!h) return fail(nullptr, MHNSW_ENOMEM, "out of memory");
    h->metric = metric;
    h->M = M;
    h->ml = ml;
    h->ef = ef_search;
    h->rng = seed;
    int r = validate(h);  // NewGraphWithConfig (graph.go:352-366)
    if (r) {
        g_create_err = h->err;
        delete h;
        return r;
    }
    if (hipGetDevice(&h->device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return fail(nullptr, MHNSW_EDEVICE, "no HIP device available");
    }
    if (hipMalloc(&h->d_stats, 16 * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&h->d_err, 4 * sizeof(int)) != hipSuccess || hipMemset(h->d_err, 0, 4 * sizeof(int)) != hipSuccess ||
        hipMalloc(&h->h16err, sizeof(float)) != hipSuccess || hipMemset(h->h16err, 0, sizeof(float)) != hipSuccess || hipMalloc(&h->touched_cnt, 16) != hipSuccess ||
        hipMalloc(&h->d_layer_entry, 3 * MH_MAXL * 4) != hipSuccess ||
        hipMalloc(&h->d_layers, MH_MAXL * sizeof(LayerDev)) != hipSuccess || hipEventCreate(&h->ev0) != hipSuccess ||
        hipEventCreate(&h->ev1) != hipSuccess || hipEventCreate(&h->gev0) != hipSuccess ||
        hipEventCreate(&h->gev1) != hipSuccess || hipEventCreateWithFlags(&h->scr_ev, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->meta_ev, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->ord_ev, hipEventDisableTiming) != hipSuccess || hipMemset(h->d_stats, 0, 16 * sizeof(unsigned long long)) != hipSuccess) {
        mhnsw_destroy(h);
        return fail(nullptr, MHNSW_EDEVICE, "device initialisation failed");
    }
    *out = h;
    return MHNSW_OK;
}

void mhnsw_destroy(mhnsw_index* h) {
    if (!h) return;
    if (h->scr_valid) (void)hipEventSynchronize(h->scr_ev);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    auto F = [](void* p) {
        if (p) (void)hipFree(p);
    };
    F(h->vecs);
    F(h->norms);
    F(h->h16);
    F(h->h16aux);
    F(h->keys);
    F(h->levels);
    F(h->dead);
    F(h->kid);
    F(h->kidlive);
    F(h->kprev);
    F(h->cur_entry);
    F(h->inc_cnt);
    F(h->inc_src);
    F(h->inc_dist);
    F(h->touched);
    F(h->touched_cnt);
    F(h->d_layer_entry);
    F(h->d_layers);
    F(h->d_stats);
    F(h->d_err);
    F(h->h16err);
    for (auto& L : h->layers) {
        F(L.deg);
        F(L.adj);
        F(L.adjd);
    }
    F(h->qpad.p);
    F(h->qnorm.p);
    F(h->scores.p);
    F(h->tmp.p);
    F(h->cand.p);
    F(h->border.p);
    F(h->okeys.p);
    F(h->odist.p);
    F(h->on.p);
    F(h->nq.p);
    F(h->nneg.p);
    F(h->ncd.p);
    F(h->nck.p);
    F(h->nok.p);
    F(h->ncn.p);
    F(h->nci.p);
    F(h->noff.p);
    F(h->non.p);
    F(h->nos.p);
    F(h->xsplit.p);
    F(h->xinv.p);
    F(h->qinv.p);
    F(h->xerr.p);
    F(h->h1thr.p);
    F(h->h1c.p);
    F(h->h1s.p);
    F(h->h1xw.p);
    F(h->qerr.p);
    F(h->h1region.p);
    F(h->h1bucket.p);
    F(h->h1rcnt.p);
    F(h->h1qcnt.p);
    F(h->h1ovf.p);
    F(h->qsplit.p);
    F(h->xbound.p);
    F(h->xsegd.p);
    F(h->xsegi.p);
    F(h->xmaxn.p);
    F(h->xflag.p);
    F(h->xgone.p);
    F(h->xflagged.p);
    F(h->xnflag.p);
    if (h->scr_ev) (void)hipEventDestroy(h->scr_ev);
    if (h->meta_ev) (void)hipEventDestroy(h->meta_ev);
    if (h->ord_ev) (void)hipEventDestroy(h->ord_ev);
    if (h->ord_pin) (void)hipHostFree(h->ord_pin);
    for (auto e : h->tev) (void)hipEventDestroy(e);
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    if (h->gev0) (void)hipEventDestroy(h->gev0);
    if (h->gev1) (void)hipEventDestroy(h->gev1);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

const char* mhnsw_last_error(const mhnsw_index* h) { return h ? h->err.c_str() : g_create_err.c_str(); }

int mhnsw_set_params(mhnsw_index* h, int metric, int M, double ml, int ef_search) {
    std::unique_lock<std::shared_mutex> lk(h->mu);
    if (metric != h->metric && h->screen && h->n > 0) {  // the screening copy's format follows the metric
        int r = drain(h);
        if (r) return r;
        h->metric = metric;
        if ((r = h16_rows(h, 0, h->n))) return r;
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    h->metric = metric;
    h->M = M;
    h->ml = ml;
    h->ef = ef_search;
    return MHNSW_OK;
}

int mhnsw_get_params(const mhnsw_index* h, int* metric, int* M, double* ml, int* ef_search) {
    std::shared_lock<std::shared_mutex> lk(h->mu);
    if (metric) *metric = h->metric;
    if (M) *M = h->M;
    if (ml) *ml = h->ml;
    if (ef_search) *ef_search = h->ef;
    return MHNSW_OK;
}

int mhnsw_seed(mhnsw_index* h, uint64_t seed) {
    std::unique_lock<std::shared_mutex> lk(h->mu);
    h->rng = seed;
    return MHNSW_OK;
}

int mhnsw_set_option(mhnsw_index* h, const char* name, int64_t v) {
    std::unique_lock<std::shared_mutex> lk(h->mu);
    std::string n(name ? name : "");
    if (n == "build_mode") {
        if (v != MHNSW_BUILD_COMPAT && v != MHNSW_BUILD_BATCH && v != MHNSW_BUILD_FLAT)
            return fail(h, MHNSW_EINVAL, "bad build_mode");
        if (h->n > 0 && v != h->build_mode) return fail(h, MHNSW_EINVAL, "build_mode must be set before the first Add");
        h->build_mode = (int)v;
    } else if (n == "m0") {
        if (h->n > 0) return fail(h, MHNSW_EINVAL, "m0 must be set before the first Add");
        h->m0 = (int)v;
    } else if (n == "ef_construction") {
        h->efc = (int)v;
    } else if (n == "heuristic") {
        if (v < 0 || v > 2) return fail(h, MHNSW_EINVAL, "heuristic must be 0, 1 or 2");
        h->heuristic = (int)v;
    } else if (n == "keep_pruned") {
        h->keep_pruned = (int)(v != 0);
    } else if (n == "build_expand") {
        if (v < 1 || v > 4) return fail(h, MHNSW_EINVAL, "build_expand must be in [1, 4]");
        h->build_expand = (int)v;
    } else if (n == "upper_efc") {
        if (v < 0 || v > 512) return fail(h, MHNSW_EINVAL, "upper_efc must be in [0, 512]");
        h->upper_efc = (int)v;
    } else if (n == "search_expand") {
        if (v != 1 && v != 2 && v != 4) return fail(h, MHNSW_EINVAL, "search_expand must be 1, 2 or 4");
        h->search_expand = (int)v;
    } else if (n == "prune_alpha_pct") {
        if (v < 50 || v > 400) return fail(h, MHNSW_EINVAL, "prune_alpha_pct must be in [50, 400]");
        h->alpha_pct = (int)v;
    } else if (n == "batch_min") {
        h->batch_min = (int)std::max<int64_t>(1, v);
    } else if (n == "batch_max") {
        h->batch_max = (int)std::max<int64_t>(1, v);
    } else if (n == "batch_ratio_pct") {
        h->batch_ratio_pct = (int)std::max<int64_t>(0, v);
    } else if (n == "vis_entries") {
        if (v != 0 && (v < 64 || v > 32768)) return fail(h, MHNSW_EINVAL, "vis_entries must be 0 or in [64, 32768]");
        h->vis_entries = (int)v;
    } else if (n == "vis_log2") {
        if (v < 6 || v > 15) return fail(h, MHNSW_EINVAL, "vis_log2 must be in [6, 15]");
        h->vis_log2 = (int)v;
    } else if (n == "exact_thr_rank") {
        if (v < 0 || v > 256) return fail(h, MHNSW_EINVAL, "exact_thr_rank must be in [0, 256]");
        h->exact_thr_rank = (int)v;
    } else if (n == "exact_sample") {
        if (v < 1 || v > 1 << 20) return fail(h, MHNSW_EINVAL, "exact_sample must be in [1, 2^20]");
        h->exact_sample = (int)v;
    } else if (n == "exact_kk") {
        h->exact_kk = (int)v;
    } else if (n == "exact_tile") {
        // precisions 1 / 2: 0-3 (the split GEMM's tiles); precision 3: 0, 5 or 34 (the
        // tools build, MH_EXACT_DIAG, also 30 / 31 / 32 / 36: timing diagnostics, 33: the
        // ring three slices deep)
        bool ok = (v >= 0 && v <= 3) || v == 5 || v == 34;
#ifdef MH_EXACT_DIAG
        ok = ok || v == 30 || v == 31 || v == 32 || v == 33 || v == 36 || (v >= 37 && v <= 41);
#endif
        if (!ok) return fail(h, MHNSW_EINVAL, "exact_tile must be 0-3, 5 or 34");
        h->exact_tile = (int)v;
    } else if (n == "build_mw_max") {
        if (v < 0) return fail(h, MHNSW_EINVAL, "build_mw_max must be >= 0");
        h->build_mw_max = v;
    } else if (n == "beam_mw_max_b") {
        if (v < 0) return fail(h, MHNSW_EINVAL, "beam_mw_max_b must be >= 0");
        h->beam_mw_max_b = v;
    } else if (n == "upper_ef") {
        if (v < 1 || v > 64) return fail(h, MHNSW_EINVAL, "upper_ef must be in [1, 64]");
        h->upper_ef = (int)v;
    } else if (n == "fuse_descent") {
        if (v != 0 && v != 1) return fail(h, MHNSW_EINVAL, "fuse_descent must be 0 or 1");
        h->fuse_descent = (int)v;
    } else if (n == "vis_compact") {
        if (v != 0 && v != 1) return fail(h, MHNSW_EINVAL, "vis_compact must be 0 or 1");
        h->vis_compact = (int)v;
    } else if (n == "time_build") {
        h->time_build = (int)(v != 0);
    } else if (n == "max_rows") {
        if (v < 0) return fail(h, MHNSW_EINVAL, "max_rows must be >= 0");
        h->max_rows = v;
    } else if (n == "screen") {
        if (v < 0 || v > 1) return fail(h, MHNSW_EINVAL, "screen must be 0 or 1");
        if ((int)v == h->screen) return MHNSW_OK;
        int r = drain(h);
        if (r) return r;
        HIPCHK(h, hipStreamSynchronize(h->stream));
        auto F = [](auto*& p) {
            if (p) (void)hipFree(p);
            p = nullptr;
        };
        F(h->h16);
        F(h->h16aux);
        h->h16_metric = -1;
        h->screen = (int)v;
        if (v && h->capn > 0) {  // rewrite the copy
            if ((r = grow(h, h->h16, 0, h->capn * h->pitch, 0)) || (r = grow(h, h->h16aux, 0, h->capn, 0xFF)))
                return r;
            if ((r = h16_rows(h, 0, h->n))) return r;
            HIPCHK(h, hipStreamSynchronize(h->stream));
        }
    } else if (n == "compat_waves") {
        if (v != 1 && v != 8) return fail(h, MHNSW_EINVAL, "compat_waves must be 1 or 8");
        h->compat_waves = (int)v;
    } else if (n == "exact_precision") {
        if (v < 0 || v > 3)
            return fail(h, MHNSW_EINVAL,
                        "exact_precision must be 0 (f32), 1 (bf16x3), 2 (fp16 2-product) or 3 (fp16 1-product, fused)");
        h->exact_precision = (int)v;
    } else {
        return fail(h, MHNSW_EINVAL, "unknown option '%s'", n.c_str());
    }
    return MHNSW_OK;
}

int mhnsw_get_option(const mhnsw_index* h, const char* name, int64_t* v) {
    std::shared_lock<std::shared_mutex> lk(h->mu);
    std::string n(name ? name : "");
    if (n == "build_mode") *v = h->build_mode;
    else if (n == "m0") *v = m0_of(h);
    else if (n == "ef_construction") *v = h->efc > 0 ? h->efc : h->ef;
    else if (n == "heuristic") *v = h->heuristic;
    else if (n == "keep_pruned") *v = h->keep_pruned;
    else if (n == "build_expand") *v = h->build_expand;
    else if (n == "search_expand") *v = h->search_expand;
    else if (n == "upper_efc") *v = h->upper_efc;
    else if (n == "prune_alpha_pct") *v = h->alpha_pct;
    else if (n == "batch_min") *v = h->batch_min;
    else if (n == "batch_max") *v = h->batch_max;
    else if (n == "batch_ratio_pct") *v = h->batch_ratio_pct;
    else if (n == "vis_log2") *v = h->vis_log2;
    else if (n == "vis_entries") *v = beam_vis_entries(h);
    else if (n == "exact_kk") *v = h->exact_kk;
    else if (n == "exact_sample") *v = h->exact_sample;
    else if (n == "exact_thr_rank") *v = h->exact_thr_rank;
    else if (n == "exact_precision") *v = h->exact_precision;
    else if (n == "exact_tile") *v = h->exact_tile;
    else if (n == "compat_waves") *v = h->compat_waves;
    else if (n == "upper_ef") *v = h->upper_ef;
    else if (n == "beam_mw_max_b") *v = h->beam_mw_max_b;
    else if (n == "build_mw_max") *v = h->build_mw_max;
    else if (n == "screen") *v = h->screen;
    else if (n == "fuse_descent") *v = h->fuse_descent;
    else if (n == "vis_compact") *v = h->vis_compact;
    else if (n == "time_build") *v = h->time_build;
    else if (n == "max_rows") *v = h->max_rows;
    else if (n == "strkey_relabels") *v = h->relabels;
    else if (n == "strkeys") *v = (int64_t)h->s2l.size();
    else if (n == "pitch") *v = h->pitch;
    else if (n == "capacity") *v = h->capn;
    else if (n == "last_gemm_ns") {  // read-only: the last timed exact search's fused score GEMM (HIP events)
        float ms = 0.f;
        if (!h->have_gemm_timing || hipEventSynchronize(h->gev1) != hipSuccess ||
            hipEventElapsedTime(&ms, h->gev0, h->gev1) != hipSuccess)
            return MHNSW_EINVAL;
        *v = (int64_t)std::llround((double)ms * 1e6);
    }
    else if (n == "screen_err_ppb") {  // read-only: the fp16 copy's measured margin E, parts per 1e9
        float e = 0.f;
        if (h->h16err && (hipMemcpyAsync(&e, h->h16err, sizeof(float), hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
                          hipStreamSynchronize(h->stream) != hipSuccess))
            return MHNSW_EDEVICE;
        *v = (int64_t)std::llround((double)e * 1e9);
    }
    else return MHNSW_EINVAL;
    return MHNSW_OK;
}

int mhnsw_validate(mhnsw_index* h) {
    std::shared_lock<std::shared_mutex> lk(h->mu);
    return validate(h);
}

int mhnsw_reserve(mhnsw_index* h, int64_t n, int dim) {
    std::unique_lock<std::shared_mutex> lk(h->mu);
    int r = drain(h);
    if (r) return r;
    if (!h->layers_exist) {
        if ((r = set_shape(h, dim))) return r;
    } else if (dim != h->dim) {
        return fail(h, MHNSW_EDIM, "embedding dimension mismatch: %d != %d", h->dim, dim);
    }
    if ((r = ensure_capacity(h, n))) return r;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int mhnsw_add(mhnsw_index* h, const int64_t* keys, const float* vecs, int64_t n, int dim, const int32_t* levels) {
    std::unique_lock<std::shared_mutex> lk(h->mu);
    h->add_reached = 0;  // (an Add failing before its walk reached no insert)
    int r = drain(h);
    if (r) return r;
    return add_impl(h, keys, vecs, false, n, dim, levels);
}

int mhnsw_add_device(mhnsw_index* h, const int64_t* keys, const float* d_vecs, int64_t n, int dim,
                     const int32_t* levels) {
    std::unique_lock<std::shared_mutex> lk(h->mu);
    h->add_reached = 0;  // (an Add failing before its walk reached no insert)
    HIPCHK(h, hipDeviceSynchronize());  // order after whatever produced d_vecs (and any enqueued search)
    h->scr_valid = false;
    return add_impl(h, keys, d_vecs, true, n, dim, levels);
}

int mhnsw_search(mhnsw_index* h, const float* queries, int64_t B, int dim, int k, int mode, int ef,
                 const int64_t* entry_key, int64_t* out_keys, float* out_dist, int32_t* out_n) {
    // scratch buffers are per handle: serialise host-pointer searches
    std::unique_lock<std::shared_mutex> lk(h->mu);
    return search_impl(h, queries, false, B, dim, k, mode, ef, entry_key, out_keys, out_dist, out_n, h->stream, true);
}

int mhnsw_search_device(mhnsw_index* h, const float* d_queries, int64_t B, int dim, int k, int mode, int ef,
                        int64_t* d_keys, float* d_dist, int32_t* d_n, void* stream) {
    std::unique_lock<std::shared_mutex> lk(h->mu);
    // NULL is the HIP null stream (torch's default stream handle is 0)
    return search_impl(h, d_queries, true, B, dim, k, mode, ef, nullptr, d_keys, d_dist, d_n, (hipStream_t)stream,
                       true, nullptr, true);
}

int mhnsw_device_status(mhnsw_index* h) {
    std::unique_lock<std::shared_mutex> lk(h->mu);
    if (h->scr_valid) HIPCHK(h, hipEventSynchronize(h->scr_ev));
    int err = 0;
    HIPCHK(h, hipMemcpy(&err, h->d_err + 1, sizeof(int), hipMemcpyDeviceToHost));
    if (!err) return MHNSW_OK;
    HIPCHK(h, hipMemset(h->d_err + 1, 0, sizeof(int)));
    if (err & 4) return fail(h, MHNSW_EINTERNAL, "out-of-range node id in adjacency (graph corrupt)");
    return fail(h, MHNSW_EINTERNAL, "visited set overflow (raise vis_log2)");
}

// read-locked like the reference's Len/Dims (graph.go:421,829): a concurrent Add may grow h->layers
int64_t mhnsw_len(const mhnsw_index* h) {
    std::shared_lock<std::shared_mutex> lk(h->mu);
    return h->layers.empty() ? 0 : h->layers[0].count;
}
int mhnsw_dims(const mhnsw_index* h) {
    std::shared_lock<std::shared_mutex> lk(h->mu);
    return h->layers_exist ? h->dim : 0;
}
int mhnsw_num_layers(const mhnsw_index* h) {
    std::shared_lock<std::shared_mutex> lk(h->mu);
    return (int)h->layers.size();
}
int64_t mhnsw_layer_count(const mhnsw_index* h, int l) {
    std::shared_lock<std::shared_mutex> lk(h->mu);
    return l >= 0 && l < (int)h->layers.size() ? h->layers[l].count : 0;
}

int mhnsw_contains(const mhnsw_index* h, const int64_t* keys, int64_t n, uint8_t* out) {
    std::shared_lock<std::shared_mutex> lk(h->mu);
    if (n > 0 && (!keys || !out)) return MHNSW_EINVAL;
    for (int64_t i = 0; i < n; ++i) out[i] = h->key2id.count(keys[i]) ? 1 : 0;
    return MHNSW_OK;
}

int mhnsw_add_plan(mhnsw_index* h, const int64_t* keys, int64_t n, int64_t* nwalk, int* one_by_one) {
    std::shared_lock<std::shared_mutex> lk(h->mu);
    if (n > 0 && !keys) return fail(h, MHNSW_EINVAL, "keys must be non-NULL");
    int64_t w = n;
    if (h->build_mode == MHNSW_BUILD_COMPAT) {
        std::unordered_map<int64_t, int> seen;
        for (int64_t i = 0; i < n; ++i) {
            if (h->key2id.count(keys[i]) || seen.count(keys[i])) {
                w = i + 1;
                break;
            }
            seen[keys[i]] = 1;
        }
    }
    if (nwalk) *nwalk = w;
    if (one_by_one) *one_by_one = h->build_mode == MHNSW_BUILD_COMPAT && h->any_dead ? 1 : 0;
    return MHNSW_OK;
}

int mhnsw_add_reached(const mhnsw_index* h, int64_t* reached) {
    std::shared_lock<std::shared_mutex> lk(h->mu);
    if (!reached) return fail(nullptr, MHNSW_EINVAL, "reached must be non-NULL");
    *reached = h->add_reached;
    return MHNSW_OK;
}

int mhnsw_lookup(mhnsw_index* h, int64_t key, float* out) {
    std::shared_lock<std::shared_mutex> lk(h->mu);
    const int32_t r0 = key_row_in(h, key, 0);  // graph.go:906 layers[0].nodes[key]
    if (r0 < 0) return 0;
    HIPCHK(h, hipMemcpy(out, h->vecs + (size_t)r0 * h->pitch, (size_t)h->dim * 4, hipMemcpyDeviceToHost));
    return 1;
}

int mhnsw_distance_device(int metric, const float* d_q, const float* d_X, int64_t n, int dim, float* d_out,
                          void* stream) {
    if (metric != COSINE && metric != EUCLIDEAN) return fail(nullptr, MHNSW_EINVAL, "Distance function must be set");
    if (dim <= 0) return fail(nullptr, MHNSW_EINVAL, "dimension must be positive");
    if (n <= 0) return 0;
    if (launch_sweep_raw(d_q, d_X, n, dim, metric, d_out, (hipStream_t)stream))
        return fail(nullptr, MHNSW_EDEVICE, "sweep launch failed");
    return 0;
}

int mhnsw_distance(int metric, const float* q, const float* X, int64_t n, int dim, float* out) {
    if (n <= 0) return 0;
    float *dq = nullptr, *dx = nullptr, *dout = nullptr;
    if (hipMalloc(&dq, (size_t)dim * 4) != hipSuccess || hipMalloc(&dx, (size_t)n * dim * 4) != hipSuccess ||
        hipMalloc(&dout, (size_t)n * 4) != hipSuccess)
        return fail(nullptr, MHNSW_ENOMEM, "device allocation failed");
    int r = 0;
    if (hipMemcpy(dq, q, (size_t)dim * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dx, X, (size_t)n * dim * 4, hipMemcpyHostToDevice) != hipSuccess)
        r = fail(nullptr, MHNSW_EDEVICE, "copy failed");
    if (!r) r = mhnsw_distance_device(metric, dq, dx, n, dim, dout, nullptr);
    if (!r && (hipDeviceSynchronize() != hipSuccess ||
               hipMemcpy(out, dout, (size_t)n * 4, hipMemcpyDeviceToHost) != hipSuccess))
        r = fail(nullptr, MHNSW_EDEVICE, "sweep failed");
    (void)hipFree(dq);
    (void)hipFree(dx);
    (void)hipFree(dout);
    return r;
}

int mhnsw_export_sizes(mhnsw_index* h, int64_t* N, int* dim, int* L, int* cap) {
    std::shared_lock<std::shared_mutex> lk(h->mu);
    *N = h->n;
    *dim = h->dim;
    *L = (int)h->layers.size();
    int c = 0;
    for (auto& Ly : h->layers) c = std::max(c, Ly.cap);
    *cap = c;
    return 0;
}

int mhnsw_export(mhnsw_index* h, int64_t* keys, float* vecs, int32_t* deg, int32_t* adj, int cap, int32_t* entry,
                 uint8_t* dead) {
    std::shared_lock<std::shared_mutex> lk(h->mu);
    const int64_t N = h->n;
    if (N == 0) return 0;
    if (dead) memcpy(dead, h->hdead.data(), (size_t)N);
    HIPCHK(h, hipMemcpy(keys, h->keys, N * 8, hipMemcpyDeviceToHost));
    HIPCHK(h, hipMemcpy2D(vecs, (size_t)h->dim * 4, h->vecs, (size_t)h->pitch * 4, (size_t)h->dim * 4, N,
                          hipMemcpyDeviceToHost));
    std::vector<int32_t> row;
    for (int l = 0; l < (int)h->layers.size(); ++l) {
        const Layer& L = h->layers[l];
        entry[l] = L.count > 0 ? L.entry : -1;
        HIPCHK(h, hipMemcpy(deg + (size_t)l * N, L.deg, N * 4, hipMemcpyDeviceToHost));
        row.resize((size_t)N * L.cap);
        HIPCHK(h, hipMemcpy(row.data(), L.adj, (size_t)N * L.cap * 4, hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < N; ++i) {
            const int d = deg[(size_t)l * N + i];
            if (d > cap) return fail(h, MHNSW_EINVAL, "export cap %d smaller than degree %d", cap, d);
            int32_t* o = adj + ((size_t)l * N + i) * cap;
            for (int j = 0; j < cap; ++j) o[j] = (j < d) ? row[(size_t)i * L.cap + j] : -1;
        }
    }
    return 0;
}

}  // extern "C"

extern "C" {

// graph.go:843-895 Delete / BatchDelete
// ExactIndex replace-on-Add (hybrid/exact.go:28-59) on a FLAT handle: rows of
// present keys are overwritten in place, so repeated Adds of one key neither
// grow the store nor leave dead rows for the exact path to scan.
int mhnsw_replace(mhnsw_index* h, const int64_t* keys, const float* vecs, int64_t n, int dim, uint8_t* out) {
    std::unique_lock<std::shared_mutex> lk(h->mu);
    if (int r0 = drain(h)) return r0;
    if (n > 0 && (!keys || !vecs || !out)) return fail(h, MHNSW_EINVAL, "keys, vecs and out must be non-NULL");
    if (h->build_mode != MHNSW_BUILD_FLAT) return fail(h, MHNSW_EUNSUPPORTED, "replace needs a flat (build_mode 2) handle");
    for (int64_t i = 0; i < n; ++i) out[i] = 0;
    if (n <= 0 || !h->layers_exist) return 0;
    if (dim != h->dim) return fail(h, MHNSW_EDIM, "embedding dimension mismatch: %d != %d", h->dim, dim);
    std::vector<int32_t> ids;
    std::vector<int64_t> src;
    {
        std::unordered_map<int64_t, int> seen;
        for (int64_t i = 0; i < n; ++i) {
            if (seen.count(keys[i])) return fail(h, MHNSW_EINVAL, "duplicate key %lld in replace", (long long)keys[i]);
            seen[keys[i]] = 1;
        }
    }
    for (int64_t i = 0; i < n; ++i) {
        auto it = h->key2id.find(keys[i]);
        if (it == h->key2id.end()) continue;
        out[i] = 1;
        ids.push_back(it->second);
        src.push_back(i);
    }
    if (ids.empty()) return 0;
    const int64_t m = (int64_t)ids.size();
    int r;
    // the present keys' vectors, compacted on the host, padded on the device
    std::vector<float> hv((size_t)m * dim);
    for (int64_t j = 0; j < m; ++j) std::memcpy(&hv[(size_t)j * dim], vecs + (size_t)src[j] * dim, (size_t)dim * 4);
    if ((r = ensure_buf(h, h->tmp, (size_t)m * dim + (size_t)m * h->pitch + (size_t)m))) return r;
    float* staged = h->tmp.p;
    float* padded = h->tmp.p + (size_t)m * dim;
    int32_t* dids = reinterpret_cast<int32_t*>(padded + (size_t)m * h->pitch);
    HIPCHK(h, hipMemcpyAsync(staged, hv.data(), hv.size() * 4, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipMemcpyAsync(dids, ids.data(), (size_t)m * 4, hipMemcpyHostToDevice, h->stream));
    LCHK(h, launch_pad_rows(staged, m, dim, padded, h->pitch, h->stream));
    LCHK(h, launch_scatter_rows(padded, dids, m, h->pitch, h->vecs, h->stream));
    // norms, the screening copy and the exact path's planes of the touched range
    // (rows in between are recomputed to the same values; the copies' measured
    // error maxima only grow, so their margins stay valid)
    const int64_t lo = *std::min_element(ids.begin(), ids.end()), hi = *std::max_element(ids.begin(), ids.end()) + 1;
    LCHK(h, launch_norms(h->vecs, lo, hi, h->pitch, h->lpr, h->vpl, h->norms, h->stream));
    if (h->screen & 1 && h->h16 && h->h16_metric == h->metric)
        LCHK(h, launch_h16_rows(h->vecs, h->norms, lo, hi, h->pitch, h->metric, h->h16, h->h16aux, h->h16err,
                                h->stream));
    h->xsplit_rows = std::min(h->xsplit_rows, lo);
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int mhnsw_delete(mhnsw_index* h, const int64_t* keys, int64_t n, uint8_t* out) {
    std::unique_lock<std::shared_mutex> lk(h->mu);
    if (int r0 = drain(h)) return r0;
    if (n > 0 && (!keys || !out)) return fail(h, MHNSW_EINVAL, "keys and out must be non-NULL");
    for (int64_t i = 0; i < n; ++i) out[i] = 0;
    if (n <= 0 || h->layers.empty()) return 0;
    ++h->mut_epoch;
    std::vector<uint32_t> ids, lay;  // (row, layer) in the reference's order: per key, its layers ascending
    for (int64_t i = 0; i < n; ++i) {
        auto it = h->key2id.find(keys[i]);
        if (it == h->key2id.end()) continue;  // not found (or deleted earlier in this batch)
        // graph.go:852-861: layers[l].nodes[key] of every layer -- the key's live rows
        // (usually one; more after a failed insert) hold disjoint layers
        const std::vector<int32_t> rows = key_rows(h, keys[i]);
        for (int l = 0; l < (int)h->layers.size(); ++l)
            for (int32_t id : rows)
                if (in_layer(h, id, l)) {
                    h->layers[l].count--;
                    ids.push_back((uint32_t)id);
                    lay.push_back((uint32_t)l);
                }
        const int32_t id = it->second;
        h->key2id.erase(it);
        forget_key(h, keys[i], id);
        if (h->aliased)
            HIPCHK(h, hipMemcpyAsync(h->kidlive + h->hkid[id], &kNoRow, 4, hipMemcpyHostToDevice, h->stream));
        for (int32_t r : rows) h->hdead[r] = 1;
        out[i] = 1;
    }
    if (ids.empty()) return 0;
    h->any_dead = true;
    int r;
    HIPCHK(h, hipMemcpyAsync(h->dead, h->hdead.data(), (size_t)h->n, hipMemcpyHostToDevice, h->stream));
    if ((r = zero_err(h)) || (r = sync_layer_table(h))) return r;
    DeleteArgs a;
    memset(&a, 0, sizeof(a));
    a.g = graph_view(h);
    a.stats = h->d_stats + 4;
    a.err = h->d_err;
    a.vis_log2 = h->vis_log2;
    if (h->build_mode == MHNSW_BUILD_FLAT) {
        // no links to repair: the dead flag removes the row from exact search
    } else if (h->build_mode == MHNSW_BUILD_COMPAT) {
        if ((r = ensure_buf(h, h->cand, 2 * ids.size()))) return r;
        HIPCHK(h, hipMemcpyAsync(h->cand.p, ids.data(), ids.size() * 4, hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, hipMemcpyAsync(h->cand.p + ids.size(), lay.data(), lay.size() * 4, hipMemcpyHostToDevice,
                                 h->stream));
        a.ids = h->cand.p;
        a.lay = h->cand.p + ids.size();
        a.nids = (int64_t)ids.size();
        a.M = h->M;
        const int lr = launch_delete_compat(a, h->lpr, h->vpl, h->stream);
        if (lr == -2) return fail(h, MHNSW_EUNSUPPORTED, "compat delete LDS budget exceeded (M=%d)", h->M);
        LCHK(h, lr);
    } else {
        a.n = h->n;
        a.heuristic = h->heuristic;
        a.keep_pruned = h->keep_pruned;
        for (int l = 0; l < (int)h->layers.size(); ++l) {
            a.layer = l;
            a.mcap = l == 0 ? m0_of(h) : h->M;
            LCHK(h, launch_delete_repair(a, h->lpr, h->vpl, h->stream));
        }
    }
    fix_entries(h);
    int err = 0;
    HIPCHK(h, hipMemcpyAsync(&err, h->d_err, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (err & 1) return fail(h, MHNSW_EINTERNAL, "visited set overflow (raise vis_log2)");
    if (err & 4) return fail(h, MHNSW_EINTERNAL, "out-of-range node id in adjacency (graph corrupt)");
    if (err & 8) return fail(h, MHNSW_EINTERNAL, "replenish candidate heap overflow");
    return 0;
}

// analyzer.go:20-38 Connectivity: mean len(neighbors) per non-empty layer
int mhnsw_connectivity(mhnsw_index* h, double* out, int max_layers) {
    std::shared_lock<std::shared_mutex> lk(h->mu);
    std::vector<int32_t> deg((size_t)std::max<int64_t>(h->n, 1));
    int w = 0;
    for (int l = 0; l < (int)h->layers.size(); ++l) {
        const Layer& L = h->layers[l];
        if (L.count == 0) continue;
        HIPCHK(h, hipMemcpy(deg.data(), L.deg, (size_t)h->n * 4, hipMemcpyDeviceToHost));
        double sum = 0;
        for (int64_t i = 0; i < h->n; ++i)
            if (in_layer(h, i, l) && !h->hdead[i]) sum += std::max(deg[i], 0);
        if (w < max_layers && out) out[w] = sum / (double)L.count;
        ++w;
    }
    return w;
}

int mhnsw_preview_levels(mhnsw_index* h, int64_t n, int32_t* out) {
    std::shared_lock<std::shared_mutex> lk(h->mu);
    uint64_t s = h->rng;
    bool le = h->layers_exist;
    for (int64_t i = 0; i < n; ++i) {
        out[i] = random_level(h->ml, le, live_count(h) + i, &s);
        le = true;
    }
    return 0;
}

int mhnsw_stats(const mhnsw_index* h, int64_t* out, int n) {
    mhnsw_index* hh = const_cast<mhnsw_index*>(h);
    unsigned long long d[16];
    HIPCHK(hh, hipDeviceSynchronize());
    HIPCHK(hh, hipMemcpy(d, h->d_stats, sizeof(d), hipMemcpyDeviceToHost));
    int err2[2] = {0, 0};
    HIPCHK(hh, hipMemcpy(err2, h->d_err, sizeof(err2), hipMemcpyDeviceToHost));
    const int err = err2[0] | err2[1];
    if (err & 4) return fail(hh, MHNSW_EINTERNAL, "out-of-range node id in adjacency (graph corrupt)");
    const int64_t v[13] = {(int64_t)d[0], (int64_t)d[1], (int64_t)d[2], (int64_t)d[4], (int64_t)d[5], (int64_t)d[6],
                           h->stats_host[6], (int64_t)d[3], (int64_t)d[8], (int64_t)d[9], (int64_t)d[10],
                           (int64_t)d[11], (int64_t)h->build_search_us};
    for (int i = 0; i < n && i < 13; ++i) out[i] = v[i];
    return 0;
}

int mhnsw_reset_stats(mhnsw_index* h) {
    HIPCHK(h, hipDeviceSynchronize());
    HIPCHK(h, hipMemset(h->d_stats, 0, 16 * sizeof(unsigned long long)));
    for (auto& v : h->stats_host) v = 0;
    h->build_search_us = 0;
    return 0;
}

int mhnsw_last_kernel_ms(mhnsw_index* h, float* ms) {
    if (!h->have_timing) return fail(h, MHNSW_EINVAL, "no timed search yet");
    HIPCHK(h, hipEventSynchronize(h->ev1));
    HIPCHK(h, hipEventElapsedTime(ms, h->ev0, h->ev1));
    return 0;
}

int mhnsw_merge_topk_device(const int64_t* keys_in, const float* dist_in, const int32_t* n_in, int shards, int64_t B,
                            int k, int64_t* out_keys, float* out_dist, int32_t* out_n, void* stream) {
    int r = launch_merge_topk(keys_in, dist_in, n_in, shards, B, k, out_keys, out_dist, out_n, (hipStream_t)stream);
    if (r) return fail(nullptr, r == -4 ? MHNSW_EUNSUPPORTED : MHNSW_EDEVICE, "merge launch failed (%d)", r);
    return 0;
}

}  // extern "C"
