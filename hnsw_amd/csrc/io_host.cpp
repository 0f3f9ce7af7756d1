// io_host.cpp -- the graph's exchange formats: the engine's CSR export / import,
// the reference's binary format (encode.go:15-327: Export / Import / SavedGraph)
// through codec.cpp, and Go string keys (Graph[string]) as order labels.
#include "index.hpp"

using namespace mhh;

namespace mhh {


// drop every row and layer (Graph.Import replaces the graph, encode.go:208)
void reset_graph(mhnsw_index* h) {
    (void)hipStreamSynchronize(h->stream);
    auto F = [](auto*& p) {
        if (p) (void)hipFree(p);
        p = nullptr;
    };
    F(h->vecs);
    F(h->norms);
    F(h->h16);
    F(h->h16aux);
    F(h->keys);
    F(h->levels);
    F(h->dead);
    F(h->cur_entry);
    F(h->inc_cnt);
    F(h->inc_src);
    F(h->inc_dist);
    for (auto& L : h->layers) {
        F(L.deg);
        F(L.adj);
        F(L.adjd);
    }
    h->layers.clear();
    memset(h->layers_host, 0, sizeof(h->layers_host));
    h->capn = h->n = 0;
    h->xsplit_rows = h->xsplit_plane = 0;
    h->dim = h->pitch = h->lpr = h->vpl = 0;
    h->layers_exist = h->any_dead = false;
    F(h->kid);
    F(h->kidlive);
    F(h->kprev);
    h->aliased = false;
    h->hkid.clear();
    h->hprev.clear();
    h->dead_kid.clear();
    h->key2id.clear();
    h->hlevels.clear();
    h->hmask.clear();
    h->hdead.clear();
    h->s2l.clear();
    h->l2s.clear();
    h->partial_rows = 0;
    h->xgone_epoch = ~0ull;
}

int import_csr(mhnsw_index* h, int64_t N, int dim, int L, int cap, const int64_t* keys, const float* vecs,
               const int32_t* deg, const int32_t* adj, const int32_t* entry, const uint8_t* dead) {
    if (h->n > 0) return fail(h, MHNSW_EINVAL, "import requires an empty index");
    if (L > MH_MAXL) return fail(h, MHNSW_EUNSUPPORTED, "more than %d layers", MH_MAXL);
    if (cap > 64) return fail(h, MHNSW_EUNSUPPORTED, "degree cap above 64 unsupported");
    int r;
    if ((r = set_shape(h, dim))) return r;
    if ((r = ensure_capacity(h, std::max<int64_t>(N, 1)))) return r;
    if ((r = ensure_layer(h, L - 1))) return r;
    // make every layer at least `cap` wide
    for (int l = 0; l < L; ++l) {
        Layer& Ly = h->layers[l];
        if (Ly.cap < cap) {
            (void)hipFree(Ly.adj);
            (void)hipFree(Ly.adjd);
            Ly.adj = nullptr;
            Ly.adjd = nullptr;
            Ly.cap = cap;
            if ((r = grow(h, Ly.adj, 0, h->capn * cap, 0xFF)) || (r = grow(h, Ly.adjd, 0, h->capn * cap, 0))) return r;
        }
    }
    HIPCHK(h, hipMemcpy(h->keys, keys, N * 8, hipMemcpyHostToDevice));
    if ((r = ensure_buf(h, h->tmp, (size_t)N * dim))) return r;
    HIPCHK(h, hipMemcpy(h->tmp.p, vecs, (size_t)N * dim * 4, hipMemcpyHostToDevice));
    LCHK(h, launch_pad_rows(h->tmp.p, N, dim, h->vecs, h->pitch, h->stream));
    LCHK(h, launch_norms(h->vecs, 0, N, h->pitch, h->lpr, h->vpl, h->norms, h->stream));
    if ((r = h16_rows(h, 0, N))) return r;
    h->xsplit_rows = 0;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    std::vector<int32_t> row;
    h->hlevels.assign(N, 0);
    h->hmask.assign(N, 0u);
    h->hdead.assign(N, 0);
    h->any_dead = false;
    for (int64_t i = 0; i < N && dead; ++i) {
        h->hdead[i] = dead[i] ? 1 : 0;
        h->any_dead |= dead[i] != 0;
    }
    HIPCHK(h, hipMemcpy(h->dead, h->hdead.data(), (size_t)N, hipMemcpyHostToDevice));
    for (int l = 0; l < L; ++l) {
        Layer& Ly = h->layers[l];
        HIPCHK(h, hipMemcpy(Ly.deg, deg + (size_t)l * N, N * 4, hipMemcpyHostToDevice));
        row.assign((size_t)N * Ly.cap, -1);
        Ly.count = 0;
        for (int64_t i = 0; i < N; ++i) {
            const int d = deg[(size_t)l * N + i];
            if (d != -2) {
                h->hmask[i] |= 1u << l;
                h->hlevels[i] = std::max(h->hlevels[i], l);
                if (!h->hdead[i]) Ly.count++;
            }
            for (int j = 0; j < d && j < cap; ++j) row[(size_t)i * Ly.cap + j] = adj[((size_t)l * N + i) * cap + j];
        }
        HIPCHK(h, hipMemcpy(Ly.adj, row.data(), row.size() * 4, hipMemcpyHostToDevice));
        Ly.entry = entry[l];
    }
    HIPCHK(h, hipMemcpy(h->levels, h->hlevels.data(), N * 4, hipMemcpyHostToDevice));
    // a key's live rows (disjoint layers): the newest heads its chain (key_rows)
    h->key2id.clear();
    std::vector<int32_t> prevl((size_t)N, -1);
    for (int64_t i = 0; i < N; ++i) {
        if (h->hdead[i]) continue;
        auto it = h->key2id.find(keys[i]);
        if (it != h->key2id.end()) prevl[i] = it->second;
        h->key2id[keys[i]] = (int32_t)i;
    }
    h->n = N;
    h->layers_exist = L > 0;
    // key identity: several rows of one key (a replaced or re-added key) -> kids
    std::unordered_map<int64_t, int32_t> first;
    bool dup = false;
    for (int64_t i = 0; i < N; ++i) dup |= !first.emplace(keys[i], (int32_t)i).second;
    h->dead_kid.clear();
    for (auto& kv : first)
        if (!h->key2id.count(kv.first)) h->dead_kid[kv.first] = kv.second;
    if (dup) {
        if ((r = start_alias(h))) return r;  // kid = row, then rows of repeated keys take the first one's
        std::vector<int32_t> live((size_t)N, -1);
        for (int64_t i = 0; i < N; ++i) h->hkid[i] = first[keys[i]];
        for (auto& kv : h->key2id) live[first[kv.first]] = kv.second;
        h->hprev = prevl;
        HIPCHK(h, hipMemcpy(h->kid, h->hkid.data(), (size_t)N * 4, hipMemcpyHostToDevice));
        HIPCHK(h, hipMemcpy(h->kidlive, live.data(), (size_t)N * 4, hipMemcpyHostToDevice));
        HIPCHK(h, hipMemcpy(h->kprev, h->hprev.data(), (size_t)N * 4, hipMemcpyHostToDevice));
    }
    // live rows outside layer 0 (an exported graph keeps a failed insert's upper rows):
    // the brute force skips them as the reference's Search cannot reach them
    h->partial_rows = 0;
    for (int64_t i = 0; i < N; ++i) h->partial_rows += !h->hdead[i] && !in_layer(h, i, 0);
    ++h->mut_epoch;
    return 0;
}

const char* metric_name(int m) { return m == COSINE ? "cosine" : "euclidean"; }

// ---- Go string keys: order-maintenance labels -------------------------------
constexpr int64_t SK_LO = -(int64_t(1) << 62), SK_HI = int64_t(1) << 62, SK_STEP = int64_t(1) << 32;

// Re-space every label evenly in string order and rewrite the keys stored on
// the device (every row, deleted ones included -- compat search can still
// return them) and in key2id.  Entries with label INT64_MIN are new strings
// that are not on the device yet.
int strkey_relabel(mhnsw_index* h) {
    const int64_t n = (int64_t)h->s2l.size();
    const int64_t step = (int64_t)(((uint64_t)SK_HI - (uint64_t)SK_LO) / (uint64_t)(n + 1));
    std::unordered_map<int64_t, int64_t> remap;
    remap.reserve((size_t)n * 2);
    int64_t i = 1;
    for (auto& kv : h->s2l) {
        const int64_t nl = SK_LO + i++ * step;
        if (kv.second != INT64_MIN) remap[kv.second] = nl;
        kv.second = nl;
    }
    h->l2s.clear();
    for (auto& kv : h->s2l) h->l2s[kv.second] = kv.first;
    if (h->n > 0 && !remap.empty()) {
        std::vector<int64_t> keys((size_t)h->n);
        HIPCHK(h, hipStreamSynchronize(h->stream));
        HIPCHK(h, hipMemcpy(keys.data(), h->keys, (size_t)h->n * 8, hipMemcpyDeviceToHost));
        for (auto& k : keys) {
            auto it = remap.find(k);
            if (it != remap.end()) k = it->second;
        }
        HIPCHK(h, hipMemcpy(h->keys, keys.data(), (size_t)h->n * 8, hipMemcpyHostToDevice));
    }
    std::unordered_map<int64_t, int32_t> k2;
    k2.reserve(h->key2id.size() * 2);
    for (auto& kv : h->key2id) {
        auto it = remap.find(kv.first);
        k2[it != remap.end() ? it->second : kv.first] = kv.second;
    }
    h->key2id.swap(k2);
    h->relabels++;
    return 0;
}

// Label for a new string: a fixed step past the ends, the midpoint inside;
// no room left -> relabel everything.
int strkey_insert(mhnsw_index* h, const std::string& s) {
    auto it = h->s2l.emplace(s, INT64_MIN).first;
    const bool first = it == h->s2l.begin();
    auto nx = std::next(it);
    const bool last = nx == h->s2l.end();
    const int64_t prev = first ? SK_LO : std::prev(it)->second;
    const int64_t next = last ? SK_HI : nx->second;
    int64_t lab = INT64_MIN;
    if (last && !first && next - prev > SK_STEP) lab = prev + SK_STEP;
    else if (first && !last && next - prev > SK_STEP) lab = next - SK_STEP;
    else if (next - prev >= 2) lab = prev + (next - prev) / 2;
    if (lab == INT64_MIN) return strkey_relabel(h);
    it->second = lab;
    h->l2s[lab] = s;
    return 0;
}

// import: distinct strings (file order) -> labels evenly spaced in string order
void strkey_table(mhnsw_index* h, const std::vector<std::string>& strs, std::vector<int64_t>& lab) {
    h->s2l.clear();
    h->l2s.clear();
    for (const auto& x : strs) h->s2l.emplace(x, INT64_MIN);
    (void)strkey_relabel(h);  // nothing on the device yet
    h->relabels--;
    lab.resize(strs.size());
    for (size_t i = 0; i < strs.size(); ++i) lab[i] = h->s2l[strs[i]];
}

bool key_fits(const mhnsw_index* h, int64_t k, int kind) {
    switch (kind) {
        case KEY_STRING: return h->l2s.count(k) != 0;
        case KEY_INT32: return k >= INT32_MIN && k <= INT32_MAX;
        case KEY_UINT32: return k >= 0 && k <= (int64_t)UINT32_MAX;
        case KEY_UINT64: return k >= 0;
        default: return true;
    }
}

// encode.go:128-174 Graph.Export: nodes in id (insertion) order, neighbour keys
// ascending (Go writes both in map order, which is unspecified)
int export_go(mhnsw_index* h, int key_kind, std::vector<uint8_t>& out) {
    if (!key_kind_ok(key_kind)) return fail(h, MHNSW_EINVAL, "unsupported key kind %d", key_kind);
    int r = validate(h);
    if (r) return r;
    GoWriter w;
    w.strs = &h->l2s;
    w.varint(1);  // encodingVersion
    w.varint(h->M);
    w.f64(h->ml);
    w.varint(h->ef);
    w.str(metric_name(h->metric));
    const int L = (int)h->layers.size();
    w.varint(L);
    const int64_t N = h->n;
    std::vector<int64_t> keys((size_t)std::max<int64_t>(N, 1));
    std::vector<float> vecs((size_t)std::max<int64_t>(N, 1) * std::max(h->dim, 1));
    if (N > 0) {
        HIPCHK(h, hipMemcpy(keys.data(), h->keys, N * 8, hipMemcpyDeviceToHost));
        HIPCHK(h, hipMemcpy2D(vecs.data(), (size_t)h->dim * 4, h->vecs, (size_t)h->pitch * 4, (size_t)h->dim * 4, N,
                              hipMemcpyDeviceToHost));
    }
    std::vector<int32_t> deg, adj;
    std::vector<int64_t> nb;
    for (int l = 0; l < L; ++l) {
        const Layer& Ly = h->layers[l];
        deg.resize((size_t)N);
        adj.resize((size_t)N * Ly.cap);
        if (N > 0) {
            HIPCHK(h, hipMemcpy(deg.data(), Ly.deg, N * 4, hipMemcpyDeviceToHost));
            HIPCHK(h, hipMemcpy(adj.data(), Ly.adj, (size_t)N * Ly.cap * 4, hipMemcpyDeviceToHost));
        }
        w.varint(Ly.count);
        for (int64_t i = 0; i < N; ++i) {
            if (!in_layer(h, i, l) || h->hdead[i]) continue;
            if (!key_fits(h, keys[i], key_kind)) return fail(h, MHNSW_EINVAL, "key %lld does not fit the key type", (long long)keys[i]);
            w.key(keys[i], key_kind);
            w.floats(vecs.data() + (size_t)i * h->dim, h->dim);
            const int d = std::min(std::max(deg[i], 0), Ly.cap);
            nb.clear();
            for (int j = 0; j < d; ++j) nb.push_back(keys[(size_t)adj[(size_t)i * Ly.cap + j]]);
            std::sort(nb.begin(), nb.end());
            w.varint(d);
            for (int64_t k : nb) w.key(k, key_kind);
        }
    }
    out.swap(w.out);
    return 0;
}

// encode.go:178-262 Graph.Import.  Neighbour keys that are not nodes of the
// same layer (dangling edges to deleted nodes in a Go-written file) become nil
// map entries in the reference; they are dropped here.
int import_go(mhnsw_index* h, const uint8_t* buf, int64_t size, int key_kind) {
    GoGraph gg;
    const std::string e = go_decode(buf, (size_t)std::max<int64_t>(size, 0), key_kind, gg);
    if (!e.empty()) return fail(h, MHNSW_EINVAL, "%s", e.c_str());
    h->M = (int)gg.M;
    h->ml = gg.ml;
    h->ef = (int)gg.ef;
    h->metric = gg.dist == "cosine" ? COSINE : EUCLIDEAN;
    const int L = (int)gg.layers.size();
    const int64_t N = L ? (int64_t)gg.layers[0].keys.size() : 0;
    reset_graph(h);
    if (key_kind == KEY_STRING) {  // ordinals -> evenly spaced labels in string order
        std::vector<int64_t> lab;
        strkey_table(h, gg.strkeys, lab);
        for (auto& Ly : gg.layers) {
            for (auto& k : Ly.keys) k = lab[(size_t)k];
            for (auto& k : Ly.nb_keys) k = lab[(size_t)k];
        }
    }
    if (N == 0) return 0;
    if (L > MH_MAXL) return fail(h, MHNSW_EUNSUPPORTED, "more than %d layers", MH_MAXL);
    std::unordered_map<int64_t, int32_t> id;
    id.reserve((size_t)N * 2);
    for (int64_t j = 0; j < N; ++j) id[gg.layers[0].keys[(size_t)j]] = (int32_t)j;
    std::vector<int32_t> deg((size_t)L * N, -2), entry((size_t)L, -1);
    std::vector<uint8_t> member((size_t)N);
    std::vector<std::vector<int32_t>> rows((size_t)L);  // resolved neighbour ids, CSR per layer
    std::vector<std::vector<int64_t>> roff((size_t)L);
    int maxd = 0;
    for (int l = 0; l < L; ++l) {
        const GoLayer& G = gg.layers[(size_t)l];
        std::fill(member.begin(), member.end(), 0);
        std::vector<int32_t> ids(G.keys.size());
        for (size_t j = 0; j < G.keys.size(); ++j) {
            auto it = id.find(G.keys[j]);
            if (it == id.end())
                return fail(h, MHNSW_EINVAL, "node %lld of layer %d is missing from layer 0", (long long)G.keys[j], l);
            ids[j] = it->second;
            member[(size_t)it->second] = 1;
            if (entry[(size_t)l] < 0 || it->second < entry[(size_t)l]) entry[(size_t)l] = it->second;
        }
        std::vector<int32_t>& R = rows[(size_t)l];
        std::vector<int64_t>& O = roff[(size_t)l];
        O.assign((size_t)N + 1, 0);
        // resolve neighbours, bucket by node id
        std::vector<int32_t> cnt((size_t)N, 0);
        std::vector<int32_t> tmp;
        std::vector<int64_t> tmpo(G.keys.size() + 1, 0);
        for (size_t j = 0; j < G.keys.size(); ++j) {
            for (int64_t t = G.nb_off[j]; t < G.nb_off[j + 1]; ++t) {
                auto it = id.find(G.nb_keys[(size_t)t]);
                if (it != id.end() && member[(size_t)it->second]) tmp.push_back(it->second);
            }
            tmpo[j + 1] = (int64_t)tmp.size();
            cnt[(size_t)ids[j]] = (int32_t)(tmpo[j + 1] - tmpo[j]);
            maxd = std::max(maxd, cnt[(size_t)ids[j]]);
        }
        for (int64_t i = 0; i < N; ++i) O[(size_t)i + 1] = O[(size_t)i] + cnt[(size_t)i];
        R.assign((size_t)O[(size_t)N], 0);
        for (size_t j = 0; j < G.keys.size(); ++j) {
            const int32_t i = ids[j];
            deg[(size_t)l * N + i] = cnt[(size_t)i];  // a decoded map is never nil (encode.go:237)
            std::copy(tmp.begin() + tmpo[j], tmp.begin() + tmpo[j + 1], R.begin() + O[(size_t)i]);
        }
    }
    int cap = 0;
    for (int l = 0; l < L; ++l) cap = std::max(cap, cap_of(h, l));
    cap = std::max(cap, maxd);
    if (cap > 64) return fail(h, MHNSW_EUNSUPPORTED, "degree %d above 64 unsupported", maxd);
    std::vector<int32_t> adj((size_t)L * N * cap, -1);
    for (int l = 0; l < L; ++l)
        for (int64_t i = 0; i < N; ++i)
            for (int64_t t = roff[(size_t)l][(size_t)i]; t < roff[(size_t)l][(size_t)i + 1]; ++t)
                adj[((size_t)l * N + i) * cap + (size_t)(t - roff[(size_t)l][(size_t)i])] = rows[(size_t)l][(size_t)t];
    return import_csr(h, N, gg.dim, L, cap, gg.layers[0].keys.data(), gg.vals0.data(), deg.data(), adj.data(),
                      entry.data(), nullptr);
}

}  // namespace mhh

extern "C" {


int mhnsw_import(mhnsw_index* h, int64_t N, int dim, int L, int cap, const int64_t* keys, const float* vecs,
                 const int32_t* deg, const int32_t* adj, const int32_t* entry, const uint8_t* dead) {
    std::unique_lock<std::shared_mutex> lk(h->mu);
    int r = drain(h);
    if (r) return r;
    return import_csr(h, N, dim, L, cap, keys, vecs, deg, adj, entry, dead);
}

int mhnsw_export_go(mhnsw_index* h, int key_kind, uint8_t* buf, int64_t cap, int64_t* size) {
    std::shared_lock<std::shared_mutex> lk(h->mu);
    std::vector<uint8_t> out;
    int r = export_go(h, key_kind, out);
    if (r) return r;
    if (size) *size = (int64_t)out.size();
    if (!buf) return 0;
    if (cap < (int64_t)out.size())
        return fail(h, MHNSW_EINVAL, "buffer too small: need %lld bytes", (long long)out.size());
    memcpy(buf, out.data(), out.size());
    return 0;
}

int mhnsw_import_go(mhnsw_index* h, const uint8_t* buf, int64_t size, int key_kind) {
    std::unique_lock<std::shared_mutex> lk(h->mu);
    int r = drain(h);
    if (r) return r;
    return import_go(h, buf, size, key_kind);
}

// encode.go:301-327 SavedGraph.Save (renameio): write a uniquely named temp file
// in the target directory, fsync it, then rename it over path.  Concurrent
// Saves (the read lock allows them) never share a temp file.
int mhnsw_save(mhnsw_index* h, const char* path, int key_kind) {
    std::shared_lock<std::shared_mutex> lk(h->mu);
    std::vector<uint8_t> out;
    int r = export_go(h, key_kind, out);
    if (r) return r;
    std::string tmpl = std::string(path) + ".tmp.XXXXXX";
    std::vector<char> name(tmpl.begin(), tmpl.end());
    name.push_back('\0');
    const int fd = mkstemp(name.data());
    if (fd < 0) return fail(h, MHNSW_EINVAL, "create temp file for %s failed", path);
    size_t off = 0;
    bool ok = true;
    while (ok && off < out.size()) {
        const ssize_t w = write(fd, out.data() + off, out.size() - off);
        if (w < 0 && errno == EINTR) continue;
        ok = w > 0;
        if (ok) off += (size_t)w;
    }
    ok = ok && fsync(fd) == 0;
    ok = (close(fd) == 0) && ok;
    if (!ok) {
        unlink(name.data());
        return fail(h, MHNSW_EINVAL, "write %s failed", name.data());
    }
    if (rename(name.data(), path) != 0) {
        unlink(name.data());
        return fail(h, MHNSW_EINVAL, "rename to %s failed", path);
    }
    return 0;
}

// encode.go:280-299 LoadSavedGraph: a missing or empty file leaves the graph empty
int mhnsw_load(mhnsw_index* h, const char* path, int key_kind) {
    std::unique_lock<std::shared_mutex> lk(h->mu);
    if (int r0 = drain(h)) return r0;
    FILE* f = fopen(path, "rb");
    if (!f) return 0;
    std::vector<uint8_t> buf;
    uint8_t tmp[1 << 16];
    size_t got;
    while ((got = fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + got);
    fclose(f);
    if (buf.empty()) return 0;
    const int r = import_go(h, buf.data(), (int64_t)buf.size(), key_kind);
    if (r) return fail(h, r, "import: %s", h->err.c_str());
    return 0;
}

// graph.go:1116-1537 SearchWithNegative(s) / BatchSearchWithNegatives
}  // extern "C"

// ---- Go string keys (Graph[string]) ------------------------------------------
int mhnsw_strkeys_encode(mhnsw_index* h, const char* blob, const int64_t* offs, int64_t n, int assign,
                         int64_t* out) {
    std::unique_lock<std::shared_mutex> lk(h->mu);
    if (n < 0) return fail(h, MHNSW_EINVAL, "negative key count");
    if (assign) {  // a re-spacing rewrites the stored keys enqueued searches read
        if (int r0 = drain(h)) return r0;
    }
    std::vector<std::string> ks((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        if (offs[i + 1] < offs[i]) return fail(h, MHNSW_EINVAL, "bad string offsets");
        ks[(size_t)i].assign(blob + offs[i], (size_t)(offs[i + 1] - offs[i]));
    }
    int r;
    if (assign) {
        std::vector<const std::string*> fresh;
        for (const auto& x : ks)
            if (!h->s2l.count(x)) fresh.push_back(&x);
        std::sort(fresh.begin(), fresh.end(), [](const std::string* a, const std::string* b) { return *a < *b; });
        fresh.erase(std::unique(fresh.begin(), fresh.end(), [](const std::string* a, const std::string* b) { return *a == *b; }),
                    fresh.end());
        if (!fresh.empty()) {
            if (fresh.size() * 4 > h->s2l.size()) {  // bulk: one even re-spacing
                for (const auto* x : fresh) h->s2l.emplace(*x, INT64_MIN);
                if ((r = strkey_relabel(h))) return r;
            } else {
                for (const auto* x : fresh)
                    if ((r = strkey_insert(h, *x))) return r;
            }
        }
    }
    for (int64_t i = 0; i < n; ++i) {
        auto it = h->s2l.find(ks[(size_t)i]);
        out[i] = it == h->s2l.end() ? INT64_MIN : it->second;
    }
    return MHNSW_OK;
}

int mhnsw_strkeys_decode(mhnsw_index* h, const int64_t* labels, int64_t n, char* blob, int64_t cap, int64_t* offs,
                         int64_t* need) {
    std::shared_lock<std::shared_mutex> lk(h->mu);
    int64_t tot = 0;
    for (int64_t i = 0; i < n; ++i) {
        auto it = h->l2s.find(labels[i]);
        if (it != h->l2s.end()) tot += (int64_t)it->second.size();
    }
    if (need) *need = tot;
    if (!blob || cap < tot) return MHNSW_OK;
    int64_t o = 0;
    for (int64_t i = 0; i < n; ++i) {
        offs[i] = o;
        auto it = h->l2s.find(labels[i]);
        if (it == h->l2s.end()) continue;
        memcpy(blob + o, it->second.data(), it->second.size());
        o += (int64_t)it->second.size();
    }
    offs[n] = o;
    return MHNSW_OK;
}

