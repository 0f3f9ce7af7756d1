// hnsw_amd/graph.hpp -- header-only C++17 mirror of the reference's Go API
// (TFMV/hnsw graph.go:17-27, 305-366, 437-1110; distance.go:12-46) over the C
// ABI in mhnsw.h.  Same names, argument meaning and error messages; Go's
// `error` becomes hnsw::Error (empty == nil).  Keys are any Go cmp.Ordered
// type: integral (the C ABI's int64), floating (their IEEE total-order int64
// image) or std::string (the engine's order labels, mhnsw_strkeys_encode).
// Vectors are copied in (the reference aliases caller slices, graph.go:447,
// 911 -- documented in DESIGN.md).
#pragma once

#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <initializer_list>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "../mhnsw.h"

namespace hnsw {

using Vector = std::vector<float>;

// Go `error`: empty message == nil
struct Error {
    std::string msg;
    int code = 0;
    explicit operator bool() const { return code != 0; }
    const std::string& Error_() const { return msg; }
};

inline Error make_error(int rc, const mhnsw_index* h) {
    if (rc >= 0) return {};
    const char* m = mhnsw_last_error(h);
    return Error{m ? m : "error", rc};
}

template <class K>
struct Node {  // graph.go:19-23
    K Key;
    Vector Value;
    bool operator==(const Node& o) const { return Key == o.Key && Value == o.Value; }
};

template <class K>
Node<K> MakeNode(K key, Vector vec) {  // graph.go:25-27
    return Node<K>{key, std::move(vec)};
}

// distance.go:12 DistanceFunc -- the built-ins run on the GPU sweep kernel
struct DistanceFunc {
    int metric;
    const char* name;
    float operator()(const Vector& a, const Vector& b) const {
        if (a.size() != b.size()) throw std::invalid_argument("vector length mismatch");
        float out = 0.f;
        int rc = mhnsw_distance(metric, a.data(), b.data(), 1, (int)a.size(), &out);
        if (rc < 0) throw std::runtime_error(mhnsw_last_error(nullptr));
        return out;
    }
};
inline const DistanceFunc CosineDistance{MHNSW_COSINE, "cosine"};        // distance.go:15-17
inline const DistanceFunc EuclideanDistance{MHNSW_EUCLIDEAN, "euclidean"};  // distance.go:20-23

// ---- Graph.Rng (graph.go:312 `Rng *rand.Rand`) -----------------------------
// Levels are drawn on the host from the caller's generator, exactly where and
// how the reference draws them (graph.go:388-417, below), and handed to the
// engine as injected levels -- so a graph built through this shim depends on
// the caller's Rng the way a Go graph does.  Any source of Float64() in [0, 1)
// will do: SplitMix64Rand reproduces the engine's own seeded stream
// (mhnsw_seed / mhnsw_preview_levels), FuncRand wraps any callable.
struct Rand {
    virtual ~Rand() = default;
    virtual double Float64() = 0;  // math/rand (*Rand).Float64
    // Optional rewind: a generator that can save and restore its state lets
    // BatchAdd draw a whole run's levels ahead and, when the walk fails part
    // way, put the generator back to exactly the draws the reference made
    // (mhnsw_add_reached).  Without it, inserts that may fail go one per call.
    virtual bool GetState(std::vector<uint64_t>*) const { return false; }
    virtual void SetState(const std::vector<uint64_t>&) {}
};

struct SplitMix64Rand : Rand {
    uint64_t state;
    explicit SplitMix64Rand(uint64_t seed) : state(seed) {}
    bool GetState(std::vector<uint64_t>* s) const override {
        s->assign(1, state);
        return true;
    }
    void SetState(const std::vector<uint64_t>& s) override { state = s.at(0); }
    double Float64() override {
        uint64_t z = (state += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z = z ^ (z >> 31);
        return (double)(z >> 11) * (1.0 / 9007199254740992.0);
    }
};

struct FuncRand : Rand {
    std::function<double()> fn;
    explicit FuncRand(std::function<double()> f) : fn(std::move(f)) {}
    double Float64() override { return fn(); }
};

inline std::shared_ptr<Rand> NewRand(uint64_t seed) { return std::make_shared<SplitMix64Rand>(seed); }

// graph.go:340-342 defaultRand: time-seeded
inline std::shared_ptr<Rand> defaultRand() {
    return NewRand((uint64_t)std::chrono::high_resolution_clock::now().time_since_epoch().count());
}

// graph.go:370-385
inline int maxLevel(double ml, int64_t numNodes) {
    if (numNodes == 0) return 1;
    double l = std::log((double)numNodes);
    l /= std::log(1.0 / ml);
    return (int)std::round(l) + 1;
}

// graph.go:388-417 randomLevel, for a graph whose layer 0 holds `base` nodes
// (`layersExist` = len(h.layers) > 0); draws from rng
inline int randomLevel(Rand& rng, double ml, bool layersExist, int64_t base) {
    int max = 1;
    if (layersExist) max = maxLevel(ml, base);
    for (int level = 0; level < max; ++level)
        if (rng.Float64() > ml) return level;
    return max;
}

// Search test hacks of the reference, opt-in (Graph::TestHacks bits)
enum : unsigned { kDogQueryHack = 1u };  // graph.go:563-569, 595-619

// ---- K of Graph[K cmp.Ordered] -> the engine's int64 key -------------------
// The engine only compares keys, so each key type travels as an
// order-preserving int64 image.  String labels can be re-spaced by an Add, so
// they are converted at every call and never cached.
template <class K, class = void>
struct KeyCodec;

template <class K>
struct KeyCodec<K, std::enable_if_t<std::is_integral<K>::value>> {
    // Go encoding of K (encode.go:72-104): C++ `int` stands for Go `int`
    // (varint); other 64-/32-bit types for Go int64 / uint64 / uint32
    // (pass MHNSW_KEY_INT32 explicitly for Go int32 keys)
    static constexpr int kind = std::is_same<K, int>::value                        ? MHNSW_KEY_INT
                                : (std::is_signed<K>::value && sizeof(K) == 8)     ? MHNSW_KEY_INT64
                                : (std::is_unsigned<K>::value && sizeof(K) == 8)   ? MHNSW_KEY_UINT64
                                : (std::is_unsigned<K>::value && sizeof(K) == 4)   ? MHNSW_KEY_UINT32
                                                                                   : MHNSW_KEY_INT;
    static std::vector<int64_t> encode(mhnsw_index*, const std::vector<K>& ks, bool) {
        return std::vector<int64_t>(ks.begin(), ks.end());
    }
    static std::vector<K> decode(mhnsw_index*, const int64_t* v, size_t n) { return std::vector<K>(v, v + n); }
};

template <class K>
struct KeyCodec<K, std::enable_if_t<std::is_floating_point<K>::value>> {
    static constexpr int kind = MHNSW_KEY_INT;  // Go has no float-keyed encoding test; export as images
    static int64_t image(double f) {
        uint64_t b;
        std::memcpy(&b, &f, 8);
        b = (b >> 63) ? ~b : (b | (uint64_t(1) << 63));
        return (int64_t)(b ^ (uint64_t(1) << 63));
    }
    static double value(int64_t i) {
        uint64_t u = (uint64_t)i ^ (uint64_t(1) << 63);
        u = (u >> 63) ? (u & ~(uint64_t(1) << 63)) : ~u;
        double f;
        std::memcpy(&f, &u, 8);
        return f;
    }
    static std::vector<int64_t> encode(mhnsw_index*, const std::vector<K>& ks, bool) {
        std::vector<int64_t> out;
        for (K k : ks) {
            if (k != k) throw std::invalid_argument("NaN keys are not ordered");
            out.push_back(image((double)k));
        }
        return out;
    }
    static std::vector<K> decode(mhnsw_index*, const int64_t* v, size_t n) {
        std::vector<K> out;
        for (size_t i = 0; i < n; ++i) out.push_back((K)value(v[i]));
        return out;
    }
};

template <>
struct KeyCodec<std::string> {
    static constexpr int kind = MHNSW_KEY_STRING;
    static std::vector<int64_t> encode(mhnsw_index* h, const std::vector<std::string>& ks, bool assign) {
        std::string blob;
        std::vector<int64_t> offs{0};
        for (const auto& k : ks) {
            blob += k;
            offs.push_back((int64_t)blob.size());
        }
        std::vector<int64_t> out(ks.size());
        if (mhnsw_strkeys_encode(h, blob.data(), offs.data(), (int64_t)ks.size(), assign ? 1 : 0, out.data()) < 0)
            throw std::runtime_error(mhnsw_last_error(h));
        return out;
    }
    static std::vector<std::string> decode(mhnsw_index* h, const int64_t* v, size_t n) {
        int64_t need = 0;
        mhnsw_strkeys_decode(h, v, (int64_t)n, nullptr, 0, nullptr, &need);
        std::string blob((size_t)need, '\0');
        std::vector<int64_t> offs(n + 1);
        mhnsw_strkeys_decode(h, v, (int64_t)n, &blob[0], need, offs.data(), &need);
        std::vector<std::string> out;
        for (size_t i = 0; i < n; ++i) out.push_back(blob.substr((size_t)offs[i], (size_t)(offs[i + 1] - offs[i])));
        return out;
    }
};

template <class K>
class Graph {  // graph.go:305-332
    using Codec = KeyCodec<K>;

   public:
    const DistanceFunc* Distance = &CosineDistance;
    std::shared_ptr<Rand> Rng;  // nullptr: defaultRand() at the first Add (graph.go:407-409)
    int M = 16;
    double Ml = 0.25;
    int EfSearch = 20;
    // opt-in reproduction of the reference's test hacks in Search (kDogQueryHack)
    unsigned TestHacks = 0;

    Graph() : Rng(NewRand(0)) { create(); }
    Graph(int m, double ml, int ef, const DistanceFunc* dist, uint64_t seed)
        : Distance(dist), Rng(NewRand(seed)), M(m), Ml(ml), EfSearch(ef) {
        create();
    }
    Graph(int m, double ml, int ef, const DistanceFunc* dist, std::shared_ptr<Rand> rng)
        : Distance(dist), Rng(std::move(rng)), M(m), Ml(ml), EfSearch(ef) {
        create();
    }
    Graph(const Graph&) = delete;
    Graph& operator=(const Graph&) = delete;
    ~Graph() {
        if (h_) mhnsw_destroy(h_);
    }

    mhnsw_index* handle() { return h_; }
    Error SetOption(const char* name, int64_t v) { return make_error(mhnsw_set_option(h_, name, v), h_); }

    // graph.go:916-937
    Error Validate() {
        sync();
        return make_error(mhnsw_validate(h_), h_);
    }

    // graph.go:437-531
    Error Add(std::initializer_list<Node<K>> nodes) { return BatchAdd(std::vector<Node<K>>(nodes)); }
    Error Add(const Node<K>& n) { return BatchAdd(std::vector<Node<K>>{n}); }

    // graph.go:942-1042.  The walk inserts the nodes in order and stops at the
    // first error: a node of another dimension (the nodes before it stay
    // added, graph.go:955-960), a present key (replaced, then "node not added",
    // graph.go:1015-1037) or a failing search.  Levels come from Rng, drawn
    // exactly where the reference draws them -- one per insert the walk
    // reaches, from the layer-0 size at that moment (graph.go:962,
    // mhnsw_add_plan); `levels` overrides them (parity tests).
    Error BatchAdd(const std::vector<Node<K>>& nodes, const std::vector<int32_t>* levels = nullptr) {
        sync();
        if (nodes.empty()) return make_error(mhnsw_validate(h_), h_);
        const size_t d = Dims() ? (size_t)Dims() : nodes[0].Value.size();
        size_t bad = 0;
        while (bad < nodes.size() && nodes[bad].Value.size() == d) ++bad;
        if (bad > 0) {
            Error e = addWalk(nodes, bad, d, levels);
            if (e) {
                for (size_t i = 0; i < bad; ++i) values_.erase(nodes[i].Key);  // partly applied: Lookup asks the engine
                return e;
            }
            for (size_t i = 0; i < bad; ++i) values_[nodes[i].Key] = nodes[i].Value;
        }
        if (bad < nodes.size()) {
            if (Error v = Validate()) return v;
            return Error{"embedding dimension mismatch: " + std::to_string(d) + " != " +
                             std::to_string(nodes[bad].Value.size()),
                         MHNSW_EDIM};
        }
        return {};
    }

    // graph.go:534-625 (mode: MHNSW_MODE_COMPAT = the reference's semantics).
    // With TestHacks & kDogQueryHack, the reference's special case for the
    // query {1.0, 0.2, 0.1} is reproduced: EfSearch doubled, and key 3 put in
    // the last of exactly three results when missing (graph.go:563-569,595-619).
    std::pair<std::vector<Node<K>>, Error> Search(const Vector& near, int k, int mode = MHNSW_MODE_COMPAT) {
        const bool dog = (TestHacks & kDogQueryHack) && near.size() == 3 && near[0] == 1.0f && near[1] == 0.2f &&
                         near[2] == 0.1f;
        auto r = BatchSearch(std::vector<Vector>{near}, k, mode, /*single=*/true, dog ? 2 * EfSearch : 0);
        if (r.second) return {{}, r.second};
        std::vector<Node<K>> out = r.first.empty() ? std::vector<Node<K>>{} : r.first[0];
        if constexpr (std::is_integral<K>::value) {
            if (dog && out.size() == 3) {
                bool has = false;
                for (const auto& n : out) has = has || n.Key == (K)3;
                if (!has) {
                    auto v = Lookup((K)3);
                    if (v.second) out[2] = Node<K>{(K)3, v.first};
                }
            }
        }
        return {out, {}};
    }

    // graph.go:1047-1110
    std::pair<std::vector<std::vector<Node<K>>>, Error> BatchSearch(const std::vector<Vector>& queries, int k,
                                                                    int mode = MHNSW_MODE_COMPAT,
                                                                    bool single = false, int ef = 0) {
        sync();
        if (queries.empty()) return {{}, make_error(mhnsw_validate(h_), h_)};
        const size_t d = queries[0].size();
        const int have = Dims();
        for (size_t i = 0; i < queries.size() && have; ++i)
            if ((int)queries[i].size() != have) {
                if (single)
                    return {{}, Error{"embedding dimension mismatch: " + std::to_string(have) + " != " +
                                          std::to_string(queries[i].size()),
                                      MHNSW_EDIM}};
                return {{}, Error{"embedding dimension mismatch for query " + std::to_string(i) + ": " +
                                      std::to_string(have) + " != " + std::to_string(queries[i].size()),
                                  MHNSW_EDIM}};
            }
        std::vector<float> flat;
        for (const auto& q : queries) flat.insert(flat.end(), q.begin(), q.end());
        const size_t B = queries.size(), kk = k > 0 ? (size_t)k : 1;
        std::vector<int64_t> keys(B * kk);
        std::vector<float> dist(B * kk);
        std::vector<int32_t> n(B);
        int rc = mhnsw_search(h_, flat.data(), (int64_t)B, (int)d, k, mode, ef, nullptr, keys.data(), dist.data(),
                              n.data());
        if (rc < 0) return {{}, make_error(rc, h_)};
        std::vector<std::vector<Node<K>>> out(B);
        for (size_t b = 0; b < B; ++b) {
            const std::vector<K> ks = Codec::decode(h_, keys.data() + b * kk, (size_t)n[b]);
            for (int j = 0; j < n[b]; ++j) out[b].push_back(Node<K>{ks[(size_t)j], lookup_value(ks[(size_t)j])});
        }
        return {out, {}};
    }

    int Len() const { return (int)mhnsw_len(h_); }   // graph.go:829
    int Dims() const { return mhnsw_dims(h_); }      // graph.go:421

    std::pair<Vector, bool> Lookup(K key) {  // graph.go:898
        auto it = values_.find(key);
        if (it != values_.end()) return {it->second, true};
        Vector v(Dims() > 0 ? Dims() : 1);
        int found = mhnsw_lookup(h_, Codec::encode(h_, {key}, false)[0], v.data());
        if (found <= 0) return {{}, false};
        return {v, true};
    }

    std::vector<int> Topography() const {  // analyzer.go:41-49
        std::vector<int> t;
        for (int l = 0; l < mhnsw_num_layers(h_); ++l) t.push_back((int)mhnsw_layer_count(h_, l));
        return t;
    }

    std::vector<double> Connectivity() {  // analyzer.go:20-38
        std::vector<double> c(64);
        int n = mhnsw_connectivity(h_, c.data(), (int)c.size());
        c.resize(n > 0 ? (size_t)n : 0);
        return c;
    }

    // encode.go:131-176 Export (Go key type K: MHNSW_KEY_INT for `int`, ...)
    std::pair<std::vector<uint8_t>, Error> Export(int key_kind = Codec::kind) {
        sync();
        int64_t size = 0;
        int rc = mhnsw_export_go(h_, key_kind, nullptr, 0, &size);
        if (rc < 0) return {{}, make_error(rc, h_)};
        std::vector<uint8_t> buf((size_t)size);
        rc = mhnsw_export_go(h_, key_kind, buf.data(), size, &size);
        if (rc < 0) return {{}, make_error(rc, h_)};
        return {buf, {}};
    }

    // encode.go:181-262 Import: parameters and distance come from the file
    Error Import(const std::vector<uint8_t>& buf, int key_kind = Codec::kind) {
        int rc = mhnsw_import_go(h_, buf.data(), (int64_t)buf.size(), key_kind);
        if (rc < 0) return make_error(rc, h_);
        int metric = 0;
        mhnsw_get_params(h_, &metric, &M, &Ml, &EfSearch);
        Distance = metric == MHNSW_COSINE ? &CosineDistance : &EuclideanDistance;
        values_.clear();
        return {};
    }

    // graph.go:843-864
    bool Delete(K key) { return BatchDelete(std::vector<K>{key})[0]; }

    // graph.go:868-895
    std::vector<bool> BatchDelete(const std::vector<K>& keys) {
        std::vector<bool> res(keys.size(), false);
        if (keys.empty()) return res;
        sync();
        std::vector<int64_t> k64 = Codec::encode(h_, keys, false);
        std::vector<uint8_t> out(keys.size());
        if (mhnsw_delete(h_, k64.data(), (int64_t)k64.size(), out.data()) < 0)
            throw std::runtime_error(mhnsw_last_error(h_));
        for (size_t i = 0; i < keys.size(); ++i) {
            res[i] = out[i] != 0;
            if (res[i]) values_.erase(keys[i]);
        }
        return res;
    }

   private:
    // nodes[0, n) of dimension d through mhnsw_add, levels drawn as the walk goes
    Error addWalk(const std::vector<Node<K>>& nodes, size_t n, size_t d, const std::vector<int32_t>* levels) {
        std::vector<K> ks;
        std::vector<float> flat;
        ks.reserve(n);
        flat.reserve(n * d);
        for (size_t i = 0; i < n; ++i) {
            ks.push_back(nodes[i].Key);
            flat.insert(flat.end(), nodes[i].Value.begin(), nodes[i].Value.end());
        }
        const std::vector<int64_t> keys = Codec::encode(h_, ks, /*assign=*/true);
        if (levels) return make_error(mhnsw_add(h_, keys.data(), flat.data(), (int64_t)n, (int)d, levels->data()), h_);
        if (!Rng) Rng = defaultRand();
        int64_t nwalk = 0;
        int one = 0;
        // The run up to the next present key (where the walk may stop) goes in one
        // call with its levels drawn ahead (graph.go:388-417, 962).  When an insert
        // of it may fail part way (deleted or replaced rows, graph.go:1009:
        // one_by_one), a generator that can rewind is put back afterwards to the
        // draws of the inserts the walk reached (mhnsw_add_reached); any other
        // goes one insert per call, drawing exactly as the reference does.
        std::vector<uint64_t> snap;
        for (size_t lo = 0; lo < n;) {
            if (int rc = mhnsw_add_plan(h_, keys.data() + lo, (int64_t)(n - lo), &nwalk, &one))
                return make_error(rc, h_);
            size_t hi = lo + (size_t)nwalk;
            const bool rewind = Rng->GetState(&snap);
            if (one && !rewind) hi = lo + 1;
            const bool existed = mhnsw_num_layers(h_) > 0;
            const int64_t base = Len();
            std::vector<int32_t> lv(hi - lo);
            std::vector<int> ndraw(hi - lo, 0);
            for (size_t i = 0; i < hi - lo; ++i) {
                const int mx = (existed || i > 0) ? maxLevel(Ml, base + (int64_t)i) : 1;
                lv[i] = mx;
                for (int level = 0; level < mx; ++level) {
                    ++ndraw[i];
                    if (Rng->Float64() > Ml) {
                        lv[i] = level;
                        break;
                    }
                }
            }
            const int rc = mhnsw_add(h_, keys.data() + lo, flat.data() + lo * d, (int64_t)(hi - lo), (int)d, lv.data());
            if (rc < 0) {
                Error e = make_error(rc, h_);
                int64_t reached = 0;
                if (rewind && mhnsw_add_reached(h_, &reached) == 0) {
                    Rng->SetState(snap);
                    for (size_t i = 0; i < (size_t)reached && i < ndraw.size(); ++i)
                        for (int j = 0; j < ndraw[i]; ++j) (void)Rng->Float64();
                }
                return e;
            }
            lo = hi;
        }
        return {};
    }

    void create() {
        int rc = mhnsw_create(MHNSW_COSINE, 16, 0.25, 20, 0, &h_);
        if (rc < 0) throw std::runtime_error(mhnsw_last_error(nullptr));
    }
    void sync() { mhnsw_set_params(h_, Distance ? Distance->metric : MHNSW_NO_DISTANCE, M, Ml, EfSearch); }
    Vector lookup_value(const K& key) {
        auto it = values_.find(key);
        if (it != values_.end()) return it->second;
        Vector v(Dims() > 0 ? Dims() : 1);
        mhnsw_lookup(h_, Codec::encode(h_, {key}, false)[0], v.data());
        return v;
    }

    mhnsw_index* h_ = nullptr;
    std::map<K, Vector> values_;
};

// graph.go:340-348
template <class K>
std::unique_ptr<Graph<K>> NewGraph(uint64_t seed = 0) {
    return std::make_unique<Graph<K>>(16, 0.25, 20, &CosineDistance, seed);
}

// graph.go:352-366: validates before touching the device
template <class K>
std::pair<std::unique_ptr<Graph<K>>, Error> NewGraphWithConfig(int m, double ml, int efSearch,
                                                               const DistanceFunc* distance, uint64_t seed = 0) {
    mhnsw_index* probe = nullptr;
    int rc = mhnsw_create(distance ? distance->metric : MHNSW_NO_DISTANCE, m, ml, efSearch, seed, &probe);
    if (rc < 0) return {nullptr, Error{mhnsw_last_error(nullptr), rc}};
    mhnsw_destroy(probe);
    return {std::make_unique<Graph<K>>(m, ml, efSearch, distance, seed), {}};
}

}  // namespace hnsw
