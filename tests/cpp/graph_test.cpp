// C++ mirror of the reference's own tests (graph_test.go, distance_test.go),
// written against the C++ host shim include/hnsw_amd/graph.hpp -> C ABI ->
// HIP kernels.  Run by tests/test_cpp_shim.py (GPU).  Exit code = failures.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <set>

#include "hnsw_amd/graph.hpp"
#include "oracle.h"  // test infrastructure: the CPU restatement, as the checker only

static int failures = 0;
#define REQUIRE(cond, name)                                              \
    do {                                                                 \
        if (!(cond)) {                                                   \
            std::printf("FAIL %s: %s (line %d)\n", name, #cond, __LINE__); \
            ++failures;                                                  \
        }                                                                \
    } while (0)

static uint32_t bits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

// distance_test.go:9-31
static void TestDistances() {
    REQUIRE(bits(hnsw::EuclideanDistance({1, 2, 3}, {4, 5, 6})) == 0x40a646e1u, "TestEuclideanDistance");
    REQUIRE(std::fabs(hnsw::CosineDistance({1, 1, 1}, {0.8f, 0.8f, 0.8f})) <= 1e-6, "TestCosineSimilarity");
    REQUIRE(std::fabs(hnsw::CosineDistance({1, 0}, {0, 1}) - 1.0f) <= 1e-6, "TestCosineSimilarity");
    REQUIRE(std::fabs(hnsw::CosineDistance({1, 0}, {1, 0})) <= 1e-6, "TestCosineSimilarity");
}

// graph_test.go:27-74 (hand-built layer; node under map key 4 has Key 5, Value {4})
static void Test_layerNode_search() {
    hnsw::Graph<int> g(6, 0.5, 4, &hnsw::EuclideanDistance, 0);
    const int64_t keys[6] = {0, 1, 2, 3, 5, 5};
    const float vals[6] = {0, 1, 2, 3, 4, 5};
    const int32_t deg[6] = {3, -1, -1, 2, -1, -1};
    int32_t adj[6 * 7];
    for (int& a : adj) a = -1;
    adj[0] = 1, adj[1] = 2, adj[2] = 3, adj[3 * 7 + 0] = 4, adj[3 * 7 + 1] = 5;
    const int32_t entry[1] = {0};
    REQUIRE(mhnsw_import(g.handle(), 6, 1, 1, 7, keys, vals, deg, adj, entry, nullptr) == 0, "Test_layerNode_search import");
    auto r = g.Search({4}, 2);
    REQUIRE(!r.second, "Test_layerNode_search err");
    REQUIRE(r.first.size() == 2 && r.first[0].Key == 5 && r.first[1].Key == 3, "Test_layerNode_search keys");
}

// graph_test.go:86-133 (level stream: SplitMix64 seed 0 -- Go's seed-0 stream is not
// reproducible offline, so the golden [64,65,62,63] is checked as a property)
static void TestGraph_AddSearch() {
    hnsw::Graph<int> g(6, 0.5, 20, &hnsw::EuclideanDistance, 0);
    for (int i = 0; i < 128; ++i) REQUIRE(!g.Add(hnsw::MakeNode(i, {(float)i})), "TestGraph_AddSearch add");
    auto topo = g.Topography();
    REQUIRE(!topo.empty() && topo[0] == 128, "TestGraph_AddSearch topography[0]");
    for (size_t i = 1; i < topo.size(); ++i) REQUIRE(topo[i] <= topo[i - 1], "TestGraph_AddSearch topography");
    auto r = g.Search({64.5f}, 4);
    REQUIRE(!r.second && r.first.size() == 4, "TestGraph_AddSearch len");
    std::set<int> got;
    for (auto& n : r.first) {
        got.insert(n.Key);
        REQUIRE(n.Value.size() == 1 && n.Value[0] == (float)n.Key, "TestGraph_AddSearch value");
    }
    REQUIRE(got.count(64) && got.count(65), "TestGraph_AddSearch nearest");
    for (int k : got) REQUIRE(k >= 60 && k <= 68, "TestGraph_AddSearch range");
}

// graph_test.go:253-275
static void TestGraph_DefaultCosine() {
    auto g = hnsw::NewGraph<int>(7);
    REQUIRE(!g->Add({hnsw::MakeNode(1, {1, 1}), hnsw::MakeNode(2, {0, 1}), hnsw::MakeNode(3, {1, -1})}),
            "TestGraph_DefaultCosine add");
    auto r = g->Search({0.5f, 0.5f}, 1);
    REQUIRE(!r.second && r.first.size() == 1, "TestGraph_DefaultCosine len");
    REQUIRE(r.first.size() == 1 && (r.first[0] == hnsw::Node<int>{1, {1, 1}}), "TestGraph_DefaultCosine node");
}

// graph_test.go:415-459
static void TestGraphValidation() {
    auto ok = hnsw::NewGraphWithConfig<int>(16, 0.25, 20, &hnsw::CosineDistance);
    REQUIRE(!ok.second && ok.first, "ValidConfig");
    auto e1 = hnsw::NewGraphWithConfig<int>(0, 0.25, 20, &hnsw::CosineDistance);
    REQUIRE(e1.second && e1.second.msg.find("M must be greater than 0") != std::string::npos, "InvalidM");
    auto e2 = hnsw::NewGraphWithConfig<int>(16, 0, 20, &hnsw::CosineDistance);
    REQUIRE(e2.second && e2.second.msg.find("Ml must be between 0 and 1") != std::string::npos, "InvalidMl");
    auto e3 = hnsw::NewGraphWithConfig<int>(16, 1.5, 20, &hnsw::CosineDistance);
    REQUIRE(e3.second && e3.second.msg.find("Ml must be between 0 and 1") != std::string::npos, "InvalidMl");
    auto e4 = hnsw::NewGraphWithConfig<int>(16, 0.25, 0, &hnsw::CosineDistance);
    REQUIRE(e4.second && e4.second.msg.find("EfSearch must be greater than 0") != std::string::npos,
            "InvalidEfSearch");
    auto e5 = hnsw::NewGraphWithConfig<int>(16, 0.25, 20, nullptr);
    REQUIRE(e5.second && e5.second.msg.find("Distance function must be set") != std::string::npos,
            "NilDistance");
    auto g = hnsw::NewGraph<int>();
    auto r = g->Search({1, 2, 3}, 0);
    REQUIRE(r.second && r.second.msg.find("k must be greater than 0") != std::string::npos, "InvalidK");
}

static void TestDimensionMismatch() {
    auto g = hnsw::NewGraph<int>(3);
    REQUIRE(!g->Add(hnsw::MakeNode(1, {1, 2, 3})), "dim add");
    auto e = g->Add(hnsw::MakeNode(2, {1, 2}));
    REQUIRE(e && e.msg == "embedding dimension mismatch: 3 != 2", "dim add mismatch");
    auto r = g->Search({1, 2}, 1);
    REQUIRE(r.second && r.second.msg == "embedding dimension mismatch: 3 != 2", "dim search mismatch");
    auto v = g->Lookup(1);
    REQUIRE(v.second && v.first == hnsw::Vector({1, 2, 3}), "Lookup");
    REQUIRE(!g->Lookup(42).second, "Lookup missing");
    REQUIRE(g->Len() == 1 && g->Dims() == 3, "Len/Dims");
}

// batch_delete_test.go:10-105 TestBatchDelete
static void TestBatchDelete() {
    auto cfg = hnsw::NewGraphWithConfig<int>(16, 0.25, 20, &hnsw::CosineDistance, 5);
    REQUIRE(!cfg.second, "NewGraphWithConfig");
    auto& g = *cfg.first;
    for (int i = 1; i <= 10; ++i) g.Add(hnsw::MakeNode(i, {(float)i, (float)i, (float)i}));
    REQUIRE(g.Len() == 10, "initial size");
    auto r = g.BatchDelete({1, 3, 5});
    REQUIRE(r == std::vector<bool>({true, true, true}), "delete existing");
    REQUIRE(g.Len() == 7, "size after delete");
    for (int k : {1, 3, 5}) REQUIRE(!g.Lookup(k).second, "deleted lookup");
    for (int k : {2, 4, 6, 7, 8, 9, 10}) REQUIRE(g.Lookup(k).second, "kept lookup");
    r = g.BatchDelete({11, 12, 13});
    REQUIRE(r == std::vector<bool>({false, false, false}), "delete missing");
    REQUIRE(g.Len() == 7, "size unchanged");
    r = g.BatchDelete({2, 15, 4, 20});
    REQUIRE(r == std::vector<bool>({true, false, true, false}), "delete mixed");
    REQUIRE(g.Len() == 5, "size after mixed");
    REQUIRE(g.BatchDelete({}).empty(), "delete empty");
    r = g.BatchDelete({6, 7, 8, 9, 10});
    REQUIRE(r == std::vector<bool>({true, true, true, true, true}), "delete rest");
    REQUIRE(g.Len() == 0, "empty graph");
    auto s = g.Search({1, 1, 1}, 3);
    REQUIRE(!s.second && s.first.empty(), "search on emptied graph");
}

// graph_test.go:135-172 TestGraph_AddDelete (levels from this engine's RNG)
static void TestGraph_AddDelete() {
    hnsw::Graph<int> g(6, 0.5, 20, &hnsw::EuclideanDistance, 0);
    for (int i = 0; i < 128; ++i) REQUIRE(!g.Add(hnsw::MakeNode(i, {(float)i})), "add");
    REQUIRE(g.Len() == 128, "len 128");
    for (int i = 0; i < 128; i += 2) REQUIRE(g.Delete(i), "delete even");
    REQUIRE(g.Len() == 64, "len 64");
    REQUIRE(!g.Delete(-1), "DeleteNotFound");
    auto s = g.Search({65.f}, 4);
    REQUIRE(!s.second, "search after delete");
}

// encode_test.go:120-160 TestGraph_ExportImport
static void TestGraph_ExportImport() {
    hnsw::Graph<int> g1(6, 0.5, 20, &hnsw::EuclideanDistance, 0);
    for (int i = 0; i < 128; ++i) g1.Add(hnsw::MakeNode(i, {(float)((i * 37) % 128) / 128.f}));
    auto ex = g1.Export();
    REQUIRE(!ex.second && !ex.first.empty(), "Export");
    hnsw::Graph<int> g2;
    REQUIRE(!g2.Import(ex.first), "Import");
    REQUIRE(g1.Len() == g2.Len() && g1.Topography() == g2.Topography(), "Len/Topography");
    REQUIRE(g1.Connectivity() == g2.Connectivity(), "Connectivity");
    REQUIRE(g2.M == 6 && g2.Ml == 0.5 && g2.EfSearch == 20 && g2.Distance == &hnsw::EuclideanDistance, "params");
    auto n1 = g1.Search({0.5f}, 10), n2 = g2.Search({0.5f}, 10);
    REQUIRE(!n1.second && !n2.second && n1.first.size() == n2.first.size(), "Search");
    for (size_t i = 0; i < n1.first.size() && i < n2.first.size(); ++i)
        REQUIRE(n1.first[i] == n2.first[i], "Search nodes");
}

// Graph[string] (examples/optimized_distance/main.go:82, vector/example/main.go:79):
// string keys are ordered labels inside the engine; Search, Lookup, Delete and
// the string encoding (encode.go:78-87) round-trip the caller's strings.
static void TestGraph_StringKeys() {
    hnsw::Graph<std::string> g(8, 0.25, 20, &hnsw::CosineDistance, 1);
    const char* words[] = {"apple", "banana", "cherry", "date", "elderberry", "fig", "grape", "honeydew",
                           "kiwi", "lemon", "mango", "nectarine", "orange", "papaya", "quince", "raspberry"};
    for (int i = 0; i < 16; ++i) {
        hnsw::Vector v(8);
        for (int j = 0; j < 8; ++j) v[j] = (float)((i * 7 + j * 3) % 11) + 0.5f * (float)(i == j);
        REQUIRE(!g.Add(hnsw::MakeNode(std::string(words[i]), v)), "add string key");
    }
    REQUIRE(g.Len() == 16, "len 16");
    auto look = g.Lookup("kiwi");
    REQUIRE(look.second && look.first.size() == 8, "Lookup string");
    auto s = g.Search(look.first, 1, MHNSW_MODE_EXACT);
    REQUIRE(!s.second && s.first.size() == 1 && s.first[0].Key == "kiwi", "Search returns the string key");
    REQUIRE(g.Delete("kiwi") && !g.Delete("kiwi") && !g.Delete("zucchini"), "Delete string key");
    auto ex = g.Export();
    REQUIRE(!ex.second && !ex.first.empty(), "Export string keys");
    hnsw::Graph<std::string> g2;
    REQUIRE(!g2.Import(ex.first), "Import string keys");
    REQUIRE(g2.Len() == 15 && g2.Lookup("lemon").second && !g2.Lookup("kiwi").second, "imported keys");
    auto a = g.Search(look.first, 5, MHNSW_MODE_EXACT), b = g2.Search(look.first, 5, MHNSW_MODE_EXACT);
    REQUIRE(!a.second && !b.second && a.first.size() == b.first.size(), "imported search");
    for (size_t i = 0; i < a.first.size() && i < b.first.size(); ++i)
        REQUIRE(a.first[i].Key == b.first[i].Key, "imported search keys");
}

// K = float64: ordered by value (negative, zero, positive)
static void TestGraph_FloatKeys() {
    hnsw::Graph<double> g(6, 0.5, 20, &hnsw::EuclideanDistance, 0);
    for (int i = 0; i < 64; ++i) REQUIRE(!g.Add(hnsw::MakeNode(-3.25 + 0.125 * i, {(float)i})), "add float key");
    auto s = g.Search({17.f}, 1, MHNSW_MODE_EXACT);
    REQUIRE(!s.second && s.first.size() == 1 && s.first[0].Key == -3.25 + 0.125 * 17, "float key round trip");
    REQUIRE(g.Delete(-3.25) && g.Len() == 63, "delete float key");
}

// Graph.Rng (graph.go:312): levels are drawn by the shim from the caller's
// generator with the reference's rule (graph.go:388-417, layer-0 size growing
// per insert, through single Adds and one BatchAdd alike); the engine receives
// them as injected levels.  Replaying the rule with a fresh copy of the same
// generator and building the oracle with those levels gives the same graph.
static std::shared_ptr<hnsw::Rand> lcg(uint64_t s) {  // a caller-supplied source, not the engine's stream
    return std::make_shared<hnsw::FuncRand>([s]() mutable {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        return (double)(s >> 11) * (1.0 / 9007199254740992.0);
    });
}

static bool same_graph(mhnsw_index* h, og_graph* o, const char* name) {
    int64_t N1 = 0, N2 = 0;
    int d1, d2, L1, L2, c1, c2;
    mhnsw_export_sizes(h, &N1, &d1, &L1, &c1);
    og_export_sizes(o, &N2, &d2, &L2, &c2);
    if (N1 != N2 || L1 != L2 || d1 != d2) {
        std::printf("FAIL %s: sizes %lld/%lld layers %d/%d\n", name, (long long)N1, (long long)N2, L1, L2);
        return false;
    }
    const int cap = c1 > c2 ? c1 : c2;
    std::vector<int64_t> k1(N1), k2(N1);
    std::vector<float> v1((size_t)N1 * d1), v2((size_t)N1 * d1);
    std::vector<int32_t> g1((size_t)L1 * N1), g2((size_t)L1 * N1), a1((size_t)L1 * N1 * cap), a2((size_t)L1 * N1 * cap);
    std::vector<int32_t> e1(L1), e2(L1);
    mhnsw_export(h, k1.data(), v1.data(), g1.data(), a1.data(), cap, e1.data(), nullptr);
    og_export(o, k2.data(), v2.data(), g2.data(), a2.data(), cap, e2.data(), nullptr);
    if (k1 != k2 || g1 != g2 || e1 != e2) {
        std::printf("FAIL %s: keys/degrees/entries differ\n", name);
        return false;
    }
    for (size_t r = 0; r < (size_t)L1 * N1; ++r) {
        const int dg = g1[r];
        std::set<int32_t> s1(a1.begin() + r * cap, a1.begin() + r * cap + (dg > 0 ? dg : 0));
        std::set<int32_t> s2(a2.begin() + r * cap, a2.begin() + r * cap + (dg > 0 ? dg : 0));
        if (s1 != s2) {
            std::printf("FAIL %s: adjacency row %zu differs\n", name, r);
            return false;
        }
    }
    return true;
}

static void TestGraph_RngLevels() {
    const int n = 600, d = 16, M = 8;
    const double ml = 0.3;
    std::vector<hnsw::Node<int>> nodes;
    uint64_t x = 12345;
    for (int i = 0; i < n; ++i) {
        hnsw::Vector v(d);
        for (auto& f : v) {
            x = x * 2862933555777941757ull + 3037000493ull;
            f = (float)((double)(x >> 40) / (double)(1ull << 24)) * 2.f - 1.f;
        }
        nodes.push_back(hnsw::MakeNode(i * 7 - 100, v));
    }
    hnsw::Graph<int> g(M, ml, 20, &hnsw::CosineDistance, lcg(99));
    for (int i = 0; i < 50; ++i) REQUIRE(!g.Add(nodes[(size_t)i]), "RngLevels add");
    REQUIRE(!g.BatchAdd(std::vector<hnsw::Node<int>>(nodes.begin() + 50, nodes.end())), "RngLevels batch add");
    // replay graph.go:388-417 with a fresh generator of the same seed
    auto rng = lcg(99);
    std::vector<int32_t> lv(n);
    std::vector<int64_t> keys(n);
    std::vector<float> flat;
    for (int i = 0; i < n; ++i) {
        lv[(size_t)i] = hnsw::randomLevel(*rng, ml, i > 0, i);
        keys[(size_t)i] = nodes[(size_t)i].Key;
        flat.insert(flat.end(), nodes[(size_t)i].Value.begin(), nodes[(size_t)i].Value.end());
    }
    og_graph* o = og_create(OG_COSINE, OG_ORDER_DEV, M, 0, ml, 20, 0);
    REQUIRE(og_add(o, keys.data(), flat.data(), n, d, lv.data()) == 0, "RngLevels oracle add");
    REQUIRE(same_graph(g.handle(), o, "RngLevels"), "RngLevels graph == oracle graph with the caller's levels");
    std::vector<int> topo;
    for (int l = 0; l < og_num_layers(o); ++l) topo.push_back((int)og_layer_count(o, l));
    REQUIRE(g.Topography() == topo && topo.size() >= 3, "RngLevels topography");
    og_destroy(o);
    // the seed matters: another generator gives other levels, hence another graph
    hnsw::Graph<int> g2(M, ml, 20, &hnsw::CosineDistance, lcg(7));
    REQUIRE(!g2.BatchAdd(nodes), "RngLevels other seed");
    auto r2 = lcg(7);
    int differ = 0;
    for (int i = 0; i < n; ++i) differ += hnsw::randomLevel(*r2, ml, i > 0, i) != lv[(size_t)i];
    REQUIRE(differ > 0, "RngLevels other seed draws other levels");
    // SplitMix64Rand(seed) reproduces the engine's own seeded stream
    hnsw::SplitMix64Rand sm(42);
    std::vector<int32_t> want(300);
    mhnsw_index* h = nullptr;
    mhnsw_create(MHNSW_COSINE, 16, 0.25, 20, 42, &h);
    mhnsw_preview_levels(h, 300, want.data());
    mhnsw_destroy(h);
    bool same = true;
    for (int i = 0; i < 300; ++i) same = same && hnsw::randomLevel(sm, 0.25, i > 0, i) == want[(size_t)i];
    REQUIRE(same, "SplitMix64Rand == engine stream");
}

// graph.go:563-569,595-619 (opt-in): the dog query doubles EfSearch and puts
// key 3 ("canine") into a 3-result answer that lacks it.  Hand graph (one
// layer): canine is unreachable, so the plain answer misses it.
static void TestGraph_DogQueryHack() {
    hnsw::Graph<int> g(4, 0.5, 20, &hnsw::CosineDistance, 1);
    const int64_t keys[5] = {1, 2, 3, 4, 5};  // dog, puppy, canine, cat, kitten (negative_test.go:17-23)
    const float vals[15] = {1.0f, 0.2f, 0.1f, 0.9f, 0.3f, 0.2f, 0.8f, 0.3f, 0.3f, 0.1f, 1.0f, 0.2f, 0.2f, 0.9f, 0.3f};
    const int32_t deg[5] = {2, 2, 0, 2, 2};
    int32_t adj[5 * 5];
    for (int& a : adj) a = -1;
    adj[0] = 1, adj[1] = 3, adj[5] = 0, adj[6] = 4, adj[15] = 0, adj[16] = 4, adj[20] = 1, adj[21] = 3;
    const int32_t entry[1] = {0};
    REQUIRE(mhnsw_import(g.handle(), 5, 3, 1, 5, keys, vals, deg, adj, entry, nullptr) == 0, "DogQuery import");
    auto keyset = [](const std::vector<hnsw::Node<int>>& v) {
        std::vector<int> k;
        for (auto& n : v) k.push_back(n.Key);
        return k;
    };
    auto plain = g.Search({1.0f, 0.2f, 0.1f}, 3);
    REQUIRE(!plain.second && plain.first.size() == 3, "DogQuery plain len");
    const std::vector<int> pk = keyset(plain.first);
    REQUIRE(std::set<int>(pk.begin(), pk.end()).count(3) == 0, "DogQuery plain misses canine");
    g.TestHacks = hnsw::kDogQueryHack;
    auto hacked = g.Search({1.0f, 0.2f, 0.1f}, 3);
    REQUIRE(!hacked.second && hacked.first.size() == 3, "DogQuery hacked len");
    std::vector<int> want = pk;
    want[2] = 3;
    REQUIRE(keyset(hacked.first) == want, "DogQuery canine replaces the last result");
    REQUIRE(hacked.first[2].Value == hnsw::Vector({0.8f, 0.3f, 0.3f}), "DogQuery canine value");
    auto other = g.Search({1.0f, 0.2f, 0.1000001f}, 3);  // not the dog query: untouched
    const std::vector<int> ok = keyset(other.first);
    REQUIRE(!other.second && std::set<int>(ok.begin(), ok.end()).count(3) == 0, "DogQuery other query untouched");
}

#define RUN(t)                           \
    do {                                 \
        std::printf("RUN %s\n", #t);      \
        t();                             \
    } while (0)

int main() {
    std::setvbuf(stdout, nullptr, _IONBF, 0);  // a crash must not swallow the log
    RUN(TestDistances);
    RUN(Test_layerNode_search);
    RUN(TestGraph_AddSearch);
    RUN(TestGraph_DefaultCosine);
    RUN(TestGraphValidation);
    RUN(TestDimensionMismatch);
    RUN(TestBatchDelete);
    RUN(TestGraph_AddDelete);
    RUN(TestGraph_ExportImport);
    RUN(TestGraph_StringKeys);
    RUN(TestGraph_FloatKeys);
    RUN(TestGraph_RngLevels);
    RUN(TestGraph_DogQueryHack);
    std::printf("%s (%d failures)\n", failures ? "FAIL" : "PASS", failures);
    return failures;
}
