// codec.cpp -- encode.go's binary graph format (see codec.hpp).  Plain host
// C++: the GPU side only ever sees the CSR arrays api.cpp builds from it.
#include "codec.hpp"

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <unordered_set>

namespace mh {

bool key_kind_ok(int kind) { return kind >= KEY_INT && kind <= KEY_STRING; }

// ---- writer -----------------------------------------------------------------
void GoWriter::varint(int64_t v) {  // binary.PutVarint
    uint64_t ux = (uint64_t)v << 1;
    if (v < 0) ux = ~ux;
    while (ux >= 0x80) {
        out.push_back((uint8_t)(ux | 0x80));
        ux >>= 7;
    }
    out.push_back((uint8_t)ux);
}

void GoWriter::f64(double v) {
    uint8_t b[8];
    memcpy(b, &v, 8);  // little-endian host (x86-64)
    out.insert(out.end(), b, b + 8);
}

void GoWriter::str(const std::string& s) {
    varint((int64_t)s.size());
    out.insert(out.end(), s.begin(), s.end());
}

void GoWriter::floats(const float* v, int n) {
    varint(n);
    const uint8_t* p = reinterpret_cast<const uint8_t*>(v);
    out.insert(out.end(), p, p + (size_t)n * 4);
}

void GoWriter::key(int64_t k, int kind) {
    uint8_t b[8];
    switch (kind) {
        case KEY_INT:
            varint(k);
            return;
        case KEY_INT64:
        case KEY_UINT64:
            memcpy(b, &k, 8);
            out.insert(out.end(), b, b + 8);
            return;
        case KEY_STRING: {
            static const std::string empty;
            auto it = strs ? strs->find(k) : decltype(strs->find(k)){};
            str(strs && it != strs->end() ? it->second : empty);
            return;
        }
        default: {
            const uint32_t u = (uint32_t)k;
            memcpy(b, &u, 4);
            out.insert(out.end(), b, b + 4);
        }
    }
}

// ---- reader -----------------------------------------------------------------
namespace {

struct Reader {
    const uint8_t* p;
    size_t n, i = 0;
    GoGraph* g = nullptr;                           // KEY_STRING intern table
    std::unordered_map<std::string, int64_t> sidx;
    // Go errors: io.EOF when nothing could be read, io.ErrUnexpectedEOF when a
    // value is cut short, binary's overflow error for an over-long varint.
    std::string varint(int64_t& v) {
        uint64_t x = 0;
        unsigned s = 0;
        for (int k = 0; k < 10; ++k) {
            if (i >= n) return k == 0 ? "EOF" : "unexpected EOF";
            const uint8_t b = p[i++];
            if (b < 0x80) {
                if (k == 9 && b > 1) return "binary: varint overflows a 64-bit integer";
                x |= (uint64_t)b << s;
                v = (int64_t)(x >> 1);
                if (x & 1) v = ~v;
                return "";
            }
            x |= (uint64_t)(b & 0x7f) << s;
            s += 7;
        }
        return "binary: varint overflows a 64-bit integer";
    }
    std::string bytes(void* dst, size_t m) {
        if (m == 0) return "";
        if (i >= n) return "EOF";
        if (n - i < m) return "unexpected EOF";
        memcpy(dst, p + i, m);
        i += m;
        return "";
    }
    std::string key(int64_t& k, int kind) {
        switch (kind) {
            case KEY_INT:
                return varint(k);
            case KEY_INT64:
            case KEY_UINT64:
                return bytes(&k, 8);
            case KEY_INT32: {
                int32_t v;
                std::string e = bytes(&v, 4);
                k = v;
                return e;
            }
            case KEY_STRING: {  // encode.go:35-45: varint length, then the bytes
                int64_t ln = 0;
                std::string e = varint(ln);
                if (!e.empty()) return e;
                if (ln < 0 || (size_t)ln > n - i) return "unexpected EOF";
                std::string s((const char*)p + i, (size_t)ln);
                i += (size_t)ln;
                auto it = sidx.find(s);
                if (it == sidx.end()) {
                    it = sidx.emplace(s, (int64_t)g->strkeys.size()).first;
                    g->strkeys.push_back(s);
                }
                k = it->second;
                return "";
            }
            default: {
                uint32_t v;
                std::string e = bytes(&v, 4);
                k = v;
                return e;
            }
        }
    }
};

const char* key_type_name(int kind) {
    static const char* names[] = {"*int", "*int64", "*int32", "*uint64", "*uint32", "*string"};
    return names[kind];
}

std::string fmt(const char* f, ...) __attribute__((format(printf, 1, 2)));
std::string fmt(const char* f, ...) {
    char b[512];
    va_list ap;
    va_start(ap, f);
    vsnprintf(b, sizeof(b), f, ap);
    va_end(ap);
    return b;
}

}  // namespace

// encode.go:178-262 Graph.Import
std::string go_decode(const uint8_t* buf, size_t n, int key_kind, GoGraph& g) {
    if (!key_kind_ok(key_kind)) return fmt("unsupported key kind %d", key_kind);
    Reader r{buf, n};
    r.g = &g;
    g.strkeys.clear();
    std::string e;
    // multiBinaryRead(r, &version, &h.M, &h.Ml, &h.EfSearch, &dist)
    if (!(e = r.varint(g.version)).empty()) return "reading *int at index 0: " + e;
    if (!(e = r.varint(g.M)).empty()) return "reading *int at index 1: " + e;
    if (!(e = r.bytes(&g.ml, 8)).empty()) return "reading *float64 at index 2: " + e;
    if (!(e = r.varint(g.ef)).empty()) return "reading *int at index 3: " + e;
    int64_t ln = 0;
    if (!(e = r.varint(ln)).empty()) return "reading *string at index 4: " + e;
    if (ln < 0 || (size_t)ln > n) return "reading *string at index 4: unexpected EOF";
    g.dist.assign((size_t)ln, '\0');
    if (!(e = r.bytes(&g.dist[0], (size_t)ln)).empty()) return "reading *string at index 4: " + e;
    if (g.dist != "cosine" && g.dist != "euclidean") return fmt("unknown distance function \"%s\"", g.dist.c_str());
    if (g.version != 1) return fmt("incompatible encoding version: %lld", (long long)g.version);
    int64_t nl = 0;
    if (!(e = r.varint(nl)).empty()) return e;
    if (nl < 0 || nl > 64) return fmt("unsupported number of layers: %lld", (long long)nl);
    g.layers.assign((size_t)nl, GoLayer{});
    g.dim = -1;
    std::vector<float> vec;
    for (int64_t l = 0; l < nl; ++l) {
        int64_t nn = 0;
        if (!(e = r.varint(nn)).empty()) return e;
        if (nn < 0 || (size_t)nn > n) return fmt("decoding node 0: reading %s at index 0: unexpected EOF", key_type_name(key_kind));
        GoLayer& L = g.layers[(size_t)l];
        L.keys.resize((size_t)nn);
        L.nb_off.assign((size_t)nn + 1, 0);
        std::unordered_set<int64_t> seen;
        seen.reserve((size_t)nn * 2);
        for (int64_t j = 0; j < nn; ++j) {
            int64_t key = 0, vl = 0, nnb = 0;
            if (!(e = r.key(key, key_kind)).empty())
                return fmt("decoding node %lld: reading %s at index 0: %s", (long long)j, key_type_name(key_kind), e.c_str());
            if (!(e = r.varint(vl)).empty())
                return fmt("decoding node %lld: reading *[]float32 at index 1: %s", (long long)j, e.c_str());
            if (vl < 0 || (size_t)vl > n / 4 + 1)
                return fmt("decoding node %lld: reading *[]float32 at index 1: unexpected EOF", (long long)j);
            vec.resize((size_t)vl);
            if (!(e = r.bytes(vec.data(), (size_t)vl * 4)).empty())
                return fmt("decoding node %lld: reading *[]float32 at index 1: %s", (long long)j, e.c_str());
            if (!(e = r.varint(nnb)).empty())
                return fmt("decoding node %lld: reading *int at index 2: %s", (long long)j, e.c_str());
            if (nnb < 0 || (size_t)nnb > n) return fmt("decoding neighbor 0 for node %lld: unexpected EOF", (long long)j);
            if (!seen.insert(key).second) {
                if (key_kind == KEY_STRING)
                    return fmt("duplicate key %s in layer %lld", g.strkeys[(size_t)key].c_str(), (long long)l);
                return fmt("duplicate key %lld in layer %lld", (long long)key, (long long)l);
            }
            if (g.dim < 0) g.dim = (int)vl;
            if ((int)vl != g.dim) return fmt("embedding dimension mismatch: %d != %lld", g.dim, (long long)vl);
            L.keys[(size_t)j] = key;
            if (l == 0) g.vals0.insert(g.vals0.end(), vec.begin(), vec.end());
            for (int64_t k = 0; k < nnb; ++k) {
                int64_t nk = 0;
                if (!(e = r.key(nk, key_kind)).empty())
                    return fmt("decoding neighbor %lld for node %lld: %s", (long long)k, (long long)j, e.c_str());
                L.nb_keys.push_back(nk);
            }
            L.nb_off[(size_t)j + 1] = (int64_t)L.nb_keys.size();
        }
    }
    if (g.dim < 0) g.dim = 0;
    return "";
}

}  // namespace mh
