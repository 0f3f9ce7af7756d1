// codec.hpp -- the reference's binary graph format (encode.go:128-262), host
// side only.  Export writes, Import reads:
//
//   varint version(=1) | varint M | f64 Ml | varint EfSearch | string distance
//   varint nLayers
//   per layer: varint nNodes
//     per node: key | []float32 value | varint nNeighbors | nNeighbors x key
//
// `varint` is Go's binary.PutVarint (zig-zag, 7-bit groups, encode.go:72-76),
// a string / []float32 is a varint length followed by the bytes / LE floats
// (encode.go:78-95), and f64 / fixed-width keys go through binary.Write
// little-endian (encode.go:97-104).  A Go `int` key is a varint; int64 /
// int32 / uint64 / uint32 keys are fixed-width (the type switch only
// special-cases `int`, encode.go:72).  A `string` key is a varint length
// followed by its bytes (encode.go:78-87); on the engine side string keys are
// int64 order labels (api.cpp, mhnsw_strkeys_encode), so the writer is handed
// the label -> string table and the reader interns the strings it meets.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <unordered_map>
#include <vector>

namespace mh {

enum KeyKind { KEY_INT = 0, KEY_INT64 = 1, KEY_INT32 = 2, KEY_UINT64 = 3, KEY_UINT32 = 4, KEY_STRING = 5 };

struct GoLayer {
    std::vector<int64_t> keys;    // node keys in file order
    std::vector<int64_t> nb_off;  // CSR offsets into nb_keys (size nodes + 1)
    std::vector<int64_t> nb_keys; // neighbour keys in file order
};

struct GoGraph {
    int64_t version = 1;
    int64_t M = 0;
    double ml = 0;
    int64_t ef = 0;
    std::string dist;
    int dim = 0;
    std::vector<float> vals0;     // layer-0 values, file order (nodes x dim)
    std::vector<GoLayer> layers;
    std::vector<std::string> strkeys;  // KEY_STRING: keys hold ordinals into this table
};

// Byte writer (Go encoders).
struct GoWriter {
    std::vector<uint8_t> out;
    void varint(int64_t v);
    void f64(double v);
    void str(const std::string& s);
    void floats(const float* v, int n);  // []float32
    void key(int64_t k, int kind);
    const std::unordered_map<int64_t, std::string>* strs = nullptr;  // KEY_STRING labels
};

// Parse a whole file.  Returns "" on success, else the error text (Import's
// messages where the reference has one: "unknown distance function %q",
// "incompatible encoding version: %d", Go's varint / EOF errors).
std::string go_decode(const uint8_t* buf, size_t n, int key_kind, GoGraph& g);

bool key_kind_ok(int kind);

}  // namespace mh
