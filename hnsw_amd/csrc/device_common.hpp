// device_common.hpp -- wave64 building blocks shared by every HIP kernel of the
// engine (gfx950 / CDNA4 only).
//
//  * Row-distance engine: one query held in VGPRs (float4 per lane), candidate
//    rows gathered straight from the row-major HBM vector store with 16-B
//    coalesced loads (a 768-d row = 3 x 1 KiB wave-instructions), per-lane
//    fmaf accumulation, then a transposed reduce-scatter over the lanes of a
//    row so that G rows finish in log2(lanes) shuffle steps instead of G*6.
//    The summation tree is the canonical order restated in oracle/oracle.c
//    (og_dev_sum): element e -> lane (e/4) mod 64, fmaf in ascending e,
//    butterfly over offsets 32..1 -- so distances are bitwise reproducible.
//  * Sorted candidate list across lanes (ef <= 64*R entries, R per lane),
//    ballot/popcount insertion, used by beam search and top-k merges.
//  * LDS open-addressing visited set (CAS probes, bounded).
//  * Go container/heap restatement on LDS arrays (compat semantics,
//    heap/heap.go + graph.go:94-170), executed redundantly by every lane.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MH_MAXL 32

namespace mh {

constexpr uint32_t ID_MASK = 0x7FFFFFFFu;
constexpr uint32_t EXP_BIT = 0x80000000u;
constexpr uint32_t EMPTY_ID = 0x7FFFFFFFu;
constexpr uint32_t VIS_EMPTY = 0xFFFFFFFFu;

enum Metric { COSINE = 0, EUCLIDEAN = 1 };

// one layer of the graph in HBM (fixed-stride adjacency rows)
struct LayerDev {
    int32_t* deg;  // [cap_nodes]: -2 absent, -1 nil neighbour map, >=0 degree
    int32_t* adj;  // [cap_nodes * cap] internal ids
    float* adjd;   // [cap_nodes * cap] edge distances (batch build)
    int cap;
    int pad_;
};

struct GraphDev {
    const float* vecs;        // [cap_nodes * pitch] row-major, zero padded
    const float* norms;       // [cap_nodes] canonical |x|
    const int64_t* keys;      // [cap_nodes]
    const LayerDev* layers;   // [nlayers] device table (read-only in kernels)
    int pitch;
    int dim;
    int metric;
    int nlayers;
    uint32_t capn;  // rows allocated: every gathered id is checked against it
    int* err;       // bit 4: out-of-range id seen (load clamped, no fault)
    const uint8_t* dead;  // [cap_nodes] 1 = deleted (nullptr until the first Delete)
    // fp16 screening copy (nullptr = off), only ever used to skip candidates
    // whose f32 distance provably exceeds the list's worst ("The fp16 screening copy").
    //   cosine: row r is fp16(x / |x| * 2^14) (no per-row value needed);
    //           NaN halves mark a row the screen must never reject
    //   L2:     row r is fp16(x * 2^e) with max|x_i| 2^e in [2^14, 2^15);
    //           h16aux[r] = {2^-e, |x|}, NaN 2^-e marks a never-rejected row
    const uint16_t* h16;      // [cap_nodes * pitch]
    const float2* h16aux;     // [cap_nodes] (L2)
    // [1] max over the copy's rows of the measured relative rounding |y' - y| / |y|
    // (<= 2^-11 by construction; replaces 2^-11 in the screening bounds)
    const float* h16err;
    // key identity (compat semantics: the reference's maps are keyed by K, so a
    // replaced or re-added key leaves several rows with one key; every map
    // operation compares kids).  nullptr until the first such row: kid == row.
    const int32_t* kid;   // [cap_nodes] the first row that ever held this row's key
    int32_t* kidlive;     // [cap_nodes] by kid: the key's newest live row (-1 none)
    // [cap_nodes] the next older live row of the same key (-1 none): a key can
    // hold live nodes in several layers at once (a failed insert leaves its node
    // in the layers above the failing one, graph.go:1009; a later insert of the
    // key below them adds another), one per layer map, in disjoint layers
    const int32_t* kprev;
};

__device__ __forceinline__ bool is_dead(const GraphDev& g, uint32_t id) { return g.dead && g.dead[id]; }
__device__ __forceinline__ uint32_t kid_of(const GraphDev& g, uint32_t id) {
    return g.kid ? (uint32_t)g.kid[id] : id;
}

// `layer.nodes[key] != nil` (graph.go:576-578): present in layer l and not deleted
__device__ __forceinline__ bool is_member(const GraphDev& g, int l, uint32_t id) {
    return id < g.capn && g.layers[l].deg[id] != -2 && !is_dead(g, id);
}

// bounds guard for gathered ids: records the violation and clamps to row 0
__device__ __forceinline__ uint32_t guard_id(const GraphDev& g, uint32_t id) {
    if (id >= g.capn) {
        atomicOr(g.err, 4);
        return 0u;
    }
    return id;
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ float rl_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ uint32_t rl_u(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ int rl_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ int64_t rl_i64(int64_t v, int l) {
    int lo = __builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, l);
    int hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ uint32_t shfl_u(uint32_t v, int src) { return (uint32_t)__shfl((int)v, src, 64); }
// push-style permute: lane l's value lands in lane dst(l)
__device__ __forceinline__ uint32_t push_to(uint32_t v, int dst) {
    return (uint32_t)__builtin_amdgcn_ds_permute(dst << 2, (int)v);
}

__device__ __forceinline__ bool lt_di(float d1, uint32_t i1, float d2, uint32_t i2) {
    return d1 < d2 || (d1 == d2 && i1 < i2);
}

constexpr int ilog2(int x) { return x <= 1 ? 0 : 1 + ilog2(x >> 1); }

// ---------------------------------------------------------------------------
// dimension configuration: LPR lanes per row, VPL float4 per lane
// ---------------------------------------------------------------------------
template <int LPR_, int VPL_>
struct Cfg {
    static constexpr int LPR = LPR_;
    static constexpr int VPL = VPL_;
    static constexpr int RPI = 64 / LPR_;          // rows per wave-instruction
    static constexpr int PITCH = LPR_ * 4 * VPL_;  // floats per stored row
    static constexpr int LOG_LPR = ilog2(LPR_);
};

template <class C>
struct QReg {
    float4 v[C::VPL];
};

template <class C>
__device__ __forceinline__ void load_query(QReg<C>& q, const float* qp) {
    const int sub = lane_id() & (C::LPR - 1);
#pragma unroll
    for (int v = 0; v < C::VPL; ++v) q.v[v] = *reinterpret_cast<const float4*>(qp + sub * 4 + v * C::LPR * 4);
}

// butterfly within an LPR-lane segment, offsets LPR/2 .. 1 (canonical tree; the
// 64-lane levels above LPR only ever add +0.0f for d <= 4*LPR)
template <int LPR>
__device__ __forceinline__ float seg_allreduce(float x) {
#pragma unroll
    for (int o = LPR / 2; o >= 1; o >>= 1) x = x + __shfl_xor(x, o, 64);
    return x;
}

template <class C>
__device__ __forceinline__ float query_norm(const QReg<C>& q) {
    float acc = 0.f;
#pragma unroll
    for (int v = 0; v < C::VPL; ++v) {
        acc = fmaf(q.v[v].x, q.v[v].x, acc);
        acc = fmaf(q.v[v].y, q.v[v].y, acc);
        acc = fmaf(q.v[v].z, q.v[v].z, acc);
        acc = fmaf(q.v[v].w, q.v[v].w, acc);
    }
    return sqrtf(seg_allreduce<C::LPR>(acc));
}

// branch-free select (keeps register arrays out of scratch: a `c ? p[i] : p[j]`
// on an array is otherwise rewritten into a dynamically indexed stack load)
__device__ __forceinline__ float bsel(uint32_t mask, float a, float b) {
    return __uint_as_float((__float_as_uint(a) & mask) | (__float_as_uint(b) & ~mask));
}

// Transposed reduce-scatter of G per-lane partials over an LPR-lane segment.
// On return lane l holds the full sum of row g(l) = (l % LPR) >> (LOG_LPR - log2 G).
template <int G, int LPR>
__device__ __forceinline__ float reduce_rows(float (&p)[G]) {
    static_assert(G >= 1 && G <= LPR && (G & (G - 1)) == 0, "G must be a power of two <= LPR");
    const int lane = lane_id();
#pragma unroll
    for (int s = 0; (LPR >> (s + 1)) >= 1; ++s) {
        const int o = LPR >> (s + 1);
        const int cnt = G >> s;
        if (cnt > 1) {
            const int half = cnt >> 1;
            const uint32_t up = (lane & o) ? 0xFFFFFFFFu : 0u;
#pragma unroll
            for (int i = 0; i < half; ++i) {
                const float lo = p[i], hi = p[i + half];
                const float send = bsel(up, lo, hi);
                const float keep = bsel(up, hi, lo);
                p[i] = keep + __shfl_xor(send, o, 64);
            }
        } else {
            p[0] = p[0] + __shfl_xor(p[0], o, 64);
        }
    }
    return p[0];
}

template <class C, int G>
struct RowMap {
    static constexpr int LG = ilog2(G);
    static constexpr int T = G * C::RPI;  // rows per group
    // row-in-group index that lane l owns after reduce_rows
    __device__ static __forceinline__ int owned_row(int l) {
        const int g = (l & (C::LPR - 1)) >> (C::LOG_LPR - LG);
        return g * C::RPI + l / C::LPR;
    }
    // lane that owns row t of the group
    __device__ static __forceinline__ int owner(int t) {
        const int g = t / C::RPI, s = t % C::RPI;
        return s * C::LPR + (g << (C::LOG_LPR - LG));
    }
    // row-in-group index that register g of lane l computes
    __device__ static __forceinline__ int reg_row(int g, int l) { return g * C::RPI + l / C::LPR; }
};

// Evaluate up to T = G*RPI rows.  row_id(t) supplies the internal id of row t
// (t < n); returns, in every lane, the canonical dot (or squared L2) sum of the
// row the lane owns (RowMap::owned_row).
template <class C, int G, bool L2>
__device__ __forceinline__ float eval_rows(const QReg<C>& q, const float* __restrict__ X, int pitch,
                                           const uint32_t (&ids)[G], const bool (&valid)[G]) {
    const int sub = lane_id() & (C::LPR - 1);
    float4 x[G][C::VPL];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const float* rp = X + (size_t)ids[g] * (size_t)pitch + sub * 4;
#pragma unroll
        for (int v = 0; v < C::VPL; ++v) {
            if (valid[g])
                x[g][v] = *reinterpret_cast<const float4*>(rp + v * C::LPR * 4);
            else
                x[g][v] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    float p[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        float acc = 0.f;
#pragma unroll
        for (int v = 0; v < C::VPL; ++v) {
            if (L2) {
                float t0 = x[g][v].x - q.v[v].x, t1 = x[g][v].y - q.v[v].y;
                float t2 = x[g][v].z - q.v[v].z, t3 = x[g][v].w - q.v[v].w;
                acc = fmaf(t0, t0, acc);
                acc = fmaf(t1, t1, acc);
                acc = fmaf(t2, t2, acc);
                acc = fmaf(t3, t3, acc);
            } else {
                acc = fmaf(x[g][v].x, q.v[v].x, acc);
                acc = fmaf(x[g][v].y, q.v[v].y, acc);
                acc = fmaf(x[g][v].z, q.v[v].z, acc);
                acc = fmaf(x[g][v].w, q.v[v].w, acc);
            }
        }
        p[g] = acc;
    }
    return reduce_rows<G, C::LPR>(p);
}

// N consecutive dwords from a 4-byte aligned address, in 16-B loads then one
// 8-B / 4-B tail (rows of the screening copies are lane-contiguous).
template <int N>
__device__ __forceinline__ void load_dwords(const int* p, int (&x)[N]) {
#pragma unroll
    for (int k = 0; k + 4 <= N; k += 4) {
        const int4 t = *reinterpret_cast<const int4*>(p + k);
        x[k] = t.x, x[k + 1] = t.y, x[k + 2] = t.z, x[k + 3] = t.w;
    }
    constexpr int R = N % 4, B = N - N % 4;
    if constexpr (R == 3) {
        typedef int i3 __attribute__((ext_vector_type(3)));
        const i3 t = *reinterpret_cast<const i3*>(p + B);
        x[B] = t.x, x[B + 1] = t.y, x[B + 2] = t.z;
    } else if constexpr (R == 2) {
        const int2 t = *reinterpret_cast<const int2*>(p + B);
        x[B] = t.x, x[B + 1] = t.y;
    } else if constexpr (R == 1) {
        x[B] = p[B];
    }
}

// Approximate sums from the fp16 screening copy, same lane/element mapping
// as eval_rows, rows stored lane-contiguous (lane sub's 4*VPL halves at
// [sub*4*VPL, (sub+1)*4*VPL) of the row: one 16-B + one 8-B load at 768-d).  Dot: sum q_i * h_i.  L2: sum (q_i - h_i * inv_g)^2 with inv[g]
// the row's unscale.
template <class C, int G, bool L2>
__device__ __forceinline__ float eval_rows_h16(const QReg<C>& q, const uint16_t* __restrict__ H, int pitch,
                                               const uint32_t (&ids)[G], const bool (&valid)[G],
                                               const float (&inv)[G]) {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    const int sub = lane_id() & (C::LPR - 1);
    h4 x[G][C::VPL];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        // lane-contiguous rows (k_h16_rows): this lane's 8*VPL bytes are adjacent
        int d[2 * C::VPL];
        if (valid[g]) {
            load_dwords<2 * C::VPL>(reinterpret_cast<const int*>(H + (size_t)ids[g] * (size_t)pitch + sub * 4 * C::VPL), d);
        } else {
#pragma unroll
            for (int k = 0; k < 2 * C::VPL; ++k) d[k] = 0;
        }
#pragma unroll
        for (int v = 0; v < C::VPL; ++v) x[g][v] = __builtin_bit_cast(h4, make_int2(d[2 * v], d[2 * v + 1]));
    }
    float p[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        float acc = 0.f;
#pragma unroll
        for (int v = 0; v < C::VPL; ++v) {
            const float x0 = (float)x[g][v].x, x1 = (float)x[g][v].y, x2 = (float)x[g][v].z, x3 = (float)x[g][v].w;
            if (L2) {
                const float t0 = fmaf(x0, inv[g], -q.v[v].x), t1 = fmaf(x1, inv[g], -q.v[v].y);
                const float t2 = fmaf(x2, inv[g], -q.v[v].z), t3 = fmaf(x3, inv[g], -q.v[v].w);
                acc = fmaf(t0, t0, acc);
                acc = fmaf(t1, t1, acc);
                acc = fmaf(t2, t2, acc);
                acc = fmaf(t3, t3, acc);
            } else {
                acc = fmaf(x0, q.v[v].x, acc);
                acc = fmaf(x1, q.v[v].y, acc);
                acc = fmaf(x2, q.v[v].z, acc);
                acc = fmaf(x3, q.v[v].w, acc);
            }
        }
        p[g] = acc;
    }
    return reduce_rows<G, C::LPR>(p);
}

// Lane-contiguous row copies (the fp16 screening copy, eval_rows_h16): the
// 4*VPL elements lane `sub` needs (sub*4 + v*LPR*4 + j, the same elements as
// in eval_rows) are adjacent, so a lane's part of a row is one or two loads.
__host__ __device__ constexpr int lc_vpl(int pitch) { return pitch >= 256 ? pitch / 256 : 1; }

// Screening bounds ("The fp16 screening copy"), with y the row the fp16 copy stands for
// (x / |x|_f32 for cosine, x for L2) and |y' - y| <= E |y|, E = the measured
// maximum over the copy's rows (k_h16_rows, f64, rounded up; it includes the
// cosine normalisation), at most 2^-11 (+ 2u) -- the bounds below are written
// with 2^-11, the kernels use E:
//   cosine: |S / |q|_f32 - (the f32 cosine term)| <= 2^-11 + 2 gamma + 8u
//           (Cauchy-Schwarz; gamma = accumulation bound of one f32 dot,
//           < 2^-18 for dim <= 4096), so approx > wd + 2^-11 + 2^-16 => f32 > wd
//   L2:     | |q - x'| - |q - x| | <= |x' - x| <= 2^-11 |x|  (triangle inequality)
//           + relative rounding of both computed distances (< 2^-16)
// Valid while no intermediate over/underflows: rows are screened only when
// 2^-50 <= max|x_i| <= 2^50 and queries when 2^-40 <= |q| <= 2^40.
constexpr float H16_COS_SCALE = 6.103515625e-05f;                      // 2^-14
constexpr float H16_DELTA_COS = 0.00048828125f + 0.0000152587890625f;  // 2^-11 + 2^-16
constexpr float H16_REL_L2 = 1.0f - 0.000030517578125f;                // 1 - 2^-15
constexpr float H16_ABS_L2 = 0.00048828125f * 1.000030517578125f;      // 2^-11 (1 + 2^-15)
constexpr float H16_MIN_L2 = 8.881784197001252e-16f;                   // 2^-50
__device__ __forceinline__ bool h16_query_ok(float qn) {
    return qn >= 9.094947017729282e-13f && qn <= 1.099511627776e12f;  // [2^-40, 2^40]; false for NaN
}
// true when the f32 distance of this row is certainly > wd (s: eval_rows_h16 sum)
// margins for a measured E: cosine E + 2^-16, L2 E (1 + 2^-15)
__device__ __forceinline__ float h16_margin_cos(float e) { return e + 0.0000152587890625f; }
__device__ __forceinline__ float h16_margin_l2(float e) { return e * 1.000030517578125f; }
__device__ __forceinline__ bool h16_rejects_cos(float s, float qn, float wd, float mcos) {
    const float da = 1.0f - (s * H16_COS_SCALE) / qn;
    return da > wd + mcos;
}
__device__ __forceinline__ bool h16_rejects_l2(float s, float xn, float wd, float ml2) {
    const float da = sqrtf(s);
    return da >= H16_MIN_L2 && da * H16_REL_L2 - ml2 * xn > wd;
}

// The other side, for the neighbour-selection screen: true when the f32
// distance is certainly < lo (same bounds as the rejects, mirrored, with the
// relative slack doubled for the rounding of the upper bound itself).
__device__ __forceinline__ bool h16_below_cos(float s, float qn, float lo, float mcos) {
    const float da = 1.0f - (s * H16_COS_SCALE) / qn;
    return da < lo - mcos;
}
__device__ __forceinline__ bool h16_below_l2(float s, float xn, float lo, float ml2) {
    const float da = sqrtf(s);
    return da >= H16_MIN_L2 && da * (2.0f - H16_REL_L2 * H16_REL_L2) + ml2 * xn * (2.0f - H16_REL_L2) < lo;
}

// finalize a canonical sum into a distance (distance.go:15-23 semantics)
__device__ __forceinline__ float finalize(int metric, float s, float xn, float qn) {
    if (metric == COSINE) return 1.0f - s / (xn * qn);
    return sqrtf(s);
}

// ---------------------------------------------------------------------------
// LDS visited set
// ---------------------------------------------------------------------------
__device__ __forceinline__ void vis_clear(uint32_t* tab, int size) {
    uint4* t4 = reinterpret_cast<uint4*>(tab);
    const uint4 e = make_uint4(VIS_EMPTY, VIS_EMPTY, VIS_EMPTY, VIS_EMPTY);
    for (int i = lane_id(); i < size / 4; i += 64) t4[i] = e;
    if (lane_id() < (size & 3)) tab[(size & ~3) + lane_id()] = VIS_EMPTY;  // a size that is not a multiple of 4
}

// 0 = already visited, 1 = newly recorded, 2 = table congested (not recorded)
__device__ __forceinline__ int vis_probe(uint32_t* tab, int mask, uint32_t id) {
    uint32_t h = (id * 0x9E3779B1u) ^ (id >> 15);
    h &= (uint32_t)mask;
#pragma unroll 1
    for (int p = 0; p < 48; ++p) {
        uint32_t old = atomicCAS(&tab[h], VIS_EMPTY, id);
        if (old == VIS_EMPTY) return 1;
        if (old == id) return 0;
        h = (h + 1) & (uint32_t)mask;
    }
    return 2;
}

// The same set over any size (the beam search sizes it to the LDS its
// occupancy leaves): multiply-high range reduction, linear probing with wrap.
__device__ __forceinline__ int vis_probe_n(uint32_t* tab, uint32_t size, uint32_t id) {
    uint32_t h = __umulhi((id * 0x9E3779B1u) ^ (id >> 15), size);
#pragma unroll 1
    for (int p = 0; p < 48; ++p) {
        uint32_t old = atomicCAS(&tab[h], VIS_EMPTY, id);
        if (old == VIS_EMPTY) return 1;
        if (old == id) return 0;
        h = h + 1 == size ? 0u : h + 1;
    }
    return 2;
}

// Compact set (beam search, node ids < 2^24): 16-bit entries, exact.  A
// bijection x of the 24-bit id splits into a home slot (its low 13 bits) and a
// tag (its high 11 bits); the entry stores tag | disp << 11, disp = slot - home
// (linear probing without wrap, 0..30, over 8,192 + 32 slots).  Slot and entry
// together give back x, hence the id: a match is the id itself, never a false
// positive.  0xFFFF (tag 2047 with disp 31, which never occurs) is empty.  Two
// entries share a 32-bit LDS word; an insert is a CAS of the whole word.  It
// holds 8,192 ids in 16 KiB where the 32-bit set holds 5,120 in 20 KiB.
constexpr int VIS16_HOMES = 1 << 13;
constexpr int VIS16_SLOTS = VIS16_HOMES + 32;
constexpr int VIS16_WORDS = VIS16_SLOTS / 2;  // 32-bit words (16,448 B)
constexpr int VIS16_MAXD = 31;                // probes per id (disp 0..30)
__device__ __forceinline__ uint32_t vis16_mix(uint32_t id) {  // a bijection on [0, 2^24)
    uint32_t x = (id * 0x9E3779u) & 0xFFFFFFu;  // odd multiplier: invertible mod 2^24
    x ^= x >> 12;                                 // invertible xorshift
    return (x * 0x2C1B3Du) & 0xFFFFFFu;           // odd again
}
// 0 = already visited, 1 = newly recorded, 2 = congested (not recorded)
__device__ __forceinline__ int vis16_probe(uint32_t* tab, uint32_t id) {
    const uint32_t x = vis16_mix(id);
    const uint32_t home = x & (uint32_t)(VIS16_HOMES - 1), tag = x >> 13;
    uint32_t cur = 0xFFFFFFFFu;  // guess: the word is empty (the CAS returns it as it is)
#pragma unroll 1
    for (uint32_t d = 0; d < (uint32_t)VIS16_MAXD; ++d) {
        const uint32_t s = home + d;
        const uint32_t want = tag | (d << 11);
        const uint32_t sh = (s & 1u) << 4;
        uint32_t* w = tab + (s >> 1);
        if (d > 0 && !(s & 1u)) cur = 0xFFFFFFFFu;  // a new word: guess again (an odd slot's word is known)
#pragma unroll 1
        for (;;) {
            const uint32_t e = (cur >> sh) & 0xFFFFu;
            if (e == want) return 0;
            if (e != 0xFFFFu) break;  // another id's: the next slot
            const uint32_t nw = (cur & ~(0xFFFFu << sh)) | (want << sh);
            const uint32_t old = atomicCAS(w, cur, nw);
            if (old == cur) return 1;
            cur = old;  // the word held something else: look again
        }
    }
    return 2;
}

// ---------------------------------------------------------------------------
// sorted list across lanes: entry index i = r*64 + lane, ordered by (d, id)
// ---------------------------------------------------------------------------
template <int R>
struct BList {
    float d[R];
    uint32_t i[R];  // id | EXP_BIT when expanded; EMPTY_ID when empty
};

template <int R>
__device__ __forceinline__ void bl_init(BList<R>& L) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
        L.d[r] = __int_as_float(0x7f800000);
        L.i[r] = EMPTY_ID;
    }
}

template <int R>
__device__ __forceinline__ void bl_at(const BList<R>& L, int idx, float& d, uint32_t& id) {
    const int rr = idx >> 6, ll = idx & 63;
    d = __int_as_float(0x7f800000);
    id = EMPTY_ID;
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (r == rr) {
            d = rl_f(L.d[r], ll);
            id = rl_u(L.i[r], ll);
        }
}

// one-lane shift up across the wave (lane l gets lane l-1, lane 0 gets
// `in`): DPP wave_shr:1, no LDS permute on the list's insertion path
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v, uint32_t in) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)in, (int)v, 0x138, 0xf, 0xf, false);
}

// insert (d,u) keeping the best `ef` entries; returns true when inserted.
// Registers wholly before the insertion point keep their entries and
// registers past ef stay empty (uniform branches); the ones in between shift
// by one entry, highest first so that each reads its predecessor's last lane
// before that register moves.
template <int R>
__device__ __forceinline__ bool bl_insert(BList<R>& L, int ef, float d, uint32_t u) {
    if (!(d == d)) return false;  // NaN never enters the list
    float wd;
    uint32_t wi;
    bl_at(L, ef - 1, wd, wi);
    if (!lt_di(d, u, wd, wi & ID_MASK)) return false;
    bool dup = false;
#pragma unroll
    for (int r = 0; r < R; ++r) dup |= ((L.i[r] & ID_MASK) == u);
    if (__ballot(dup)) return false;
    int pos = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) pos += __popcll(__ballot(lt_di(L.d[r], L.i[r] & ID_MASK, d, u)));
    const int lane = lane_id();
#pragma unroll
    for (int r = R - 1; r >= 0; --r) {
        if (r * 64 >= ef) continue;   // empty, stays empty
        if (r * 64 + 63 < pos) break;  // this register and the ones below are unchanged
        const uint32_t cd = r > 0 ? rl_u(__float_as_uint(L.d[r > 0 ? r - 1 : 0]), 63) : 0u;
        const uint32_t ci = r > 0 ? rl_u(L.i[r > 0 ? r - 1 : 0], 63) : EMPTY_ID;
        const float sd = __uint_as_float(wave_shr1(__float_as_uint(L.d[r]), cd));
        const uint32_t si = wave_shr1(L.i[r], ci);
        const int idx = r * 64 + lane;
        if (idx > pos) {
            L.d[r] = sd;
            L.i[r] = si;
        } else if (idx == pos) {
            L.d[r] = d;
            L.i[r] = u;
        }
        if (idx >= ef) {
            L.d[r] = __int_as_float(0x7f800000);
            L.i[r] = EMPTY_ID;
        }
    }
    return true;
}

// pick the first unexpanded entry, mark it expanded; returns EMPTY_ID if none
template <int R>
__device__ __forceinline__ uint32_t bl_next(BList<R>& L) {
    const int lane = lane_id();
    int sel_r = -1, sel_l = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        unsigned long long m = __ballot(((L.i[r] & EXP_BIT) == 0) && (L.i[r] != EMPTY_ID));
        if (sel_r < 0 && m) {
            sel_r = r;
            sel_l = __ffsll((long long)m) - 1;
        }
    }
    if (sel_r < 0) return EMPTY_ID;
    uint32_t id = EMPTY_ID;
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (r == sel_r) {
            id = rl_u(L.i[r], sel_l);
            if (lane == sel_l) L.i[r] |= EXP_BIT;
        }
    return id;
}

// ---------------------------------------------------------------------------
// Go container/heap on LDS arrays (heap/heap.go + container/heap), executed
// identically by every lane (uniform control flow, same-address LDS traffic).
// ---------------------------------------------------------------------------
struct GHeap {
    float* d;
    uint32_t* id;
    int n;
};

__device__ __forceinline__ bool gh_less(const GHeap& h, int i, int j) { return h.d[i] < h.d[j]; }
__device__ __forceinline__ void gh_swap(GHeap& h, int i, int j) {
    float td = h.d[i];
    uint32_t ti = h.id[i];
    float jd = h.d[j];
    uint32_t ji = h.id[j];
    h.d[i] = jd;
    h.id[i] = ji;
    h.d[j] = td;
    h.id[j] = ti;
}
__device__ __forceinline__ void gh_up(GHeap& h, int j) {
    for (;;) {
        int i = (j - 1) / 2;
        if (i == j || !gh_less(h, j, i)) break;
        gh_swap(h, i, j);
        j = i;
    }
}
__device__ __forceinline__ bool gh_down(GHeap& h, int i0, int n) {
    int i = i0;
    for (;;) {
        int j1 = 2 * i + 1;
        if (j1 >= n || j1 < 0) break;
        int j = j1;
        int j2 = j1 + 1;
        if (j2 < n && gh_less(h, j2, j1)) j = j2;
        if (!gh_less(h, j, i)) break;
        gh_swap(h, i, j);
        i = j;
    }
    return i > i0;
}
__device__ __forceinline__ void gh_push(GHeap& h, float d, uint32_t id) {
    h.d[h.n] = d;
    h.id[h.n] = id;
    h.n++;
    gh_up(h, h.n - 1);
}
__device__ __forceinline__ void gh_pop(GHeap& h, float& d, uint32_t& id) {
    int n = h.n - 1;
    gh_swap(h, 0, n);
    gh_down(h, 0, n);
    h.n--;
    d = h.d[h.n];
    id = h.id[h.n];
}
// PopLast == Remove(Len()-1): i == n, no swap (heap/heap.go:73-81)
__device__ __forceinline__ void gh_poplast(GHeap& h) { h.n--; }

// The same heap with slot i in lane i (capacity 64), for the compat walks'
// small heaps (ef + 1 and k + 1 entries): the sift loops run on readlane /
// writelane instead of dependent LDS round trips.  Sifts move a hole instead
// of swapping; the slots end up exactly where Go's swap loops put them.
struct RHeap {
    float d = 0.f;
    uint32_t id = 0u;
    int n = 0;
};
__device__ __forceinline__ void rh_set(RHeap& h, int j, float d, uint32_t id) {
    const bool me = lane_id() == j;  // (no writelane builtin in this compiler: compare + select)
    h.d = me ? d : h.d;
    h.id = me ? id : h.id;
}
// element (xd, xi) entering at slot j, moved up (heap.go up: Less(j, parent))
__device__ __forceinline__ void rh_up(RHeap& h, int j, float xd, uint32_t xi) {
    while (j > 0) {
        const int p = (j - 1) / 2;
        const float pd = rl_f(h.d, p);
        if (!(xd < pd)) break;
        rh_set(h, j, pd, rl_u(h.id, p));
        j = p;
    }
    rh_set(h, j, xd, xi);
}
// element (xd, xi) at slot i, moved down within [0, n) (heap.go down)
__device__ __forceinline__ void rh_down(RHeap& h, int i, int n, float xd, uint32_t xi) {
    for (;;) {
        const int j1 = 2 * i + 1;
        if (j1 >= n) break;
        int j = j1;
        float jd = rl_f(h.d, j1);
        if (j1 + 1 < n) {
            const float d2 = rl_f(h.d, j1 + 1);
            if (d2 < jd) {
                j = j1 + 1;
                jd = d2;
            }
        }
        if (!(jd < xd)) break;
        rh_set(h, i, jd, rl_u(h.id, j));
        i = j;
    }
    rh_set(h, i, xd, xi);
}

// one interface over both heaps (compat_layer is written against it)
__device__ __forceinline__ void hp_push(GHeap& h, float d, uint32_t id) { gh_push(h, d, id); }
__device__ __forceinline__ void hp_pop(GHeap& h, float& d, uint32_t& id) { gh_pop(h, d, id); }
__device__ __forceinline__ void hp_poplast(GHeap& h) { h.n--; }
__device__ __forceinline__ float hp_d(const GHeap& h, int i) { return h.d[i]; }
__device__ __forceinline__ uint32_t hp_id(const GHeap& h, int i) { return h.id[i]; }
__device__ __forceinline__ void hp_store(const GHeap&, float*, uint32_t*) {}  // already in place
__device__ __forceinline__ void hp_push(RHeap& h, float d, uint32_t id) {
    rh_up(h, h.n, d, id);
    h.n++;
}
__device__ __forceinline__ void hp_pop(RHeap& h, float& d, uint32_t& id) {
    const int n1 = h.n - 1;
    d = rl_f(h.d, 0);
    id = rl_u(h.id, 0);
    if (n1 > 0) rh_down(h, 0, n1, rl_f(h.d, n1), rl_u(h.id, n1));
    h.n = n1;
}
__device__ __forceinline__ void hp_poplast(RHeap& h) { h.n--; }
__device__ __forceinline__ float hp_d(const RHeap& h, int i) { return rl_f(h.d, i); }
__device__ __forceinline__ uint32_t hp_id(const RHeap& h, int i) { return rl_u(h.id, i); }
__device__ __forceinline__ void hp_store(const RHeap& h, float* d, uint32_t* id) {
    if (lane_id() < h.n) {
        d[lane_id()] = h.d;
        id[lane_id()] = h.id;
    }
}

// ---------------------------------------------------------------------------
// Ascending (key, id) order of lanes 0..cnt-1 (cnt uniform, <= 64; lanes >= cnt
// keep their values): each lane counts the entries before it -- cnt uniform
// readlanes, no cross-lane latency chain -- and one permute scatters them.
// Equal pairs (duplicate entries) keep lane order.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void rank_sort(int64_t& key, uint32_t& id, int cnt) {
    const int lane = lane_id();
    const uint32_t klo = (uint32_t)(uint64_t)key, khi = (uint32_t)((uint64_t)key >> 32);
    int r = 0;
#pragma unroll 8
    for (int j = 0; j < cnt; ++j) {
        const int64_t kj = (int64_t)(((uint64_t)rl_u(khi, j) << 32) | rl_u(klo, j));
        const uint32_t ij = rl_u(id, j);
        r += (kj < key || (kj == key && (ij < id || (ij == id && j < lane)))) ? 1 : 0;
    }
    const int dst = lane < cnt ? r : lane;
    const uint32_t nlo = push_to(klo, dst), nhi = push_to(khi, dst);
    id = push_to(id, dst);
    key = (int64_t)(((uint64_t)nhi << 32) | nlo);
}

// Tools-only cycle accounting of the compat walk (tools/Makefile.build with
// BFLAGS=-DMH_COMPAT_PROF): per-phase clock deltas summed in LDS by the walking
// wave and printed by the kernel at exit.  Compiled out of the product.
#ifdef MH_COMPAT_PROF
__shared__ unsigned long long mh_cprof[24];
#define CPROF_T(v) long long v = clock64()
#define CPROF_ADD(v, s)                                                                 \
    do {                                                                                \
        const long long n_ = clock64();                                                 \
        if (lane_id() == 0) atomicAdd(&mh_cprof[s], (unsigned long long)(n_ - (v)));    \
        v = n_;                                                                         \
    } while (0)
#define CPROF_CNT(s, x)                                                                 \
    do {                                                                                \
        if (lane_id() == 0) atomicAdd(&mh_cprof[s], (unsigned long long)(x));           \
    } while (0)
#else
#define CPROF_T(v)
#define CPROF_ADD(v, s)
#define CPROF_CNT(s, x)
#endif

}  // namespace mh
