// engine.hpp -- host-side launch interface between the C ABI (api.cpp) and the
// HIP kernels (search.hip, build.hip, exact.hip).  No torch types anywhere.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.hpp"

namespace mh {

// supported dimension configurations (lanes per row, float4 per lane)
struct DimCfgId {
    int lpr, vpl;
};
inline bool pick_cfg(int dim, int& lpr, int& vpl) {
    if (dim <= 0) return false;
    if (dim <= 64) { lpr = 16; vpl = 1; return true; }
    if (dim <= 128) { lpr = 32; vpl = 1; return true; }
    if (dim <= 256) { lpr = 64; vpl = 1; return true; }
    if (dim <= 512) { lpr = 64; vpl = 2; return true; }
    if (dim <= 768) { lpr = 64; vpl = 3; return true; }
    if (dim <= 1024) { lpr = 64; vpl = 4; return true; }
    if (dim <= 1536) { lpr = 64; vpl = 6; return true; }
    if (dim <= 2048) { lpr = 64; vpl = 8; return true; }
    if (dim <= 3072) { lpr = 64; vpl = 12; return true; }
    if (dim <= 4096) { lpr = 64; vpl = 16; return true; }
    return false;
}
inline int pitch_of(int lpr, int vpl) { return lpr * 4 * vpl; }

struct SearchArgs {
    GraphDev g;
    const float* q;  // padded queries [B * pitch]
    int64_t B;
    int k, ef, top;
    uint32_t entry;               // top-layer entry (internal id)
    const int32_t* layer_entry;   // [nlayers] policy entry per layer (compat)
    int64_t* out_keys;            // [B*k]
    float* out_dist;              // [B*k]
    int32_t* out_n;               // [B]
    int32_t* out_ids;             // [B*k] internal ids (nullable)
    unsigned long long* stats;    // [0]=dist evals [1]=expansions [2]=visited resets
                                  // [8]=rows screened in fp16 [9]=rows evaluated in f32 (beam)
    int* err;                     // set to nonzero on visited overflow (compat)
    int vis_log2;                 // compat: 2^vis_log2-entry visited set
    int vis_n;                    // beam: visited-set entries (the LDS it takes: 4 * vis_n bytes per wave)
    int vis16 = 0;                // beam: the compact 16-bit set in that LDS instead (ids < 2^24)
    int upper_ef;                 // beam: width of the upper-layer descent (1 = greedy, the reference's k = 1)
    int64_t mw_max_b;             // beam: batches up to this size run a workgroup per query (0 = never)
    int expand = 1;               // beam: entries expanded per layer-0 step (1, 2 or 4; beam_layer XW)
};

// negative-example re-ranking epilogue (graph.go:1116-1537)
struct NegArgs {
    GraphDev g;
    const float* neg;          // padded negative rows [total * pitch]
    const int32_t* neg_off;    // [B + 1] row offsets of each query's negatives
    const int32_t* cand_ids;   // [B * kx] Search(near, kx) internal ids
    const float* cand_d;       // [B * kx] their distances to the query
    const int32_t* cand_n;     // [B]
    int64_t B;
    int kx, k;
    float w;
    int flags;                 // bit 0: the reference's key 7..9 boost (test hack)
    int64_t* out_keys;         // [B * k]
    float* out_score;          // [B * k]
    int32_t* out_n;            // [B]
};
constexpr int NEG_MAX_CAND = 256;
int launch_negatives(const NegArgs& a, int lpr, int vpl, hipStream_t s);

int launch_pad_rows(const float* src, int64_t n, int dim, float* dst, int pitch, hipStream_t s);
int launch_scatter_rows(const float* src, const int32_t* ids, int64_t n, int pitch, float* dst, hipStream_t s);
// err: running max of the rows' measured relative rounding (GraphDev::h16err)
int launch_h16_rows(const float* X, const float* norms, int64_t n0, int64_t n1, int pitch, int metric, uint16_t* H,
                    float2* aux, float* err, hipStream_t s);
int launch_norms(const float* X, int64_t n0, int64_t n1, int pitch, int lpr, int vpl, float* out, hipStream_t s);
int launch_sweep(const float* q, const float* X, int64_t n, int pitch, int lpr, int vpl, int metric, float* out,
                 hipStream_t s);
int launch_sweep_raw(const float* q, const float* X, int64_t n, int dim, int metric, float* out, hipStream_t s);
int launch_search_beam(const SearchArgs& a, int lpr, int vpl, hipStream_t s);
int launch_search_compat(const SearchArgs& a, int lpr, int vpl, hipStream_t s);

// ---- build ----
struct CompatBuildArgs {
    GraphDev g;
    int64_t n0, n1;               // insert internal ids [n0, n1) in order
    const int32_t* levels;        // [cap_nodes] level of each node
    const int32_t* layer_entry;   // [MH_MAXL] first node id of each layer (-1 none)
    int top0;                     // len(g.layers) - 1 before this batch (-1: no layers)
    int M, ef;
    unsigned long long* stats;    // [0]=dist evals [1]=expansions
    int* err;                     // [0] error bits; on "no nodes found" (bit 2): [2] layer, [3] row
    int vis_log2;
    // BatchAdd of a present key (graph.go:1015-1024), after the fresh inserts:
    int rep_level;                // its level (-1: none)
    int rep_i0;                   // the layer whose search precedes the sweep
    uint32_t rep_a, rep_b;        // its rows above i0 (EMPTY_ID: none needed) / from i0 down
    const int32_t* rep_entry;     // [MH_MAXL] entry() of each layer at its turn (the row itself: empty then)
    const int32_t* rep_sweep;     // [MH_MAXL] row the sweep deletes + isolates in layer l (-1 none)
    int spec;                     // set by the launch: the eviction-staging area fits in LDS
};
int launch_build_compat(const CompatBuildArgs& a, int lpr, int vpl, int waves, hipStream_t s);  // waves: 1 or 8

// ---- delete (graph.go:843-895) ----
struct DeleteArgs {
    GraphDev g;
    const uint32_t* ids;          // compat: internal ids in BatchDelete order ...
    const uint32_t* lay;          // ... each isolated in layer lay[i] only (graph.go:852-861 walks a key's
                                  //     layers; a key's nodes can be several rows in disjoint layers)
    int64_t nids;
    int64_t n;                    // repair: rows [0, n)
    int layer;                    // repair: layer being repaired
    int M;                        // compat: the reference's cap (M on every layer)
    int mcap;                     // repair: row cap of this layer
    int heuristic, keep_pruned;   // repair: selection rule (as the batched insert)
    unsigned long long* stats;    // [0]=dist evals
    int* err;
    int vis_log2;
};
constexpr int REPAIR_POOL = 256;  // candidate pool per repaired row (oracle: OG_REPAIR_POOL)
int launch_delete_compat(const DeleteArgs& a, int lpr, int vpl, hipStream_t s);
int launch_delete_repair(const DeleteArgs& a, int lpr, int vpl, hipStream_t s);

struct BatchBuildArgs {
    GraphDev g;
    int layer;
    int64_t n0, n1;               // batch of new internal ids
    const int32_t* levels;
    uint32_t* cur_entry;          // [cap_nodes] per-node descent entry (in/out)
    int ef;                       // efConstruction
    int mcap;                     // neighbors to select on this layer
    int heuristic;                // 0 closest-M, 1 HNSW heuristic on the new row, 2 also on overflowing rows
    int keep_pruned;              // fill the new row with pruned candidates up to mcap
    int expand;                   // entries expanded per step of the layer search (1 or 2; beam_layer XW)
    float alpha;                  // diversity slack: drop c when alpha * d(c, kept) < d(u, c) (1 = HNSW Alg. 4)
    int32_t* inc_cnt;             // [cap_nodes] incoming request counters (zero between batches)
    uint32_t* inc_src;            // [cap_nodes * inc_cap]
    float* inc_dist;              // [cap_nodes * inc_cap]
    int inc_cap;
    uint32_t* touched;            // [batch * mcap]
    int32_t* touched_cnt;         // [1]
    unsigned long long* stats;    // [0]=dist evals [1]=expansions [2]=dropped requests
    int vis_log2;
    const uint32_t* order;        // nullable: node of workgroup b is order[b] (b < count), nodes sorted by
    int64_t count;                //   level descending so that level >= layer is a prefix
    int64_t mw_max = 0;           // launches of at most this many inserts: one workgroup of 4 waves per insert
    int vis16 = 0;                // the layer searches' visited set is the compact 16-bit one (ids < 2^24)
};
int launch_build_batch_search(const BatchBuildArgs& a, int lpr, int vpl, hipStream_t s);
// greedy descent of every node u in [n0, n1) through layers a.layer .. levels[u] + 1
int launch_build_batch_descend(const BatchBuildArgs& a, int lpr, int vpl, hipStream_t s);
int launch_build_batch_commit(const BatchBuildArgs& a, int lpr, int vpl, int64_t n_touched, hipStream_t s);

// ---- exact / merge ----
// Brute-force path: approximate scores on MFMA (f32-input, or the bf16x3 split
// hi*hi + hi*lo + lo*hi), top-kk preselection, canonical re-rank of the kk,
// then a per-query certificate that no row outside the kk can belong to the
// canonical top-k; uncertified queries are redone by a full canonical sweep.
struct ExactArgs {
    const float* X;       // [N * pitch]
    const float* xnorm;   // [N]
    const uint8_t* dead;  // [N] 1 = deleted row (nullable)
    int64_t N;
    const float* Q;       // [B * pitch]
    const float* qnorm;   // [B] canonical |q|
    int64_t B;
    int pitch, dim, metric;
    float* scores;        // [B * ldS] workspace
    int64_t ldS;          // row stride of scores (multiple of 4, >= N)
    int kk;               // preselect width (<= 64)
    uint32_t* cand;       // [B * kk]
    float* bound;         // [B] k_select: kk-th preselected score (+inf when fewer)
    int nseg;             // k_select: row segments per query (<= 16), each seglen rows (multiple of 1024)
    int64_t seglen;
    float* seg_d;         // [B * nseg * kk] per-segment best scores / ids
    uint32_t* seg_i;
    const uint8_t* only;  // k_select: skip rows b with only[b] == 0 (nullable)
    const uint16_t* Xh;   // split mode: bf16 hi / lo planes of X, K-blocked (k_split_rows)
    const uint16_t* Xl;
    int64_t ldXs;         // rows per K-block of the X planes
    const uint16_t* Qh;   // split mode: bf16 hi / lo planes of Q, K-blocked
    const uint16_t* Ql;
    int64_t ldQs;
    const float* xinv;    // fp16 2-product mode: per-row / per-query unscale 2^-e (NaN: outside the bound)
    const float* qinv;
    // fp16 1-product ring (exact_precision 3)
    int tile_stride;          // sample pass: score every tile_stride-th row tile (1: every tile)
    int64_t nsample_tiles;    // ... how many (compact columns [0, nsample_tiles * BN) of scores)
    const float* ring_c;      // [>= roundup(B, 256)] filter constants (k_ring_prep; +inf pads)
    const float* ring_s;      // [same] L2: 1 / qi
    uint2* region;            // [tiles * rcap] passing pairs {row off | query off << 16, acc}
    int32_t* region_cnt;      // [tiles] pairs per tile (may exceed rcap: overflow)
    int rcap;                 // entries per tile region
    const float4* xw;         // [N] k_h1_pp: per-row filter constants (k_h1_rowconst)
};
int launch_exact_scores(const ExactArgs& a, hipStream_t s);     // f32-input MFMA
int launch_exact_scores_x3(const ExactArgs& a, int tile, hipStream_t s);  // bf16x3 split MFMA
// fp16 2-product split: (qh + ql) . xh on v_mfma_f32_32x32x16_f16 (Xl unused)
int launch_exact_scores_x2h(const ExactArgs& a, int tile, hipStream_t s);
// fp16 1-product ring: every score of the sampled row tiles, or the fused filter into regions
int launch_h1_sample(const ExactArgs& a, int variant, hipStream_t s);
int launch_h1_filter(const ExactArgs& a, int variant, hipStream_t s);
constexpr int H1_BN = 256;   // row tile of every launch_h1_* variant
constexpr int H1_BSUB = 16;     // sub-buckets per query (k_bucket)
constexpr int H1_CSTRIDE = 32;  // sub-bucket counters one 128-B line apart (no same-line atomics)
constexpr int H1_REC = 10;      // uint2 per record of the record-mode filter: {mb | lane << 8, 0}, pad, 16 accumulators
int h1_tile_bm(int variant);  // query tile of a variant (128 or 256)
bool h1_timing_diag(int variant);   // exact_tile 7-9, 11-13, 15-17, 19-20: timing diagnostics (no results)
int h1_region_split(int variant);   // regions per tile of the fused filter (rcap is split evenly)
bool h1_records(int variant);       // the variant's regions hold records (k_h1_pp16 REC), not pairs
int h1_effective_variant(int variant, int pitch, int64_t ld);  // the variant a search runs (0 -> default)
int launch_h1_rowconst(const float* xinv, const float* xnorm, const uint8_t* dead, int64_t n, int metric, float4* xw,
                       hipStream_t s);
int launch_ring_prep(const float* thr, const float* qnorm, const float* qinv, int64_t B, int metric, float* c,
                     float* sq, hipStream_t s);
// qcnt [B * H1_BSUB * H1_CSTRIDE], bucket [B * H1_BSUB * scap]
int launch_bucket(const uint2* region, const int32_t* region_cnt, int rcap, int64_t ntiles, int64_t nqt, int BM,
                  int BN, int64_t B, int32_t* qcnt, uint2* bucket, int scap, uint8_t* qovf, int rsub, int rec,
                  const ExactArgs& a, hipStream_t s);
int launch_select_bucket(const ExactArgs& a, const int32_t* qcnt, const uint2* bucket, int scap, const uint8_t* qovf,
                         const float* thr, hipStream_t s);
// err (nullable): running max of the rows' relative fp16 rounding |x' - x| / |x|
int launch_split_h16(const float* src, int64_t r0, int64_t r1, int pitch, int64_t rows, uint16_t* hi, uint16_t* lo,
                     float* inv, float* err, hipStream_t s);
int launch_exact_select(const ExactArgs& a, hipStream_t s);
int launch_split_rows(const float* src, int64_t r0, int64_t r1, int pitch, int64_t rows, uint16_t* hi, uint16_t* lo,
                      hipStream_t s);
int launch_max_norm(const float* norms, int64_t n, float* out, hipStream_t s);

// certificate of the re-rank (nullable pieces disable it)
struct CertArgs {
    const float* bound;          // [B] from k_select; nullptr = no certificate
    const float* qnorm;          // [B]
    const float* xmax;           // [1] largest row norm (L2)
    float eps_cos;               // cosine: |approx - canonical| distance bound
    float eps_dot, c_l2;         // L2: 2*eps_dot*|q|*xmax + c_l2*(|q|+xmax)^2 bounds |approx - canonical^2|
    uint8_t* flag;               // [B] out: 1 = not certified
    int32_t* flagged;            // [B] out: list of uncertified rows
    int32_t* nflag;              // [1] out: list length
    unsigned long long* stats;   // [0] += uncertified queries
    const uint8_t* only;         // re-rank only rows with only[b] != 0 (nullable)
    const float* xerr;           // fp16 2-product scores: max relative row rounding, added to the bound (nullable)
    const float* qerr;           // fp16 1-product scores: max relative query rounding of the batch (nullable)
};
int launch_rerank(const float* Q, const GraphDev& g, const uint32_t* cand, int kk, int64_t B, int lpr, int vpl, int k,
                  int64_t* out_keys, float* out_dist, int32_t* out_n, int32_t* out_ids, const CertArgs& c,
                  hipStream_t s);
// canonical distances of every row for the flagged queries (overwrites their score rows)
int launch_exact_fallback(const float* Q, const GraphDev& g, int64_t N, const int32_t* flagged, const int32_t* nflag,
                          float* scores, int64_t ldS, int lpr, int vpl, hipStream_t s);

// the fused path's fallback: canonical distances of every row streamed into per-segment
// top-kk lists (a.seg_d / a.seg_i, k_select's layout) for the queries a.only flags, then
// k_select_merge -> a.cand, a.bound (no score matrix)
int launch_fallback_select(const float* Q, const GraphDev& g, const ExactArgs& a, int lpr, int vpl, hipStream_t s);
int launch_merge_topk(const int64_t* keys_in, const float* dist_in, const int32_t* n_in, int shards, int64_t B,
                      int k, int64_t* out_keys, float* out_dist, int32_t* out_n, hipStream_t s);

}  // namespace mh
