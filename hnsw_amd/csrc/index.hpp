// index.hpp -- the engine's per-handle host state (struct mhnsw_index) and the
// host helpers shared by the C ABI's translation units: api.cpp (lifecycle,
// options, Add / Delete / build scheduling), search_host.cpp (search and
// exact-path orchestration), io_host.cpp (export / import, encode.go format,
// string keys).  Host only: no device code here.
#pragma once
#include <hip/hip_runtime.h>

#include <errno.h>
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <functional>
#include <unordered_map>
#include <vector>

#include "../../include/mhnsw.h"
#include "codec.hpp"
#include "engine.hpp"

using namespace mh;

namespace mhh {

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
};

struct Layer {
    int32_t* deg = nullptr;
    int32_t* adj = nullptr;
    float* adjd = nullptr;
    int cap = 0;
    int64_t count = 0;
    int32_t entry = -1;
};

}  // namespace mhh

using mhh::DevBuf;
using mhh::Layer;

struct mhnsw_index {
    // public fields (graph.go:305-326)
    int metric = COSINE;
    int M = 16;
    double ml = 0.25;
    int ef = 20;
    uint64_t rng = 0;
    // engine options
    int build_mode = MHNSW_BUILD_COMPAT;
    int m0 = 0;  // 0 => 2*M in batch mode, M in compat mode
    int efc = 0; // 0 => EfSearch
    int heuristic = 1;
    int keep_pruned = 0;
    int build_expand = 4;     // batched insert: entries expanded per step of its layer searches (1-4)
    int upper_efc = 0;        // batched insert: candidate list of the layers above 0 (0 = efConstruction)
    int search_expand = 1;    // beam search: entries expanded per layer-0 step (1, 2, 4; 1 = standard)
    int alpha_pct = 100;
    int batch_min = 1, batch_max = 65536, batch_ratio_pct = 5;
    int vis_log2 = 12;
    int vis_entries = 0;      // beam search's visited set; 0 = 1.25 * 2^vis_log2 (beam_vis_entries)
    int vis_compact = 1;      // beam search: the compact 16-bit visited set when ids < 2^24 and it fits
    int exact_kk = 0;
    int exact_sample = 64;   // fused preselection: row tiles in the threshold sample (at most; stride = ceil(tiles / this))
    int exact_thr_rank = 0;  // fused preselection: the sample's J-th best is the threshold (0 = max(k, kk / 8))
    int exact_precision = 3;  // scores: 0 f32-input MFMA, 1 bf16x3 split, 2 fp16 2-product split,
                              // 3 fp16 1-product with the fused preselection (all certified, same results)
    int exact_tile = 0;       // GEMM variant (exact.hip: launch_split_scores, launch_h1)
    int compat_waves = 8;     // compat insert: waves scoring each distance batch (1 = the walking wave alone)
    int upper_ef = 1;         // beam search: upper-layer descent width
    int64_t beam_mw_max_b = 512;  // beam search: batches up to this size run one workgroup of 4 waves per query
    int64_t build_mw_max = 256;   // batched insert: launches of at most this many inserts run 4 waves per insert
    int screen = 1;           // beam search / batched insert fp16 screening copy (results unchanged)
    int fuse_descent = 1;     // batched insert: all greedy descents of a batch in one launch (same graph)
    int time_build = 0;       // batched insert: time its search kernels with HIP events (stats [12])
    int64_t max_rows = 0;     // row capacity limit (0 = none): an Add past it fails with MHNSW_ENOMEM, index unchanged
    std::vector<hipEvent_t> tev;  // event pairs around the timed launches of the current Add
    size_t tev_used = 0;
    double build_search_us = 0;
    // shape
    int dim = 0, pitch = 0, lpr = 0, vpl = 0;
    bool layers_exist = false;
    int64_t n = 0, capn = 0;
    int device = 0;
    hipStream_t stream = nullptr;
    // device state
    float* vecs = nullptr;
    float* norms = nullptr;
    uint16_t* h16 = nullptr;  // fp16 screening copy [capn * pitch] (screen = 1)
    float2* h16aux = nullptr;  // [capn] L2 screening {unscale, |x|}
    int h16_metric = -1;       // metric the copies were written for
    float* h16err = nullptr;   // [1] the copy's measured max relative rounding (screening margin)
    int64_t* keys = nullptr;
    int32_t* levels = nullptr;
    uint8_t* dead = nullptr;  // [capn] deleted rows (graph.go:843-864)
    bool any_dead = false;
    // key identity (compat; GraphDev::kid): allocated at the first replaced or re-added key
    int32_t* kid = nullptr;      // [capn] first row that held the row's key
    int32_t* kidlive = nullptr;  // [capn] by kid: the key's newest live row (-1 none)
    int32_t* kprev = nullptr;    // [capn] the next older live row of the same key (-1 none; GraphDev::kprev)
    bool aliased = false;
    uint32_t* cur_entry = nullptr;
    int32_t* inc_cnt = nullptr;
    uint32_t* inc_src = nullptr;
    float* inc_dist = nullptr;
    int inc_cap = 64;
    uint32_t* touched = nullptr;
    size_t touched_cap = 0;
    int32_t* touched_cnt = nullptr;
    int32_t* d_layer_entry = nullptr;
    LayerDev* d_layers = nullptr;
    LayerDev layers_host[MH_MAXL] = {};
    unsigned long long* d_stats = nullptr;
    // d_err[0]: error word of the current synchronous call (zeroed per call);
    // d_err[1]: sticky word of *_device searches, which return before their
    // kernels run -- read and cleared by mhnsw_device_status
    int* d_err = nullptr;
    std::vector<mhh::Layer> layers;
    // scratch
    DevBuf<float> qpad, qnorm, scores, tmp;
    DevBuf<uint32_t> cand;
    DevBuf<uint32_t> border;           // batched insert: batch nodes by level, descending
    uint32_t* ord_pin = nullptr;       // ... staged in pinned memory
    int64_t ord_cap = 0;
    hipEvent_t ord_ev = nullptr;       // the staging copy has been consumed
    bool ord_pending = false;
    DevBuf<int64_t> okeys;
    DevBuf<float> odist;
    DevBuf<int32_t> on;
    DevBuf<float> nq, nneg, ncd;  // negatives: queries, padded negative rows, candidate distances
    DevBuf<int64_t> nck, nok;
    DevBuf<int32_t> ncn, nci, noff, non;
    DevBuf<float> nos;
    // exact path: cached bf16 hi/lo planes of the first xsplit_rows rows (rows are
    // immutable once added; import resets), per-chunk query planes, certificate state
    DevBuf<uint16_t> xsplit, qsplit;
    int64_t xsplit_rows = 0, xsplit_plane = 0;  // rows converted; plane stride they were written with
    int xsplit_kind = 0;                        // 1: bf16 hi/lo planes, 2: fp16 hi plane + xinv (exact_precision)
    DevBuf<float> xinv, qinv;                   // exact_precision 2: per-row / per-query unscale
    DevBuf<float> xerr;                         // ... and the rows' max relative fp16 rounding
    // exact_precision 3 (fp16 1-product, fused preselection): sample thresholds,
    // filter constants, tile regions + counts, per-query buckets, the queries' rounding
    DevBuf<float> h1thr, h1c, h1s, qerr;
    DevBuf<float> h1xw;  // [4 capn] per-row filter constants of k_h1_pp16 (k_h1_rowconst)
    DevBuf<uint2> h1region, h1bucket;
    DevBuf<int32_t> h1rcnt, h1qcnt;
    DevBuf<uint8_t> h1ovf;
    DevBuf<float> xbound, xmaxn, xsegd;
    DevBuf<uint32_t> xsegi;
    DevBuf<uint8_t> xflag;
    DevBuf<uint8_t> xgone;     // exact path: rows to skip when some live row is not in layer 0
    int64_t add_reached = 0;   // inserts the last Add's walk reached (mhnsw_add_reached)
    int64_t partial_rows = 0;  // rows neither deleted nor in layer 0 (left by failed inserts, graph.go:1009)
    uint64_t mut_epoch = 0;            // bumped by every Add / Delete / Import: row membership may have changed
    uint64_t xgone_epoch = ~0ull;      // the epoch xgone was built at
    DevBuf<int32_t> xflagged, xnflag;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t gev0 = nullptr, gev1 = nullptr;  // the exact path's score GEMM (first query chunk)
    bool have_gemm_timing = false;
    // cross-stream ordering: a *_device search returns once enqueued on the
    // caller's stream; the next call on another stream (or a mutation) must
    // not reuse scratch / rewrite the graph under it
    hipEvent_t scr_ev = nullptr, meta_ev = nullptr;
    hipStream_t scr_stream = nullptr;
    bool scr_valid = false;
    bool have_timing = false;
    // host mirrors
    std::unordered_map<int64_t, int32_t> key2id;  // live keys only
    // Go string keys (Graph[string]): order-maintenance labels -- every string
    // ever added maps to an int64 label in lexicographic order, so the engine's
    // key comparisons (compat expansion order, tie-breaks) see the string order
    std::map<std::string, int64_t> s2l;
    std::unordered_map<int64_t, std::string> l2s;
    int64_t relabels = 0;
    std::vector<int32_t> hlevels;
    std::vector<uint32_t> hmask;  // bit l: row is in layer l (compat may promote into emptied layers)
    std::vector<uint8_t> hdead;
    std::vector<int32_t> hkid;                       // kid mirror (aliased only)
    std::vector<int32_t> hprev;                      // kprev mirror (aliased only)
    std::unordered_map<int64_t, int32_t> dead_kid;   // deleted keys -> kid, for a later re-add
    int64_t stats_host[8] = {0};
    std::string err;
    mutable std::shared_mutex mu;
};

namespace mhh {

extern thread_local std::string g_create_err;

#define HIPCHK(h, x)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) return fail(h, MHNSW_EDEVICE, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)

#define LCHK(h, x)                                                              \
    do {                                                                        \
        int r_ = (x);                                                           \
        if (r_ != 0) return fail(h, r_ == -4 ? MHNSW_EUNSUPPORTED : MHNSW_EDEVICE, "kernel launch failed (%d) at %s", r_, #x); \
    } while (0)

int fail(mhnsw_index* h, int code, const char* fmt, ...);
int validate(mhnsw_index* h);
int max_level(double ml, int64_t num);
double rng_next(uint64_t* s);
int random_level(double ml, bool layers_exist, int64_t count, uint64_t* rng);
int m0_of(const mhnsw_index* h);
int cap_of(const mhnsw_index* h, int l);
int ensure_layer(mhnsw_index* h, int l);
int ensure_caps(mhnsw_index* h);
int ensure_capacity(mhnsw_index* h, int64_t need);
int sync_layer_table(mhnsw_index* h);
GraphDev graph_view(const mhnsw_index* h);
int64_t live_count(const mhnsw_index* h);
int top_live_layer(const mhnsw_index* h);
bool in_layer(const mhnsw_index* h, int64_t id, int l);
void fix_entries(mhnsw_index* h);
int set_shape(mhnsw_index* h, int dim);
int set_deg(mhnsw_index* h, int l, int64_t id, int32_t v);
int sync_layer_entries(mhnsw_index* h);
int zero_err(mhnsw_index* h);
int run_batch_layers(mhnsw_index* h, int64_t a0, int64_t a1, int top, uint32_t entry);
int run_build_batch(mhnsw_index* h, int64_t n0, int64_t n1, int top, uint32_t entry,
                    const std::function<void()>& while_gpu = nullptr);
int h16_rows(mhnsw_index* h, int64_t r0, int64_t r1);
int32_t kid_of_row(const mhnsw_index* h, int64_t r);
int set_kidlive(mhnsw_index* h, int32_t kid, int32_t row);
int start_alias(mhnsw_index* h);
void forget_key(mhnsw_index* h, int64_t key, int32_t row);
std::vector<int32_t> key_rows(const mhnsw_index* h, int64_t key);
int32_t key_row_in(const mhnsw_index* h, int64_t key, int l);
int add_step(mhnsw_index* h, const int64_t* keys, const float* vecs, bool vecs_on_device, int64_t n, int dim, const int32_t* levels, int64_t* reached, int64_t* cont_out);
int add_impl(mhnsw_index* h, const int64_t* keys, const float* vecs, bool vecs_on_device, int64_t n, int dim, const int32_t* levels);
int beam_vis_entries(const mhnsw_index* h);
int drain(mhnsw_index* h);
int search_impl(mhnsw_index* h, const float* queries, bool on_device, int64_t B, int dim, int k, int mode, int ef, const int64_t* entry_key, int64_t* okeys, float* odist, int32_t* on, hipStream_t s, bool timing, int32_t* out_ids = nullptr, bool sticky = false);
int order_meta(mhnsw_index* h, hipStream_t s);
int search_body(mhnsw_index* h, const float* queries, bool on_device, int64_t B, int dim, int k, int mode, int ef, const int64_t* entry_key, int64_t* okeys, float* odist, int32_t* on, hipStream_t s, bool timing, int32_t* out_ids, bool sticky);
void reset_graph(mhnsw_index* h);
int import_csr(mhnsw_index* h, int64_t N, int dim, int L, int cap, const int64_t* keys, const float* vecs, const int32_t* deg, const int32_t* adj, const int32_t* entry, const uint8_t* dead);
const char* metric_name(int m);
int strkey_relabel(mhnsw_index* h);
int strkey_insert(mhnsw_index* h, const std::string& s);
void strkey_table(mhnsw_index* h, const std::vector<std::string>& strs, std::vector<int64_t>& lab);
bool key_fits(const mhnsw_index* h, int64_t k, int kind);
int export_go(mhnsw_index* h, int key_kind, std::vector<uint8_t>& out);
int import_go(mhnsw_index* h, const uint8_t* buf, int64_t size, int key_kind);


template <class T>
int ensure_buf(mhnsw_index* h, DevBuf<T>& b, size_t n) {
    if (b.n >= n) return 0;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.n = 0;
    size_t want = std::max(n, b.n * 2);
    if (hipMalloc(&b.p, want * sizeof(T)) != hipSuccess) return fail(h, MHNSW_ENOMEM, "device allocation of %zu bytes failed", want * sizeof(T));
    b.n = want;
    return 0;
}

template <class T>
int grow(mhnsw_index* h, T*& p, int64_t old_elems, int64_t new_elems, int fill_byte, bool fill32 = false,
         uint32_t fill_val = 0) {
    T* np = nullptr;
    if (hipMalloc(&np, (size_t)new_elems * sizeof(T)) != hipSuccess)
        return fail(h, MHNSW_ENOMEM, "device allocation of %lld bytes failed", (long long)(new_elems * sizeof(T)));
    if (fill32)
        HIPCHK(h, hipMemsetD32Async((hipDeviceptr_t)np, (int)fill_val, (size_t)new_elems * sizeof(T) / 4, h->stream));
    else if (fill_byte >= 0)
        HIPCHK(h, hipMemsetAsync(np, fill_byte, (size_t)new_elems * sizeof(T), h->stream));
    if (p && old_elems > 0) HIPCHK(h, hipMemcpyAsync(np, p, (size_t)old_elems * sizeof(T), hipMemcpyDeviceToDevice, h->stream));
    if (p) {
        HIPCHK(h, hipStreamSynchronize(h->stream));
        (void)hipFree(p);
    }
    p = np;
    return 0;
}

}  // namespace mhh
