// device_search.hpp -- per-wave layer searches shared by the search kernels
// (search.hip) and the build kernels (build.hip).
//
//   beam_layer   : sorted-list best-first search (standard HNSW Alg. 2 stop
//                  rule), restated in oracle/oracle.c beam_layer_search.
//   compat_layer : graph.go:94-170 layerNode.search with the reference's heap
//                  quirks (Max()/PopLast() act on the last array slot, result
//                  in heap order, greedy stop), restated in oracle/oracle.c
//                  compat_layer_search.
#pragma once
#include "device_common.hpp"

namespace mh {

// Loads of mutable graph state.  COH = true inside the sequential build /
// delete kernels, which rewrite adjacency while searching: relaxed atomics
// keep the compiler off the (incoherent) scalar cache.  Only one wave ever
// reads or writes graph state there (the multi-wave build's workers score
// immutable rows), so wavefront scope suffices -- and it keeps the loads in
// the vector L1 (workgroup scope would add sc0, sending every dependent load
// of the walk to L2); the wave's own program order and __syncthreads /
// ev.sync() order its lanes.
// The pointers come from the layer table, so the compiler cannot tell their
// address space: the casts make these global (not flat) operations, which do
// not count against lgkmcnt (a flat load holds up every LDS wait behind it).
typedef __attribute__((address_space(1))) int32_t g_i32;
template <bool COH>
__device__ __forceinline__ int32_t ld_i32(const int32_t* p) {
    const g_i32* gp = (const g_i32*)p;
    if constexpr (COH)
        return __hip_atomic_load(gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    else
        return *gp;
}
__device__ __forceinline__ void st_i32(int32_t* p, int32_t v) {
    __hip_atomic_store((g_i32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

// `layers[l].nodes[*elevator]` (graph.go:497, 574): the layer's node of the
// elevator row's KEY -- the key's live row that is a member of layer l (its
// newest, then the older ones through kprev), else nil (EMPTY_ID).  The
// elevator itself may be a replaced or deleted node that a dangling edge led to.
template <bool COH>
__device__ __forceinline__ uint32_t resolve_member(const GraphDev& g, int l, uint32_t e) {
    if (g.kidlive) {
        int32_t r = ld_i32<COH>(g.kidlive + kid_of(g, e));
        for (int hop = 0; hop < MH_MAXL && r >= 0 && (uint32_t)r < g.capn; ++hop) {  // (rows hold disjoint layers)
            if (ld_i32<COH>(g.layers[l].deg + r) != -2 && !is_dead(g, (uint32_t)r)) return (uint32_t)r;
            r = g.kprev ? ld_i32<COH>(g.kprev + r) : -1;
        }
        return EMPTY_ID;
    }
    if (e >= g.capn || ld_i32<COH>(g.layers[l].deg + e) == -2 || is_dead(g, e)) return EMPTY_ID;
    return e;
}

// Evaluate the distances of candidate ids held in lanes 0..cnt-1 of `cid`
// against the query; sink(dist, id) is called in row order (uniformly).
template <class C, int G, class Sink>
__device__ __forceinline__ void eval_list(const GraphDev& g, const QReg<C>& q, float qn, uint32_t cid, int cnt,
                                          int metric, Sink&& sink) {
    using RM = RowMap<C, G>;
    const int lane = lane_id();
    for (int base = 0; base < cnt; base += RM::T) {
        uint32_t ids[G];
        bool valid[G];
#pragma unroll
        for (int gg = 0; gg < G; ++gg) {
            const int t = base + RM::reg_row(gg, lane);
            valid[gg] = t < cnt;
            if constexpr (C::RPI == 1)
                ids[gg] = rl_u(cid, (base + gg) & 63);
            else
                ids[gg] = shfl_u(cid, t & 63);
            ids[gg] = valid[gg] ? guard_id(g, ids[gg]) : 0u;
        }
        float s;
        if (metric == EUCLIDEAN)
            s = eval_rows<C, G, true>(q, g.vecs, g.pitch, ids, valid);
        else
            s = eval_rows<C, G, false>(q, g.vecs, g.pitch, ids, valid);
        const int town = base + RM::owned_row(lane);
        const uint32_t idown = shfl_u(cid, town & 63);
        float xn = 1.f;
        if (metric == COSINE && town < cnt) xn = g.norms[guard_id(g, idown)];
        const float dist = finalize(metric, s, xn, qn);
#pragma unroll
        for (int t = 0; t < RM::T; ++t) {
            if (base + t >= cnt) break;
            sink(rl_f(dist, RM::owner(t)), rl_u(cid, (base + t) & 63));
        }
    }
}

// compact the lanes where `keep` holds into lanes 0..popc-1 (order preserving)
__device__ __forceinline__ uint32_t compact(uint32_t v, bool keep, int& cnt) {
    const unsigned long long m = __ballot(keep);
    cnt = __popcll(m);
    const int lane = lane_id();
    const int before = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
    const int dst = keep ? before : cnt + (lane - before);
    return push_to(v, dst);
}

// Screened evaluation for the sorted-list searches: candidates whose fp16
// screening distance proves the f32 distance exceeds `wd` (the list's worst
// entry before this batch, which only decreases) are dropped; the rest go
// through eval_list, so every distance that reaches the sink is the canonical
// f32 one and the list evolves exactly as without the screen.
// Returns the number of rows evaluated in f32.
template <class C, int G, class Sink>
__device__ __forceinline__ int eval_screened(const GraphDev& g, const QReg<C>& q, float qn, uint32_t cid, int cnt,
                                             int metric, float wd, Sink&& sink, unsigned long long& s16,
                                             float margin) {
    constexpr int GH = (2 * G <= C::LPR) ? 2 * G : G;
    using RM = RowMap<C, GH>;
    const int lane = lane_id();
    if (!g.h16) {
        eval_list<C, G>(g, q, qn, cid, cnt, metric, sink);
        return cnt;
    }
    s16 += cnt;
    bool rej = false;  // lane t: candidate t is rejected
    for (int base = 0; base < cnt; base += RM::T) {
        uint32_t ids[GH];
        bool valid[GH];
        float inv[GH];
#pragma unroll
        for (int gg = 0; gg < GH; ++gg) {
            const int t = base + RM::reg_row(gg, lane);
            valid[gg] = t < cnt;
            if constexpr (C::RPI == 1)
                ids[gg] = rl_u(cid, (base + gg) & 63);
            else
                ids[gg] = shfl_u(cid, t & 63);
            ids[gg] = valid[gg] ? guard_id(g, ids[gg]) : 0u;
        }
        const int town = base + RM::owned_row(lane);
        bool r = false;
        if (metric == EUCLIDEAN) {
            float xn[GH];
#pragma unroll
            for (int gg = 0; gg < GH; ++gg) {
                const float2 ax = g.h16aux[ids[gg]];
                inv[gg] = ax.x;
                xn[gg] = ax.y;
            }
            const float s = eval_rows_h16<C, GH, true>(q, g.h16, g.pitch, ids, valid, inv);
            // the owner of row town computed it in register (town - base) / RPI
            float xo = xn[0];
#pragma unroll
            for (int gg = 1; gg < GH; ++gg)
                if (RM::reg_row(gg, lane) == town - base) xo = xn[gg];
            if (town < cnt) r = h16_rejects_l2(s, xo, wd, margin);
        } else {
#pragma unroll
            for (int gg = 0; gg < GH; ++gg) inv[gg] = 1.f;
            const float s = eval_rows_h16<C, GH, false>(q, g.h16, g.pitch, ids, valid, inv);
            if (town < cnt) r = h16_rejects_cos(s, qn, wd, margin);
        }
        // hand row t's verdict from its owner lane to lane t
        const int t = lane - base;
        const int src = (t >= 0 && t < RM::T) ? RM::owner(t) : lane;
        const bool rt = __shfl((int)r, src, 64) != 0;
        if (t >= 0 && t < RM::T) rej = rt;
    }
    int cnt2;
    const uint32_t cid2 = compact(cid, lane < cnt && !rej, cnt2);
    if (cnt2 > 0) eval_list<C, G>(g, q, qn, cid2, cnt2, metric, sink);
    return cnt2;
}

// Two-sided screen of the rows cid[0, cnt) against a stored row held as the
// "query" q (norm qn), for the selection rule "r drops c when alpha d(c, r) <
// d(u, c)": lane t gets +1 when row t's f32 distance is certainly > hi_t, -1
// when it is certainly < lo_t, 0 when the fp16 estimate cannot tell (those go
// to the canonical f32 path).  lo_t / hi_t: row t's bounds, in lane t (or the
// same in every lane).  Rows outside the copy's range are always 0.
template <class C, int G>
__device__ __forceinline__ int screen_pairs(const GraphDev& g, const QReg<C>& q, float qn, uint32_t cid, int cnt,
                                            int metric, float lo_t, float hi_t, float margin) {
    constexpr int GH = (2 * G <= C::LPR) ? 2 * G : G;
    using RM = RowMap<C, GH>;
    const int lane = lane_id();
    int cls = 0;
    for (int base = 0; base < cnt; base += RM::T) {
        uint32_t ids[GH];
        bool valid[GH];
        float inv[GH];
#pragma unroll
        for (int gg = 0; gg < GH; ++gg) {
            const int t = base + RM::reg_row(gg, lane);
            valid[gg] = t < cnt;
            if constexpr (C::RPI == 1)
                ids[gg] = rl_u(cid, (base + gg) & 63);
            else
                ids[gg] = shfl_u(cid, t & 63);
            ids[gg] = valid[gg] ? guard_id(g, ids[gg]) : 0u;
        }
        const int town = base + RM::owned_row(lane);
        const float lo = __shfl(lo_t, town & 63, 64), hi = __shfl(hi_t, town & 63, 64);
        int c = 0;
        if (metric == EUCLIDEAN) {
            float xn[GH];
#pragma unroll
            for (int gg = 0; gg < GH; ++gg) {
                const float2 ax = g.h16aux[ids[gg]];
                inv[gg] = ax.x;
                xn[gg] = ax.y;
            }
            const float s = eval_rows_h16<C, GH, true>(q, g.h16, g.pitch, ids, valid, inv);
            float xo = xn[0];
#pragma unroll
            for (int gg = 1; gg < GH; ++gg)
                if (RM::reg_row(gg, lane) == town - base) xo = xn[gg];
            if (town < cnt) c = h16_rejects_l2(s, xo, hi, margin) ? 1 : h16_below_l2(s, xo, lo, margin) ? -1 : 0;
        } else {
#pragma unroll
            for (int gg = 0; gg < GH; ++gg) inv[gg] = 1.f;
            const float s = eval_rows_h16<C, GH, false>(q, g.h16, g.pitch, ids, valid, inv);
            if (town < cnt) c = h16_rejects_cos(s, qn, hi, margin) ? 1 : h16_below_cos(s, qn, lo, margin) ? -1 : 0;
        }
        const int t = lane - base;
        const int src = (t >= 0 && t < RM::T) ? RM::owner(t) : lane;
        const int ct = __shfl(c, src, 64);
        if (t >= 0 && t < RM::T) cls = ct;
    }
    return cls;
}

struct WaveStats {
    unsigned long long E = 0, X = 0, resets = 0;
    unsigned long long S = 0, F = 0;  // rows screened on the fp16 copy / rows evaluated in f32
#ifdef MH_PROF_BEAM
    // (tools-only build, tools/Makefile.beam: shader-clock cycles of the layer-0
    // beam spent in list insertions, in candidate scoring, and in all)
    unsigned long long c_ins = 0, c_score = 0, c_all = 0;
#endif
};

// Orders the lanes of ONE wave (compiler ordering only: a wave's vector memory
// and LDS operations are performed in issue order, so a lane's load after
// another lane's store to the same address sees it -- no waitcnt for the
// store's acknowledgement).  The sequential walks mutate graph state from a
// single wave; nothing else reads it while they run.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// How the sequential (compat) walks evaluate distances and order their own
// lanes.  WaveEval: everything on the calling wave (a 64-thread workgroup, so
// __syncthreads only orders this wave).  The multi-wave build evaluator
// (build.hip MwEval) has the same interface and spreads each batch of rows
// over the workgroup's other waves.
struct WaveEval {
    static constexpr bool kPairs = false;  // no batched per-row scoring (build.hip MwEval::pairs)
    uint32_t* list = nullptr;  // LDS candidate list (run_list)
    template <class C, int G, class Sink>
    __device__ __forceinline__ void run(const GraphDev& g, const QReg<C>& q, float qn, uint32_t cid, int cnt,
                                        int metric, Sink&& sink) const {
        eval_list<C, G>(g, q, qn, cid, cnt, metric, sink);
    }
    // rows list[0, cnt), sink called in list order
    template <class C, int G, class Sink>
    __device__ __forceinline__ void run_list(const GraphDev& g, const QReg<C>& q, float qn, int cnt, int metric,
                                             Sink&& sink) const {
        for (int b = 0; b < cnt; b += 64) {
            const int c = min(64, cnt - b);
            const uint32_t cid = lane_id() < c ? list[b + lane_id()] : 0u;
            eval_list<C, G>(g, q, qn, cid, c, metric, sink);
        }
    }
    // rows list[0, cnt): distance e into outd[e], the row into outi[e]
    template <class C, int G>
    __device__ __forceinline__ void score(const GraphDev& g, const QReg<C>& q, float qn, int cnt, int metric,
                                          float* outd, uint32_t* outi) const {
        int t = 0;
        run_list<C, G>(g, q, qn, cnt, metric, [&](float d, uint32_t u) {
            if (lane_id() == 0) {
                outd[t] = d;
                outi[t] = u;
            }
            ++t;
        });
    }
    __device__ __forceinline__ void sync() const { wave_sync(); }
};

// the visited set's fill at which beam_layer forgets (3/4; a tools build may
// set another fraction to measure the probe-length / re-evaluation trade)
// beam_layer's visited set: vsize > 0 the 32-bit set of vsize entries, vsize < 0
// the compact 16-bit set (device_common.hpp VIS16_*; the query searches, ids < 2^24)
__device__ __forceinline__ int vis_any_probe(uint32_t* vis, int vsize, uint32_t id) {
    return vsize < 0 ? vis16_probe(vis, id) : vis_probe_n(vis, (uint32_t)vsize, id);
}
__device__ __forceinline__ void vis_any_clear(uint32_t* vis, int vsize) { vis_clear(vis, vsize < 0 ? VIS16_WORDS : vsize); }
__device__ __forceinline__ int vis_any_cap(int vsize) { return vsize < 0 ? VIS16_HOMES : vsize; }

#ifndef MH_VIS_FULL
#define MH_VIS_FULL(n) (((n) >> 1) + ((n) >> 2))
#endif

// Batched list update (the query search's 256- and 512-entry lists, beam_layer
// MERGE): a step's candidates that beat the list's worst entry are collected,
// one per lane, and merged into the list once per step instead of one
// bl_insert each.  bl_insert keeps the best ef of the list and everything
// offered to it, whatever the order (it drops a candidate only when it is no
// better than the worst entry or already listed), so the merge leaves the list
// bl_insert would, expansion marks included.  Fast path, every distance finite
// and distinct: each candidate ranked among the candidates (one compare per
// candidate) and in the list (binary search over the list's distances in LDS,
// A), every list entry moved down by the candidates ranked at or before it,
// and both written into A at their new places and read back (distances, then
// ids).  A candidate whose distance equals a listed one (the same row met
// again, or equal rows) or any infinite distance sends the buffer through
// bl_insert instead.  LDS scratch M: A = M[0, 512) (the list), the k <= 64
// candidates in M[512 + j] (distance) and M[576 + j] (id), in arrival order.
constexpr int BL_MERGE_WORDS = 640;
template <int R>
__device__ __forceinline__ void bl_merge(BList<R>& L, int ef, int k, float* M) {
    const int lane = lane_id();
    const float INF = __int_as_float(0x7f800000);
    float* A = M;
    wave_sync();  // (the buffer was written by lane 0)
    const float bd = lane < k ? M[512 + lane] : INF;
    const uint32_t bi = lane < k ? reinterpret_cast<const uint32_t*>(M)[576 + lane] : EMPTY_ID;
    const float d = bd;
    const uint32_t id = bi;
    bool slow = __ballot(lane < k && !(bd < INF)) != 0;
    int rk = 0;  // lane j < k: the candidates below candidate j
    int lb = 0;  // lane j < k: the list entries (of the first ef) below candidate j
    if (!slow) {
        int eq = 0;
        for (int j = 0; j < k; ++j) {
            const float dj = rl_f(bd, j);
            rk += dj < bd ? 1 : 0;
            eq += dj == bd ? 1 : 0;
        }
        slow = __ballot(lane < k && eq > 1) != 0;
    }
    if (!slow) {
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (r * 64 + lane < ef) A[r * 64 + lane] = L.d[r];
        wave_sync();
        if (lane < k) {
            // lower bound over A[0, ef); a candidate is below the worst entry, so lb < ef
#pragma unroll
            for (int step = R * 32; step >= 1; step >>= 1) {
                const int t = lb + step - 1;
                if (t < ef && A[t] < d) lb += step;
            }
        }
        slow = __ballot(lane < k && (lb >= ef || A[lb] == d)) != 0;
        wave_sync();
    }
    if (slow) {
        for (int j = 0; j < k; ++j) bl_insert(L, ef, rl_f(bd, j), rl_u(bi, j));
        return;
    }
    int sh[R];
#pragma unroll
    for (int r = 0; r < R; ++r) sh[r] = 0;
    for (int j = 0; j < k; ++j) {
        const int lj = rl_i(lb, j);
#pragma unroll
        for (int r = 0; r < R; ++r) sh[r] += (r * 64 + lane >= lj) ? 1 : 0;
    }
    const int pos = rk + lb;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = r * 64 + lane;
        if (i < ef && i + sh[r] < ef) A[i + sh[r]] = L.d[r];
    }
    if (lane < k && pos < ef) A[pos] = d;
    wave_sync();
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (r * 64 + lane < ef) L.d[r] = A[r * 64 + lane];
    wave_sync();
    uint32_t* AI = reinterpret_cast<uint32_t*>(A);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = r * 64 + lane;
        if (i < ef && i + sh[r] < ef) AI[i + sh[r]] = L.i[r];
    }
    if (lane < k && pos < ef) AI[pos] = id;
    wave_sync();
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (r * 64 + lane < ef) L.i[r] = AI[r * 64 + lane];
    wave_sync();
}

// How beam_layer scores one batch of new candidates (ids in lanes 0..cnt-1 of
// cid) and hands the survivors to its sink: WaveBatch does it on the calling
// wave; the multi-wave single-query kernel (beam.hpp MwBatch) spreads the rows
// over the workgroup's waves.  Returns the rows evaluated in f32.
struct WaveBatch {
    template <class C, int G, bool SCREEN, class Sink>
    __device__ __forceinline__ int score(const GraphDev& g, const QReg<C>& q, float qn, uint32_t cid, int cnt,
                                         float wd, bool screen, float margin, Sink&& sink,
                                         unsigned long long& s16) const {
        if (SCREEN && screen && wd < __int_as_float(0x7f800000))
            return eval_screened<C, G>(g, q, qn, cid, cnt, g.metric, wd, sink, s16, margin);
        eval_list<C, G>(g, q, qn, cid, cnt, g.metric, sink);
        return cnt;
    }
};

// ---------------------------------------------------------------------------
// beam: sorted list of <= ef entries; stop when every entry is expanded
// ---------------------------------------------------------------------------
// XW: entries expanded per step.  1 is the standard best-first search (the
// oracle's beam_layer_search with xw 1).  XW > 1 (the batched insert's layer
// searches, option "build_expand"; the query search's layer 0, option
// "search_expand"): the XW best unexpanded entries are expanded together --
// their adjacency rows fetched in one round trip and their new neighbours
// evaluated in batches of up to 64 against the worst entry before the step --
// fewer dependent round trips for a search whose expansions yield few new
// candidates.  The oracle restates it (beam_layer_search's xw).
// MH_SCREEN_PAD (a build flag for tools/ variants, default 0): widens the
// screen's margin, to measure how the rejections fall off with a looser bound
#ifndef MH_SCREEN_PAD
#define MH_SCREEN_PAD 0.f
#endif
// MERGE (the query search's layer 0 at ef > 128): the step's candidates go
// through bl_merge once per step, with `mrg` (BL_MERGE_WORDS of LDS) as its
// scratch.
template <class C, int R, int G, bool COH = false, bool SCREEN = false, int XW = 1, bool MERGE = false,
          class BEv = WaveBatch>
__device__ __forceinline__ void beam_layer(const GraphDev& g, int layer, uint32_t entry, int ef, const QReg<C>& q, float qn,
                           BList<R>& L, uint32_t* vis, int vsize, WaveStats& st, const BEv& bev = BEv(),
                           float* mrg = nullptr) {
    const int lane = lane_id();
    bl_init(L);
    if (entry == EMPTY_ID) return;
    vis_any_clear(vis, vsize);
    wave_sync();  // (the list and the visited set belong to this wave alone)
    if (lane == 0) vis_any_probe(vis, vsize, entry);
    int vcount = 1;
    eval_list<C, G>(g, q, qn, entry, 1, g.metric, [&](float d, uint32_t u) { bl_insert(L, ef, d, u); });
    st.E += 1;
    st.F += 1;
    const bool screen = SCREEN && h16_query_ok(qn);
    float margin = 0.f;  // the copy's measured rounding -> the metric's screening margin
    if constexpr (SCREEN) {
        const float e = g.h16err ? *g.h16err : 0.00048828125f;
        margin = g.metric == EUCLIDEAN ? h16_margin_l2(e) : h16_margin_cos(e);
        margin += MH_SCREEN_PAD;
    }
    const int32_t* degp = g.layers[layer].deg;
    const int32_t* adjp = g.layers[layer].adj;
    const int capl = g.layers[layer].cap;
#ifdef MH_PROF_BEAM
    const unsigned long long tl0 = clock64();
    struct AllClock {  // adds the layer-0 search's cycles at every exit
        WaveStats& st;
        unsigned long long t0;
        int layer;
        __device__ ~AllClock() {
            if (layer == 0) st.c_all += clock64() - t0;
        }
    } all_clock{st, tl0, layer};
#endif
    for (;;) {
        uint32_t cur[XW];
        cur[0] = bl_next(L);
        if (cur[0] == EMPTY_ID) break;
#pragma unroll
        for (int w = 1; w < XW; ++w) cur[w] = bl_next(L);
        // the adjacency rows are loaded together with their degrees (rows are
        // cap wide, so lanes past the degree read allocated, ignored slots):
        // one dependent round trip per step
        int32_t rowv[XW];
        int deg[XW];
#pragma unroll
        for (int w = 0; w < XW; ++w) {
            rowv[w] = -1;
            deg[w] = 0;
            if (cur[w] != EMPTY_ID) {
                st.X += 1;
                const uint32_t cg = guard_id(g, cur[w]);
                rowv[w] = lane < capl ? ld_i32<COH>(adjp + (size_t)cg * capl + lane) : -1;
                deg[w] = min(uni(ld_i32<COH>(degp + cg)), capl);
            }
        }
        uint32_t cids[XW];
        int cnts[XW];
#pragma unroll
        for (int w = 0; w < XW; ++w) {
            const bool have = lane < deg[w];
            uint32_t nb = have ? (uint32_t)rowv[w] : 0u;
            int pr = 0;
            if (have && nb != 0xFFFFFFFFu) {
                nb = guard_id(g, nb);
                pr = vis_any_probe(vis, vsize, nb);
            }
            vcount += __popcll(__ballot(pr == 1));
            cids[w] = compact(nb, pr != 0, cnts[w]);
        }
        // the new neighbours of consecutive expanded entries share a batch while
        // they fit the wave
        if constexpr (XW >= 2) {
            int b = 0;
#pragma unroll
            for (int w = 1; w < XW; ++w) {
                if (cnts[b] + cnts[w] <= 64) {
                    const uint32_t cw = shfl_u(cids[w], (lane - cnts[b]) & 63);
#pragma unroll
                    for (int v = 0; v < w; ++v)  // (static register indices)
                        if (v == b && lane >= cnts[v]) cids[v] = cw;
#pragma unroll
                    for (int v = 0; v < w; ++v)
                        if (v == b) cnts[v] += cnts[w];
                    cnts[w] = 0;
                } else {
                    b = w;
                }
            }
        }
        float wd = __int_as_float(0x7f800000);
        uint32_t wi = EMPTY_ID;
        if constexpr (SCREEN || MERGE) bl_at(L, ef - 1, wd, wi);  // the worst before the step: it only decreases during it
        int bk = 0;  // MERGE: the step's candidates below that worst, in mrg's buffer
        // the batches are taken from slot 0 and the slots shifted down, so every
        // register index is static whether or not the compiler unrolls this loop
        // (a large score() body can keep it rolled)
        for (int w = 0; w < XW; ++w) {
            const int cnt = cnts[0];
            const uint32_t cid = cids[0];
#pragma unroll
            for (int v = 0; v + 1 < XW; ++v) {
                cnts[v] = cnts[v + 1];
                cids[v] = cids[v + 1];
            }
            cnts[XW - 1] = 0;
            if (cnt == 0) continue;
            st.E += cnt;
            if constexpr (MERGE) {
                {
                    if (bk + cnt > 64) {  // (a batch adds at most cnt)
                        bl_merge(L, ef, bk, mrg);
                        bk = 0;
                    }
                    auto sink = [&](float d, uint32_t u) {
                        if (lt_di(d, u, wd, wi & ID_MASK)) {
                            if (lane == 0) {
                                mrg[512 + bk] = d;
                                reinterpret_cast<uint32_t*>(mrg)[576 + bk] = u;
                            }
                            ++bk;
                        }
                    };
                    st.F += bev.template score<C, G, SCREEN>(g, q, qn, cid, cnt, wd, screen, margin, sink, st.S);
                    continue;
                }
            }
#ifdef MH_PROF_BEAM
            const unsigned long long t0 = clock64();
            unsigned long long ti = 0;
            auto sink = [&](float d, uint32_t u) {
                const unsigned long long a = clock64();
                bl_insert(L, ef, d, u);
                ti += clock64() - a;
            };
            st.F += bev.template score<C, G, SCREEN>(g, q, qn, cid, cnt, wd, screen, margin, sink, st.S);
            if (layer == 0) {
                st.c_ins += ti;
                st.c_score += clock64() - t0 - ti;
            }
#else
            auto sink = [&](float d, uint32_t u) { bl_insert(L, ef, d, u); };
            st.F += bev.template score<C, G, SCREEN>(g, q, qn, cid, cnt, wd, screen, margin, sink, st.S);
#endif
        }
        if constexpr (MERGE) {
            if (bk > 0) bl_merge(L, ef, bk, mrg);
        }
        if (vcount > MH_VIS_FULL(vis_any_cap(vsize))) {  // reset: results unchanged
            wave_sync();
            vis_any_clear(vis, vsize);
            wave_sync();
            // the list's members stay visited: they are the neighbourhood the
            // next expansions keep meeting (fewer re-evaluations)
            int seeded = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t id = L.i[r];
                const bool ins = id != EMPTY_ID && vis_any_probe(vis, vsize, id & ID_MASK) == 1;
                seeded += __popcll(__ballot(ins));
            }
            wave_sync();
            vcount = seeded;
            st.resets += 1;
        }
    }
}

// ---------------------------------------------------------------------------
// several waves per query (or insert): wave 0 runs the list, the visited set
// and the expansions; each batch of new candidates is split over the waves
// (screen + f32 on each wave's rows, in one round trip instead of one per 16
// rows) and the survivors come back to wave 0's list.  The list is the best ef
// of everything inserted whatever the insertion order, so the results are the
// one-wave kernel's bit for bit (k_search_beam_mw, k_batch_search_mw).
// ---------------------------------------------------------------------------
constexpr int BMW_WAVES = 4;
constexpr int BMW_SCORE = 0, BMW_EXIT = 1;
struct BmwShare {
    int cmd, cnt;
    float wd;
    int pad_;
    uint32_t list[64];
    int scnt[BMW_WAVES];
    float sd[BMW_WAVES * 64];
    uint32_t si[BMW_WAVES * 64];
};

// everything handed between the waves is in LDS (rows and norms are only read)
__device__ __forceinline__ void bmw_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// wave w's rows of the posted batch, [w*ch, min(cnt, (w+1)*ch)): screened
// against the posted worst, survivors (f32 distance, id) into sd / si
template <class C, int G, bool SCREEN>
__device__ __forceinline__ int bmw_share(const GraphDev& g, const QReg<C>& q, float qn, BmwShare* sh, int w,
                                         bool screen, float margin, unsigned long long& s16) {
    const int lane = lane_id();
    const int cnt = uni(sh->cnt);
    const float wd = __int_as_float(uni(__float_as_int(sh->wd)));
    const int ch = (cnt + BMW_WAVES - 1) / BMW_WAVES;
    const int t0 = w * ch;
    const int c = min(cnt - t0, ch);
    int k = 0, f = 0;
    if (c > 0) {
        const uint32_t cid = lane < c ? sh->list[t0 + lane] : 0u;
        auto sink = [&](float d, uint32_t u) {
            if (lane == 0) {
                sh->sd[w * 64 + k] = d;
                sh->si[w * 64 + k] = u;
            }
            ++k;
        };
        f = WaveBatch().template score<C, G, SCREEN>(g, q, qn, cid, c, wd, screen, margin, sink, s16);
    }
    if (lane == 0) sh->scnt[w] = k;
    return f;
}

struct MwBatch {
    BmwShare* sh;
    template <class C, int G, bool SCREEN, class Sink>
    __device__ __forceinline__ int score(const GraphDev& g, const QReg<C>& q, float qn, uint32_t cid, int cnt,
                                         float wd, bool screen, float margin, Sink&& sink,
                                         unsigned long long& s16) const {
        const int lane = lane_id();
        if (lane < cnt) sh->list[lane] = cid;
        if (lane == 0) {
            sh->cmd = BMW_SCORE;
            sh->cnt = cnt;
            sh->wd = wd;
        }
        bmw_barrier();  // post
        const int f = bmw_share<C, G, SCREEN>(g, q, qn, sh, 0, screen, margin, s16);
        bmw_barrier();  // collect
#pragma unroll
        for (int w = 0; w < BMW_WAVES; ++w) {
            const int n = uni(sh->scnt[w]);
            const float dv = lane < n ? sh->sd[w * 64 + lane] : 0.f;
            const uint32_t iv = lane < n ? sh->si[w * 64 + lane] : 0u;
            for (int t = 0; t < n; ++t) sink(rl_f(dv, t), rl_u(iv, t));
        }
        return f;  // this wave's rows (the others count theirs)
    }
};


// ---------------------------------------------------------------------------
// compat: graph.go:94-170 verbatim semantics on LDS Go-heaps
// ---------------------------------------------------------------------------
struct CompatSmem {
    uint32_t* vis;
    int vlog2;
    float* cd;
    uint32_t* ci;  // candidates heap [ef+2]
    float* rd;
    uint32_t* ri;  // result heap [k+2]
};

// HP: GHeap (LDS arrays S.cd/S.ci and S.rd/S.ri) or RHeap (one slot per lane,
// when ef + 1 and k + 1 fit the wave); the result heap ends in S.rd / S.ri
// either way, in heap order.
template <class C, int G, bool COH, class Ev, class HP>
__device__ __forceinline__ int compat_layer_h(const GraphDev& g, int layer, uint32_t entry, int k, int ef,
                                              const QReg<C>& q, float qn, CompatSmem& S, WaveStats& st, int& err,
                                              const Ev& ev, HP cand, HP res) {
    const int lane = lane_id();
    const int vsize = 1 << S.vlog2, vmask = vsize - 1;
    vis_clear(S.vis, vsize);
    ev.sync();
    float d0 = 0.f;
    ev.template run<C, G>(g, q, qn, entry, 1, g.metric, [&](float d, uint32_t) { d0 = d; });  // graph.go:112
    st.E += 1;
    if (lane == 0) vis_probe(S.vis, vmask, kid_of(g, entry));  // graph.go:123 visited[n.Key]
    hp_push(cand, d0, entry);                          // graph.go:109-114
    hp_push(res, hp_d(cand, 0), hp_id(cand, 0));       // graph.go:122
    const int32_t* degp = g.layers[layer].deg;
    const int32_t* adjp = g.layers[layer].adj;
    const int capl = g.layers[layer].cap;
    while (cand.n > 0) {
        float cdist;
        uint32_t cur;
        hp_pop(cand, cdist, cur);  // graph.go:127
        bool improved = false;
        const uint32_t cg = guard_id(g, cur);
        // the row is loaded with its degree (one round trip, entries past deg ignored)
        const int32_t rowv = lane < capl ? ld_i32<COH>(adjp + (size_t)cg * capl + lane) : -1;
        const int deg = min(uni(ld_i32<COH>(degp + cg)), capl);
        if (deg < 0) continue;  // graph.go:131-133 (nil neighbor map)
        st.X += 1;
        const bool have = lane < deg;
        uint32_t nb = 0xFFFFFFFFu;
        int64_t key = INT64_MAX;
        if (have) {
            nb = guard_id(g, (uint32_t)rowv);
            key = g.keys[nb];
        }
        rank_sort(key, nb, deg);  // graph.go:137-138 ascending key order
        int pr = 0;
        if (lane < deg) pr = vis_probe(S.vis, vmask, kid_of(g, nb));  // graph.go:141-144 (by key)
        if (__ballot(pr == 2)) err = 1;                   // exact visited set required here
        int cnt;
        const uint32_t cid = compact(nb, pr == 1, cnt);
        st.E += cnt;
        CPROF_T(tq);
        ev.template run<C, G>(g, q, qn, cid, cnt, g.metric, [&](float dist, uint32_t u) {  // graph.go:146-159
            improved = improved || (res.n > 0 && dist < hp_d(res, 0));
            if (res.n < k) {
                hp_push(res, dist, u);
            } else if (dist < hp_d(res, res.n - 1)) {
                hp_poplast(res);
                hp_push(res, dist, u);
            }
            hp_push(cand, dist, u);
            if (cand.n > ef) hp_poplast(cand);
        });
        CPROF_ADD(tq, 22);
        CPROF_CNT(23, cnt);
        if (!improved && res.n >= k) break;  // graph.go:164-166
    }
    hp_store(res, S.rd, S.ri);
    return res.n;
}

template <class C, int G, bool COH = false, class Ev = WaveEval>
__device__ __forceinline__ int compat_layer(const GraphDev& g, int layer, uint32_t entry, int k, int ef, const QReg<C>& q, float qn,
                            CompatSmem& S, WaveStats& st, int& err, const Ev& ev = Ev()) {
    if (entry == EMPTY_ID) return 0;
    if (ef < 64 && k < 64)  // at most ef + 1 / k + 1 entries at a time
        return compat_layer_h<C, G, COH>(g, layer, entry, k, ef, q, qn, S, st, err, ev, RHeap{}, RHeap{});
    return compat_layer_h<C, G, COH>(g, layer, entry, k, ef, q, qn, S, st, err, ev, GHeap{S.cd, S.ci, 0},
                                     GHeap{S.rd, S.ri, 0});
}

}  // namespace mh
