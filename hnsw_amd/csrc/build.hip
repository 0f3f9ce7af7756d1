// build.hip -- insert path (Graph.Add / BatchAdd, graph.go:437-531, 942-1042).
//
// k_build_compat: the reference's strictly sequential insert, verbatim
//   semantics (per-layer compat search with k = M, bidirectional addNeighbor
//   with "evict the worst of M+1" (graph.go:41-81) and one-directional
//   replenish from neighbours-of-neighbours ranked by CosineDistance
//   (graph.go:172-219)).  One wave walks the inserts in order; every distance
//   batch is spread over the 64 lanes.  Graph state is rewritten while it is
//   searched, so adjacency goes through relaxed atomics + __syncthreads.
//
// k_batch_search / k_batch_commit: throughput insert.  A batch of new nodes is
//   searched in parallel against the graph as it stood before the batch (one
//   wave per node, beam search with efConstruction), each node selects its
//   neighbours (HNSW heuristic or closest-M) and writes its own row; reverse
//   edges are proposed into per-target slots and committed by one wave per
//   touched node, keeping the best cap by (distance, id) -- the M-neighbour
//   selection of graph.go:55-80 generalised to a set of proposals, and
//   independent of arrival order.
#include "device_search.hpp"
#include "engine.hpp"

namespace mh {

__device__ __forceinline__ void build_sync() { __syncthreads(); }

// ---------------------------------------------------------------------------
// compat build
// ---------------------------------------------------------------------------
// The walks below run on ONE wave (the "master"): every graph mutation, heap
// and visited-set operation happens there, in the reference's order.  Only
// distance batches are delegated, through the evaluator policy `Ev`:
// WaveEval evaluates on the master itself; MwEval (k_build_compat_mw) hands a
// batch to all waves of the workgroup and gets the distances back in LDS, in
// the same order.  Distances are the canonical ones whichever wave computes
// them (eval_rows), so both evaluators give identical graphs.
struct BuildSmem {
    CompatSmem cs;
    float* hd;  // replenish heap
    uint32_t* hi;
    int hcap;
    uint32_t* radj;  // replenish: staged neighbour rows (hcap entries)
    int64_t* rkey;   // ... and their keys
    // eviction speculation (k_build_compat_mw): the neighbourhood's rows as the
    // layer's addNeighbor pairs start, each followed by the new node, and the
    // distances of every such entry to its row's owner (stride pstride)
    int32_t* prow = nullptr;  // [pgroups * pstride] entry i of neighbour j's row
    int* pdeg = nullptr;      // [pgroups] its degree (-1 nil)
    float* pdist = nullptr;   // [pgroups * pstride] distance of entry i to neighbour j (entry deg: the new node)
    int pgroups = 0, pstride = 0;
};

// Rows are loaded together with their degree (one round trip; entries past
// the degree are ignored): the sequential walk is bound by dependent loads.
// list_remove_in: n's row already in registers (lane i: entry i, d entries);
// both are updated to the row after the removal, so the next step on n (the
// replenish after an eviction) needs no reload.
template <class Ev>
__device__ __forceinline__ void list_remove_in(const GraphDev& g, int l, uint32_t n, int32_t& rv, int& d, uint32_t v,
                                               const Ev& ev) {
    const int lane = lane_id();
    if (d <= 0) return;
    // delete(n.neighbors, v.Key): the entry of v's key, whichever row it holds
    const bool hit = lane < d && kid_of(g, guard_id(g, (uint32_t)rv)) == kid_of(g, v);
    const unsigned long long m = __ballot(hit);
    if (!m) return;
    const int pos = __ffsll((long long)m) - 1;
    const int32_t last = __shfl(rv, d - 1, 64);
    ev.sync();
    if (lane == 0) {
        st_i32(g.layers[l].adj + (size_t)n * g.layers[l].cap + pos, last);
        st_i32(g.layers[l].deg + n, d - 1);
    }
    ev.sync();
    if (lane == pos) rv = last;
    d = d - 1;
}
template <class C, int G, class Ev>
__device__ __forceinline__ void list_remove(const GraphDev& g, int l, uint32_t n, uint32_t v, const Ev& ev) {
    const int lane = lane_id();
    const int capl = g.layers[l].cap;
    int32_t rv = lane < capl ? ld_i32<true>(g.layers[l].adj + (size_t)n * capl + lane) : -1;
    int d = uni(ld_i32<true>(g.layers[l].deg + n));  // uniform: scalar loop bounds
    list_remove_in(g, l, n, rv, d, v, ev);
}

// graph.go:50 n.neighbors[nw.Key] = nw: overwrite the entry of nw's key (which
// may hold another row of that key), else append; returns the new degree and,
// in *rowout (nullable), the row after the assignment (lane i: entry i)
template <class Ev>
__device__ __forceinline__ int list_append(const GraphDev& g, int l, uint32_t n, uint32_t nw, const Ev& ev,
                           int32_t* rowout = nullptr) {
    const int lane = lane_id();
    const int capl = g.layers[l].cap;
    int32_t* row = g.layers[l].adj + (size_t)n * capl;
    const int32_t rv = lane < capl ? ld_i32<true>(row + lane) : -1;
    int d = uni(ld_i32<true>(g.layers[l].deg + n));
    if (d < 0) d = 0;  // graph.go:46-48 allocate the map
    const bool pres = lane < d && kid_of(g, guard_id(g, (uint32_t)rv)) == kid_of(g, nw);
    const unsigned long long pm = __ballot(pres);
    const bool present = pm != 0;
    const int pos = present ? __ffsll((long long)pm) - 1 : d;
    const int nd = uni(present ? d : d + 1);  // (computed outside the lane-0 stores: stays scalar)
    ev.sync();
    if (lane == 0) {
        st_i32(row + pos, (int32_t)nw);
        st_i32(g.layers[l].deg + n, nd);
    }
    ev.sync();
    if (rowout) *rowout = lane == pos ? (int32_t)nw : rv;
    return nd;
}

// graph.go:172-219 when the outcome does not depend on the walk order.  With
// one row per key (no replaced keys: g.kid == nullptr) the candidates are a SET
// -- neighbours of neighbours, minus n and its neighbours, one per key -- and
// when the pops it takes are strict minima (no NaN, no tie at any pop) every
// heap shape pops the same rows in the same order.  So: stage the rows without
// their keys, collect the set through the visited table in any lane order,
// score it, and check the pops before making any of them.  Returns false
// (nothing changed) when a NaN or a tie needs the reference's exact push
// order; replenish then takes the ordered walk.
template <class C, int G, class Ev>
__device__ __forceinline__ bool replenish_set(const GraphDev& g, int l, uint32_t n, int m, int dn, int32_t rv, BuildSmem& S,
                              WaveStats& st, int& err, const Ev& ev) {
    const int lane = lane_id();
    const int capl = g.layers[l].cap;
    const uint32_t mine = lane < dn ? guard_id(g, (uint32_t)rv) : 0u;
    const int mydeg = lane < dn ? min(ld_i32<true>(g.layers[l].deg + mine), capl) : -1;
    const int tot = min(dn * capl, S.hcap);
    const int vsize = 1 << S.cs.vlog2, vmask = vsize - 1;
    vis_clear(S.cs.vis, vsize);
    ev.sync();
    if (lane == 0) vis_probe(S.cs.vis, vmask, n);     // graph.go:184
    if (lane < dn) vis_probe(S.cs.vis, vmask, mine);  // graph.go:187-189
    ev.sync();
    int ncand = 0;
    constexpr int U = 4;  // rows' entries in flight per pass
    for (int e0 = 0; e0 < tot; e0 += 64 * U) {
        int32_t x[U];
        int dj[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {  // uniform trip count: the shuffles see every lane
            const int e = e0 + u * 64 + lane;
            const int j = min(e / capl, 63), i = e % capl;
            const uint32_t nb = shfl_u(mine, j);
            x[u] = e < tot && j < dn ? ld_i32<true>(g.layers[l].adj + (size_t)nb * capl + i) : -1;
            dj[u] = __shfl(mydeg, j, 64);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = e0 + u * 64 + lane;
            const int i = e % capl;
            uint32_t v = EMPTY_ID;
            if (e < tot && i < dj[u]) v = guard_id(g, (uint32_t)x[u]);
            int pr = 0;
            if (v != EMPTY_ID) pr = vis_probe(S.cs.vis, vmask, v);  // graph.go:198-201
            if (__ballot(pr == 2)) err = 1;
            int cnt;
            const uint32_t cid = compact(v, pr == 1, cnt);
            if (ncand + cnt > S.hcap) {
                err |= 8;
                cnt = S.hcap - ncand;
            }
            if (lane < cnt) ev.list[ncand + lane] = cid;
            ncand += cnt;
        }
    }
    ev.sync();
    st.E += ncand;
    CPROF_CNT(19, ncand);
    {
        QReg<C> q;
        load_query(q, g.vecs + (size_t)n * g.pitch);
        ev.template score<C, G>(g, q, g.norms[n], ncand, COSINE, S.hd, S.hi);  // graph.go:204 hard-coded cosine
    }
    ev.sync();
    bool anynan = false;
    for (int e = lane; e < ncand; e += 64) anynan |= !(S.hd[e] == S.hd[e]);
    const int need = min(m - dn, ncand);  // each pop adds a new key: deg grows by one
    if (__ballot(anynan) || need > 64) return false;
    uint32_t popped = 0xFFFFFFFFu;  // lane p: the candidate index of pop p
    for (int p = 0; p < need; ++p) {
        float mv = __int_as_float(0x7f800000);
        int mi = -1;
        for (int e = lane; e < ncand; e += 64) {
            bool gone = false;
            for (int j = 0; j < p; ++j) gone |= rl_u(popped, j) == (uint32_t)e;
            const float v = S.hd[e];
            if (!gone && (mi < 0 || v < mv)) {
                mv = v;
                mi = e;
            }
        }
        float wm = mi < 0 ? __int_as_float(0x7f800000) : mv;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) wm = fminf(wm, __shfl_xor(wm, o, 64));
        int eq = 0;
        for (int e = lane; e < ncand; e += 64) {
            bool gone = false;
            for (int j = 0; j < p; ++j) gone |= rl_u(popped, j) == (uint32_t)e;
            eq += (!gone && S.hd[e] == wm) ? 1 : 0;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) eq += __shfl_xor(eq, o, 64);
        if (eq != 1) return false;  // a tie: the heap's shape decides
        const unsigned long long own = __ballot(mi >= 0 && mv == wm);
        const int bi = __shfl(mi, __ffsll((long long)own) - 1, 64);
        if (lane == p) popped = (uint32_t)bi;
    }
    CPROF_CNT(15, 1);
    for (int p = 0; p < need; ++p) list_append(g, l, n, S.hi[rl_u(popped, p)], ev);  // graph.go:213-218
    return true;
}

// graph.go:172-219.  The neighbours' rows and keys are staged in LDS in one
// pass (instead of one dependent load chain per neighbour); the candidates are
// then collected in the reference's walk order (neighbours, then their
// neighbours, both in ascending key order -- the map-order stand-in) for all
// rows at once, and ONE distance batch scores them all; the heap sees the
// pushes in the same order as a per-neighbour loop would produce.
template <class C, int G, class Ev>
__device__ __forceinline__ void replenish(const GraphDev& g, int l, uint32_t n, int m, BuildSmem& S, WaveStats& st, int& err,
                          const Ev& ev, const int32_t* known_row = nullptr, int known_deg = 0) {
    const int lane = lane_id();
    const int capl = g.layers[l].cap;
    // n's row and degree: from the caller's registers when it just changed them
    const int32_t rv = known_row ? *known_row : lane < capl ? ld_i32<true>(g.layers[l].adj + (size_t)n * capl + lane) : -1;
    int dn = known_row ? known_deg : uni(ld_i32<true>(g.layers[l].deg + n));
    if (dn < 0) dn = 0;
    if (dn >= m) return;
    CPROF_T(tr);
    CPROF_CNT(18, 1);
    if (!g.kid) {
        const bool done = replenish_set<C, G>(g, l, n, m, dn, rv, S, st, err, ev);
        CPROF_ADD(tr, 14);
        if (done) return;
        CPROF_CNT(20, 1);
    }
    uint32_t mine = 0xFFFFFFFFu;
    int64_t key = INT64_MAX;
    if (lane < dn) {
        mine = guard_id(g, (uint32_t)rv);
        key = g.keys[mine];
    }
    rank_sort(key, mine, dn);
    // stage every neighbour's row (deg, entries, keys) -- rows j < dn, j-major
    const int mydeg = lane < dn ? min(ld_i32<true>(g.layers[l].deg + mine), capl) : -1;
    const int tot = min(dn * capl, S.hcap);
    for (int e0 = 0; e0 < tot; e0 += 64) {  // uniform trip count: the shuffles see every lane
        const int e = e0 + lane;
        const int j = min(e / capl, 63), i = e % capl;
        const uint32_t nb = shfl_u(mine, j);
        // the entry load goes out before the degree is needed (masked below)
        const int32_t ev_ = e < tot && j < dn ? ld_i32<true>(g.layers[l].adj + (size_t)nb * capl + i) : -1;
        const int dj = __shfl(mydeg, j, 64);
        uint32_t th = 0xFFFFFFFFu;
        int64_t tk = INT64_MAX;
        if (e < tot && i < dj) {
            th = guard_id(g, (uint32_t)ev_);
            tk = g.keys[th];
        }
        if (e < tot) {
            S.radj[e] = th;
            S.rkey[e] = tk;
        }
    }
    ev.sync();
    CPROF_ADD(tr, 5);
    // The reference's walk (graph.go:184-210): visited = {n} + n's neighbours;
    // then each neighbour j in key order, each of its neighbours in key order,
    // collecting the ones not yet visited.  All rows at once: (1) every entry's
    // rank in its row's key order gives its walk position j*capl + rank in
    // S.hi (EMPTY past the row's degree); (2) a walk entry is collected when it
    // is not n, not one of n's neighbours and not seen at an earlier position.
    uint32_t* W = S.hi;
    for (int e0 = 0; e0 < tot; e0 += 64) {  // uniform trip count for the shuffle
        const int e = e0 + lane;
        const int j = min(e / capl, 63), i = e % capl;
        const int dj = __shfl(mydeg, j, 64);
        if (e < tot) {
            const uint32_t v = S.radj[e];
            const int64_t kv = S.rkey[e];
            const int row = j * capl;
            if (i < dj) {
                int r = 0;
#pragma unroll 8
                for (int i2 = 0; i2 < dj && row + i2 < tot; ++i2) {
                    const int64_t k2 = S.rkey[row + i2];
                    const uint32_t v2 = S.radj[row + i2];
                    r += (k2 < kv || (k2 == kv && (v2 < v || (v2 == v && i2 < i)))) ? 1 : 0;
                }
                W[row + r] = v;
            } else {
                W[e] = EMPTY_ID;
            }
        }
    }
    ev.sync();
    CPROF_ADD(tr, 6);
    const int vsize = 1 << S.cs.vlog2, vmask = vsize - 1;
    vis_clear(S.cs.vis, vsize);
    ev.sync();
    if (lane == 0) vis_probe(S.cs.vis, vmask, kid_of(g, n));     // graph.go:184 visited[n.Key]
    if (lane < dn) vis_probe(S.cs.vis, vmask, kid_of(g, mine));  // graph.go:187-189
    ev.sync();
    int ncand = 0;
    for (int e0 = 0; e0 < tot; e0 += 64) {  // 64 walk positions at a time, in order
        const int e = e0 + lane;
        const uint32_t v = e < tot ? W[e] : EMPTY_ID;
        const uint32_t kv = v != EMPTY_ID ? kid_of(g, v) : EMPTY_ID;  // graph.go:198 visited[k]: by key
        bool first = v != EMPTY_ID;  // not repeated at a lower lane of this chunk
#pragma unroll 9
        for (int l2 = 0; l2 < 63; ++l2) first = first && !(l2 < lane && rl_u(kv, l2) == kv);
        int pr = 0;
        if (first) pr = vis_probe(S.cs.vis, vmask, kv);  // earlier chunks and the pre-visited set
        if (__ballot(pr == 2)) err = 1;
        int cnt;
        const uint32_t cid = compact(v, pr == 1, cnt);
        if (ncand + cnt > S.hcap) {
            err |= 8;
            cnt = S.hcap - ncand;
        }
        if (lane < cnt) ev.list[ncand + lane] = cid;
        ncand += cnt;
    }
    ev.sync();
    CPROF_ADD(tr, 7);
    CPROF_CNT(19, ncand);
    st.E += ncand;
    // distances in push order (the reference pushes each into its heap)
    {
        QReg<C> q;
        load_query(q, g.vecs + (size_t)n * g.pitch);
        const float qn = g.norms[n];
        ev.template score<C, G>(g, q, qn, ncand, COSINE, S.hd, S.hi);  // graph.go:204 hard-coded cosine
    }
    ev.sync();
    CPROF_ADD(tr, 8);
    // graph.go:213-218 (len < m before every add: addNeighbor cannot evict).
    // Every Pop returns the heap's minimum.  While no distance is NaN and the
    // minimum of what is left is unique, that is the arg-min whatever shape
    // the heap has, so the pushes are skipped.  Otherwise the heap is built in
    // place by replaying the pushes (element e of the push-order array is the
    // e-th push), the pops made so far are replayed, and the walk continues on
    // the heap exactly as the reference's.
    bool anynan = false;
    for (int e = lane; e < ncand; e += 64) anynan |= !(S.hd[e] == S.hd[e]);
    bool fast = __ballot(anynan) == 0ull;
    uint32_t popped = 0xFFFFFFFFu;  // fast path: lane j holds the index of the j-th pop
    int npop = 0;
    GHeap h{S.hd, S.hi, 0};
    auto gone = [&](int e) {
        bool r = false;
        for (int j = 0; j < npop; ++j) r |= rl_u(popped, j) == (uint32_t)e;
        return r;
    };
    auto replay = [&]() {
        for (int e = 0; e < ncand; ++e) {
            h.n = e + 1;
            gh_up(h, e);
        }
        for (int j = 0; j < npop; ++j) {
            float bd;
            uint32_t bb;
            gh_pop(h, bd, bb);
        }
        fast = false;
    };
    if (!fast) replay();
    for (;;) {
        int cur = uni(ld_i32<true>(g.layers[l].deg + n));
        if (cur < 0) cur = 0;
        if (cur >= m) break;
        uint32_t best;
        if (fast) {
            if (npop >= ncand) break;
            float mv = __int_as_float(0x7f800000);
            int mi = -1;
            for (int e = lane; e < ncand; e += 64) {
                const float v = S.hd[e];
                if (!gone(e) && (mi < 0 || v < mv)) {
                    mv = v;
                    mi = e;
                }
            }
            float wm = mi < 0 ? __int_as_float(0x7f800000) : mv;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) wm = fminf(wm, __shfl_xor(wm, o, 64));
            int eq = 0;
            for (int e = lane; e < ncand; e += 64) eq += (!gone(e) && S.hd[e] == wm) ? 1 : 0;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) eq += __shfl_xor(eq, o, 64);
            if (eq == 1 && npop < 64) {
                const unsigned long long own = __ballot(mi >= 0 && mv == wm);
                const int bi = __shfl(mi, __ffsll((long long)own) - 1, 64);
                best = S.hi[bi];
                if (lane == npop) popped = (uint32_t)bi;
                ++npop;
            } else {
                replay();  // a tie at the minimum: the heap's shape decides
            }
        }
        if (!fast) {
            if (h.n <= 0) break;
            float bd;
            gh_pop(h, bd, best);
        }
        list_append(g, l, n, best, ev);
    }
    CPROF_ADD(tr, 9);
}

// What add_neighbor(n, nw) needs from before its own append, staged for the
// whole neighbourhood at once (compat_insert): n's row and degree, and the
// distance from n to each entry (entry deg: to nw).
struct EvictSpec {
    const int32_t* row;
    int deg;
    const float* dist;
};

// graph.go:41-81.  Returns the evicted neighbour (EMPTY_ID: none).
template <class C, int G, class Ev>
__device__ __forceinline__ uint32_t add_neighbor(const GraphDev& g, int l, uint32_t n, uint32_t nw, int m, BuildSmem& S,
                                                 WaveStats& st, int& err, const Ev& ev,
                                                 bool have_sp = false, EvictSpec sp = {}) {
    const int lane = lane_id();
    const int capl = g.layers[l].cap;
    int32_t rv;
    int d;
    float worst_d = -__int_as_float(0x7f800000);
    uint32_t worst = EMPTY_ID;
    bool decided = false;
    CPROF_T(ta);
    QReg<C> q;
    float qn = 0.f;
    if (have_sp) {
        // the append of list_append from the staged row (graph.go:50), then the
        // staged distances: entry i of the row after it is the old entry i, or
        // nw where nw went (the slot of its key, else slot deg)
        const int d0 = sp.deg < 0 ? 0 : sp.deg;  // graph.go:46-48 allocate the map
        const int32_t r0 = lane < capl ? sp.row[lane] : -1;
        const bool pres = lane < d0 && kid_of(g, guard_id(g, (uint32_t)r0)) == kid_of(g, nw);
        const unsigned long long pm = __ballot(pres);
        const int pos = pm ? __ffsll((long long)pm) - 1 : d0;
        d = uni(pm ? d0 : d0 + 1);
        ev.sync();
        if (lane == 0) {
            st_i32(g.layers[l].adj + (size_t)n * capl + pos, (int32_t)nw);
            st_i32(g.layers[l].deg + n, d);
        }
        ev.sync();
        rv = lane == pos ? (int32_t)nw : r0;
        CPROF_ADD(ta, 1);
        if (d <= m) return EMPTY_ID;
        CPROF_CNT(17, 1);
        st.E += d;
        const float dl = lane < d ? sp.dist[lane == pos ? d0 : lane] : -__int_as_float(0x7f800000);
        const bool nan = __ballot(lane < d && !(dl == dl)) != 0ull;
        float wm = dl;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) wm = fmaxf(wm, __shfl_xor(wm, o, 64));
        const unsigned long long at = __ballot(lane < d && dl == wm);
        if (!nan && __popcll(at) == 1) {  // a unique maximum: the map order is irrelevant
            worst = (uint32_t)guard_id(g, (uint32_t)__shfl(rv, __ffsll((long long)at) - 1, 64));
            worst_d = wm;
            decided = true;
        } else {
            load_query(q, g.vecs + (size_t)n * g.pitch);
            qn = g.norms[n];
        }
    } else {
        // n's row goes out with the append's loads (one round trip for both; most
        // appends overflow the row and evict)
        load_query(q, g.vecs + (size_t)n * g.pitch);
        qn = g.norms[n];
        d = list_append(g, l, n, nw, ev, &rv);
        CPROF_ADD(ta, 1);
        if (d <= m) return EMPTY_ID;
        CPROF_CNT(17, 1);
        st.E += d;
    }
    uint32_t nb = lane < d ? guard_id(g, (uint32_t)rv) : 0xFFFFFFFFu;
    if (!decided) {
        // graph.go:60-71 takes the first maximum in map order.  A unique maximum and
        // no NaN make the order irrelevant: score the row as it lies, and rank it
        // by key (the map-order stand-in) only when a tie or a NaN needs it.
        int nmax = 0;
        bool nan = false;
        if (!have_sp) {
            ev.template run<C, G>(g, q, qn, nb, d, g.metric, [&](float dd, uint32_t u) {
                nan |= !(dd == dd);
                if (dd > worst_d || worst == EMPTY_ID) {
                    worst_d = dd;
                    worst = u;
                    nmax = 1;
                } else if (dd == worst_d) {
                    ++nmax;
                }
            });
        }
        if (have_sp || nan || nmax > 1) {
            int64_t key = lane < d ? g.keys[nb] : INT64_MAX;
            rank_sort(key, nb, d);  // Go map order -> ascending key
            worst_d = -__int_as_float(0x7f800000);
            worst = EMPTY_ID;
            st.E += d;
            ev.template run<C, G>(g, q, qn, nb, d, g.metric, [&](float dd, uint32_t u) {  // graph.go:60-71
                if (dd > worst_d || worst == EMPTY_ID) {
                    worst_d = dd;
                    worst = u;
                }
            });
        }
    }
    CPROF_ADD(ta, 2);
    if (worst == EMPTY_ID) return EMPTY_ID;
    {
        int dd = d;
        list_remove_in(g, l, n, rv, dd, worst, ev);  // graph.go:74 (n's row is in registers since the append)
    }
    // worst's row, read after that removal (worst may be n itself)
    int32_t wrow = lane < capl ? ld_i32<true>(g.layers[l].adj + (size_t)worst * capl + lane) : -1;
    int wdeg = uni(ld_i32<true>(g.layers[l].deg + worst));
    if (wdeg >= 0) list_remove_in(g, l, worst, wrow, wdeg, n, ev);  // graph.go:76-78
    CPROF_ADD(ta, 3);
    replenish<C, G>(g, l, worst, m, S, st, err, ev, &wrow, wdeg);  // graph.go:79
    CPROF_ADD(ta, 4);
    return worst;
}

// Stage EvictSpec for add_neighbor(c_j, nw), j < cnt (lane j of nbh: c_j): the
// rows as they stand now, and one MW_PAIRS batch of every entry's distance to
// its row's owner plus nw's.  False when the staging area is too small (then
// every pair takes the plain path).
template <class C, int G, class Ev>
__device__ __forceinline__ bool stage_evictions(const GraphDev& g, int l, uint32_t nbh, int cnt, uint32_t nw,
                                                BuildSmem& S, const Ev& ev) {
    const int lane = lane_id();
    const int capl = g.layers[l].cap;
    if (!S.prow || cnt > S.pgroups || capl + 1 > S.pstride || cnt <= 0) return false;
    const int ps = S.pstride;
    const int tot = cnt * capl;
    for (int e0 = 0; e0 < tot; e0 += 64) {  // uniform trip count: the shuffles see every lane
        const int e = e0 + lane;
        const int j = min(e / capl, 63), i = e % capl;
        const uint32_t c = shfl_u(nbh, j);
        if (e < tot) S.prow[j * ps + i] = ld_i32<true>(g.layers[l].adj + (size_t)c * capl + i);
    }
    const int dj = lane < cnt ? ld_i32<true>(g.layers[l].deg + guard_id(g, nbh)) : -1;  // lane j: c_j's degree
    if (lane < cnt) S.pdeg[lane] = dj;
    ev.sync();
    // the pairs table: entries of row j (past its degree: none), then nw
    for (int e0 = 0; e0 < cnt * ps; e0 += 64) {
        const int e = e0 + lane;
        const int j = min(e / ps, 63), i = e % ps;
        const int djj = __shfl(dj, j, 64);
        const int dd = djj < 0 ? 0 : min(djj, capl);
        if (e < cnt * ps && i < dd) ev.pc[e] = (int32_t)guard_id(g, (uint32_t)S.prow[j * ps + i]);
        if (e < cnt * ps && i == dd) ev.pc[e] = (int32_t)nw;
    }
    if (lane < cnt) {
        ev.pq[lane] = nbh;
        ev.pn[lane] = (dj < 0 ? 0 : min(dj, capl)) + 1;
    }
    ev.sync();
    ev.template pairs<C, G>(g, cnt, g.metric);
    return true;
}

// graph.go:221-235 isolate: neighbours in ascending key order (the map-order
// stand-in) drop their backlink and are replenished; the deleted node's own
// row stays (the reference keeps the layerNode behind one-directional edges).
template <class C, int G, class Ev>
__device__ __forceinline__ void isolate(const GraphDev& g, int l, uint32_t n, int m, BuildSmem& S, WaveStats& st, int& err,
                        const Ev& ev) {
    const int lane = lane_id();
    const int capl = g.layers[l].cap;
    const int dn = min(uni(ld_i32<true>(g.layers[l].deg + n)), capl);
    if (dn < 0) return;  // nil neighbour map
    uint32_t mine = 0xFFFFFFFFu;
    int64_t key = INT64_MAX;
    if (lane < dn) {
        mine = guard_id(g, (uint32_t)ld_i32<true>(g.layers[l].adj + (size_t)n * capl + lane));
        key = g.keys[mine];
    }
    rank_sort(key, mine, dn);
    for (int j = 0; j < dn; ++j) {
        const uint32_t x = rl_u(mine, j);
        int32_t xrow = lane < capl ? ld_i32<true>(g.layers[l].adj + (size_t)x * capl + lane) : -1;
        int xdeg = uni(ld_i32<true>(g.layers[l].deg + x));
        if (xdeg < 0) continue;                            // neighbor.neighbors == nil
        list_remove_in(g, l, x, xrow, xdeg, n, ev);        // graph.go:232 delete(neighbor.neighbors, n.Key)
        replenish<C, G>(g, l, x, m, S, st, err, ev, &xrow, xdeg);  // graph.go:232
    }
}

// ---- multi-wave evaluator ----------------------------------------------------
// Protocol block in LDS.  The master posts a batch (query registers, ids,
// metric) and hits a workgroup barrier; every wave scores its share of the
// rows into dist[]; a second barrier hands the distances back.  Workers sit in
// mw_worker's loop between the two barriers until the master posts EXIT.
struct MwHdr {
    int cmd, cnt, metric;
    float qn;
};
constexpr int MW_EVAL = 0, MW_EXIT = 1, MW_PAIRS = 2;

// Everything exchanged here lives in LDS (workers read only immutable rows from
// HBM), so the fences order LDS alone: the master's graph stores are not waited
// for at every hand-off.
__device__ __forceinline__ void mw_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// rows [0, cnt) of ids, wave w of nw: canonical distances into dist[]
template <class C, int G>
__device__ __forceinline__ void mw_share(const GraphDev& g, const QReg<C>& q, float qn, const uint32_t* ids,
                                         float* dist, int cnt, int metric, int w, int nw) {
    using RM = RowMap<C, G>;
    constexpr int GROUP = C::LPR >> RM::LG;
    const int lane = lane_id();
    for (int base = w * RM::T; base < cnt; base += nw * RM::T) {
        uint32_t rid[G];
        bool valid[G];
#pragma unroll
        for (int gg = 0; gg < G; ++gg) {
            const int t = base + RM::reg_row(gg, lane);
            valid[gg] = t < cnt;
            rid[gg] = valid[gg] ? guard_id(g, ids[t]) : 0u;
        }
        const float s = metric == EUCLIDEAN ? eval_rows<C, G, true>(q, g.vecs, g.pitch, rid, valid)
                                            : eval_rows<C, G, false>(q, g.vecs, g.pitch, rid, valid);
        const int town = base + RM::owned_row(lane);
        if (town < cnt && (lane & (GROUP - 1)) == 0) {
            const float xn = metric == COSINE ? g.norms[guard_id(g, ids[town])] : 1.f;
            dist[town] = finalize(metric, s, xn, qn);
        }
    }
}

template <class C>
struct MwEval {
    static constexpr bool kPairs = true;
    MwHdr* hdr;
    float4* qbuf;     // [VPL * 64] the master's query registers, lane-major
    uint32_t* list;   // ids of the posted batch (also replenish's candidate list)
    float* dist;      // [cap] distances back
    int nw;
    // MW_PAIRS: group j scores rows pc[j * ps, + pn[j]) against row pq[j] into pd
    uint32_t* pq = nullptr;
    int* pn = nullptr;
    int32_t* pc = nullptr;
    float* pd = nullptr;
    int ps = 0;
    template <class C2, int G, class Sink>
    __device__ __forceinline__ void run_list(const GraphDev& g, const QReg<C2>& q, float qn, int cnt, int metric,
                                             Sink&& sink, bool sinks = true) const {
        if (cnt <= 0) return;
        const int lane = lane_id();
#pragma unroll
        for (int v = 0; v < C2::VPL; ++v) qbuf[v * 64 + lane] = q.v[v];
        if (lane == 0) {
            hdr->cmd = MW_EVAL;
            hdr->cnt = cnt;
            hdr->metric = metric;
            hdr->qn = qn;
        }
        CPROF_T(tp);
        mw_barrier();  // post
        mw_share<C2, G>(g, q, qn, list, dist, cnt, metric, 0, nw);
        mw_barrier();  // collect
        CPROF_ADD(tp, 11);
        // the results go through registers: the sink loop reads lanes, not LDS
        for (int b = 0; sinks && b < cnt; b += 64) {
            const int c = min(64, cnt - b);
            const float dv = lane < c ? dist[b + lane] : 0.f;
            const uint32_t iv = lane < c ? list[b + lane] : 0u;
            for (int t = 0; t < c; ++t) sink(rl_f(dv, t), rl_u(iv, t));
        }
        CPROF_ADD(tp, 12);
    }
    template <class C2, int G, class Sink>
    __device__ __forceinline__ void run(const GraphDev& g, const QReg<C2>& q, float qn, uint32_t cid, int cnt,
                                        int metric, Sink&& sink) const {
        if (cnt <= 0) return;
        if (lane_id() < cnt) list[lane_id()] = cid;
        run_list<C2, G>(g, q, qn, cnt, metric, sink);
    }
    // rows list[0, cnt): distance e into outd[e], the row into outi[e]
    template <class C2, int G>
    __device__ __forceinline__ void score(const GraphDev& g, const QReg<C2>& q, float qn, int cnt, int metric,
                                          float* outd, uint32_t* outi) const {
        run_list<C2, G>(g, q, qn, cnt, metric, [](float, uint32_t) {}, false);
        for (int e = lane_id(); e < cnt; e += 64) {
            outd[e] = dist[e];
            outi[e] = list[e];
        }
    }
    // every group j of the posted pairs table scored by the waves (pq / pn / pc
    // written by the caller), distances into pd
    template <class C2, int G>
    __device__ __forceinline__ void pairs(const GraphDev& g, int ngroups, int metric) const;
    // the master's own lanes only (workers never touch graph state)
    __device__ __forceinline__ void sync() const { wave_sync(); }
};

// MW_PAIRS, wave w of nw: whole groups j = w, w + nw, ... (each group's rows
// against its own owner row, loaded here)
template <class C, int G>
__device__ __forceinline__ void mw_pairs_share(const GraphDev& g, const MwEval<C>& ev, int ngroups, int metric, int w,
                                               int nw) {
    for (int j = w; j < ngroups; j += nw) {
        const uint32_t o = guard_id(g, uni(ev.pq[j]));
        QReg<C> q;
        load_query(q, g.vecs + (size_t)o * g.pitch);
        mw_share<C, G>(g, q, g.norms[o], reinterpret_cast<const uint32_t*>(ev.pc) + (size_t)j * ev.ps,
                       ev.pd + (size_t)j * ev.ps, uni(ev.pn[j]), metric, 0, 1);
    }
}

template <class C, int G>
__device__ __forceinline__ void mw_worker(const GraphDev& g, const MwEval<C>& ev, int w) {
    for (;;) {
        mw_barrier();
        const int cmd = ev.hdr->cmd;
        if (cmd == MW_EXIT) break;
        if (cmd == MW_PAIRS) {
            mw_pairs_share<C, G>(g, ev, ev.hdr->cnt, ev.hdr->metric, w, ev.nw);
        } else {
            QReg<C> q;
            const int lane = lane_id();
#pragma unroll
            for (int v = 0; v < C::VPL; ++v) q.v[v] = ev.qbuf[v * 64 + lane];
            mw_share<C, G>(g, q, ev.hdr->qn, ev.list, ev.dist, ev.hdr->cnt, ev.hdr->metric, w, ev.nw);
        }
        mw_barrier();
    }
}

template <class C>
template <class C2, int G>
__device__ __forceinline__ void MwEval<C>::pairs(const GraphDev& g, int ngroups, int metric) const {
    if (ngroups <= 0) return;
    if (lane_id() == 0) {
        hdr->cmd = MW_PAIRS;
        hdr->cnt = ngroups;
        hdr->metric = metric;
    }
    mw_barrier();  // post
    mw_pairs_share<C, G>(g, *this, ngroups, metric, 0, nw);
    mw_barrier();  // collect
}

// The sequential kernels re-read a layer's descriptor (row cap, adjacency and
// degree arrays) at every step of the walk; from HBM each read is one more
// dependent round trip (vector loads: the walk's own stores could alias the
// table, so the scalar cache is out).  A copy in LDS makes it a few dozen
// cycles.  Returns the graph view to walk with.
__device__ __forceinline__ GraphDev lds_layers(const GraphDev& g, LayerDev* tab) {
    for (int i = threadIdx.x; i < g.nlayers; i += blockDim.x) tab[i] = g.layers[i];
    __syncthreads();
    GraphDev v = g;
    v.layers = tab;
    return v;
}

// LDS of the compat walks: visited set, compat heaps, replenish heap + staging
__device__ __forceinline__ uint32_t* build_smem(uint32_t* p, int vis_log2, int M, int ef, BuildSmem& S) {
    S.cs.vis = p;
    S.cs.vlog2 = vis_log2;
    p += 1 << vis_log2;
    S.cs.cd = reinterpret_cast<float*>(p);
    p += ef + 2;
    S.cs.ci = p;
    p += ef + 2;
    S.cs.rd = reinterpret_cast<float*>(p);
    p += M + 2;
    S.cs.ri = p;
    p += M + 2;
    const int hcap = (M + 1) * (M + 1) + 2;  // >= any neighbours-of-neighbours list
    S.hcap = hcap;
    S.hd = reinterpret_cast<float*>(p);
    p += hcap;
    S.hi = p;
    p += hcap;
    S.radj = p;
    p += hcap;
    p += (reinterpret_cast<uintptr_t>(p) & 4) ? 1 : 0;  // 8-B align
    S.rkey = reinterpret_cast<int64_t*>(p);
    p += 2 * hcap;
    return p;
}
__host__ __device__ constexpr size_t build_smem_words(int vis_log2, int M, int ef) {
    return ((size_t)1 << vis_log2) + 2 * (size_t)(ef + 2) + 2 * (size_t)(M + 2) + 5 * (size_t)((M + 1) * (M + 1) + 2) + 1;
}

// One insert of graph.go:942-1042 (BatchAdd; Add is the same walk), by the
// master wave.  Rows: id_a for the layers above i0, id_b from i0 down (the same
// row for a fresh key).  ent[l]: the layer's entry() at its turn, or the
// inserted row itself when the layer is empty then (graph.go:990-993).  i0 >= 0
// (a present key, graph.go:1015-1024): after layer i0's search every layer
// holding the key deletes and isolates it (sweep[l], ascending), and the key's
// live row becomes id_b.  Returns false on the reference's "no nodes found in
// neighborhood search" (layer in *fail_layer).
template <class C, int G, class Ev>
__device__ __forceinline__ bool compat_insert(const CompatBuildArgs& a, BuildSmem& S, const Ev& ev, WaveStats& st, int& err,
                              int level, int top, uint32_t id_a, uint32_t id_b, int i0, const int32_t* ent,
                              const int32_t* sweep, int& fail_layer) {
    const int lane = lane_id();
    QReg<C> q;
    load_query(q, a.g.vecs + (size_t)id_b * a.g.pitch);
    const float qn = a.g.norms[id_b];
    uint32_t elevator = EMPTY_ID;
    for (int l = top; l >= 0; --l) {  // graph.go:980
        const uint32_t id = l > i0 ? id_a : id_b;
        if (ent[l] == (int32_t)id) {  // graph.go:990-993: empty layer, no search
            ev.sync();
            if (lane == 0) st_i32(a.g.layers[l].deg + id, -1);
            ev.sync();
            continue;
        }
        // graph.go:997-1003: layer.nodes[*elevator] -- nil once that key has no node here
        uint32_t sp = ent[l] < 0 ? EMPTY_ID : (uint32_t)ent[l];
        if (elevator != EMPTY_ID) sp = resolve_member<true>(a.g, l, elevator);
        int cnt = 0;
        CPROF_T(ts);
        if (sp != EMPTY_ID) cnt = compat_layer<C, G, true>(a.g, l, sp, a.M, a.ef, q, qn, S.cs, st, err, ev);  // :1005
        CPROF_ADD(ts, 0);
        if (cnt == 0) {  // search(nil) -> "no nodes found in neighborhood search"
            fail_layer = l;
            return false;
        }
        elevator = S.cs.ri[0];  // graph.go:1013
        if (level >= l) {       // graph.go:1015-1032
            const uint32_t nbh = lane < cnt ? S.cs.ri[lane] : 0u;
            if (l == i0) {
                CPROF_T(ti);
                for (int l2 = 0; l2 < a.g.nlayers; ++l2)  // graph.go:1018-1023
                    if (sweep[l2] >= 0) isolate<C, G>(a.g, l2, (uint32_t)sweep[l2], a.M, S, st, err, ev);
                ev.sync();
                if (lane == 0) st_i32(a.g.kidlive + kid_of(a.g, id_b), (int32_t)id_b);
                CPROF_ADD(ti, 10);
            }
            ev.sync();
            if (lane == 0) st_i32(a.g.layers[l].deg + id, -1);
            ev.sync();
            CPROF_T(tn);
            // Eviction speculation: the neighbourhood's rows and their distances
            // are staged in one batch; pair j uses them unless an earlier pair of
            // this loop changed c_j's row -- which only an eviction of c_j does
            // (an addNeighbor pair writes its own two rows, and the evicted row
            // with its replenish): then it reads the row as usual.
            bool staged = false;
            if constexpr (Ev::kPairs) staged = stage_evictions<C, G>(a.g, l, nbh, cnt, id, S, ev);
            uint32_t evicted = EMPTY_ID;  // lane k: the k-th row evicted in this loop
            int nev = 0;
            for (int j = 0; j < cnt; ++j) {
                const uint32_t c = rl_u(nbh, j);
                const bool fresh = staged && nev < 64 && __ballot(lane < nev && evicted == c) == 0ull;
                // the staged row is read only when fresh (S.pdeg / S.prow are null without staging)
                const EvictSpec sp = fresh ? EvictSpec{S.prow + j * S.pstride, uni(S.pdeg[j]), S.pdist + j * S.pstride}
                                           : EvictSpec{nullptr, 0, nullptr};
                const uint32_t w1 = add_neighbor<C, G>(a.g, l, c, id, a.M, S, st, err, ev, fresh, sp);
                if (w1 != EMPTY_ID) {
                    if (lane == nev) evicted = w1;
                    ++nev;
                }
                const uint32_t w2 = add_neighbor<C, G>(a.g, l, id, c, a.M, S, st, err, ev);
                if (w2 != EMPTY_ID) {
                    if (lane == nev) evicted = w2;
                    ++nev;
                }
            }
            CPROF_ADD(tn, 13);
        }
    }
    return true;
}

// graph.go:942-1042 for the fresh inserts [n0, n1), then the replacing insert
// (a.rep_level >= 0), in order; the first failing insert ends the walk
template <class C, int G, class Ev>
__device__ __forceinline__ void compat_inserts(const CompatBuildArgs& a, BuildSmem& S, const Ev& ev, WaveStats& st, int& err) {
    int top = a.top0;
    int fail_layer = -1;
    int64_t fail_row = -1;
    for (int64_t i = a.n0; i < a.n1; ++i) {
        const uint32_t id = (uint32_t)i;
        const int level = a.levels[i];
        top = max(top, level);
        if (!compat_insert<C, G>(a, S, ev, st, err, level, top, id, id, -1, a.layer_entry, a.rep_sweep,
                                 fail_layer)) {
            fail_row = i;
            break;
        }
        if (err) break;
    }
    if (fail_row < 0 && !err && a.rep_level >= 0) {
        top = max(top, a.rep_level);
        if (!compat_insert<C, G>(a, S, ev, st, err, a.rep_level, top, a.rep_a, a.rep_b, a.rep_i0, a.rep_entry,
                                 a.rep_sweep, fail_layer))
            fail_row = a.rep_b;
    }
    if (fail_row >= 0) {
        err |= 2;
        if (lane_id() == 0) {
            a.err[2] = fail_layer;
            a.err[3] = (int)fail_row;
        }
    }
}

template <class C, int G>
__global__ __launch_bounds__(64) void k_build_compat(CompatBuildArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    __shared__ LayerDev ltab[MH_MAXL];
    a.g = lds_layers(a.g, ltab);
    BuildSmem S;
    uint32_t* p = build_smem(smem, a.vis_log2, a.M, a.ef, S);
    WaveEval ev;
    ev.list = p;
    WaveStats st;
    int err = 0;
    compat_inserts<C, G>(a, S, ev, st, err);
    if (lane_id() == 0) {
        atomicAdd(&a.stats[0], st.E);
        atomicAdd(&a.stats[1], st.X);
        if (err) atomicOr(a.err, err);
    }
}

// The same walk with distance batches spread over NW waves (the sequential
// insert is latency-bound: one wave keeps too few rows in flight).
template <class C, int G, int NW>
__global__ __launch_bounds__(64 * NW) void k_build_compat_mw(CompatBuildArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    __shared__ LayerDev ltab[MH_MAXL];
    a.g = lds_layers(a.g, ltab);
    BuildSmem S;
    uint32_t* p = build_smem(smem, a.vis_log2, a.M, a.ef, S);
    MwEval<C> ev;
    p += (4 - (reinterpret_cast<uintptr_t>(p) >> 2) % 4) % 4;  // 16-B align: qbuf is read/written as float4
    ev.hdr = reinterpret_cast<MwHdr*>(p);
    p += 4;
    ev.qbuf = reinterpret_cast<float4*>(p);
    p += 4 * 64 * C::VPL;
    ev.list = p;
    p += S.hcap;
    ev.dist = reinterpret_cast<float*>(p);
    p += S.hcap;
    ev.nw = NW;
    // eviction speculation staging (stage_evictions): M groups of M + 2, when
    // the launch found room for it
    S.pgroups = a.spec ? a.M : 0;
    S.pstride = a.M + 2;
    const int pt = S.pgroups * S.pstride;
    S.prow = a.spec ? reinterpret_cast<int32_t*>(p) : nullptr;
    p += pt;
    // without staging (large M: the launch found no room) every staging pointer
    // stays null -- they lie past the dynamic LDS allocation
    ev.pc = a.spec ? reinterpret_cast<int32_t*>(p) : nullptr;
    p += pt;
    ev.pd = a.spec ? reinterpret_cast<float*>(p) : nullptr;
    S.pdist = ev.pd;
    p += pt;
    S.pdeg = a.spec ? reinterpret_cast<int*>(p) : nullptr;
    p += 64;
    ev.pq = a.spec ? p : nullptr;
    p += 64;
    ev.pn = a.spec ? reinterpret_cast<int*>(p) : nullptr;
    ev.ps = S.pstride;
    const int wave = threadIdx.x >> 6;
    if (wave != 0) {
        mw_worker<C, G>(a.g, ev, wave);
        return;
    }
    WaveStats st;
    int err = 0;
#ifdef MH_COMPAT_PROF
    if (lane_id() < 24) mh_cprof[lane_id()] = 0;
    __builtin_amdgcn_wave_barrier();
    CPROF_T(tk);
    CPROF_CNT(16, a.n1 - a.n0);
#endif
    compat_inserts<C, G>(a, S, ev, st, err);
#ifdef MH_COMPAT_PROF
    CPROF_ADD(tk, 21);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    if (lane_id() == 0) {
        for (int i = 0; i < 24; ++i) printf("cprof %d %llu\n", i, mh_cprof[i]);
    }
#endif
    if (lane_id() == 0) ev.hdr->cmd = MW_EXIT;
    mw_barrier();  // releases the workers
    if (lane_id() == 0) {
        atomicAdd(&a.stats[0], st.E);
        atomicAdd(&a.stats[1], st.X);
        if (err) atomicOr(a.err, err);
    }
}

constexpr int MW_WAVES = 8;
// dynamic LDS a sequential kernel may ask for: 160 KiB less its static layer
// table (and the tools-only counters)
constexpr size_t CW_LDS_MAX = 160 * 1024 - MH_MAXL * sizeof(LayerDev) - 256;

template <class C, int G>
static int launch_build_compat_t(const CompatBuildArgs& a, int waves, hipStream_t s) {
    const size_t base = build_smem_words(a.vis_log2, a.M, a.ef);
    const int hcap = (a.M + 1) * (a.M + 1) + 2;
    if (waves <= 1 || C::VPL >= 16) {  // 4096-d: the walking wave alone (register budget)
        const size_t lds = (base + hcap) * 4;
        if (lds > CW_LDS_MAX) return -2;
        hipLaunchKernelGGL((k_build_compat<C, G>), dim3(1), dim3(64), lds, s, a);
    } else {
        const size_t spec = 3 * (size_t)a.M * (a.M + 2) + 3 * 64;  // eviction speculation staging
        const size_t core = (base + 3 + 4 + 4 * 64 * (size_t)C::VPL + 2 * (size_t)hcap) * 4;
        CompatBuildArgs b = a;
        b.spec = core + spec * 4 <= CW_LDS_MAX ? 1 : 0;  // large M: no staging (same graph)
        const size_t lds = core + (b.spec ? spec * 4 : 0);
        if (lds > CW_LDS_MAX) return -2;
        hipLaunchKernelGGL((k_build_compat_mw<C, G, MW_WAVES>), dim3(1), dim3(64 * MW_WAVES), lds, s, b);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------------------
// batched build
// ---------------------------------------------------------------------------
// One kept row r (f32 row qr, norm rn) applied to every candidate still
// standing after list position pos (entry e = k * 64 + lane of the NR
// registers: bit k of live / dropped, id ids[k] & ID_MASK, d(u, c) ed[k] --
// the list's own registers, nothing copied): a candidate is dropped
// when alpha d(c, r) < d(u, c) -- decided by a two-sided screen of the
// candidates' fp16 rows against per-row thresholds, the undecided pairs in
// f32 (the neighbour selection of k_batch_search and k_batch_commit).
template <class C, int G, int NR>
__device__ __forceinline__ void drop_pass(const GraphDev& g, const QReg<C>& qr, float rn, int pos,
                                          uint32_t live, uint32_t& dropped, const uint32_t (&ids)[NR],
                                          const float (&ed)[NR], float alpha, float margin, WaveStats& st) {
    const int lane = lane_id();
    const bool scr = h16_query_ok(rn);
    st.F += 1;  // the kept row
    // (the body is too large to unroll: register r's id / distance are picked by
    // a small unrolled select, which keeps the list's registers out of scratch)
    for (int r = 0; r < NR; ++r) {
        uint32_t idr = ids[0];
        float edr = ed[0];
#pragma unroll
        for (int k = 1; k < NR; ++k) {  // bitwise selects: a `?:` chain is folded back into an indexed load
            const uint32_t mk = k == r ? 0xFFFFFFFFu : 0u;
            idr = (ids[k] & mk) | (idr & ~mk);
            edr = bsel(mk, ed[k], edr);
        }
        const bool cand = ((live & ~dropped) >> r & 1u) && r * 64 + lane >= pos;
        const unsigned long long m = __ballot(cand);
        if (!m) continue;
        const int cnt = __popcll(m);
        const int before =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        const int dst = cand ? before : cnt + (lane - before);
        const uint32_t cc = push_to(idr & ID_MASK, dst);
        const float cd = __uint_as_float(push_to(__float_as_uint(edr), dst));
        st.E += cnt;
        // with t = d(u, c) / alpha: an estimate proving d(c, r) > t (1 + 2^-20)
        // keeps c, one proving d(c, r) < t (1 - 2^-20) drops it; the brackets
        // absorb the roundings of t and of the rule's product, so
        // fl(alpha d) >= d(u, c) above and < below
        const float t = cd / alpha;
        int cls = 0;
        if (scr) {
            cls = screen_pairs<C, G>(g, qr, rn, cc, cnt, g.metric, t * (1.0f - 0x1p-20f),
                                     t * (1.0f + 0x1p-20f), margin);
            st.S += cnt;
        }
        if (!(cd > 0.f)) cls = 0;  // as the candidate-major loop: no screen for d(u, c) <= 0
        bool dr = lane < cnt && cls < 0;
        const bool und = lane < cnt && cls == 0;
        const unsigned long long mu = __ballot(und);
        if (mu) {
            const int nu = __popcll(mu);
            const int bu =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(mu >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mu, 0));
            const int du = und ? bu : nu + (lane - bu);
            const uint32_t cu = push_to(cc, du);
            const float dcu = __uint_as_float(push_to(__float_as_uint(cd), du));
            st.F += nu;
            bool dk = false;
            int k = 0;
            eval_list<C, G>(g, qr, rn, cu, nu, g.metric, [&](float dcs, uint32_t) {
                const bool drop = alpha * dcs < rl_f(dcu, k);
                if (lane == k) dk = drop;
                ++k;
            });
            const int dks = __shfl((int)dk, du, 64);  // all lanes: a shuffle reads inactive lanes as 0
            dr = dr || (und && dks != 0);
        }
        const int drs = __shfl((int)dr, dst, 64);
        if (cand && drs != 0) dropped |= 1u << r;
    }
}

// the insert searches' visited set: 2^vis_log2 32-bit entries, or (vis16) the
// compact set -- 8,192 ids in 16 KiB where 2^12 entries held 4,096 (fewer
// resets, fewer re-evaluated candidates; the same lists, so the same graph)
__device__ __forceinline__ int batch_vsize(const BatchBuildArgs& a) { return a.vis16 ? -1 : 1 << a.vis_log2; }
__host__ __device__ inline int batch_vis_words(const BatchBuildArgs& a) {
    return a.vis16 ? std::max(1 << a.vis_log2, VIS16_WORDS) : 1 << a.vis_log2;
}
static size_t batch_lds(const BatchBuildArgs& a) { return (size_t)4 * batch_vis_words(a); }

// Greedy descent (ef = 1) of every new node through the layers above its own
// level, all layers in one launch.  Every layer l is read before its commit
// (run_batch_layers commits layer l only after this kernel), exactly what the
// per-layer descent inside k_batch_search reads, so the graph is the same.
template <class C, int G, bool SCREEN>
__global__ __launch_bounds__(64) void k_batch_descend(BatchBuildArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int64_t u64 = a.n0 + blockIdx.x;
    if (u64 >= a.n1) return;
    const uint32_t u = (uint32_t)u64;
    const int lv = a.levels[u];
    if (lv >= a.layer) return;
    WaveStats st;
    QReg<C> q;
    load_query(q, a.g.vecs + (size_t)u * a.g.pitch);
    const float qn = a.g.norms[u];
    uint32_t ep = a.cur_entry[u];
    for (int l = a.layer; l > lv; --l) {
        BList<1> L1;
        beam_layer<C, 1, G, false, SCREEN>(a.g, l, ep, 1, q, qn, L1, smem, batch_vsize(a), st);
        float d;
        uint32_t id;
        bl_at(L1, 0, d, id);
        if (id != EMPTY_ID) ep = id & ID_MASK;
    }
    if (lane_id() == 0) {
        a.cur_entry[u] = ep;
        atomicAdd(&a.stats[0], st.E);
        atomicAdd(&a.stats[1], st.X);
        atomicAdd(&a.stats[6], st.S);
        atomicAdd(&a.stats[7], st.F);
    }
}

#ifndef MH_BUILD_WPS
#define MH_BUILD_WPS 1
#endif
// One insert u of a batch at layer a.layer: greedy descent above u's level,
// else the layer search (efConstruction), the neighbour selection and the
// reverse proposals.  bev scores the search's candidate batches (WaveBatch:
// this wave; MwBatch: the workgroup's waves, k_batch_search_mw).
template <class C, int R, int G, bool SCREEN, int XW, class BEv>
__device__ __forceinline__ void batch_insert(const BatchBuildArgs& a, uint32_t u, const QReg<C>& q, float qn,
                                             uint32_t* smem, WaveStats& st, const BEv& bev) {
    const int lane = lane_id();
    const int l = a.layer;
    const uint32_t ep = a.cur_entry[u];
    if (a.levels[u] < l) {  // above the node's level: greedy descent only
        BList<1> L1;
        beam_layer<C, 1, G, false, SCREEN, 1>(a.g, l, ep, 1, q, qn, L1, smem, batch_vsize(a), st, bev);
        float d;
        uint32_t id;
        bl_at(L1, 0, d, id);
        if (lane == 0 && id != EMPTY_ID) a.cur_entry[u] = id & ID_MASK;
    } else {
        BList<R> L;
        // lists of 256 / 512 entries on the one-wave kernel merge each step's
        // candidates at once (bl_merge; scratch after the visited set, sized by
        // launch_batch_search_t)
        constexpr bool MRG = R >= 4 && std::is_same<BEv, WaveBatch>::value;
        float* mrg = MRG ? reinterpret_cast<float*>(smem + batch_vis_words(a)) : nullptr;
        beam_layer<C, R, G, false, SCREEN, XW, MRG>(a.g, l, ep, a.ef, q, qn, L, smem, batch_vsize(a), st, bev, mrg);
        float d0;
        uint32_t i0;
        bl_at(L, 0, d0, i0);
        if (lane == 0 && i0 != EMPTY_ID) a.cur_entry[u] = i0 & ID_MASK;
        // neighbour selection
        bool sel_screen = false;
        float margin = 0.f;
        if constexpr (SCREEN) {
            sel_screen = a.g.h16 != nullptr && a.alpha > 0.f;
            const float e = a.g.h16err ? *a.g.h16err : 0.00048828125f;
            margin = a.g.metric == EUCLIDEAN ? h16_margin_l2(e) : h16_margin_cos(e);
        }
        uint32_t sel = 0;
        float seld = 0.f;
        int nsel = 0;
        const int nl = a.ef;
        // Screened: the same rule applied kept-row-major.  A candidate is kept
        // iff no kept row before it drops it, so each kept row r can be applied
        // at once to every later candidate still standing (one batched
        // two-sided screen of their fp16 rows, r's f32 row the query, and the
        // undecided pairs in f32); the next candidate standing is kept.
        // d(c, r) == d(r, c) bitwise (commutative products, norms multiplied
        // both ways round), so every decision is the candidate-major loop's
        // below (the unscreened path): the same graph (test_gpu_screen.py
        // compares with screen 0).  A candidate meets kept rows only until the
        // first one drops it, and the kept rows, not the candidates, are read
        // in f32: 15.4k -> 10.0k pair evaluations and 1.38k -> 0.99k f32 rows
        // per insert on the bench index.
        const bool rowmajor = SCREEN && sel_screen && a.heuristic;
        if (rowmajor) {
            uint32_t live = 0u, dropped = 0u;  // bit r: entry r * 64 + lane
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (L.i[r] != EMPTY_ID && r * 64 + lane < nl && !is_dead(a.g, L.i[r] & ID_MASK)) live |= 1u << r;
            int pos = 0;
            while (nsel < a.mcap) {
                int idx = -1;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const unsigned long long m = __ballot(((live & ~dropped) >> r & 1u) && r * 64 + lane >= pos);
                    if (idx < 0 && m) idx = r * 64 + __ffsll((long long)m) - 1;
                }
                if (idx < 0) break;
                float dc;
                uint32_t c;
                bl_at(L, idx, dc, c);
                c &= ID_MASK;
                if (lane == nsel) {
                    sel = c;
                    seld = dc;
                }
                ++nsel;
                pos = idx + 1;
                if (nsel >= a.mcap) break;
                QReg<C> qr;
                load_query(qr, a.g.vecs + (size_t)c * a.g.pitch);
                drop_pass<C, G, R>(a.g, qr, a.g.norms[c], pos, live, dropped, L.i, L.d, a.alpha, margin, st);
            }
        }
        for (int i = 0; !rowmajor && i < nl && nsel < a.mcap; ++i) {
            float dc;
            uint32_t c;
            bl_at(L, i, dc, c);
            if (c == EMPTY_ID) break;
            c &= ID_MASK;
            if (is_dead(a.g, c)) continue;
            bool good = true;
            if (a.heuristic && nsel > 0) {  // HNSW Alg. 4: drop c if closer to a kept neighbour than to u
                QReg<C> qc;
                load_query(qc, a.g.vecs + (size_t)c * a.g.pitch);
                const float cn = a.g.norms[c];
                st.E += nsel;
                auto rule = [&](float dcs, uint32_t) {
                    if (a.alpha * dcs < dc) good = false;
                };
                st.F += nsel + 1;  // the candidate's row and the kept rows, in f32
                eval_list<C, G>(a.g, qc, cn, sel, nsel, a.g.metric, rule);
            }
            if (good) {
                if (lane == nsel) {
                    sel = c;
                    seld = dc;
                }
                ++nsel;
            }
        }
        if (a.keep_pruned && nsel < a.mcap) {  // Malkov Alg. 4 keepPrunedConnections
            for (int i = 0; i < nl && nsel < a.mcap; ++i) {
                float dc;
                uint32_t c;
                bl_at(L, i, dc, c);
                if (c == EMPTY_ID) break;
                c &= ID_MASK;
                if (is_dead(a.g, c)) continue;
                if (__ballot(lane < nsel && sel == c)) continue;
                if (lane == nsel) {
                    sel = c;
                    seld = dc;
                }
                ++nsel;
            }
        }
        const int capl = a.g.layers[l].cap;
        if (lane < nsel) {
            a.g.layers[l].adj[(size_t)u * capl + lane] = (int32_t)sel;
            a.g.layers[l].adjd[(size_t)u * capl + lane] = seld;
            const int slot = atomicAdd(&a.inc_cnt[sel], 1);
            if (slot < a.inc_cap) {
                a.inc_src[(size_t)sel * a.inc_cap + slot] = u;
                a.inc_dist[(size_t)sel * a.inc_cap + slot] = seld;
            } else {
                atomicAdd(&a.stats[2], 1ull);
            }
            if (slot == 0) {
                const int t = atomicAdd(a.touched_cnt, 1);
                a.touched[t] = sel;
            }
        }
        if (lane == 0) a.g.layers[l].deg[u] = nsel;
    }
}

__device__ __forceinline__ void batch_stats(const BatchBuildArgs& a, const WaveStats& st) {
    if (lane_id() == 0) {
        atomicAdd(&a.stats[0], st.E);
        atomicAdd(&a.stats[1], st.X);
        atomicAdd(&a.stats[6], st.S);
        atomicAdd(&a.stats[7], st.F);
    }
}

__device__ __forceinline__ bool batch_node(const BatchBuildArgs& a, uint32_t& u) {
    if (a.order) {
        if (blockIdx.x >= a.count) return false;
        u = a.order[blockIdx.x];
    } else {
        const int64_t u64 = a.n0 + blockIdx.x;
        if (u64 >= a.n1) return false;
        u = (uint32_t)u64;
    }
    return true;
}

template <class C, int R, int G, bool SCREEN, int XW>
__global__ __launch_bounds__(64, MH_BUILD_WPS) void k_batch_search(BatchBuildArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t u;
    if (!batch_node(a, u)) return;
    WaveStats st;
    QReg<C> q;
    load_query(q, a.g.vecs + (size_t)u * a.g.pitch);
    const float qn = a.g.norms[u];
    batch_insert<C, R, G, SCREEN, XW>(a, u, q, qn, smem, st, WaveBatch());
    batch_stats(a, st);
}

// Narrow launches (few inserts: the first batches of a build, the upper layers
// of every batch) leave most of the chip idle and each insert's ~550 dependent
// expansions on one wave: one workgroup of BMW_WAVES waves per insert splits
// every candidate batch over the waves (k_search_beam_mw's protocol).  Same
// graph as k_batch_search, bit for bit (the list keeps the best ef of what is
// inserted, whatever the order; the screen tests the pre-batch worst on every
// wave).
template <class C, int R, int G, bool SCREEN, int XW>
__global__ __launch_bounds__(64 * BMW_WAVES) void k_batch_search_mw(BatchBuildArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    __shared__ BmwShare sh;
    uint32_t u;
    if (!batch_node(a, u)) return;  // (whole workgroup)
    const int wave = threadIdx.x >> 6;
    WaveStats st;
    QReg<C> q;
    load_query(q, a.g.vecs + (size_t)u * a.g.pitch);
    const float qn = a.g.norms[u];
    if (wave == 0) {
        batch_insert<C, R, G, SCREEN, XW>(a, u, q, qn, smem, st, MwBatch{&sh});
        if (lane_id() == 0) sh.cmd = BMW_EXIT;
        bmw_barrier();  // releases the other waves
    } else {
        const bool screen = SCREEN && h16_query_ok(qn);
        float margin = 0.f;
        if constexpr (SCREEN) {
            const float e = a.g.h16err ? *a.g.h16err : 0.00048828125f;
            margin = a.g.metric == EUCLIDEAN ? h16_margin_l2(e) : h16_margin_cos(e);
        }
        for (;;) {
            bmw_barrier();
            if (sh.cmd == BMW_EXIT) break;
            st.F += bmw_share<C, G, SCREEN>(a.g, q, qn, &sh, wave, screen, margin, st.S);
            bmw_barrier();
        }
    }
    batch_stats(a, st);
}

// One wave per touched node v: merge v's row with the proposals it received.
// (existing U proposals) is ranked by (dist to v, id); when it fits the row it
// is written in rank order, otherwise the best `cap` are kept -- or, with
// heuristic >= 2, HNSW's diversity rule (Alg. 4) is applied on overflow: a
// candidate is dropped when it is closer to an already kept neighbour than to v.
template <class C, int G>
__global__ __launch_bounds__(64) void k_batch_commit(BatchBuildArgs a) {
    __shared__ float sd[128];
    __shared__ uint32_t si[128];
    __shared__ float rd[128];
    __shared__ uint32_t ri[128];
    const int lane = lane_id();
    const int n_t = *a.touched_cnt;
    // grid-stride over the touched rows: a bounded grid (at most 32,768
    // workgroups) instead of one workgroup per row the batch could touch (mcap
    // per insert: 8M for a 200k batch at M0 40, nearly all of which would only
    // read the count and exit)
    for (int t = blockIdx.x; t < n_t; t += gridDim.x) {
        const uint32_t v = a.touched[t];
        const int l = a.layer;
        const int capl = a.g.layers[l].cap;
        const int keep_cap = min(capl, a.mcap);
        int32_t* row = a.g.layers[l].adj + (size_t)v * capl;
        float* rowd = a.g.layers[l].adjd + (size_t)v * capl;
        int d = a.g.layers[l].deg[v];
        if (d < 0) d = 0;
        int nin = a.inc_cnt[v];
        if (nin > a.inc_cap) nin = a.inc_cap;
        const int tot = d + nin;
        for (int e = lane; e < 128; e += 64) {
            float dd = __int_as_float(0x7f800000);
            uint32_t ii = EMPTY_ID;
            if (e < d) {
                ii = (uint32_t)row[e];
                dd = rowd[e];
            } else if (e < tot) {
                ii = a.inc_src[(size_t)v * a.inc_cap + (e - d)];
                dd = a.inc_dist[(size_t)v * a.inc_cap + (e - d)];
            }
            sd[e] = dd;
            si[e] = ii;
        }
        __syncthreads();
        // rank = number of entries ordered before this one by (dist, id)
        for (int h = 0; h < 2; ++h) {
            const int e = lane + 64 * h;
            const float md = sd[e];
            const uint32_t mi = si[e];
            int rank = 0;
            for (int f = 0; f < tot; ++f) rank += lt_di(sd[f], si[f], md, mi) ? 1 : 0;
            if (e < tot) {
                rd[rank] = md;
                ri[rank] = mi;
            }
        }
        __syncthreads();
        int nkeep = 0;
        if (tot <= keep_cap || a.heuristic < 2) {
            nkeep = min(tot, keep_cap);
            for (int e = lane; e < nkeep; e += 64) {
                row[e] = (int32_t)ri[e];
                rowd[e] = rd[e];
            }
        } else {
            uint32_t kept = 0;   // lane j holds the j-th kept id
            float keptd = 0.f;
            WaveStats st;
            // with the fp16 copy: kept-row-major, as k_batch_search's selection
            // (drop_pass; the same decisions as the candidate-major loop below)
            const bool rowmajor = a.g.h16 != nullptr && a.alpha > 0.f;
            if (rowmajor) {
                const float e = a.g.h16err ? *a.g.h16err : 0.00048828125f;
                const float margin = a.g.metric == EUCLIDEAN ? h16_margin_l2(e) : h16_margin_cos(e);
                uint32_t live = 0u, dropped = 0u;
                uint32_t eid[2];
                float ed[2];
    #pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int e2 = lane + 64 * h;
                    if (e2 < tot) live |= 1u << h;
                    eid[h] = e2 < tot ? guard_id(a.g, ri[e2]) : 0u;
                    ed[h] = rd[e2];
                }
                int pos = 0;
                while (nkeep < keep_cap) {
                    int idx = -1;
    #pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const unsigned long long m = __ballot(((live & ~dropped) >> h & 1u) && h * 64 + lane >= pos);
                        if (idx < 0 && m) idx = h * 64 + __ffsll((long long)m) - 1;
                    }
                    if (idx < 0) break;
                    const uint32_t c = ri[idx];
                    if (lane == nkeep) {
                        kept = c;
                        keptd = rd[idx];
                    }
                    ++nkeep;
                    pos = idx + 1;
                    if (nkeep >= keep_cap) break;
                    QReg<C> qr;
                    const uint32_t cg = guard_id(a.g, c);
                    load_query(qr, a.g.vecs + (size_t)cg * a.g.pitch);
                    drop_pass<C, G, 2>(a.g, qr, a.g.norms[cg], pos, live, dropped, eid, ed, a.alpha, margin, st);
                }
            }
            for (int i = 0; !rowmajor && i < tot && nkeep < keep_cap; ++i) {
                const uint32_t c = ri[i];
                const float dcv = rd[i];
                bool good = true;
                if (nkeep > 0) {
                    QReg<C> qc;
                    load_query(qc, a.g.vecs + (size_t)guard_id(a.g, c) * a.g.pitch);
                    const float cn = a.g.norms[guard_id(a.g, c)];
                    st.E += nkeep;
                    st.F += nkeep + 1;  // the candidate's row and the kept rows, in f32
                    eval_list<C, G>(a.g, qc, cn, kept, nkeep, a.g.metric, [&](float dcs, uint32_t) {
                        if (a.alpha * dcs < dcv) good = false;
                    });
                }
                if (good) {
                    if (lane == nkeep) {
                        kept = c;
                        keptd = dcv;
                    }
                    ++nkeep;
                }
            }
            if (lane < nkeep) {
                row[lane] = (int32_t)kept;
                rowd[lane] = keptd;
            }
            if (lane == 0) {  // the pruning's rows count as the insert's reads (bench.py build roofline)
                atomicAdd(&a.stats[0], st.E);
                atomicAdd(&a.stats[6], st.S);
                atomicAdd(&a.stats[7], st.F);
            }
        }
        if (lane == 0) {
            a.g.layers[l].deg[v] = nkeep;
            a.inc_cnt[v] = 0;
        }
        __syncthreads();  // (the LDS rank arrays are reused by the next row)
    }
}

// ---------------------------------------------------------------------------
// delete (graph.go:843-895)
// ---------------------------------------------------------------------------
// Delete / BatchDelete with the reference's semantics: one wave walks the keys
// in order and every layer holding the node (graph.go:852-861).
template <class C, int G>
__global__ __launch_bounds__(64) void k_delete_compat(DeleteArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    __shared__ LayerDev ltab[MH_MAXL];
    a.g = lds_layers(a.g, ltab);
    const int lane = lane_id();
    BuildSmem S;
    uint32_t* p = build_smem(smem, a.vis_log2, a.M, 0, S);
    WaveEval ev;
    ev.list = p;
    WaveStats st;
    int err = 0;
    for (int64_t i = 0; i < a.nids; ++i) {
        const uint32_t id = a.ids[i];
        const int l = (int)a.lay[i];
        if (uni(ld_i32<true>(a.g.layers[l].deg + id)) == -2) continue;
        isolate<C, G>(a.g, l, id, a.M, S, st, err, ev);
    }
    if (lane == 0) {
        atomicAdd(&a.stats[0], st.E);
        if (err) atomicOr(a.err, err);
    }
}

// Batched-graph repair, one wave per row of layer a.layer: a live row that
// points at a deleted node is rebuilt from its live neighbours plus the rows
// of its deleted neighbours (gather order, first REPAIR_POOL kept), ranked by
// (distance, id) and selected like k_batch_search (diversity heuristic,
// optional keep-pruned fill).  Deleted rows are only read and live rows are
// only written by their owner, so rows are independent.  Restated in
// oracle/oracle.c repair_layer.
template <class C, int G>
__global__ __launch_bounds__(64) void k_delete_repair(DeleteArgs a) {
    __shared__ uint32_t pid[REPAIR_POOL];
    __shared__ float pd[REPAIR_POOL];
    __shared__ uint32_t sid[REPAIR_POOL];
    __shared__ float sdd[REPAIR_POOL];
    const int64_t v64 = blockIdx.x;
    if (v64 >= a.n) return;
    const uint32_t v = (uint32_t)v64;
    const int lane = lane_id();
    const int l = a.layer;
    if (a.g.dead[v]) return;
    const int capl = a.g.layers[l].cap;
    const int d = min(a.g.layers[l].deg[v], capl);
    if (d <= 0) return;
    int32_t* row = a.g.layers[l].adj + (size_t)v * capl;
    float* rowd = a.g.layers[l].adjd + (size_t)v * capl;
    const uint32_t nb = lane < d ? guard_id(a.g, (uint32_t)row[lane]) : 0u;
    const bool nd = lane < d && a.g.dead[nb];
    const unsigned long long mdead = __ballot(nd);
    if (!mdead) return;
    const unsigned long long below = (1ull << lane) - 1ull;
    const unsigned long long mlive = __ballot(lane < d && !nd);
    if (lane < d && !nd) pid[__popcll(mlive & below)] = nb;
    int np = __popcll(mlive);
    for (unsigned long long m = mdead; m; m &= m - 1) {
        const int j = __ffsll((long long)m) - 1;
        const uint32_t x = rl_u(nb, j);
        const int dx = min(a.g.layers[l].deg[x], capl);
        if (dx <= 0) continue;
        const uint32_t y = lane < dx ? guard_id(a.g, (uint32_t)a.g.layers[l].adj[(size_t)x * capl + lane]) : 0u;
        const bool ok = lane < dx && y != v && !a.g.dead[y];
        const unsigned long long my = __ballot(ok);
        const int pos = np + __popcll(my & below);
        if (ok && pos < REPAIR_POOL) pid[pos] = y;
        np = min(np + __popcll(my), REPAIR_POOL);
    }
    __syncthreads();
    QReg<C> q;
    load_query(q, a.g.vecs + (size_t)v * a.g.pitch);
    const float qn = a.g.norms[v];
    const float inf = __int_as_float(0x7f800000);
    WaveStats st;
    for (int base = 0; base < np; base += 64) {
        const int cnt = min(64, np - base);
        const uint32_t cid = lane < cnt ? pid[base + lane] : 0u;
        int t = base;
        st.E += cnt;
        eval_list<C, G>(a.g, q, qn, cid, cnt, a.g.metric, [&](float dd, uint32_t) {
            if (lane == 0) pd[t] = dd != dd ? inf : dd;  // NaN (zero vectors) ranks last
            ++t;
        });
    }
    __syncthreads();
    for (int e = lane; e < np; e += 64) {  // rank by (dist, id); duplicates keep gather order
        const float md = pd[e];
        const uint32_t mi = pid[e];
        int rank = 0;
        for (int f = 0; f < np; ++f) {
            const float fd = pd[f];
            const uint32_t fi = pid[f];
            rank += (lt_di(fd, fi, md, mi) || (fd == md && fi == mi && f < e)) ? 1 : 0;
        }
        sdd[rank] = md;
        sid[rank] = mi;
    }
    __syncthreads();
    uint32_t kept = 0;  // lane j holds the j-th kept id
    float keptd = 0.f;
    int nkeep = 0;
    for (int i = 0; i < np && nkeep < a.mcap; ++i) {
        const uint32_t c = sid[i];
        if (i > 0 && c == sid[i - 1]) continue;
        const float dcv = sdd[i];
        bool good = true;
        if (a.heuristic && nkeep > 0) {
            QReg<C> qc;
            load_query(qc, a.g.vecs + (size_t)c * a.g.pitch);
            const float cn = a.g.norms[c];
            st.E += nkeep;
            eval_list<C, G>(a.g, qc, cn, kept, nkeep, a.g.metric, [&](float dcs, uint32_t) {
                if (dcs < dcv) good = false;
            });
        }
        if (good) {
            if (lane == nkeep) {
                kept = c;
                keptd = dcv;
            }
            ++nkeep;
        }
    }
    if (a.keep_pruned) {
        for (int i = 0; i < np && nkeep < a.mcap; ++i) {
            const uint32_t c = sid[i];
            if (i > 0 && c == sid[i - 1]) continue;
            if (__ballot(lane < nkeep && kept == c)) continue;
            if (lane == nkeep) {
                kept = c;
                keptd = sdd[i];
            }
            ++nkeep;
        }
    }
    if (lane < nkeep) {
        row[lane] = (int32_t)kept;
        rowd[lane] = keptd;
    }
    if (lane == 0) {
        a.g.layers[l].deg[v] = nkeep;
        atomicAdd(&a.stats[0], st.E);
    }
}

template <class C, int G>
static int launch_delete_compat_t(const DeleteArgs& a, hipStream_t s) {
    const size_t words = build_smem_words(a.vis_log2, a.M, 0) + (size_t)((a.M + 1) * (a.M + 1) + 2);
    if (words * 4 > CW_LDS_MAX) return -2;
    hipLaunchKernelGGL((k_delete_compat<C, G>), dim3(1), dim3(64), words * 4, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <class C, int G>
static int launch_batch_descend_t(const BatchBuildArgs& a, hipStream_t s) {
    const size_t lds = batch_lds(a);
    const int64_t n = a.n1 - a.n0;
    if (n <= 0) return 0;
    if (a.g.h16)
        hipLaunchKernelGGL((k_batch_descend<C, G, true>), dim3((unsigned)n), dim3(64), lds, s, a);
    else
        hipLaunchKernelGGL((k_batch_descend<C, G, false>), dim3((unsigned)n), dim3(64), lds, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <class C, int R, int G>
static int launch_batch_search_t(const BatchBuildArgs& a, hipStream_t s) {
    const size_t lds_mw = batch_lds(a);
    const size_t lds = lds_mw + (R >= 4 ? 4 * BL_MERGE_WORDS : 0);  // (the one-wave kernel's merge scratch)
    const int64_t n = a.order ? a.count : a.n1 - a.n0;
    if (n <= 0) return 0;
    // fp16 screening: same graph, fewer bytes per candidate; XW = a.expand as a
    // template argument (one search variant per kernel keeps it spill-free)
    const bool narrow = a.g.h16 && n <= a.mw_max;  // a narrow launch: a workgroup per insert
    if (narrow && a.expand == 4)
        hipLaunchKernelGGL((k_batch_search_mw<C, R, G, true, 4>), dim3((unsigned)n), dim3(64 * BMW_WAVES), lds_mw, s, a);
    else if (narrow && a.expand == 3)
        hipLaunchKernelGGL((k_batch_search_mw<C, R, G, true, 3>), dim3((unsigned)n), dim3(64 * BMW_WAVES), lds_mw, s, a);
    else if (narrow && a.expand == 2)
        hipLaunchKernelGGL((k_batch_search_mw<C, R, G, true, 2>), dim3((unsigned)n), dim3(64 * BMW_WAVES), lds_mw, s, a);
    else if (a.g.h16 && a.expand == 4)
        hipLaunchKernelGGL((k_batch_search<C, R, G, true, 4>), dim3((unsigned)n), dim3(64), lds, s, a);
    else if (a.g.h16 && a.expand == 3)
        hipLaunchKernelGGL((k_batch_search<C, R, G, true, 3>), dim3((unsigned)n), dim3(64), lds, s, a);
    else if (a.g.h16 && a.expand == 2)
        hipLaunchKernelGGL((k_batch_search<C, R, G, true, 2>), dim3((unsigned)n), dim3(64), lds, s, a);
    else if (a.g.h16)
        hipLaunchKernelGGL((k_batch_search<C, R, G, true, 1>), dim3((unsigned)n), dim3(64), lds, s, a);
    else if (a.expand == 4)
        hipLaunchKernelGGL((k_batch_search<C, R, G, false, 4>), dim3((unsigned)n), dim3(64), lds, s, a);
    else if (a.expand == 3)
        hipLaunchKernelGGL((k_batch_search<C, R, G, false, 3>), dim3((unsigned)n), dim3(64), lds, s, a);
    else if (a.expand == 2)
        hipLaunchKernelGGL((k_batch_search<C, R, G, false, 2>), dim3((unsigned)n), dim3(64), lds, s, a);
    else
        hipLaunchKernelGGL((k_batch_search<C, R, G, false, 1>), dim3((unsigned)n), dim3(64), lds, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// build.hip is compiled once per part (MH_PART 0-3, Makefile) so that the
// configurations' kernels compile in parallel; each part instantiates its
// share of the configurations, and part 0 also holds the dispatchers, which
// ask each part in turn (-3: configuration not in that part).
// (MH_NO_PARTS: templates only, for ISA inspection of one instantiation)
#ifndef MH_NO_PARTS
#ifndef MH_PART
#define MH_PART 0
#endif
#if MH_PART == 0
#define MH_FOR_EACH_CFG(X) X(16, 1, 2) X(32, 1, 4) X(64, 1, 8)
#elif MH_PART == 1
#define MH_FOR_EACH_CFG(X) X(64, 2, 8) X(64, 3, 8)
#elif MH_PART == 2
#define MH_FOR_EACH_CFG(X) X(64, 4, 4) X(64, 6, 4)
#else
#define MH_FOR_EACH_CFG(X) X(64, 8, 2) X(64, 12, 1) X(64, 16, 1)
#endif
#define MH_CAT2(a, b) a##b
#define MH_CAT(a, b) MH_CAT2(a, b)
#define MH_PARTFN(f) MH_CAT(f##_part, MH_PART)

// every part's entry points (defined below, one set per part)
#define MH_DECL_PARTS(P)                                                                           \
    int launch_build_compat_part##P(const CompatBuildArgs& a, int lpr, int vpl, int waves, hipStream_t s); \
    int launch_build_batch_descend_part##P(const BatchBuildArgs& a, int lpr, int vpl, hipStream_t s); \
    int launch_build_batch_search_part##P(const BatchBuildArgs& a, int lpr, int vpl, hipStream_t s);  \
    int launch_build_batch_commit_part##P(const BatchBuildArgs& a, int lpr, int vpl, int64_t mt, hipStream_t s); \
    int launch_delete_compat_part##P(const DeleteArgs& a, int lpr, int vpl, hipStream_t s);           \
    int launch_delete_repair_part##P(const DeleteArgs& a, int lpr, int vpl, hipStream_t s);
MH_DECL_PARTS(0)
MH_DECL_PARTS(1)
MH_DECL_PARTS(2)
MH_DECL_PARTS(3)
#undef MH_DECL_PARTS

int MH_PARTFN(launch_build_compat)(const CompatBuildArgs& a, int lpr, int vpl, int waves, hipStream_t s) {
    // the sequential build keeps three query rows live (search / addNeighbor /
    // replenish): up to 4 rows in flight per group to 768-d, 2 above (spill-free)
#define X_(L, V, G) \
    if (lpr == L && vpl == V)    \
        return launch_build_compat_t<Cfg<L, V>, (V <= 3 ? (G < 4 ? G : 4) : (G < 2 ? G : 2))>(a, waves, s);
    MH_FOR_EACH_CFG(X_)
#undef X_
    return -3;
}

int MH_PARTFN(launch_build_batch_descend)(const BatchBuildArgs& a, int lpr, int vpl, hipStream_t s) {
#define X_(L, V, G) \
    if (lpr == L && vpl == V) return launch_batch_descend_t<Cfg<L, V>, G>(a, s);
    MH_FOR_EACH_CFG(X_)
#undef X_
    return -3;
}

// MH_BUILD_GMAX (a build flag, default 8): cap on the rows in flight per wave
// step of the batched insert's search kernel
#ifndef MH_BUILD_GMAX
#define MH_BUILD_GMAX 8
#endif
int MH_PARTFN(launch_build_batch_search)(const BatchBuildArgs& a, int lpr, int vpl, hipStream_t s) {
#define X_(L, V, G)                                                                                    \
    if (lpr == L && vpl == V) {                                                                        \
        constexpr int GB = G < MH_BUILD_GMAX ? G : MH_BUILD_GMAX;                                      \
        if (a.ef <= 64) return launch_batch_search_t<Cfg<L, V>, 1, GB>(a, s);                          \
        if (a.ef <= 128) return launch_batch_search_t<Cfg<L, V>, 2, GB>(a, s);                         \
        if (a.ef <= 256) return launch_batch_search_t<Cfg<L, V>, 4, GB>(a, s);                         \
        if (a.ef <= 512) return launch_batch_search_t<Cfg<L, V>, 8, GB>(a, s);                         \
        return -4;                                                                                     \
    }
    MH_FOR_EACH_CFG(X_)
#undef X_
    return -3;
}

int MH_PARTFN(launch_build_batch_commit)(const BatchBuildArgs& a, int lpr, int vpl, int64_t max_touched, hipStream_t s) {
    if (max_touched <= 0) return 0;
#define X_(L, V, G)                                                                                   \
    if (lpr == L && vpl == V) {                                                                       \
        hipLaunchKernelGGL((k_batch_commit<Cfg<L, V>, (G < 4 ? G : 4)>), dim3((unsigned)std::min<int64_t>(max_touched, 32768)), \
                           dim3(64), 0, s, a);                                                        \
        return hipGetLastError() == hipSuccess ? 0 : -1;                                              \
    }
    MH_FOR_EACH_CFG(X_)
#undef X_
    return -3;
}

int MH_PARTFN(launch_delete_compat)(const DeleteArgs& a, int lpr, int vpl, hipStream_t s) {
    if (a.nids <= 0) return 0;
#define X_(L, V, G) \
    if (lpr == L && vpl == V) return launch_delete_compat_t<Cfg<L, V>, (G < 2 ? G : 2)>(a, s);
    MH_FOR_EACH_CFG(X_)
#undef X_
    return -3;
}

int MH_PARTFN(launch_delete_repair)(const DeleteArgs& a, int lpr, int vpl, hipStream_t s) {
    if (a.n <= 0) return 0;
#define X_(L, V, G)                                                                                      \
    if (lpr == L && vpl == V) {                                                                          \
        hipLaunchKernelGGL((k_delete_repair<Cfg<L, V>, (G < 4 ? G : 4)>), dim3((unsigned)a.n), dim3(64), 0, s, \
                           a);                                                                           \
        return hipGetLastError() == hipSuccess ? 0 : -1;                                                 \
    }
    MH_FOR_EACH_CFG(X_)
#undef X_
    return -3;
}

#if MH_PART == 0
#define MH_ASK_PARTS(call)                       \
    {                                            \
        int r_;                                  \
        if ((r_ = call(0)) != -3) return r_;     \
        if ((r_ = call(1)) != -3) return r_;     \
        if ((r_ = call(2)) != -3) return r_;     \
        return call(3);                          \
    }
int launch_build_compat(const CompatBuildArgs& a, int lpr, int vpl, int waves, hipStream_t s) {
#define C_(P) launch_build_compat_part##P(a, lpr, vpl, waves, s)
    MH_ASK_PARTS(C_)
#undef C_
}
int launch_build_batch_descend(const BatchBuildArgs& a, int lpr, int vpl, hipStream_t s) {
#define C_(P) launch_build_batch_descend_part##P(a, lpr, vpl, s)
    MH_ASK_PARTS(C_)
#undef C_
}
int launch_build_batch_search(const BatchBuildArgs& a, int lpr, int vpl, hipStream_t s) {
#define C_(P) launch_build_batch_search_part##P(a, lpr, vpl, s)
    MH_ASK_PARTS(C_)
#undef C_
}
int launch_build_batch_commit(const BatchBuildArgs& a, int lpr, int vpl, int64_t max_touched, hipStream_t s) {
#define C_(P) launch_build_batch_commit_part##P(a, lpr, vpl, max_touched, s)
    MH_ASK_PARTS(C_)
#undef C_
}
int launch_delete_compat(const DeleteArgs& a, int lpr, int vpl, hipStream_t s) {
#define C_(P) launch_delete_compat_part##P(a, lpr, vpl, s)
    MH_ASK_PARTS(C_)
#undef C_
}
int launch_delete_repair(const DeleteArgs& a, int lpr, int vpl, hipStream_t s) {
#define C_(P) launch_delete_repair_part##P(a, lpr, vpl, s)
    MH_ASK_PARTS(C_)
#undef C_
}
#undef MH_ASK_PARTS
#endif
#endif  // MH_NO_PARTS

}  // namespace mh
