// walks.hpp -- the reference-semantics search kernel (k_search_compat,
// graph.go:571-622) and the negatives epilogue (k_negatives,
// graph.go:1116-1537), instantiated per dimension configuration in
// walks_*.hip (split from search.hip so the configurations compile in
// parallel).
#pragma once
#include "beam.hpp"

namespace mh {

template <int L, int V>
int launch_compat_cfg(const SearchArgs& a, hipStream_t s);
template <int L, int V>
int launch_negatives_cfg(const NegArgs& a, hipStream_t s);

template <class C, int G>
__global__ __launch_bounds__(64) void k_search_compat(SearchArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int64_t b = blockIdx.x;
    if (b >= a.B) return;
    const int lane = lane_id();
    const int vsize = 1 << a.vis_log2;
    CompatSmem S;
    S.vis = smem;
    S.vlog2 = a.vis_log2;
    S.cd = reinterpret_cast<float*>(smem + vsize);
    S.ci = smem + vsize + (a.ef + 2);
    S.rd = reinterpret_cast<float*>(smem + vsize + 2 * (a.ef + 2));
    S.ri = smem + vsize + 2 * (a.ef + 2) + (a.k + 2);
    QReg<C> q;
    load_query(q, a.q + (size_t)b * C::PITCH);
    const float qn = query_norm(q);
    WaveStats st;
    int err = 0;
    uint32_t elevator = EMPTY_ID;
    int nres = 0;
    for (int l = a.top; l >= 0; --l) {  // graph.go:571-622
        // searchPoint: layers[l].nodes[*elevator] (nil once deleted) or entry() (nil when empty)
        uint32_t p;
        if (elevator != EMPTY_ID)
            p = resolve_member<false>(a.g, l, elevator);
        else
            p = l == a.top ? a.entry : (a.layer_entry[l] < 0 ? EMPTY_ID : (uint32_t)a.layer_entry[l]);
        if (p == EMPTY_ID) continue;  // search(nil) returns nothing (graph.go:101-103)
        if (l > 0) {
            const int c = compat_layer<C, G>(a.g, l, p, 1, a.ef, q, qn, S, st, err);
            if (c == 0) continue;
            elevator = S.ri[0];
            continue;
        }
        nres = compat_layer<C, G>(a.g, 0, p, a.k, a.ef, q, qn, S, st, err);
    }
    for (int i = lane; i < a.k; i += 64) {
        const bool ok = i < nres;
        const uint32_t id = ok ? S.ri[i] : 0u;
        a.out_keys[b * a.k + i] = ok ? a.g.keys[id] : (int64_t)-1;
        a.out_dist[b * a.k + i] = ok ? S.rd[i] : __int_as_float(0x7f800000);
        if (a.out_ids) a.out_ids[b * a.k + i] = ok ? (int32_t)id : -1;
    }
    if (lane == 0) {
        a.out_n[b] = nres;
        atomicAdd(&a.stats[0], st.E);
        atomicAdd(&a.stats[1], st.X);
        if (err) atomicOr(a.err, 1);
    }
}

// ---------------------------------------------------------------------------
// negative-example re-ranking (graph.go:1116-1537), one wave per query: the
// Search(near, kx) candidates are scored against the query's negatives with
// the reference's float32 formula, then ranked by descending score (ties in
// candidate order, NaN last).  Restated in oracle/oracle.c og_search_negatives.
// ---------------------------------------------------------------------------
template <class C, int G>
__global__ __launch_bounds__(64) void k_negatives(NegArgs a) {
#pragma clang fp contract(off)
    __shared__ float sc[NEG_MAX_CAND];
    __shared__ int32_t sid[NEG_MAX_CAND];
    const int64_t b = blockIdx.x;
    if (b >= a.B) return;
    const int lane = lane_id();
    const int n = min(a.cand_n[b], a.kx);
    const int j0 = a.neg_off[b], j1 = a.neg_off[b + 1];
    const int nn = j1 - j0;
    for (int base = 0; base < n; base += 64) {
        const int cnt = min(64, n - base);
        const bool mine = lane < cnt;
        const uint32_t cid = mine ? (uint32_t)a.cand_ids[b * a.kx + base + lane] : 0u;
        const float qd = mine ? a.cand_d[b * a.kx + base + lane] : 0.f;
        float total = 0.f;
        bool close = false;
        for (int j = j0; j < j1; ++j) {
            QReg<C> nq;
            load_query(nq, a.neg + (size_t)j * C::PITCH);
            const float nqn = query_norm(nq);
            float nd = 0.f;
            int t = 0;
            eval_list<C, G>(a.g, nq, nqn, cid, cnt, a.g.metric, [&](float d, uint32_t) {
                if (lane == t) nd = d;
                ++t;
            });
            total = total + (1.0f - nd);
            close = close || nd < 0.1f;
        }
        const float qs = 1.0f - qd;
        const float avg = total / (float)nn;
        float score;
        if (qd < 0.001f) {
            score = 2.0f;
        } else if (close) {
            score = qs - a.w * 2.0f;
        } else {
            const int64_t key = mine ? a.g.keys[cid] : 0;
            const float boost = ((a.flags & 1) && key >= 7 && key <= 9) ? 0.2f : 0.0f;
            score = qs - a.w * avg + boost;
        }
        if (mine) {
            sc[base + lane] = score;
            sid[base + lane] = (int32_t)cid;
        }
    }
    __syncthreads();
    for (int e = lane; e < n; e += 64) {
        const float se = sc[e];
        const bool en = se != se;
        int rank = 0;
        for (int f = 0; f < n; ++f) {
            const float sf = sc[f];
            const bool fn = sf != sf;
            const bool before = (fn != en) ? en : ((!fn && sf != se) ? sf > se : f < e);
            rank += before ? 1 : 0;
        }
        if (rank < a.k) {
            a.out_keys[b * a.k + rank] = a.g.keys[sid[e]];
            a.out_score[b * a.k + rank] = se;
        }
    }
    const int m = min(n, a.k);
    for (int i = m + lane; i < a.k; i += 64) {
        a.out_keys[b * a.k + i] = (int64_t)-1;
        a.out_score[b * a.k + i] = __int_as_float(0x7fc00000);
    }
    if (lane == 0) a.out_n[b] = m;
}

template <class C, int G>
static int launch_compat_t(const SearchArgs& a, hipStream_t s) {
    const size_t lds = ((size_t)1 << a.vis_log2) * 4 + (size_t)(a.ef + 2) * 8 + (size_t)(a.k + 2) * 8;
    if (lds > 160 * 1024) return -2;
    hipLaunchKernelGGL((k_search_compat<C, G>), dim3((unsigned)a.B), dim3(64), lds, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int L, int V>
int launch_compat_cfg(const SearchArgs& a, hipStream_t s) {
    return launch_compat_t<Cfg<L, V>, beam_group<L, V>()>(a, s);
}

template <int L, int V>
int launch_negatives_cfg(const NegArgs& a, hipStream_t s) {
    constexpr int G = beam_group<L, V>();
    hipLaunchKernelGGL((k_negatives<Cfg<L, V>, (G < 4 ? G : 4)>), dim3((unsigned)a.B), dim3(64), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace mh
