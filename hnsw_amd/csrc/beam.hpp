// beam.hpp -- the batched beam search kernel (k_search_beam) and the
// dimension-configuration list, shared by search.hip (dispatch) and the
// beam_*.hip translation units that instantiate it per configuration (split
// so that the kernel's 4 list widths x 2 screen modes x 10 configurations
// compile in parallel).
#pragma once
#include "device_search.hpp"
#include "engine.hpp"

namespace mh {

// group width per configuration (rows in flight per wave step)
#define MH_FOR_EACH_CFG(X)      \
    X(16, 1, 2)                 \
    X(32, 1, 4)                 \
    X(64, 1, 8)                 \
    X(64, 2, 8)                 \
    X(64, 3, 8)                 \
    X(64, 4, 4)                 \
    X(64, 6, 4)                 \
    X(64, 8, 2)            \
    X(64, 12, 1)           \
    X(64, 16, 1)

// XW: entries expanded per step of the layer-0 search (option "search_expand";
// 1 = the standard best-first search).  XW 1 is instantiated in beam_a-d.hip,
// XW 2 and 4 in beam_x2a/b.hip and beam_x4a/b.hip.
template <int L, int V, int XW>
int launch_beam_cfg(const SearchArgs& a, hipStream_t s);

// ---------------------------------------------------------------------------
// batched search: one wave per query
// ---------------------------------------------------------------------------
// One query b: greedy descent, the layer-0 beam, and its first k live entries
// into the outputs.  BEv scores each batch of candidates (beam_layer).
// the visited set's LDS words (the merge scratch follows it)
__host__ __device__ inline int beam_vis_words(const SearchArgs& a) { return a.vis16 ? VIS16_WORDS : a.vis_n; }

template <class C, int R, int G, bool SCREEN, int XW, class BEv>
__device__ __forceinline__ void beam_query(const SearchArgs& a, int64_t b, const QReg<C>& q, float qn, uint32_t* smem,
                                           WaveStats& st, const BEv& bev) {
    const int lane = lane_id();
    const int vsz = a.vis16 ? -1 : a.vis_n;  // (beam_layer: < 0 selects the compact set)
    uint32_t ep = a.entry;
    {
        BList<1> L1;
        for (int l = a.top; l >= 1; --l) {  // greedy descent, ef = 1
            if (a.g.layers[l].deg[ep] == -2) {  // not in this layer: restart at its entry
                const int32_t e = a.layer_entry[l];
                if (e < 0) continue;
                ep = (uint32_t)e;
            }
            beam_layer<C, 1, G, false, SCREEN, 1>(a.g, l, ep, a.upper_ef, q, qn, L1, smem, vsz, st, bev);
            float d;
            uint32_t id;
            bl_at(L1, 0, d, id);
            if (id != EMPTY_ID) ep = id & ID_MASK;
        }
    }
    BList<R> L;
    const int efl = a.ef > a.k ? a.ef : a.k;
    if (a.g.layers[0].deg[ep] == -2) ep = (uint32_t)a.layer_entry[0];
    // lists of 256 / 512 entries merge each step's candidates at once, with the
    // LDS past the visited set as scratch (launch_beam_t sizes the LDS for it;
    // the default compact set leaves room in the 20 KiB a 2-wave SIMD allows)
    constexpr bool MRG = R >= 4;
    float* mrg = MRG ? reinterpret_cast<float*>(smem + beam_vis_words(a)) : nullptr;
    beam_layer<C, R, G, false, SCREEN, XW, MRG>(a.g, 0, ep, efl, q, qn, L, smem, vsz, st, bev, mrg);
    // compact the sorted list into the first k live entries (deleted rows
    // route the search but are never returned)
    int nvalid = 0;
    const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t id = L.i[r] & ID_MASK;
        const bool ok = L.i[r] != EMPTY_ID && !is_dead(a.g, id);
        const unsigned long long m = __ballot(ok);
        const int pos = nvalid + __popcll(m & below);
        if (ok && pos < a.k) {
            a.out_keys[b * a.k + pos] = a.g.keys[id];
            a.out_dist[b * a.k + pos] = L.d[r];
            if (a.out_ids) a.out_ids[b * a.k + pos] = (int32_t)id;
        }
        nvalid += __popcll(m);
    }
    nvalid = min(nvalid, a.k);
    for (int i = nvalid + lane; i < a.k; i += 64) {
        a.out_keys[b * a.k + i] = (int64_t)-1;
        a.out_dist[b * a.k + i] = __int_as_float(0x7f800000);
        if (a.out_ids) a.out_ids[b * a.k + i] = -1;
    }
    if (lane == 0) a.out_n[b] = nvalid;
}

__device__ __forceinline__ void beam_stats(const SearchArgs& a, const WaveStats& st) {
    if (lane_id() == 0) {
        atomicAdd(&a.stats[0], st.E);
        atomicAdd(&a.stats[1], st.X);
        if (st.resets) atomicAdd(&a.stats[2], st.resets);
        atomicAdd(&a.stats[8], st.S);
        atomicAdd(&a.stats[9], st.F);
#ifdef MH_PROF_BEAM
        // (tools-only: the slots the batched insert uses, read back as build_screened /
        // build_f32_rows / exact_uncertified)
        atomicAdd(&a.stats[10], st.c_ins);
        atomicAdd(&a.stats[11], st.c_score);
        atomicAdd(&a.stats[3], st.c_all);
#endif
    }
}

// MH_BEAM_WIDE_G / MH_BEAM_WIDE_WAVES (build flags, for tools/ variants): rows
// in flight per wave step and the waves per SIMD the compiler must fit, for the
// 512-entry list (R = 8); 0 = the configuration's G and 2 waves
#ifndef MH_BEAM_WIDE_G
#define MH_BEAM_WIDE_G 0
#endif
#ifndef MH_BEAM_WIDE_WAVES
#define MH_BEAM_WIDE_WAVES 2
#endif
template <class C, int R, int G, bool SCREEN, int XW>
__global__ __attribute__((amdgpu_flat_work_group_size(64, 64), amdgpu_waves_per_eu(R >= 8 ? MH_BEAM_WIDE_WAVES : 2)))
void k_search_beam(SearchArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int64_t b = blockIdx.x;
    if (b >= a.B) return;
    QReg<C> q;
    load_query(q, a.q + (size_t)b * C::PITCH);
    const float qn = query_norm(q);
    WaveStats st;
    beam_query<C, R, G, SCREEN, XW>(a, b, q, qn, smem, st, WaveBatch());
    beam_stats(a, st);
}

// ---------------------------------------------------------------------------
// small batches (the reference's ParallelSearch, graph.go:631-790: one query's
// neighbour distances fanned out over workers): one workgroup of BMW_WAVES
// waves per query.  Wave 0 runs the list, the visited set and the expansions
// exactly as k_search_beam; each batch of new candidates is split over the
// waves (screen + f32 on each wave's rows, in one round trip instead of one
// per 16 rows), and the survivors come back to wave 0's list.  The list is the
// best ef of everything inserted whatever the insertion order, so the results
// are k_search_beam's bit for bit (test_gpu_parity.py: batches below and above
// BMW_MAX_B compared).
// ---------------------------------------------------------------------------
// (BmwShare, MwBatch: device_search.hpp, shared with the batched insert)
template <class C, int R, int G, bool SCREEN>
__global__ __launch_bounds__(64 * BMW_WAVES) void k_search_beam_mw(SearchArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    __shared__ BmwShare sh;
    const int64_t b = blockIdx.x;
    if (b >= a.B) return;  // (whole workgroup)
    const int wave = threadIdx.x >> 6;
    QReg<C> q;
    load_query(q, a.q + (size_t)b * C::PITCH);
    const float qn = query_norm(q);
    WaveStats st;
    if (wave == 0) {
        beam_query<C, R, G, SCREEN, 1>(a, b, q, qn, smem, st, MwBatch{&sh});
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
    beam_stats(a, st);
}

template <class C, int R, int G, int XW>
static int launch_beam_t(const SearchArgs& a, hipStream_t s) {
    const size_t lds = (size_t)4 * (size_t)(R >= 4 ? std::max(a.vis_n, beam_vis_words(a) + BL_MERGE_WORDS) : a.vis_n);
    // small batch: a workgroup per query (the standard search only; a wider
    // expansion runs the one-wave kernel at every batch size)
    if constexpr (XW == 1) {
        if (R <= 2 && a.B <= a.mw_max_b) {
            if (a.g.h16)
                hipLaunchKernelGGL((k_search_beam_mw<C, R, G, true>), dim3((unsigned)a.B), dim3(64 * BMW_WAVES), lds, s,
                                   a);
            else
                hipLaunchKernelGGL((k_search_beam_mw<C, R, G, false>), dim3((unsigned)a.B), dim3(64 * BMW_WAVES), lds,
                                   s, a);
            return hipGetLastError() == hipSuccess ? 0 : -1;
        }
    }
    if (a.g.h16)
        hipLaunchKernelGGL((k_search_beam<C, R, G, true, XW>), dim3((unsigned)a.B), dim3(64), lds, s, a);
    else
        hipLaunchKernelGGL((k_search_beam<C, R, G, false, XW>), dim3((unsigned)a.B), dim3(64), lds, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// group width G of configuration (L, V), from MH_FOR_EACH_CFG
template <int L, int V>
constexpr int beam_group() {
#define X_(L_, V_, G_) \
    if (L == L_ && V == V_) return G_;
    MH_FOR_EACH_CFG(X_)
#undef X_
    return 0;
}

template <int L, int V, int XW>
int launch_beam_cfg(const SearchArgs& a, hipStream_t s) {
    constexpr int G = beam_group<L, V>();
    const int efl = a.ef > a.k ? a.ef : a.k;
    if (efl <= 64) return launch_beam_t<Cfg<L, V>, 1, G, XW>(a, s);
    if (efl <= 128) return launch_beam_t<Cfg<L, V>, 2, G, XW>(a, s);
    if (efl <= 256) return launch_beam_t<Cfg<L, V>, 4, G, XW>(a, s);
    constexpr int GW = MH_BEAM_WIDE_G > 0 && MH_BEAM_WIDE_G < G ? MH_BEAM_WIDE_G : G;
    if (efl <= 512) return launch_beam_t<Cfg<L, V>, 8, GW, XW>(a, s);
    return -4;
}

}  // namespace mh
