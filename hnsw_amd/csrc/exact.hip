// exact.hip -- brute-force path (BASELINE config 5) and the multi-GPU merge.
//
//  k_scores : dense batched-query x base-block GEMM on the f32-input MFMA
//             (v_mfma_f32_32x32x2_f32, exact f32, no xf32 on gfx950) with the
//             metric epilogue fused (cosine: 1 - dot/(|q||x|); L2: |q|^2 +
//             |x|^2 - 2 q.x).  128x128x32 block tile, 4 waves of 64x64, LDS
//             double-buffered, rows padded to 36 floats so the 16-lane groups
//             of ds_read_b128 hit distinct 16-B slots.
//  k_select : per query, stream its score row and keep the best kk (<= 64)
//             (score, id) in a lane-per-entry sorted list (threshold filter).
//  k_rerank : recompute the kk candidates with the canonical distance engine
//             and keep the best k by (distance, id) -- bit-identical to the
//             oracle's brute force whenever the true top-k is inside the
//             GEMM top-kk.
//  k_merge  : per query, merge S shard top-k lists by (distance, key).
#include "device_search.hpp"
#include "engine.hpp"

namespace mh {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int EBM = 128, EBN = 128, EBK = 32, ELD = EBK + 4;

__global__ __launch_bounds__(256) void k_scores(ExactArgs a) {
    __shared__ __attribute__((aligned(16))) float sQ[2][EBM * ELD];
    __shared__ __attribute__((aligned(16))) float sX[2][EBN * ELD];
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    // XCD-aware order: consecutive query tiles of one base block share an XCD
    const int64_t nqt = (a.B + EBM - 1) / EBM;
    const int64_t bid = blockIdx.x;
    const int64_t qt = bid % nqt, nt = bid / nqt;
    const int64_t q0 = qt * EBM, n0 = nt * EBN;

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // staging: each thread moves 4 float4 of Q and 4 float4 of X per K-step
    float4 rq[4], rx[4];
    auto gload = [&](int k0) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int e = tid + t * 256;  // 0..1023 float4 slots: row = e/8, c4 = e%8
            const int row = e >> 3, c4 = e & 7;
            const int64_t qr = q0 + row, xr = n0 + row;
            rq[t] = qr < a.B ? *reinterpret_cast<const float4*>(a.Q + (size_t)qr * a.pitch + k0 + c4 * 4)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
            rx[t] = xr < a.N ? *reinterpret_cast<const float4*>(a.X + (size_t)xr * a.pitch + k0 + c4 * 4)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int e = tid + t * 256;
            const int row = e >> 3, c4 = e & 7;
            *reinterpret_cast<float4*>(&sQ[buf][row * ELD + c4 * 4]) = rq[t];
            *reinterpret_cast<float4*>(&sX[buf][row * ELD + c4 * 4]) = rx[t];
        }
    };

    const int nk = a.pitch / EBK;
    gload(0);
    lstore(0);
    __syncthreads();
    const int li = lane & 31, lh = lane >> 5;
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) gload((kt + 1) * EBK);
#pragma unroll
        for (int kb = 0; kb < EBK / 8; ++kb) {
            float4 fa[2], fb[2];
#pragma unroll
            for (int i = 0; i < 2; ++i)
                fa[i] = *reinterpret_cast<const float4*>(&sQ[cur][(wm * 64 + i * 32 + li) * ELD + kb * 8 + lh * 4]);
#pragma unroll
            for (int j = 0; j < 2; ++j)
                fb[j] = *reinterpret_cast<const float4*>(&sX[cur][(wn * 64 + j * 32 + li) * ELD + kb * 8 + lh * 4]);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].x, fb[j].x, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].y, fb[j].y, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].z, fb[j].z, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].w, fb[j].w, acc[i][j], 0, 0, 0);
                }
        }
        if (kt + 1 < nk) {
            lstore(cur ^ 1);
        }
        __syncthreads();
    }
    // epilogue: D[i][j] col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
    const float inf = __int_as_float(0x7f800000);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int64_t xr = n0 + wn * 64 + j * 32 + li;
        if (xr >= a.N) continue;
        const bool xok = !(a.dead && a.dead[xr]);
        const float xn = a.xnorm[xr];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t qr = q0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (qr >= a.B) continue;
                const float dot = acc[i][j][r];
                const float qn = a.qnorm[qr];
                float sc = a.metric == COSINE ? 1.0f - dot / (qn * xn) : fmaf(-2.f, dot, qn * qn + xn * xn);
                if (!xok || !(sc == sc)) sc = inf;
                a.scores[(size_t)qr * a.ldS + xr] = sc;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// top-kk preselect per query row (one wave per query)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_select(ExactArgs a) {
    const int64_t b = blockIdx.x;
    if (b >= a.B) return;
    const int lane = lane_id();
    const float* row = a.scores + (size_t)b * a.ldS;
    const float inf = __int_as_float(0x7f800000);
    BList<1> L;
    bl_init(L);
    const int kk = a.kk;
    float worst = inf;
    constexpr int U = 4;
    for (int64_t base = 0; base < a.N; base += 256 * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t e = base + u * 256 + lane * 4;
            v[u] = e < a.ldS ? *reinterpret_cast<const float4*>(row + e) : make_float4(inf, inf, inf, inf);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float vv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int64_t e = base + u * 256 + lane * 4 + c;
                const float x = e < a.N ? vv[c] : inf;
                unsigned long long m = __ballot(x < worst);
                while (m) {
                    const int src = __ffsll((long long)m) - 1;
                    m &= m - 1;
                    const float d = rl_f(x, src);
                    const uint32_t id = (uint32_t)(base + u * 256 + src * 4 + c);
                    if (bl_insert(L, kk, d, id)) {
                        float wd;
                        uint32_t wi;
                        bl_at(L, kk - 1, wd, wi);
                        worst = wi == EMPTY_ID ? inf : wd;
                    }
                }
            }
        }
    }
    if (lane < kk) a.cand[b * kk + lane] = (L.i[0] == EMPTY_ID) ? EMPTY_ID : (L.i[0] & ID_MASK);
}

// ---------------------------------------------------------------------------
// canonical re-rank of the kk candidates -> best k by (distance, id)
// ---------------------------------------------------------------------------
template <class C, int G>
__global__ __launch_bounds__(64) void k_rerank(const float* __restrict__ Q, GraphDev g, const uint32_t* cand, int kk,
                                               int64_t B, int k, int64_t* out_keys, float* out_dist, int32_t* out_n,
                                               int32_t* out_ids) {
    const int64_t b = blockIdx.x;
    if (b >= B) return;
    const int lane = lane_id();
    QReg<C> q;
    load_query(q, Q + (size_t)b * C::PITCH);
    const float qn = query_norm(q);
    const uint32_t c = lane < kk ? cand[b * kk + lane] : EMPTY_ID;
    int cnt;
    const uint32_t cid = compact(c, c != EMPTY_ID, cnt);
    BList<1> L;
    bl_init(L);
    eval_list<C, G>(g, q, qn, cid, cnt, g.metric, [&](float d, uint32_t u) { bl_insert(L, k, d, u); });
    const bool ok = lane < k && L.i[0] != EMPTY_ID;
    if (lane < k) {
        const uint32_t id = L.i[0] & ID_MASK;
        out_keys[b * k + lane] = ok ? g.keys[id] : (int64_t)-1;
        out_dist[b * k + lane] = ok ? L.d[0] : __int_as_float(0x7f800000);
        if (out_ids) out_ids[b * k + lane] = ok ? (int32_t)id : -1;
    }
    const int nv = __popcll(__ballot(ok));
    if (lane == 0) out_n[b] = nv;
}

// ---------------------------------------------------------------------------
// merge S shard lists (each sorted, n_in valid) -> best k by (distance, key)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_merge(const int64_t* keys_in, const float* dist_in, const int32_t* n_in,
                                              int S, int64_t B, int k, int64_t* out_keys, float* out_dist,
                                              int32_t* out_n) {
    extern __shared__ __attribute__((aligned(16))) unsigned char msm[];
    float* sd = reinterpret_cast<float*>(msm);
    int64_t* sk = reinterpret_cast<int64_t*>(msm + ((size_t)S * k * 4 + 15) / 16 * 16);
    const int64_t b = blockIdx.x;
    if (b >= B) return;
    const int lane = lane_id();
    const int tot = S * k;
    for (int e = lane; e < tot; e += 64) {
        const int s = e / k, j = e % k;
        const int nv = n_in[(size_t)s * B + b];
        const bool ok = j < nv;
        sd[e] = ok ? dist_in[((size_t)s * B + b) * k + j] : __int_as_float(0x7f800000);
        sk[e] = ok ? keys_in[((size_t)s * B + b) * k + j] : INT64_MAX;
    }
    __syncthreads();
    int nvalid = 0;
    for (int e = lane; e < tot; e += 64) {
        const float d = sd[e];
        const int64_t key = sk[e];
        const bool valid = key != INT64_MAX || d < __int_as_float(0x7f800000);
        int rank = 0;
        for (int f = 0; f < tot; ++f) {
            const float od = sd[f];
            const int64_t ok = sk[f];
            rank += (od < d || (od == d && (ok < key || (ok == key && f < e)))) ? 1 : 0;
        }
        if (valid && rank < k) {
            out_keys[b * k + rank] = key;
            out_dist[b * k + rank] = d;
        }
        nvalid += valid ? 1 : 0;
    }
    for (int o = 32; o >= 1; o >>= 1) nvalid += __shfl_xor(nvalid, o, 64);
    const int nout = nvalid < k ? nvalid : k;
    for (int j = nout + lane; j < k; j += 64) {
        out_keys[b * k + j] = -1;
        out_dist[b * k + j] = __int_as_float(0x7f800000);
    }
    if (lane == 0) out_n[b] = nout;
}

// ---------------------------------------------------------------------------
int launch_exact_scores(const ExactArgs& a, hipStream_t s) {
    if (a.B <= 0 || a.N <= 0) return 0;
    if (a.pitch % EBK) return -5;
    const int64_t nqt = (a.B + EBM - 1) / EBM, nnt = (a.N + EBN - 1) / EBN;
    hipLaunchKernelGGL(k_scores, dim3((unsigned)(nqt * nnt)), dim3(256), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_exact_select(const ExactArgs& a, hipStream_t s) {
    if (a.B <= 0) return 0;
    if (a.kk < 1 || a.kk > 64) return -4;
    hipLaunchKernelGGL(k_select, dim3((unsigned)a.B), dim3(64), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

#define MH_FOR_EACH_CFG(X) \
    X(16, 1, 2)            \
    X(32, 1, 4)            \
    X(64, 1, 8)            \
    X(64, 2, 8)            \
    X(64, 3, 8)            \
    X(64, 4, 4)            \
    X(64, 6, 4)            \
    X(64, 8, 2)

int launch_rerank(const float* Q, const GraphDev& g, const uint32_t* cand, int kk, int64_t B, int lpr, int vpl, int k,
                  int64_t* out_keys, float* out_dist, int32_t* out_n, int32_t* out_ids, hipStream_t s) {
    if (B <= 0) return 0;
    if (k > 64 || kk > 64) return -4;
#define X_(L, V, G)                                                                                           \
    if (lpr == L && vpl == V) {                                                                               \
        hipLaunchKernelGGL((k_rerank<Cfg<L, V>, G>), dim3((unsigned)B), dim3(64), 0, s, Q, g, cand, kk, B, k, \
                           out_keys, out_dist, out_n, out_ids);                                               \
        return hipGetLastError() == hipSuccess ? 0 : -1;                                                      \
    }
    MH_FOR_EACH_CFG(X_)
#undef X_
    return -3;
}

int launch_merge_topk(const int64_t* keys_in, const float* dist_in, const int32_t* n_in, int shards, int64_t B, int k,
                      int64_t* out_keys, float* out_dist, int32_t* out_n, hipStream_t s) {
    if (B <= 0) return 0;
    const size_t lds = ((size_t)shards * k * 4 + 15) / 16 * 16 + (size_t)shards * k * 8;
    if (lds > 64 * 1024) return -4;
    hipLaunchKernelGGL(k_merge, dim3((unsigned)B), dim3(64), lds, s, keys_in, dist_in, n_in, shards, B, k, out_keys,
                       out_dist, out_n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace mh
