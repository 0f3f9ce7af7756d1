// search.hip -- query-side kernels: row padding, canonical norms, the batched
// distance sweep (DistanceFunc, distance.go:12-23) and the batched layer
// descent + layer-0 search (Graph.Search / BatchSearch, graph.go:534-625,
// 1047-1110) in compat and beam modes.  One wave64 workgroup per query: the
// query lives in VGPRs, the visited set in LDS, the candidate list in VGPRs
// across lanes; candidate rows are gathered from HBM with 1-KiB coalesced
// wave loads.
#include "beam.hpp"
#include "walks.hpp"

namespace mh {
// instantiated in beam_*.hip / walks_*.hip
#define X_(L, V, G)                                                                    \
    extern template int launch_beam_cfg<L, V, 1>(const SearchArgs&, hipStream_t);    \
    extern template int launch_beam_cfg<L, V, 2>(const SearchArgs&, hipStream_t);    \
    extern template int launch_beam_cfg<L, V, 4>(const SearchArgs&, hipStream_t);    \
    extern template int launch_compat_cfg<L, V>(const SearchArgs&, hipStream_t);     \
    extern template int launch_negatives_cfg<L, V>(const NegArgs&, hipStream_t);
MH_FOR_EACH_CFG(X_)
#undef X_
}  // namespace mh

namespace mh {

__global__ void k_pad_rows(const float* __restrict__ src, int64_t n, int dim, float* __restrict__ dst, int pitch) {
    const int64_t total = n * (int64_t)pitch;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / pitch;
        const int c = (int)(i - r * pitch);
        dst[i] = c < dim ? src[r * dim + c] : 0.f;
    }
}

int launch_pad_rows(const float* src, int64_t n, int dim, float* dst, int pitch, hipStream_t s) {
    if (n <= 0) return 0;
    int64_t total = n * pitch;
    int grid = (int)((total + 255) / 256);
    if (grid > 65536) grid = 65536;
    hipLaunchKernelGGL(k_pad_rows, dim3(grid), dim3(256), 0, s, src, n, dim, dst, pitch);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// dst row ids[i] <- padded row i of src (rows already padded to pitch)
__global__ void k_scatter_rows(const float* __restrict__ src, const int32_t* __restrict__ ids, int64_t n, int pitch,
                               float* __restrict__ dst) {
    const int64_t total = n * (int64_t)pitch;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / pitch;
        dst[(size_t)ids[r] * pitch + (i - r * pitch)] = src[i];
    }
}

int launch_scatter_rows(const float* src, const int32_t* ids, int64_t n, int pitch, float* dst, hipStream_t s) {
    if (n <= 0) return 0;
    int64_t total = n * pitch;
    int64_t grid = (total + 255) / 256;
    if (grid > 65536) grid = 65536;
    hipLaunchKernelGGL(k_scatter_rows, dim3((unsigned)grid), dim3(256), 0, s, src, ids, n, pitch, dst);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// canonical |x| per row: one wave handles RPI rows per step
template <class C>
__global__ __launch_bounds__(256) void k_norms(const float* __restrict__ X, int64_t n0, int64_t n1, int pitch,
                                               float* __restrict__ out) {
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    const int64_t gw = (int64_t)blockIdx.x * 4 + wave;
    const int64_t row = n0 + gw * C::RPI + lane / C::LPR;
    const int sub = lane & (C::LPR - 1);
    float acc = 0.f;
    if (row < n1) {
        const float* rp = X + (size_t)row * pitch + sub * 4;
#pragma unroll
        for (int v = 0; v < C::VPL; ++v) {
            float4 x = *reinterpret_cast<const float4*>(rp + v * C::LPR * 4);
            acc = fmaf(x.x, x.x, acc);
            acc = fmaf(x.y, x.y, acc);
            acc = fmaf(x.z, x.z, acc);
            acc = fmaf(x.w, x.w, acc);
        }
    }
    acc = seg_allreduce<C::LPR>(acc);
    if (row < n1 && sub == 0) out[row] = sqrtf(acc);
}

// distance of one query against n rows (mhnsw_distance)
template <class C, int G>
__global__ __launch_bounds__(256) void k_sweep(const float* __restrict__ qp, const float* __restrict__ X, int64_t n,
                                               int pitch, int metric, float* __restrict__ out) {
    using RM = RowMap<C, G>;
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    const int64_t base = ((int64_t)blockIdx.x * 4 + wave) * RM::T;
    QReg<C> q;
    load_query(q, qp);
    const float qn = query_norm(q);
    uint32_t ids[G];
    bool valid[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int64_t r = base + RM::reg_row(g, lane);
        valid[g] = r < n;
        ids[g] = valid[g] ? (uint32_t)r : 0u;
    }
    // rows of the sweep operand are addressed relative to X directly
    float s = metric == EUCLIDEAN ? eval_rows<C, G, true>(q, X, pitch, ids, valid)
                                  : eval_rows<C, G, false>(q, X, pitch, ids, valid);
    const int64_t rown = base + RM::owned_row(lane);
    float xn = 1.f;
    // canonical |x| of the owned row: a second transposed pass (L1/L2-hot rows)
    if (metric == COSINE) {
        float p[G];
        const int sub = lane & (C::LPR - 1);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float acc = 0.f;
            if (valid[g]) {
                const float* rp = X + (size_t)ids[g] * pitch + sub * 4;
#pragma unroll
                for (int v = 0; v < C::VPL; ++v) {
                    float4 x = *reinterpret_cast<const float4*>(rp + v * C::LPR * 4);
                    acc = fmaf(x.x, x.x, acc);
                    acc = fmaf(x.y, x.y, acc);
                    acc = fmaf(x.z, x.z, acc);
                    acc = fmaf(x.w, x.w, acc);
                }
            }
            p[g] = acc;
        }
        xn = sqrtf(reduce_rows<G, C::LPR>(p));
    }
    const float d = finalize(metric, s, xn, qn);
    // the owning lane of each row is the first lane of its reduction group
    constexpr int GROUP = C::LPR >> RM::LG;
    if (rown < n && (lane & (GROUP - 1)) == 0) out[rown] = d;
}

// Allocation-free sweep over raw rows (dim-contiguous, any alignment): one
// wave per row, lane l owns elements e with (e/4) mod 64 == l (canonical order).
__global__ __launch_bounds__(256) void k_sweep_raw(const float* __restrict__ q, const float* __restrict__ X,
                                                   int64_t n, int dim, int metric, float* __restrict__ out) {
    const int lane = lane_id();
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    const float* x = X + (size_t)row * dim;
    float acc = 0.f, xx = 0.f, qq = 0.f;
    for (int base = 4 * lane; base < dim; base += 256) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = base + j;
            if (e < dim) {
                const float a = x[e], b = q[e];
                if (metric == EUCLIDEAN) {
                    const float t = a - b;
                    acc = fmaf(t, t, acc);
                } else {
                    acc = fmaf(a, b, acc);
                    xx = fmaf(a, a, xx);
                    qq = fmaf(b, b, qq);
                }
            }
        }
    }
    acc = seg_allreduce<64>(acc);
    if (metric == COSINE) {
        xx = seg_allreduce<64>(xx);
        qq = seg_allreduce<64>(qq);
    }
    if (lane == 0) out[row] = finalize(metric, acc, sqrtf(xx), sqrtf(qq));
}

// The same sweep for 16-B aligned rows with dim % 4 == 0 (the common case):
// lane l loads its elements as float4 (one 1-KiB wave instruction per 256
// elements), the query and its canonical |q| stay in registers for every row
// of a grid-stride loop, RP rows in flight per step (4 up to 1,024-d, else 2),
// read with non-temporal loads (each row is read once: no point keeping it in
// the caches).  Identical arithmetic order, so identical bits.  HBM-bound:
// n * dim * 4 bytes per query.
// (MH_SWEEP_RP / MH_SWEEP_GRID(_L2) / MH_SWEEP_NT: build flags for tools/ variants --
// rows in flight up to 1,024-d, the grid caps, non-temporal row loads)
#ifndef MH_SWEEP_RP
#define MH_SWEEP_RP 4
#endif
#ifndef MH_SWEEP_GRID
#define MH_SWEEP_GRID 16384
#endif
#ifndef MH_SWEEP_GRID_L2
#define MH_SWEEP_GRID_L2 65536
#endif
#ifndef MH_SWEEP_NT
#define MH_SWEEP_NT 1
#endif
template <int VPL>
__global__ __launch_bounds__(256) void k_sweep_raw4(const float* __restrict__ q, const float* __restrict__ X,
                                                    int64_t n, int dim, int metric, float* __restrict__ out) {
    constexpr int RP = VPL <= 4 ? MH_SWEEP_RP : 2;
    const int lane = lane_id();
    const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t nw = (int64_t)gridDim.x * 4;
    float4 qv[VPL];
    float qq = 0.f;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
        const int e = v * 256 + 4 * lane;
        qv[v] = e < dim ? *reinterpret_cast<const float4*>(q + e) : make_float4(0.f, 0.f, 0.f, 0.f);
        if (e < dim) {
            qq = fmaf(qv[v].x, qv[v].x, qq);
            qq = fmaf(qv[v].y, qv[v].y, qq);
            qq = fmaf(qv[v].z, qv[v].z, qq);
            qq = fmaf(qv[v].w, qv[v].w, qq);
        }
    }
    const float qn = metric == COSINE ? sqrtf(seg_allreduce<64>(qq)) : 1.f;
    for (int64_t r0 = gw * RP; r0 < n; r0 += nw * RP) {
        float4 xv[RP][VPL];
#pragma unroll
        for (int h = 0; h < RP; ++h) {
            const int64_t row = r0 + h < n ? r0 + h : r0;
            const float* x = X + (size_t)row * dim;
#pragma unroll
            for (int v = 0; v < VPL; ++v) {
                const int e = v * 256 + 4 * lane;
                typedef float f4v __attribute__((ext_vector_type(4)));
                f4v t = {0.f, 0.f, 0.f, 0.f};
                if (e < dim)
                    t = MH_SWEEP_NT ? __builtin_nontemporal_load(reinterpret_cast<const f4v*>(x + e))
                                    : *reinterpret_cast<const f4v*>(x + e);
                xv[h][v] = make_float4(t.x, t.y, t.z, t.w);
            }
        }
#pragma unroll
        for (int h = 0; h < RP; ++h) {
            float acc = 0.f, xx = 0.f;
#pragma unroll
            for (int v = 0; v < VPL; ++v) {
                if (v * 256 + 4 * lane >= dim) continue;
                const float4 a = xv[h][v], b = qv[v];
                if (metric == EUCLIDEAN) {
                    float t = a.x - b.x;
                    acc = fmaf(t, t, acc);
                    t = a.y - b.y;
                    acc = fmaf(t, t, acc);
                    t = a.z - b.z;
                    acc = fmaf(t, t, acc);
                    t = a.w - b.w;
                    acc = fmaf(t, t, acc);
                } else {
                    acc = fmaf(a.x, b.x, acc);
                    xx = fmaf(a.x, a.x, xx);
                    acc = fmaf(a.y, b.y, acc);
                    xx = fmaf(a.y, a.y, xx);
                    acc = fmaf(a.z, b.z, acc);
                    xx = fmaf(a.z, a.z, xx);
                    acc = fmaf(a.w, b.w, acc);
                    xx = fmaf(a.w, a.w, xx);
                }
            }
            acc = seg_allreduce<64>(acc);
            if (metric == COSINE) xx = seg_allreduce<64>(xx);
            if (lane == 0 && r0 + h < n) out[r0 + h] = finalize(metric, acc, sqrtf(xx), qn);
        }
    }
}

int launch_sweep_raw(const float* q, const float* X, int64_t n, int dim, int metric, float* out, hipStream_t s) {
    if (n <= 0) return 0;
    const bool vec = dim % 4 == 0 && dim <= 4096 && ((uintptr_t)q & 15) == 0 && ((uintptr_t)X & 15) == 0;
    if (vec) {
        const int vpl = (dim + 255) / 256;
        // grid cap: cosine keeps a grid-stride loop over 16,384 workgroups (each
        // wave reduces |q| once); L2 (no |q|) runs one 16-row block per
        // workgroup up to 65,536 (profiles/r06_sweep_variants.txt)
        const int grid = (int)std::min<int64_t>((n + 15) / 16, metric == EUCLIDEAN ? MH_SWEEP_GRID_L2 : MH_SWEEP_GRID);
#define SW_(V)                                                                                            \
    if (vpl <= V) {                                                                                       \
        hipLaunchKernelGGL(k_sweep_raw4<V>, dim3((unsigned)grid), dim3(256), 0, s, q, X, n, dim, metric, out); \
        return hipGetLastError() == hipSuccess ? 0 : -1;                                                  \
    }
        SW_(1) SW_(2) SW_(3) SW_(4) SW_(6) SW_(8) SW_(12) SW_(16)
#undef SW_
    }
    hipLaunchKernelGGL(k_sweep_raw, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, q, X, n, dim, metric, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <class C>
static int launch_norms_t(const float* X, int64_t n0, int64_t n1, int pitch, float* out, hipStream_t s) {
    const int64_t rows = n1 - n0;
    if (rows <= 0) return 0;
    const int64_t waves = (rows + C::RPI - 1) / C::RPI;
    const int grid = (int)((waves + 3) / 4);
    hipLaunchKernelGGL(k_norms<C>, dim3(grid), dim3(256), 0, s, X, n0, n1, pitch, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <class C, int G>
static int launch_sweep_t(const float* q, const float* X, int64_t n, int pitch, int metric, float* out,
                          hipStream_t s) {
    if (n <= 0) return 0;
    constexpr int T = G * C::RPI;
    const int64_t waves = (n + T - 1) / T;
    const int grid = (int)((waves + 3) / 4);
    hipLaunchKernelGGL((k_sweep<C, G>), dim3(grid), dim3(256), 0, s, q, X, n, pitch, metric, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------------------
// fp16 screening copy of rows [n0, n1) (device_common.hpp GraphDev::h16), one
// wave per row; norms[r] (canonical |x|) must already be written.
//   cosine: fp16(x_i * (1/|x|) * 2^14); rows outside the screen's validity
//           range (max|x_i| not in [2^-50, 2^50], any non-finite value) get
//           NaN halves, which make every screening test on them false
//   L2:     fp16(x_i * 2^e), max|x_i| 2^e in [2^14, 2^15) (exact power of two);
//           aux[r] = {2^-e, |x|}, 2^-e = NaN outside the validity range
// Rounding is to nearest; the bounds are in device_common.hpp (H16_*).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_h16_rows(const float* __restrict__ X, const float* __restrict__ norms,
                                                  int64_t n0, int64_t n1, int pitch, int metric,
                                                  uint16_t* __restrict__ H, float2* __restrict__ aux,
                                                  float* __restrict__ err) {
    const int lane = lane_id();
    const int64_t r = n0 + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n1) return;
    const float* xp = X + (size_t)r * pitch;
    float m = 0.f;
    bool fin = true;
    for (int e = lane * 4; e < pitch; e += 256) {
        const float4 v = *reinterpret_cast<const float4*>(xp + e);
        fin = fin && isfinite(v.x) && isfinite(v.y) && isfinite(v.z) && isfinite(v.w);
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    fin = __ballot(!fin) == 0ull;
    const float xn = norms[r];
    const bool ok = fin && m >= 8.881784197001252e-16f && m <= 1.125899906842624e15f &&  // [2^-50, 2^50]
                    xn > 0.f && isfinite(xn);
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    const _Float16 hnan = __builtin_bit_cast(_Float16, (uint16_t)0x7E00);
    int k = 0;
    if (ok) (void)frexpf(m, &k);  // m = f * 2^k, f in [0.5, 1)
    const int ex = 15 - k;        // m * 2^ex in [2^14, 2^15)
    const float rx = ok ? 16384.0f / xn : 0.f;
    // the row's measured rounding against y = x / |x|_f32 (cosine) or x (L2), in f64
    double e2 = 0.0, y2 = 0.0;
    const double inx = ok ? 1.0 / (double)xn : 0.0;
    for (int e = lane * 4; e < pitch; e += 256) {
        const float4 v = *reinterpret_cast<const float4*>(xp + e);
        h4 o;
        if (!ok)
            o = metric == COSINE ? h4{hnan, hnan, hnan, hnan} : h4{0, 0, 0, 0};
        else if (metric == COSINE)
            o = h4{(_Float16)(v.x * rx), (_Float16)(v.y * rx), (_Float16)(v.z * rx), (_Float16)(v.w * rx)};
        else
            o = h4{(_Float16)ldexpf(v.x, ex), (_Float16)ldexpf(v.y, ex), (_Float16)ldexpf(v.z, ex),
                   (_Float16)ldexpf(v.w, ex)};
        if (ok) {
            const float xv[4] = {v.x, v.y, v.z, v.w};
            const _Float16 ov[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const double y = metric == COSINE ? (double)xv[c] * inx : (double)xv[c];
                const double yq = metric == COSINE ? (double)(float)ov[c] * 0x1p-14 : ldexp((double)(float)ov[c], -ex);
                e2 = fma(yq - y, yq - y, e2);
                y2 = fma(y, y, y2);
            }
        }
        // lane-contiguous layout (eval_rows_h16)
        *reinterpret_cast<h4*>(H + (size_t)r * pitch + lane * 4 * lc_vpl(pitch) + (e >> 8) * 4) = o;
    }
    if (lane == 0) aux[r] = make_float2(ok ? ldexpf(1.f, -ex) : __int_as_float(0x7fc00000), xn);
    if (err && ok) {  // rows outside the range never reject: they do not count
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            e2 += __shfl_xor(e2, o, 64);
            y2 += __shfl_xor(y2, o, 64);
        }
        // relative to |y| (cosine: |y| = |x| / |x|_f32 ~ 1), padded for the f64 sums and the rounding to f32
        const float rel = y2 > 0.0 ? (float)(sqrt(e2 / y2) * (1.0 + 1e-6)) : 0.f;
        if (lane == 0) atomicMax(reinterpret_cast<unsigned int*>(err), __float_as_uint(rel));
    }
}

int launch_h16_rows(const float* X, const float* norms, int64_t n0, int64_t n1, int pitch, int metric, uint16_t* H,
                    float2* aux, float* err, hipStream_t s) {
    const int64_t rows = n1 - n0;
    if (rows <= 0) return 0;
    hipLaunchKernelGGL(k_h16_rows, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, X, norms, n0, n1, pitch, metric,
                       H, aux, err);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_norms(const float* X, int64_t n0, int64_t n1, int pitch, int lpr, int vpl, float* out, hipStream_t s) {
#define X_(L, V, G) \
    if (lpr == L && vpl == V) return launch_norms_t<Cfg<L, V>>(X, n0, n1, pitch, out, s);
    MH_FOR_EACH_CFG(X_)
#undef X_
    return -3;
}

int launch_sweep(const float* q, const float* X, int64_t n, int pitch, int lpr, int vpl, int metric, float* out,
                 hipStream_t s) {
#define X_(L, V, G) \
    if (lpr == L && vpl == V) return launch_sweep_t<Cfg<L, V>, G>(q, X, n, pitch, metric, out, s);
    MH_FOR_EACH_CFG(X_)
#undef X_
    return -3;
}

int launch_search_beam(const SearchArgs& a, int lpr, int vpl, hipStream_t s) {
    if (a.B <= 0) return 0;
#define X_(L, V, G)                                                   \
    if (lpr == L && vpl == V)                                         \
        return a.expand == 4 ? launch_beam_cfg<L, V, 4>(a, s)         \
               : a.expand == 2 ? launch_beam_cfg<L, V, 2>(a, s)       \
                               : launch_beam_cfg<L, V, 1>(a, s);
    MH_FOR_EACH_CFG(X_)
#undef X_
    return -3;
}

int launch_negatives(const NegArgs& a, int lpr, int vpl, hipStream_t s) {
    if (a.B <= 0) return 0;
    if (a.kx > NEG_MAX_CAND) return -4;
#define X_(L, V, G) \
    if (lpr == L && vpl == V) return launch_negatives_cfg<L, V>(a, s);
    MH_FOR_EACH_CFG(X_)
#undef X_
    return -3;
}

int launch_search_compat(const SearchArgs& a, int lpr, int vpl, hipStream_t s) {
    if (a.B <= 0) return 0;
#define X_(L, V, G) \
    if (lpr == L && vpl == V) return launch_compat_cfg<L, V>(a, s);
    MH_FOR_EACH_CFG(X_)
#undef X_
    return -3;
}

}  // namespace mh
