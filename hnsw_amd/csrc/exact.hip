// exact.hip -- brute-force path (BASELINE config 5) and the multi-GPU merge.
//
//  k_scores : dense batched-query x base-block GEMM on the f32-input MFMA
//             (v_mfma_f32_32x32x2_f32, exact f32, no xf32 on gfx950) with the
//             metric epilogue fused (cosine: 1 - dot/(|q||x|); L2: |q|^2 +
//             |x|^2 - 2 q.x).  128x128x32 block tile, 4 waves of 64x64, LDS
//             double-buffered, rows padded to 36 floats so the 16-lane groups
//             of ds_read_b128 hit distinct 16-B slots.
//  k_scores_x3 : the same scores from the bf16x3 split (x = hi + lo, both
//             bf16; q.x ~ qh.xh + qh.xl + ql.xh on v_mfma_f32_32x32x16_bf16,
//             16x the f32-input rate per instruction), 256x256 block tile,
//             8 waves of 128x64, operands staged by LDS-DMA into a 4-deep
//             ring of swizzled buffers (three K-stages in flight).
//  k_select : per query, stream its score row and keep the best kk (<= 256)
//             (score, id) in a lane-per-entry sorted list (threshold filter);
//             the kk-th score is the query's preselection bound.
//  k_rerank : recompute the kk candidates with the canonical distance engine,
//             keep the best k by (distance, id), and certify the query: with
//             eps bounding |approx - canonical| for every row, no row left
//             out of the kk can enter the canonical top-k when the k-th
//             canonical distance is below bound - eps.  Uncertified queries
//             are redone exactly (k_exact_fallback: canonical distances of
//             every row, then select + re-rank), so the output is the
//             oracle's brute force bit for bit.
//  k_merge  : per query, merge S shard top-k lists by (distance, key).
#include <algorithm>
#include <type_traits>
#include <utility>

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
// bf16x3 split path
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int X3K = 16;  // K-block of the split planes = GEMM K-stage (one 32x32x16 MFMA step)

// round-to-nearest-even f32 -> bf16 bits (NaN stays NaN)
__device__ __forceinline__ uint32_t bf16_rne(float v) {
    const uint32_t u = __float_as_uint(v);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ float bf16_val(uint32_t h) { return __uint_as_float(h << 16); }

// x = hi + lo + r with hi = bf16(x), lo = bf16(x - hi) (x - hi is exact in f32),
// |r| <= 2^-16 |x|.  Rows [r0, r1) of a pitch-strided f32 array go to K-blocked
// planes: element (row, k) at ((k / 16) * rows + row) * 16 + k % 16, so one GEMM
// K-stage of consecutive rows is a single contiguous run.
__global__ void k_split_rows(const float* __restrict__ src, int64_t r0, int64_t r1, int pitch, int64_t rows,
                             uint16_t* __restrict__ hi, uint16_t* __restrict__ lo) {
    const int q4 = pitch / 4;
    const int64_t total = (r1 - r0) * (int64_t)q4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t row = r0 + i / q4;
        const int k = (int)(i % q4) * 4;
        const float4 v = *reinterpret_cast<const float4*>(src + row * (int64_t)pitch + k);
        const uint32_t a0 = bf16_rne(v.x), a1 = bf16_rne(v.y), a2 = bf16_rne(v.z), a3 = bf16_rne(v.w);
        const uint32_t b0 = bf16_rne(v.x - bf16_val(a0)), b1 = bf16_rne(v.y - bf16_val(a1));
        const uint32_t b2 = bf16_rne(v.z - bf16_val(a2)), b3 = bf16_rne(v.w - bf16_val(a3));
        const int64_t o = ((int64_t)(k / X3K) * rows + row) * X3K + (k % X3K);
        *reinterpret_cast<uint2*>(hi + o) = make_uint2(a0 | (a1 << 16), a2 | (a3 << 16));
        *reinterpret_cast<uint2*>(lo + o) = make_uint2(b0 | (b1 << 16), b2 | (b3 << 16));
    }
}

int launch_split_rows(const float* src, int64_t r0, int64_t r1, int pitch, int64_t rows, uint16_t* hi, uint16_t* lo,
                      hipStream_t s) {
    if (r1 <= r0) return 0;
    if (pitch % X3K || r1 > rows) return -5;
    const int64_t total = (r1 - r0) * (int64_t)pitch / 4;
    const int grid = (int)std::min<int64_t>((total + 255) / 256, 8192);
    hipLaunchKernelGGL(k_split_rows, dim3(grid), dim3(256), 0, s, src, r0, r1, pitch, rows, hi, lo);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// fp16 planes for the 2-product split (exact_precision 2): row r is scaled by
// 2^e (max|x_i| 2^e in [2^14, 2^15), a power of two, so exact) and hi =
// fp16(x 2^e); with `lo` also lo = fp16(x 2^e - hi) (queries: hi + lo carries
// 22 bits).  inv[r] = 2^-e.  A row the error bound does not cover (a
// non-finite value, or max|x_i| outside [2^-40, 2^40] and not 0) gets inv =
// NaN: the GEMM epilogue scores it -inf, so a row is always preselected (and
// re-ranked canonically) and a query always fails its certificate (and is
// redone by the canonical sweep).  Same K-blocked layout as k_split_rows; one
// wave per row.
__global__ __launch_bounds__(256) void k_split_h16(const float* __restrict__ src, int64_t r0, int64_t r1, int pitch,
                                                   int64_t rows, uint16_t* __restrict__ hi, uint16_t* __restrict__ lo,
                                                   float* __restrict__ inv, float* __restrict__ err) {
    const int lane = threadIdx.x & 63;
    const int64_t row = r0 + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= r1) return;
    const float* xp = src + row * (int64_t)pitch;
    float m = 0.f;
    bool fin = true;
    for (int k = lane * 4; k < pitch; k += 256) {
        const float4 v = *reinterpret_cast<const float4*>(xp + k);
        fin = fin && isfinite(v.x) && isfinite(v.y) && isfinite(v.z) && isfinite(v.w);
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    fin = __ballot(!fin) == 0ull;
    const bool ok = fin && (m == 0.f || (m >= 9.094947017729282e-13f && m <= 1.099511627776e12f));
    int ex = 0;
    if (ok && m > 0.f) {
        int kx;
        (void)frexpf(m, &kx);
        ex = 15 - kx;
    }
    double e2 = 0.0, x2 = 0.0;  // |hi 2^-e - x|^2 and |x|^2, exact enough in f64
    for (int k = lane * 4; k < pitch; k += 256) {
        const float4 v = *reinterpret_cast<const float4*>(xp + k);
        const float w[4] = {ldexpf(v.x, ex), ldexpf(v.y, ex), ldexpf(v.z, ex), ldexpf(v.w, ex)};
        const float xv[4] = {v.x, v.y, v.z, v.w};
        uint16_t h[4], l[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const _Float16 hh = ok ? (_Float16)w[c] : (_Float16)0.f;
            h[c] = __builtin_bit_cast(uint16_t, hh);
            l[c] = __builtin_bit_cast(uint16_t, ok ? (_Float16)(w[c] - (float)hh) : (_Float16)0.f);
            const double dv = ldexp((double)(float)hh, -ex) - (double)xv[c];
            e2 = fma(dv, dv, e2);
            x2 = fma((double)xv[c], (double)xv[c], x2);
        }
        const int64_t o = ((int64_t)(k / X3K) * rows + row) * X3K + (k % X3K);
        *reinterpret_cast<uint2*>(hi + o) = make_uint2(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16));
        if (lo) *reinterpret_cast<uint2*>(lo + o) = make_uint2(l[0] | ((uint32_t)l[1] << 16), l[2] | ((uint32_t)l[3] << 16));
    }
    if (lane == 0) inv[row] = ok ? ldexpf(1.f, -ex) : __int_as_float(0x7fc00000);
    if (err && ok) {  // the row's relative rounding |x' - x| / |x|, rounded up, into the running max
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            e2 += __shfl_xor(e2, o, 64);
            x2 += __shfl_xor(x2, o, 64);
        }
        const float rel = x2 > 0.0 ? (float)(sqrt(e2 / x2) * (1.0 + 1e-6)) : 0.f;
        if (lane == 0) atomicMax(reinterpret_cast<unsigned int*>(err), __float_as_uint(rel));
    }
}

int launch_split_h16(const float* src, int64_t r0, int64_t r1, int pitch, int64_t rows, uint16_t* hi, uint16_t* lo,
                     float* inv, float* err, hipStream_t s) {
    if (r1 <= r0) return 0;
    if (pitch % X3K || r1 > rows) return -5;
    hipLaunchKernelGGL(k_split_h16, dim3((unsigned)((r1 - r0 + 3) / 4)), dim3(256), 0, s, src, r0, r1, pitch, rows, hi,
                       lo, inv, err);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// largest row norm (NaN skipped) into *out (zeroed by the caller)
__global__ __launch_bounds__(256) void k_max_norm(const float* __restrict__ norms, int64_t n, float* out) {
    float m = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float v = norms[i];
        if (v > m) m = v;
    }
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<unsigned int*>(out), __float_as_uint(m));
}

int launch_max_norm(const float* norms, int64_t n, float* out, hipStream_t s) {
    if (n <= 0) return 0;
    const int grid = (int)std::min<int64_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(k_max_norm, dim3(grid), dim3(256), 0, s, norms, n, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Split-operand GEMM modes (planes of A = queries, B = rows, all K-blocked by 16):
//   RING_X3 bf16x3     q.x ~ ql.xh + qh.xl + qh.xh  (A hi+lo, B hi+lo)
//   RING_H2 fp16 2-pr. q.x ~ ql.xh + qh.xh          (A hi+lo, B hi; rows rounded once)
//   RING_H1 fp16 1-pr. q.x ~ qh.xh                  (A hi,    B hi; both rounded once)
enum { RING_X3 = 0, RING_H2 = 1, RING_H1 = 2 };

// Block tile BM (queries) x BN (rows) = (WAVES_M*TM*32) x (WAVES_N*TN*32).  One
// ring stage = S K-blocks of 16.  LDS image of one K-block: [A hi][A lo][B hi]
// [B lo] (planes the mode uses), each rows x 16 halves (two 16-B chunks per
// row); chunk c of row r sits at chunk position c ^ ((r >> 3) & 1), so the 16
// consecutive rows one quarter of a ds_read_b128 touches land in 16 distinct
// 16-B slots of the 256-B bank window.
template <int WAVES_M, int WAVES_N, int TM, int TN, int MODE, int S>
struct RingTile {
    static constexpr int BM = WAVES_M * TM * 32, BN = WAVES_N * TN * 32;
    static constexpr int NT = 64 * WAVES_M * WAVES_N, NW = WAVES_M * WAVES_N;
    static constexpr int APL = MODE == RING_H1 ? 1 : 2;  // query planes
    static constexpr int XPL = MODE == RING_X3 ? 2 : 1;  // row planes
    static constexpr int KBE = (APL * BM + XPL * BN) * X3K;  // 16-bit elements of one K-block image
    static constexpr int STAGE = KBE * S;
    static constexpr int KB_PIECES = KBE * 2 / 1024;  // 1-KiB LDS-DMA pieces per K-block
    static constexpr int PIECES = KB_PIECES * S;
    static_assert(PIECES % NW == 0, "DMA split");
    static constexpr int PER = PIECES / NW;
};

__device__ __forceinline__ int swz16(int r, int c) { return r * X3K + ((c ^ ((r >> 3) & 1)) << 3); }

__device__ __forceinline__ void x3_dma(const uint16_t* src, uint16_t* lds) {
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                     (__attribute__((address_space(3))) void*)(lds), 16, 0, 0);
}

// Fragments of one 16-deep K-block (base = the K-block's image) for a wave's
// TM x TN tiles, and their MFMAs.  ring_stage reads every K-block of a stage
// before the first MFMA, so the LDS latency of block s+1 hides behind the
// MFMAs of block s (the compiler's lgkmcnt waits become partial).
template <class T, int TM, int TN>
struct RingFrag {
    u32x4 ah[TM], al[TM], bh[TN], bl[TN];
};

template <class T, int TM, int TN>
__device__ __forceinline__ void ring_load(const uint16_t* base, RingFrag<T, TM, TN>& f, int wm, int wn, int li, int lh) {
    const uint16_t* Ah = base;
    const uint16_t* Al = base + T::BM * X3K;
    const uint16_t* Bh = base + T::APL * T::BM * X3K;
    const uint16_t* Bl = Bh + T::BN * X3K;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int r = wm * TM * 32 + i * 32 + li;
        f.ah[i] = *reinterpret_cast<const u32x4*>(Ah + swz16(r, lh));
        if constexpr (T::APL == 2) f.al[i] = *reinterpret_cast<const u32x4*>(Al + swz16(r, lh));
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int r = wn * TN * 32 + j * 32 + li;
        f.bh[j] = *reinterpret_cast<const u32x4*>(Bh + swz16(r, lh));
        if constexpr (T::XPL == 2) f.bl[j] = *reinterpret_cast<const u32x4*>(Bl + swz16(r, lh));
    }
}

template <class T, int MODE, int TM, int TN>
__device__ __forceinline__ void ring_mma(const RingFrag<T, TM, TN>& f, f32x16 (&acc)[TM][TN]) {
    typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            if constexpr (MODE == RING_X3) {  // small cross terms first, the dominant hi*hi last
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, f.al[i]),
                                                                    __builtin_bit_cast(bf16x8, f.bh[j]), acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, f.ah[i]),
                                                                    __builtin_bit_cast(bf16x8, f.bl[j]), acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, f.ah[i]),
                                                                    __builtin_bit_cast(bf16x8, f.bh[j]), acc[i][j], 0, 0, 0);
            } else {
                if constexpr (MODE == RING_H2)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, f.al[i]),
                                                                       __builtin_bit_cast(f16x8, f.bh[j]), acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, f.ah[i]),
                                                                   __builtin_bit_cast(f16x8, f.bh[j]), acc[i][j], 0, 0, 0);
            }
        }
}

template <class T, int MODE, int TM, int TN, int S>
__device__ __forceinline__ void ring_stage(const uint16_t* buf, f32x16 (&acc)[TM][TN], int wm, int wn, int li,
                                           int lh) {
    RingFrag<T, TM, TN> f[S];
#pragma unroll
    for (int sb = 0; sb < S; ++sb) ring_load<T, TM, TN>(buf + sb * T::KBE, f[sb], wm, wn, li, lh);
    // priority 1 while this wave's MFMA cluster issues (cdna_hip_programming.md T5:
    // keeps the cluster between the barriers instead of among the DMA issues)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int sb = 0; sb < S; ++sb) ring_mma<T, MODE, TM, TN>(f[sb], acc);
    __builtin_amdgcn_s_setprio(0);
}

// the score of one (query, row) pair from its accumulator -- the one formula
// every consumer of split scores uses (write epilogue, candidate select), so
// a score is the same float wherever it is computed.  Outside the fp16 bound
// (NaN unscale): -inf, always preselected / never certified.
__device__ __forceinline__ float split_score(int mode, int metric, float acc, float xi, float qi, float qn, float xn) {
    const float dot = mode != RING_X3 ? acc * xi * qi : acc;
    float sc = metric == COSINE ? 1.0f - dot / (qn * xn) : fmaf(-2.f, dot, qn * qn + xn * xn);
    if (!(sc == sc)) sc = __int_as_float(0x7f800000);
    if (mode != RING_X3 && !(xi == xi && qi == qi)) sc = -__int_as_float(0x7f800000);
    return sc;
}

// Staged by LDS-DMA (global_load_lds_dwordx4: 1 KiB per wave instruction
// straight into LDS -- no staging registers, no ds_write pass) into a ring of
// R buffers, R separate __shared__ objects so the compiler's wait counting can
// tell which buffer a pending DMA targets.  Stage t lives in buffer t % R.
// Step t: wait for this wave's stage-t pieces (vmcnt leaves stages t+1 ..
// t+R-2 in flight), barrier (everyone's stage t landed, everyone finished step
// t-1), issue stage t+R-1 into the buffer step t-1 read, multiply.  The loop is
// unrolled by R; DMA issue is unconditional (past the end it re-reads the last
// K-blocks into a buffer nobody reads) so the in-flight count is the same
// every step.  A lane's source chunk is pre-swizzled on the global side so the
// linear LDS-DMA image matches swz16().
//
// Epilogues: EPI 0 writes every score (nsample_tiles > 0: only row tiles 0,
// tile_stride, 2 tile_stride, ..., into a compact [B x ns] sample matrix); EPI 1 keeps
// only the pairs that can beat the query's threshold (RingFilter, below) --
// the fused top-k: no score matrix.
template <int WAVES_M, int WAVES_N, int TM, int TN, int MODE, int S, int R, int EPI>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void k_scores_ring(ExactArgs a) {
    using T = RingTile<WAVES_M, WAVES_N, TM, TN, MODE, S>;
    static_assert(R >= 2 && R <= 4, "ring depth");
    // B0's tail: the tile's region counter (EPI 1)
    __shared__ __attribute__((aligned(16))) uint16_t B0[T::STAGE + 8];
    __shared__ __attribute__((aligned(16))) uint16_t B1[T::STAGE];
    __shared__ __attribute__((aligned(16))) uint16_t B2[R > 2 ? T::STAGE : 8];
    __shared__ __attribute__((aligned(16))) uint16_t B3[R > 3 ? T::STAGE : 8];
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    // XCD-aware tile order: round-robin dispatch puts block i on XCD i % 8; give
    // every XCD a contiguous run of logical tiles, query tiles fastest, so one
    // base tile is read into an XCD's L2 once and reused by all query tiles.
    const int64_t nqt = (a.B + T::BM - 1) / T::BM;
    const int64_t nnt = EPI == 0 && a.nsample_tiles > 0 ? a.nsample_tiles : (a.N + T::BN - 1) / T::BN;
    const int64_t nblk = nqt * nnt;
    const int64_t per = nblk / 8, rem = nblk % 8;
    const int64_t xcd = blockIdx.x % 8, idx = blockIdx.x / 8;
    const int64_t logical = xcd < rem ? xcd * (per + 1) + idx : rem * (per + 1) + (xcd - rem) * per + idx;
    const int64_t qt = logical % nqt, nt = logical / nqt;
    const int64_t q0 = qt * T::BM;
    const int64_t n0 = (EPI == 0 && a.nsample_tiles > 0 ? nt * a.tile_stride : nt) * T::BN;
    int* const tile_ctr = reinterpret_cast<int*>(B0 + T::STAGE);
    if (EPI == 1 && tid == 0) *tile_ctr = 0;  // ordered before the epilogue by the mainloop's barriers

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // this wave's DMA pieces.  A piece = 32 rows x 32 B of one plane of one
    // K-block.  Its source is a wave-uniform base (plane + first row of the
    // tile + the stage's K-blocks: scalar registers, advanced by scalar adds)
    // plus a per-lane 32-bit byte offset (row within the tile, chunk, K-block
    // within the stage), so each piece is one global_load_lds with an SGPR base
    // and no per-stage vector address arithmetic.  Rows past B / N are clamped
    // to the last row (valid loads; their products land in outputs never stored).
    const int wv = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform piece numbers
    const char* pb[T::PER];
    int64_t pstep[T::PER];  // bytes per ring stage (uniform)
    uint32_t poff[T::PER];
    int lofs[T::PER];
#pragma unroll
    for (int j = 0; j < T::PER; ++j) {
        const int I = wv * T::PER + j;
        const int sblk = I / T::KB_PIECES, Ik = I % T::KB_PIECES;
        const int apieces = T::APL * T::BM / 32;
        int r;
        const uint16_t* base;
        int64_t row0, rmax, ld;
        if (Ik < apieces) {
            const int plane = Ik / (T::BM / 32);
            r = (Ik % (T::BM / 32)) * 32 + (lane >> 1);
            base = plane ? a.Ql : a.Qh;
            row0 = q0;
            rmax = a.B - 1;
            ld = a.ldQs;
        } else {
            const int I2 = Ik - apieces;
            const int plane = I2 / (T::BN / 32);
            r = (I2 % (T::BN / 32)) * 32 + (lane >> 1);
            base = plane ? a.Xl : a.Xh;
            row0 = n0;
            rmax = a.N - 1;
            ld = a.ldXs;
        }
        const int c = (lane & 1) ^ ((r >> 3) & 1);
        pb[j] = reinterpret_cast<const char*>(base + row0 * X3K);
        pstep[j] = ld * X3K * S * 2;
        poff[j] = (uint32_t)(((min(row0 + r, rmax) - row0) * X3K + c * 8 + (int64_t)sblk * ld * X3K) * 2);
        lofs[j] = I * 512;
    }
    const int nst = a.pitch / (X3K * S);  // ring stages
    const int li = lane & 31, lh = lane >> 5;
    // issue() is called for stages 0, 1, 2, ... in order: each piece's base
    // advances by one stage per call and stops at the last stage (past the end
    // the DMA re-reads it), a scalar add instead of a 64-bit multiply per piece
    int next_st = 0;
    auto issue = [&](uint16_t* buf, int st) {
        (void)st;
        const bool adv = next_st < nst - 1;
        ++next_st;
#pragma unroll
        for (int j = 0; j < T::PER; ++j) {
            // the stage's base in scalar registers, the lane's offset added last:
            // global_load_lds with an SGPR base and a 32-bit VGPR offset
            const uint64_t ub = reinterpret_cast<uint64_t>(pb[j]);
            if (adv) pb[j] += pstep[j];
            const uint64_t sb = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)ub) |
                                ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(ub >> 32)) << 32);
            x3_dma(reinterpret_cast<const uint16_t*>(reinterpret_cast<const char*>(sb) + poff[j]), buf + lofs[j]);
        }
    };
    auto stage = [&](const uint16_t* buf) { ring_stage<T, MODE, TM, TN, S>(buf, acc, wm, wn, li, lh); };
    // vmcnt(PER * (R - 2)): this wave's pieces of the R-2 newest stages stay in flight
    constexpr int NWT = T::PER * (R - 2);
    constexpr int WAIT = (NWT & 15) | ((NWT >> 4) << 14) | (0x7 << 4) | (0xF << 8);
    uint16_t* const bufs[4] = {B0, B1, B2, B3};
#pragma unroll
    for (int p = 0; p < R - 1; ++p) issue(bufs[p], p);
    for (int kt = 0; kt < nst; kt += R) {
#pragma unroll
        for (int u = 0; u < R; ++u) {
            __builtin_amdgcn_s_waitcnt(WAIT);
            __builtin_amdgcn_s_barrier();
            issue(bufs[(u + R - 1) % R], kt + u + R - 1);
            if (u == 0 || kt + u < nst) stage(bufs[u]);
        }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): no DMA may land after the workgroup ends
    // accumulator layout: D col = lane&31 (base row), row = (r&3) + 8*(r>>2) + 4*(lane>>5) (query)
    if constexpr (EPI == 0) {
        const int64_t col0 = EPI == 0 && a.nsample_tiles > 0 ? nt * T::BN : n0;  // sample: compact columns
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int64_t xr = n0 + wn * TN * 32 + j * 32 + li;
            if (xr >= a.N) continue;
            const bool xok = !(a.dead && a.dead[xr]);
            const float xn = a.xnorm[xr];
            const float xi = MODE != RING_X3 ? a.xinv[xr] : 1.f;
            const int64_t col = col0 + wn * TN * 32 + j * 32 + li;
#pragma unroll
            for (int i = 0; i < TM; ++i) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int64_t qr = q0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                    if (qr >= a.B) continue;
                    const float qi = MODE != RING_X3 ? a.qinv[qr] : 1.f;
                    float sc = split_score(MODE, a.metric, acc[i][j][r], xi, qi, a.qnorm[qr], xn);
                    if (!xok) sc = __int_as_float(0x7f800000);
                    a.scores[(size_t)qr * a.ldS + col] = sc;
                }
            }
        }
    } else {
        // Fused preselection.  A pair can matter only if its score is <= the
        // query's threshold t_q (an upper bound on the query's kk-th best
        // score, from the sample pass).  The test is done on the accumulator:
        //   cosine: score <= t  <=>  acc >= (1 - t) |q| |x| / (xi qi) = c_q w_r
        //   L2:     score <= t  <=>  acc >= a_q / xi + b_r / qi
        // with c_q, a_q lowered and b_r scaled down by 2^-19..2^-20 relative
        // (k_ring_prep), far more than the roundings of either side, so a pair
        // whose exact score is <= t always passes; extra passes are harmless
        // (k_select_bucket recomputes split_score).  Passing pairs go to this
        // wave's slice of the tile's region: {row offset | query offset << 16, acc}.
        bool rok[TN];
        float w0[TN], w1[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int64_t xr = n0 + wn * TN * 32 + j * 32 + li;
            rok[j] = xr < a.N && !(a.dead && a.dead[xr]);
            const int64_t xc = xr < a.N ? xr : a.N - 1;
            const float xi = a.xinv[xc], xn = a.xnorm[xc];
            if (a.metric == COSINE) {
                w0[j] = xn / xi;  // xi is a power of two (or NaN: every query passes the row)
                w1[j] = 0.f;
            } else {
                w0[j] = 1.f / xi;
                w1[j] = xn * xn * 0.5f * (1.0f - 0x1p-20f) / xi;
            }
        }
        // Passing pairs go to the tile's region {row off | query off << 16, score}
        // (split_score, the exact float the sample pass and k_select use).  One
        // pass, per element an fma and a compare (t = acc - bound; !(t < 0) keeps
        // NaN bounds, rows outside the fp16 bound, passing) and a wave-uniform
        // branch on the ballot; only a ballot with passes (a few per wave-tile)
        // takes an LDS add for its slots.
        uint2* reg = a.region + logical * (int64_t)a.rcap;
        unsigned long long rokm[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) rokm[j] = __builtin_amdgcn_ballot_w64(rok[j]);
        auto epi = [&](auto cos_tag) {
            constexpr bool COS = decltype(cos_tag)::value;
#pragma unroll
            for (int i = 0; i < TM; ++i) {
#pragma unroll
                for (int r4 = 0; r4 < 4; ++r4) {
                    const int64_t qb = q0 + wm * TM * 32 + i * 32 + 8 * r4 + 4 * lh;  // 4 consecutive queries
                    const float4 c4 = *reinterpret_cast<const float4*>(a.ring_c + qb);
                    const float cq[4] = {c4.x, c4.y, c4.z, c4.w};
                    float sq[4] = {0.f, 0.f, 0.f, 0.f};
                    if constexpr (!COS) {
                        const float4 s4 = *reinterpret_cast<const float4*>(a.ring_s + qb);
                        sq[0] = s4.x, sq[1] = s4.y, sq[2] = s4.z, sq[3] = s4.w;
                    }
#pragma unroll
                    for (int r1 = 0; r1 < 4; ++r1) {
#pragma unroll
                        for (int j = 0; j < TN; ++j) {
                            const int r = r4 * 4 + r1;
                            const float v = acc[i][j][r];
                            float t;
                            if constexpr (COS)
                                t = fmaf(-cq[r1], w0[j], v);
                            else
                                t = v - fmaf(cq[r1], w0[j], w1[j] * sq[r1]);
                            const unsigned long long m = __builtin_amdgcn_ballot_w64(!(t < 0.f)) & rokm[j];
                            if (m) {
                                const bool pass = (m >> lane) & 1ull;
                                const int first = __ffsll((long long)m) - 1;
                                int base = 0;
                                if (lane == first) base = atomicAdd(tile_ctr, __popcll(m));
                                base = __shfl(base, first, 64);
                                const int qo = wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                                // every counted slot is written (a padded query, q >= B, can pass
                                // on a NaN bound; k_bucket skips it).  The raw accumulator is
                                // stored: k_bucket turns it into split_score's float.
                                if (pass) {
                                    const int e = base + __builtin_amdgcn_mbcnt_hi(
                                                             (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
                                    const int ro = wn * TN * 32 + j * 32 + li;
                                    if (e < a.rcap)
                                        reg[e] = make_uint2((uint32_t)ro | ((uint32_t)qo << 16), __float_as_uint(v));
                                }
                            }
                        }
                    }
                }
            }
        };
        if (a.metric == COSINE)
            epi(std::true_type{});
        else
            epi(std::false_type{});
        __syncthreads();
        if (tid == 0) a.region_cnt[logical] = *tile_ctr;
    }
}

template <int WM_, int WN_, int TM_, int TN_, int MODE, int S, int R, int EPI>
static int launch_ring_t(const ExactArgs& a, hipStream_t s) {
    using T = RingTile<WM_, WN_, TM_, TN_, MODE, S>;
    if (a.pitch % (X3K * S)) return -5;
    const int64_t nqt = (a.B + T::BM - 1) / T::BM;
    const int64_t nnt = EPI == 0 && a.nsample_tiles > 0 ? a.nsample_tiles : (a.N + T::BN - 1) / T::BN;
    hipLaunchKernelGGL((k_scores_ring<WM_, WN_, TM_, TN_, MODE, S, R, EPI>), dim3((unsigned)(nqt * nnt)), dim3(T::NT),
                       0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int MODE>
static int launch_split_scores(const ExactArgs& a, int tile, hipStream_t s) {
    if (a.B <= 0 || a.N <= 0) return 0;
    if (a.pitch % X3K) return -5;
    // tile 0: the measured best per split (config 5: bf16x3 256 x 256, fp16 128 x 256)
    if (tile == 0) tile = MODE == RING_H2 ? 1 : 3;
    switch (tile) {
        case 1: return launch_ring_t<2, 4, 2, 2, MODE, 1, 4, 0>(a, s);  // 128 x 256, 8 waves of 64 x 64
        case 2: return launch_ring_t<2, 2, 2, 2, MODE, 1, 4, 0>(a, s);  // 128 x 128, 4 waves of 64 x 64
        default: return launch_ring_t<2, 4, 4, 2, MODE, 1, 4, 0>(a, s);  // 256 x 256, 8 waves of 128 x 64
    }
}
int launch_exact_scores_x3(const ExactArgs& a, int tile, hipStream_t s) { return launch_split_scores<RING_X3>(a, tile, s); }
int launch_exact_scores_x2h(const ExactArgs& a, int tile, hipStream_t s) { return launch_split_scores<RING_H2>(a, tile, s); }

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
constexpr int G_BM = 256, G_BN = 256;  // k_h1_pp16 tile: queries x rows

static int device_cus() {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
            cus = v;
        else
            cus = 256;
    }
    return cus;
}

// s_waitcnt vmcnt(v) (6-bit count: bits 3:0 and 15:14; lgkm / exp untouched)
constexpr int vmcnt_imm(int v) { return 0x0F70 | (v & 15) | (((v >> 4) & 3) << 14); }
// s_waitcnt vmcnt(BASE + extra) for a wave-uniform extra in [0, sizeof...(I)); a
// larger extra waits vmcnt(BASE) (more than needed, never less)
template <int BASE, int... I>
__device__ __forceinline__ void wait_vm_plus(int extra, std::integer_sequence<int, I...>) {
    const bool done = ((extra == I ? (__builtin_amdgcn_s_waitcnt(vmcnt_imm(BASE + I)), true) : false) || ...);
    if (!done) __builtin_amdgcn_s_waitcnt(vmcnt_imm(BASE));
}

#define MH_DSR(dst, addr, off) asm volatile("ds_read_b128 %0, %1 offset:" #off : "=v"(dst) : "v"(addr))

// ---------------------------------------------------------------------------
// k_h1_pp16: the fp16 1-product scores (exact_precision 3) as a persistent,
// two-group ping-pong stream of 256 x 256 tiles (queries x rows) on
// v_mfma_f32_16x16x32_f16.  Waves 0-3 (group 0, query rows 0-127) and 4-7
// (group 1, rows 128-255) hold one wave on every SIMD; group 1 runs one
// barrier behind group 0, so in every barrier interval one wave of a SIMD
// multiplies (32 MFMAs, s_setprio 1) while the other reads its next fragments
// and issues its share of the LDS-DMA, and the roles swap at the barrier.  Per
// wave (a 128 x 64 tile: 8 x 4 blocks of 16 x 16) and 32-deep K-slice:
//   R: 12 ds_read_b128 (8 A, 4 B fragments) from the slice's ring slot, the
//      wave's 4 DMA pieces of slice x + D (group 0 the A image, group 1 the B
//      image), barrier
//   M: lgkmcnt(0), 32 MFMAs, the tile's epilogue after its last slice, barrier
// The counted vmcnt(4 (D - 1)) before the barrier that precedes group 0's R
// phase (group 0: end of M, group 1: end of R) retires slice x + 1 for every
// wave while D - 1 younger slices stay in flight across the barriers.
//   ring: NS = 4 slots of one K-slice (32 KiB: A 256 rows x 64 B, then B);
//         16-B chunk c of image row r at slot c ^ ((r >> 2) & 3): the four
//         16-lane groups of a fragment read hit 16 distinct 16-B slots.
//   DMA:  a piece = 16 image rows x 64 B = one contiguous 1 KiB run of the
//         16-blocked plane (lane l: row 16 P + l / 4, chunk (l & 3) ^ swizzle).
//   WAR:  slice x + D overwrites the slot of slice x + D - NS, whose last reads
//         (group 1) retired two barrier intervals earlier: NS >= D + 2.
// Tile order: each XCD walks a contiguous run of logical tiles, query tiles
// fastest, so a row tile enters that XCD's L2 once (blockIdx.x % 8 = XCD).
// EPI 0 writes every score of the (sampled) row tiles; EPI 1 is the fused
// filter (records, below): the per-tile filter constants arrive by LDS-DMA at
// the tile's first slice, double-buffered by tile parity.
// DIAG (timing diagnostics, tools build only -- MH_EXACT_DIAG): 1 no epilogue,
// 4 the filter's tests without the record stores (no pair passes: every query
// takes the canonical fallback, results stay exact); without an epilogue and
// without results: 5 no LDS-DMA after the prologue's slices, 6 no fragment
// reads after the first slice's, 7 no barriers in the main loop.
// ---------------------------------------------------------------------------
// STG (round 6, exact_tile 40, tools build): the slices through registers instead of LDS-DMA
// -- each wave loads its pieces of slice x + 2 (global_load_dwordx4, issued in
// R(x)) and writes the previous interval's pieces, slice x + 1, into the ring
// (ds_write_b128, R(x)), so a slice is in LDS one interval before it is read;
// the writes are retired (lgkmcnt) before the barrier that ends the writer's R
// phase.  The same LDS image, so the same scores bit for bit -- but 14 % slower
// than the LDS-DMA ring (the staged loads and writes cost more issue than the
// DMA pieces they replace), so it stays a measurement.
template <int EPI, int DIAG = 0, int NS = 4, int D = 2, int STG = 0>
__global__ __launch_bounds__(512) void k_h1_pp16(ExactArgs a) {
    constexpr int PS = 2;
    // WAR: slice x + D overwrites the slot of slice x + D - NS.  NS >= D + 2: its
    // last reads (group 1) retired two barrier intervals earlier.  NS = D + 1
    // (RSYNC): group 1 retires its fragment reads before the barrier that ends
    // its R phase, so they are done when group 0 issues that DMA one interval on.
    static_assert(NS >= D + 1 && D >= 1, "ring depth");
    constexpr bool RSYNC = NS < D + 2;
    constexpr int RB = 32 * PS;                // image row bytes (16 PS halves of K)
    constexpr int SL = (G_BM + G_BN) * RB;     // one slice: A then B image
    constexpr int CPR = 2 * PS, RPP = 32 / PS;  // 16-B chunks per row, rows per 1-KiB piece
    // EPI 1: per tile (double-buffered by tile parity) the filter constants, by
    // LDS-DMA: 256 rows x {w0, w1, dead, -} (4 KiB), then c and s of 256 queries
    constexpr int CST = 6144, CSTB = NS * SL;
    constexpr bool NOEPI = DIAG == 1 || DIAG >= 5;  // timing diagnostics without an epilogue
    constexpr bool CONSTS = EPI == 1 && !NOEPI;  // the filter constants' LDS copy (not read without an epilogue)
    __shared__ __attribute__((aligned(16))) uint8_t ring[NS * SL + (CONSTS ? 2 * CST : 0)];
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 2, wc = wave & 3;
    const int g = __builtin_amdgcn_readfirstlane(wr);
    const int wcs = __builtin_amdgcn_readfirstlane(wc);
    const int64_t nqt = (a.B + G_BM - 1) / G_BM;
    const int64_t nnt = EPI == 0 && a.nsample_tiles > 0 ? a.nsample_tiles : (a.N + G_BN - 1) / G_BN;
    const int64_t nblk = nqt * nnt;
    const int W = gridDim.x, xcd = blockIdx.x % 8, jx = blockIdx.x / 8;
    const int wx = W / 8 + (xcd < W % 8 ? 1 : 0);
    const int64_t per = nblk / 8, rem = nblk % 8;
    const int64_t lo = xcd < rem ? xcd * (per + 1) : rem * (per + 1) + (xcd - rem) * per;
    const int64_t hi = lo + per + (xcd < rem ? 1 : 0);
    const int64_t first = lo + jx;
    const int64_t ntile = first < hi ? (hi - first + wx - 1) / wx : 0;
    const int nkt = a.pitch / (X3K * PS);  // K-slices per tile
    const int64_t S = ntile * nkt;
    if (S == 0) return;  // uniform over the workgroup

    // DMA: this wave's 2 PS pieces of a slice's A (group 0) or B (group 1) image;
    // lane l: row RPP P + l / CPR, chunk (l % CPR) ^ swizzle(row) = K-block c / 2, half c % 2
    const int rr0 = wcs * 2 * PS * RPP + lane / CPR;  // piece i: + RPP i
    const int64_t ld = g == 0 ? a.ldQs : a.ldXs;
    const int dc = (lane % CPR) ^ (PS == 1 ? (lane >> 4) & 1 : (lane >> 4) & 3);
    const uint32_t pk = (uint32_t)((dc >> 1) * ld * 32 + (dc & 1) * 16);
    const char* const plane = reinterpret_cast<const char*>(g == 0 ? a.Qh : a.Xh);
    auto sbase = [](const char* p) {
        const uint64_t u = reinterpret_cast<uint64_t>(p);
        return reinterpret_cast<const char*>((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u) |
                                             ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(u >> 32))
                                              << 32));
    };
    int64_t p_tile = 0;
    int p_kt = 0, p_slot = 0;
    const char* p_base = nullptr;  // the producer tile's first row in K-block 0
    int p_lim = 0;                 // its last valid image row (rows past B / N clamp to it)
    auto p_set = [&]() {
        const int64_t L = first + p_tile * wx;
        const int64_t qt = L % nqt, nt = L / nqt;
        const int64_t r0 = g == 0 ? qt * G_BM : (EPI == 0 && a.nsample_tiles > 0 ? nt * a.tile_stride : nt) * G_BN;
        p_base = plane + r0 * 32;
        p_lim = (int)min<int64_t>(255, (g == 0 ? a.B : a.N) - 1 - r0);
    };
    auto produce = [&]() {  // this wave's pieces of the producer slice, then advance it
        const char* base = sbase(p_base + (int64_t)p_kt * PS * ld * 32);
#pragma unroll
        for (int i = 0; i < 2 * PS; ++i) {
            const uint32_t off = (uint32_t)min(rr0 + RPP * i, p_lim) * 32 + pk;
            uint8_t* dst = ring + p_slot * SL + g * (G_BM * RB) + (wcs * 2 * PS + i) * 1024;
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(base + off),
                                             (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
        }
        if (++p_slot == NS) p_slot = 0;
        if (++p_kt == nkt) {
            p_kt = 0;
            if (++p_tile < ntile) p_set();
        }
    };
    // STG: this wave's pieces of the producer slice into registers, then advance
    // it; stage_write puts the held pieces into their ring slot
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) const u32x4 gu32x4;
    u32x4 stv[2 * PS];
    int st_slot = -1;  // ring slot of the held pieces (-1: none)
    auto stage_load = [&]() {
        const char* base = sbase(p_base + (int64_t)p_kt * PS * ld * 32);
#pragma unroll
        for (int i = 0; i < 2 * PS; ++i) {
            const uint32_t off = (uint32_t)min(rr0 + RPP * i, p_lim) * 32 + pk;
            stv[i] = *(gu32x4*)(base + off);
        }
        st_slot = p_slot;
        if (++p_slot == NS) p_slot = 0;
        if (++p_kt == nkt) {
            p_kt = 0;
            if (++p_tile < ntile) p_set();
        }
    };
    auto stage_write = [&]() {
        if (st_slot < 0) return;
#pragma unroll
        for (int i = 0; i < 2 * PS; ++i)
            *reinterpret_cast<u32x4*>(ring + st_slot * SL + g * (G_BM * RB) + (wcs * 2 * PS + i) * 1024 + lane * 16) =
                stv[i];
        st_slot = -1;
    };

    f32x4 acc[8][4];  // 16 x 16 blocks: queries wr 128 + 16 mb .., rows wc 64 + 16 nb ..
    const f32x4 zacc = {};  // a tile's first MFMAs accumulate onto zero (no clearing pass)
    const uint32_t ring_lds = (uint32_t)reinterpret_cast<uintptr_t>(ring);
    // fragment of a 16-row block (v_mfma_f32_16x16x32_f16): row lane & 15, logical
    // chunk lane / 16 (halves 8 (lane / 16) .. of the 32-deep slice), swizzled like
    // the DMA image: slot = chunk ^ ((row >> 2) & 3)
    const uint32_t lfix = (lane & 15) * RB + ((((lane >> 4) ^ ((lane >> 2) & 3)) & 3) << 4);
    const uint32_t offA = wr * 128 * RB, offB = G_BM * RB + wc * 64 * RB;
    const int fr = lane & 15, fq = lane >> 4;  // accumulator: column (row) fr, queries 4 fq + j
    float keep = 0.f;  // DIAG: keeps the MFMAs / tests live
    int nst = 0;  // vector-memory ops besides the slice pieces since the last counted wait

    // The fused filter, in records: per lane four rows (nb) and, per 16-query
    // block row mb, four queries; a pair passes unless acc - c_q w_x < 0 (cosine;
    // L2 acc - (c_q w0_x + w1_x s_q) < 0), every constant from the tile's LDS copy.
    // A lane with a passing pair in block row mb stores that row's 16 accumulators
    // as one record ({mb | lane << 8, 0}, pad, 4 x float4 = H1_REC uint2) in its
    // wave's eighth of the tile's region; k_bucket_rec re-applies the identical
    // test to each.  A block's largest value is tested first (one ballot per 16
    // queries).
    auto epilogue = [&](int64_t L, int64_t ctile) {
        const int64_t qt = L % nqt, nt = L / nqt;
        const int64_t q0 = qt * G_BM;
        const int64_t n0 = (EPI == 0 && a.nsample_tiles > 0 ? nt * a.tile_stride : nt) * G_BN;
        if constexpr (NOEPI) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) keep += acc[i][j][r];
        } else if constexpr (EPI == 0) {
            const int64_t col0 = a.nsample_tiles > 0 ? nt * G_BN : n0;  // sample: compact columns
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) {
                const int ro = wc * 64 + nb * 16 + fr;
                const int64_t xr = n0 + ro;
                if (xr >= a.N) continue;
                const bool xok = !(a.dead && a.dead[xr]);
                const float xn = a.xnorm[xr], xi = a.xinv[xr];
#pragma unroll
                for (int mb = 0; mb < 8; ++mb)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int64_t qr = q0 + wr * 128 + mb * 16 + 4 * fq + r;
                        if (qr >= a.B) continue;
                        float sc = split_score(RING_H1, a.metric, acc[mb][nb][r], xi, a.qinv[qr], a.qnorm[qr], xn);
                        if (!xok) sc = __int_as_float(0x7f800000);
                        a.scores[(size_t)qr * a.ldS + col0 + ro] = sc;
                    }
            }
        } else {
            const uint32_t cb = ring_lds + CSTB + (uint32_t)(ctile & 1) * CST;
            f32x4 xw[4];
#pragma unroll
            for (int nb = 0; nb < 4; ++nb)
                asm volatile("ds_read_b128 %0, %1" : "=v"(xw[nb]) : "v"(cb + (uint32_t)(wc * 64 + nb * 16 + fr) * 16));
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(xw[0]), "+v"(xw[1]), "+v"(xw[2]), "+v"(xw[3]));
            __builtin_amdgcn_sched_barrier(0);
            bool rok[4], rsp[4];
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) {
                rok[nb] = n0 + wc * 64 + nb * 16 + fr < a.N && xw[nb][2] == 0.f;
                // a row whose w0 is not finite (or 0) always takes the exact per-pair tests
                rsp[nb] = rok[nb] && (!(fabsf(xw[nb][0]) < __builtin_inff()) || xw[nb][0] == 0.f);
            }
            int cnt = 0;  // wave-uniform
            const int rcw = a.rcap / (8 * H1_REC);  // records per wave region
            uint2* regr = a.region + (L * 8 + wave) * (int64_t)(rcw * H1_REC);
            int lid = lane;
            asm volatile("" : "+v"(lid));
            auto filt = [&](auto cos_tag) {
                constexpr bool COS = decltype(cos_tag)::value;
                auto tval = [&](int mb, int nb, int r, const f32x4& c4, const f32x4& s4) {
                    const float v = acc[mb][nb][r];
                    if constexpr (COS)
                        return fmaf(-c4[r], xw[nb][0], v);
                    else
                        return v - fmaf(c4[r], xw[nb][0], xw[nb][1] * s4[r]);
                };
#pragma unroll
                for (int mb = 0; mb < 8; ++mb) {
                    __builtin_amdgcn_sched_barrier(0);
                    // queries wr 128 + 16 mb + 4 fq + 0..3
                    f32x4 c4, s4 = {};
                    const uint32_t qa = cb + 4096 + (uint32_t)(wr * 128 + mb * 16 + 4 * fq) * 4;
                    asm volatile("ds_read_b128 %0, %1" : "=v"(c4) : "v"(qa));
                    if constexpr (!COS) {
                        asm volatile("ds_read_b128 %0, %1 offset:1024" : "=v"(s4) : "v"(qa));
                        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(c4), "+v"(s4));
                    } else {
                        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(c4));
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    bool hit = false;
#pragma unroll
                    for (int nb = 0; nb < 4; ++nb) {
                        float mx = -__builtin_inff();
#pragma unroll
                        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, tval(mb, nb, r, c4, s4));
                        hit |= (rok[nb] && !(mx < 0.f)) || rsp[nb];
                    }
                    if constexpr (DIAG == 4) {
                        keep += (float)__builtin_amdgcn_ballot_w64(hit);
                    } else {
                        const unsigned long long m = __builtin_amdgcn_ballot_w64(hit);
                        if (m) {
                            const int rk = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
                            if (hit) {
                                const int slot = min(cnt + rk, rcw - 1);  // past the capacity: the last record (flagged)
                                uint2* rec = regr + (int64_t)slot * H1_REC;
                                rec[0] = make_uint2((uint32_t)mb | ((uint32_t)lid << 8), 0u);
                                float4* ra = reinterpret_cast<float4*>(rec + 2);
#pragma unroll
                                for (int nb = 0; nb < 4; ++nb)
                                    ra[nb] = make_float4(acc[mb][nb][0], acc[mb][nb][1], acc[mb][nb][2], acc[mb][nb][3]);
                            }
                            nst += 5;  // (at least 5 store instructions: never an over-count)
                            cnt += __popcll(m);
                        }
                    }
                }
            };
            if (a.metric == COSINE)
                filt(std::true_type{});
            else
                filt(std::false_type{});
            if (lane == 0) a.region_cnt[L * 8 + wave] = cnt;  // (DIAG 4: 0)
            ++nst;
        }
    };

    constexpr int VMC = vmcnt_imm(2 * PS * (D - 1));
    constexpr int VMCNT0 = 0x0F70;
    auto wait_vmc = [&]() {
        if (nst > 0) {
            wait_vm_plus<2 * PS * (D - 1)>(nst, std::make_integer_sequence<int, 59>{});  // (vmcnt <= 63)
        } else {
            __builtin_amdgcn_s_waitcnt(VMC);
        }
    };
    p_set();
    int64_t ps = 0;
    if constexpr (STG) {
        stage_load();  // slice 0 into the ring now, slice 1 held
        stage_write();
        ++ps;
        if (ps < S) {
            stage_load();
            ++ps;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
        for (; ps < D && ps < S; ++ps) produce();
        if (D <= S)
            __builtin_amdgcn_s_waitcnt(VMC);
        else
            __builtin_amdgcn_s_waitcnt(VMCNT0);
    }
    __builtin_amdgcn_s_barrier();
    if (g == 1 && DIAG != 7) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind

    int64_t c_tile = 0;
    int c_kt = 0, c_slot = 0;
    f16x8 fa[8], fb[4];
    for (int64_t x = 0; x < S; ++x) {
        // R: fragments of slice x, DMA of slice x + D
        const uint32_t sb = ring_lds + (uint32_t)c_slot * SL;
        if (++c_slot == NS) c_slot = 0;
        if (DIAG != 6 || x == 0) {
            const uint32_t va = sb + offA + lfix, vb = sb + offB + lfix;
            MH_DSR(fa[0], va, 0);
            MH_DSR(fa[1], va, 1024);
            MH_DSR(fa[2], va, 2048);
            MH_DSR(fa[3], va, 3072);
            MH_DSR(fa[4], va, 4096);
            MH_DSR(fa[5], va, 5120);
            MH_DSR(fa[6], va, 6144);
            MH_DSR(fa[7], va, 7168);
            MH_DSR(fb[0], vb, 0);
            MH_DSR(fb[1], vb, 1024);
            MH_DSR(fb[2], vb, 2048);
            MH_DSR(fb[3], vb, 3072);
        }
        if (CONSTS && c_kt == 0) {
            // the filter constants of this tile (read by its epilogue, nkt - 1 >= D
            // slices later: retired by the counted waits in between)
            const int64_t L = first + c_tile * wx;
            const int64_t q0 = (L % nqt) * G_BM, n0 = (L / nqt) * G_BN;
            uint8_t* cd = ring + CSTB + (int)(c_tile & 1) * CST;
            const float* src;
            uint8_t* dst;
            if (g == 0) {
                src = (wcs & 1 ? a.ring_s : a.ring_c) + q0 + lane * 4;
                dst = cd + 4096 + (wcs & 1) * 1024;
            } else {
                src = reinterpret_cast<const float*>(a.xw + min<int64_t>(n0 + wcs * 64 + lane, a.N - 1));
                dst = cd + wcs * 1024;
            }
            if (g == 1 || wcs < 2) {
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                                 (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
                ++nst;
            }
        }
        if constexpr (STG) {
            stage_write();  // slice x + 1
            if (ps < S) {
                stage_load();  // slice x + 2
                ++ps;
            }
        } else if (ps < S) {
            if constexpr (DIAG != 5) produce();
            ++ps;
        }
        const bool tail = x + 1 + D > S;  // fewer than D slices left in flight: retire them all
        if (STG && g == 1) {
            // this wave's slice writes land before the barrier after which group 0 reads them
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        } else if (g == 1) {
            if (tail)
                __builtin_amdgcn_s_waitcnt(VMCNT0);
            else
                wait_vmc();
            nst = 0;
            if constexpr (RSYNC)
                asm volatile("s_waitcnt lgkmcnt(0)"
                             : "+v"(fa[0]), "+v"(fa[1]), "+v"(fa[2]), "+v"(fa[3]), "+v"(fa[4]), "+v"(fa[5]),
                               "+v"(fa[6]), "+v"(fa[7]), "+v"(fb[0]), "+v"(fb[1]), "+v"(fb[2]), "+v"(fb[3]));
        }
        if constexpr (DIAG != 7) __builtin_amdgcn_s_barrier();
        // M: 32 MFMAs (+ the epilogue after a tile's last slice)
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(fa[0]), "+v"(fa[1]), "+v"(fa[2]), "+v"(fa[3]), "+v"(fa[4]), "+v"(fa[5]), "+v"(fa[6]),
                       "+v"(fa[7]), "+v"(fb[0]), "+v"(fb[1]), "+v"(fb[2]), "+v"(fb[3]));
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        if (c_kt == 0) {
#pragma unroll
            for (int m = 0; m < 8; ++m)
#pragma unroll
                for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[m], fb[n], zacc, 0, 0, 0);
        } else {
#pragma unroll
            for (int m = 0; m < 8; ++m)
#pragma unroll
                for (int n = 0; n < 4; ++n)
                    acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[m], fb[n], acc[m][n], 0, 0, 0);
        }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if (++c_kt == nkt) {
            if constexpr (STG && CONSTS) __builtin_amdgcn_s_waitcnt(VMCNT0);  // the tile's filter constants (LDS-DMA)
            epilogue(first + c_tile * wx, c_tile);
            c_kt = 0;
            ++c_tile;
        }
        if (g == 0 && !STG) {
            if (tail)
                __builtin_amdgcn_s_waitcnt(VMCNT0);
            else
                wait_vmc();
            nst = 0;
        }
        if constexpr (DIAG != 7) __builtin_amdgcn_s_barrier();
    }
    if (g == 0 && DIAG != 7) __builtin_amdgcn_s_barrier();  // evens the barrier count
    __builtin_amdgcn_s_waitcnt(VMCNT0);
    if constexpr (DIAG > 0) {
        if (lane == 0 && keep == -1.0e38f) a.region_cnt[0] = 1;
    }
}

template <int EPI, int DIAG = 0, int NS = 4, int D = 2, int STG = 0>
static int launch_h1_pp16_t(const ExactArgs& a, hipStream_t s) {
    if (a.pitch % (X3K * 2)) return -5;
    if (std::max(a.ldQs, a.ldXs) * 32 + G_BM * 32 >= ((int64_t)1 << 32)) return -5;  // 32-bit DMA offsets
    const int64_t nqt = (a.B + G_BM - 1) / G_BM;
    const int64_t nnt = EPI == 0 && a.nsample_tiles > 0 ? a.nsample_tiles : (a.N + G_BN - 1) / G_BN;
    const int64_t nblk = nqt * nnt;
    const int64_t W = std::min<int64_t>(nblk, std::max(8, device_cus() / 8 * 8));
    hipLaunchKernelGGL((k_h1_pp16<EPI, DIAG, NS, D, STG>), dim3((unsigned)W), dim3(512), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

#undef MH_DSR

// ---------------------------------------------------------------------------
// fp16 1-product path with the fused preselection (exact_precision 3)
// ---------------------------------------------------------------------------
// exact_tile for precision 3: 0 / 34 = k_h1_pp16 (the default); 5 = the ring
// kernel's fused filter (k_scores_ring, 128 x 256 tiles, 32-deep stages, 3
// buffers, two workgroups per CU), which also runs every shape k_h1_pp16 does
// not admit (fewer than 3 K-slices per tile, DMA offsets past 32 bits).  The
// tools build (MH_EXACT_DIAG) adds 30 / 31: k_h1_pp16 with no epilogue / the
// filter's tests without the record stores.
template <int EPI>
static int launch_h1(const ExactArgs& a, int variant, hipStream_t s) {
    if (a.B <= 0 || a.N <= 0) return 0;
    switch (variant) {
        case 5: return launch_ring_t<2, 4, 2, 2, RING_H1, 2, 3, EPI>(a, s);
#ifdef MH_EXACT_DIAG
        case 30: return launch_h1_pp16_t<EPI, EPI ? 1 : 0>(a, s);
        case 31: return launch_h1_pp16_t<EPI, EPI ? 4 : 0>(a, s);
        case 32: return launch_h1_pp16_t<EPI, EPI ? 1 : 0, 5, 3>(a, s);  // no epilogue, 3 slices in flight (160 KiB ring)
        case 36: return launch_h1_pp16_t<EPI, EPI ? 1 : 0, 4, 3>(a, s);  // no epilogue, 3 in flight, 4-slot ring (RSYNC)
        case 33: return launch_h1_pp16_t<EPI, 0, 4, 3>(a, s);  // with the epilogue, 3 in flight (RSYNC)
        case 37: return launch_h1_pp16_t<EPI, EPI ? 5 : 0>(a, s);  // no epilogue, no DMA after the prologue
        case 38: return launch_h1_pp16_t<EPI, EPI ? 6 : 0>(a, s);  // no epilogue, no fragment reads after slice 0
        case 39: return launch_h1_pp16_t<EPI, EPI ? 7 : 0>(a, s);  // no epilogue, no main-loop barriers
#endif
#ifdef MH_EXACT_DIAG
        // slices staged through registers (STG): the same results, measured slower
        // (3.35 vs 2.94 ms on configs[4], profiles/r06_gemm_diag.txt)
        case 40: return launch_h1_pp16_t<EPI, 0, 4, 2, 1>(a, s);
        case 41: return launch_h1_pp16_t<EPI, EPI ? 1 : 0, 4, 2, 1>(a, s);  // STG, no epilogue
#endif
        default: return launch_h1_pp16_t<EPI>(a, s);
    }
}
int h1_tile_bm(int variant) { return variant == 5 ? 128 : 256; }
// The variant a search runs: k_h1_pp16 (34) needs at least D + 1 = 3 K-slices per
// tile (the filter constants staged at a tile's first slice must have landed by
// its epilogue) and 32-bit DMA offsets -- otherwise the ring (5).
int h1_effective_variant(int variant, int pitch, int64_t ld) {
    const int v = variant == 0 ? 34 : variant;
    if (v == 5) return 5;
    const int dslices = v == 33 || v == 32 || v == 36 ? 3 : 2;  // slices in flight (33, 32, 36: tools build)
    if (pitch % (X3K * 2) || pitch / (X3K * 2) < dslices + 1 || ld * 32 + G_BM * 32 >= ((int64_t)1 << 32)) return 5;
    return v;
}

// Per row the fused filter's constants {w0, w1, dead, 0} (k_h1_pp16 stages them per
// tile by DMA): cosine w0 = |x| / xi; L2 w0 = 1 / xi, w1 = |x|^2 (1 - 2^-20) / (2 xi)
__global__ void k_h1_rowconst(const float* xinv, const float* xnorm, const uint8_t* dead, int64_t n, int metric,
                              float4* xw) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float xi = xinv[i], xn = xnorm[i];
    float w0, w1;
    if (metric == COSINE) {
        w0 = xn / xi;
        w1 = 0.f;
    } else {
        w0 = 1.f / xi;
        w1 = xn * xn * 0.5f * (1.0f - 0x1p-20f) / xi;
    }
    xw[i] = make_float4(w0, w1, dead && dead[i] ? 1.f : 0.f, 0.f);
}
int launch_h1_rowconst(const float* xinv, const float* xnorm, const uint8_t* dead, int64_t n, int metric, float4* xw,
                       hipStream_t s) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_h1_rowconst, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, xinv, xnorm, dead, n, metric,
                       xw);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
// tools build (MH_EXACT_DIAG): the timing diagnostics, which let no pair pass
bool h1_timing_diag(int variant) {
    return variant == 30 || variant == 31 || variant == 32 || variant == 36 || (variant >= 37 && variant <= 39) ||
           variant == 41;
}
// regions per tile of a variant's fused filter (k_h1_pp16: one per wave)
int h1_region_split(int variant) { return variant == 5 ? 1 : 8; }  // (an effective variant)
// the variant's regions hold records (H1_REC uint2 each: a lane's 16 accumulators of one
// block row, tested by k_bucket_rec) instead of passing pairs
bool h1_records(int variant) { return variant != 5; }
int launch_h1_sample(const ExactArgs& a, int variant, hipStream_t s) { return launch_h1<0>(a, variant, s); }
int launch_h1_filter(const ExactArgs& a, int variant, hipStream_t s) { return launch_h1<1>(a, variant, s); }

// Per query: the epilogue filter's constants from the sample threshold t_q (the
// kk-th best sample score; the sample is a subset of the rows scored with the
// same arithmetic, so t_q bounds the query's kk-th best score from above).
//   cosine: c = ((1 - t) - 2^-19) |q| / qi, then scaled by (1 -+ 2^-20) toward -inf
//   L2:     c = a = (|q|^2 - t - 2^-20 (|q|^2 + |t|)) / (2 qi), s = 1 / qi
// A query the bound does not cover (NaN qi, t not finite) gets c = +inf: no row
// passes for it except rows outside the bound; k_select_bucket sends it to the
// canonical fallback.
__global__ void k_ring_prep(const float* thr, const float* qnorm, const float* qinv, int64_t B, int64_t Bpad,
                            int metric, float* c, float* sq) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= Bpad) return;
    if (b >= B) {  // pads of the last query tile: nothing passes
        c[b] = __int_as_float(0x7f800000);
        sq[b] = 0.f;
        return;
    }
    const float t = thr[b], qn = qnorm[b], qi = qinv[b];
    const bool ok = isfinite(t) && qi == qi;
    float cv, sv = 0.f;
    if (metric == COSINE) {
        const double v = ((1.0 - (double)t) - 0x1p-19) * (double)qn / (double)qi;
        cv = (float)(v >= 0 ? v * (1.0 - 0x1p-20) : v * (1.0 + 0x1p-20));
    } else {
        const double q2 = (double)qn * (double)qn;
        cv = (float)((q2 - (double)t - 0x1p-20 * (q2 + fabs((double)t))) * 0.5 / (double)qi);
        sv = 1.f / qi;
    }
    c[b] = ok ? cv : __int_as_float(0x7f800000);
    sq[b] = ok ? sv : 0.f;
}

int launch_ring_prep(const float* thr, const float* qnorm, const float* qinv, int64_t B, int metric, float* c,
                     float* sq, hipStream_t s) {
    if (B <= 0) return 0;
    const int64_t Bpad = (B + 255) / 256 * 256;  // covers every variant's query tile
    hipLaunchKernelGGL(k_ring_prep, dim3((unsigned)((Bpad + 255) / 256)), dim3(256), 0, s, thr, qnorm, qinv, B, Bpad,
                       metric, c, sq);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Regions -> per-query buckets: one wave per row/query tile.  A query's
// bucket is split in H1_BSUB sub-buckets (row tile nt goes to nt % H1_BSUB), each with
// its own counter, so the appends of the ~N/256 tiles that feed one query do
// not all serialise on one address.  A region (or sub-bucket) whose count
// exceeds its capacity lost pairs: every query of the tile (or that query) is
// marked, and k_select_bucket sends it to the canonical fallback.
__global__ __launch_bounds__(64) void k_bucket(const uint2* region, const int32_t* region_cnt, int rcap, int64_t ntiles,
                                               int64_t nqt, int BM, int BN, int64_t B, int32_t* qcnt, uint2* bucket,
                                               int scap, uint8_t* qovf, int rsub, int rec, ExactArgs a) {
    // one wave per region: rsub regions of rcap / rsub entries per tile
    const int64_t ri = blockIdx.x;
    if (ri >= ntiles * rsub) return;
    const int64_t t = ri / rsub;
    rcap /= rsub;
    const int cap = rsub > 1 ? rcap - 1 : rcap;  // k_h1_pp: the last slot of a wave's region is its trash slot
    const int lane = lane_id();
    const int64_t nt = t / nqt;
    const int64_t q0 = (t % nqt) * BM, n0 = nt * BN;
    const int sub = (int)(nt % H1_BSUB);
    const int n = region_cnt[ri];
    if (n > cap) {
        for (int64_t q = q0 + lane; q < q0 + BM && q < B; q += 64) qovf[q] = 1;
    }
    const int m = min(n, cap);
    const uint2* reg = region + ri * (int64_t)rcap;
    for (int e = lane; e < m; e += 64) {
        const uint2 v = reg[e];
        const int64_t q = q0 + (v.x >> 16);
        if (q >= B) continue;
        const uint32_t row = (uint32_t)(n0 + (v.x & 0xFFFFu));
        // the epilogue stored the raw accumulator: its score, split_score's float
        const float sc = split_score(RING_H1, a.metric, __uint_as_float(v.y), a.xinv[row], a.qinv[q], a.qnorm[q],
                                     a.xnorm[row]);
        const int pos = atomicAdd(&qcnt[(q * H1_BSUB + sub) * H1_CSTRIDE], 1);
        if (pos < scap) bucket[(q * H1_BSUB + sub) * scap + pos] = make_uint2(row, __float_as_uint(sc));
    }
}

// Record mode (k_h1_pp16<1, 0, 1>): one workgroup per tile, wave w takes region w
// (the tile's wave w: queries 128 (w / 4) .., rows 64 (w % 4) ..).  The tile's
// filter constants are staged in LDS once; 16 lanes take one record (lane
// 4 nb + r: accumulator r of row block nb), apply the GEMM's test to it and
// append the passing pairs as k_bucket does.
__global__ __launch_bounds__(512) void k_bucket_rec(const uint2* region, const int32_t* region_cnt, int rcap,
                                                    int64_t nqt, int64_t B, int32_t* qcnt, uint2* bucket, int scap,
                                                    uint8_t* qovf, ExactArgs a) {
    // the tile's constants, row and query norms in LDS; the wave's count and its
    // first 16 records are loaded beside them (a region holds >= 64 records, so
    // the loads past the count stay inside it and are discarded): one round trip
    // before the tests instead of a chain of dependent loads per record
    constexpr int U = 4;  // records per lane group in flight (16 per wave)
    __shared__ float sc_c[256], sc_s[256], sx_i[256], sx_n[256], sq_i[256], sq_n[256];
    __shared__ float4 sc_w[256];
    const int64_t t = blockIdx.x;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int64_t nt = t / nqt;
    const int64_t q0 = (t % nqt) * 256, n0 = nt * 256;
    const int sub = (int)(nt % H1_BSUB);
    const int rpw = rcap / 8, rcw = rpw / H1_REC;  // uint2 / records per wave region
    const int64_t ri = t * 8 + w;
    const int n = region_cnt[ri];
    const uint2* reg = region + ri * (int64_t)rpw;
    const int pr = lane & 15;
    uint32_t hd[U];
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint2* rec = reg + (int64_t)((lane >> 4) + 4 * u) * H1_REC;
        hd[u] = rec[0].x;
        v[u] = reinterpret_cast<const float*>(rec + 2)[pr];
    }
    if (tid < 256) {
        sc_c[tid] = a.ring_c[q0 + tid];  // (ring_c / ring_s are padded to the 256-query tile)
        sc_s[tid] = a.metric == COSINE ? 0.f : a.ring_s[q0 + tid];
        const int64_t row = min<int64_t>(n0 + tid, a.N - 1), q = min<int64_t>(q0 + tid, B - 1);
        sc_w[tid] = a.xw[row];
        sx_i[tid] = a.xinv[row];
        sx_n[tid] = a.xnorm[row];
        sq_i[tid] = a.qinv[q];
        sq_n[tid] = a.qnorm[q];
    }
    __syncthreads();
    if (n > rcw) {
        for (int64_t q = q0 + (w >> 2) * 128 + lane; q < q0 + (w >> 2) * 128 + 128 && q < B; q += 64) qovf[q] = 1;
    }
    const int m = min(n, rcw);
    const int wr = w >> 2, wc = w & 3, nb = pr >> 2, r = pr & 3;
    for (int e0 = 0; e0 < m; e0 += 4 * U) {
        if (e0 > 0) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = min(e0 + (lane >> 4) + 4 * u, rcw - 1);
                const uint2* rec = reg + (int64_t)e * H1_REC;
                hd[u] = rec[0].x;
                v[u] = reinterpret_cast<const float*>(rec + 2)[pr];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = e0 + (lane >> 4) + 4 * u;
            if (e >= m) break;
            const int mb = (int)(hd[u] & 0xFFu), sl = (int)(hd[u] >> 8);
            const int ro = wc * 64 + nb * 16 + (sl & 15), qo = wr * 128 + mb * 16 + 4 * (sl >> 4) + r;
            const int64_t row = n0 + ro, q = q0 + qo;
            const float4 xw = sc_w[ro];
            // the fused filter's test (k_h1_pp16), on the same accumulator and constants
            float tv;
            if (a.metric == COSINE)
                tv = fmaf(-sc_c[qo], xw.x, v[u]);
            else
                tv = v[u] - fmaf(sc_c[qo], xw.x, xw.y * sc_s[qo]);
            if (!(tv < 0.f) && row < a.N && xw.z == 0.f && q < B) {
                const float sc = split_score(RING_H1, a.metric, v[u], sx_i[ro], sq_i[qo], sq_n[qo], sx_n[ro]);
                const int pos = atomicAdd(&qcnt[(q * H1_BSUB + sub) * H1_CSTRIDE], 1);
                if (pos < scap) bucket[(q * H1_BSUB + sub) * scap + pos] = make_uint2((uint32_t)row, __float_as_uint(sc));
            }
        }
    }
}

int launch_bucket(const uint2* region, const int32_t* region_cnt, int rcap, int64_t ntiles, int64_t nqt, int BM,
                  int BN, int64_t B, int32_t* qcnt, uint2* bucket, int scap, uint8_t* qovf, int rsub, int rec,
                  const ExactArgs& a, hipStream_t s) {
    if (ntiles <= 0) return 0;
    if (rsub < 1 || rcap % rsub || (rec && (rsub != 8 || BM != 256 || BN != 256 || (rcap / rsub) % H1_REC))) return -5;
    if (rec) {
        hipLaunchKernelGGL(k_bucket_rec, dim3((unsigned)ntiles), dim3(512), 0, s, region, region_cnt, rcap, nqt, B, qcnt,
                           bucket, scap, qovf, a);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    hipLaunchKernelGGL(k_bucket, dim3((unsigned)(ntiles * rsub)), dim3(64), 0, s, region, region_cnt, rcap, ntiles, nqt,
                       BM, BN, B, qcnt, bucket, scap, qovf, rsub, rec, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// One wave per query: the best kk (score, row) of its sub-buckets (scores as
// the epilogue computed them with split_score).  Bound t: every row outside
// the bucket scored above t_q (the filter passes every score <= t_q), every
// bucket row past the best kk scored >= the kk-th, so t = min(t_q, kk-th best)
// (t_q alone when the bucket holds fewer than kk).  A query with an overflowed
// region or sub-bucket, or an unusable threshold, gets t = -inf: its
// certificate fails and the canonical fallback recomputes it.
template <int R>
__global__ __launch_bounds__(256) void k_select_bucket(ExactArgs a, const int32_t* qcnt, const uint2* bucket, int scap,
                                                       const uint8_t* qovf, const float* thr) {
    // four waves per query, wave w takes sub-buckets w, w+4, ...; wave 0 merges
    __shared__ float md[4 * 64 * R];
    __shared__ uint32_t mi[4 * 64 * R];
    __shared__ int mbad;
    const int64_t b = blockIdx.x;
    if (b >= a.B) return;
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    const float inf = __int_as_float(0x7f800000);
    const float tq = thr[b], qi = a.qinv[b];
    const bool usable0 = !qovf[b] && isfinite(tq) && qi == qi;
    if (threadIdx.x == 0) mbad = 0;
    __syncthreads();
    const int kk = a.kk;
    auto scan = [&](BList<R>& L, const uint2* bk, int m) {
        float worst;
        {
            float wd;
            uint32_t wi;
            bl_at(L, kk - 1, wd, wi);
            worst = wi == EMPTY_ID ? inf : wd;
        }
        for (int base = 0; base < m; base += 64) {
            const int e = base + lane;
            float x = inf;
            uint32_t row = 0;
            if (e < m) {
                const uint2 v = bk[e];
                row = v.x;
                x = __uint_as_float(v.y);
            }
            unsigned long long msk = __ballot(x <= worst && x < inf);
            while (msk) {
                const int src = __ffsll((long long)msk) - 1;
                msk &= msk - 1;
                const float d = rl_f(x, src);
                const uint32_t id = (uint32_t)__shfl((int)row, src, 64);
                if (bl_insert(L, kk, d, id)) {
                    float wd;
                    uint32_t wi;
                    bl_at(L, kk - 1, wd, wi);
                    worst = wi == EMPTY_ID ? inf : wd;
                }
            }
        }
    };
    BList<R> L;
    bl_init(L);
    if (usable0) {
        for (int sb = wave; sb < H1_BSUB; sb += 4) {
            const int n = qcnt[(b * H1_BSUB + sb) * H1_CSTRIDE];
            if (n > scap) {
                if (lane == 0) mbad = 1;
                break;
            }
            scan(L, bucket + (b * H1_BSUB + sb) * (int64_t)scap, n);
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        md[(wave * R + r) * 64 + lane] = L.d[r];
        mi[(wave * R + r) * 64 + lane] = L.i[r] == EMPTY_ID ? EMPTY_ID : (L.i[r] & ID_MASK);
    }
    __syncthreads();
    if (wave != 0) return;
    const bool usable = usable0 && !mbad;
    // merge the other three lists into wave 0's
    for (int w = 1; w < 4 && usable; ++w) {
        float worst;
        {
            float wd;
            uint32_t wi;
            bl_at(L, kk - 1, wd, wi);
            worst = wi == EMPTY_ID ? inf : wd;
        }
        for (int r = 0; r < R; ++r) {
            const float x = md[(w * R + r) * 64 + lane];
            const uint32_t row = mi[(w * R + r) * 64 + lane];
            unsigned long long msk = __ballot(row != EMPTY_ID && x <= worst);
            while (msk) {
                const int src = __ffsll((long long)msk) - 1;
                msk &= msk - 1;
                const float d = rl_f(x, src);
                const uint32_t id = (uint32_t)__shfl((int)row, src, 64);
                if (bl_insert(L, kk, d, id)) {
                    float wd;
                    uint32_t wi;
                    bl_at(L, kk - 1, wd, wi);
                    worst = wi == EMPTY_ID ? inf : wd;
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int idx = r * 64 + lane;
        if (idx < kk) a.cand[b * kk + idx] = (!usable || L.i[r] == EMPTY_ID) ? EMPTY_ID : (L.i[r] & ID_MASK);
    }
    float kd;
    uint32_t ki;
    bl_at(L, kk - 1, kd, ki);
    if (lane == 0) a.bound[b] = !usable ? -inf : (ki != EMPTY_ID ? fminf(kd, tq) : tq);
}

int launch_select_bucket(const ExactArgs& a, const int32_t* qcnt, const uint2* bucket, int scap, const uint8_t* qovf,
                         const float* thr, hipStream_t s) {
    if (a.B <= 0) return 0;
    if (a.kk < 1 || a.kk > 256) return -4;
    if (a.kk <= 64)
        hipLaunchKernelGGL(k_select_bucket<1>, dim3((unsigned)a.B), dim3(256), 0, s, a, qcnt, bucket, scap, qovf, thr);
    else if (a.kk <= 128)
        hipLaunchKernelGGL(k_select_bucket<2>, dim3((unsigned)a.B), dim3(256), 0, s, a, qcnt, bucket, scap, qovf, thr);
    else
        hipLaunchKernelGGL(k_select_bucket<4>, dim3((unsigned)a.B), dim3(256), 0, s, a, qcnt, bucket, scap, qovf, thr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------------------
// top-kk preselect per query row (one wave per query)
// ---------------------------------------------------------------------------
// One wave per (query, row segment): the segment's best kk (score, id).  With
// nseg segments per query the score matrix is streamed by B * nseg waves
// instead of B (a 1024-query batch is only 4 waves per CU).
template <int R>
__global__ __launch_bounds__(64) void k_select(ExactArgs a) {
    const int64_t b = blockIdx.x / a.nseg;
    const int sg = (int)(blockIdx.x % a.nseg);
    if (b >= a.B) return;
    if (a.only && !a.only[b]) return;
    const int lane = lane_id();
    const float* row = a.scores + (size_t)b * a.ldS;
    const float inf = __int_as_float(0x7f800000);
    BList<R> L;
    bl_init(L);
    const int kk = a.kk;
    float worst = inf;
    constexpr int U = 4;
    const int64_t seg = a.seglen;  // multiple of 256 * U
    const int64_t lo = (int64_t)sg * seg, hi = min(lo + seg, a.N);
    for (int64_t base = lo; base < hi; base += 256 * U) {
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
                const float x = e < hi ? vv[c] : inf;
                // <=: a row tying the kk-th score may still win on its id (rows
                // arrive c-interleaved, not in id order); +inf never enters
                unsigned long long m = __ballot(x <= worst && x < inf);
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
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int idx = r * 64 + lane;
        if (idx < kk) {
            const size_t o = ((size_t)b * a.nseg + sg) * kk + idx;
            a.seg_d[o] = L.d[r];
            a.seg_i[o] = L.i[r] == EMPTY_ID ? EMPTY_ID : (L.i[r] & ID_MASK);
        }
    }
}

// Merge a query's nseg segment lists: the best kk by (score, id) and the
// kk-th score (the certificate's bound; +inf when fewer than kk rows scored).
constexpr int SEL_MERGE_MAX = 1024;  // nseg * kk
__global__ __launch_bounds__(64) void k_select_merge(ExactArgs a) {
    __shared__ float sd[SEL_MERGE_MAX];
    __shared__ uint32_t si[SEL_MERGE_MAX];
    const int64_t b = blockIdx.x;
    if (b >= a.B) return;
    if (a.only && !a.only[b]) return;
    const int lane = lane_id();
    const int kk = a.kk, n = a.nseg * kk;
    const float inf = __int_as_float(0x7f800000);
    for (int e = lane; e < n; e += 64) {
        const size_t o = (size_t)b * n + e;
        const uint32_t id = a.seg_i[o];
        sd[e] = id == EMPTY_ID ? inf : a.seg_d[o];
        si[e] = id;
    }
    __syncthreads();
    for (int e = lane; e < kk; e += 64) a.cand[b * kk + e] = EMPTY_ID;
    float kth = inf;
    // every segment list is sorted by (score, id) with its empty slots (+inf,
    // EMPTY_ID) at the tail: an entry's rank is its position in its own list
    // plus, per other list, the length of the prefix ordered before it
    for (int e = lane; e < n; e += 64) {
        const uint32_t id = si[e];
        if (id == EMPTY_ID) continue;
        const float d = sd[e];
        const int s0 = e / kk;
        int rank = e - s0 * kk;
        for (int sg = 0; sg < a.nseg; ++sg) {
            if (sg == s0) continue;
            const float* ld = sd + sg * kk;
            const uint32_t* li = si + sg * kk;
            int lo = 0, hi = kk;  // first slot not ordered before (d, id)
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (li[mid] != EMPTY_ID && lt_di(ld[mid], li[mid], d, id))
                    lo = mid + 1;
                else
                    hi = mid;
            }
            rank += lo;
        }
        if (rank < kk) a.cand[b * kk + rank] = id;
        if (rank == kk - 1) kth = d;
    }
    for (int o = 32; o >= 1; o >>= 1) kth = fminf(kth, __shfl_xor(kth, o, 64));
    if (lane == 0 && a.bound) a.bound[b] = kth;
}

// ---------------------------------------------------------------------------
// canonical re-rank of the kk candidates -> best k by (distance, id)
// ---------------------------------------------------------------------------
template <class C, int G, int R>
__global__ __launch_bounds__(64) void k_rerank(const float* __restrict__ Q, GraphDev g, const uint32_t* cand, int kk,
                                               int64_t B, int k, int64_t* out_keys, float* out_dist, int32_t* out_n,
                                               int32_t* out_ids, CertArgs c) {
    const int64_t b = blockIdx.x;
    if (b >= B) return;
    if (c.only && !c.only[b]) return;
    const int lane = lane_id();
    QReg<C> q;
    load_query(q, Q + (size_t)b * C::PITCH);
    const float qn = query_norm(q);
    BList<R> L;
    bl_init(L);
    for (int c0 = 0; c0 < kk; c0 += 64) {
        const uint32_t cc = c0 + lane < kk ? cand[b * kk + c0 + lane] : EMPTY_ID;
        int cnt;
        const uint32_t cid = compact(cc, cc != EMPTY_ID, cnt);
        eval_list<C, G>(g, q, qn, cid, cnt, g.metric, [&](float d, uint32_t u) { bl_insert(L, k, d, u); });
    }
    int nv = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int idx = r * 64 + lane;
        const bool okr = idx < k && L.i[r] != EMPTY_ID;
        if (idx < k) {
            const uint32_t id = L.i[r] & ID_MASK;
            out_keys[b * k + idx] = okr ? g.keys[id] : (int64_t)-1;
            out_dist[b * k + idx] = okr ? L.d[r] : __int_as_float(0x7f800000);
            if (out_ids) out_ids[b * k + idx] = okr ? (int32_t)id : -1;
        }
        nv += __popcll(__ballot(okr));
    }
    if (lane == 0) out_n[b] = nv;
    if (c.bound) {
        const float t = c.bound[b];
        bool cert = true;
        if (t < __int_as_float(0x7f800000)) {  // rows were left out of the preselection
            float dk;
            uint32_t ik;
            bl_at(L, k - 1, dk, ik);
            if (ik == EMPTY_ID) {
                cert = false;
            } else if (g.metric == COSINE) {
                // measured roundings: rows' ex (and queries' eq, 1-product) ->
                // |q'.x' - q.x| <= (ex + eq + ex eq) |q| |x|
                const double xe = c.xerr ? (double)*c.xerr : 0.0, qe = c.qerr ? (double)*c.qerr : 0.0;
                const double ex = 1.01 * (1.0 + 1e-4) * (xe + qe + xe * qe);
                cert = (double)dk < (double)t - (double)c.eps_cos - ex;
            } else {
                const double qnd = c.qnorm[b], xm = *c.xmax;
                const double xe = c.xerr ? (double)*c.xerr : 0.0, qe = c.qerr ? (double)*c.qerr : 0.0;
                const double ed = c.eps_dot + 1.01 * (xe + qe + xe * qe);
                const double delta = 2.0 * ed * qnd * xm + c.c_l2 * (qnd + xm) * (qnd + xm);
                cert = (double)dk * (double)dk < (double)t - delta;
            }
        }
        if (lane == 0) {
            c.flag[b] = cert ? 0 : 1;
            if (!cert) {
                c.flagged[atomicAdd(c.nflag, 1)] = (int32_t)b;
                atomicAdd(c.stats, 1ull);
            }
        }
    }
}

// Canonical distance of every row for each uncertified query (the same
// arithmetic as the re-rank: eval_rows + stored canonical norms + finalize),
// written over that query's score row; deleted rows get +inf.  Blocks stride
// over row groups; with no flagged query every block exits at once.
template <class C, int G>
__global__ __launch_bounds__(256) void k_exact_fallback(const float* __restrict__ Q, GraphDev g, int64_t N,
                                                        const int32_t* flagged, const int32_t* nflag,
                                                        float* __restrict__ scores, int64_t ldS) {
    using RM = RowMap<C, G>;
    constexpr int GROUP = C::LPR >> RM::LG;
    const int nf = *nflag;
    if (nf == 0) return;
    const int lane = lane_id();
    const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t nw = (int64_t)gridDim.x * 4;
    const int64_t ngroups = (N + RM::T - 1) / RM::T;
    for (int f = 0; f < nf; ++f) {
        const int64_t b = flagged[f];
        QReg<C> q;
        load_query(q, Q + (size_t)b * C::PITCH);
        const float qn = query_norm(q);
        for (int64_t grp = gw; grp < ngroups; grp += nw) {
            const int64_t base = grp * RM::T;
            uint32_t ids[G];
            bool valid[G];
#pragma unroll
            for (int gg = 0; gg < G; ++gg) {
                const int64_t r = base + RM::reg_row(gg, lane);
                valid[gg] = r < N;
                ids[gg] = valid[gg] ? (uint32_t)r : 0u;
            }
            const float sacc = g.metric == EUCLIDEAN ? eval_rows<C, G, true>(q, g.vecs, g.pitch, ids, valid)
                                                     : eval_rows<C, G, false>(q, g.vecs, g.pitch, ids, valid);
            const int64_t rown = base + RM::owned_row(lane);
            if (rown < N && (lane & (GROUP - 1)) == 0) {
                const float xn = g.metric == COSINE ? g.norms[rown] : 1.f;
                float d = finalize(g.metric, sacc, xn, qn);
                if (g.dead && g.dead[rown]) d = __int_as_float(0x7f800000);
                scores[(size_t)b * ldS + rown] = d;
            }
        }
    }
}

// The fused path's fallback (precision 3): for each uncertified query, the
// canonical distance of every row (k_exact_fallback's arithmetic) streamed
// straight into a top-kk per row segment -- no score matrix.  Block (b, s):
// query b (flag[b] set, else it exits at once), segment s of nseg; its 4 waves
// take a quarter of the segment each, keep the best kk by (distance, id), and
// wave 0 merges the four lists (LDS) into the segment's list, in k_select's
// layout for k_select_merge.  Deleted rows and NaN distances never enter.
template <class C, int G, int R>
__global__ __launch_bounds__(256) void k_fallback_select(const float* __restrict__ Q, GraphDev g, int64_t N,
                                                         const uint8_t* __restrict__ flag, int kk, int nseg,
                                                         int64_t seglen, float* seg_d, uint32_t* seg_i) {
    using RM = RowMap<C, G>;
    constexpr int GROUP = C::LPR >> RM::LG;
    __shared__ float md[4 * 64 * R];
    __shared__ uint32_t mi[4 * 64 * R];
    const int64_t b = blockIdx.x / nseg;
    const int sg = (int)(blockIdx.x % nseg);
    if (!flag[b]) return;
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const float inf = __int_as_float(0x7f800000);
    QReg<C> q;
    load_query(q, Q + (size_t)b * C::PITCH);
    const float qn = query_norm(q);
    const int64_t lo = (int64_t)sg * seglen, hi = min(lo + seglen, N);
    const int64_t sub = (max<int64_t>(hi - lo, 0) + 3) / 4;
    const int64_t wlo = lo + w * sub, whi = min(wlo + sub, hi);
    BList<R> L;
    bl_init(L);
    float worst = inf;
    for (int64_t base = wlo; base < whi; base += RM::T) {
        uint32_t ids[G];
        bool valid[G];
#pragma unroll
        for (int gg = 0; gg < G; ++gg) {
            const int64_t r = base + RM::reg_row(gg, lane);
            valid[gg] = r < whi;
            ids[gg] = valid[gg] ? (uint32_t)r : 0u;
        }
        const float sacc = g.metric == EUCLIDEAN ? eval_rows<C, G, true>(q, g.vecs, g.pitch, ids, valid)
                                                 : eval_rows<C, G, false>(q, g.vecs, g.pitch, ids, valid);
        const int64_t rown = base + RM::owned_row(lane);
        const bool own = rown < whi && (lane & (GROUP - 1)) == 0;
        float d = inf;
        if (own) {
            const float xn = g.metric == COSINE ? g.norms[rown] : 1.f;
            d = finalize(g.metric, sacc, xn, qn);
            if (g.dead && g.dead[rown]) d = inf;
        }
        // <=: a row tying the kk-th distance may still win on its id
        unsigned long long m = __ballot(own && d <= worst && d < inf);
        while (m) {
            const int src = __ffsll((long long)m) - 1;
            m &= m - 1;
            if (bl_insert(L, kk, rl_f(d, src), (uint32_t)rl_u((uint32_t)rown, src))) {
                float wd;
                uint32_t wi;
                bl_at(L, kk - 1, wd, wi);
                worst = wi == EMPTY_ID ? inf : wd;
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        md[(w * R + r) * 64 + lane] = L.d[r];
        mi[(w * R + r) * 64 + lane] = L.i[r];
    }
    __syncthreads();
    if (w != 0) return;
    for (int ow = 1; ow < 4; ++ow)
        for (int e = 0; e < kk; ++e) {
            const uint32_t id = mi[(ow * R + (e >> 6)) * 64 + (e & 63)];  // (uniform reads: every lane the same entry)
            if (id == EMPTY_ID) break;
            bl_insert(L, kk, md[(ow * R + (e >> 6)) * 64 + (e & 63)], id & ID_MASK);
        }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int idx = r * 64 + lane;
        if (idx < kk) {
            const size_t o = ((size_t)b * nseg + sg) * kk + idx;
            seg_d[o] = L.d[r];
            seg_i[o] = L.i[r] == EMPTY_ID ? EMPTY_ID : (L.i[r] & ID_MASK);
        }
    }
}

// ---------------------------------------------------------------------------
// merge S shard lists (each sorted, n_in valid) -> best k by (distance, key)
// ---------------------------------------------------------------------------
// Total order on distances: the float order with -0 == +0, every NaN after
// +inf (NaN distances come back from compat searches over zero rows), and the
// padding of short lists after everything.  Ranks are then a permutation, so
// every output slot below min(k, valid) is written exactly once.
__device__ __forceinline__ uint32_t merge_ord(float d, bool valid) {
    if (!valid) return 0xFFFFFFFFu;
    if (d != d) return 0xFFFFFFFEu;
    uint32_t u = __float_as_uint(d == 0.0f ? 0.0f : d);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ __launch_bounds__(64) void k_merge(const int64_t* keys_in, const float* dist_in, const int32_t* n_in,
                                              int S, int64_t B, int k, int64_t* out_keys, float* out_dist,
                                              int32_t* out_n) {
    extern __shared__ __attribute__((aligned(16))) unsigned char msm[];
    uint32_t* so = reinterpret_cast<uint32_t*>(msm);
    int64_t* sk = reinterpret_cast<int64_t*>(msm + ((size_t)S * k * 4 + 15) / 16 * 16);
    const int64_t b = blockIdx.x;
    if (b >= B) return;
    const int lane = lane_id();
    const int tot = S * k;
    for (int e = lane; e < tot; e += 64) {
        const int s = e / k, j = e % k;
        const int nv = n_in[(size_t)s * B + b];
        const bool ok = j < nv;
        so[e] = merge_ord(ok ? dist_in[((size_t)s * B + b) * k + j] : 0.0f, ok);
        sk[e] = ok ? keys_in[((size_t)s * B + b) * k + j] : INT64_MAX;
    }
    __syncthreads();
    int nvalid = 0;
    for (int e = lane; e < tot; e += 64) {
        const uint32_t d = so[e];
        const int64_t key = sk[e];
        const bool valid = d != 0xFFFFFFFFu;
        int rank = 0;
        for (int f = 0; f < tot; ++f) {
            const uint32_t od = so[f];
            const int64_t ok = sk[f];
            rank += (od < d || (od == d && (ok < key || (ok == key && f < e)))) ? 1 : 0;
        }
        if (valid && rank < k) {
            const int s = e / k, j = e % k;
            out_keys[b * k + rank] = key;
            out_dist[b * k + rank] = dist_in[((size_t)s * B + b) * k + j];
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
    if (a.kk < 1 || a.kk > 256 || a.nseg < 1 || a.nseg * a.kk > SEL_MERGE_MAX || a.seglen % 1024) return -4;
    const dim3 grid((unsigned)(a.B * a.nseg));
    if (a.kk <= 64)
        hipLaunchKernelGGL(k_select<1>, grid, dim3(64), 0, s, a);
    else if (a.kk <= 128)
        hipLaunchKernelGGL(k_select<2>, grid, dim3(64), 0, s, a);
    else
        hipLaunchKernelGGL(k_select<4>, grid, dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_select_merge, dim3((unsigned)a.B), dim3(64), 0, s, a);
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
    X(64, 8, 2)            \
    X(64, 12, 1)           \
    X(64, 16, 1)

int launch_rerank(const float* Q, const GraphDev& g, const uint32_t* cand, int kk, int64_t B, int lpr, int vpl, int k,
                  int64_t* out_keys, float* out_dist, int32_t* out_n, int32_t* out_ids, const CertArgs& c,
                  hipStream_t s) {
    if (B <= 0) return 0;
    if (k > 256 || kk > 256 || k > kk) return -4;
#define X_(L, V, G)                                                                                              \
    if (lpr == L && vpl == V) {                                                                                  \
        if (k <= 64)                                                                                             \
            hipLaunchKernelGGL((k_rerank<Cfg<L, V>, G, 1>), dim3((unsigned)B), dim3(64), 0, s, Q, g, cand, kk, B, k, \
                               out_keys, out_dist, out_n, out_ids, c);                                           \
        else                                                                                                     \
            hipLaunchKernelGGL((k_rerank<Cfg<L, V>, G, 4>), dim3((unsigned)B), dim3(64), 0, s, Q, g, cand, kk, B, k, \
                               out_keys, out_dist, out_n, out_ids, c);                                           \
        return hipGetLastError() == hipSuccess ? 0 : -1;                                                         \
    }
    MH_FOR_EACH_CFG(X_)
#undef X_
    return -3;
}

int launch_exact_fallback(const float* Q, const GraphDev& g, int64_t N, const int32_t* flagged, const int32_t* nflag,
                          float* scores, int64_t ldS, int lpr, int vpl, hipStream_t s) {
    if (N <= 0) return 0;
#define X_(L, V, G)                                                                                          \
    if (lpr == L && vpl == V) {                                                                              \
        hipLaunchKernelGGL((k_exact_fallback<Cfg<L, V>, (G < 4 ? G : 4)>), dim3(1024), dim3(256), 0, s, Q, g, N, \
                           flagged, nflag, scores, ldS);                                                     \
        return hipGetLastError() == hipSuccess ? 0 : -1;                                                     \
    }
    MH_FOR_EACH_CFG(X_)
#undef X_
    return -3;
}

int launch_fallback_select(const float* Q, const GraphDev& g, const ExactArgs& a, int lpr, int vpl, hipStream_t s) {
    if (a.B <= 0 || a.N <= 0) return 0;
    if (a.kk < 1 || a.kk > 256 || a.nseg < 1 || a.nseg * a.kk > SEL_MERGE_MAX || !a.only) return -4;
    const dim3 grid((unsigned)(a.B * a.nseg));
#define X_(L, V, G)                                                                                            \
    if (lpr == L && vpl == V) {                                                                                \
        constexpr int GF = G < 4 ? G : 4;                                                                      \
        if (a.kk <= 64)                                                                                        \
            hipLaunchKernelGGL((k_fallback_select<Cfg<L, V>, GF, 1>), grid, dim3(256), 0, s, Q, g, a.N, a.only, \
                               a.kk, a.nseg, a.seglen, a.seg_d, a.seg_i);                                       \
        else if (a.kk <= 128)                                                                                  \
            hipLaunchKernelGGL((k_fallback_select<Cfg<L, V>, GF, 2>), grid, dim3(256), 0, s, Q, g, a.N, a.only, \
                               a.kk, a.nseg, a.seglen, a.seg_d, a.seg_i);                                       \
        else                                                                                                   \
            hipLaunchKernelGGL((k_fallback_select<Cfg<L, V>, GF, 4>), grid, dim3(256), 0, s, Q, g, a.N, a.only, \
                               a.kk, a.nseg, a.seglen, a.seg_d, a.seg_i);                                       \
        hipLaunchKernelGGL(k_select_merge, dim3((unsigned)a.B), dim3(64), 0, s, a);                            \
        return hipGetLastError() == hipSuccess ? 0 : -1;                                                       \
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
