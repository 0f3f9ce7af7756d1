// search_host.cpp -- host orchestration of the searches (graph.go:534-625,
// 1047-1110, 1116-1537): argument checks with the reference's error texts,
// stream ordering of the *_device calls, the beam / compat launches, and the
// exact path (score GEMM, fused preselection, bucket select, canonical re-rank,
// certificate, fallback); the negative-example re-ranking.
#include "index.hpp"

using namespace mhh;

namespace mhh {

// Mutations (Add / Delete / Reserve / Import) first let every enqueued
// search finish: they rewrite or reallocate what those kernels read.
// The beam search kernel is held to 2 waves per SIMD by its VGPRs (8 per CU),
// which leaves 20 KiB of the CU's 160 KiB LDS per wave: its visited set takes
// 1.25 * 2^vis_log2 entries (5,120 at the default), fewer resets at large ef.
int beam_vis_entries(const mhnsw_index* h) {
    if (h->vis_entries > 0) return h->vis_entries;
    return std::min(32768, 5 << (h->vis_log2 - 2));
}

int drain(mhnsw_index* h) {
    if (h->scr_valid) HIPCHK(h, hipEventSynchronize(h->scr_ev));
    h->scr_valid = false;
    return 0;
}

int search_body(mhnsw_index* h, const float* queries, bool on_device, int64_t B, int dim, int k, int mode, int ef,
                const int64_t* entry_key, int64_t* okeys, float* odist, int32_t* on, hipStream_t s, bool timing,
                int32_t* out_ids, bool sticky);

// every search: order after the previous scratch user (another stream), and
// after the metadata copies this call makes on the handle's stream.  sticky:
// the kernels report into d_err[1] (an asynchronous *_device search the caller
// checks with mhnsw_device_status); otherwise into d_err[0], zeroed first.
int search_impl(mhnsw_index* h, const float* queries, bool on_device, int64_t B, int dim, int k, int mode, int ef,
                const int64_t* entry_key, int64_t* okeys, float* odist, int32_t* on, hipStream_t s, bool timing,
                int32_t* out_ids, bool sticky) {
    if (h->scr_valid && h->scr_stream != s) HIPCHK(h, hipStreamWaitEvent(s, h->scr_ev, 0));
    const int r = search_body(h, queries, on_device, B, dim, k, mode, ef, entry_key, okeys, odist, on, s, timing,
                              out_ids, sticky);
    HIPCHK(h, hipEventRecord(h->scr_ev, s));
    h->scr_stream = s;
    h->scr_valid = true;
    return r;
}

// the search kernels run on the caller's stream; metadata goes up on the handle's
int order_meta(mhnsw_index* h, hipStream_t s) {
    if (s == h->stream) return 0;
    HIPCHK(h, hipEventRecord(h->meta_ev, h->stream));
    HIPCHK(h, hipStreamWaitEvent(s, h->meta_ev, 0));
    return 0;
}

int search_body(mhnsw_index* h, const float* queries, bool on_device, int64_t B, int dim, int k, int mode, int ef,
                const int64_t* entry_key, int64_t* okeys, float* odist, int32_t* on, hipStream_t s, bool timing,
                int32_t* out_ids, bool sticky) {
    int r = validate(h);
    if (r) return r;
    h->have_gemm_timing = false;  // last_gemm_ns describes this search or none
    if (k <= 0) return fail(h, MHNSW_EK, "k must be greater than 0, got %d", k);  // graph.go:542-544
    if (h->layers_exist && h->dim != dim) {                                          // graph.go:547-552
        if (B == 1) return fail(h, MHNSW_EDIM, "embedding dimension mismatch: %d != %d", h->dim, dim);
        return fail(h, MHNSW_EDIM, "embedding dimension mismatch for query %d: %d != %d", 0, h->dim, dim);
    }
    if (mode < 0 || mode > 2) return fail(h, MHNSW_EINVAL, "unknown search mode %d", mode);
    if (h->build_mode == MHNSW_BUILD_FLAT && mode != MHNSW_MODE_EXACT)
        return fail(h, MHNSW_EUNSUPPORTED, "flat index (build_mode 2) supports exact search only");
    if (B <= 0) return 0;
    if (!h->layers_exist || live_count(h) == 0) {  // graph.go:554-556: nil, nil
        if (on_device)
            HIPCHK(h, hipMemsetAsync(on, 0, B * 4, s));
        else
            memset(on, 0, B * 4);
        return 0;
    }
    if (ef <= 0) ef = h->ef;
    const int top = top_live_layer(h);
    uint32_t entry = (uint32_t)h->layers[top].entry;
    if (entry_key) {
        const int32_t e = key_row_in(h, *entry_key, top);
        if (e < 0) return fail(h, MHNSW_EINVAL, "entry key %lld not in top layer", (long long)*entry_key);
        entry = (uint32_t)e;
    }
    if ((r = ensure_buf(h, h->qpad, (size_t)B * h->pitch))) return r;
    const float* qsrc = queries;
    if (!on_device) {
        if ((r = ensure_buf(h, h->tmp, (size_t)B * dim))) return r;
        HIPCHK(h, hipMemcpyAsync(h->tmp.p, queries, (size_t)B * dim * 4, hipMemcpyHostToDevice, s));
        qsrc = h->tmp.p;
    }
    LCHK(h, launch_pad_rows(qsrc, B, dim, h->qpad.p, h->pitch, s));
    int64_t* dk = okeys;
    float* dd = odist;
    int32_t* dn = on;
    if (!on_device) {
        if ((r = ensure_buf(h, h->okeys, (size_t)B * k)) || (r = ensure_buf(h, h->odist, (size_t)B * k)) ||
            (r = ensure_buf(h, h->on, (size_t)B)))
            return r;
        dk = h->okeys.p;
        dd = h->odist.p;
        dn = h->on.p;
    }
    int* errw = sticky ? h->d_err + 1 : h->d_err;
    if (!sticky) HIPCHK(h, hipMemsetAsync(h->d_err, 0, sizeof(int), s));
    if (mode == MHNSW_MODE_EXACT) {
        if (k > 256) return fail(h, MHNSW_EUNSUPPORTED, "exact mode supports k <= 256");
        const bool split = h->exact_precision != 0;
        // fp16 1-product with the fused preselection (needs one full sample tile of rows)
        const bool h1 = h->exact_precision == 3 && h->n >= H1_BN;
        const bool h2 = h->exact_precision >= 2;  // fp16 row plane (1- and 2-product)
        // preselect width: the fp16 2-product scores carry a ~2x larger error bound, so the
        // kk-th score must sit further from the k-th distance for the certificate
        const int kk = h->exact_kk > 0 ? std::min(256, std::max(h->exact_kk, k))
                                       : std::min(256, h2 ? std::max(2 * k, 64) : std::max(2 * k, k + 16));
        const int64_t ldS = (h->n + 255) / 256 * 256;
        const int64_t budget = (int64_t)4 << 30;  // score workspace bytes
        int64_t qc = std::max<int64_t>(1, std::min<int64_t>(B, budget / (ldS * 4)));
        qc = std::min<int64_t>(qc, 4096);
        if ((r = ensure_buf(h, h->qnorm, (size_t)B)) ||
            (r = ensure_buf(h, h->cand, (size_t)qc * kk)) || (r = ensure_buf(h, h->xbound, (size_t)qc)) ||
            (r = ensure_buf(h, h->xflag, (size_t)qc)) || (r = ensure_buf(h, h->xflagged, (size_t)qc)) ||
            (r = ensure_buf(h, h->xnflag, 1)) || (r = ensure_buf(h, h->xmaxn, 1)))
            return r;
        // selection: enough (query, row-segment) waves to stream the score rows at full rate
        auto segs = [&](int64_t rows, int& ns, int64_t& sl) {
            ns = (int)std::min<int64_t>(16, std::max<int64_t>(1, (16384 + qc - 1) / qc));
            ns = (int)std::max<int64_t>(1, std::min<int64_t>(ns, (rows + 4095) / 4096));
            ns = std::max(1, std::min(ns, 1024 / kk));  // merge holds nseg * kk entries
            sl = ((rows + ns - 1) / ns + 1023) / 1024 * 1024;
        };
        int nseg;
        int64_t seglen;
        segs(h->n, nseg, seglen);
        if ((r = ensure_buf(h, h->xsegd, (size_t)qc * nseg * kk)) || (r = ensure_buf(h, h->xsegi, (size_t)qc * nseg * kk)))
            return r;
        // fused preselection (h1): the sample = every stride-th full row tile (about 32
        // tiles), its J-th best score per query is the threshold (J = kk when the
        // sample is every tile); a row passes at a rate of ~J / sample rows
        // the GEMM variant this search runs (exact_tile 0: the default, k_h1_pp16; a shape
        // it does not admit runs the ring kernel's filter)
        const int ev = h1_effective_variant(h->exact_tile, h->pitch, std::max<int64_t>(qc, h->capn));
        const int bm = h1_tile_bm(ev);
        const int64_t nnt = (h->n + H1_BN - 1) / H1_BN, nqt = (qc + bm - 1) / bm;
        const int stride = (int)std::max<int64_t>(1, std::min<int64_t>(128, (nnt + h->exact_sample - 1) / h->exact_sample));
        const int64_t nsamp = h1 ? ((h->n / H1_BN) - 1) / stride + 1 : 0;  // sampled full tiles
        const int J = stride < 8 ? kk : h->exact_thr_rank > 0 ? std::min(kk, std::max(k, h->exact_thr_rank)) : std::max(k, kk / 8);
        // the score workspace: every (query, row) score (precisions 0-2, and their
        // fallback), or only the sample's (fused path: its fallback streams distances
        // into per-segment lists, k_fallback_select)
        if ((r = ensure_buf(h, h->scores, (size_t)qc * (h1 ? (size_t)std::max<int64_t>(nsamp, 1) * H1_BN : (size_t)ldS))))
            return r;
        int sseg = 1;
        int64_t sseglen = 0;
        if (h1) {
            segs(nsamp * H1_BN, sseg, sseglen);
            sseg = std::max(1, std::min(sseg, 1024 / J));
        }
        // pairs per tile region / per query sub-bucket: 4x what the threshold lets
        // through on average (~J N / ns per query, ~bm J BN / ns per tile), with floors
        const int64_t ns = std::max<int64_t>(1, nsamp * H1_BN);
        // (a multiple of 8: k_h1_pp16 splits each tile's region among its 8 waves)
        // record-mode variants: per wave 4x the expected records (<= one per passing pair,
        // at most 8 block rows x 64 lanes), H1_REC uint2 each
        const int rcap = h1_records(ev)
                             ? 8 * H1_REC * (int)std::min<int64_t>(512, std::max<int64_t>(64, 4 * bm * J * H1_BN / ns / 8))
                             : (int)std::min<int64_t>((int64_t)bm * H1_BN, std::max<int64_t>(2048, 4 * bm * J * H1_BN / ns) + 7) / 8 * 8;
        const int rsub = h1_region_split(ev);
        const int scap = (int)std::min<int64_t>(std::max<int64_t>(h->n, 1),
                                                std::max<int64_t>(512, 8 * J * h->n / ns / H1_BSUB));
        if (h1 && ((r = ensure_buf(h, h->h1thr, (size_t)qc)) || (r = ensure_buf(h, h->h1c, (size_t)nqt * bm + 256)) ||
                   (r = ensure_buf(h, h->h1s, (size_t)nqt * bm + 256)) ||
                   (r = ensure_buf(h, h->h1region, (size_t)nqt * nnt * rcap)) ||
                   (r = ensure_buf(h, h->h1rcnt, (size_t)nqt * nnt * rsub)) ||
                   (r = ensure_buf(h, h->h1xw, (size_t)std::max<int64_t>(h->n, 1) * 4)) ||
                   (r = ensure_buf(h, h->h1qcnt, (size_t)qc * H1_BSUB * H1_CSTRIDE)) || (r = ensure_buf(h, h->h1ovf, (size_t)qc)) ||
                   (r = ensure_buf(h, h->h1bucket, (size_t)qc * H1_BSUB * scap)) || (r = ensure_buf(h, h->qerr, 1)) ||
                   (r = ensure_buf(h, h->xsegd, (size_t)qc * sseg * J)) ||
                   (r = ensure_buf(h, h->xsegi, (size_t)qc * sseg * J))))
            return r;
        if (split) {
            const int64_t plane = h->capn * h->pitch;
            const int kind = h2 ? 2 : 1;
            if (h->xsplit.n < (size_t)plane * 2 || h->xsplit_plane != plane || h->xsplit_kind != kind) {
                if ((r = ensure_buf(h, h->xsplit, (size_t)plane * 2))) return r;
                h->xsplit_rows = 0;
                h->xsplit_plane = plane;
                h->xsplit_kind = kind;
            }
            if ((r = ensure_buf(h, h->qsplit, (size_t)qc * h->pitch * 2))) return r;
            if (h2 && ((r = ensure_buf(h, h->xinv, (size_t)h->capn)) || (r = ensure_buf(h, h->qinv, (size_t)qc)) ||
                       (r = ensure_buf(h, h->xerr, 1))))
                return r;
        }
        LCHK(h, launch_norms(h->qpad.p, 0, B, h->pitch, h->lpr, h->vpl, h->qnorm.p, s));
        if ((r = sync_layer_table(h)) || (r = order_meta(h, s))) return r;
        GraphDev g = graph_view(h);
        g.err = errw;
        // rows the brute force skips: deleted ones, and the live rows of a failed
        // insert that never reached layer 0 (graph.go:1009 leaves them in upper
        // layers only; Search cannot return them)
        const uint8_t* xdead = h->any_dead ? h->dead : nullptr;
        if (h->partial_rows && h->xgone_epoch != h->mut_epoch) {  // rebuilt only after a mutation
            // a Delete or a replacement sweep may have killed the last partial rows
            std::vector<uint8_t> gone((size_t)h->n);
            int64_t partial = 0;
            for (int64_t i = 0; i < h->n; ++i) {
                const bool p = !h->hdead[i] && !in_layer(h, i, 0);
                partial += p;
                gone[i] = h->hdead[i] || p;
            }
            h->partial_rows = partial;
            if (partial) {
                if ((r = ensure_buf(h, h->xgone, (size_t)std::max<int64_t>(h->n, 1)))) return r;
                HIPCHK(h, hipMemcpyAsync(h->xgone.p, gone.data(), (size_t)h->n, hipMemcpyHostToDevice, s));
                HIPCHK(h, hipStreamSynchronize(s));
            }
            h->xgone_epoch = h->mut_epoch;
        }
        if (h->partial_rows) xdead = h->xgone.p;
        g.dead = xdead;
        // certificate constants (u = 2^-24; gamma_n = n u / (1 - n u) bounds any
        // order of n-term f32 summation relative to the sum of magnitudes)
        const double u = std::ldexp(1.0, -24);
        auto gam = [&](double nn) { return nn * u / (1.0 - nn * u); };
        // products per element: f32 1, bf16x3 3, fp16 2-product 2, fp16 1-product 1.  Split
        // error: bf16x3 drops ql.xl and the planes' tails (3.02 * 2^-16); fp16 2-product
        // rounds the rows to fp16 (2^-11 |x|, Cauchy-Schwarz) and the queries to hi + lo
        // (2^-21); fp16 1-product rounds both once
        const double g_mfma = gam((h1 ? 1.0 : h2 ? 2.0 : split ? 3.0 : 1.0) * h->pitch + 1);
        // (fp16: the rows' part -- and the queries' in the 1-product -- is the measured
        // max |x' - x| / |x| <= 2^-11, added on the device)
        const double e_split = h1 ? 0.0 : h2 ? std::ldexp(1.0, -21) : split ? 3.02 * std::ldexp(1.0, -16) : 0.0;
        const double g_can = gam(4.0 * h->vpl + 8);  // canonical: 4*VPL fmaf per lane + 6 butterfly levels
        CertArgs cert{};
        cert.qnorm = h->qnorm.p;
        cert.xmax = h->xmaxn.p;
        cert.eps_cos = (float)(1.01 * ((g_mfma + e_split + g_can) * (1.0 + 1e-4) + 16 * u));
        cert.eps_dot = (float)(1.01 * (g_mfma + e_split + g_can));
        cert.c_l2 = (float)(1.01 * (2.0 * gam(4.0 * h->vpl + 10) + 16 * u));
        cert.flag = h->xflag.p;
        cert.flagged = h->xflagged.p;
        cert.nflag = h->xnflag.p;
        cert.stats = h->d_stats + 3;
        cert.xerr = h2 ? h->xerr.p : nullptr;
        cert.qerr = h1 ? h->qerr.p : nullptr;
        if (timing) HIPCHK(h, hipEventRecord(h->ev0, s));
        if (split && h->xsplit_rows < h->n) {
            uint16_t* xh = h->xsplit.p;
            uint16_t* xl = h->xsplit.p + (size_t)h->capn * h->pitch;
            if (h2) {
                if (h->xsplit_rows == 0) HIPCHK(h, hipMemsetAsync(h->xerr.p, 0, sizeof(float), s));
                LCHK(h, launch_split_h16(h->vecs, h->xsplit_rows, h->n, h->pitch, h->capn, xh, nullptr, h->xinv.p,
                                         h->xerr.p, s));
            }
            else
                LCHK(h, launch_split_rows(h->vecs, h->xsplit_rows, h->n, h->pitch, h->capn, xh, xl, s));
            h->xsplit_rows = h->n;
        }
        if (h->metric == EUCLIDEAN) {
            HIPCHK(h, hipMemsetAsync(h->xmaxn.p, 0, sizeof(float), s));
            LCHK(h, launch_max_norm(h->norms, h->n, h->xmaxn.p, s));
        }
        for (int64_t q0 = 0; q0 < B; q0 += qc) {
            const int64_t nb = std::min(qc, B - q0);
            ExactArgs a{};
            a.X = h->vecs;
            a.xnorm = h->norms;
            a.dead = xdead;
            a.N = h->n;
            a.Q = h->qpad.p + (size_t)q0 * h->pitch;
            a.qnorm = h->qnorm.p + q0;
            a.B = nb;
            a.pitch = h->pitch;
            a.dim = h->dim;
            a.metric = h->metric;
            a.scores = h->scores.p;
            a.ldS = ldS;
            a.kk = kk;
            a.cand = h->cand.p;
            a.bound = h->xbound.p;
            a.nseg = nseg;
            a.seglen = seglen;
            a.seg_d = h->xsegd.p;
            a.seg_i = h->xsegi.p;
            int64_t* ok_ = dk + q0 * k;
            float* od_ = dd + q0 * k;
            int32_t* on_ = dn + q0;
            int32_t* oi_ = out_ids ? out_ids + q0 * k : nullptr;
            if (split) {
                a.Xh = h->xsplit.p;
                a.Xl = h->xsplit.p + (size_t)h->capn * h->pitch;
                a.ldXs = h->capn;
                a.Qh = h->qsplit.p;
                a.Ql = h->qsplit.p + (size_t)qc * h->pitch;
                a.ldQs = qc;
                if (h1) {
                    a.xinv = h->xinv.p;
                    a.qinv = h->qinv.p;
                    HIPCHK(h, hipMemsetAsync(h->qerr.p, 0, sizeof(float), s));
                    LCHK(h, launch_split_h16(a.Q, 0, nb, h->pitch, qc, h->qsplit.p, nullptr, h->qinv.p, h->qerr.p, s));
                    // 1. sample: every score of the sampled row tiles -> the kk-th best per query
                    ExactArgs as = a;
                    as.tile_stride = stride;
                    as.nsample_tiles = nsamp;
                    as.ldS = nsamp * H1_BN;
                    LCHK(h, launch_h1_sample(as, ev, s));
                    as.N = nsamp * H1_BN;
                    as.kk = J;
                    as.nseg = sseg;
                    as.seglen = sseglen;
                    as.bound = h->h1thr.p;
                    LCHK(h, launch_exact_select(as, s));
                    // 2. the full GEMM keeps the pairs that can beat it; 3. per-query buckets; 4. top-kk
                    LCHK(h, launch_ring_prep(h->h1thr.p, a.qnorm, a.qinv, nb, h->metric, h->h1c.p, h->h1s.p, s));
                    HIPCHK(h, hipMemsetAsync(h->h1qcnt.p, 0, (size_t)nb * H1_BSUB * H1_CSTRIDE * 4, s));
                    HIPCHK(h, hipMemsetAsync(h->h1ovf.p, 0, (size_t)nb, s));
                    a.tile_stride = 1;
                    a.ring_c = h->h1c.p;
                    a.ring_s = h->h1s.p;
                    a.region = h->h1region.p;
                    a.region_cnt = h->h1rcnt.p;
                    a.rcap = rcap;
                    a.xw = reinterpret_cast<const float4*>(h->h1xw.p);
                    if (q0 == 0)
                        LCHK(h, launch_h1_rowconst(h->xinv.p, h->norms, xdead, h->n, h->metric,
                                                   reinterpret_cast<float4*>(h->h1xw.p), s));
                    if (timing && q0 == 0) HIPCHK(h, hipEventRecord(h->gev0, s));
                    LCHK(h, launch_h1_filter(a, ev, s));
                    if (timing && q0 == 0) {
                        HIPCHK(h, hipEventRecord(h->gev1, s));
                        h->have_gemm_timing = true;
                    }
                    const int64_t bqt = (nb + bm - 1) / bm;
                    LCHK(h, launch_bucket(h->h1region.p, h->h1rcnt.p, rcap, bqt * nnt, bqt, bm, H1_BN, nb, h->h1qcnt.p,
                                          h->h1bucket.p, scap, h->h1ovf.p, rsub, h1_records(ev) ? 1 : 0, a, s));
                    LCHK(h, launch_select_bucket(a, h->h1qcnt.p, h->h1bucket.p, scap, h->h1ovf.p, h->h1thr.p, s));
                } else if (h2) {
                    a.xinv = h->xinv.p;
                    a.qinv = h->qinv.p;
                    LCHK(h, launch_split_h16(a.Q, 0, nb, h->pitch, qc, h->qsplit.p, h->qsplit.p + (size_t)qc * h->pitch,
                                             h->qinv.p, nullptr, s));
                    LCHK(h, launch_exact_scores_x2h(a, h->exact_tile, s));
                } else {
                    LCHK(h, launch_split_rows(a.Q, 0, nb, h->pitch, qc, h->qsplit.p,
                                              h->qsplit.p + (size_t)qc * h->pitch, s));
                    LCHK(h, launch_exact_scores_x3(a, h->exact_tile, s));
                }
            } else {
                LCHK(h, launch_exact_scores(a, s));
            }
            if (!h1) LCHK(h, launch_exact_select(a, s));
            if (h1 && h1_timing_diag(ev)) continue;  // timing diagnostic: no re-rank, no results
            HIPCHK(h, hipMemsetAsync(h->xnflag.p, 0, sizeof(int32_t), s));
            CertArgs c1 = cert;
            c1.bound = h->xbound.p;
            c1.qnorm = h->qnorm.p + q0;
            LCHK(h, launch_rerank(a.Q, g, h->cand.p, kk, nb, h->lpr, h->vpl, k, ok_, od_, on_, oi_, c1, s));
            // uncertified queries: canonical distances of every row, then select + re-rank again
            ExactArgs a2 = a;
            a2.only = h->xflag.p;
            a2.bound = nullptr;
            if (h1) {
                LCHK(h, launch_fallback_select(a.Q, g, a2, h->lpr, h->vpl, s));
            } else {
                LCHK(h, launch_exact_fallback(a.Q, g, h->n, h->xflagged.p, h->xnflag.p, h->scores.p, ldS, h->lpr,
                                              h->vpl, s));
                LCHK(h, launch_exact_select(a2, s));
            }
            CertArgs c2{};
            c2.only = h->xflag.p;
            LCHK(h, launch_rerank(a.Q, g, h->cand.p, kk, nb, h->lpr, h->vpl, k, ok_, od_, on_, oi_, c2, s));
        }
        if (timing) HIPCHK(h, hipEventRecord(h->ev1, s));
        if (h->exact_precision == 3 && h->n >= H1_BN && h1_timing_diag(ev))
            return fail(h, MHNSW_EUNSUPPORTED, "exact_tile %d is a timing diagnostic: no results", h->exact_tile);
    } else {
        if ((r = sync_layer_entries(h))) return r;
        if ((r = sync_layer_table(h)) || (r = order_meta(h, s))) return r;
        SearchArgs a;
        a.g = graph_view(h);
        a.g.err = errw;
        a.q = h->qpad.p;
        a.B = B;
        a.k = k;
        a.ef = ef;
        a.top = top;
        a.entry = entry;
        a.layer_entry = h->d_layer_entry;
        a.out_keys = dk;
        a.out_dist = dd;
        a.out_n = dn;
        a.out_ids = out_ids;
        a.stats = h->d_stats;
        a.err = errw;
        a.vis_log2 = h->vis_log2;
        a.vis_n = beam_vis_entries(h);
        // the compact set holds 8,192 ids in 16 KiB (the 32-bit set 5,120 in 20 KiB):
        // fewer resets at large ef, the same results either way.  Below ef 129 the
        // 32-bit set rarely fills and its single-CAS probe is the cheaper one
        // (the compact probe cost 1 % at the headline ef 64).
        // (only where the compact set holds more ids than the 32-bit one in the LDS
        // it is given: a user who raised vis_entries past 8,192 keeps that set)
        a.vis16 = h->vis_compact && std::max(ef, k) > 128 && h->capn <= (int64_t(1) << 24) &&
                  (int64_t)a.vis_n >= (int64_t)VIS16_WORDS && a.vis_n < VIS16_HOMES;
        a.upper_ef = h->upper_ef;
        a.mw_max_b = h->beam_mw_max_b;
        a.expand = h->search_expand;
        if (mode == MHNSW_MODE_BEAM) {
            if (std::max(ef, k) > 512) return fail(h, MHNSW_EUNSUPPORTED, "beam mode supports max(ef,k) <= 512");
            if (timing) HIPCHK(h, hipEventRecord(h->ev0, s));
            LCHK(h, launch_search_beam(a, h->lpr, h->vpl, s));
            if (timing) HIPCHK(h, hipEventRecord(h->ev1, s));
        } else {
            if (timing) HIPCHK(h, hipEventRecord(h->ev0, s));
            int lr = launch_search_compat(a, h->lpr, h->vpl, s);
            if (lr == -2) return fail(h, MHNSW_EUNSUPPORTED, "compat search LDS budget exceeded (ef=%d, k=%d)", ef, k);
            LCHK(h, lr);
            if (timing) HIPCHK(h, hipEventRecord(h->ev1, s));
        }
    }
    h->have_timing = timing;
    h->stats_host[6] += B;
    if (!on_device) {
        HIPCHK(h, hipMemcpyAsync(okeys, dk, (size_t)B * k * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipMemcpyAsync(odist, dd, (size_t)B * k * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipMemcpyAsync(on, dn, (size_t)B * 4, hipMemcpyDeviceToHost, s));
        int err = 0;
        HIPCHK(h, hipMemcpyAsync(&err, h->d_err, sizeof(int), hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipStreamSynchronize(s));
        if (err & 4) return fail(h, MHNSW_EINTERNAL, "out-of-range node id in adjacency (graph corrupt)");
        if (err) return fail(h, MHNSW_EINTERNAL, "visited set overflow (raise vis_log2)");
    }
    return 0;
}

}  // namespace mhh

extern "C" {

int mhnsw_search_negatives(mhnsw_index* h, const float* queries, int64_t B, int dim, const float* negatives,
                           const int32_t* neg_count, int k, float neg_weight, int mode, int ef, int flags,
                           int64_t* out_keys, float* out_score, int32_t* out_n) {
    std::unique_lock<std::shared_mutex> lk(h->mu);
    int r = validate(h);
    if (r) return r;
    if (k <= 0) return fail(h, MHNSW_EK, "k must be greater than 0, got %d", k);
    if (!(neg_weight >= 0.0f && neg_weight <= 1.0f))
        return fail(h, MHNSW_EINVAL, "negWeight must be between 0.0 and 1.0, got %f", (double)neg_weight);
    if (h->layers_exist && h->dim != dim)
        return fail(h, MHNSW_EDIM, "query embedding dimension mismatch: %d != %d", h->dim, dim);
    if (B <= 0) return 0;
    for (int64_t b = 0; b < B; ++b) out_n[b] = 0;
    if (!h->layers_exist || live_count(h) == 0) return 0;  // graph.go:1144-1146
    const int kx = std::max(3 * k, 10);                    // graph.go:1150-1153
    if (kx > NEG_MAX_CAND) return fail(h, MHNSW_EUNSUPPORTED, "negatives support k <= %d", NEG_MAX_CAND / 3);
    // queries without negatives are a plain Search(near, k) (graph.go:1395-1398)
    std::vector<int64_t> plain, rer;
    std::vector<int32_t> off(1, 0);
    for (int64_t b = 0; b < B; ++b) {
        if (neg_count[b] < 0) return fail(h, MHNSW_EINVAL, "negative count %d for query %lld", neg_count[b], (long long)b);
        (neg_count[b] == 0 ? plain : rer).push_back(b);
    }
    const int64_t ntot = [&] {
        int64_t t = 0;
        for (int64_t b = 0; b < B; ++b) t += neg_count[b];
        return t;
    }();
    hipStream_t s = h->stream;
    if (!plain.empty()) {
        std::vector<float> q(plain.size() * (size_t)dim);
        for (size_t i = 0; i < plain.size(); ++i)
            memcpy(&q[i * dim], queries + (size_t)plain[i] * dim, (size_t)dim * 4);
        std::vector<int64_t> kk(plain.size() * (size_t)k);
        std::vector<float> dd(plain.size() * (size_t)k);
        std::vector<int32_t> nn(plain.size());
        if ((r = search_impl(h, q.data(), false, (int64_t)plain.size(), dim, k, mode, ef, nullptr, kk.data(), dd.data(),
                             nn.data(), s, false)))
            return r;
        for (size_t i = 0; i < plain.size(); ++i) {
            memcpy(out_keys + (size_t)plain[i] * k, &kk[i * k], (size_t)k * 8);
            memcpy(out_score + (size_t)plain[i] * k, &dd[i * k], (size_t)k * 4);
            out_n[plain[i]] = nn[i];
        }
    }
    if (rer.empty()) return 0;
    const int64_t R = (int64_t)rer.size();
    // gather the re-ranked queries and their negatives
    std::vector<float> q((size_t)R * dim), ng((size_t)std::max<int64_t>(ntot, 1) * dim);
    std::vector<int64_t> noff_b((size_t)B + 1, 0);
    for (int64_t b = 0; b < B; ++b) noff_b[(size_t)b + 1] = noff_b[(size_t)b] + neg_count[b];
    int64_t w = 0;
    for (int64_t i = 0; i < R; ++i) {
        const int64_t b = rer[(size_t)i];
        memcpy(&q[(size_t)i * dim], queries + (size_t)b * dim, (size_t)dim * 4);
        memcpy(&ng[(size_t)w * dim], negatives + (size_t)noff_b[(size_t)b] * dim, (size_t)neg_count[b] * dim * 4);
        w += neg_count[b];
        off.push_back((int32_t)w);
    }
    if ((r = ensure_buf(h, h->nq, (size_t)R * dim)) || (r = ensure_buf(h, h->nneg, (size_t)std::max<int64_t>(w, 1) * h->pitch)) ||
        (r = ensure_buf(h, h->nck, (size_t)R * kx)) || (r = ensure_buf(h, h->ncd, (size_t)R * kx)) ||
        (r = ensure_buf(h, h->nci, (size_t)R * kx)) || (r = ensure_buf(h, h->ncn, (size_t)R)) ||
        (r = ensure_buf(h, h->noff, (size_t)R + 1)) || (r = ensure_buf(h, h->nok, (size_t)R * k)) ||
        (r = ensure_buf(h, h->nos, (size_t)R * k)) || (r = ensure_buf(h, h->non, (size_t)R)))
        return r;
    HIPCHK(h, hipMemcpyAsync(h->nq.p, q.data(), q.size() * 4, hipMemcpyHostToDevice, s));
    HIPCHK(h, hipMemcpyAsync(h->noff.p, off.data(), off.size() * 4, hipMemcpyHostToDevice, s));
    if (w > 0) {
        if ((r = ensure_buf(h, h->tmp, (size_t)w * dim))) return r;
        HIPCHK(h, hipMemcpyAsync(h->tmp.p, ng.data(), (size_t)w * dim * 4, hipMemcpyHostToDevice, s));
        LCHK(h, launch_pad_rows(h->tmp.p, w, dim, h->nneg.p, h->pitch, s));
    }
    // candidates: Search(near, kx) in the requested mode, internal ids kept
    if ((r = search_impl(h, h->nq.p, true, R, dim, kx, mode, ef, nullptr, h->nck.p, h->ncd.p, h->ncn.p, s, false,
                         h->nci.p)))
        return r;
    if ((r = sync_layer_table(h))) return r;
    NegArgs a;
    a.g = graph_view(h);
    a.neg = h->nneg.p;
    a.neg_off = h->noff.p;
    a.cand_ids = h->nci.p;
    a.cand_d = h->ncd.p;
    a.cand_n = h->ncn.p;
    a.B = R;
    a.kx = kx;
    a.k = k;
    a.w = neg_weight;
    a.flags = flags;
    a.out_keys = h->nok.p;
    a.out_score = h->nos.p;
    a.out_n = h->non.p;
    LCHK(h, launch_negatives(a, h->lpr, h->vpl, s));
    std::vector<int64_t> kk((size_t)R * k);
    std::vector<float> ss((size_t)R * k);
    std::vector<int32_t> nn((size_t)R);
    HIPCHK(h, hipMemcpyAsync(kk.data(), h->nok.p, kk.size() * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipMemcpyAsync(ss.data(), h->nos.p, ss.size() * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipMemcpyAsync(nn.data(), h->non.p, nn.size() * 4, hipMemcpyDeviceToHost, s));
    int err = 0;  // the candidate search and the re-ranking report into d_err[0]
    HIPCHK(h, hipMemcpyAsync(&err, h->d_err, sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipStreamSynchronize(s));
    if (err & 4) return fail(h, MHNSW_EINTERNAL, "out-of-range node id in adjacency (graph corrupt)");
    if (err) return fail(h, MHNSW_EINTERNAL, "visited set overflow (raise vis_log2)");
    for (int64_t i = 0; i < R; ++i) {
        const int64_t b = rer[(size_t)i];
        memcpy(out_keys + (size_t)b * k, &kk[(size_t)i * k], (size_t)k * 8);
        memcpy(out_score + (size_t)b * k, &ss[(size_t)i * k], (size_t)k * 4);
        out_n[b] = nn[(size_t)i];
    }
    return 0;
}

}  // extern "C"
