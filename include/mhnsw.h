/*
 * mhnsw.h -- C ABI of the MI355X-native HNSW engine (libmhnsw.so).
 *
 * This is the drop-in boundary for the hot path of TFMV/hnsw (Go): the
 * distance sweep -> layer-0 greedy/beam search -> M-neighbour selection on
 * insert.  Every entry point is plain C (pointers + sizes, no torch types) so
 * the Go package can bind it through cgo; see INTEGRATION.md for the binding
 * a maintainer would add.  Each declaration names the reference interface it
 * replaces (paths relative to the reference repository root).
 *
 * Conventions
 *  - Keys are int64 (the reference's Graph[int]); vectors are float32,
 *    row-major, `dim` contiguous floats per row.
 *  - Host-pointer entry points copy their inputs before returning (the cgo
 *    rule forbids C from retaining Go pointers).  *_device entry points take
 *    device pointers and enqueue asynchronously on the given HIP stream
 *    (NULL = the HIP null stream, as in the HIP/CUDA runtime convention).
 *  - Return value: MHNSW_OK (0) or a negative error class; the message, with
 *    the reference's wording where one exists, is mhnsw_last_error(h).
 *  - Concurrency mirrors graph.go:328 (sync.RWMutex): searches may run
 *    concurrently on one handle; add/import are exclusive.
 */
#ifndef MHNSW_H
#define MHNSW_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mhnsw_index mhnsw_index;

/* DistanceFunc identities (distance.go:25-28 distanceFuncs registry) */
#define MHNSW_NO_DISTANCE (-1) /* Graph.Distance == nil */
#define MHNSW_COSINE 0         /* distance.go:15 CosineDistance */
#define MHNSW_EUCLIDEAN 1      /* distance.go:20 EuclideanDistance */

/* search modes */
#define MHNSW_MODE_COMPAT 0 /* graph.go:94-170 semantics, results in heap order */
#define MHNSW_MODE_BEAM 1   /* standard HNSW best-first (ef), sorted results   */
#define MHNSW_MODE_EXACT 2  /* brute force (MFMA scores + canonical re-rank)   */

/* build modes (option "build_mode") */
#define MHNSW_BUILD_COMPAT 0 /* graph.go:437-531 sequential Add semantics */
#define MHNSW_BUILD_BATCH 1  /* batched parallel insert (throughput)      */
#define MHNSW_BUILD_FLAT 2   /* vector store only, exact search (hnsw-extensions/hybrid/exact.go ExactIndex) */

/* error classes */
#define MHNSW_OK 0
#define MHNSW_EINVAL (-1)       /* Validate() failure / bad argument          */
#define MHNSW_EDIM (-2)         /* "embedding dimension mismatch: %d != %d"   */
#define MHNSW_EK (-3)           /* "k must be greater than 0, got %d"         */
#define MHNSW_ENOMEM (-4)
#define MHNSW_EDEVICE (-5)      /* HIP runtime / kernel launch failure         */
#define MHNSW_EUNSUPPORTED (-6) /* outside this build's supported envelope     */
#define MHNSW_EINTERNAL (-7)

/* ---- lifecycle: NewGraph / NewGraphWithConfig (graph.go:340-366) ----
 * Binds the handle to the current HIP device.  Fails with the Validate()
 * message (graph.go:916-937) when the configuration is invalid; the message is
 * then available from mhnsw_last_error(NULL). */
int mhnsw_create(int metric, int M, double ml, int ef_search, uint64_t seed, mhnsw_index **out);
void mhnsw_destroy(mhnsw_index *h);
const char *mhnsw_last_error(const mhnsw_index *h);

/* ---- public Graph fields (graph.go:305-326): Distance, M, Ml, EfSearch, Rng ---- */
int mhnsw_set_params(mhnsw_index *h, int metric, int M, double ml, int ef_search);
int mhnsw_get_params(const mhnsw_index *h, int *metric, int *M, double *ml, int *ef_search);
int mhnsw_seed(mhnsw_index *h, uint64_t seed); /* Rng = rand.New(rand.NewSource(seed)) analogue */
/* engine options: "build_mode", "m0" (layer-0 degree cap, batch mode),
 * "ef_construction" (<= 512), "heuristic" (0 closest-M, 1 HNSW heuristic on new rows,
 * 2 also when a reverse edge overflows a row), "keep_pruned", "prune_alpha_pct"
 * (heuristic slack x100: c is dropped when alpha*d(c,kept) < d(u,c); 100 = HNSW
 * Alg. 4), "batch_min", "batch_max", "batch_ratio_pct" (batched insert: each batch holds this
 * % of the rows already indexed, default 5 -- a batch is searched against the index as it
 * stood before it, so larger batches build faster but link a batch's rows to each other
 * only through reverse edges: adding 1,000 rows to a 5,100-row index in one 20 % batch
 * left 16 % of them unreachable by their own vector at ef 64), "vis_log2" (compat / build visited sets:
 * 2^n entries), "vis_entries" (beam search's visited set, 0 = 1.25 * 2^vis_log2),
 * "build_expand" (batched insert: entries expanded per step of its layer
 * searches, 1-4, default 4 -- they fetch their adjacency rows in one round
 * trip and evaluate their new neighbours as one batch), "upper_efc" (batched
 * insert: the candidate list of its searches in the layers above 0, 0 (default) =
 * efConstruction on every layer; those rows hold M neighbours and their
 * searches are narrow launches -- 128 builds the 1M bench index 22 % faster at
 * the same recall), "search_expand" (beam
 * mode: entries expanded per step of the layer-0 search, 1 (default, the
 * standard best-first search), 2 or 4 -- the best unexpanded entries are taken
 * together, their adjacency rows fetched in one round trip and their new
 * neighbours scored as one batch; a different search from 1 (results can
 * differ), bit-identical to the oracle's og_set_search_expand; always the
 * one-wave kernel), "exact_kk",
 * "exact_thr_rank" (precision 3: the threshold is the sample's J-th best score,
 * J = max(k, this) capped at kk; 0 (default) = max(k, kk / 8)),
 * "exact_sample" (precision 3: at most this many row tiles form the threshold
 * sample, every ceil(tiles / this)-th, default 64),
 * "exact_precision" (exact-mode scoring: 0 f32-input MFMA, 1 bf16x3 split MFMA,
 * 2 fp16 2-product split MFMA, 3 (default) fp16 1-product MFMA with the top-kk
 * preselection fused into the GEMM epilogue; all preselect, re-rank canonically
 * and certify, so results are identical),
 * "exact_tile" (GEMM variant, 0 = the measured best per precision; precisions 1/2:
 * 1 128x256, 2 128x128, 3 256x256 ring tiles; precision 3: 34 (the default)
 * the persistent two-group ping-pong stream k_h1_pp16 on 16x16x32 MFMAs with
 * the fused filter storing per-lane records of a block row's accumulators,
 * 5 the ring kernel's fused filter (128x256), which also runs every shape
 * k_h1_pp16 does not admit), "compat_waves" (1 or 8 waves scoring the compat insert's
 * distance batches), "upper_ef" (beam mode: upper-layer descent width, 1 =
 * greedy), "beam_mw_max_b" (beam mode, ef and k <= 128: batches of at most this
 * many queries run one workgroup of 4 waves per query -- the single-query
 * latency path of ParallelSearch, graph.go:631-790; default 512, 0 = never;
 * results are identical either way; the standard search only: search_expand 2 / 4
 * run the one-wave kernel), "build_mw_max" (batched insert with the screening
 * copy, build_expand 2-4: a layer launch of at most this many inserts runs one
 * workgroup of 4 waves per insert, the candidate batches of its searches split
 * over the waves; default 256, 0 = never; the same graph either way), "vis_compact" (beam mode at max(ef, k) > 128 and batched insert at
 * efConstruction > 128, default 1: when node
 * ids are below 2^24 the visited set stores 16-bit entries -- 8,192 ids in 16 KiB
 * of LDS, where the beam search's 32-bit set holds 5,120 in 20 KiB and the
 * insert's (vis_log2 12) 4,096 in 16 KiB -- so a large-ef search resets it less;
 * exact, the same results and graph either way), "screen" (beam mode and batched insert, default 1: keep an fp16
 * copy of the rows; a candidate is skipped only when the copy proves the f32
 * distance rejects it, so results are unchanged);
 * "max_rows" (row capacity limit, 0 = none: an Add that would need more rows
 * fails with MHNSW_ENOMEM and leaves the index, its key maps and its Rng as
 * they were);
 * read-only: "pitch", "capacity", "strkeys", "strkey_relabels", "last_gemm_ns" (device
 *            time of the last timed exact search's fused fp16 score GEMM, first query chunk),
 *            "screen_err_ppb" (the fp16 screening copy's measured max relative
 *            rounding E, the margin its rejects use, in parts per 1e9) */
int mhnsw_set_option(mhnsw_index *h, const char *name, int64_t value);
int mhnsw_get_option(const mhnsw_index *h, const char *name, int64_t *value);
/* Graph.Validate (graph.go:916-937) */
int mhnsw_validate(mhnsw_index *h);
/* pre-size device storage for n vectors of `dim` floats */
int mhnsw_reserve(mhnsw_index *h, int64_t n, int dim);

/* ---- Graph.Add / Graph.BatchAdd (graph.go:437-531, 942-1042) ----
 * levels: NULL draws each level like randomLevel (graph.go:388-417) from the
 * handle's RNG; non-NULL injects them (a host drawing from its own Rng, or
 * parity testing).  COMPAT build mode follows BatchAdd's walk: the nodes are
 * inserted in order; a node whose key is already present (in the index or
 * earlier in the batch) replaces the key's nodes -- after its layer search,
 * every layer holding the key deletes and isolates it (graph.go:1015-1024) --
 * and when layer 0 held the key the walk stops with "node not added"
 * (MHNSW_EINTERNAL; graph.go:1035-1037: Len() did not grow); a key whose nodes
 * sat only in upper layers (left by a failed insert) leaves Len() one higher,
 * and the walk goes on.  A failing insert ("no nodes found in
 * neighborhood search", graph.go:1009) also ends the walk, leaving the graph as
 * the reference leaves it.  Add of a present key deadlocks in the reference
 * (graph.go:511-513 -> Delete re-locks, :844); here it is BatchAdd's walk.
 * BATCH / FLAT build modes reject a present key (MHNSW_EUNSUPPORTED). */
int mhnsw_add(mhnsw_index *h, const int64_t *keys, const float *vecs, int64_t n, int dim, const int32_t *levels);
/* same, vectors already in HBM (keys/levels stay host pointers) */
int mhnsw_add_device(mhnsw_index *h, const int64_t *keys, const float *d_vecs, int64_t n, int dim,
                     const int32_t *levels);
/* For hosts that draw levels from their own Rng (graph.go:962: one draw per
 * insert the walk reaches, from the layer-0 size at that moment): *nwalk = the
 * inserts up to and including the first key already present (or repeated) --
 * where a COMPAT walk may stop (it does when that key's node holds a layer at
 * or below the new level); *one_by_one = 1 when an insert may fail with "no
 * nodes found in neighborhood search" (the index holds deleted or replaced
 * rows).  A host draws nwalk levels, adds those nodes, and repeats with the
 * rest until done or an error ends the walk.  When one_by_one is set, a host
 * that can rewind its Rng still adds the nwalk nodes in one call: after an
 * error, mhnsw_add_reached says how many inserts the walk got to (the draws
 * the reference made, graph.go:962); the host rewinds and redraws that many.
 * A host that cannot rewind adds one node per call instead. */
int mhnsw_add_plan(mhnsw_index *h, const int64_t *keys, int64_t n, int64_t *nwalk, int *one_by_one);
/* The inserts the last mhnsw_add / mhnsw_add_device walk reached, counting a
 * replacing insert ("node not added") and a failing one ("no nodes found in
 * neighborhood search", graph.go:1009) -- i.e. the levels it consumed; 0 after
 * an error that left the index untouched (validation, dimension, capacity). */
int mhnsw_add_reached(const mhnsw_index *h, int64_t *reached);

/* ---- Graph.Search / Graph.BatchSearch (graph.go:534-625, 1047-1110) ----
 * B queries of `dim` floats; outputs hold B*k slots; out_n[b] results for
 * query b.  ef <= 0 uses EfSearch.  entry_key (nullable) replaces the
 * arbitrary layer.entry() (graph.go:250-258) of the top layer. */
int mhnsw_search(mhnsw_index *h, const float *queries, int64_t B, int dim, int k, int mode, int ef,
                 const int64_t *entry_key, int64_t *out_keys, float *out_dist, int32_t *out_n);
int mhnsw_search_device(mhnsw_index *h, const float *d_queries, int64_t B, int dim, int k, int mode, int ef,
                        int64_t *d_keys, float *d_dist, int32_t *d_n, void *stream);
/* Errors of *_device searches.  mhnsw_search_device returns once its kernels
 * are enqueued, so what they detect (a compat search whose visited set
 * overflows -- the reference's visited map is exact, graph.go:141-144 -- or an
 * out-of-range id in the adjacency) cannot be its return value: it accumulates
 * in a per-handle word.  This call waits for the last enqueued search, returns
 * MHNSW_OK or MHNSW_EINTERNAL with the message of the host-pointer path, and
 * clears the word. */
int mhnsw_device_status(mhnsw_index *h);

/* ---- SearchWithNegative(s) / BatchSearchWithNegatives (graph.go:1116-1537) ----
 * Query b's negatives are the next neg_count[b] rows of `negatives` (B*dim
 * queries, sum(neg_count)*dim negatives).  Candidates = Search(near,
 * max(3k,10)) in `mode`; scored in float32 as the reference (graph.go:1174-
 * 1210 / 1300-1345) and returned by descending score (ties in candidate
 * order, NaN last).  neg_count[b] == 0 runs a plain Search(near, k)
 * (out_score then holds distances).  flags bit 0 enables the reference's
 * key 7..9 boost (a test hack, graph.go:1338-1344).  k <= 85. */
int mhnsw_search_negatives(mhnsw_index *h, const float *queries, int64_t B, int dim, const float *negatives,
                           const int32_t *neg_count, int k, float neg_weight, int mode, int ef, int flags,
                           int64_t *out_keys, float *out_score, int32_t *out_n);

/* ---- Len / Dims / Lookup / Analyzer.Topography (graph.go:829, 421, 898; analyzer.go:41) ----
 * Lookup reads layer 0 (graph.go:906) and copies the key's vector. */
int64_t mhnsw_len(const mhnsw_index *h);
int mhnsw_dims(const mhnsw_index *h);
int mhnsw_lookup(mhnsw_index *h, int64_t key, float *out_vec); /* 1 found, 0 absent, <0 error */
/* out[i] = 1 when keys[i] has a live node (the `_, ok := layer.nodes[key]` test
 * of graph.go:1016 / hybrid/exact.go:30, without copying vectors) */
int mhnsw_contains(const mhnsw_index *h, const int64_t *keys, int64_t n, uint8_t *out);
int mhnsw_num_layers(const mhnsw_index *h);
int64_t mhnsw_layer_count(const mhnsw_index *h, int layer);
/* Analyzer.Connectivity (analyzer.go:20-38): mean neighbour count of each
 * non-empty layer; returns how many layers it has (writes min(that, max_layers)) */
int mhnsw_connectivity(mhnsw_index *h, double *out, int max_layers);

/* ---- Graph.Delete / Graph.BatchDelete (graph.go:843-895) ----
 * out[i] = 1 when keys[i] was present.  COMPAT build mode runs the reference's
 * isolate + replenish per key (graph.go:172-235: the deleted row keeps its
 * edges and stays reachable through one-directional links, as in Go); BATCH
 * build mode repairs every row that points at a deleted node in parallel.
 * Deleted rows are never returned by BEAM or EXACT searches. */
int mhnsw_delete(mhnsw_index *h, const int64_t *keys, int64_t n, uint8_t *out);

/* ---- ExactIndex replace-on-Add (hnsw-extensions/hybrid/exact.go:28-59: Add of
 * a present key is a map assignment) ----
 * FLAT build mode only (a vector store without links).  For every key present,
 * its row's vector is overwritten in place (norms, the fp16 screening copy and
 * the exact path's split planes follow); out[i] = 1 when keys[i] was present,
 * 0 otherwise (the caller adds those).  Keys must be distinct.  Nothing is
 * written unless every argument is valid. */
int mhnsw_replace(mhnsw_index *h, const int64_t *keys, const float *vecs, int64_t n, int dim, uint8_t *out);

/* ---- DistanceFunc (distance.go:12-23): batched sweep of one query over n rows ---- */
int mhnsw_distance(int metric, const float *q, const float *X, int64_t n, int dim, float *out);
int mhnsw_distance_device(int metric, const float *d_q, const float *d_X, int64_t n, int dim, float *d_out,
                          void *stream);

/* ---- graph exchange (CSR view of encode.go's layer/neighbour structure) ----
 * keys[N], vecs[N*dim], deg[L*N] (-2 absent, -1 nil map, >=0 degree),
 * adj[L*N*cap] internal ids (row-major, -1 padded), entry[L] (-1: empty
 * layer), dead[N] (1 = deleted row; nullable). */
int mhnsw_export_sizes(mhnsw_index *h, int64_t *N, int *dim, int *L, int *cap);
int mhnsw_export(mhnsw_index *h, int64_t *keys, float *vecs, int32_t *deg, int32_t *adj, int cap, int32_t *entry,
                 uint8_t *dead);
int mhnsw_import(mhnsw_index *h, int64_t N, int dim, int L, int cap, const int64_t *keys, const float *vecs,
                 const int32_t *deg, const int32_t *adj, const int32_t *entry, const uint8_t *dead);

/* ---- the reference's binary format (encode.go:128-262) and SavedGraph (encode.go:264-327) ----
 * key_kind = the Go key type K: MHNSW_KEY_INT (Go `int`, varint-encoded),
 * MHNSW_KEY_INT64 / _INT32 / _UINT64 / _UINT32 (fixed-width little-endian).
 * Export: *size receives the byte count; buf == NULL only sizes.  Nodes are
 * written in insertion order and neighbour keys ascending (Go: map order).
 * Import replaces the graph (M, Ml, EfSearch and the distance come from the
 * file) and reports the reference's errors ("unknown distance function %q",
 * "incompatible encoding version: %d", ...).  Save writes a unique temp file
 * next to path, fsyncs it and renames it over path (renameio, encode.go:320);
 * Load of a missing or empty file leaves the graph empty. */
enum { MHNSW_KEY_INT = 0, MHNSW_KEY_INT64 = 1, MHNSW_KEY_INT32 = 2, MHNSW_KEY_UINT64 = 3, MHNSW_KEY_UINT32 = 4,
       MHNSW_KEY_STRING = 5 /* Go string keys: the labels of mhnsw_strkeys_encode */ };
int mhnsw_export_go(mhnsw_index *h, int key_kind, uint8_t *buf, int64_t cap, int64_t *size);
int mhnsw_import_go(mhnsw_index *h, const uint8_t *buf, int64_t size, int key_kind);
int mhnsw_save(mhnsw_index *h, const char *path, int key_kind);
int mhnsw_load(mhnsw_index *h, const char *path, int key_kind);

/* levels randomLevel() would draw for the next n Adds (does not consume the RNG) */
int mhnsw_preview_levels(mhnsw_index *h, int64_t n, int32_t *out);

/* counters: [0] search distance evals, [1] search expansions, [2] visited-set
 * resets, [3] build distance evals, [4] build expansions, [5] dropped reverse
 * proposals, [6] searches issued, [7] exact-mode queries whose preselection
 * could not be certified and were redone by a full canonical sweep, [8] beam
 * candidates screened on the fp16 copy, [9] beam candidates evaluated in f32,
 * [10] batched-insert candidates screened on the fp16 copy, [11] batched-insert
 * rows read in f32 (search evaluations + neighbour-selection rows), [12]
 * device time of the batched insert's kernels (descent, layer searches,
 * commits) in microseconds (option "time_build" = 1: HIP events around each
 * layer's launches) */
int mhnsw_stats(const mhnsw_index *h, int64_t *out, int n);
int mhnsw_reset_stats(mhnsw_index *h);
/* device time of the last search's main kernel (HIP events on its stream) */
int mhnsw_last_kernel_ms(mhnsw_index *h, float *ms);

/* ---- Go string keys (Graph[string], graph.go:305 K = string) ----
 * The engine compares keys only by order (graph.go:137 expansion order, map
 * order stand-ins), so a string key travels as an int64 order label: every
 * string ever added gets a label and labels follow lexicographic (Go string)
 * order.  encode: n strings (blob + offs[n+1]) -> labels; with `assign` new
 * strings get labels (a new string between two adjacent labels may re-space
 * all labels: the stored keys are rewritten, so earlier labels go stale --
 * hosts convert at every call, never cache), without it unknown strings give
 * INT64_MIN.  decode: labels -> strings (blob + offs[n+1]); `need` = bytes;
 * blob == NULL or cap < need only reports `need`.  Unknown labels decode to
 * "".  Options "strkeys" / "strkey_relabels" report the table size and the
 * number of re-spacings. */
int mhnsw_strkeys_encode(mhnsw_index *h, const char *blob, const int64_t *offs, int64_t n, int assign,
                         int64_t *out);
int mhnsw_strkeys_decode(mhnsw_index *h, const int64_t *labels, int64_t n, char *blob, int64_t cap,
                         int64_t *offs, int64_t *need);

/* ---- multi-GPU: merge per-shard top-k lists (device pointers) ----
 * inputs [shards][B][k] (+ n_in [shards][B]); output best k by (dist, key). */
int mhnsw_merge_topk_device(const int64_t *keys_in, const float *dist_in, const int32_t *n_in, int shards,
                            int64_t B, int k, int64_t *out_keys, float *out_dist, int32_t *out_n, void *stream);

#ifdef __cplusplus
}
#endif
#endif
