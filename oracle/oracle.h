/*
 * oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C99) of the TFMV/hnsw hot path, used as the parity
 * checker for the HIP engine in hnsw_amd/.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library, and only as a checker
 * or as the timed CPU baseline.  The product path never links or calls it.
 *
 * Reference (read-only, Go, cannot be compiled here: no Go toolchain, no vek
 * module source):
 *   distance.go:15-23        CosineDistance / EuclideanDistance
 *   heap/heap.go:1-95        Heap wrapper over Go container/heap
 *   graph.go:41-81           layerNode.addNeighbor
 *   graph.go:94-170          layerNode.search            (compat search)
 *   graph.go:172-219         layerNode.replenish
 *   graph.go:250-258         layer.entry                 (made deterministic)
 *   graph.go:370-417         maxLevel / randomLevel      (RNG made injectable)
 *   graph.go:437-531         Graph.Add
 *   graph.go:534-625         Graph.Search
 *   graph.go:221-235, 843-895 isolate / Delete / BatchDelete
 *   graph.go:916-937         Graph.Validate
 *   graph.go:1047-1110       Graph.BatchSearch
 *   parquet/graph.go:924-1076, arrow/graph.go:576-659   beam-search precedent
 *
 * Parity pinning: see oracle.c header and tests/test_oracle_golden.py.
 */
#ifndef MHNSW_ORACLE_H
#define MHNSW_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OG_COSINE = 0, OG_EUCLIDEAN = 1 };
/* Distance summation order.
 *  OG_ORDER_REF: sequential fp32 (mul then add), the Go fallback of vek32.
 *  OG_ORDER_DEV: the engine's canonical order -- element e goes to lane
 *                (e/4) mod 64, each lane accumulates with fmaf in ascending
 *                e, then a butterfly over offsets 32,16,8,4,2,1.  Cosine uses
 *                1 - dot/(|a|*|b|) with |x| = sqrtf(canonical sum x*x). */
enum { OG_ORDER_REF = 0, OG_ORDER_DEV = 1 };
enum { OG_MODE_COMPAT = 0, OG_MODE_BEAM = 1, OG_MODE_EXACT = 2 };

/* Error classes (mirrors include/mhnsw.h). */
#define OG_OK 0
#define OG_EINVAL (-1)
#define OG_EDIM (-2)
#define OG_EK (-3)
#define OG_ENOMEM (-4)
#define OG_EUNSUPPORTED (-6)
#define OG_EINTERNAL (-7)

typedef struct og_graph og_graph;

/* ---- distances (distance.go:15-23) ---- */
float og_distance(int metric, int order, const float *a, const float *b, int dim);
float og_dev_sum(const float *a, const float *b, int dim, int square_diff);
float og_dev_norm(const float *a, int dim);

/* ---- Go container/heap restatement (heap/heap.go) on (dist,id) pairs ----
 * ops: 0=push(d,id) 1=pop 2=poplast.  Applies a sequence of ops to an
 * initially empty heap; writes the popped ids in order to out_popped and the
 * final heap array (heap order) to out_d/out_id.  Returns final length. */
int og_heap_run(const int *ops, const float *op_d, const int32_t *op_id, int nops,
                float *out_d, int32_t *out_id, int32_t *out_popped, int *n_popped);

/* ---- levels (graph.go:370-417) ---- */
int og_max_level(double ml, int64_t num_nodes);         /* -1 if ml == 0 */
double og_rng_next(uint64_t *state);                    /* SplitMix64 -> [0,1) */

/* ---- graph ---- */
og_graph *og_create(int metric, int order, int M, int M0, double ml, int ef, uint64_t seed);
void og_destroy(og_graph *g);
const char *og_last_error(og_graph *g);
int og_set_params(og_graph *g, int M, double ml, int ef, int metric);
/* switch the summation order of later distances (the norms are kept for both) */
int og_set_order(og_graph *g, int order);
/* beam mode: entries expanded per step of the layer-0 search (1 = standard, 2, 4);
 * the engine's option "search_expand" */
int og_set_search_expand(og_graph *g, int xw);
int og_validate(og_graph *g);
int64_t og_len(og_graph *g);
int og_dims(og_graph *g);
int og_num_layers(og_graph *g);
int64_t og_layer_count(og_graph *g, int layer);
int32_t og_layer_entry(og_graph *g, int layer);
/* draw the level the next Add would use (consumes RNG) */
int og_random_level(og_graph *g);
/* levels the next n Adds would draw (layer-0 size growing per insert; RNG untouched) */
int og_preview_levels(og_graph *g, int64_t n, int32_t *out);

/* Graph.Add (compat, sequential). levels may be NULL (drawn from the RNG). */
int og_add(og_graph *g, const int64_t *keys, const float *vecs, int64_t n, int dim,
           const int32_t *levels);

/* Graph.Search / BatchSearch.  mode: OG_MODE_*.  entry_key NULL => policy entry
 * (first node inserted into the top layer).  ef <= 0 => EfSearch.  Outputs are
 * B*k slots; out_n[b] = results written for query b.  For compat mode the
 * order is the reference's heap order (heap/heap.go:93-95); beam/exact modes
 * are sorted by (dist, id). */
int og_search(og_graph *g, const float *queries, int64_t B, int dim, int k, int mode,
              int ef, const int64_t *entry_key, int64_t *out_keys, float *out_dist, int32_t *out_n);
/* same, queries split over nthreads pthreads (concurrent Search, graph.go:535 RLock) */
int og_search_mt(og_graph *g, const float *queries, int64_t B, int dim, int k, int mode,
                 int ef, const int64_t *entry_key, int64_t *out_keys, float *out_dist,
                 int32_t *out_n, int nthreads);

/* SearchWithNegative(s) / BatchSearchWithNegatives (graph.go:1116-1537): the
 * negatives of query b are the next neg_count[b] rows of `negatives`; flags
 * bit 0 enables the reference's key-7..9 boost (test hack).  out_score holds
 * the combined scores (descending). */
int og_search_negatives(og_graph *g, const float *queries, int64_t B, int dim, const float *negatives,
                        const int32_t *neg_count, int k, float neg_weight, int mode, int ef, int flags,
                        int64_t *out_keys, float *out_score, int32_t *out_n);

/* layerNode.search on one layer from an explicit entry id (graph.go:94-170) */
int og_layer_search_compat(og_graph *g, int layer, int32_t entry_id, int k, int ef,
                           const float *q, int32_t *out_ids, float *out_d);

/* Graph.Delete / BatchDelete (graph.go:843-895).  mode 0: the reference's
 * isolate + replenish per key (graph.go:172-235); mode 1: the engine's
 * batched-graph repair (see oracle.c repair_layer).  out[i] = 1 if deleted. */
int og_delete(og_graph *g, const int64_t *keys, int64_t n, int mode, int heuristic, int keep_pruned,
              uint8_t *out);

/* ---- graph exchange (same format as mhnsw_export/mhnsw_import) ----
 * keys[N], vecs[N*dim], per layer: deg[N] (-2 absent, -1 nil map, >=0),
 * adj[N*cap] (internal ids), entry[L], dead[N] (nullable). */
int og_export_sizes(og_graph *g, int64_t *N, int *dim, int *L, int *cap);
int og_export(og_graph *g, int64_t *keys, float *vecs, int32_t *deg, int32_t *adj, int cap,
              int32_t *entry, uint8_t *dead);
int og_import(og_graph *g, int64_t N, int dim, int L, int cap, const int64_t *keys,
              const float *vecs, const int32_t *deg, const int32_t *adj, const int32_t *entry,
              const uint8_t *dead);

/* counters: [0]=distance evals (search), [1]=expansions (search),
 * [2]=distance evals (build), [3]=expansions (build) */
void og_stats(og_graph *g, int64_t *out4);
void og_reset_stats(og_graph *g);

#ifdef __cplusplus
}
#endif
#endif
