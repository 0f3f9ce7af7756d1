/*
 * oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + timed CPU baseline).
 *
 * Plain-C99 restatement of the TFMV/hnsw hot path (see oracle.h for the list of
 * reference file:line anchors).  The reference is pure Go and cannot be built
 * in this image (no Go toolchain, no github.com/viterin/vek v0.4.2 source), so
 * parity is pinned by:
 *   - the reference's own golden tests, re-expressed as fixtures in
 *     tests/golden/ and checked by tests/test_oracle_golden.py
 *     (distance_test.go:9-31, heap/heap_test.go:17-34, graph_test.go:14-74,
 *      graph_test.go:86-133 (as a property: Go math/rand seed-0 stream is not
 *      reproducible offline), graph_test.go:253-275, graph_test.go:415-459);
 *   - vek32's arithmetic is restated as sequential fp32 (OG_ORDER_REF), which
 *     reproduces distance_test.go:12's exact bits 0x40a646e1 for sqrt(27).
 *
 * Deterministic choices where the reference is nondeterministic (documented in
 * DESIGN.md "Quirks"):
 *   - Go map iteration order (graph.go:60, 137, 187-197) -> ascending (key, id);
 *     graph.go:137-138 already sorts neighbor keys for search.
 *   - layer.entry() (graph.go:250-258, arbitrary map element) -> the first node
 *     inserted into that layer that is still present, or an injected key.
 *   - Rng.Float64() (graph.go:410) -> SplitMix64, or injected levels.
 *   - Add() of an existing key deadlocks in the reference (graph.go:438,511-513
 *     -> Delete re-locks at :844); here every Add follows BatchAdd's inline
 *     replacement (graph.go:1015-1024), including its "node not added" error
 *     (graph.go:1035-1037: Len() did not grow).
 * Keys vs nodes: the reference's maps are keyed by K, its nodes are objects.
 * A row here is one node object; several rows can carry one key (a replaced or
 * deleted node stays reachable through one-directional edges).  Every map
 * operation therefore goes by key: rows carry kid (the first row ever holding
 * the key) and neighbour sets, visited sets and layer lookups compare kids.
 *   - Search()'s "dog" test hack (graph.go:563-569, 595-619) is not restated.
 */
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* distances                                                                 */
/* ------------------------------------------------------------------------ */

/* distance.go:15-17 -> 1 - vek32.CosineSimilarity(a,b); vek's generic Go path
 * accumulates dot, |a|^2, |b|^2 sequentially in fp32. */
static float ref_cosine(const float *a, const float *b, int dim) {
    float dot = 0.f, aa = 0.f, bb = 0.f;
    for (int i = 0; i < dim; ++i) {
        float p = a[i] * b[i];
        dot = dot + p;
        p = a[i] * a[i];
        aa = aa + p;
        p = b[i] * b[i];
        bb = bb + p;
    }
    return 1.0f - dot / (sqrtf(aa) * sqrtf(bb));
}

/* distance.go:20-23 -> vek32.Distance = sqrt(sum (a-b)^2) */
static float ref_euclid(const float *a, const float *b, int dim) {
    float s = 0.f;
    for (int i = 0; i < dim; ++i) {
        float t = a[i] - b[i];
        float p = t * t;
        s = s + p;
    }
    return sqrtf(s);
}

/* canonical device order: lane(e) = (e/4) mod 64, per-lane fmaf in ascending
 * e, butterfly over offsets 32..1.  square_diff: accumulate (a-b)^2. */
float og_dev_sum(const float *a, const float *b, int dim, int square_diff) {
    float p[64];
    for (int l = 0; l < 64; ++l) p[l] = 0.f;
    for (int e = 0; e < dim; ++e) {
        int lane = (e >> 2) & 63;
        if (square_diff) {
            float t = a[e] - b[e];
            p[lane] = fmaf(t, t, p[lane]);
        } else {
            p[lane] = fmaf(a[e], b[e], p[lane]);
        }
    }
    for (int o = 32; o >= 1; o >>= 1) {
        float q[64];
        for (int l = 0; l < 64; ++l) q[l] = p[l] + p[l ^ o];
        for (int l = 0; l < 64; ++l) p[l] = q[l];
    }
    return p[0];
}

float og_dev_norm(const float *a, int dim) { return sqrtf(og_dev_sum(a, a, dim, 0)); }

static float dev_cosine_n(const float *a, const float *b, int dim, float na, float nb) {
    float dot = og_dev_sum(a, b, dim, 0);
    return 1.0f - dot / (na * nb);
}

float og_distance(int metric, int order, const float *a, const float *b, int dim) {
    if (order == OG_ORDER_REF)
        return metric == OG_COSINE ? ref_cosine(a, b, dim) : ref_euclid(a, b, dim);
    if (metric == OG_COSINE) return dev_cosine_n(a, b, dim, og_dev_norm(a, dim), og_dev_norm(b, dim));
    return sqrtf(og_dev_sum(a, b, dim, 1));
}

/* ------------------------------------------------------------------------ */
/* Go container/heap restatement (heap/heap.go + container/heap)             */
/* ------------------------------------------------------------------------ */

typedef struct {
    float d;
    int32_t id;
} cand_t;

typedef struct {
    cand_t *a;
    int n, cap;
} gheap;

static int gh_reserve(gheap *h, int cap) {
    if (cap <= h->cap) return 0;
    cand_t *na = (cand_t *)realloc(h->a, sizeof(cand_t) * (size_t)cap);
    if (!na) return -1;
    h->a = na;
    h->cap = cap;
    return 0;
}
static inline int gh_less(const gheap *h, int i, int j) { return h->a[i].d < h->a[j].d; }
static inline void gh_swap(gheap *h, int i, int j) {
    cand_t t = h->a[i];
    h->a[i] = h->a[j];
    h->a[j] = t;
}
/* container/heap up(): i := (j-1)/2 with Go truncating division */
static void gh_up(gheap *h, int j) {
    for (;;) {
        int i = (j - 1) / 2;
        if (i == j || !gh_less(h, j, i)) break;
        gh_swap(h, i, j);
        j = i;
    }
}
static int gh_down(gheap *h, int i0, int n) {
    int i = i0;
    for (;;) {
        int j1 = 2 * i + 1;
        if (j1 >= n || j1 < 0) break;
        int j = j1;
        int j2 = j1 + 1;
        if (j2 < n && gh_less(h, j2, j1)) j = j2;
        if (!gh_less(h, j, i)) break;
        gh_swap(h, i, j);
        i = j;
    }
    return i > i0;
}
/* heap.go:62 Push -> container/heap.Push */
static void gh_push(gheap *h, float d, int32_t id) {
    if (h->n >= h->cap) gh_reserve(h, h->cap ? h->cap * 2 : 16);
    h->a[h->n].d = d;
    h->a[h->n].id = id;
    h->n++;
    gh_up(h, h->n - 1);
}
/* heap.go:69 Pop -> container/heap.Pop */
static cand_t gh_pop(gheap *h) {
    int n = h->n - 1;
    gh_swap(h, 0, n);
    gh_down(h, 0, n);
    h->n--;
    return h->a[h->n];
}
/* heap.go:79 Remove -> container/heap.Remove */
static cand_t gh_remove(gheap *h, int i) {
    int n = h->n - 1;
    if (n != i) {
        gh_swap(h, i, n);
        if (!gh_down(h, i, n)) gh_up(h, i);
    }
    h->n--;
    return h->a[h->n];
}
/* heap.go:73 PopLast = Remove(Len()-1): drops the last array slot */
static cand_t gh_poplast(gheap *h) { return gh_remove(h, h->n - 1); }

int og_heap_run(const int *ops, const float *op_d, const int32_t *op_id, int nops, float *out_d,
                int32_t *out_id, int32_t *out_popped, int *n_popped) {
    gheap h = {0};
    int np = 0;
    gh_reserve(&h, 16);
    for (int i = 0; i < nops; ++i) {
        if (ops[i] == 0) {
            gh_push(&h, op_d[i], op_id[i]);
        } else if (h.n > 0) {
            cand_t c = ops[i] == 1 ? gh_pop(&h) : gh_poplast(&h);
            out_popped[np++] = c.id;
        }
    }
    for (int i = 0; i < h.n; ++i) {
        out_d[i] = h.a[i].d;
        out_id[i] = h.a[i].id;
    }
    *n_popped = np;
    int n = h.n;
    free(h.a);
    return n;
}

/* ------------------------------------------------------------------------ */
/* levels: graph.go:370-417                                                  */
/* ------------------------------------------------------------------------ */

int og_max_level(double ml, int64_t num_nodes) {
    if (ml == 0) return -1; /* "ml must be greater than 0" */
    if (num_nodes == 0) return 1;
    double l = log((double)num_nodes);
    l /= log(1.0 / ml);
    return (int)round(l) + 1; /* Go math.Round: half away from zero */
}

/* SplitMix64 -> uniform double in [0,1) with 53 random bits.  Stand-in for
 * Go's math/rand Float64 (graph.go:410), whose seed-0 stream cannot be
 * regenerated offline.  The engine's host code implements the same draw. */
double og_rng_next(uint64_t *state) {
    uint64_t z = (*state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z = z ^ (z >> 31);
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

/* ------------------------------------------------------------------------ */
/* graph                                                                     */
/* ------------------------------------------------------------------------ */

typedef struct {
    int32_t *deg; /* -2 absent, -1 nil neighbor map, >=0 count */
    int32_t *adj; /* [cap_nodes * acap] */
    int64_t count;
    int32_t entry;
} og_layer;

typedef struct {
    uint32_t *visited;
    uint32_t stamp;
    int64_t nvis;
    gheap c1, c2;
} og_scratch;

struct og_graph {
    int metric, order;
    int xw; /* beam mode: entries expanded per layer-0 step (og_set_search_expand; 1 = standard) */
    int M, M0, ef;
    double ml;
    uint64_t rng;
    int dim;
    int layers_exist;
    int64_t n, cap_nodes;
    int acap;
    int64_t *keys;
    int32_t *kid;  /* [cap_nodes] key identity: the first row that held keys[row] */
    /* [cap_nodes] the next older live row of the same key (-1 none).  A key can
     * hold live nodes in several layers at once -- a failed insert leaves its
     * node in the layers above the failing one (graph.go:1009), a later insert of
     * the key below them adds another -- each layer's map holding one of them:
     * hget(key) is the newest, prev_live links the rest (disjoint layers). */
    int32_t *prev_live;
    float *vecs;
    float *norms;
    uint8_t *dead; /* [cap_nodes] 1 = deleted (graph.go:843-864); rows stay for dangling edges */
    int nlayers;
    og_layer *layers;
    /* key -> id hash (open addressing, linear probe) */
    int64_t *hkeys;
    int32_t *hvals;
    int64_t hcap;
    /* key -> kid (every key ever added; never deleted) */
    int64_t *kkeys;
    int32_t *kvals;
    int64_t kcap, kn;
    og_scratch scr;
    int64_t stats[4];
    char err[256];
};

static int set_err(og_graph *g, int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g->err, sizeof(g->err), fmt, ap);
    va_end(ap);
    return code;
}

const char *og_last_error(og_graph *g) { return g->err; }

static uint64_t hmix(int64_t k) {
    uint64_t z = (uint64_t)k * 0x9E3779B97F4A7C15ull;
    return z ^ (z >> 29);
}

/* slot values: -1 empty, -2 tombstone (deleted key), >= 0 id */
static int32_t hget(og_graph *g, int64_t key) {
    if (!g->hcap) return -1;
    uint64_t m = (uint64_t)g->hcap - 1, h = hmix(key) & m;
    for (;;) {
        if (g->hvals[h] == -1) return -1;
        if (g->hvals[h] >= 0 && g->hkeys[h] == key) return g->hvals[h];
        h = (h + 1) & m;
    }
}

static void hdel(og_graph *g, int64_t key) {
    if (!g->hcap) return;
    uint64_t m = (uint64_t)g->hcap - 1, h = hmix(key) & m;
    for (;;) {
        if (g->hvals[h] == -1) return;
        if (g->hvals[h] >= 0 && g->hkeys[h] == key) {
            g->hvals[h] = -2;
            return;
        }
        h = (h + 1) & m;
    }
}

static int hput(og_graph *g, int64_t key, int32_t val);
static int hgrow(og_graph *g) {
    int64_t ocap = g->hcap;
    int64_t *ok = g->hkeys;
    int32_t *ov = g->hvals;
    int64_t ncap = ocap ? ocap * 2 : 1024;
    g->hkeys = (int64_t *)malloc(sizeof(int64_t) * (size_t)ncap);
    g->hvals = (int32_t *)malloc(sizeof(int32_t) * (size_t)ncap);
    if (!g->hkeys || !g->hvals) return -1;
    for (int64_t i = 0; i < ncap; ++i) g->hvals[i] = -1;
    g->hcap = ncap;
    for (int64_t i = 0; i < ocap; ++i)
        if (ov[i] >= 0) hput(g, ok[i], ov[i]);
    free(ok);
    free(ov);
    return 0;
}
static int hput(og_graph *g, int64_t key, int32_t val) {
    if ((g->n + 1) * 2 > g->hcap && hgrow(g)) return -1;
    uint64_t m = (uint64_t)g->hcap - 1, h = hmix(key) & m;
    while (g->hvals[h] >= 0 && g->hkeys[h] != key) h = (h + 1) & m;
    g->hkeys[h] = key;
    g->hvals[h] = val;
    return 0;
}

/* key -> kid, insert-or-get (kid = `row` for a key never seen) */
static int32_t kid_get(og_graph *g, int64_t key, int32_t row) {
    if ((g->kn + 1) * 2 > g->kcap) {
        int64_t ocap = g->kcap;
        int64_t *ok = g->kkeys;
        int32_t *ov = g->kvals;
        int64_t ncap = ocap ? ocap * 2 : 1024;
        g->kkeys = (int64_t *)malloc(sizeof(int64_t) * (size_t)ncap);
        g->kvals = (int32_t *)malloc(sizeof(int32_t) * (size_t)ncap);
        if (!g->kkeys || !g->kvals) return -1;
        for (int64_t i = 0; i < ncap; ++i) g->kvals[i] = -1;
        g->kcap = ncap;
        for (int64_t i = 0; i < ocap; ++i) {
            if (ov[i] < 0) continue;
            uint64_t m = (uint64_t)ncap - 1, h = hmix(ok[i]) & m;
            while (g->kvals[h] >= 0) h = (h + 1) & m;
            g->kkeys[h] = ok[i];
            g->kvals[h] = ov[i];
        }
        free(ok);
        free(ov);
    }
    uint64_t m = (uint64_t)g->kcap - 1, h = hmix(key) & m;
    while (g->kvals[h] >= 0) {
        if (g->kkeys[h] == key) return g->kvals[h];
        h = (h + 1) & m;
    }
    g->kkeys[h] = key;
    g->kvals[h] = row;
    g->kn++;
    return row;
}

og_graph *og_create(int metric, int order, int M, int M0, double ml, int ef, uint64_t seed) {
    og_graph *g = (og_graph *)calloc(1, sizeof(og_graph));
    if (!g) return NULL;
    g->metric = metric;
    g->order = order;
    g->xw = 1;
    g->M = M;
    g->M0 = M0 > 0 ? M0 : M;
    g->ml = ml;
    g->ef = ef;
    g->rng = seed;
    g->acap = (g->M0 > g->M ? g->M0 : g->M) + 1;
    if (g->acap < 2) g->acap = 2;
    return g;
}

static void free_layers(og_graph *g) {
    for (int i = 0; i < g->nlayers; ++i) {
        free(g->layers[i].deg);
        free(g->layers[i].adj);
    }
    free(g->layers);
    g->layers = NULL;
    g->nlayers = 0;
}

void og_destroy(og_graph *g) {
    if (!g) return;
    free_layers(g);
    free(g->keys);
    free(g->kid);
    free(g->prev_live);
    free(g->vecs);
    free(g->norms);
    free(g->dead);
    free(g->hkeys);
    free(g->hvals);
    free(g->kkeys);
    free(g->kvals);
    free(g->scr.visited);
    free(g->scr.c1.a);
    free(g->scr.c2.a);
    free(g);
}

/* graph.go:916-937 */
int og_validate(og_graph *g) {
    if (g->M <= 0) return set_err(g, OG_EINVAL, "M must be greater than 0, got %d", g->M);
    if (g->ml <= 0 || g->ml >= 1)
        return set_err(g, OG_EINVAL, "Ml must be between 0 and 1 (exclusive), got %f", g->ml);
    if (g->ef <= 0) return set_err(g, OG_EINVAL, "EfSearch must be greater than 0, got %d", g->ef);
    if (g->metric != OG_COSINE && g->metric != OG_EUCLIDEAN)
        return set_err(g, OG_EINVAL, "Distance function must be set");
    g->err[0] = 0;
    return OG_OK;
}

int og_set_params(og_graph *g, int M, double ml, int ef, int metric) {
    g->M = M;
    g->ml = ml;
    g->ef = ef;
    g->metric = metric;
    return OG_OK;
}

/* the engine's option "search_expand" (beam.hpp / device_search.hpp beam_layer XW) */
int og_set_search_expand(og_graph *g, int xw) {
    if (xw != 1 && xw != 2 && xw != 4) return set_err(g, OG_EINVAL, "search_expand must be 1, 2 or 4");
    g->xw = xw;
    return OG_OK;
}

int og_set_order(og_graph *g, int order) {
    if (order != OG_ORDER_REF && order != OG_ORDER_DEV) return set_err(g, OG_EINVAL, "unknown order %d", order);
    g->order = order;
    return OG_OK;
}

int64_t og_len(og_graph *g) { return g->nlayers ? g->layers[0].count : 0; }
int og_dims(og_graph *g) { return g->layers_exist ? g->dim : 0; }
int og_num_layers(og_graph *g) { return g->nlayers; }
int64_t og_layer_count(og_graph *g, int l) { return l >= 0 && l < g->nlayers ? g->layers[l].count : 0; }
int32_t og_layer_entry(og_graph *g, int l) { return l >= 0 && l < g->nlayers ? g->layers[l].entry : -1; }

void og_stats(og_graph *g, int64_t *o) { memcpy(o, g->stats, sizeof(g->stats)); }
void og_reset_stats(og_graph *g) { memset(g->stats, 0, sizeof(g->stats)); }

static int ensure_nodes(og_graph *g, int64_t need) {
    if (need <= g->cap_nodes) return 0;
    int64_t nc = g->cap_nodes ? g->cap_nodes : 64;
    while (nc < need) nc *= 2;
    int64_t *nk = (int64_t *)realloc(g->keys, sizeof(int64_t) * (size_t)nc);
    if (!nk) return -1;
    g->keys = nk;
    int32_t *nkid = (int32_t *)realloc(g->kid, sizeof(int32_t) * (size_t)nc);
    if (!nkid) return -1;
    g->kid = nkid;
    float *nv = (float *)realloc(g->vecs, sizeof(float) * (size_t)nc * (size_t)(g->dim ? g->dim : 1));
    if (!nv) return -1;
    g->vecs = nv;
    float *nn = (float *)realloc(g->norms, sizeof(float) * (size_t)nc);
    if (!nn) return -1;
    g->norms = nn;
    uint8_t *dd = (uint8_t *)realloc(g->dead, (size_t)nc);
    if (!dd) return -1;
    for (int64_t i = g->cap_nodes; i < nc; ++i) dd[i] = 0;
    g->dead = dd;
    int32_t *pl = (int32_t *)realloc(g->prev_live, sizeof(int32_t) * (size_t)nc);
    if (!pl) return -1;
    for (int64_t i = g->cap_nodes; i < nc; ++i) pl[i] = -1;
    g->prev_live = pl;
    uint32_t *vis = (uint32_t *)realloc(g->scr.visited, sizeof(uint32_t) * (size_t)nc);
    if (!vis) return -1;
    for (int64_t i = g->cap_nodes; i < nc; ++i) vis[i] = 0;
    g->scr.visited = vis;
    for (int l = 0; l < g->nlayers; ++l) {
        og_layer *L = &g->layers[l];
        int32_t *d = (int32_t *)realloc(L->deg, sizeof(int32_t) * (size_t)nc);
        int32_t *a = (int32_t *)realloc(L->adj, sizeof(int32_t) * (size_t)nc * (size_t)g->acap);
        if (!d || !a) return -1;
        for (int64_t i = g->cap_nodes; i < nc; ++i) d[i] = -2;
        L->deg = d;
        L->adj = a;
    }
    g->cap_nodes = nc;
    return 0;
}

static int add_layer(og_graph *g) {
    og_layer *nl = (og_layer *)realloc(g->layers, sizeof(og_layer) * (size_t)(g->nlayers + 1));
    if (!nl) return -1;
    g->layers = nl;
    og_layer *L = &g->layers[g->nlayers];
    L->count = 0;
    L->entry = -1;
    int64_t c = g->cap_nodes ? g->cap_nodes : 1;
    L->deg = (int32_t *)malloc(sizeof(int32_t) * (size_t)c);
    L->adj = (int32_t *)malloc(sizeof(int32_t) * (size_t)c * (size_t)g->acap);
    if (!L->deg || !L->adj) return -1;
    for (int64_t i = 0; i < c; ++i) L->deg[i] = -2;
    g->nlayers++;
    return 0;
}

/* adjacency capacity must hold M+1 (addNeighbor overflows by one, graph.go:50) */
static int ensure_acap(og_graph *g, int need) {
    if (need <= g->acap) return 0;
    for (int l = 0; l < g->nlayers; ++l) {
        og_layer *L = &g->layers[l];
        int32_t *a = (int32_t *)malloc(sizeof(int32_t) * (size_t)(g->cap_nodes ? g->cap_nodes : 1) * (size_t)need);
        if (!a) return -1;
        for (int64_t i = 0; i < g->cap_nodes; ++i)
            for (int j = 0; j < L->deg[i] && L->deg[i] > 0; ++j) a[i * need + j] = L->adj[i * g->acap + j];
        free(L->adj);
        L->adj = a;
    }
    g->acap = need;
    return 0;
}

static inline uint32_t next_stamp(og_scratch *s, int64_t n) {
    if (++s->stamp == 0) {
        memset(s->visited, 0, sizeof(uint32_t) * (size_t)n);
        s->stamp = 1;
    }
    return s->stamp;
}

static inline const float *vec_of(const og_graph *g, int32_t id) { return g->vecs + (size_t)id * (size_t)g->dim; }

/* `layer.nodes[key]` is non-nil: present in the layer and not deleted */
static inline int member(const og_graph *g, int l, int32_t id) {
    return id >= 0 && l >= 0 && l < g->nlayers && g->layers[l].deg[id] != -2 && !g->dead[id];
}

/* `layer.nodes[*elevator]` (graph.go:497, 574): the layer's node of the row's
 * KEY -- the key's live row when it is a member of layer l, else nil.  The
 * elevator row itself may be a replaced or deleted node reached through a
 * dangling edge. */
static inline int32_t key_row_in(og_graph *g, int64_t key, int l) {
    for (int32_t r = hget(g, key); r >= 0; r = g->prev_live[r])
        if (member(g, l, r)) return r;
    return -1;
}
static inline int32_t resolve(og_graph *g, int l, int32_t row) { return key_row_in(g, g->keys[row], l); }

/* highest layer with a live node (empty top layers are skipped by Search:
 * entry() == nil -> search() == nil -> continue, graph.go:572-582) */
static int top_live_layer(const og_graph *g) {
    int top = g->nlayers - 1;
    while (top > 0 && g->layers[top].count == 0) --top;
    return top;
}

/* distance(node, target) as used by search (graph.go:112, 146) */
static inline float dist_q(const og_graph *g, int32_t id, const float *q, float qn) {
    const float *x = vec_of(g, id);
    if (g->order == OG_ORDER_REF)
        return g->metric == OG_COSINE ? ref_cosine(x, q, g->dim) : ref_euclid(x, q, g->dim);
    if (g->metric == OG_COSINE) return 1.0f - og_dev_sum(x, q, g->dim, 0) / (g->norms[id] * qn);
    return sqrtf(og_dev_sum(x, q, g->dim, 1));
}

/* dist(a.Value, b.Value) between stored nodes with an explicit metric
 * (graph.go:64 uses g.Distance; graph.go:204 hard-codes CosineDistance) */
static inline float dist_nodes(const og_graph *g, int32_t a, int32_t b, int metric) {
    const float *x = vec_of(g, a), *y = vec_of(g, b);
    if (g->order == OG_ORDER_REF)
        return metric == OG_COSINE ? ref_cosine(x, y, g->dim) : ref_euclid(x, y, g->dim);
    if (metric == OG_COSINE) return 1.0f - og_dev_sum(x, y, g->dim, 0) / (g->norms[a] * g->norms[b]);
    return sqrtf(og_dev_sum(x, y, g->dim, 1));
}

/* neighbor list in Go-map-iteration stand-in order: ascending (key, id) */
static const og_graph *g_sort_ctx;
static int cmp_by_key(const void *pa, const void *pb) {
    int32_t a = *(const int32_t *)pa, b = *(const int32_t *)pb;
    int64_t ka = g_sort_ctx->keys[a], kb = g_sort_ctx->keys[b];
    if (ka != kb) return ka < kb ? -1 : 1;
    return a < b ? -1 : (a > b);
}
static int sorted_neighbors(const og_graph *g, const og_layer *L, int32_t n, int32_t *out) {
    int d = L->deg[n];
    if (d <= 0) return d < 0 ? 0 : 0;
    memcpy(out, L->adj + (size_t)n * g->acap, sizeof(int32_t) * (size_t)d);
    g_sort_ctx = g;
    qsort(out, (size_t)d, sizeof(int32_t), cmp_by_key);
    return d;
}

/* graph.go:94-170 layerNode.search (compat semantics, heap quirks Q1-Q4) */
static int compat_layer_search(og_graph *g, og_scratch *s, int layer, int32_t entry, int k, int ef,
                               const float *q, float qn, int32_t *oid, float *od, int64_t *nd, int64_t *nx) {
    if (entry < 0 || layer < 0 || layer >= g->nlayers) return 0;
    og_layer *L = &g->layers[layer];
    gheap *cand = &s->c1, *res = &s->c2;
    cand->n = 0;
    res->n = 0;
    gh_reserve(cand, ef + 2);
    gh_reserve(res, k + 2);
    int32_t *nb = (int32_t *)malloc(sizeof(int32_t) * (size_t)g->acap);
    uint32_t st = next_stamp(s, g->cap_nodes);

    gh_push(cand, dist_q(g, entry, q, qn), entry); /* graph.go:109-114 */
    (*nd)++;
    gh_push(res, cand->a[0].d, cand->a[0].id); /* graph.go:122 result.Push(candidates.Min()) */
    s->visited[g->kid[entry]] = st;             /* graph.go:123 visited[n.Key] */

    while (cand->n > 0) {
        cand_t cur = gh_pop(cand); /* graph.go:127 */
        int improved = 0;
        if (L->deg[cur.id] < 0) continue; /* graph.go:131-133: nil neighbor map */
        (*nx)++;
        int d = sorted_neighbors(g, L, cur.id, nb); /* graph.go:137-138 */
        for (int j = 0; j < d; ++j) {
            int32_t v = nb[j];
            if (s->visited[g->kid[v]] == st) continue; /* graph.go:141-143 (by key) */
            s->visited[g->kid[v]] = st;
            float dist = dist_q(g, v, q, qn); /* graph.go:146 */
            (*nd)++;
            improved = improved || (res->n > 0 && dist < res->a[0].d); /* graph.go:147 */
            if (res->n < k) {
                gh_push(res, dist, v);
            } else if (dist < res->a[res->n - 1].d) { /* Max() = last slot */
                gh_poplast(res);
                gh_push(res, dist, v);
            }
            gh_push(cand, dist, v); /* graph.go:155-159 */
            if (cand->n > ef) gh_poplast(cand);
        }
        if (!improved && res->n >= k) break; /* graph.go:164-166 */
    }
    free(nb);
    for (int i = 0; i < res->n; ++i) {
        oid[i] = res->a[i].id;
        od[i] = res->a[i].d;
    }
    return res->n; /* heap order, graph.go:169 */
}

int og_layer_search_compat(og_graph *g, int layer, int32_t entry_id, int k, int ef, const float *q,
                           int32_t *out_ids, float *out_d) {
    float qn = og_dev_norm(q, g->dim);
    return compat_layer_search(g, &g->scr, layer, entry_id, k, ef, q, qn, out_ids, out_d, &g->stats[0],
                               &g->stats[1]);
}

/* ---- sorted-list beam search (standard HNSW Alg. 2; precedent
 *      parquet/graph.go:924-1076, arrow/graph.go:576-659) ----
 * List of <= ef entries sorted by (dist, id); an entry is inserted iff the list
 * has room or (d,id) < last; terminate when every entry is expanded.  NaN
 * distances are never inserted.  Equivalent to the candidate/result two-heap
 * formulation with the stop rule cand.min > result.max && |result| >= ef. */
typedef struct {
    float d;
    int32_t id;
    int exp;
} bentry;

static inline int blt(float d1, int32_t i1, float d2, int32_t i2) { return d1 < d2 || (d1 == d2 && i1 < i2); }

static int beam_insert(bentry *lst, int *n, int ef, float d, int32_t id) {
    if (d != d) return 0;
    if (*n == ef && !blt(d, id, lst[ef - 1].d, lst[ef - 1].id)) return 0;
    for (int i = 0; i < *n; ++i)
        if (lst[i].id == id) return 0;
    int p = 0;
    while (p < *n && blt(lst[p].d, lst[p].id, d, id)) ++p;
    int last = *n < ef ? *n : ef - 1;
    for (int i = last; i > p; --i) lst[i] = lst[i - 1];
    lst[p].d = d;
    lst[p].id = id;
    lst[p].exp = 0;
    if (*n < ef) (*n)++;
    return 1;
}

/* xw: entries expanded per step.  1 is the standard search above.  xw > 1 (the
 * engine's "search_expand" / "build_expand", device_search.hpp beam_layer XW):
 * the xw first unexpanded entries of the list are all marked expanded, then
 * their rows' unvisited neighbours are scored and inserted, row by row.  The
 * list after a step is the best ef of its entries and the step's candidates
 * whatever the insertion order, so the engine may score the step's candidates
 * in any order and batching. */
static int beam_layer_search(og_graph *g, og_scratch *s, int layer, int32_t entry, int ef, const float *q,
                             float qn, bentry *lst, int64_t *nd, int64_t *nx, int xw) {
    if (entry < 0 || layer < 0 || layer >= g->nlayers) return 0;
    og_layer *L = &g->layers[layer];
    uint32_t st = next_stamp(s, g->cap_nodes);
    int n = 0;
    s->visited[entry] = st;
    beam_insert(lst, &n, ef, dist_q(g, entry, q, qn), entry);
    (*nd)++;
    if (xw < 1) xw = 1;
    if (xw > 4) xw = 4;
    for (;;) {
        int32_t cur[4];
        int nc = 0;
        for (int i = 0; i < n && nc < xw; ++i)
            if (!lst[i].exp) {
                lst[i].exp = 1;
                cur[nc++] = lst[i].id;
            }
        if (nc == 0) break;
        for (int w = 0; w < nc; ++w) {
            int deg = L->deg[cur[w]];
            (*nx)++;
            if (deg <= 0) continue;
            const int32_t *nb = L->adj + (size_t)cur[w] * g->acap;
            for (int j = 0; j < deg; ++j) {
                int32_t v = nb[j];
                if (v < 0 || s->visited[v] == st) continue;
                s->visited[v] = st;
                float d = dist_q(g, v, q, qn);
                (*nd)++;
                beam_insert(lst, &n, ef, d, v);
            }
        }
    }
    return n;
}

/* ---- graph.go:172-219 replenish, graph.go:41-81 addNeighbor ---- */
/* delete(n.neighbors, v.Key): the entry of v's key, whichever row it holds */
static void list_remove(const og_graph *g, og_layer *L, int32_t n, int32_t v) {
    const int acap = g->acap;
    int d = L->deg[n];
    int32_t *a = L->adj + (size_t)n * acap;
    for (int j = 0; j < d; ++j)
        if (g->kid[a[j]] == g->kid[v]) {
            a[j] = a[d - 1];
            L->deg[n] = d - 1;
            return;
        }
}

static void add_neighbor(og_graph *g, int layer, int32_t n, int32_t nw, int m, int metric);

static void replenish(og_graph *g, int layer, int32_t n, int m) {
    og_layer *L = &g->layers[layer];
    int dn = L->deg[n] < 0 ? 0 : L->deg[n];
    if (dn >= m) return; /* graph.go:173-175 (len(nil map) == 0) */
    og_scratch *s = &g->scr;
    uint32_t st = next_stamp(s, g->cap_nodes);
    s->visited[g->kid[n]] = st; /* graph.go:184 visited[n.Key] */
    int32_t *mine = (int32_t *)malloc(sizeof(int32_t) * (size_t)g->acap);
    int32_t *theirs = (int32_t *)malloc(sizeof(int32_t) * (size_t)g->acap);
    int nm = sorted_neighbors(g, L, n, mine);
    for (int j = 0; j < nm; ++j) s->visited[g->kid[mine[j]]] = st; /* graph.go:187-189 */
    gheap cand = {0};
    gh_reserve(&cand, 2 * m + 2);
    for (int j = 0; j < nm; ++j) { /* graph.go:192-210 */
        int32_t nb = mine[j];
        if (L->deg[nb] < 0) continue;
        int nt = sorted_neighbors(g, L, nb, theirs);
        for (int t = 0; t < nt; ++t) {
            int32_t c = theirs[t];
            if (s->visited[g->kid[c]] == st) continue; /* graph.go:198 visited[k] */
            s->visited[g->kid[c]] = st;
            float d = dist_nodes(g, c, n, OG_COSINE); /* graph.go:204 hard-coded cosine */
            g->stats[2]++;
            gh_push(&cand, d, c);
        }
    }
    free(mine);
    free(theirs);
    /* graph.go:213-218: no eviction can happen here (len < m before each add) */
    while (cand.n > 0 && (L->deg[n] < 0 ? 0 : L->deg[n]) < m) {
        cand_t best = gh_pop(&cand);
        add_neighbor(g, layer, n, best.id, m, OG_COSINE);
    }
    free(cand.a);
}

static void add_neighbor(og_graph *g, int layer, int32_t n, int32_t nw, int m, int metric) {
    og_layer *L = &g->layers[layer];
    if (n < 0 || nw < 0) return;
    if (L->deg[n] < 0) L->deg[n] = 0; /* graph.go:46-48 */
    int32_t *a = L->adj + (size_t)n * g->acap;
    int d = L->deg[n];
    int present = 0;
    for (int j = 0; j < d; ++j)
        if (g->kid[a[j]] == g->kid[nw]) { /* graph.go:50 n.neighbors[newNode.Key] = newNode: */
            a[j] = nw;                     /* the key's entry is overwritten */
            present = 1;
        }
    if (!present) {
        a[d] = nw;
        L->deg[n] = ++d;
    }
    if (d <= m) return; /* graph.go:51-53 */
    int32_t *nb = (int32_t *)malloc(sizeof(int32_t) * (size_t)g->acap);
    int nn = sorted_neighbors(g, L, n, nb);
    float worst_d = -INFINITY;
    int32_t worst = -1;
    for (int j = 0; j < nn; ++j) { /* graph.go:60-71 */
        float dd = dist_nodes(g, nb[j], n, metric);
        g->stats[2]++;
        if (dd > worst_d || worst < 0) {
            worst_d = dd;
            worst = nb[j];
        }
    }
    free(nb);
    if (worst >= 0) { /* graph.go:73-80 */
        list_remove(g, L, n, worst);
        if (L->deg[worst] >= 0) list_remove(g, L, worst, n);
        replenish(g, layer, worst, m);
    }
}

int og_random_level(og_graph *g) {
    int max = 1;
    if (g->layers_exist) {
        if (g->ml == 0) return -1;
        max = og_max_level(g->ml, og_len(g)); /* graph.go:400 */
    }
    for (int level = 0; level < max; ++level) {
        double r = og_rng_next(&g->rng);
        if (r > g->ml) return level; /* graph.go:410-413 */
    }
    return max;
}

/* levels the next n Adds would draw (graph.go:388-417 with the layer-0 size
 * growing by one per insert); does not consume the RNG */
int og_preview_levels(og_graph *g, int64_t n, int32_t *out) {
    uint64_t s = g->rng;
    int le = g->layers_exist;
    int64_t cnt = og_len(g);
    for (int64_t i = 0; i < n; ++i) {
        int max = 1;
        if (le) max = og_max_level(g->ml, cnt + i);
        int lv = max;
        for (int level = 0; level < max; ++level) {
            if (og_rng_next(&s) > g->ml) {
                lv = level;
                break;
            }
        }
        out[i] = lv;
        le = 1;
    }
    return OG_OK;
}

static void isolate(og_graph *g, int l, int32_t n, int m);

/* graph.go:1015-1024: BatchAdd found the key in layer i0 (after that layer's
 * search): every layer holding the key -- the key's old nodes (one per layer,
 * from one or several rows), and the new node's own upper row A in the layers
 * above i0 -- deletes it and isolates it, in layer order.  The rows stay behind
 * their one-directional edges, like Delete's. */
static void replace_sweep(og_graph *g, int64_t key, int32_t ida, int32_t idb) {
    int nl = g->nlayers > 0 ? g->nlayers : 1;
    int32_t *rows = (int32_t *)malloc(sizeof(int32_t) * (size_t)nl);
    for (int l = 0; l < g->nlayers; ++l) {
        rows[l] = key_row_in(g, key, l);
        if (rows[l] < 0 && ida >= 0 && g->layers[l].deg[ida] != -2) rows[l] = ida;
    }
    for (int32_t r = hget(g, key); r >= 0; r = g->prev_live[r]) g->dead[r] = 1;
    if (ida >= 0) g->dead[ida] = 1;
    for (int l = 0; l < g->nlayers; ++l) {
        if (rows[l] < 0) continue;
        g->layers[l].count--; /* delete(l.nodes, key) */
        isolate(g, l, rows[l], g->M);
    }
    free(rows);
    hput(g, key, idb);
    g->prev_live[idb] = -1;
}

static void fix_entries(og_graph *g);

/* graph.go:942-1042 Graph.BatchAdd (sequential, compat; Add is the same walk,
 * graph.go:437-531, minus its deadlock on a present key) */
int og_add(og_graph *g, const int64_t *keys, const float *vecs, int64_t n, int dim, const int32_t *levels) {
    int rc = og_validate(g);
    if (rc) return rc;
    if (ensure_acap(g, (g->M > g->M0 ? g->M : g->M0) + 1)) return set_err(g, OG_ENOMEM, "out of memory");
    for (int64_t i = 0; i < n; ++i) {
        int64_t key = keys[i];
        const float *vec = vecs + (size_t)i * (size_t)dim;
        if (g->layers_exist && g->dim != dim) /* graph.go:955-960 */
            return set_err(g, OG_EDIM, "embedding dimension mismatch: %d != %d", g->dim, dim);
        if (!g->layers_exist) g->dim = dim;
        int level = levels ? levels[i] : og_random_level(g); /* graph.go:962 */
        if (level < 0) return set_err(g, OG_EINVAL, "invalid level: %d", level);
        if (ensure_nodes(g, g->n + 2)) return set_err(g, OG_ENOMEM, "out of memory");
        while (level >= g->nlayers) /* graph.go:967-969 */
            if (add_layer(g)) return set_err(g, OG_ENOMEM, "out of memory");
        g->layers_exist = 1;
        /* a present key: the first layer (from the top) at or below the insert
         * level whose map holds it is where the replacement happens; Len() then
         * stays put -- "node not added" -- only when layer 0 held it */
        int32_t head = hget(g, key);
        int i0 = -1;
        for (int l = level; head >= 0 && l >= 0; --l)
            if (key_row_in(g, key, l) >= 0) {
                i0 = l;
                break;
            }
        const int in0 = head >= 0 && key_row_in(g, key, 0) >= 0;
        /* rows: the new node's layers above i0 (deleted again by the sweep) get a
         * row of their own, A; B holds it from i0 down */
        int need_a = 0;
        for (int l = g->nlayers - 1; i0 >= 0 && l > i0; --l) need_a |= g->layers[l].count == 0 || l <= level;
        int32_t ida = -1, idb;
        if (need_a) ida = (int32_t)g->n++;
        idb = (int32_t)g->n++;
        int32_t kid = kid_get(g, key, ida >= 0 ? ida : idb);
        if (kid < 0) return set_err(g, OG_ENOMEM, "out of memory");
        for (int32_t id = ida >= 0 ? ida : idb; id <= idb; ++id) {
            g->keys[id] = key;
            g->kid[id] = kid;
            memcpy(g->vecs + (size_t)id * dim, vec, sizeof(float) * (size_t)dim);
            g->norms[id] = og_dev_norm(vec, dim);
        }
        if (i0 < 0) { /* a fresh node: the key's newest live row (older ones stay in their layers) */
            if (hput(g, key, idb)) return set_err(g, OG_ENOMEM, "out of memory");
            g->prev_live[idb] = head;
        }
        float qn = g->norms[idb];
        int32_t elevator = -1;
        int32_t *nbh = (int32_t *)malloc(sizeof(int32_t) * (size_t)(g->M + 2));
        float *nbd = (float *)malloc(sizeof(float) * (size_t)(g->M + 2));
        for (int l = g->nlayers - 1; l >= 0; --l) { /* graph.go:980 */
            og_layer *L = &g->layers[l];
            const int32_t id = l > i0 && ida >= 0 ? ida : idb;
            if (L->count == 0) { /* graph.go:990-993 */
                L->deg[id] = -1;
                L->count = 1;
                L->entry = id;
                continue;
            }
            /* graph.go:997-1003: layer.nodes[*elevator] is nil once that key has
             * no node in this layer -> search(nil) -> error below */
            int32_t sp = elevator >= 0 ? resolve(g, l, elevator) : L->entry;
            int cnt = compat_layer_search(g, &g->scr, l, sp, g->M, g->ef, vec, qn, nbh, nbd, &g->stats[2],
                                          &g->stats[3]); /* graph.go:1005 */
            if (cnt == 0) {
                free(nbh);
                free(nbd);
                /* graph.go:1009 returns here: the node keeps the layers above */
                int any_b = 0, any_a = 0;
                for (int l2 = 0; l2 < g->nlayers; ++l2) {
                    any_b |= g->layers[l2].deg[idb] != -2;
                    any_a |= ida >= 0 && g->layers[l2].deg[ida] != -2;
                }
                if (i0 < 0 && !any_b) { /* in none of them: the key is as before */
                    if (head >= 0)
                        hput(g, key, head);
                    else
                        hdel(g, key);
                } else if (i0 >= 0 && l >= i0) { /* before the sweep: the new node joins the key's rows */
                    const int32_t placed = any_a ? ida : any_b ? idb : -1;
                    if (placed >= 0) {
                        hput(g, key, placed);
                        g->prev_live[placed] = head;
                    }
                }
                fix_entries(g);
                return set_err(g, OG_EINTERNAL, "no nodes found in neighborhood search");
            }
            elevator = nbh[0]; /* graph.go:1013 */
            if (level >= l) {  /* graph.go:1015-1032 */
                if (l == i0) replace_sweep(g, key, ida, idb);
                L->deg[id] = -1;
                L->count++;
                for (int j = 0; j < cnt; ++j) {
                    add_neighbor(g, l, nbh[j], id, g->M, g->metric);
                    add_neighbor(g, l, id, nbh[j], g->M, g->metric);
                }
            }
        }
        free(nbh);
        free(nbd);
        if (i0 >= 0 && in0) { /* graph.go:1035-1037: Len() did not grow -> the batch stops here */
            fix_entries(g);
            return set_err(g, OG_EINTERNAL, "node not added");
        }
        if (i0 >= 0) fix_entries(g); /* the sweep may have emptied an entry; the walk goes on */
    }
    return OG_OK;
}

/* ---- graph.go:843-895 Delete / BatchDelete ----------------------------- */

/* graph.go:221-235 isolate: for each neighbour (ascending key = the map-order
 * stand-in) drop the backlink and replenish the neighbour.  The deleted
 * node's own map is left intact (the reference keeps the layerNode alive
 * behind one-directional edges), and replenish may even re-link it. */
static void isolate(og_graph *g, int l, int32_t n, int m) {
    og_layer *L = &g->layers[l];
    if (L->deg[n] < 0) return; /* nil neighbor map */
    int32_t *nb = (int32_t *)malloc(sizeof(int32_t) * (size_t)g->acap);
    int d = sorted_neighbors(g, L, n, nb);
    for (int j = 0; j < d; ++j) {
        int32_t x = nb[j];
        if (L->deg[x] < 0) continue; /* neighbor.neighbors == nil */
        list_remove(g, L, x, n); /* graph.go:232 delete(neighbor.neighbors, n.Key) */
        replenish(g, l, x, m);
    }
    free(nb);
}

typedef struct {
    float d;
    int32_t id;
} rp_t;
static int rp_cmp(const void *a, const void *b) {
    const rp_t *x = (const rp_t *)a, *y = (const rp_t *)b;
    if (blt(x->d, x->id, y->d, y->id)) return -1;
    if (blt(y->d, y->id, x->d, x->id)) return 1;
    return 0;
}

/* Batched-graph repair (engine semantics, k_delete_repair): every live row of
 * layer l that points at a deleted node is rebuilt from its live neighbours
 * plus the neighbours of its deleted neighbours (gather order: row order,
 * capped at OG_REPAIR_POOL), ranked by (distance, id) and selected like the
 * batched insert (HNSW diversity heuristic, optional keep-pruned fill).  Rows
 * of deleted nodes are read, never written, so rows are independent. */
#define OG_REPAIR_POOL 256
static void repair_layer(og_graph *g, int l, int mcap, int heuristic, int keep_pruned) {
    og_layer *L = &g->layers[l];
    rp_t *pool = (rp_t *)malloc(sizeof(rp_t) * OG_REPAIR_POOL);
    int32_t *sel = (int32_t *)malloc(sizeof(int32_t) * (size_t)g->acap);
    for (int64_t v = 0; v < g->n; ++v) {
        int d = L->deg[v];
        if (g->dead[v] || d <= 0) continue;
        const int32_t *row = L->adj + (size_t)v * g->acap;
        int hit = 0;
        for (int j = 0; j < d; ++j) hit |= g->dead[row[j]];
        if (!hit) continue;
        int np = 0;
        for (int j = 0; j < d && np < OG_REPAIR_POOL; ++j)
            if (!g->dead[row[j]]) pool[np++].id = row[j];
        for (int j = 0; j < d; ++j) {
            int32_t x = row[j];
            if (!g->dead[x] || L->deg[x] <= 0) continue;
            const int32_t *xr = L->adj + (size_t)x * g->acap;
            for (int t = 0; t < L->deg[x] && np < OG_REPAIR_POOL; ++t)
                if (xr[t] != (int32_t)v && !g->dead[xr[t]]) pool[np++].id = xr[t];
        }
        for (int i = 0; i < np; ++i) {
            float dd = dist_nodes(g, pool[i].id, (int32_t)v, g->metric);
            pool[i].d = dd != dd ? INFINITY : dd; /* NaN (zero vectors) ranks last */
            g->stats[2]++;
        }
        qsort(pool, (size_t)np, sizeof(rp_t), rp_cmp);
        int ns = 0;
        for (int i = 0; i < np && ns < mcap; ++i) {
            if (i > 0 && pool[i].id == pool[i - 1].id) continue;
            int good = 1;
            if (heuristic && ns > 0)
                for (int s2 = 0; s2 < ns; ++s2) {
                    g->stats[2]++;
                    if (dist_nodes(g, sel[s2], pool[i].id, g->metric) < pool[i].d) good = 0;
                }
            if (good) sel[ns++] = pool[i].id;
        }
        if (keep_pruned)
            for (int i = 0; i < np && ns < mcap; ++i) {
                if (i > 0 && pool[i].id == pool[i - 1].id) continue;
                int have = 0;
                for (int s2 = 0; s2 < ns; ++s2) have |= sel[s2] == pool[i].id;
                if (!have) sel[ns++] = pool[i].id;
            }
        int32_t *w = L->adj + (size_t)v * g->acap;
        for (int i = 0; i < ns; ++i) w[i] = sel[i];
        L->deg[v] = ns;
    }
    free(pool);
    free(sel);
}

/* lowest-id live member, the deterministic stand-in for entry() (graph.go:250-258) */
static void fix_entries(og_graph *g) {
    for (int l = 0; l < g->nlayers; ++l) {
        og_layer *L = &g->layers[l];
        if (member(g, l, L->entry)) continue;
        L->entry = -1;
        for (int64_t i = 0; i < g->n; ++i)
            if (member(g, l, (int32_t)i)) {
                L->entry = (int32_t)i;
                break;
            }
    }
}

int og_delete(og_graph *g, const int64_t *keys, int64_t n, int mode, int heuristic, int keep_pruned, uint8_t *out) {
    int any = 0;
    int32_t *rows = (int32_t *)malloc(sizeof(int32_t) * (size_t)(g->nlayers > 0 ? g->nlayers : 1));
    for (int64_t i = 0; i < n; ++i) {
        int32_t head = hget(g, keys[i]);
        out[i] = 0;
        if (head < 0 || g->nlayers == 0) continue;
        /* layers[l].nodes[key] of every layer (the key's rows hold disjoint layers) */
        for (int l = 0; l < g->nlayers; ++l) rows[l] = key_row_in(g, keys[i], l);
        for (int32_t r = head; r >= 0; r = g->prev_live[r]) g->dead[r] = 1;
        hdel(g, keys[i]);
        any = 1;
        for (int l = 0; l < g->nlayers; ++l) { /* graph.go:852-861 */
            if (rows[l] < 0) continue;
            g->layers[l].count--;
            out[i] = 1;
            if (mode == 0) isolate(g, l, rows[l], g->M); /* cap M on every layer (Q13) */
        }
    }
    free(rows);
    if (any && mode == 1)
        for (int l = 0; l < g->nlayers; ++l) repair_layer(g, l, l == 0 ? g->M0 : g->M, heuristic, keep_pruned);
    if (any) fix_entries(g);
    return OG_OK;
}

/* one query of Graph.Search (graph.go:534-625) / BatchSearch loop body
 * (graph.go:1076-1106), compat or beam, or exact brute force */
typedef struct {
    int32_t *ids;
    float *ds;
    bentry *lst;
    int64_t st[2];
} qbuf;

static int search_one(og_graph *g, og_scratch *s, qbuf *qb, const float *q, int dim, int k, int mode, int ef,
                      int32_t entry, int64_t *ok, float *odd, int32_t *oid) {
    float qn = og_dev_norm(q, dim);
    int top = top_live_layer(g);
    if (mode == OG_MODE_EXACT) {
        int n = 0;
        og_layer *L0 = &g->layers[0];
        for (int32_t v = 0; v < (int32_t)g->n; ++v) {
            if (L0->deg[v] == -2 || g->dead[v]) continue;
            beam_insert(qb->lst, &n, k, dist_q(g, v, q, qn), v);
            qb->st[0]++;
        }
        for (int i = 0; i < n; ++i) {
            ok[i] = g->keys[qb->lst[i].id];
            odd[i] = qb->lst[i].d;
            if (oid) oid[i] = qb->lst[i].id;
        }
        return n;
    }
    if (mode == OG_MODE_COMPAT) {
        int32_t elevator = -1;
        for (int l = top; l >= 0; --l) { /* graph.go:571-622 */
            /* searchPoint = layers[l].entry() (nil when empty), or
             * layers[l].nodes[*elevator] (nil when that node was deleted) */
            int32_t p = elevator >= 0 ? resolve(g, l, elevator)
                                      : (l == top ? entry : (g->layers[l].count > 0 ? g->layers[l].entry : -1));
            if (l > 0) {
                int c = compat_layer_search(g, s, l, p, 1, ef, q, qn, qb->ids, qb->ds, &qb->st[0], &qb->st[1]);
                if (c == 0) continue;
                elevator = qb->ids[0];
                continue;
            }
            int c = compat_layer_search(g, s, 0, p, k, ef, q, qn, qb->ids, qb->ds, &qb->st[0], &qb->st[1]);
            for (int i = 0; i < c; ++i) {
                ok[i] = g->keys[qb->ids[i]];
                odd[i] = qb->ds[i];
                if (oid) oid[i] = qb->ids[i];
            }
            return c;
        }
        return 0;
    }
    int efl = ef > k ? ef : k;
    int32_t p = entry;
    for (int l = top; l >= 1; --l) {
        if (g->layers[l].deg[p] == -2) p = g->layers[l].entry; /* not a member of this layer */
        int c = beam_layer_search(g, s, l, p, 1, q, qn, qb->lst, &qb->st[0], &qb->st[1], 1);
        if (c > 0) p = qb->lst[0].id;
    }
    if (g->layers[0].deg[p] == -2) p = g->layers[0].entry;
    int c = beam_layer_search(g, s, 0, p, efl, q, qn, qb->lst, &qb->st[0], &qb->st[1], g->xw);
    /* deleted rows still route the search (their edges stay) but are not returned */
    int nout = 0;
    for (int i = 0; i < c && nout < k; ++i) {
        if (g->dead[qb->lst[i].id]) continue;
        ok[nout] = g->keys[qb->lst[i].id];
        odd[nout] = qb->lst[i].d;
        if (oid) oid[nout] = qb->lst[i].id;
        ++nout;
    }
    return nout;
}

static int search_prologue(og_graph *g, int64_t B, int dim, int k, const int64_t *entry_key, int32_t *entry,
                           int32_t *out_n) {
    int rc = og_validate(g);
    if (rc) return rc;
    if (k <= 0) return set_err(g, OG_EK, "k must be greater than 0, got %d", k);
    if (g->layers_exist && g->dim != dim) {
        if (B == 1) return set_err(g, OG_EDIM, "embedding dimension mismatch: %d != %d", g->dim, dim);
        return set_err(g, OG_EDIM, "embedding dimension mismatch for query %d: %d != %d", 0, g->dim, dim);
    }
    for (int64_t b = 0; b < B; ++b) out_n[b] = 0;
    *entry = -1;
    if (!g->layers_exist || og_len(g) == 0) return 1; /* graph.go:554-556: nil, nil */
    int top = top_live_layer(g);
    *entry = g->layers[top].entry;
    if (entry_key) {
        int32_t e = key_row_in(g, *entry_key, top);
        if (e < 0)
            return set_err(g, OG_EINVAL, "entry key %lld not in top layer", (long long)*entry_key);
        *entry = e;
    }
    return 0;
}

static int qbuf_init(qbuf *qb, int cap) {
    qb->ids = (int32_t *)malloc(sizeof(int32_t) * (size_t)(cap + 2));
    qb->ds = (float *)malloc(sizeof(float) * (size_t)(cap + 2));
    qb->lst = (bentry *)malloc(sizeof(bentry) * (size_t)(cap + 2));
    qb->st[0] = qb->st[1] = 0;
    return (qb->ids && qb->ds && qb->lst) ? 0 : -1;
}
static void qbuf_free(qbuf *qb) {
    free(qb->ids);
    free(qb->ds);
    free(qb->lst);
}

/* graph.go:534-625 Search / graph.go:1047-1110 BatchSearch */
int og_search(og_graph *g, const float *queries, int64_t B, int dim, int k, int mode, int ef,
              const int64_t *entry_key, int64_t *out_keys, float *out_dist, int32_t *out_n) {
    int32_t entry;
    int rc = search_prologue(g, B, dim, k, entry_key, &entry, out_n);
    if (rc) return rc > 0 ? OG_OK : rc;
    if (ef <= 0) ef = g->ef;
    qbuf qb;
    if (qbuf_init(&qb, ef > k ? ef : k)) return set_err(g, OG_ENOMEM, "out of memory");
    for (int64_t b = 0; b < B; ++b)
        out_n[b] = search_one(g, &g->scr, &qb, queries + (size_t)b * dim, dim, k, mode, ef, entry,
                              out_keys + (size_t)b * k, out_dist + (size_t)b * k, NULL);
    g->stats[0] += qb.st[0];
    g->stats[1] += qb.st[1];
    qbuf_free(&qb);
    return OG_OK;
}

/* concurrent Search under the read lock (graph_benchmark_test.go:70-89
 * BenchmarkConcurrentSearch): queries split over nthreads pthreads */
typedef struct {
    og_graph *g;
    const float *q;
    int64_t b0, b1;
    int dim, k, mode, ef;
    int32_t entry;
    int64_t *ok;
    float *od;
    int32_t *on;
    int64_t st[2];
} mt_arg;

static void *mt_worker(void *p) {
    mt_arg *a = (mt_arg *)p;
    og_scratch s = {0};
    s.visited = (uint32_t *)calloc((size_t)a->g->cap_nodes, sizeof(uint32_t));
    qbuf qb;
    qbuf_init(&qb, a->ef > a->k ? a->ef : a->k);
    for (int64_t b = a->b0; b < a->b1; ++b)
        a->on[b] = search_one(a->g, &s, &qb, a->q + (size_t)b * a->dim, a->dim, a->k, a->mode, a->ef, a->entry,
                              a->ok + (size_t)b * a->k, a->od + (size_t)b * a->k, NULL);
    a->st[0] = qb.st[0];
    a->st[1] = qb.st[1];
    qbuf_free(&qb);
    free(s.visited);
    free(s.c1.a);
    free(s.c2.a);
    return NULL;
}

int og_search_mt(og_graph *g, const float *queries, int64_t B, int dim, int k, int mode, int ef,
                 const int64_t *entry_key, int64_t *out_keys, float *out_dist, int32_t *out_n, int nthreads) {
    int32_t entry;
    int rc = search_prologue(g, B, dim, k, entry_key, &entry, out_n);
    if (rc) return rc > 0 ? OG_OK : rc;
    if (ef <= 0) ef = g->ef;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    mt_arg args[256];
    int64_t per = (B + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; ++t) {
        mt_arg *a = &args[t];
        a->g = g;
        a->q = queries;
        a->b0 = t * per < B ? t * per : B;
        a->b1 = (t + 1) * per < B ? (t + 1) * per : B;
        a->dim = dim;
        a->k = k;
        a->mode = mode;
        a->ef = ef;
        a->entry = entry;
        a->ok = out_keys;
        a->od = out_dist;
        a->on = out_n;
        pthread_create(&th[t], NULL, mt_worker, a);
    }
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        g->stats[0] += args[t].st[0];
        g->stats[1] += args[t].st[1];
    }
    return OG_OK;
}

/* ---- graph.go:1116-1537 SearchWithNegative(s) / BatchSearchWithNegatives ----
 * Candidates = Search(near, max(3k, 10)) in the chosen mode; each candidate is
 * scored in float32 exactly as the reference:
 *   qd = Distance(cand, near), qs = 1 - qd
 *   total += 1 - Distance(cand, neg_j) (in order), avg = total / n
 *   qd < 0.001 -> 2.0; any Distance(cand, neg_j) < 0.1 -> qs - w*2.0;
 *   else qs - w*avg (+ 0.2 for keys 7..9 with flags & 1: the test hack Q11)
 * then ordered by descending score.  Go's slices.SortFunc is not stable, so
 * ties keep candidate order here, and NaN scores (zero vectors) go last.
 * A query with no negatives is a plain Search(near, k) (graph.go:1395-1398). */
typedef struct {
    float score;
    int pos;
} negsc_t;
static int negsc_cmp(const void *a, const void *b) {
    const negsc_t *x = (const negsc_t *)a, *y = (const negsc_t *)b;
    int xn = x->score != x->score, yn = y->score != y->score;
    if (xn != yn) return xn - yn;
    if (!xn && x->score != y->score) return x->score > y->score ? -1 : 1;
    return x->pos - y->pos;
}

int og_search_negatives(og_graph *g, const float *queries, int64_t B, int dim, const float *negatives,
                        const int32_t *neg_count, int k, float neg_weight, int mode, int ef, int flags,
                        int64_t *out_keys, float *out_score, int32_t *out_n) {
    int32_t entry;
    if (neg_weight < 0.0f || neg_weight > 1.0f)
        return set_err(g, OG_EINVAL, "negWeight must be between 0.0 and 1.0, got %f", (double)neg_weight);
    int rc = search_prologue(g, B, dim, k, NULL, &entry, out_n);
    if (rc) return rc > 0 ? OG_OK : rc;
    if (ef <= 0) ef = g->ef;
    int kx = 3 * k < 10 ? 10 : 3 * k;
    qbuf qb;
    if (qbuf_init(&qb, (ef > kx ? ef : kx) + k)) return set_err(g, OG_ENOMEM, "out of memory");
    int64_t *ck = (int64_t *)malloc(sizeof(int64_t) * (size_t)kx);
    float *cd = (float *)malloc(sizeof(float) * (size_t)kx);
    int32_t *ci = (int32_t *)malloc(sizeof(int32_t) * (size_t)kx);
    negsc_t *sc = (negsc_t *)malloc(sizeof(negsc_t) * (size_t)kx);
    const float *neg = negatives;
    for (int64_t b = 0; b < B; ++b) {
        const float *q = queries + (size_t)b * dim;
        const int nn = neg_count[b];
        int64_t *okb = out_keys + (size_t)b * k;
        float *osb = out_score + (size_t)b * k;
        if (nn == 0) { /* plain Search */
            out_n[b] = search_one(g, &g->scr, &qb, q, dim, k, mode, ef, entry, okb, osb, NULL);
            continue;
        }
        int c = search_one(g, &g->scr, &qb, q, dim, kx, mode, ef, entry, ck, cd, ci);
        for (int i = 0; i < c; ++i) {
            const float qd = cd[i];
            const float qs = 1.0f - qd;
            float total = 0.0f;
            int close = 0;
            for (int j = 0; j < nn; ++j) {
                const float *nv = neg + (size_t)j * dim;
                const float nd = dist_q(g, ci[i], nv, og_dev_norm(nv, dim));
                total += 1.0f - nd;
                if (nd < 0.1f) close = 1;
            }
            const float avg = total / (float)nn;
            float score;
            if (qd < 0.001f)
                score = 2.0f;
            else if (close)
                score = qs - neg_weight * 2.0f;
            else {
                const float boost = ((flags & 1) && ck[i] >= 7 && ck[i] <= 9) ? 0.2f : 0.0f;
                score = qs - neg_weight * avg + boost;
            }
            sc[i].score = score;
            sc[i].pos = i;
        }
        qsort(sc, (size_t)c, sizeof(negsc_t), negsc_cmp);
        const int m = c < k ? c : k;
        for (int i = 0; i < m; ++i) {
            okb[i] = ck[sc[i].pos];
            osb[i] = sc[i].score;
        }
        out_n[b] = m;
        neg += (size_t)nn * dim;
    }
    g->stats[0] += qb.st[0];
    g->stats[1] += qb.st[1];
    free(ck);
    free(cd);
    free(ci);
    free(sc);
    qbuf_free(&qb);
    return OG_OK;
}

/* ---- exchange ---- */
int og_export_sizes(og_graph *g, int64_t *N, int *dim, int *L, int *cap) {
    *N = g->n;
    *dim = g->dim;
    *L = g->nlayers;
    *cap = g->acap;
    return OG_OK;
}

int og_export(og_graph *g, int64_t *keys, float *vecs, int32_t *deg, int32_t *adj, int cap, int32_t *entry,
              uint8_t *dead) {
    if (cap < g->acap) {
        for (int l = 0; l < g->nlayers; ++l)
            for (int64_t i = 0; i < g->n; ++i)
                if (g->layers[l].deg[i] > cap) return set_err(g, OG_EINVAL, "export cap too small");
    }
    memcpy(keys, g->keys, sizeof(int64_t) * (size_t)g->n);
    memcpy(vecs, g->vecs, sizeof(float) * (size_t)g->n * (size_t)g->dim);
    if (dead) memcpy(dead, g->dead, (size_t)g->n);
    for (int l = 0; l < g->nlayers; ++l) {
        og_layer *L = &g->layers[l];
        entry[l] = L->entry;
        for (int64_t i = 0; i < g->n; ++i) {
            int d = L->deg[i];
            deg[(size_t)l * g->n + i] = d;
            int32_t *o = adj + ((size_t)l * g->n + i) * cap;
            for (int j = 0; j < cap; ++j) o[j] = (j < d) ? L->adj[(size_t)i * g->acap + j] : -1;
        }
    }
    return OG_OK;
}

int og_import(og_graph *g, int64_t N, int dim, int L, int cap, const int64_t *keys, const float *vecs,
              const int32_t *deg, const int32_t *adj, const int32_t *entry, const uint8_t *dead) {
    free_layers(g);
    free(g->keys);
    free(g->vecs);
    free(g->norms);
    free(g->dead);
    g->dead = NULL;
    free(g->scr.visited);
    free(g->hkeys);
    free(g->hvals);
    free(g->kid);
    free(g->kkeys);
    free(g->kvals);
    g->kid = NULL;
    g->kkeys = NULL;
    g->kvals = NULL;
    g->kcap = g->kn = 0;
    g->keys = NULL;
    g->vecs = NULL;
    g->norms = NULL;
    g->scr.visited = NULL;
    g->hkeys = NULL;
    g->hvals = NULL;
    g->hcap = 0;
    g->cap_nodes = 0;
    g->n = 0;
    g->dim = dim;
    int need = (g->M > g->M0 ? g->M : g->M0) + 1;
    g->acap = cap > need ? cap : need;
    if (ensure_nodes(g, N > 0 ? N : 1)) return set_err(g, OG_ENOMEM, "out of memory");
    for (int l = 0; l < L; ++l)
        if (add_layer(g)) return set_err(g, OG_ENOMEM, "out of memory");
    /* add_layer sized for cap_nodes already */
    memcpy(g->keys, keys, sizeof(int64_t) * (size_t)N);
    memcpy(g->vecs, vecs, sizeof(float) * (size_t)N * (size_t)dim);
    g->n = N;
    for (int64_t i = 0; i < N; ++i) {
        g->norms[i] = og_dev_norm(vecs + (size_t)i * dim, dim);
        g->dead[i] = dead ? dead[i] : 0;
        g->kid[i] = kid_get(g, keys[i], (int32_t)i);
        g->prev_live[i] = -1;
        if (!g->dead[i]) { /* the newest live row heads the key's chain */
            g->prev_live[i] = hget(g, keys[i]);
            hput(g, keys[i], (int32_t)i);
        }
    }
    for (int l = 0; l < L; ++l) {
        og_layer *Ly = &g->layers[l];
        Ly->count = 0;
        Ly->entry = entry[l];
        for (int64_t i = 0; i < N; ++i) {
            int d = deg[(size_t)l * N + i];
            Ly->deg[i] = d;
            if (d != -2 && !g->dead[i]) Ly->count++;
            for (int j = 0; j < d; ++j) Ly->adj[(size_t)i * g->acap + j] = adj[((size_t)l * N + i) * cap + j];
        }
    }
    g->layers_exist = L > 0;
    return OG_OK;
}
