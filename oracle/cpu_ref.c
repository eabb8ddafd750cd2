/*
 * cpu_ref.c -- TEST INFRASTRUCTURE ONLY: a second, independent CPU restatement
 * (in C) of the Orleans dispatch hot path.  It is the bench's cpu_baseline
 * ("port") and cross-checks oracle.py bit-for-bit.  Never linked into or called
 * by libgraindispatch.
 *
 * Two modes:
 *   faithful  follows the reference data structures:
 *             - ring: linear scan from the end under one mutex
 *               (LocalGrainDirectory.CalculateTargetSilo, LocalGrainDirectory.cs:512-541)
 *             - directory: chained hash map keyed by GrainId, .NET Dictionary style
 *               (GrainDirectoryPartition.partitionData, GrainDirectoryPartition.cs:215;
 *               lookup under lock(lockable) :393)
 *             - enqueue: per-activation growable FIFO append
 *               (ActivationData.waiting.Add, ActivationData.cs:604-605)
 *   fast      binary-search ring, open-addressing table, parallel stable counting sort.
 *
 * Hash restated from JenkinsHash.cs:85-105 / UniqueKey.cs:272-293 (TypeCodeData, N0, N1).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define M32 0xFFFFFFFFu

/* ------------------------------------------------------------------ Jenkins */
#define JMIX(a, b, c)                   \
    do {                                \
        a -= b; a -= c; a ^= (c >> 13); \
        b -= c; b -= a; b ^= (a << 8);  \
        c -= a; c -= b; c ^= (b >> 13); \
        a -= b; a -= c; a ^= (c >> 12); \
        b -= c; b -= a; b ^= (a << 16); \
        c -= a; c -= b; c ^= (b >> 5);  \
        a -= b; a -= c; a ^= (c >> 3);  \
        b -= c; b -= a; b ^= (a << 10); \
        c -= a; c -= b; c ^= (b >> 15); \
    } while (0)

uint32_t cpu_jenkins_u64x3(uint64_t u1, uint64_t u2, uint64_t u3) {
    uint32_t a = 0x9e3779b9u, b = a, c = 0;
    a += (uint32_t)u1; b += (uint32_t)(u1 >> 32); c += (uint32_t)u2;
    JMIX(a, b, c);
    a += (uint32_t)(u2 >> 32); b += (uint32_t)u3; c += (uint32_t)(u3 >> 32);
    JMIX(a, b, c);
    c += 24;
    JMIX(a, b, c);
    return c;
}

static inline uint32_t grain_hash(const uint64_t* k) { return cpu_jenkins_u64x3(k[2], k[0], k[1]); }

/* ------------------------------------------------------------------ directory */
typedef struct {
    uint64_t n0, n1, tcd;
    uint32_t act, silo;
    int32_t next;      /* chain (faithful) */
    int32_t hash;      /* cached (int)uniform hash */
} entry_t;

typedef struct cpu_dir {
    int faithful;
    pthread_mutex_t lock;
    /* faithful: buckets + entries (.NET Dictionary shape) */
    int32_t* buckets;
    uint64_t nbuckets;
    entry_t* entries;
    uint64_t count, cap_entries;
    /* fast: open addressing, power of two */
    entry_t* slots;
    uint8_t* used;
    uint64_t mask;
} cpu_dir;

static int is_prime(uint64_t x) {
    if (x < 2) return 0;
    for (uint64_t d = 2; d * d <= x; ++d)
        if (x % d == 0) return 0;
    return 1;
}

cpu_dir* cpu_dir_new(int faithful, uint64_t capacity_hint) {
    cpu_dir* d = (cpu_dir*)calloc(1, sizeof(cpu_dir));
    d->faithful = faithful;
    pthread_mutex_init(&d->lock, NULL);
    if (capacity_hint < 16) capacity_hint = 16;
    if (faithful) {
        uint64_t p = capacity_hint | 1;
        while (!is_prime(p)) p += 2;
        d->nbuckets = p;
        d->buckets = (int32_t*)malloc(p * sizeof(int32_t));
        memset(d->buckets, 0xFF, p * sizeof(int32_t));
        d->cap_entries = capacity_hint;
        d->entries = (entry_t*)malloc(d->cap_entries * sizeof(entry_t));
    } else {
        uint64_t c = 1;
        while (c < 2 * capacity_hint) c <<= 1;
        d->mask = c - 1;
        d->slots = (entry_t*)calloc(c, sizeof(entry_t));
        d->used = (uint8_t*)calloc(c, 1);
    }
    return d;
}

void cpu_dir_free(cpu_dir* d) {
    if (!d) return;
    free(d->buckets); free(d->entries); free(d->slots); free(d->used);
    pthread_mutex_destroy(&d->lock);
    free(d);
}

static inline int key_eq(const entry_t* e, const uint64_t* k) {
    return e->n0 == k[0] && e->n1 == k[1] && e->tcd == k[2];
}

static const entry_t* dir_find(cpu_dir* d, const uint64_t* k, uint32_t h) {
    if (d->faithful) {
        /* Dictionary<GrainId,..>: hashCode = GetHashCode() & 0x7FFFFFFF (GrainId hash = (int)uniform) */
        const int32_t hc = (int32_t)(h & 0x7FFFFFFFu);
        for (int32_t i = d->buckets[(uint64_t)hc % d->nbuckets]; i >= 0; i = d->entries[i].next)
            if (d->entries[i].hash == hc && key_eq(&d->entries[i], k)) return &d->entries[i];
        return NULL;
    }
    uint64_t s = h & d->mask;
    for (;;) {
        if (!d->used[s]) return NULL;
        if (key_eq(&d->slots[s], k)) return &d->slots[s];
        s = (s + 1) & d->mask;
    }
}

/* AddSingleActivation (GrainDirectoryPartition.cs:304-326): first registration wins. */
void cpu_dir_register(cpu_dir* d, const uint64_t* keys, const uint32_t* acts, const uint32_t* silos, uint64_t n,
                      uint32_t* out_act, uint32_t* out_silo, uint8_t* out_ins) {
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t* k = keys + 3 * i;
        const uint32_t h = grain_hash(k);
        const entry_t* f = dir_find(d, k, h);
        if (f) {
            out_act[i] = f->act; out_silo[i] = f->silo; out_ins[i] = 0;
            continue;
        }
        entry_t e = {k[0], k[1], k[2], acts[i], silos[i], -1, (int32_t)(h & 0x7FFFFFFFu)};
        if (d->faithful) {
            if (d->count == d->cap_entries) {
                d->cap_entries *= 2;
                d->entries = (entry_t*)realloc(d->entries, d->cap_entries * sizeof(entry_t));
            }
            const uint64_t b = (uint64_t)e.hash % d->nbuckets;
            e.next = d->buckets[b];
            d->entries[d->count] = e;
            d->buckets[b] = (int32_t)d->count;
        } else {
            uint64_t s = h & d->mask;
            while (d->used[s]) s = (s + 1) & d->mask;
            d->slots[s] = e;
            d->used[s] = 1;
        }
        d->count++;
        out_act[i] = acts[i]; out_silo[i] = silos[i]; out_ins[i] = 1;
    }
}

/* ------------------------------------------------------------------ ring */
static const uint64_t MT_N0 = 0x11E0C21E01145FECull, MT_N1 = 0x9B012447FBD00591ull, MT_TCD = 2ull << 56;

static uint32_t ring_pos_scan(int mode, const uint32_t* pts, uint32_t n, uint32_t h) {
    if (mode == 0) {               /* LocalGrainDirectory.cs:521-538 */
        for (int64_t i = (int64_t)n - 1; i >= 0; --i)
            if ((int32_t)pts[i] <= (int32_t)h) return (uint32_t)i;
        return n - 1;
    }
    for (uint32_t i = 0; i < n; ++i) {
        if (mode == 1 ? ((int64_t)(int32_t)pts[i] >= (int64_t)h) : (pts[i] >= h)) return i;
    }
    return 0;
}

static uint32_t ring_pos_bsearch(int mode, const uint32_t* pts, uint32_t n, uint32_t h) {
    uint32_t lo = 0, hi = n;   /* count of the prefix satisfying the monotone predicate */
    while (lo < hi) {
        const uint32_t mid = (lo + hi) / 2;
        const uint32_t p = pts[mid];
        const int pred = mode == 0 ? ((int32_t)p <= (int32_t)h) : mode == 1 ? ((int32_t)p < 0 || p < h) : (p < h);
        if (pred) lo = mid + 1; else hi = mid;
    }
    if (mode == 0) return lo == 0 ? n - 1 : lo - 1;
    return lo == n ? 0 : lo;
}

typedef struct {
    cpu_dir* d; int faithful, mode; const uint32_t *pts, *own; uint32_t npts;
    const uint64_t* keys; uint64_t lo, hi; uint32_t my_silo, seed_silo;
    uint8_t* st; uint32_t *silo, *act;
} route_job;

static void* route_worker(void* arg) {
    route_job* j = (route_job*)arg;
    for (uint64_t i = j->lo; i < j->hi; ++i) {
        const uint64_t* k = j->keys + 3 * i;
        const uint32_t cat = (uint32_t)(k[2] >> 56);
        if (cat == 1) { j->st[i] = 2; j->silo[i] = j->my_silo; j->act[i] = M32; continue; }
        if (k[0] == MT_N0 && k[1] == MT_N1 && k[2] == MT_TCD) { j->st[i] = 3; j->silo[i] = j->seed_silo; j->act[i] = M32; continue; }
        if (cat == 6 || cat == 7) { j->st[i] = 4; j->silo[i] = M32; j->act[i] = M32; continue; }
        const uint32_t h = grain_hash(k);
        uint32_t owner;
        if (j->faithful) {
            pthread_mutex_lock(&j->d->lock);          /* lock(membershipCache) */
            owner = j->own[ring_pos_scan(j->mode, j->pts, j->npts, h)];
            pthread_mutex_unlock(&j->d->lock);
            pthread_mutex_lock(&j->d->lock);          /* lock(lockable) */
        } else {
            owner = j->own[ring_pos_bsearch(j->mode, j->pts, j->npts, h)];
        }
        const entry_t* e = dir_find(j->d, k, h);
        if (j->faithful) pthread_mutex_unlock(&j->d->lock);
        if (e) { j->st[i] = 0; j->silo[i] = e->silo; j->act[i] = e->act; }
        else { j->st[i] = 1; j->silo[i] = owner; j->act[i] = M32; }
    }
    return NULL;
}

int cpu_route(cpu_dir* d, int faithful, int mode, const uint32_t* pts, const uint32_t* own, uint32_t npts,
              const uint64_t* keys, uint64_t n, uint32_t my_silo, uint32_t seed_silo, uint8_t* st, uint32_t* silo,
              uint32_t* act, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    route_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        route_job j = {d, faithful, mode, pts, own, npts, keys, n * t / nthreads, n * (t + 1) / nthreads,
                       my_silo, seed_silo, st, silo, act};
        jobs[t] = j;
        if (nthreads == 1) route_worker(&jobs[0]);
        else pthread_create(&th[t], NULL, route_worker, &jobs[t]);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    return 0;
}

/* ------------------------------------------------------------------ bucketing */
typedef struct { uint32_t* v; uint32_t len, cap; } fifo_t;

/* Fast mode: a parallel two-level stable partition, O(n + n_act) work in all, no O(n_act) pass per
 * thread.  Level 1: each thread counts the high digit key >> s of its contiguous slice (H <= 4,096
 * digits), one serial scan over [digit][thread], each thread scatters (index, key) stably.  Level 2:
 * the threads take high-digit buckets from a shared counter; a bucket's 2^s activations get a private
 * counting sort (counts, exclusive scan written as their offsets, stable placement).  */
typedef struct {
    const uint32_t* act; uint64_t lo, hi; uint32_t n_act, shift, H; uint64_t* hist; uint32_t *tk, *ti, *perm, *off;
    int phase; uint32_t* next; const uint64_t* bstart; uint32_t* cnt;
} bk_job;

static void* bucket_worker(void* arg) {
    bk_job* j = (bk_job*)arg;
    if (j->phase == 0) {
        for (uint64_t i = j->lo; i < j->hi; ++i) {
            const uint32_t a = j->act[i] < j->n_act ? j->act[i] : j->n_act;
            j->hist[a >> j->shift]++;
        }
    } else if (j->phase == 1) {
        for (uint64_t i = j->lo; i < j->hi; ++i) {
            const uint32_t a = j->act[i] < j->n_act ? j->act[i] : j->n_act;
            const uint64_t p = j->hist[a >> j->shift]++;
            j->tk[p] = a;
            j->ti[p] = (uint32_t)i;
        }
    } else {
        const uint32_t L = 1u << j->shift;
        for (;;) {
            const uint32_t b = __atomic_fetch_add(j->next, 1u, __ATOMIC_RELAXED);
            if (b >= j->H) break;
            const uint64_t s0 = j->bstart[b], s1 = j->bstart[b + 1];
            const uint64_t k0 = (uint64_t)b << j->shift;
            const uint64_t nk = (uint64_t)j->n_act + 1 - k0 < L ? (uint64_t)j->n_act + 1 - k0 : L;
            memset(j->cnt, 0, nk * sizeof(uint32_t));
            for (uint64_t p = s0; p < s1; ++p) j->cnt[j->tk[p] - k0]++;
            uint64_t run = s0;
            for (uint64_t a = 0; a < nk; ++a) {
                const uint32_t c = j->cnt[a];
                j->off[k0 + a] = (uint32_t)run;
                j->cnt[a] = (uint32_t)run;
                run += c;
            }
            for (uint64_t p = s0; p < s1; ++p) j->perm[j->cnt[j->tk[p] - k0]++] = j->ti[p];
        }
    }
    return NULL;
}

static void run_jobs(bk_job* jobs, int nthreads) {
    pthread_t th[256];
    if (nthreads == 1) { bucket_worker(&jobs[0]); return; }
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, bucket_worker, &jobs[t]);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

/* Stable partition by activation: faithful = per-activation FIFO append
 * (ActivationData.cs:604-605), fast = the parallel two-level partition above. */
int cpu_bucket(int faithful, const uint32_t* act, uint64_t n, uint32_t n_act, uint32_t* perm, uint32_t* off,
               int nthreads) {
    const uint64_t nb = (uint64_t)n_act + 1;
    if (faithful) {
        fifo_t* q = (fifo_t*)calloc(nb, sizeof(fifo_t));
        for (uint64_t i = 0; i < n; ++i) {
            const uint32_t a = act[i] < n_act ? act[i] : n_act;
            fifo_t* f = &q[a];
            if (f->len == f->cap) {
                f->cap = f->cap ? 2 * f->cap : 4;
                f->v = (uint32_t*)realloc(f->v, f->cap * sizeof(uint32_t));
            }
            f->v[f->len++] = (uint32_t)i;
        }
        uint64_t pos = 0;
        for (uint64_t a = 0; a < nb; ++a) {
            off[a] = (uint32_t)pos;
            if (q[a].len) memcpy(perm + pos, q[a].v, q[a].len * sizeof(uint32_t));
            pos += q[a].len;
            free(q[a].v);
        }
        off[nb] = (uint32_t)pos;
        free(q);
        return 0;
    }
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    /* s: low bits sorted per bucket (2^s counters, <= 256 KB a thread), leaving <= 4,096 high digits */
    uint32_t kb = 1;
    while (kb < 32 && (nb - 1) >> kb) ++kb;
    const uint32_t shift = kb > 12 ? (kb - 12 < 16 ? (kb - 12 > 6 ? kb - 12 : 6) : 16) : 6;
    const uint32_t H = (uint32_t)(((nb - 1) >> shift) + 1);
    uint64_t* hist = (uint64_t*)calloc((uint64_t)nthreads * H, sizeof(uint64_t));
    uint64_t* bstart = (uint64_t*)malloc(((uint64_t)H + 1) * sizeof(uint64_t));
    uint32_t* tk = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
    uint32_t* ti = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
    uint32_t* cnt = (uint32_t*)malloc((uint64_t)nthreads << shift << 2);
    uint32_t next = 0;
    bk_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        bk_job j = {act, n * t / nthreads, n * (t + 1) / nthreads, n_act, shift, H, hist + (uint64_t)t * H,
                    tk, ti, perm, off, 0, &next, bstart, cnt + ((uint64_t)t << shift)};
        jobs[t] = j;
    }
    run_jobs(jobs, nthreads);
    uint64_t run = 0;
    for (uint32_t d = 0; d < H; ++d) {          /* [digit][thread]: thread slices in batch order */
        bstart[d] = run;
        for (int t = 0; t < nthreads; ++t) {
            const uint64_t c = hist[(uint64_t)t * H + d];
            hist[(uint64_t)t * H + d] = run;
            run += c;
        }
    }
    bstart[H] = run;
    for (int t = 0; t < nthreads; ++t) jobs[t].phase = 1;
    run_jobs(jobs, nthreads);
    for (int t = 0; t < nthreads; ++t) jobs[t].phase = 2;
    run_jobs(jobs, nthreads);
    off[nb] = (uint32_t)n;
    free(hist); free(bstart); free(tk); free(ti); free(cnt);
    return 0;
}

/* Micro-batch form of the bucketing (BASELINE cfg 5, the CPU side of gd_microbatch_run): the
 * activations present in a small batch, ascending, each with its messages in arrival order
 * (ActivationData.waiting FIFO append, ActivationData.cs:604-605).  Work is O(n + k log k) for k
 * distinct activations -- no O(n_act) pass per batch.  counts[n_act + 1] is caller scratch that is
 * zero on entry and left zero on return. */
static int cmp_u32(const void* a, const void* b) {
    const uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return x < y ? -1 : x > y;
}

int cpu_bucket_runs(const uint32_t* act, uint64_t n, uint32_t n_act, uint32_t* counts, uint32_t* perm,
                    uint32_t* run_act, uint32_t* run_start, uint32_t* n_runs) {
    uint32_t k = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t a = act[i] < n_act ? act[i] : n_act;
        if (counts[a]++ == 0) run_act[k++] = a;
    }
    qsort(run_act, k, sizeof(uint32_t), cmp_u32);
    uint32_t pos = 0;
    for (uint32_t r = 0; r < k; ++r) {
        const uint32_t c = counts[run_act[r]];
        run_start[r] = pos;
        counts[run_act[r]] = pos;   /* now the write cursor */
        pos += c;
    }
    run_start[k] = pos;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t a = act[i] < n_act ? act[i] : n_act;
        perm[counts[a]++] = (uint32_t)i;
    }
    for (uint32_t r = 0; r < k; ++r) counts[run_act[r]] = 0;
    *n_runs = k;
    return 0;
}
