// eng_core.hip -- libgraindispatch: scratch, launches, the probe index and measured choices, the route and bucketing drivers, the exchange partition.
// Shared handle and helpers: gd_engine.h.
#include "gd_engine.h"


namespace gdx {

thread_local std::string g_tls_error = "";



}  // namespace gdx


namespace gdx {

int set_err(gd_handle* h, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (h) h->err = buf;
    g_tls_error = buf;
    return code;
}


// A bucketing gd_route_bucket_device left running on the bucket stream (gd_set_bucket_stream) uses the
// handle's scratch (u32_a..d, hist, partials, m3): every entry point that takes scratch on the handle's
// own stream waits for it first (ensure() calls this).  The route itself takes no scratch,
// so the next batch's route still overlaps this batch's bucketing.
int bfence(gd_handle* h) {
    if (!h->b_pending || !h->bstream || h->bstream == h->stream) return GD_OK;
    HIP_TRY(h, hipEventRecord(h->b_fence_ev, h->bstream));
    HIP_TRY(h, hipStreamWaitEvent(h->stream, h->b_fence_ev, 0));
    h->b_pending = false;
    return GD_OK;
}

int ensure(gd_handle* h, DevBuf& b, size_t bytes) {
    GD_TRY(bfence(h));
    return ensure_own(h, b, bytes);
}

// ensure() for a buffer no bucketing touches (the directory batches' dir_scr): no bfence.
int ensure_own(gd_handle* h, DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes && b.p) return GD_OK;
    if (b.p) {
        HIP_TRY(h, hipStreamSynchronize(h->stream));
        HIP_TRY(h, hipFree(b.p));
        b.p = nullptr;
        b.bytes = 0;
    }
    size_t want = std::max<size_t>(bytes, 256);
    hipError_t e = hipMalloc(&b.p, want);
    if (e != hipSuccess) return set_err(h, GD_ENOMEM, "hipMalloc(%zu): %s", want, hipGetErrorString(e));
    b.bytes = want;
    return GD_OK;
}

void free_buf(DevBuf& b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}

int name_id(gd_handle* h, const char* name) {
    for (size_t i = 0; i < h->tnames.size(); ++i)
        if (h->tnames[i] == name) return (int)i;
    h->tnames.emplace_back(name);
    h->tms.push_back(0.0);
    h->tcount.push_back(0);
    return (int)h->tnames.size() - 1;
}

hipEvent_t take_event(gd_handle* h) {
    if (!h->event_pool.empty()) {
        hipEvent_t e = h->event_pool.back();
        h->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}


int resolve_timing(gd_handle* h) {
    if (h->pending.empty()) return GD_OK;
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    if (h->bstream) HIP_TRY(h, hipStreamSynchronize(h->bstream));
    if (h->xstream) HIP_TRY(h, hipStreamSynchronize(h->xstream));
    if (h->pstream) HIP_TRY(h, hipStreamSynchronize(h->pstream));
    for (auto& t : h->pending) {
        float ms = 0.f;
        HIP_TRY(h, hipEventElapsedTime(&ms, t.a, t.b));
        h->tms[t.name] += ms;
        h->tcount[t.name] += 1;
        h->event_pool.push_back(t.a);
        h->event_pool.push_back(t.b);
    }
    h->pending.clear();
    return GD_OK;
}


int check_ring(gd_handle* h) {
    if (h->ring_mode < 0 || h->ring_n == 0) return set_err(h, GD_ESTATE, "no ring installed (gd_ring_set)");
    return GD_OK;
}

RingArgs ring_args(gd_handle* h) {
    return RingArgs{(const uint32_t*)h->ring_pts.p, (const uint32_t*)h->ring_own.p, h->ring_n, h->ring_top,
                    h->cfg.my_silo, h->cfg.seed_silo};
}

TableArgs table_args(gd_handle* h) {
    return TableArgs{h->slots, h->capacity - 1, h->ctr, (const uint32_t*)h->dir_valid.p, h->n_valid};
}

bool host_silo_valid(const gd_handle* h, uint32_t silo) {
    return h->n_valid == 0 || silo >= h->n_valid || h->valid_host[silo];
}

size_t ring_lds(gd_handle* h) { return (size_t)h->ring_n * 2 * sizeof(uint32_t); }

// The striped live / tomb deltas (gd_kernels.h CTR_STRIPES) into the counters, before a read-back.
int fold_counters(gd_handle* h, DevCounters* c) {
    hipLaunchKernelGGL(k_ctr_fold, dim3(1), dim3(64), 0, h->stream, c);
    HIP_TRY(h, hipGetLastError());
    return GD_OK;
}

int pull_counters(gd_handle* h) {
    GD_TRY(fold_counters(h, h->ctr));
    HIP_TRY(h, hipMemcpyAsync(&h->ctr_host, h->ctr, sizeof(DevCounters), hipMemcpyDeviceToHost, h->stream));
    if (h->cx_built && h->cxi_ctr.p)   // the index counters ride along (cx_ensure's rebuild rule)
        HIP_TRY(h, hipMemcpyAsync(&h->cx_ctr_host, h->cxi_ctr.p, sizeof(CxCounters), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    h->ctr_stale = false;
    h->pending_in = 0;
    // every batch enqueued so far is done: the index is pure again if no batch left anything out
    if (h->tab_track == 0 && h->cx_built && h->cxi_ctr.p)
        h->cx8_pure = h->cx8_ok && h->cx8_layout.ntypes == 1 && h->cx_ctr_host.out8 == 0;
    return GD_OK;
}

int alloc_table(gd_handle* h, unsigned long long cap, Slot** out) {
    if (cap > (1ull << 32)) return set_err(h, GD_EINVAL, "table of %llu slots: at most 2^32 (home_slot)", cap);
    Slot* s = nullptr;
    hipError_t e = hipMalloc(&s, cap * sizeof(Slot));
    if (e != hipSuccess) return set_err(h, GD_ENOMEM, "table hipMalloc(%llu slots): %s", cap, hipGetErrorString(e));
    e = hipMemsetAsync(s, 0, cap * sizeof(Slot), h->stream);
    if (e != hipSuccess) {
        (void)hipFree(s);
        return set_err(h, GD_EHIP, "table memset: %s", hipGetErrorString(e));
    }
    *out = s;
    return GD_OK;
}

int alloc_vtag(gd_handle* h, unsigned long long cap, uint32_t** out) {
    uint32_t* v = nullptr;
    hipError_t e = hipMalloc(&v, cap * sizeof(uint32_t));
    if (e != hipSuccess) return set_err(h, GD_ENOMEM, "version tags hipMalloc(%llu): %s", cap, hipGetErrorString(e));
    e = hipMemsetAsync(v, 0, cap * sizeof(uint32_t), h->stream);
    if (e != hipSuccess) {
        (void)hipFree(v);
        return set_err(h, GD_EHIP, "version tags memset: %s", hipGetErrorString(e));
    }
    *out = v;
    return GD_OK;
}

unsigned long long pow2_at_least(unsigned long long x) {
    unsigned long long c = 1024;
    while (c < x) c <<= 1;
    return c;
}

// ---- compact probe indexes (gd_cx.h) ----------------------------------------------
bool cx_current(const gd_handle* h) {
    return h->cx_built && h->cx_slots_at == h->slots && h->cx_cap_at == h->capacity && h->cx_gen_at == h->tab_gen;
}

TabTrack::TabTrack(gd_handle* hh) : h(hh), was_current(cx_current(hh)) {
    ++h->tab_track;
    h->cx8_pure = false;                 // until a read-back after the batch shows the index still pure
}

static uint32_t bit_len(uint64_t x) {
    uint32_t b = 0;
    while (x) {
        ++b;
        x >>= 1;
    }
    return b;
}

CxBuild cx_build_args(gd_handle* h) {
    return CxBuild{(uint4*)h->cxi_tab.p, (unsigned long long*)h->cxi_types.p,
                   h->cx8_ok ? (unsigned long long*)h->cx8_tab.p : nullptr, h->cx8_layout};
}

// Grid of the table-wide index passes: CXT_IT slots a thread a round, at most 16 workgroups a CU.
static uint32_t cx_grid(gd_handle* h) {
    return std::max<uint32_t>(1, std::min<uint64_t>(blocks_for(h->capacity, BLOCK * CXT_IT), (uint64_t)h->n_cu * 16));
}

// The full build: k_cx_types, one read-back (types, counts, widths), the 8-B layout, k_cx_project.
// The 8-B index takes the most populous types (up to CX8_TYPES) and the activation / silo widths of the
// live entries; fewer types when the three fields would not fit 31 bits, narrower activations last
// (wider ones are then redirect entries: their keys probe the directory).
static int cx_build(gd_handle* h) {
    const auto t0 = std::chrono::steady_clock::now();
    const unsigned long long cap = h->capacity;
    GD_TRY(ensure(h, h->cxi_tab, cap * 16));
    GD_TRY(ensure(h, h->cx8_tab, cap * 8));
    GD_TRY(ensure(h, h->cxi_types, CX_TYPES * 12));
    GD_TRY(ensure(h, h->cxi_ctr, sizeof(CxCounters)));
    unsigned long long* types = (unsigned long long*)h->cxi_types.p;
    uint32_t* counts = (uint32_t*)(types + CX_TYPES);
    CxCounters* ctr = (CxCounters*)h->cxi_ctr.p;
    HIP_TRY(h, hipMemsetAsync(types, 0xFF, CX_TYPES * 8, h->stream));
    HIP_TRY(h, hipMemsetAsync(counts, 0, CX_TYPES * 4, h->stream));
    HIP_TRY(h, hipMemsetAsync(ctr, 0, sizeof(CxCounters), h->stream));
    const dim3 g(cx_grid(h)), b(BLOCK);
    GD_TRY(launch(h, "k_cx_types", g, b, 0, k_cx_types, (const Slot*)h->slots, cap, types, counts, ctr));
    CxCounters c{};
    unsigned long long ht[CX_TYPES];
    uint32_t hc[CX_TYPES];
    HIP_TRY(h, hipMemcpyAsync(&c, ctr, sizeof c, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipMemcpyAsync(ht, types, sizeof ht, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipMemcpyAsync(hc, counts, sizeof hc, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    std::vector<std::pair<uint32_t, unsigned long long>> by_count;
    for (uint32_t t = 0; t < CX_TYPES; ++t)
        if (ht[t] != CX_NO_TYPE) by_count.emplace_back(hc[t], ht[t]);
    std::stable_sort(by_count.begin(), by_count.end(),
                     [](const auto& x, const auto& y) { return x.first > y.first; });
    uint32_t n8 = (uint32_t)std::min<size_t>(CX8_TYPES, by_count.size());
    uint32_t ab = std::max<uint32_t>(2, bit_len((uint64_t)c.act_max + 2));
    const uint32_t sb = std::max<uint32_t>(1, bit_len((uint64_t)c.silo_max + 1));
    for (;;) {
        const uint32_t tb = n8 > 1 ? bit_len(n8 - 1) : 0;
        if (ab + sb + tb <= 31) break;
        if (tb > 0) {
            n8 = 1u << (tb - 1);                       // fewer types before narrower activations
            continue;
        }
        ab = sb + tb >= 29 ? 0 : 31 - sb - tb;
        break;
    }
    Cx8Args p8{};
    p8.slots = (const uint4*)h->cx8_tab.p;
    p8.cap = cap;
    p8.ntypes = n8;
    for (uint32_t k = 0; k < n8; ++k) p8.tcd[k] = by_count[k].second;
    p8.ab = ab;
    p8.sb = sb;
    h->cx8_layout = p8;
    h->cx8_ok = ab >= 2;
    uint32_t held8 = 0;
    for (uint32_t k = 0; k < n8; ++k) held8 += by_count[k].first;
    h->cx_held8_at = held8;
    GD_TRY(launch(h, "k_cx_project", g, b, 0, k_cx_project, (const Slot*)h->slots, cap, cx_build_args(h), ctr));
    HIP_TRY(h, hipMemcpyAsync(&h->cx_ctr_host, ctr, sizeof(CxCounters), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    h->cx_ok = true;
    h->cx_built = true;
    h->cx_out8_at = h->cx_ctr_host.out8;              // the build's own: the baseline of the rebuild rule
    h->cx8_pure = h->cx8_ok && h->cx8_layout.ntypes == 1 && h->cx_ctr_host.out8 == 0;
    h->cx_builds++;
    h->cx_build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return GD_OK;
}

// Re-projects the slots a directory batch touched (slot_of[n]) when the indexes were current before it.
// Only enqueued: its counters come back with the next pull_counters, and when the batches' new entries
// no longer fit the 8-B layout (a new grain class, wider activations or silos) beyond an eighth of the
// entries it held, cx_ensure rebuilds with a new layout.
int cx_sync(gd_handle* h, TabTrack& tt, const uint32_t* slot_of, uint32_t n) {
    tt.synced = true;
    if (!tt.was_current || n == 0) return GD_OK;   // a stale index stays stale: the next large route rebuilds
    GD_TRY(launch(h, "k_cx_sync", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), 0, k_cx_sync, slot_of, n,
                  (const Slot*)h->slots, cx_build_args(h), (CxCounters*)h->cxi_ctr.p));
    h->cx_synced += n;
    return GD_OK;
}

// A directory batch that projects its slots inside its commit kernel: true (and the batch counted as
// synced) when the indexes were current before it; false leaves a stale index stale.
bool cx_inline(gd_handle* h, TabTrack& tt, uint32_t n) {
    tt.synced = true;
    if (!tt.was_current || !h->cx_ok) return false;
    h->cx_synced += n;
    return true;
}

// The index for the current table: rebuilt (two streaming passes + one host sync) when the table
// changed since the last build by a write that did not re-project its slots (gd_dir_rehash, clear,
// merge, silo removal, split, handoff); false when GD_OPT_PROBE = 0.  n: the messages of the launch
// asking.  A stale index is rebuilt only for a launch of at least capacity / 16 messages: a small route
// after such a change takes the directory probe instead of a full-table pass and a host sync (ADVICE
// r03); the next large launch rebuilds.
int cx_ensure(gd_handle* h, bool* ok, uint64_t n) {
    *ok = false;
    if (!h->cx_mode || !h->slots || h->capacity < CX8_GROUP) return GD_OK;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;   // a captured graph keeps the directory probe
    HIP_TRY(h, hipStreamIsCapturing(h->stream, &cs));
    if (cs != hipStreamCaptureStatusNone) return GD_OK;
    if (cx_current(h)) {
        const CxCounters& c = h->cx_ctr_host;
        if (!(h->cx8_ok && c.out8 > h->cx_out8_at && c.out8 - h->cx_out8_at > h->cx_held8_at / 8 + 4096)) {
            *ok = h->cx_ok;
            return GD_OK;
        }
        h->tab_gen++;                               // the 8-B layout no longer fits the directory: rebuild
    }
    if (h->cx_mode == 1 && n < h->capacity / 16) return GD_OK;
    GD_TRY(cx_build(h));
    for (auto& kt : h->cx_tune) {                   // a new table: measure the probes again (not the bucketing)
        if (kt.first / (64 * 32) == GD_TUNE_BUCKET) continue;
        auto& t = kt.second;
        for (int v = 0; v < gd_handle::CXV; ++v) {
            if (t.pending[v]) (void)hipEventSynchronize(t.b[v]);
            t.best[v] = 1e30f;
            t.pending[v] = false;
        }
        t.pick = -1;
        t.round = 0;
    }
    h->cx_slots_at = h->slots;
    h->cx_cap_at = h->capacity;
    h->cx_gen_at = h->tab_gen;
    *ok = h->cx_ok;
    return GD_OK;
}

// The probe variant for a launch of `kind` (0 keys, 1 N1s, 2 fan-out, 3 node ids) over n messages when
// the index is available: 0 the index read in 64-B groups, 1 the directory, 2 the index read one 16-B
// slot at a time.  GD_CX=2: always 0.  GD_CX=1 times the three on the first six eligible launches of the
// kind and size class (bit length of n: the fan-out's hops differ 10x in size, and per-message cost
// with them), twice each in turn, between HIP events read back without a stream sync at the next
// choice, and keeps the fastest per message.  All give the same results; which is fastest depends on
// the key distribution (a Zipf-hot set favours small reads, a uniform one the index's group reads,
// DESIGN 5).  nvar: the variants this launch kind has (2: no 16-B-read form).  *meas: the tune entry
// this launch is timed into (key * CXV + variant), or -1.
// The tune entry's key: kind, size class (bit length of n), a second shape class.
int tune_key(int kind, uint64_t n, int sub) {
    int cls = 0;
    while (cls < 63 && (n >> cls) > 1) ++cls;
    return (kind * 64 + cls) * 32 + std::max(0, std::min(31, sub));
}

// Variants of a tune kind (GD_TUNE_*): the 24-B-key and N1 probes have three, the rest two.
int tune_nvar(int kind) { return kind <= 1 ? 4 : (kind <= 3 ? 3 : 2); }

// Variants a launch of `kind` has on this handle now: kinds 0 / 1 and 2 / 3 have the 8-B index as their
// last variant only where it is built (cx_ensure), kind 4 (the bucketing form) always two.
int tune_nvar_now(const gd_handle* h, int kind) {
    if (kind <= 1) return h->cx8_ok ? 4 : 3;
    if (kind <= 3) return h->cx8_ok ? 3 : 2;
    return 2;
}

// Folds the entry's finished timings in (events read without a stream sync, unless the entry has
// timed every variant twice and only waits for them) and picks when every variant is timed.
void tune_resolve(gd_handle::CxTune& t, int nvar) {
    constexpr int V = gd_handle::CXV;
    bool any_pending = false;
    for (int v = 0; v < V; ++v) {
        if (!t.pending[v]) continue;
        if (hipEventQuery(t.b[v]) != hipSuccess && t.pick < 0 && t.round >= 2 * nvar) (void)hipEventSynchronize(t.b[v]);
        if (hipEventQuery(t.b[v]) == hipSuccess) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, t.a[v], t.b[v]) == hipSuccess && t.n[v])
                t.best[v] = std::min(t.best[v], ms / (float)t.n[v]);
            t.pending[v] = false;
        }
        any_pending = any_pending || t.pending[v];
    }
    if (t.pick < 0 && t.round >= 2 * nvar && !any_pending) {
        t.pick = 0;
        for (int v = 1; v < nvar; ++v)
            if (t.best[v] < t.best[t.pick]) t.pick = v;
    }
}

// The probe variant for a launch of `kind` (0 keys, 1 N1s, 2 fan-out, 3 node ids) over n messages when
// the index is available: 0 the index read in 64-B groups, 1 the directory, 2 the index read one 16-B
// slot at a time; kind 4: the bucketing form.  A variant pinned by gd_tune_set is taken at once.
// Else the first launches of the kind and size class (bit length of n: the fan-out's hops differ 10x
// in size, and per-message cost with them) time the variants, twice each in turn, between HIP events
// read back without a stream sync at the next choice, and the fastest per message is kept (or the one
// gd_tune_agree settled on).  All give the same results; which is fastest depends on the key
// distribution (a Zipf-hot set favours small reads, a uniform one the index's group reads).
// nvar: the variants this launch kind has.  *meas: the tune entry this launch is timed into
// (key * CXV + variant), or -1.
int tune_choose(gd_handle* h, int kind, uint64_t n, int* meas, int nvar, int sub) {
    constexpr int V = gd_handle::CXV;
    *meas = -1;
    if (h->tune_pin[kind] >= 0 && h->tune_pin[kind] < nvar) return h->tune_pin[kind];
    const int key = tune_key(kind, n, sub);
    auto& t = h->cx_tune[key];
    if (t.pick >= nvar || (t.pick < 0 && t.nvar && t.nvar != nvar)) {
        // a pick (gd_tune_agree's, or this entry's own) of a variant this launch does not have -- the
        // 8-B index not built here, or no longer -- or timings taken over another variant set: measure
        // again over the variants this launch has
        for (int v = 0; v < V; ++v) {
            if (t.pending[v] && t.b[v]) (void)hipEventSynchronize(t.b[v]);
            t.pending[v] = false;
            t.best[v] = 1e30f;
            t.n[v] = 0;
        }
        t.pick = -1;
        t.round = 0;
    }
    t.nvar = nvar;
    tune_resolve(t, nvar);
    if (t.pick >= 0) return t.pick;
    const int v = t.round % nvar;
    if (t.round < 2 * nvar && !t.pending[v]) {
        if (!t.a[v]) (void)hipEventCreate(&t.a[v]);
        if (!t.b[v]) (void)hipEventCreate(&t.b[v]);
        *meas = key * V + v;
        ++t.round;
        h->measured_launch = true;
    }
    return v;
}

int cx_choose(gd_handle* h, int kind, uint64_t n, int* meas, int nvar) {
    *meas = -1;
    // variants: 0 index groups, 1 directory; kinds 0 / 1: 2 index slots, 3 the 8-B index; kinds 2 / 3:
    // 2 the 8-B index (when built: nvar says)
    if (h->cx_mode == 2) return 0;
    if (h->cx_mode == 3) return kind <= 1 && nvar > 2 ? 2 : 0;
    if (h->cx_mode == 4) return kind <= 1 ? (nvar > 3 ? 3 : 0) : ((kind == 2 || kind == 3) && nvar > 2 ? 2 : 0);
    return tune_choose(h, kind, n, meas, nvar);
}


Cx8Args cx8_args(gd_handle* h) { return h->cx8_layout; }

CxArgs cx_args(gd_handle* h) {
    return CxArgs{(const uint4*)h->cxi_tab.p, h->capacity, (const unsigned long long*)h->cxi_types.p};
}

// ---- route -------------------------------------------------------------------
// The tune entry's second class for the bucketing form (kind 4): the messages a 1,024-activation range
// holds, as a bit length (it decides whether ranges are staged in LDS).
int bucket_sub(uint64_t n, uint32_t n_act) {
    int per_range = 0;
    while (per_range < 31 && ((uint64_t)n / ((n_act >> MSD_SHIFT) + 1) >> per_range) > 1) ++per_range;
    return per_range;
}

template <int MODE, int M, bool NT>
int route_launch(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t* silo, uint32_t* act, uint8_t* status) {
    bool cx = false;
    GD_TRY(cx_ensure(h, &cx, n));
    int meas = -1;
    const int var = cx ? cx_choose(h, 0, n, &meas, h->cx8_ok ? 4 : 3) : 1;
    CxMeasure m(h, meas, n);
    if (var == 3 && h->cx8_pure)             // nothing to fall back to the directory for (gd_engine.h cx8_pure)
        return launch(h, "k_route", dim3(blocks_for(n, BLOCK * M)), dim3(BLOCK), ring_lds(h),
                      k_route_m<MODE, M, NT, 0, false, (int)CX_GROUP, true, true>, keys, n, ring_args(h),
                      table_args(h), silo, act, status, 0ull, h->route_xcd ? 1u : 0u, (const uint32_t*)nullptr, 0u,
                      (uint32_t*)nullptr, CxArgs{}, cx8_args(h));
    if (var == 3)
        return launch(h, "k_route", dim3(blocks_for(n, BLOCK * M)), dim3(BLOCK), ring_lds(h),
                      k_route_m<MODE, M, NT, 0, false, (int)CX_GROUP, true>, keys, n, ring_args(h), table_args(h), silo,
                      act, status, 0ull, h->route_xcd ? 1u : 0u, (const uint32_t*)nullptr, 0u, (uint32_t*)nullptr,
                      CxArgs{}, cx8_args(h));
    if (var == 0)
        return launch(h, "k_route", dim3(blocks_for(n, BLOCK * M)), dim3(BLOCK), ring_lds(h),
                      k_route_m<MODE, M, NT, 0, true>, keys, n, ring_args(h), table_args(h), silo, act, status, 0ull,
                      h->route_xcd ? 1u : 0u, (const uint32_t*)nullptr, 0u, (uint32_t*)nullptr, cx_args(h), Cx8Args{});
    if (var == 2)
        return launch(h, "k_route", dim3(blocks_for(n, BLOCK * M)), dim3(BLOCK), ring_lds(h),
                      k_route_m<MODE, M, NT, 0, true, 1>, keys, n, ring_args(h), table_args(h), silo, act, status,
                      0ull, h->route_xcd ? 1u : 0u, (const uint32_t*)nullptr, 0u, (uint32_t*)nullptr, cx_args(h), Cx8Args{});
    return launch(h, "k_route", dim3(blocks_for(n, BLOCK * M)), dim3(BLOCK), ring_lds(h), k_route_m<MODE, M, NT>, keys,
                  n, ring_args(h), table_args(h), silo, act, status, 0ull, h->route_xcd ? 1u : 0u,
                  (const uint32_t*)nullptr, 0u, (uint32_t*)nullptr, CxArgs{}, Cx8Args{});
}

// The probe index up to which the routes read their key stream non-temporally (route_mode).
constexpr uint64_t ROUTE_NT_INDEX_BYTES = 64ull << 20;

// Keys given as N1 alone (u64, or u32 with n1w = 4) with one TypeCodeData (a compact exchange
// receive); not in cache mode.
template <int MODE>
int route_n1_mode(gd_handle* h, const gd_key* k, uint32_t n1w, uint64_t tcd, uint32_t n, uint32_t* silo,
                  uint32_t* act, uint8_t* status, const uint32_t* rcnt, uint32_t world, uint32_t* src) {
    const dim3 g(blocks_for(n, BLOCK)), b(BLOCK);
    const uint32_t xcd = h->route_xcd ? 1u : 0u;
    bool cx = false;
    GD_TRY(cx_ensure(h, &cx, n));
    int meas = -1;
    const int var = cx ? cx_choose(h, 1, n, &meas, h->cx8_ok ? 4 : 3) : 1;
    CxMeasure m(h, meas, n);
    // the N1 stream non-temporal under route_mode's rule (world-1 exchange pipeline: 0.5791 -> 0.5773 ms,
    // profiles/r05_route_n1_nt_ab.txt)
    const bool nt = (uint64_t)h->capacity * 8u <= ROUTE_NT_INDEX_BYTES;
    if (var == 3 && nt && n1w == 4)
        return launch(h, "k_route", g, b, ring_lds(h), k_route_m<MODE, 1, true, 4, false, (int)CX_GROUP, true>, k, n,
                      ring_args(h), table_args(h), silo, act, status, tcd, xcd, rcnt, world, src, CxArgs{},
                      cx8_args(h));
    if (var == 3 && nt)
        return launch(h, "k_route", g, b, ring_lds(h), k_route_m<MODE, 1, true, 8, false, (int)CX_GROUP, true>, k, n,
                      ring_args(h), table_args(h), silo, act, status, tcd, xcd, rcnt, world, src, CxArgs{},
                      cx8_args(h));
    if (var == 3 && n1w == 4)
        return launch(h, "k_route", g, b, ring_lds(h), k_route_m<MODE, 1, false, 4, false, (int)CX_GROUP, true>, k, n,
                      ring_args(h), table_args(h), silo, act, status, tcd, xcd, rcnt, world, src, CxArgs{},
                      cx8_args(h));
    if (var == 3)
        return launch(h, "k_route", g, b, ring_lds(h), k_route_m<MODE, 1, false, 8, false, (int)CX_GROUP, true>, k, n,
                      ring_args(h), table_args(h), silo, act, status, tcd, xcd, rcnt, world, src, CxArgs{},
                      cx8_args(h));
    if (var == 0 && n1w == 4)
        return launch(h, "k_route", g, b, ring_lds(h), k_route_m<MODE, 1, false, 4, true>, k, n, ring_args(h),
                      table_args(h), silo, act, status, tcd, xcd, rcnt, world, src, cx_args(h), Cx8Args{});
    if (var == 0)
        return launch(h, "k_route", g, b, ring_lds(h), k_route_m<MODE, 1, false, 8, true>, k, n, ring_args(h),
                      table_args(h), silo, act, status, tcd, xcd, rcnt, world, src, cx_args(h), Cx8Args{});
    if (var == 2 && n1w == 4)
        return launch(h, "k_route", g, b, ring_lds(h), k_route_m<MODE, 1, false, 4, true, 1>, k, n, ring_args(h),
                      table_args(h), silo, act, status, tcd, xcd, rcnt, world, src, cx_args(h), Cx8Args{});
    if (var == 2)
        return launch(h, "k_route", g, b, ring_lds(h), k_route_m<MODE, 1, false, 8, true, 1>, k, n, ring_args(h),
                      table_args(h), silo, act, status, tcd, xcd, rcnt, world, src, cx_args(h), Cx8Args{});
    if (n1w == 4)
        return launch(h, "k_route", g, b, ring_lds(h), k_route_m<MODE, 1, false, 4>, k, n, ring_args(h), table_args(h),
                      silo, act, status, tcd, xcd, rcnt, world, src, CxArgs{}, Cx8Args{});
    return launch(h, "k_route", g, b, ring_lds(h), k_route_m<MODE, 1, false, 8>, k, n, ring_args(h), table_args(h),
                  silo, act, status, tcd, xcd, rcnt, world, src, CxArgs{}, Cx8Args{});
}

// src (optional): also the sender rank of every message, from the per-sender counts rcnt[world].
int route_n1_device(gd_handle* h, const void* n1s, uint32_t n1w, uint64_t tcd, uint32_t n, uint32_t* silo,
                    uint32_t* act, uint8_t* status, const uint32_t* rcnt, uint32_t world,
                    uint32_t* src) {
    GD_TRY(check_ring(h));
    h->routed += n;
    const gd_key* k = reinterpret_cast<const gd_key*>(n1s);
    switch (h->ring_mode) {
        case GD_RING_DIRECTORY:
            return route_n1_mode<GD_RING_DIRECTORY>(h, k, n1w, tcd, n, silo, act, status, rcnt, world, src);
        case GD_RING_CONSISTENT:
            return route_n1_mode<GD_RING_CONSISTENT>(h, k, n1w, tcd, n, silo, act, status, rcnt, world, src);
        default: return route_n1_mode<GD_RING_VIRTUAL_BUCKETS>(h, k, n1w, tcd, n, silo, act, status, rcnt, world, src);
    }
}

// The owner's region-mapped probe (k_route_region) over m received messages: 24-B keys (n1w = 0) or
// N1s with one TypeCodeData; seg from k_region_segments.  Not in cache mode.
template <int MODE>
int route_region_mode(gd_handle* h, const void* k, uint32_t n1w, uint64_t tcd, uint32_t m, const uint32_t* seg,
                      uint32_t world, uint32_t* silo, uint32_t* act, uint8_t* status) {
    const dim3 g(N_REGIONS * std::max<uint32_t>(1, blocks_for(m, N_REGIONS * BLOCK))), b(BLOCK);
    const gd_key* kk = reinterpret_cast<const gd_key*>(k);
    if (n1w == 4)
        return launch(h, "k_route", g, b, ring_lds(h), k_route_region<MODE, 4>, kk, m, ring_args(h), table_args(h),
                      silo, act, status, tcd, seg, world);
    if (n1w == 8)
        return launch(h, "k_route", g, b, ring_lds(h), k_route_region<MODE, 8>, kk, m, ring_args(h), table_args(h),
                      silo, act, status, tcd, seg, world);
    return launch(h, "k_route", g, b, ring_lds(h), k_route_region<MODE, 0>, kk, m, ring_args(h), table_args(h), silo,
                  act, status, 0ull, seg, world);
}

int route_region_device(gd_handle* h, const void* k, uint32_t n1w, uint64_t tcd, uint32_t m, const uint32_t* seg,
                        uint32_t world, uint32_t* silo, uint32_t* act, uint8_t* status) {
    GD_TRY(check_ring(h));
    h->routed += m;
    switch (h->ring_mode) {
        case GD_RING_DIRECTORY:
            return route_region_mode<GD_RING_DIRECTORY>(h, k, n1w, tcd, m, seg, world, silo, act, status);
        case GD_RING_CONSISTENT:
            return route_region_mode<GD_RING_CONSISTENT>(h, k, n1w, tcd, m, seg, world, silo, act, status);
        default:
            return route_region_mode<GD_RING_VIRTUAL_BUCKETS>(h, k, n1w, tcd, m, seg, world, silo, act, status);
    }
}

// A cache-sized probe index (<= 64 MB of 8-B slots: BASELINE cfg 2's 16 MB): one message a thread (2
// measured no faster, profiles/r03_route_cx_ab.txt) and the 24-B key stream read non-temporally, so it
// does not push the index out of L2 (k_route 0.292 -> 0.285 ms, the step 0.415 -> 0.406 ms).  A larger
// one (cfg 3's 2 GB, its Zipf-hot part in L2 and the MALL): temporal reads (0.882 against 0.905 ms
// non-temporal; profiles/r05_route_nt_ab.txt) and two messages a thread, two dependent key -> probe
// chains in flight (0.878 -> 0.863 ms; 4: 0.963; profiles/r05_route_m_ab.txt).  act is stored
// temporally either way: the bucketing's histogram reads it next.
template <int MODE>
int route_mode(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t* silo, uint32_t* act, uint8_t* status) {
    const uint64_t index_bytes = (uint64_t)h->capacity * 8u;
    if (index_bytes <= ROUTE_NT_INDEX_BYTES) return route_launch<MODE, 1, true>(h, keys, n, silo, act, status);
    return route_launch<MODE, 2, false>(h, keys, n, silo, act, status);
}

// gd_route_bound_device: k_route_bound over the current 8-B index, with route_mode's key-stream rule.
int route_bound_device(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t* silo, uint32_t* act,
                       uint8_t* status) {
    GD_TRY(check_ring(h));
    bool cx = false;
    GD_TRY(cx_ensure(h, &cx, n));
    if (!cx || !h->cx8_ok) return set_err(h, GD_EINVAL, "route bound: the directory has no 8-B probe index");
    const uint32_t xcd = h->route_xcd ? 1u : 0u;
    const unsigned long long mask = h->capacity - 1ull;
    // two messages a thread: the fastest of the forms measured (profiles/r06_route_bound_forms.json: one
    // a thread 0.328-0.336 ms with or without the ring-staging barrier and non-temporal keys, two 0.286,
    // four 0.288; k_route 0.288)
    const bool nt = (uint64_t)h->capacity * 8u <= ROUTE_NT_INDEX_BYTES;
    const dim3 g2(blocks_for(n, BLOCK * 2));
    if (nt)
        return launch(h, "k_route_bound", g2, dim3(BLOCK), ring_lds(h), k_route_bound<2, true>, keys, n, mask,
                      cx8_args(h), silo, act, status, xcd);
    return launch(h, "k_route_bound", g2, dim3(BLOCK), ring_lds(h), k_route_bound<2, false>, keys, n, mask,
                  cx8_args(h), silo, act, status, xcd);
}


// touch = false (LocalLookup mode only): leave the batch's generation updates to the KeyExt pass
// that follows, so plain and KeyExt cache hits are numbered in one batch order.
int route_device(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t* silo, uint32_t* act, uint8_t* status,
                 bool touch) {
    GD_TRY(check_ring(h));
    h->routed += n;
    if (h->cache_max) return route_cached(h, keys, n, silo, act, status, touch);
    switch (h->ring_mode) {
        case GD_RING_DIRECTORY: return route_mode<GD_RING_DIRECTORY>(h, keys, n, silo, act, status);
        case GD_RING_CONSISTENT: return route_mode<GD_RING_CONSISTENT>(h, keys, n, silo, act, status);
        default: return route_mode<GD_RING_VIRTUAL_BUCKETS>(h, keys, n, silo, act, status);
    }
}

KxArgs kx_args(gd_handle* h) {
    return KxArgs{h->kx_slots, h->kx_cap ? h->kx_cap - 1 : 0ull, h->kx_maxp, (const uint8_t*)h->kx_heap.p,
                  (const uint32_t*)h->dir_valid.p, h->n_valid};
}

template <int MODE>
int route_keyext_t(gd_handle* h, const gd_key* keys, const ExtArgs& x, uint32_t n, uint32_t* silo, uint32_t* act,
                   uint8_t* st) {
    return launch(h, "k_route_keyext", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), ring_lds(h), k_route_keyext<MODE>,
                  keys, n, x, ring_args(h), kx_args(h), silo, act, st);
}

// The KeyExt pass (gd_keyext.h) over the messages route_device left at GD_ROUTE_KEYEXT.  In
// LocalLookup (cache) mode it follows route_device(..., touch = false) over the same batch: the
// KeyExt LocalLookup, then the generation updates of every cache hit of the batch.
int keyext_pass(gd_handle* h, const gd_key* keys, const ExtArgs& x, uint32_t n, uint32_t* silo, uint32_t* act,
                uint8_t* st) {
    if (n == 0) return GD_OK;
    if (h->cache_max) return route_cached_keyext(h, keys, x, n, silo, act, st);
    switch (h->ring_mode) {
        case GD_RING_DIRECTORY: return route_keyext_t<GD_RING_DIRECTORY>(h, keys, x, n, silo, act, st);
        case GD_RING_CONSISTENT: return route_keyext_t<GD_RING_CONSISTENT>(h, keys, x, n, silo, act, st);
        default: return route_keyext_t<GD_RING_VIRTUAL_BUCKETS>(h, keys, x, n, silo, act, st);
    }
}

int ring_owner_device(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t* silo) {
    GD_TRY(check_ring(h));
    const dim3 g(blocks_for(n, BLOCK)), b(BLOCK);
    const RingArgs r = ring_args(h);
    const TableArgs t = table_args(h);
    const size_t lds = ring_lds(h);
    switch (h->ring_mode) {
        case GD_RING_DIRECTORY:
            return launch(h, "k_ring_owner", g, b, lds, k_route<GD_RING_DIRECTORY, false>, keys, n, r, t, silo,
                          (uint32_t*)nullptr, (uint8_t*)nullptr);
        case GD_RING_CONSISTENT:
            return launch(h, "k_ring_owner", g, b, lds, k_route<GD_RING_CONSISTENT, false>, keys, n, r, t, silo,
                          (uint32_t*)nullptr, (uint8_t*)nullptr);
        default:
            return launch(h, "k_ring_owner", g, b, lds, k_route<GD_RING_VIRTUAL_BUCKETS, false>, keys, n, r, t, silo,
                          (uint32_t*)nullptr, (uint8_t*)nullptr);
    }
}

// ---- scans -------------------------------------------------------------------
// Scan of data[0..n) into out (default: in place).
template <class Op>
int scan_device(gd_handle* h, uint32_t* data, uint32_t n, bool reverse, bool inclusive, const char* tag,
                uint32_t* out) {
    if (n == 0) return GD_OK;
    if (!out) out = data;
    // too many 1,024-entry tiles to fold but few 4,096-entry ones: the wide tiles, 2 launches
    if (blocks_for(n, SCAN_TILE) > 2048 && blocks_for(n, 4 * SCAN_TILE) <= 4096) {
        const uint32_t nbw = blocks_for(n, 4 * SCAN_TILE);
        GD_TRY(ensure(h, h->partials, (size_t)nbw * sizeof(uint32_t)));
        uint32_t* part = (uint32_t*)h->partials.p;
        GD_TRY(launch(h, "k_scan_reduce", dim3(nbw), dim3(BLOCK), 0, k_scan_reduce<Op, 16>, (const uint32_t*)data, n,
                      reverse, part));
        return launch(h, "k_scan_down", dim3(nbw), dim3(BLOCK), 0, k_scan_down<Op, 16>, (const uint32_t*)data, out, n,
                      reverse, inclusive, (const uint32_t*)part, nbw);
    }
    const uint32_t nb = blocks_for(n, SCAN_TILE);
    GD_TRY(ensure(h, h->partials, (size_t)nb * sizeof(uint32_t)));
    uint32_t* part = (uint32_t*)h->partials.p;
    (void)tag;
    GD_TRY(launch(h, "k_scan_reduce", dim3(nb), dim3(BLOCK), 0, k_scan_reduce<Op>, (const uint32_t*)data, n, reverse, part));
    // few blocks (<= 2048: each block then reads <= 8 aggregates per thread): every block folds its
    // predecessors' aggregates itself (2 launches);
    // many: the aggregates are scanned in between -- by the same two-launch fold scan one level
    // up while that has <= 1024 blocks (4 launches), else by one block (3 launches)
    const bool fold = nb <= 2048;
    if (!fold) {
        const uint32_t nb2 = blocks_for(nb, SCAN_TILE);
        if (nb2 <= 1024) {
            GD_TRY(ensure(h, h->partials2, (size_t)nb2 * sizeof(uint32_t)));
            uint32_t* part2 = (uint32_t*)h->partials2.p;
            // partials are in logical order already: scan them forward, exclusive, in place
            GD_TRY(launch(h, "k_scan_reduce", dim3(nb2), dim3(BLOCK), 0, k_scan_reduce<Op>, (const uint32_t*)part, nb,
                          false, part2));
            GD_TRY(launch(h, "k_scan_down", dim3(nb2), dim3(BLOCK), 0, k_scan_down<Op>, (const uint32_t*)part, part, nb,
                          false, false, (const uint32_t*)part2, nb2));
        } else {
            GD_TRY(launch(h, "k_scan_partials", dim3(1), dim3(BLOCK), 0, k_scan_partials<Op>, part, nb));
        }
    }
    return launch(h, "k_scan_down", dim3(nb), dim3(BLOCK), 0, k_scan_down<Op>, (const uint32_t*)data, out, n, reverse,
                  inclusive, (const uint32_t*)part, fold ? nb : 0u);
}

// ---- K3 bucketing -------------------------------------------------------------
template <int BITS, int NT, int IT>
int radix_pass_t(gd_handle* h, const uint32_t* kin, const uint32_t* vin, uint32_t n, uint32_t clamp, uint32_t shift,
                 uint32_t* kout, uint32_t* vout, bool first,
                 uint32_t* offsets, uint32_t* rank_out, FillArgs fill, Pack pk) {
    constexpr uint32_t TILE = NT * IT;
    const uint32_t tiles = blocks_for(n, TILE);
    const uint32_t R = 1u << BITS;
    // the digit-major counts, then (row scans) the R digit totals
    GD_TRY(ensure(h, h->hist, ((size_t)R * tiles + R) * sizeof(uint32_t)));
    uint32_t* hist = (uint32_t*)h->hist.p;
    // below 1024 tiles, 4 per workgroup would leave fewer workgroups than the 256 CUs; up to 12,288
    // tiles (48M keys) 4 per workgroup in reverse XCD order also leaves the scatter's keys in L2
    // (f2 hop 3, 43M keys: bucketing -8%); at cfg 3's 16,384 tiles it is neutral, one stays
    const uint32_t tpb = tiles >= 1024 && tiles <= 12288 ? 4u : 1u;
    // multi-tile histograms walk the scatter's XCD tile ranges backwards (hist_t0)
    const uint32_t hxr = h->hist_xcd && h->xcd_tiles ? 1u : 0u;
    if (pk.in) {
        // packed records: the histogram reads the u16 high-key array (bucket_device enables the
        // packing only for the 512 x 8 tiles and digits of at most 8 bits)
        if constexpr (BITS <= 8 && NT == 512 && IT == 8) {
            const uint16_t* kb16 = reinterpret_cast<const uint16_t*>(vin);
            if (tpb == 4)
                GD_TRY(launch(h, "k_radix_hist", dim3(blocks_for(tiles, 4)), dim3(NT), 0, k_radix_hist16<BITS, NT, IT, 4>,
                              kb16, n, shift - pk.b1, tiles, hist, hxr));
            else
                GD_TRY(launch(h, "k_radix_hist", dim3(tiles), dim3(NT), 0, k_radix_hist16<BITS, NT, IT, 1>, kb16, n,
                              shift - pk.b1, tiles, hist, hxr));
        } else {
            return set_err(h, GD_EINVAL, "packed radix records need 512 x 8 tiles and <= 8-bit digits");
        }
    } else if constexpr (BITS <= 9) {
        if (tpb == 4)
            GD_TRY(launch(h, "k_radix_hist", dim3(blocks_for(tiles, 4)), dim3(NT), 0, k_radix_hist_multi<BITS, NT, IT, 4>,
                          kin, n, clamp, shift, tiles, hist, fill, hxr));
        else
            GD_TRY(launch(h, "k_radix_hist", dim3(tiles), dim3(NT), 0, k_radix_hist<BITS, NT, IT>, kin, n, clamp, shift,
                          tiles, hist, fill));
    } else {
        GD_TRY(launch(h, "k_radix_hist", dim3(tiles), dim3(NT), 0, k_radix_hist<BITS, NT, IT>, kin, n, clamp, shift, tiles,
                      hist, fill));
    }
    // one scan launch per digit row (the scatter adds the digit bases), or the device-wide
    // reduce + down-sweep over all R * tiles counts (GD_RADIX_ROWSCAN=0)
    const uint32_t* totals = hist + (size_t)R * tiles;
    h->last_totals = totals;
    h->last_digits = R;
    GD_TRY(launch(h, "k_radix_rowscan", dim3(R), dim3(BLOCK), 0, k_radix_rowscan, hist, tiles, hist + (size_t)R * tiles));
    if (first)
        return launch(h, "k_radix_scatter", dim3(tiles), dim3(NT), 0, k_radix_scatter<BITS, true, NT, IT>, kin, vin, n,
                      clamp, shift, tiles, (const uint32_t*)hist, kout, vout, h->radix_rank_atomic, offsets, h->xcd_tiles,
                      rank_out, totals, pk);
    return launch(h, "k_radix_scatter", dim3(tiles), dim3(NT), 0, k_radix_scatter<BITS, false, NT, IT>, kin, vin, n,
                  clamp, shift, tiles, (const uint32_t*)hist, kout, vout, h->radix_rank_atomic, offsets, h->xcd_tiles,
                  rank_out, totals, pk);
}

template <int BITS>
int radix_pass(gd_handle* h, const uint32_t* kin, const uint32_t* vin, uint32_t n, uint32_t clamp, uint32_t shift,
               uint32_t* kout, uint32_t* vout, bool first, uint32_t* offsets, uint32_t* rank_out, FillArgs fill, Pack pk) {
    // 512 threads x 8 messages (tools/ab_bucket.py: beat 256 x 16, 1024 x 4 and 512 x 16 by 10-20 %)
    return radix_pass_t<BITS, 512, 8>(h, kin, vin, n, clamp, shift, kout, vout, first, offsets, rank_out, fill, pk);
}

int radix_dispatch(gd_handle* h, int bits, const uint32_t* kin, const uint32_t* vin, uint32_t n, uint32_t clamp,
                   uint32_t shift, uint32_t* kout, uint32_t* vout, bool first,
                 uint32_t* offsets, uint32_t* rank_out, FillArgs fill, Pack pk) {
    switch (bits) {
        case 4: return radix_pass<4>(h, kin, vin, n, clamp, shift, kout, vout, first, offsets, rank_out, fill, pk);
        case 5: return radix_pass<5>(h, kin, vin, n, clamp, shift, kout, vout, first, offsets, rank_out, fill, pk);
        case 6: return radix_pass<6>(h, kin, vin, n, clamp, shift, kout, vout, first, offsets, rank_out, fill, pk);
        case 7: return radix_pass<7>(h, kin, vin, n, clamp, shift, kout, vout, first, offsets, rank_out, fill, pk);
        case 8: return radix_pass<8>(h, kin, vin, n, clamp, shift, kout, vout, first, offsets, rank_out, fill, pk);
        case 9: return radix_pass<9>(h, kin, vin, n, clamp, shift, kout, vout, first, offsets, rank_out, fill, pk);
        case 10: return radix_pass<10>(h, kin, vin, n, clamp, shift, kout, vout, first, offsets, rank_out, fill, pk);
        default: return radix_pass<11>(h, kin, vin, n, clamp, shift, kout, vout, first, offsets, rank_out, fill, pk);
    }
}

// The one-pass form's MSD pass (gd_bucket2.h): 8K-item tiles (512 threads, two workgroups a CU, 32-B
// index runs at R ~ 1,024; 65 against 76 us on 16K tiles at cfg 2), digit min(act, n_act) >> shift.
// K16: the range-local keys as u16 (the one-pass form); else the whole clamped key as u32 (pass A of
// the three-pass form).  Leaves the digit totals in last_totals.
template <int RMAX, int KOUT, bool BALLOT>
int msd_pass(gd_handle* h, const uint32_t* acts, uint32_t n, uint32_t n_act, uint32_t R, uint32_t shift, uint32_t* k1,
             uint32_t* v1, B2Pack pk = B2Pack{0, 0, 32}, uint32_t ku = 0) {
    const uint2 clamp = make_uint2(n_act, ku ? ku : n_act);      // keys >= n_act -> ku (b2_clamp)
    const uint32_t tiles = blocks_for(n, B2_TILE);
    const uint32_t hxr = h->hist_xcd && h->xcd_tiles ? 1u : 0u;
    GD_TRY(ensure(h, h->hist, ((size_t)R * tiles + R) * sizeof(uint32_t)));
    uint32_t* hist = (uint32_t*)h->hist.p;
    // 4 tiles a histogram workgroup from 1,024 tiles up (20.3 / 21.3 / 24.7 us at cfg 2 for 1 / 2 / 4,
    // profiles/r03_msd_htpb_ab.txt: 4 is the fastest; fewer tiles leave CUs idle)
    if (tiles >= 1024)
        GD_TRY(launch(h, "k_radix_hist", dim3(blocks_for(tiles, 4)), dim3(B2_NT), 0, k_b2_hist<B2_NT, B2_IT, 4, RMAX>,
                      acts, n, clamp, R, tiles, hist, shift, hxr));
    else
        GD_TRY(launch(h, "k_radix_hist", dim3(tiles), dim3(B2_NT), 0, k_b2_hist<B2_NT, B2_IT, 1, RMAX>, acts, n, clamp,
                      R, tiles, hist, shift, hxr));
    const uint32_t* tot = hist + (size_t)R * tiles;
    GD_TRY(launch(h, "k_radix_rowscan", dim3(R), dim3(BLOCK), 0, k_radix_rowscan, hist, tiles, hist + (size_t)R * tiles));
    // GD_OPT_B2_PERSIST k > 0, the one-pass form (KEY16): k persistent workgroups a CU (a multiple of 8 in
    // all), each looping over its tiles with the next tile's loads under the current write-out.  cfg 2:
    // k_radix_scatter 0.0626 -> 0.0597 ms at k = 2, 0.087 at k = 1; pass A of the three-pass form at cfg 3
    // (Zipf, 8-K tiles) 0.173 -> 0.19 ms, so that pass keeps one workgroup a tile
    // (profiles/r05_b2_persist_ab.txt).  The ballot ranks keep it too (their persistent form spills).  The
    // persistent form addresses the activations by 32-bit byte offsets: batches up to 2^30 messages.
    bool persisted = false;
    if constexpr (KOUT == B2_KEY16 && !BALLOT) if (h->b2_persist && n <= (1u << 30)) {
        const uint32_t grid = std::min<uint32_t>(tiles, std::max<uint32_t>(8, (h->b2_persist * h->n_cu) & ~7u));
        GD_TRY(launch(h, "k_radix_scatter", dim3(grid), dim3(B2_NT), 0,
                      k_b2_scatter<B2_NT, B2_IT, RMAX, KOUT, BALLOT, true>, acts, n, clamp, R, tiles,
                      (const uint32_t*)hist, tot, k1, v1, shift, h->xcd_tiles, pk, h->b2_order));
        persisted = true;
    }
    if (!persisted)
        GD_TRY(launch(h, "k_radix_scatter", dim3(tiles), dim3(B2_NT), 0, k_b2_scatter<B2_NT, B2_IT, RMAX, KOUT, BALLOT>,
                      acts, n, clamp, R, tiles, (const uint32_t*)hist, tot, k1, v1, shift, h->xcd_tiles, pk, 0u));
    h->last_totals = tot;
    h->last_digits = R;
    return GD_OK;
}

// The one-pass two-level bucketing (gd_msd.h): a stable MSD pass on the high digit min(act, n_act) >> 10,
// then k_msd_local sorts each 1,024-activation range in LDS and writes its starts.  Needs (n_act >> 10)
// + 1 <= B2_RMAX2.
template <bool BALLOT>
int msd_bucket(gd_handle* h, const uint32_t* acts, uint32_t n, uint32_t n_act, uint32_t* perm, uint32_t* offsets,
               uint32_t* rank_out) {
    // The MSD pass clamps the keys at ku, the first key of a range past n_act's, rather than at n_act: the
    // unrouted messages (act >= n_act: directory misses, which a directory under churn sends in numbers)
    // get a range of their own, copied in order (msd_range_kp, L <= 1), instead of turning n_act's range
    // into a hot one ranked in chunks by one workgroup (1 % misses at cfg 2: k_msd_local 0.045 ->
    // 0.47 ms, tools/churn_probe.py).
    const uint32_t ku = msd_unrouted_key(n_act);
    const uint32_t R = (ku >> MSD_SHIFT) + 1;
    if (R > MSD_MAX_RANGES) return set_err(h, GD_EINVAL, "two-level bucketing: n_act too large");
    GD_TRY(ensure(h, h->u32_a, (size_t)n * 4));
    GD_TRY(ensure(h, h->u32_c, (size_t)n * 4));
    uint32_t* k1 = (uint32_t*)h->u32_a.p;
    uint32_t* v1 = (uint32_t*)h->u32_c.p;
    GD_TRY((msd_pass<B2_RMAX2, B2_KEY16, BALLOT>(h, acts, n, n_act, R, MSD_SHIFT, k1, v1, B2Pack{0, 0, 32}, ku)));
    return launch(h, "k_msd_local", dim3(std::min<uint32_t>(R, h->n_cu)), dim3(MSD_NT), 0, k_msd_local<BALLOT>,
                  (const uint16_t*)k1, (const uint32_t*)v1, h->last_totals, R, n, n_act, perm, offsets, rank_out);
}

// Three-pass form's split of k' = n_act >> 10: pass B's digit bits a (low part), pass A's kb - a.
// False when the one-pass form applies or k' needs more than 18 bits (n_act >= 2^28).
bool msd3_split(uint32_t n_act, uint32_t* a_out, uint32_t* ra_out) {
    const uint32_t km = n_act >> MSD_SHIFT;
    if (km + 1 <= MSD_MAX_RANGES) return false;
    uint32_t kb = 0;
    while (kb < 32 && (km >> kb) != 0) ++kb;
    if (kb > 18) return false;
    // pass B takes the smaller half: a 17-bit k' (BASELINE cfg 3) as 9 + 8 bits, pass B's 256 digits
    // writing twice the run length of 512 (k_seg_scatter 0.240 -> 0.218 ms, step 2.094 -> 2.035 ms,
    // profiles/r04_msd3_split_ab.jsonl)
    const uint32_t a = kb / 2;
    *a_out = a;
    *ra_out = (km >> a) + 1;
    return true;
}

// The three-pass two-level bucketing (gd_msd2.h), for n_act past the one-pass form's digit: pass A
// (MSD on d2 = k' >> a), pass B (segmented MSD on d1 = k' & (2^a - 1), one flat scan for the
// positions), then the level-2 work lists (thin ranges a wave each, staged ranges a workgroup each,
// hot ranges in chunks).  Grids of the level-2 kernels are bounded and loop over device-side counts.
template <bool BALLOT>
int msd3_bucket(gd_handle* h, const uint32_t* acts, uint32_t n, uint32_t n_act, uint32_t* perm, uint32_t* offsets,
                uint32_t* rank_out) {
    uint32_t a = 0, RA = 0;
    if (!msd3_split(n_act, &a, &RA)) return set_err(h, GD_EINVAL, "three-pass bucketing: n_act out of range");
    const uint32_t R = (n_act >> MSD_SHIFT) + 1, RB = 1u << a;
    const uint32_t tilesA = blocks_for(n, B2_TILE);
    const uint32_t tbound = blocks_for(n, SEG_TILE) + RA;
    // ranges past t_staged messages are chunked (k_l2_classify): at most n / (t_staged + 1) of them,
    // whatever GD_OPT_L2_STAGED / GD_OPT_L2_SMALL say
    const uint32_t t_staged = std::max(h->l2_small, h->l2_staged);
    const uint32_t cr_bound = std::min(R, n / (t_staged + 1) + 1);
    const uint32_t ch_bound = n / CH_CAP + cr_bound;
    GD_TRY(ensure(h, h->u32_a, (size_t)n * 4));
    GD_TRY(ensure(h, h->u32_b, (size_t)n * 4));
    GD_TRY(ensure(h, h->u32_c, (size_t)n * 4));
    GD_TRY(ensure(h, h->u32_d, (size_t)n * 4));
    DevBuf* m = h->m3;
    GD_TRY(ensure(h, m[0], (size_t)(RA + 1) * 4));                 // segment starts
    GD_TRY(ensure(h, m[1], (size_t)(RA + 1) * 4));                 // segment tile bases
    GD_TRY(ensure(h, m[2], (size_t)tbound * 4));                   // tile -> segment
    GD_TRY(ensure(h, m[3], (size_t)RB * tbound * 4));              // pass B counts, flat-scanned
    GD_TRY(ensure(h, m[4], (size_t)(R + 1) * 4));                  // range starts
    GD_TRY(ensure(h, m[5], (size_t)L2_CTR_WORDS * 4));
    GD_TRY(ensure(h, m[6], (size_t)R * 4));                        // thin ranges
    GD_TRY(ensure(h, m[7], (size_t)R * 4));                        // staged ranges
    GD_TRY(ensure(h, m[14], (size_t)R * 4));                       // mid ranges
    GD_TRY(ensure(h, m[8], (size_t)cr_bound * 4 * 4));             // chunked ranges
    // chunk-scan items: 1 a range of <= CS_DIRECT chunks, else CS_SLABS a piece of CS_ROWS chunks
    const uint32_t it_bound = cr_bound + CS_SLABS * (ch_bound / CS_DIRECT + blocks_for(ch_bound, CS_ROWS));
    GD_TRY(ensure(h, m[13], (size_t)it_bound * 4));
    GD_TRY(ensure(h, m[9], (size_t)ch_bound * 4));                 // chunk -> chunked range
    GD_TRY(ensure(h, m[10], (size_t)ch_bound * MSD_L * 4));        // per-chunk activation counts
    GD_TRY(ensure(h, m[11], (size_t)cr_bound * MSD_L * 4));        // per-range activation totals
    GD_TRY(ensure(h, m[12], (size_t)it_bound * CS_COLS * 4));        // per-item (slab x piece) column sums
    uint32_t* kA = (uint32_t*)h->u32_a.p;
    uint32_t* vA = (uint32_t*)h->u32_c.p;
    uint16_t* kB = (uint16_t*)h->u32_b.p;
    uint32_t* vB = (uint32_t*)h->u32_d.p;
    uint32_t* seg_start = (uint32_t*)m[0].p;
    uint32_t* seg_tb = (uint32_t*)m[1].p;
    uint32_t* tile_seg = (uint32_t*)m[2].p;
    uint32_t* hseg = (uint32_t*)m[3].p;
    (void)tilesA;
    // pass A: d2 = k' >> a.  Pass B needs the key's low a + 10 bits P: as a u16 of P's high bits with
    // the hb bits below them in the index word's spare top bits (6-B records) when the index leaves
    // room (BASELINE cfg 3: P 19 bits, 26-bit indices), else the whole key (8-B records)
    uint32_t ib = 1;
    while (ib < 32 && ((n - 1) >> ib) != 0) ++ib;
    const uint32_t pbits = a + MSD_SHIFT, hb = pbits > 16 ? pbits - 16 : 0;
    const bool pk = hb == 0 || ib + hb <= 32;
    const B2Pack bp{pbits, hb, hb ? ib : 32u};
    if (pk) GD_TRY((msd_pass<SEG_RMAX, B2_PACK, BALLOT>(h, acts, n, n_act, RA, MSD_SHIFT + a, kA, vA, bp)));
    else GD_TRY((msd_pass<SEG_RMAX, B2_KEY32, BALLOT>(h, acts, n, n_act, RA, MSD_SHIFT + a, kA, vA)));
    const SegIn in{(const uint16_t*)kA, (const uint32_t*)kA, (const uint32_t*)vA, hb, bp.ib};
    GD_TRY(launch(h, "k_seg_table", dim3(blocks_for(tbound, 1024)), dim3(1024), 0, k_seg_table, h->last_totals, RA, tbound, seg_start, seg_tb,
                  tile_seg, (uint32_t*)m[5].p));
    // pass B: d1 inside each d2 segment; one flat scan gives every (segment, digit, tile) its position
    if (pk)
        GD_TRY(launch(h, "k_seg_hist", dim3(tbound), dim3(SEG_NT), 0, k_seg_hist<true>, in, (const uint32_t*)tile_seg,
                      (const uint32_t*)seg_start, (const uint32_t*)seg_tb, RB, hseg));
    else
        GD_TRY(launch(h, "k_seg_hist", dim3(tbound), dim3(SEG_NT), 0, k_seg_hist<false>, in, (const uint32_t*)tile_seg,
                      (const uint32_t*)seg_start, (const uint32_t*)seg_tb, RB, hseg));
    GD_TRY(scan_device<OpAdd>(h, hseg, RB * tbound, false, false, "seg"));
    if (pk)
        GD_TRY(launch(h, "k_seg_scatter", dim3(tbound), dim3(SEG_NT), 0, k_seg_scatter<true, BALLOT>, in,
                      (const uint32_t*)tile_seg, (const uint32_t*)seg_start, (const uint32_t*)seg_tb, RB,
                      (const uint32_t*)hseg, kB, vB, h->xcd_tiles));
    else
        GD_TRY(launch(h, "k_seg_scatter", dim3(tbound), dim3(SEG_NT), 0, k_seg_scatter<false, BALLOT>, in,
                      (const uint32_t*)tile_seg, (const uint32_t*)seg_start, (const uint32_t*)seg_tb, RB,
                      (const uint32_t*)hseg, kB, vB, h->xcd_tiles));
    // level 2
    uint32_t* cr = (uint32_t*)m[8].p;
    const L2Lists l{(uint32_t*)m[4].p, (uint32_t*)m[6].p, (uint32_t*)m[7].p, (uint32_t*)m[14].p, cr, cr + cr_bound,
                    cr + 2 * cr_bound,
                    (uint32_t*)m[9].p, cr + 3 * cr_bound, (uint32_t*)m[13].p, (uint32_t*)m[5].p};
    GD_TRY(launch(h, "k_l2_classify", dim3(blocks_for(R, CL_NT)), dim3(CL_NT), 0, k_l2_classify, (const uint32_t*)hseg,
                  (const uint32_t*)seg_start, (const uint32_t*)seg_tb, a, R, n, h->l2_small,
                  std::max(h->l2_small, h->l2_mid), t_staged, l));
    // persistent grids sized to what the chip holds at once (a second round of workgroups would wait for
    // the first to finish its whole share): k_l2_small 4 a CU (32 KB of LDS, 8 waves each), the range
    // sort 1 a CU (135 KB), the chunk scatter 2 (72 KB), the chunk histogram 4 and the scan 2 a CU
    const uint32_t cu8 = (h->n_cu + 7) & ~7u;
    GD_TRY(launch(h, "k_l2_small", dim3(std::min<uint32_t>(blocks_for(R, L2_SMALL_WAVES), 4 * cu8)),
                  dim3(L2_SMALL_WAVES * WAVE), 0, k_l2_small<BALLOT>, (const uint16_t*)kB, (const uint32_t*)vB, l, n, n_act, perm,
                  offsets, rank_out));
    GD_TRY(launch(h, "k_msd_local_mid", dim3(std::min<uint32_t>(R, 3 * cu8)), dim3(MSD_MID_NT), 0,
                  k_msd_local_list<MSD_MID_NT, MSD_MID_RW, BALLOT>, (const uint16_t*)kB, (const uint32_t*)vB,
                  (const uint32_t*)l.rs, (const uint32_t*)l.mid, (const uint32_t*)(l.ctr + 5), n, n_act, perm, offsets,
                  rank_out));
    GD_TRY(launch(h, "k_msd_local", dim3(std::min<uint32_t>(R, cu8)), dim3(MSD_NT), 0, k_msd_local_list<MSD_NT, MSD_RW, BALLOT>,
                  (const uint16_t*)kB, (const uint32_t*)vB, (const uint32_t*)l.rs, (const uint32_t*)l.staged,
                  (const uint32_t*)(l.ctr + 1), n, n_act, perm, offsets, rank_out));
    uint32_t* hh = (uint32_t*)m[10].p;
    uint32_t* tot = (uint32_t*)m[11].p;
    // the chunk grids are multiples of 8 (chunk_walk: one contiguous chunk range an XCD)
    GD_TRY(launch(h, "k_l2_chunk_hist", dim3(4 * cu8), dim3(CH_NT), 0, k_l2_chunk_hist,
                  (const uint16_t*)kB, l, hh));
    uint32_t* ptot = (uint32_t*)m[12].p;
    GD_TRY(launch(h, "k_l2_chunk_ptot", dim3(2 * cu8), dim3(MSD_NT), 0, k_l2_chunk_ptot, l, (const uint32_t*)hh, ptot));
    GD_TRY(launch(h, "k_l2_chunk_scan", dim3(2 * cu8), dim3(MSD_NT), 0, k_l2_chunk_scan, l, hh, (const uint32_t*)ptot,
                  tot));
    return launch(h, "k_l2_chunk_scatter", dim3(2 * cu8), dim3(CH_NT), 0, k_l2_chunk_scatter<BALLOT>,
                  (const uint16_t*)kB, (const uint32_t*)vB, l, (const uint32_t*)hh, (const uint32_t*)tot, n, n_act, perm,
                  offsets, rank_out);
}


// Stable partition of indices 0..n-1 by min(acts[i], n_act).  rank_out (optional): the inverse
// permutation, rank_out[perm[p]] = p.  Forms with identical output: LSD passes of <= 8 bits plus the
// bucket starts (bucket_lsd); for batches of at least 2^20 messages the two-level forms -- one MSD pass
// + the in-LDS range sort for n_act < 1056 x 1024 (msd_bucket), two MSD passes + the level-2 work lists
// up to n_act < 2^28 (msd3_bucket).  GD_MSD=1 (default) times the two-level form against the LSD
// passes on the first launches of each batch shape (tune_choose, kind 4) and keeps the faster, 2
// always takes the two-level form.
int bucket_device(gd_handle* h, const uint32_t* acts, uint32_t n, uint32_t n_act, uint32_t* perm, uint32_t* offsets,
                  uint32_t* rank_out) {
    if (n_act == 0xFFFFFFFFu) return set_err(h, GD_EINVAL, "n_act too large");
    if (h->bstream && h->bstream != h->stream) {
        // the bucketing scratch is the bucket stream's (gd_set_bucket_stream): a bucketing enqueued on
        // another stream waits for it
        HIP_TRY(h, hipEventRecord(h->b_ev, h->bstream));
        HIP_TRY(h, hipStreamWaitEvent(h->stream, h->b_ev, 0));
    }
    StageTime stage(h, "stage:bucket");
    uint32_t a3 = 0, ra3 = 0;
    const bool one = (msd_unrouted_key(n_act) >> MSD_SHIFT) + 1 <= MSD_MAX_RANGES;
    const bool three = !one && msd3_split(n_act, &a3, &ra3);
    if (h->msd_mode && n >= (1u << 20) && (one || three)) {
        int meas = -1;
        // keyed by the batch size and by the messages a range holds (which decide whether ranges are
        // staged in LDS): a handle bucketing 16M messages over 1M and over 10k activations keeps one
        // choice for each
        const int per_range = bucket_sub(n, n_act);
        const int var = h->msd_mode == 2 ? 1 : tune_choose(h, 4, n, &meas, 2, per_range);
        CxMeasure mm(h, meas, n);
        // ranks by ds_add_rtn lane order (default) or by ballots (GD_OPT_STABLE_RANK 0; gd_create's
        // choice on a device without that order)
        if (var == 1 && h->radix_rank_atomic)
            return one ? msd_bucket<false>(h, acts, n, n_act, perm, offsets, rank_out)
                       : msd3_bucket<false>(h, acts, n, n_act, perm, offsets, rank_out);
        if (var == 1)
            return one ? msd_bucket<true>(h, acts, n, n_act, perm, offsets, rank_out)
                       : msd3_bucket<true>(h, acts, n, n_act, perm, offsets, rank_out);
        return bucket_lsd(h, acts, n, n_act, perm, offsets, rank_out);
    }
    return bucket_lsd(h, acts, n, n_act, perm, offsets, rank_out);
}

constexpr uint32_t RADIX_MAX_BITS = 8;   // widest LSD digit (9- and 10-bit digits measured slower at cfg 3)

int bucket_lsd(gd_handle* h, const uint32_t* acts, uint32_t n, uint32_t n_act, uint32_t* perm, uint32_t* offsets,
               uint32_t* rank_out) {
    const uint32_t n_off = n_act + 2;
    if (n == 0) return launch(h, "k_fill", dim3(blocks_for(n_off, BLOCK)), dim3(BLOCK), 0, k_fill_u32, offsets, n_off, n);
    // the first pass's histogram fills the starts (n = the empty-bucket value)
    const FillArgs fill{offsets, n_off, n};
    uint32_t key_bits = 1;
    while (key_bits < 32 && (n_act >> key_bits) != 0) ++key_bits;
    const uint32_t passes = (key_bits + RADIX_MAX_BITS - 1) / RADIX_MAX_BITS;
    const uint32_t bits = std::max<uint32_t>(4, (key_bits + passes - 1) / passes);
    GD_TRY(ensure(h, h->u32_a, (size_t)n * 4));
    GD_TRY(ensure(h, h->u32_b, (size_t)n * 4));
    GD_TRY(ensure(h, h->u32_c, (size_t)n * 4));
    GD_TRY(ensure(h, h->u32_d, (size_t)n * 4));
    uint32_t* kb[2] = {(uint32_t*)h->u32_a.p, (uint32_t*)h->u32_b.p};
    uint32_t* vb[2] = {(uint32_t*)h->u32_c.p, (uint32_t*)h->u32_d.p};
    const uint32_t* kin = acts;
    const uint32_t* vin = nullptr;
    // packed records between the passes (gd_kernels.h Pack): the key bits above the first digit fit
    // a u16 and the index fits beside the first digit in a u32 (BASELINE cfg 2: 14 + 24 + 7 bits)
    uint32_t ib = 1;
    while (ib < 32 && ((n - 1) >> ib) != 0) ++ib;
    const bool pack = passes >= 2 && bits <= 8 &&
                      key_bits - bits <= 16 && ib + bits <= 32;
    for (uint32_t p = 0; p < passes; ++p) {
        uint32_t* kout = kb[p & 1];
        uint32_t* vout = (p + 1 == passes) ? perm : vb[p & 1];
        // the last pass writes the bucket starts itself (no sorted keys, no k_bucket_starts)
        const bool last = p + 1 == passes;
        const Pack pk{ib, bits, pack && p > 0, pack && p + 1 < passes};
        GD_TRY(radix_dispatch(h, (int)bits, kin, vin, n, n_act, p * bits, kout, vout, p == 0,
                              last ? offsets : nullptr, p + 1 == passes ? rank_out : nullptr,
                              p == 0 ? fill : FillArgs{nullptr, 0u, 0u}, pk));
        kin = kout;
        vin = vout;
    }
    // the last pass's digit spans <= RS_RANGE * RS_MAX_SUB activations: one workgroup per digit
    // range, carried by the pass's digit bases (GD_RANGE_SCAN=0: the device-wide scan)
    const uint32_t last_shift = (passes - 1) * bits;
    if (h->last_totals && last_shift < 32 && (1u << last_shift) <= RS_RANGE * RS_MAX_SUB)
        return launch(h, "k_starts_rangescan", dim3((n_act >> last_shift) + 1), dim3(RS_THREADS), 0, k_starts_rangescan,
                      offsets, n_act + 1, last_shift, h->last_totals, h->last_digits);
    return scan_device<OpMin>(h, offsets, n_act + 1, true, true, "offsets");
}


int sync(gd_handle* h) {
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    if (h->bstream && h->bstream != h->stream) HIP_TRY(h, hipStreamSynchronize(h->bstream));
    return GD_OK;
}

// h->h_pin holds at least `bytes` (page-locked: the small read-backs are true async copies).
int pinned_scratch(gd_handle* h, size_t bytes) {
    if (h->h_pin_bytes >= bytes) return GD_OK;
    if (h->h_pin) {
        HIP_TRY(h, hipStreamSynchronize(h->stream));
        HIP_TRY(h, hipHostFree(h->h_pin));
        h->h_pin = nullptr;
        h->h_pin_bytes = 0;
    }
    const size_t b = std::max<size_t>(bytes, 64 * 1024);
    HIP_TRY(h, hipHostMalloc(&h->h_pin, b));
    h->h_pin_bytes = b;
    return GD_OK;
}

// Surface device-side error bits after a synchronising call.
int sync_checked(gd_handle* h) {
    GD_TRY(pull_counters(h));
    if (h->ctr_host.err) {
        const uint32_t e = h->ctr_host.err;
        HIP_TRY(h, hipMemsetAsync(&h->ctr->err, 0, sizeof(uint32_t), h->stream));
        GD_TRY(sync(h));
        if (e == ERR_CTX_RANGE)
            return set_err(h, GD_EINVAL, "an ActivationDirectory entry's context index is not below n_ctx");
        if (e & ERR_UNSETTLED)
            return set_err(h, GD_ETIMEOUT, "an asynchronous registration's claims did not settle (device bits 0x%x)", e);
        return set_err(h, GD_EFULL, "device error bits 0x%x", e);
    }
    return GD_OK;
}

// maybe_grow_table without the read-back while the last copy of the counters is current (no untracked
// table write since) and, with every asynchronous registration since counted as new entries, the table
// stays at load <= 0.75.
int maybe_grow_async(gd_handle* h, uint64_t incoming) {
    if (!h->ctr_stale) {
        const unsigned long long used = h->ctr_host.live + h->ctr_host.tomb + h->pending_in + incoming;
        if (used * 4 <= h->capacity * 3) return GD_OK;
    }
    return maybe_grow_table(h, incoming);
}

int maybe_grow_table(gd_handle* h, uint64_t incoming) {
    GD_TRY(pull_counters(h));
    const unsigned long long used = h->ctr_host.live + h->ctr_host.tomb + incoming;
    if (used * 4 <= h->capacity * 3) return GD_OK;  // keep load <= 0.75
    unsigned long long cap = h->capacity;
    while ((h->ctr_host.live + incoming) * 2 > cap) cap <<= 1;
    return gd_dir_rehash(h, cap);
}

// ---- exchange partition (gd_shard.h) -------------------------------------------------
template <int MODE, bool NODES>
int shard_hist_t(gd_handle* h, const void* recs, uint32_t n, uint64_t tcd, uint32_t n_shards, uint32_t bits,
                 uint32_t tiles, uint8_t* dest, uint32_t* hist, const ExtArgs& ext, uint32_t* kdesc, uint32_t regions) {
    uint32_t* n1lo = !NODES && kdesc && h->shard_n1_copy ? (uint32_t*)h->shard_n1.p : nullptr;
    if (!NODES && !ext.len)           // no KeyExt strings in the batch: the instantiation without their path
        return launch(h, "k_shard_hist", dim3(tiles), dim3(SH_NT), ring_lds(h), k_shard_hist<MODE, NODES, false>, recs,
                      n, tcd, ring_args(h), n_shards, bits, tiles, dest, hist, ext, kdesc, n1lo, regions);
    return launch(h, "k_shard_hist", dim3(tiles), dim3(SH_NT), ring_lds(h), k_shard_hist<MODE, NODES>, recs, n, tcd,
                  ring_args(h), n_shards, bits, tiles, dest, hist, ext, kdesc, n1lo, regions);
}

template <int BITS, bool NODES>
int shard_scatter_t(gd_handle* h, const void* recs, const uint32_t* payload, const uint8_t* dest, uint32_t n,
                    uint32_t n_shards, uint32_t tiles, const uint32_t* gscan, void* out, uint32_t* out_pay,
                    const uint32_t* kdesc) {
    // keys with a compaction descriptor: the compact case by k_shard_gather, the other by the staged
    // kernel (each returns at once in the other's case)
    if constexpr (!NODES)
        if (h->pack_pay16) {         // route_multi's 2-B origin indices (KD_IDX16); keys with a descriptor
            uint16_t* op = reinterpret_cast<uint16_t*>(out_pay);
            if (h->shard_gather)
                GD_TRY(launch(h, "k_shard_scatter", dim3(tiles), dim3(SH_NT), 0, k_shard_gather<BITS, uint16_t>,
                              (const gd_key*)recs, payload, dest, n, n_shards, tiles, gscan, out, op, kdesc,
                              h->shard_n1_copy ? (const uint32_t*)h->shard_n1.p : nullptr));
            if (h->shard_gather)
                return launch(h, "k_shard_scatter", dim3(tiles), dim3(SH_NT), 0,
                              k_shard_scatter<BITS, false, true, uint16_t>, recs, payload, dest, n, n_shards, tiles,
                              gscan, out, op, kdesc);
            return launch(h, "k_shard_scatter", dim3(tiles), dim3(SH_NT), 0, k_shard_scatter<BITS, false, false, uint16_t>,
                          recs, payload, dest, n, n_shards, tiles, gscan, out, op, kdesc);
        }
    if constexpr (!NODES)
        if (h->shard_gather && kdesc) {
            GD_TRY(launch(h, "k_shard_scatter", dim3(tiles), dim3(SH_NT), 0, k_shard_gather<BITS>,
                          (const gd_key*)recs, payload, dest, n, n_shards, tiles, gscan, out, out_pay, kdesc,
                          h->shard_n1_copy ? (const uint32_t*)h->shard_n1.p : nullptr));
            return launch(h, "k_shard_scatter", dim3(tiles), dim3(SH_NT), 0, k_shard_scatter<BITS, false, true>, recs,
                          payload, dest, n, n_shards, tiles, gscan, out, out_pay, kdesc);
        }
    return launch(h, "k_shard_scatter", dim3(tiles), dim3(SH_NT), 0, k_shard_scatter<BITS, NODES>, recs, payload, dest,
                  n, n_shards, tiles, gscan, out, out_pay, kdesc);
}

template <bool NODES>
int shard_finish(gd_handle* h, const void* recs, const uint32_t* payload, uint32_t n, uint32_t n_shards, uint32_t bits,
                 uint32_t tiles, const uint8_t* dest, uint32_t* hist, void* out_recs, uint32_t* out_pay,
                 uint32_t* counts, const uint32_t* kdesc = nullptr, uint32_t group = 1);

// Stable partition of n records (gd_key or u32 node ids) by destination rank, payload alongside
// (payload == nullptr: the batch index); counts[d] per destination.  kdesc != nullptr (keys): the
// header-compaction descriptor (k_key_desc) is built, and a compact batch is written as N1 only.
// regions = N_REGIONS (keys): each rank's chunk is ordered by the grains' table region on the owner
// (then batch order), for the owner's region-mapped probe; counts stay per rank.
template <bool NODES>
int shard_pack(gd_handle* h, const void* recs, const uint32_t* payload, uint32_t n, uint64_t tcd, uint32_t n_shards,
               void* out_recs, uint32_t* out_pay, uint32_t* counts, const ExtArgs& ext,
               uint32_t* kdesc, uint32_t regions) {
    GD_TRY(check_ring(h));
    if (kdesc) HIP_TRY(h, hipMemsetAsync(kdesc, 0, 16, h->stream));
    if (n == 0) {
        if (kdesc)
            GD_TRY(launch(h, "k_key_desc", dim3(1), dim3(64), 0, k_key_desc, (const gd_key*)recs, n, kdesc,
                          h->narrow_headers ? 1u : 0u));
        return launch(h, "k_fill", dim3(1), dim3(BLOCK), 0, k_fill_u32, counts, n_shards, 0u);
    }
    if (NODES || n_shards * regions > 256) regions = 1;
    const uint32_t n_dest = n_shards * regions;
    const uint32_t tiles = blocks_for(n, SH_TILE);
    if ((uint64_t)tiles * n_dest > 0xFFFFFFFFull) return set_err(h, GD_EINVAL, "batch too large to partition");
    GD_TRY(ensure(h, h->shard_dest, (size_t)n));
    GD_TRY(ensure(h, h->shard_hist, (size_t)tiles * n_dest * 4));
    if (!NODES && kdesc) GD_TRY(ensure(h, h->shard_n1, (size_t)n * 4));
    uint8_t* dest = (uint8_t*)h->shard_dest.p;
    uint32_t* hist = (uint32_t*)h->shard_hist.p;
    uint32_t bits = 1;
    while ((1u << bits) < n_dest) ++bits;
    switch (h->ring_mode) {
        case GD_RING_DIRECTORY:
            GD_TRY((shard_hist_t<GD_RING_DIRECTORY, NODES>(h, recs, n, tcd, n_shards, bits, tiles, dest, hist, ext, kdesc,
                                                           regions)));
            break;
        case GD_RING_CONSISTENT:
            GD_TRY((shard_hist_t<GD_RING_CONSISTENT, NODES>(h, recs, n, tcd, n_shards, bits, tiles, dest, hist, ext,
                                                            kdesc, regions)));
            break;
        default:
            GD_TRY((shard_hist_t<GD_RING_VIRTUAL_BUCKETS, NODES>(h, recs, n, tcd, n_shards, bits, tiles, dest, hist,
                                                                 ext, kdesc, regions)));
    }
    return shard_finish<NODES>(h, recs, payload, n, n_shards, bits, tiles, dest, hist, out_recs, out_pay, counts,
                               kdesc, regions);
}

// Forward partition of routed messages by the rank hosting their activation (k_fwd_hist): keys
// move, out_pos[j] = the message's position in the input.
// n1 (optional): the messages' keys are u32 N1s (one TypeCodeData, N0 = 0) and move as such.
int fwd_pack(gd_handle* h, const gd_key* keys, const uint8_t* st, const uint32_t* silo, uint32_t n, uint32_t n_shards,
             uint32_t my_rank, void* out_keys, uint32_t* out_pos, uint32_t* counts, const uint32_t* n1) {
    if (n == 0)
        return launch(h, "k_fill", dim3(1), dim3(BLOCK), 0, k_fill_u32, counts, n_shards, 0u);
    const uint32_t tiles = blocks_for(n, SH_TILE);
    if ((uint64_t)tiles * n_shards > 0xFFFFFFFFull) return set_err(h, GD_EINVAL, "batch too large to partition");
    GD_TRY(ensure(h, h->shard_dest, (size_t)n));
    GD_TRY(ensure(h, h->shard_hist, (size_t)tiles * n_shards * 4));
    uint8_t* dest = (uint8_t*)h->shard_dest.p;
    uint32_t* hist = (uint32_t*)h->shard_hist.p;
    uint32_t bits = 1;
    while ((1u << bits) < n_shards) ++bits;
    GD_TRY(launch(h, "k_fwd_hist", dim3(tiles), dim3(SH_NT), 0, k_fwd_hist, st, silo, n, n_shards, my_rank, bits, tiles,
                  dest, hist));
    if (n1) return shard_finish<true>(h, n1, nullptr, n, n_shards, bits, tiles, dest, hist, out_keys, out_pos, counts);
    return shard_finish<false>(h, keys, nullptr, n, n_shards, bits, tiles, dest, hist, out_keys, out_pos, counts);
}

template <bool NODES>
int shard_finish(gd_handle* h, const void* recs, const uint32_t* payload, uint32_t n, uint32_t n_shards, uint32_t bits,
                 uint32_t tiles, const uint8_t* dest, uint32_t* hist, void* out_recs, uint32_t* out_pay,
                 uint32_t* counts, const uint32_t* kdesc, uint32_t group) {
    GD_TRY(scan_device<OpAdd>(h, hist, tiles * n_shards * group, false, false, "shard"));
    // k_shard_counts also completes the compaction descriptor (kdesc, keys only)
    GD_TRY(launch(h, "k_shard_counts", dim3(1), dim3(256), 0, k_shard_counts, (const uint32_t*)hist, tiles, n_shards, n,
                  counts, NODES ? nullptr : (const gd_key*)recs, NODES ? nullptr : const_cast<uint32_t*>(kdesc),
                  h->narrow_headers ? 1u : 0u, group));
    const uint32_t* gs = hist;
    n_shards *= group;                  // the scatter's destinations: (rank, region) pairs
    switch (bits) {
        case 1: return shard_scatter_t<1, NODES>(h, recs, payload, dest, n, n_shards, tiles, gs, out_recs, out_pay,
                                                   kdesc);
        case 2: return shard_scatter_t<2, NODES>(h, recs, payload, dest, n, n_shards, tiles, gs, out_recs, out_pay,
                                                   kdesc);
        case 3: return shard_scatter_t<3, NODES>(h, recs, payload, dest, n, n_shards, tiles, gs, out_recs, out_pay,
                                                   kdesc);
        case 4: return shard_scatter_t<4, NODES>(h, recs, payload, dest, n, n_shards, tiles, gs, out_recs, out_pay,
                                                   kdesc);
        case 5: return shard_scatter_t<5, NODES>(h, recs, payload, dest, n, n_shards, tiles, gs, out_recs, out_pay,
                                                   kdesc);
        case 6: return shard_scatter_t<6, NODES>(h, recs, payload, dest, n, n_shards, tiles, gs, out_recs, out_pay,
                                                   kdesc);
        case 7: return shard_scatter_t<7, NODES>(h, recs, payload, dest, n, n_shards, tiles, gs, out_recs, out_pay,
                                                   kdesc);
        default: return shard_scatter_t<8, NODES>(h, recs, payload, dest, n, n_shards, tiles, gs, out_recs, out_pay,
                                                  kdesc);
    }
}

// Page-locked host memory (hipHostMalloc / gd_host_alloc / hipHostRegister): copies from it are
// asynchronous.  From pageable memory HIP stages every copy, and the chunked pipeline measured
// slower than one copy each way (1.35 vs 1.42 G messages/s at cfg 2).
bool host_pinned(const void* p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// Host buffers, large batch: the PCIe copies overlap the kernels.  Chunk k's keys go up on the
// copy-in stream while chunk k-1 is probed on the handle's stream and chunk k-2's routes come
// down on the copy-out stream (PCIe is full duplex); the bucketing needs the whole batch, so only
// perm and offsets are copied after it.  Bounded by the 24-B-a-message upload instead of the sum
// of both directions.  Used when the caller's buffers are pinned (gd_host_alloc).  out_perm ==
// nullptr: gd_route (routes only, no bucketing).
int route_bucket_host_pipelined(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t n_act, uint32_t* out_silo,
                                uint32_t* out_act, uint8_t* out_status, uint32_t* out_perm, uint32_t* out_offsets) {
    if (!h->cin) HIP_TRY(h, hipStreamCreateWithFlags(&h->cin, hipStreamNonBlocking));
    if (!h->cout) HIP_TRY(h, hipStreamCreateWithFlags(&h->cout, hipStreamNonBlocking));
    const uint32_t C = h->host_chunk;
    const uint32_t nch = (uint32_t)(((uint64_t)n + C - 1) / C);
    while (h->hp_ev.size() < 2 * (size_t)nch + 2) {
        hipEvent_t e;
        HIP_TRY(h, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        h->hp_ev.push_back(e);
    }
    GD_TRY(ensure(h, h->keys_in, (size_t)n * sizeof(gd_key)));
    GD_TRY(ensure(h, h->out_a, (size_t)n * 4 + 4));
    GD_TRY(ensure(h, h->out_b, (size_t)n * 4 + 4));
    GD_TRY(ensure(h, h->out_c, (size_t)n + 4));
    const bool bucket = out_perm != nullptr;        // gd_route: routes only
    if (bucket) {
        GD_TRY(ensure(h, h->u8_a, (size_t)n * 4 + 4));
        GD_TRY(ensure(h, h->offs, ((size_t)n_act + 2) * 4));
    }
    gd_key* dk = (gd_key*)h->keys_in.p;
    uint32_t* silo = (uint32_t*)h->out_a.p;
    uint32_t* act = (uint32_t*)h->out_b.p;
    uint8_t* st = (uint8_t*)h->out_c.p;
    hipEvent_t* ev = h->hp_ev.data();
    HIP_TRY(h, hipEventRecord(ev[2 * nch], h->stream));        // earlier work on the handle's stream
    HIP_TRY(h, hipStreamWaitEvent(h->cin, ev[2 * nch], 0));
    for (uint32_t k = 0; k < nch; ++k) {
        const size_t off = (size_t)k * C;
        const uint32_t cnt = (uint32_t)std::min<size_t>(C, n - off);
        HIP_TRY(h, hipMemcpyAsync(dk + off, keys + off, (size_t)cnt * sizeof(gd_key), hipMemcpyHostToDevice, h->cin));
        HIP_TRY(h, hipEventRecord(ev[2 * k], h->cin));
        HIP_TRY(h, hipStreamWaitEvent(h->stream, ev[2 * k], 0));
        GD_TRY(route_device(h, dk + off, cnt, silo + off, act + off, st + off));
        HIP_TRY(h, hipEventRecord(ev[2 * k + 1], h->stream));
        HIP_TRY(h, hipStreamWaitEvent(h->cout, ev[2 * k + 1], 0));
        HIP_TRY(h, hipMemcpyAsync(out_silo + off, silo + off, (size_t)cnt * 4, hipMemcpyDeviceToHost, h->cout));
        HIP_TRY(h, hipMemcpyAsync(out_act + off, act + off, (size_t)cnt * 4, hipMemcpyDeviceToHost, h->cout));
        HIP_TRY(h, hipMemcpyAsync(out_status + off, st + off, cnt, hipMemcpyDeviceToHost, h->cout));
    }
    if (!bucket) {
        HIP_TRY(h, hipStreamSynchronize(h->cout));
        return sync(h);
    }
    GD_TRY(bucket_device(h, act, n, n_act, (uint32_t*)h->u8_a.p, (uint32_t*)h->offs.p));
    HIP_TRY(h, hipEventRecord(ev[2 * nch + 1], h->stream));
    HIP_TRY(h, hipStreamWaitEvent(h->cout, ev[2 * nch + 1], 0));
    HIP_TRY(h, hipMemcpyAsync(out_perm, h->u8_a.p, (size_t)n * 4, hipMemcpyDeviceToHost, h->cout));
    HIP_TRY(h, hipMemcpyAsync(out_offsets, h->offs.p, ((size_t)n_act + 2) * 4, hipMemcpyDeviceToHost, h->cout));
    HIP_TRY(h, hipStreamSynchronize(h->cout));
    return sync_checked(h);
}

}  // namespace gdx

namespace gdx {
template int scan_device<OpAdd>(gd_handle*, uint32_t*, uint32_t, bool, bool, const char*, uint32_t*);
template int scan_device<OpMin>(gd_handle*, uint32_t*, uint32_t, bool, bool, const char*, uint32_t*);
template int shard_pack<true>(gd_handle*, const void*, const uint32_t*, uint32_t, uint64_t, uint32_t, void*, uint32_t*,
                              uint32_t*, const ExtArgs&, uint32_t*, uint32_t);
template int shard_pack<false>(gd_handle*, const void*, const uint32_t*, uint32_t, uint64_t, uint32_t, void*, uint32_t*,
                               uint32_t*, const ExtArgs&, uint32_t*, uint32_t);
}  // namespace gdx
