// eng_abi.hip -- libgraindispatch: handle lifecycle, ring, directory, route / bucket entry points, options and measured choices (C ABI); the micro-batch latency path; membership split.
// Shared handle and helpers: gd_engine.h.
#include "gd_engine.h"

// ================================================================== C ABI
extern "C" {

const char* gd_last_error(const gd_handle* h) {
    if (h) return h->err.c_str();
    return g_tls_error.c_str();
}

// The stable ranks' hardware assumption (gd_msd.h k_lane_order_check): on a device that does not serve
// one wave's same-address LDS atomics in lane order, the handle ranks by ballots instead (stable by
// construction; GD_OPT_STABLE_RANK reads 0 and refuses 1 there).
static int lane_order_check(gd_handle* h) {
    uint32_t* d = nullptr;
    if (hipMalloc(&d, 256 * 4) != hipSuccess) return set_err(nullptr, GD_ENOMEM, "lane-order check buffer");
    uint32_t hbad[256] = {};
    hipLaunchKernelGGL(k_lane_order_check, dim3(1), dim3(256), 0, h->stream, d);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(hbad, d, sizeof(hbad), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return set_err(nullptr, GD_EHIP, "lane-order check: %s", hipGetErrorString(e));
    uint64_t bad = 0;
    for (uint32_t x : hbad) bad += x;
    h->lane_order = bad == 0 && !h->lane_order_forced_off;
    if (!h->lane_order) h->radix_rank_atomic = 0;
    return GD_OK;
}

int gd_create(const gd_config* cfg, gd_handle** out) {
    if (!cfg || !out) return set_err(nullptr, GD_EINVAL, "gd_create: null argument");
    if (cfg->struct_size != sizeof(gd_config)) return set_err(nullptr, GD_EINVAL, "gd_create: struct_size mismatch");
    *out = nullptr;
    gd_handle* h = new (std::nothrow) gd_handle();
    if (!h) return set_err(nullptr, GD_ENOMEM, "gd_create: out of host memory");
    h->cfg = *cfg;
    h->device = cfg->device;
    h->timing = (cfg->flags & GD_CFG_KERNEL_TIMING) != 0 ? 1 : 0;
    h->lane_order_forced_off = (cfg->flags & GD_CFG_NO_LANE_ORDER) != 0;
    hipError_t e = hipSetDevice(h->device);
    if (e != hipSuccess) {
        int r = set_err(nullptr, GD_EHIP, "hipSetDevice(%d): %s", h->device, hipGetErrorString(e));
        delete h;
        return r;
    }
    {
        int cu = 0;
        if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, h->device) == hipSuccess && cu > 0)
            h->n_cu = (uint32_t)cu;
    }
    e = hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        int r = set_err(nullptr, GD_EHIP, "hipStreamCreate: %s", hipGetErrorString(e));
        delete h;
        return r;
    }
    h->stream = h->own_stream;
    h->capacity = pow2_at_least(cfg->table_capacity ? cfg->table_capacity : (1ull << 20));
    int r = alloc_table(h, h->capacity, &h->slots);
    if (r == GD_OK) r = alloc_vtag(h, h->capacity, &h->vtag);
    if (r == GD_OK) {
        e = hipMalloc(&h->ctr, CTR_BYTES);
        if (e != hipSuccess) r = set_err(nullptr, GD_ENOMEM, "counters: %s", hipGetErrorString(e));
        else if ((e = hipMemsetAsync(h->ctr, 0, CTR_BYTES, h->stream)) != hipSuccess)
            r = set_err(nullptr, GD_EHIP, "counters memset: %s", hipGetErrorString(e));
    }
    if (r == GD_OK) {
        const uint32_t mb = cfg->max_batch ? cfg->max_batch : (1u << 24);
        (void)mb;  // scratch grows on demand; nothing pre-sized beyond the table
        r = sync(h);
    }
    if (r == GD_OK) r = lane_order_check(h);
    if (r != GD_OK) {
        gd_destroy(h);
        return r;
    }
    *out = h;
    return GD_OK;
}

namespace gdx {
}

void gd_destroy(gd_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->bstream) (void)hipStreamSynchronize(h->bstream);
    if (h->b_ev) (void)hipEventDestroy(h->b_ev);
    if (h->b_fence_ev) (void)hipEventDestroy(h->b_fence_ev);
    if (h->fan_ev) (void)hipEventDestroy(h->fan_ev);
    for (DevBuf* b : {&h->ring_pts, &h->ring_own, &h->keys_in, &h->u32_a, &h->u32_b, &h->u32_c, &h->u32_d, &h->u8_a,
                      &h->out_a, &h->out_b, &h->out_c, &h->hist, &h->partials, &h->partials2, &h->offs})
        free_buf(*b);
    for (DevBuf& b : h->fr) free_buf(b);
    for (DevBuf& b : h->m3) free_buf(b);
    free_buf(h->tune_buf);
    for (DevBuf& b : h->fr_ext) free_buf(b);
    for (DevBuf& b : h->churn) free_buf(b);
    for (DevBuf& b : h->fan) free_buf(b);
    free_buf(h->fan_bnd);
    for (DevBuf& b : h->cbuf) free_buf(b);
    if (h->h_pin) (void)hipHostFree(h->h_pin);
    free_buf(h->cache_local);
    free_buf(h->shard_dest);
    free_buf(h->shard_hist);
    free_buf(h->up_last);
    comm_release(h);
    if (h->kx_slots) (void)hipFree(h->kx_slots);
    free_buf(h->kx_heap);
    for (DevBuf& b : h->kx_buf) free_buf(b);
    free_buf(h->cache_valid);
    if (h->cslots) (void)hipFree(h->cslots);
    free_buf(h->cx_heap);
    free_buf(h->cxi_tab);
    free_buf(h->cx8_tab);
    free_buf(h->reg_retry);
    for (auto& d : h->dir_scr) free_buf(d);
    free_buf(h->cxi_types);
    free_buf(h->cxi_ctr);
    for (auto& kt : h->cx_tune)
        for (int v = 0; v < gd_handle::CXV; ++v) {
            auto& t = kt.second;
            if (t.a[v]) (void)hipEventDestroy(t.a[v]);
            if (t.b[v]) (void)hipEventDestroy(t.b[v]);
        }
    if (h->cctr) (void)hipFree(h->cctr);
    if (h->slots) (void)hipFree(h->slots);
    if (h->ctr) (void)hipFree(h->ctr);
    if (h->vtag) (void)hipFree(h->vtag);
    free_buf(h->dir_valid);
    free_buf(h->act_ids);
    for (DevBuf& b : h->dirop_buf) free_buf(b);
    if (h->ad_slots) (void)hipFree(h->ad_slots);
    if (h->ad_ctr) (void)hipFree(h->ad_ctr);
    free_buf(h->ad_last);
    for (DevBuf& b : h->ad_buf) free_buf(b);
    for (DevBuf& b : h->fr_recv) free_buf(b);
    for (DevBuf& b : h->recv_scr) free_buf(b);
    for (auto& t : h->pending) {
        (void)hipEventDestroy(t.a);
        (void)hipEventDestroy(t.b);
    }
    for (auto e : h->event_pool) (void)hipEventDestroy(e);
    for (auto e : h->hp_ev) (void)hipEventDestroy(e);
    if (h->cin) (void)hipStreamDestroy(h->cin);
    if (h->cout) (void)hipStreamDestroy(h->cout);
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    delete h;
}

int gd_set_stream(gd_handle* h, void* s) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    GD_TRY(resolve_timing(h));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    h->stream = s ? (hipStream_t)s : h->own_stream;
    return GD_OK;
}

void* gd_get_stream(gd_handle* h) { return h ? (void*)h->stream : nullptr; }

int gd_host_alloc(size_t bytes, void** out) {
    if (!out) return set_err(nullptr, GD_EINVAL, "null argument");
    *out = nullptr;
    const hipError_t e = hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault);
    if (e != hipSuccess) {
        *out = nullptr;
        return set_err(nullptr, GD_ENOMEM, "hipHostMalloc(%zu): %s", bytes, hipGetErrorString(e));
    }
    return GD_OK;
}

int gd_host_free(void* p) {
    if (!p) return GD_OK;
    const hipError_t e = hipHostFree(p);
    if (e != hipSuccess) return set_err(nullptr, GD_EHIP, "hipHostFree: %s", hipGetErrorString(e));
    return GD_OK;
}

int gd_synchronize(gd_handle* h) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    HIP_TRY(h, hipSetDevice(h->device));
    if (h->pstream) HIP_TRY(h, hipStreamSynchronize(h->pstream));
    if (h->xstream) HIP_TRY(h, hipStreamSynchronize(h->xstream));
    return sync_checked(h);
}

int gd_stats_get(gd_handle* h, gd_stats* out) {
    if (!h || !out) return set_err(h, GD_EINVAL, "null argument");
    GD_TRY(pull_counters(h));
    out->routed = h->routed;
    out->table_live = h->ctr_host.live;
    out->table_tombstones = h->ctr_host.tomb;
    out->table_capacity = h->capacity;
    out->ring_points = h->ring_n;
    out->ring_mode = (uint64_t)(int64_t)h->ring_mode;
    return GD_OK;
}

int gd_index_stats_get(gd_handle* h, gd_index_stats* out) {
    if (!h || !out) return set_err(h, GD_EINVAL, "null argument");
    *out = gd_index_stats{};
    out->builds = h->cx_builds;
    out->synced_slots = h->cx_synced;
    out->last_build_ms = h->cx_build_ms;
    out->current = cx_current(h) ? 1u : 0u;
    out->types8 = h->cx8_ok ? h->cx8_layout.ntypes : 0u;
    out->act_bits8 = h->cx8_ok ? h->cx8_layout.ab : 0u;
    out->silo_bits8 = h->cx8_ok ? h->cx8_layout.sb : 0u;
    out->n0_live = h->cx_ctr_host.n0_live;
    out->out8 = h->cx_ctr_host.out8;
    return GD_OK;
}

int gd_ring_set(gd_handle* h, int mode, const uint32_t* points, const uint32_t* owner, uint32_t n) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    if (mode < GD_RING_DIRECTORY || mode > GD_RING_VIRTUAL_BUCKETS) return set_err(h, GD_EINVAL, "bad ring mode %d", mode);
    if (n == 0 || n > 4096 || !points || !owner) return set_err(h, GD_EINVAL, "ring size %u not in [1, 4096]", n);
    for (uint32_t i = 0; i < n; ++i) {
        if (owner[i] > 0xFFFEu) return set_err(h, GD_EINVAL, "ring owner %u out of range", owner[i]);
        if (i == 0) continue;
        const bool ok = (mode == GD_RING_VIRTUAL_BUCKETS) ? (points[i - 1] < points[i])
                                                          : ((int32_t)points[i - 1] <= (int32_t)points[i]);
        if (!ok) return set_err(h, GD_EINVAL, "ring points not in ring order at %u", i);
    }
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(ensure(h, h->ring_pts, (size_t)n * 4));
    GD_TRY(ensure(h, h->ring_own, (size_t)n * 4));
    HIP_TRY(h, hipMemcpyAsync(h->ring_pts.p, points, (size_t)n * 4, hipMemcpyHostToDevice, h->stream));
    HIP_TRY(h, hipMemcpyAsync(h->ring_own.p, owner, (size_t)n * 4, hipMemcpyHostToDevice, h->stream));
    GD_TRY(sync(h));
    uint32_t top = 1;
    while (top * 2 <= n) top *= 2;
    h->ring_mode = mode;
    h->ring_n = n;
    h->ring_top = top;
    h->layout_gen++;
    return GD_OK;
}

int gd_ring_owner(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t* out_silo) {
    if (!h || (n && (!keys || !out_silo))) return set_err(h, GD_EINVAL, "null argument");
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(h2d(h, h->keys_in, keys, n));
    GD_TRY(ensure(h, h->out_a, (size_t)n * 4));
    if (n) GD_TRY(ring_owner_device(h, (const gd_key*)h->keys_in.p, n, (uint32_t*)h->out_a.p));
    GD_TRY(d2h(h, out_silo, h->out_a, n));
    return sync(h);
}

int gd_ring_owner_device(gd_handle* h, const gd_key* d_keys, uint32_t n, uint32_t* d_silo) {
    if (!h || (n && (!d_keys || !d_silo))) return set_err(h, GD_EINVAL, "null argument");
    return n ? ring_owner_device(h, d_keys, n, d_silo) : GD_OK;
}

int gd_ring_lookup_hashes(gd_handle* h, const uint32_t* hashes, uint32_t n, uint32_t* out_silo) {
    if (!h || (n && (!hashes || !out_silo))) return set_err(h, GD_EINVAL, "null argument");
    GD_TRY(check_ring(h));
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(h2d(h, h->u32_a, hashes, n));
    GD_TRY(ensure(h, h->out_a, (size_t)n * 4));
    const dim3 g(blocks_for(n, BLOCK)), b(BLOCK);
    const RingArgs r = ring_args(h);
    const uint32_t* in = (const uint32_t*)h->u32_a.p;
    uint32_t* o = (uint32_t*)h->out_a.p;
    if (n) {
        if (h->ring_mode == GD_RING_DIRECTORY)
            GD_TRY(launch(h, "k_ring_hashes", g, b, ring_lds(h), k_ring_hashes<GD_RING_DIRECTORY>, in, n, r, o));
        else if (h->ring_mode == GD_RING_CONSISTENT)
            GD_TRY(launch(h, "k_ring_hashes", g, b, ring_lds(h), k_ring_hashes<GD_RING_CONSISTENT>, in, n, r, o));
        else
            GD_TRY(launch(h, "k_ring_hashes", g, b, ring_lds(h), k_ring_hashes<GD_RING_VIRTUAL_BUCKETS>, in, n, r, o));
    }
    GD_TRY(d2h(h, out_silo, h->out_a, n));
    return sync(h);
}

}  // extern "C"

namespace gdx {
// AddSingleActivation for a batch of device-resident keys / values (first registration wins, batch
// order); out_vals / out_ins are device arrays (either may be null).  Synchronous, or (async) only
// enqueued: REG_PASSES gated claim passes instead of read-back-driven relaunches, no read-back at the
// end; a device error (table full, unsettled claims) surfaces at the next synchronising call.
int register_core(gd_handle* h, const gd_key* dk, const gd_val* dvals, uint32_t n, gd_val* out_vals,
                  uint8_t* out_ins, bool async) {
    GD_TRY(async ? maybe_grow_async(h, n) : maybe_grow_table(h, n));
    const uint32_t op = ++h->dir_op;
    // the directory batches' own scratch (dir_scr): no bucketing left running on the bucket stream
    // shares it, so a batch need not wait for one (bfence) -- it overlaps the previous batch's bucketing
    GD_TRY(ensure_own(h, h->dir_scr[0], (size_t)n * 4));   // slot_of
    GD_TRY(ensure_own(h, h->dir_scr[1], (size_t)n * 4));   // k_reg_find's seen metas, then win
    GD_TRY(ensure_own(h, h->dir_scr[2], (size_t)n));       // is_new (k_reg_find writes every item's)
    GD_TRY(slot_words(h));                                 // the per-slot election words
    const dim3 g(blocks_for(n, BLOCK)), b(BLOCK);
    uint32_t* slot_of = (uint32_t*)h->dir_scr[0].p;
    uint32_t* win = (uint32_t*)h->dir_scr[1].p;
    uint8_t* is_new = (uint8_t*)h->dir_scr[2].p;
    uint32_t* last = (uint32_t*)h->up_last.p;
    const unsigned long long mask = h->capacity - 1;
    TabTrack tt(h);                                // the batch re-projects its slots into the probe indexes
    // a find with plain loads and one CAS a new grain in one launch (k_reg_find_take), then the full
    // protocol for the items that lost their CAS or met a claim of the launch; every item ending with a new
    // entry elects itself in the slot's word (the lowest batch index wins: first registration wins,
    // GrainDirectoryPartition.cs:304-326)
    const uint32_t* unsettled = nullptr;
    uint32_t* retry0 = nullptr;
    if (async) {
        if (!h->reg_retry.p) {                     // gate counters: k_reg_take / the commit keep them
            GD_TRY(ensure_own(h, h->reg_retry, REG_PASSES * sizeof(uint32_t)));
            HIP_TRY(h, hipMemsetAsync(h->reg_retry.p, 0, REG_PASSES * sizeof(uint32_t), h->stream));
        }
        uint32_t* rc = (uint32_t*)h->reg_retry.p;
        GD_TRY(launch(h, "k_reg_find_take", g, b, 0, k_reg_find_take, dk, n, h->slots, mask, h->ctr, dvals,
                      table_args(h), slot_of, is_new, win, rc, rc + 1, last));
        // a pass settles one new grain of each group colliding on a first free slot: a batch of 2^16 items
        // settles in 3 (cfg 2's 1 % churn batches: 222 deferred by the take, 3 by pass 1, none by pass 2),
        // and each gated launch costs ~1.4 us even when its gate is shut
        const uint32_t passes = n <= (1u << 16) ? REG_PASSES_SMALL : REG_PASSES;
        for (uint32_t pass = 1; pass < passes; ++pass)
            GD_TRY(launch(h, "k_reg_claim", g, b, 0, k_reg_claim_gated, dk, n, h->slots, mask, h->ctr, slot_of, is_new,
                          dvals, table_args(h), (const uint32_t*)rc + pass - 1, rc + pass, last, pass));
        unsettled = rc + passes - 1;
        retry0 = rc;
        h->pending_in += n;
    } else {
        HIP_TRY(h, hipMemsetAsync(&h->ctr->retry, 0, sizeof(uint32_t), h->stream));
        GD_TRY(launch(h, "k_reg_find_take", g, b, 0, k_reg_find_take, dk, n, h->slots, mask, h->ctr, dvals,
                      table_args(h), slot_of, is_new, win, &h->ctr->retry, (uint32_t*)nullptr, last));
        GD_TRY(pull_counters(h));
        // relaunches for the items that lost their CAS or met an unpublished claim
        for (uint32_t pass = 1; h->ctr_host.retry && !h->ctr_host.err; ++pass) {
            if (pass > 64) return set_err(h, GD_ETIMEOUT, "gd_dir_register: claims did not settle");
            HIP_TRY(h, hipMemsetAsync(&h->ctr->retry, 0, sizeof(uint32_t), h->stream));
            GD_TRY(launch(h, "k_reg_claim", g, b, 0, k_reg_claim, dk, n, h->slots, mask, h->ctr, slot_of, is_new, pass,
                          dvals, table_args(h), last));
            GD_TRY(pull_counters(h));
        }
    }
    if (cx_inline(h, tt, n))                       // the winners project their slots as they commit
        GD_TRY(launch(h, "k_reg_commit", g, b, 0, k_reg_commit_elect_cx, (const uint32_t*)slot_of,
                      (const uint8_t*)is_new, dvals, n, h->slots, h->ctr, h->vtag, op, last, win, unsettled, retry0,
                      cx_build_args(h), (CxCounters*)h->cxi_ctr.p));
    else
        GD_TRY(launch(h, "k_reg_commit", g, b, 0, k_reg_commit_elect, (const uint32_t*)slot_of, (const uint8_t*)is_new,
                      dvals, n, h->slots, h->ctr, h->vtag, op, last, win, unsettled, retry0));
    if (out_vals || out_ins)
        GD_TRY(launch(h, "k_reg_report", g, b, 0, k_reg_report, (const uint32_t*)slot_of, (const uint32_t*)win, n,
                      (const Slot*)h->slots, out_vals, out_ins));
    if (async) return GD_OK;
    GD_TRY(pull_counters(h));
    if (h->ctr_host.err) {
        const uint32_t e = h->ctr_host.err;
        HIP_TRY(h, hipMemsetAsync(&h->ctr->err, 0, sizeof(uint32_t), h->stream));
        GD_TRY(sync(h));
        return set_err(h, (e & 2) ? GD_EFULL : (e & 4) ? GD_EINVAL : GD_ETIMEOUT,
                       "gd_dir_register: device error bits 0x%x (2: table full, 4: silo index > 0xFFFE, "
                       "64: an asynchronous batch's claims did not settle)", e);
    }
    return GD_OK;
}

// RemoveActivation (Force) for a batch of device-resident keys / activations; out_removed (device, may be
// null).  Only enqueued; its own scratch (no bfence).  The first matching item of the batch removes.
int unregister_core(gd_handle* h, const gd_key* dk, const uint32_t* dacts, uint32_t n, uint8_t* out_removed) {
    const dim3 g(blocks_for(n, BLOCK)), b(BLOCK);
    const unsigned long long mask = h->capacity - 1;
    if (!out_removed) {
        // nobody asks which item removed: one launch, the CAS on the meta decides (k_unreg_cas)
        TabTrack tt(h);
        const CxBuild none{nullptr, nullptr, nullptr, Cx8Args{}};
        return launch(h, "k_unreg_cas", g, b, 0, k_unreg_cas, dk, dacts, n, h->slots, mask, h->ctr,
                      cx_inline(h, tt, n) ? cx_build_args(h) : none);
    }
    GD_TRY(ensure_own(h, h->dir_scr[0], (size_t)n * 4));
    GD_TRY(slot_words(h));
    uint32_t* slot_of = (uint32_t*)h->dir_scr[0].p;
    uint32_t* last = (uint32_t*)h->up_last.p;
    TabTrack tt(h);                               // the batch re-projects its slots into the probe indexes
    GD_TRY(launch(h, "k_unreg_find", g, b, 0, k_unreg_find_elect, dk, dacts, n, (const Slot*)h->slots, mask,
                  (const DevCounters*)h->ctr, slot_of, last));
    if (cx_inline(h, tt, n))                      // the removers project their tombstones as they commit
        return launch(h, "k_unreg_commit", g, b, 0, k_unreg_commit_elect_cx, (const uint32_t*)slot_of, n, h->slots,
                      h->ctr, last, out_removed, cx_build_args(h));
    return launch(h, "k_unreg_commit", g, b, 0, k_unreg_commit_elect, (const uint32_t*)slot_of, n, h->slots, h->ctr,
                  last, out_removed);
}

// One u32 per table slot, zero between directory batches (gd_dir_upsert's last writer, the registration
// and removal elections); (re)zeroed when the table grew.
int slot_words(gd_handle* h) {
    if (h->up_last.bytes >= h->capacity * 4) return GD_OK;
    GD_TRY(ensure_own(h, h->up_last, h->capacity * 4));
    HIP_TRY(h, hipMemsetAsync(h->up_last.p, 0, h->up_last.bytes, h->stream));
    return GD_OK;
}
}  // namespace gdx

extern "C" {

int gd_dir_register(gd_handle* h, const gd_key* keys, const gd_val* vals, uint32_t n, gd_val* out_vals,
                    uint8_t* out_inserted) {
    if (!h || (n && (!keys || !vals || !out_vals || !out_inserted))) return set_err(h, GD_EINVAL, "null argument");
    for (uint32_t i = 0; i < n; ++i)
        if (vals[i].silo > 0xFFFEu) return set_err(h, GD_EINVAL, "silo index %u out of range at %u", vals[i].silo, i);
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(h2d(h, h->keys_in, keys, n));
    GD_TRY(h2d(h, h->out_c, vals, n));     // gd_val staging
    GD_TRY(ensure(h, h->out_a, (size_t)n * sizeof(gd_val)));
    GD_TRY(ensure(h, h->out_b, (size_t)n));
    GD_TRY(register_core(h, (const gd_key*)h->keys_in.p, (const gd_val*)h->out_c.p, n, (gd_val*)h->out_a.p,
                         (uint8_t*)h->out_b.p, false));
    GD_TRY(d2h(h, out_vals, h->out_a, n));
    GD_TRY(d2h(h, out_inserted, h->out_b, n));
    return sync(h);
}

int gd_dir_register_device(gd_handle* h, const gd_key* d_keys, const gd_val* d_vals, uint32_t n, gd_val* d_out_vals,
                           uint8_t* d_out_inserted) {
    if (!h || (n && (!d_keys || !d_vals))) return set_err(h, GD_EINVAL, "null argument");
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(sync(h));                       // the caller's producers of d_keys / d_vals ran on this stream
    return register_core(h, d_keys, d_vals, n, d_out_vals, d_out_inserted, false);
}

int gd_dir_register_device_async(gd_handle* h, const gd_key* d_keys, const gd_val* d_vals, uint32_t n,
                                 gd_val* d_out_vals, uint8_t* d_out_inserted) {
    if (!h || (n && (!d_keys || !d_vals))) return set_err(h, GD_EINVAL, "null argument");
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    return register_core(h, d_keys, d_vals, n, d_out_vals, d_out_inserted, true);
}

int gd_dir_unregister_device(gd_handle* h, const gd_key* d_keys, const uint32_t* d_acts, uint32_t n,
                             uint8_t* d_out_removed) {
    if (!h || (n && (!d_keys || !d_acts))) return set_err(h, GD_EINVAL, "null argument");
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    return unregister_core(h, d_keys, d_acts, n, d_out_removed);
}

int gd_dir_upsert(gd_handle* h, const gd_key* keys, const gd_val* vals, uint32_t n, uint8_t* out_inserted) {
    if (!h || (n && (!keys || !vals))) return set_err(h, GD_EINVAL, "null argument");
    for (uint32_t i = 0; i < n; ++i)
        if (vals[i].silo > 0xFFFEu) return set_err(h, GD_EINVAL, "silo index %u out of range at %u", vals[i].silo, i);
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(bfence(h));
    GD_TRY(maybe_grow_table(h, n));
    const uint32_t op = ++h->dir_op;
    GD_TRY(h2d(h, h->keys_in, keys, n));
    GD_TRY(h2d(h, h->out_c, vals, n));            // gd_val staging
    GD_TRY(ensure(h, h->u32_a, (size_t)n * 4));   // slot_of
    GD_TRY(ensure(h, h->u8_a, (size_t)n));        // is_new
    GD_TRY(ensure(h, h->out_b, (size_t)n));
    GD_TRY(slot_words(h));                        // one u32 per slot, kept zero between calls
    HIP_TRY(h, hipMemsetAsync(h->u8_a.p, 0, n, h->stream));
    const dim3 g(blocks_for(n, BLOCK)), b(BLOCK);
    uint32_t* slot_of = (uint32_t*)h->u32_a.p;
    uint8_t* is_new = (uint8_t*)h->u8_a.p;
    uint32_t* last = (uint32_t*)h->up_last.p;
    const gd_key* dk = (const gd_key*)h->keys_in.p;
    const unsigned long long mask = h->capacity - 1;
    TabTrack tt(h);                               // the batch re-projects its slots into the probe indexes
    for (uint32_t pass = 0;; ++pass) {            // the registration's claim protocol (k_reg_claim)
        HIP_TRY(h, hipMemsetAsync(&h->ctr->retry, 0, sizeof(uint32_t), h->stream));
        GD_TRY(launch(h, "k_reg_claim", g, b, 0, k_reg_claim, dk, n, h->slots, mask, h->ctr, slot_of, is_new,
                      pass, (const gd_val*)h->out_c.p, table_args(h), (uint32_t*)nullptr));
        GD_TRY(pull_counters(h));
        if (h->ctr_host.retry == 0 || h->ctr_host.err) break;
        if (pass >= 64) return set_err(h, GD_ETIMEOUT, "gd_dir_upsert: claims did not settle");
    }
    GD_TRY(launch(h, "k_up_last", g, b, 0, k_up_last, (const uint32_t*)slot_of, n, last));
    GD_TRY(launch(h, "k_up_apply", g, b, 0, k_up_apply, (const uint32_t*)slot_of, (const uint8_t*)is_new,
                  (const gd_val*)h->out_c.p, n, (const uint32_t*)last, h->slots, h->ctr, (uint8_t*)h->out_b.p,
                  h->vtag, op));
    GD_TRY(launch(h, "k_up_clear", g, b, 0, k_up_clear, (const uint32_t*)slot_of, n, last));
    GD_TRY(cx_sync(h, tt, slot_of, n));
    if (out_inserted) GD_TRY(d2h(h, out_inserted, h->out_b, n));
    GD_TRY(pull_counters(h));
    if (h->ctr_host.err) {
        const uint32_t e = h->ctr_host.err;
        HIP_TRY(h, hipMemsetAsync(&h->ctr->err, 0, sizeof(uint32_t), h->stream));
        return set_err(h, (e & 2) ? GD_EFULL : GD_ETIMEOUT, "gd_dir_upsert: device error bits 0x%x", e);
    }
    return GD_OK;
}

int gd_dir_unregister(gd_handle* h, const gd_key* keys, const uint32_t* acts, uint32_t n, uint8_t* out_removed) {
    if (!h || (n && (!keys || !acts))) return set_err(h, GD_EINVAL, "null argument");
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(bfence(h));
    GD_TRY(h2d(h, h->keys_in, keys, n));
    GD_TRY(h2d(h, h->u32_b, acts, n));
    GD_TRY(ensure(h, h->out_b, (size_t)n));
    GD_TRY(unregister_core(h, (const gd_key*)h->keys_in.p, (const uint32_t*)h->u32_b.p, n, (uint8_t*)h->out_b.p));
    GD_TRY(d2h(h, out_removed, h->out_b, n));
    return sync(h);
}

int gd_dir_lookup(gd_handle* h, const gd_key* keys, uint32_t n, gd_val* out_vals, uint8_t* out_found) {
    if (!h || (n && (!keys || !out_vals || !out_found))) return set_err(h, GD_EINVAL, "null argument");
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(h2d(h, h->keys_in, keys, n));
    GD_TRY(ensure(h, h->out_a, (size_t)n * sizeof(gd_val)));
    GD_TRY(ensure(h, h->out_b, (size_t)n));
    GD_TRY(launch(h, "k_dir_lookup", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), 0, k_dir_lookup,
                  (const gd_key*)h->keys_in.p, n, table_args(h), (gd_val*)h->out_a.p, (uint8_t*)h->out_b.p));
    GD_TRY(d2h(h, out_vals, h->out_a, n));
    GD_TRY(d2h(h, out_found, h->out_b, n));
    return sync(h);
}

int gd_dir_clear(gd_handle* h) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, hipMemsetAsync(h->slots, 0, h->capacity * sizeof(Slot), h->stream));
    h->tab_gen++;
    HIP_TRY(h, hipMemsetAsync(h->vtag, 0, h->capacity * sizeof(uint32_t), h->stream));
    HIP_TRY(h, hipMemsetAsync(h->ctr, 0, CTR_BYTES, h->stream));   // with the striped deltas
    h->ctr_stale = true;
    if (h->kx_cap) {                   // KeyExt entries go too
        h->kx_m.assign(h->kx_cap, KxSlot{});
        h->kx_hheap.clear();
        h->kx_live = h->kx_tomb = 0;
        h->kx_maxp = 0;
        h->kx_heap_dev = 0;
        HIP_TRY(h, hipMemsetAsync(h->kx_slots, 0, h->kx_cap * sizeof(KxSlot), h->stream));
    }
    return sync(h);
}

int gd_dir_rehash(gd_handle* h, uint64_t new_capacity) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(pull_counters(h));
    const unsigned long long cap = pow2_at_least(new_capacity);
    if (cap < h->ctr_host.live) return set_err(h, GD_EINVAL, "capacity %llu below live entries", cap);
    Slot* ns = nullptr;
    GD_TRY(alloc_table(h, cap, &ns));
    uint32_t* nv = nullptr;
    if (alloc_vtag(h, cap, &nv) != GD_OK) {
        (void)hipFree(ns);
        return GD_ENOMEM;
    }
    HIP_TRY(h, hipMemsetAsync(h->ctr, 0, CTR_BYTES, h->stream));   // counters and their striped deltas
    const unsigned long long old_cap = h->capacity;
    const uint32_t g = (uint32_t)((old_cap + BLOCK - 1) / BLOCK);
    GD_TRY(launch(h, "k_rehash", dim3(g), dim3(BLOCK), 0, k_rehash, (const Slot*)h->slots, old_cap, ns, cap - 1, h->ctr,
                  (const uint32_t*)h->vtag, nv));
    GD_TRY(sync(h));
    HIP_TRY(h, hipFree(h->slots));
    HIP_TRY(h, hipFree(h->vtag));
    h->slots = ns;
    h->vtag = nv;
    h->capacity = cap;
    h->layout_gen++;
    h->tab_gen++;
    GD_TRY(pull_counters(h));
    if (h->ctr_host.err) return set_err(h, GD_EFULL, "rehash failed (0x%x)", h->ctr_host.err);
    return GD_OK;
}

int gd_route_device(gd_handle* h, const gd_key* d_keys, uint32_t n, uint32_t* d_silo, uint32_t* d_act, uint8_t* d_status) {
    if (!h || (n && (!d_keys || !d_silo || !d_act || !d_status))) return set_err(h, GD_EINVAL, "null argument");
    return n ? route_device(h, d_keys, n, d_silo, d_act, d_status) : GD_OK;
}

int gd_route_bound_device(gd_handle* h, const gd_key* d_keys, uint32_t n, uint32_t* d_silo, uint32_t* d_act,
                          uint8_t* d_status) {
    if (!h || (n && (!d_keys || !d_silo || !d_act || !d_status))) return set_err(h, GD_EINVAL, "null argument");
    return n ? route_bound_device(h, d_keys, n, d_silo, d_act, d_status) : GD_OK;
}

int gd_bucket_device(gd_handle* h, const uint32_t* d_acts, uint32_t n, uint32_t n_act, uint32_t* d_perm,
                     uint32_t* d_offsets) {
    if (!h || !d_offsets || (n && (!d_acts || !d_perm))) return set_err(h, GD_EINVAL, "null argument");
    return bucket_device(h, d_acts, n, n_act, d_perm, d_offsets);
}

int gd_route_bucket_device(gd_handle* h, const gd_key* d_keys, uint32_t n, uint32_t n_act, uint32_t* d_silo,
                           uint32_t* d_act, uint8_t* d_status, uint32_t* d_perm, uint32_t* d_offsets) {
    if (!h || !d_offsets || (n && (!d_keys || !d_silo || !d_act || !d_status || !d_perm)))
        return set_err(h, GD_EINVAL, "null argument");
    if (n) GD_TRY(route_device(h, d_keys, n, d_silo, d_act, d_status));
    if (!h->bstream || h->bstream == h->stream) return bucket_device(h, d_act, n, n_act, d_perm, d_offsets);
    // the bucketing on the bucket stream once this route is done; the handle's stream goes on to the
    // next batch's route (gd_set_bucket_stream)
    HIP_TRY(h, hipEventRecord(h->b_ev, h->stream));
    HIP_TRY(h, hipStreamWaitEvent(h->bstream, h->b_ev, 0));
    const hipStream_t main = h->stream;
    const bool measured_before = h->measured_launch;
    h->measured_launch = false;
    h->stream = h->bstream;
    const int r = bucket_device(h, d_act, n, n_act, d_perm, d_offsets);
    h->stream = main;
    h->b_pending = true;
    // a bucketing timed for tune_choose runs alone: the next batch's route waits for it
    if (h->measured_launch) GD_TRY(bfence(h));
    h->measured_launch = h->measured_launch || measured_before;
    return r;
}

int gd_set_bucket_stream(gd_handle* h, void* s) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(resolve_timing(h));
    GD_TRY(sync(h));
    if (s && !h->b_ev) HIP_TRY(h, hipEventCreateWithFlags(&h->b_ev, hipEventDisableTiming));
    if (s && !h->b_fence_ev) HIP_TRY(h, hipEventCreateWithFlags(&h->b_fence_ev, hipEventDisableTiming));
    h->b_pending = false;
    h->bstream = (hipStream_t)s;
    return GD_OK;
}

int gd_route(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t* out_silo, uint32_t* out_act, uint8_t* out_status) {
    if (!h || (n && (!keys || !out_silo || !out_act || !out_status))) return set_err(h, GD_EINVAL, "null argument");
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    if (h->host_chunk && n >= 2 * h->host_chunk && !h->cache_max && host_pinned(keys) && host_pinned(out_silo))
        return route_bucket_host_pipelined(h, keys, n, 0, out_silo, out_act, out_status, nullptr, nullptr);
    GD_TRY(h2d(h, h->keys_in, keys, n));
    GD_TRY(ensure(h, h->out_a, (size_t)n * 4));
    GD_TRY(ensure(h, h->out_b, (size_t)n * 4));
    GD_TRY(ensure(h, h->out_c, (size_t)n));
    GD_TRY(route_device(h, (const gd_key*)h->keys_in.p, n, (uint32_t*)h->out_a.p, (uint32_t*)h->out_b.p,
                        (uint8_t*)h->out_c.p));
    GD_TRY(d2h(h, out_silo, h->out_a, n));
    GD_TRY(d2h(h, out_act, h->out_b, n));
    GD_TRY(d2h(h, out_status, h->out_c, n));
    return sync(h);
}

int gd_bucket(gd_handle* h, const uint32_t* acts, uint32_t n, uint32_t n_act, uint32_t* out_perm, uint32_t* out_offsets) {
    if (!h || !out_offsets || (n && (!acts || !out_perm))) return set_err(h, GD_EINVAL, "null argument");
    if (n_act == 0xFFFFFFFFu) return set_err(h, GD_EINVAL, "n_act too large");
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(h2d(h, h->out_b, acts, n));
    GD_TRY(ensure(h, h->out_a, (size_t)n * 4 + 4));
    GD_TRY(ensure(h, h->offs, ((size_t)n_act + 2) * 4));
    GD_TRY(bucket_device(h, (const uint32_t*)h->out_b.p, n, n_act, (uint32_t*)h->out_a.p, (uint32_t*)h->offs.p));
    GD_TRY(d2h(h, out_perm, h->out_a, n));
    GD_TRY(d2h(h, out_offsets, h->offs, (size_t)n_act + 2));
    return sync_checked(h);
}

int gd_route_bucket(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t n_act, uint32_t* out_silo, uint32_t* out_act,
                    uint8_t* out_status, uint32_t* out_perm, uint32_t* out_offsets) {
    if (!h || !out_offsets || (n && (!keys || !out_silo || !out_act || !out_status || !out_perm)))
        return set_err(h, GD_EINVAL, "null argument");
    if (n_act == 0xFFFFFFFFu) return set_err(h, GD_EINVAL, "n_act too large");
    HIP_TRY(h, hipSetDevice(h->device));
    if (h->host_chunk && n >= 2 * h->host_chunk && !h->cache_max && host_pinned(keys) && host_pinned(out_perm))
        return route_bucket_host_pipelined(h, keys, n, n_act, out_silo, out_act, out_status, out_perm, out_offsets);
    GD_TRY(h2d(h, h->keys_in, keys, n));
    GD_TRY(ensure(h, h->out_a, (size_t)n * 4 + 4));
    GD_TRY(ensure(h, h->out_b, (size_t)n * 4 + 4));
    GD_TRY(ensure(h, h->out_c, (size_t)n + 4));
    GD_TRY(ensure(h, h->u8_a, (size_t)n * 4 + 4));   // perm
    GD_TRY(ensure(h, h->offs, ((size_t)n_act + 2) * 4));
    if (n)
        GD_TRY(route_device(h, (const gd_key*)h->keys_in.p, n, (uint32_t*)h->out_a.p, (uint32_t*)h->out_b.p,
                            (uint8_t*)h->out_c.p));
    GD_TRY(bucket_device(h, (const uint32_t*)h->out_b.p, n, n_act, (uint32_t*)h->u8_a.p, (uint32_t*)h->offs.p));
    GD_TRY(d2h(h, out_silo, h->out_a, n));
    GD_TRY(d2h(h, out_act, h->out_b, n));
    GD_TRY(d2h(h, out_status, h->out_c, n));
    GD_TRY(d2h(h, out_perm, h->u8_a, n));
    GD_TRY(d2h(h, out_offsets, h->offs, (size_t)n_act + 2));
    return sync_checked(h);
}

int gd_pack_by_shard_device(gd_handle* h, const gd_key* d_keys, uint32_t n, uint32_t n_shards, gd_key* d_send_keys,
                            uint32_t* d_send_idx, uint32_t* d_counts) {
    if (!h || !d_counts || (n && (!d_keys || !d_send_keys || !d_send_idx))) return set_err(h, GD_EINVAL, "null argument");
    if (n_shards == 0 || n_shards > 256) return set_err(h, GD_EINVAL, "n_shards %u not in [1, 256]", n_shards);
    return shard_pack<false>(h, d_keys, nullptr, n, 0, n_shards, d_send_keys, d_send_idx, d_counts);
}

int gd_pack_routes_by_rank_device(gd_handle* h, const gd_key* d_keys, const uint8_t* d_status, const uint32_t* d_silo,
                                  uint32_t n, uint32_t n_shards, uint32_t my_rank, gd_key* d_send_keys,
                                  uint32_t* d_send_pos, uint32_t* d_counts) {
    if (!h || !d_counts || (n && (!d_keys || !d_status || !d_silo || !d_send_keys || !d_send_pos)))
        return set_err(h, GD_EINVAL, "null argument");
    if (n_shards == 0 || n_shards > 256 || my_rank >= n_shards)
        return set_err(h, GD_EINVAL, "n_shards %u not in [1, 256] or my_rank %u >= n_shards", n_shards, my_rank);
    return fwd_pack(h, d_keys, d_status, d_silo, n, n_shards, my_rank, d_send_keys, d_send_pos, d_counts);
}

int gd_kernel_times(gd_handle* h, gd_kernel_time* out, uint32_t max, uint32_t* out_n) {
    if (!h || !out_n) return set_err(h, GD_EINVAL, "null argument");
    GD_TRY(resolve_timing(h));
    const uint32_t m = (uint32_t)std::min<size_t>(max, h->tnames.size());
    for (uint32_t i = 0; i < m; ++i) {
        std::memset(out[i].name, 0, sizeof out[i].name);
        std::strncpy(out[i].name, h->tnames[i].c_str(), sizeof out[i].name - 1);
        out[i].launches = h->tcount[i];
        out[i].total_ms = h->tms[i];
    }
    *out_n = (uint32_t)h->tnames.size();
    return GD_OK;
}

int gd_set_kernel_timing(gd_handle* h, int enable) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    if (enable < 0 || enable > 2) return set_err(h, GD_EINVAL, "gd_set_kernel_timing: %d (0 off, 1 launches, 2 stages)", enable);
    GD_TRY(resolve_timing(h));
    h->timing = enable;
    return GD_OK;
}

int gd_kernel_times_reset(gd_handle* h) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    GD_TRY(resolve_timing(h));
    std::fill(h->tms.begin(), h->tms.end(), 0.0);
    std::fill(h->tcount.begin(), h->tcount.end(), 0);
    return GD_OK;
}

int gd_option_set(gd_handle* h, int option, int64_t v) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    auto in = [&](int64_t lo, int64_t hi) { return v >= lo && v <= hi; };
    switch (option) {
        case GD_OPT_PROBE:
            if (!in(0, 4)) break;
            h->cx_mode = (int)v;
            return GD_OK;
        case GD_OPT_BUCKET:
            if (!in(0, 2)) break;
            h->msd_mode = (int)v;
            return GD_OK;
        case GD_OPT_L2_SMALL:
            if (!in(0, MSD_CAP)) break;
            h->l2_small = (uint32_t)v;
            return GD_OK;
        case GD_OPT_STABLE_RANK:
            if (!in(0, 1)) break;
            if (v == 1 && !h->lane_order)
                return set_err(h, GD_EINVAL, "gd_option_set: GD_OPT_STABLE_RANK 1 needs the LDS lane order this "
                               "device lacks (gd_create's check): ranks stay on ballots");
            h->radix_rank_atomic = (uint32_t)v;
            return GD_OK;
        case GD_OPT_WIRE_HEADERS:
            if (!in(0, 2)) break;
            h->compact_headers = v >= 1;
            h->narrow_headers = v == 2;
            return GD_OK;
        case GD_OPT_REGION_PROBE:
            if (!in(0, 1)) break;
            h->region_probe = v != 0;
            return GD_OK;
        case GD_OPT_IDX16:
            if (!in(0, 1)) break;
            h->idx16 = v != 0;
            return GD_OK;
        case GD_OPT_HOST_CHUNK:
            if (!in(0, 1ll << 30)) break;
            h->host_chunk = (uint32_t)v;
            return GD_OK;
        case GD_OPT_MB_ZEROCOPY:
            if (!in(0, 1)) break;
            h->mb_zero_copy = v != 0;
            return GD_OK;
        case GD_OPT_MB_SPLIT:
            if (!in(1, 64)) break;
            h->mb_split = (uint32_t)v;
            return GD_OK;
        case GD_OPT_MB_TRACE:
            if (!in(0, 1)) break;
            h->mb_trace = v != 0;
            return GD_OK;
        case GD_OPT_L2_STAGED:
            if (!in(0, MSD_CAP)) break;
            h->l2_staged = (uint32_t)v;
            return GD_OK;
        case GD_OPT_L2_MID:
            if (!in(0, MSD_MID_CAP)) break;
            h->l2_mid = (uint32_t)v;
            return GD_OK;
        case GD_OPT_B2_PERSIST:
            if (!in(0, 8)) break;
            h->b2_persist = (uint32_t)v;
            return GD_OK;
        case GD_OPT_B2_ORDER:
            if (!in(0, 1)) break;
            h->b2_order = (uint32_t)v;
            return GD_OK;
        case GD_OPT_MB_POLL:
            if (!in(0, 1)) break;
            h->mb_poll = v != 0;
            return GD_OK;
        case GD_OPT_FAN_BOUND:
            if (!in(0, 1)) break;
            h->fan_bound = v != 0;
            return GD_OK;
        default: return set_err(h, GD_EINVAL, "gd_option_set: unknown option %d", option);
    }
    return set_err(h, GD_EINVAL, "gd_option_set: option %d: value %lld out of range", option, (long long)v);
}

int gd_option_get(const gd_handle* hc, int option, int64_t* v) {
    gd_handle* h = const_cast<gd_handle*>(hc);
    if (!h || !v) return set_err(h, GD_EINVAL, "null argument");
    switch (option) {
        case GD_OPT_PROBE: *v = h->cx_mode; return GD_OK;
        case GD_OPT_BUCKET: *v = h->msd_mode; return GD_OK;
        case GD_OPT_L2_SMALL: *v = h->l2_small; return GD_OK;
        case GD_OPT_STABLE_RANK: *v = h->radix_rank_atomic; return GD_OK;
        case GD_OPT_WIRE_HEADERS: *v = h->compact_headers ? (h->narrow_headers ? 2 : 1) : 0; return GD_OK;
        case GD_OPT_REGION_PROBE: *v = h->region_probe; return GD_OK;
        case GD_OPT_IDX16: *v = h->idx16; return GD_OK;
        case GD_OPT_HOST_CHUNK: *v = h->host_chunk; return GD_OK;
        case GD_OPT_MB_ZEROCOPY: *v = h->mb_zero_copy; return GD_OK;
        case GD_OPT_MB_SPLIT: *v = h->mb_split; return GD_OK;
        case GD_OPT_MB_TRACE: *v = h->mb_trace; return GD_OK;
        case GD_OPT_L2_STAGED: *v = h->l2_staged; return GD_OK;
        case GD_OPT_L2_MID: *v = h->l2_mid; return GD_OK;
        case GD_OPT_B2_PERSIST: *v = h->b2_persist; return GD_OK;
        case GD_OPT_B2_ORDER: *v = h->b2_order; return GD_OK;
        case GD_OPT_MB_POLL: *v = h->mb_poll ? 1 : 0; return GD_OK;
        case GD_OPT_FAN_BOUND: *v = h->fan_bound ? 1 : 0; return GD_OK;
        default: return set_err(h, GD_EINVAL, "gd_option_get: unknown option %d", option);
    }
}

int gd_tune_reset(gd_handle* h) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    for (auto& kt : h->cx_tune) {
        auto& t = kt.second;
        for (int v = 0; v < gd_handle::CXV; ++v) {
            if (t.pending[v]) (void)hipEventSynchronize(t.b[v]);
            t.best[v] = 1e30f;
            t.pending[v] = false;
        }
        t.pick = -1;
        t.round = 0;
    }
    return GD_OK;
}

int gd_tune_set(gd_handle* h, int kind, int variant) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    if (kind < 0 || kind >= GD_TUNE_KINDS) return set_err(h, GD_EINVAL, "gd_tune_set: kind %d", kind);
    if (variant < -1 || variant >= tune_nvar(kind))
        return set_err(h, GD_EINVAL, "gd_tune_set: kind %d has no variant %d", kind, variant);
    h->tune_pin[kind] = variant;
    return GD_OK;
}

int gd_tune_get(gd_handle* h, int kind, uint64_t n, uint32_t sub, int* variant) {
    if (!h || !variant) return set_err(h, GD_EINVAL, "null argument");
    if (kind < 0 || kind >= GD_TUNE_KINDS) return set_err(h, GD_EINVAL, "gd_tune_get: kind %d", kind);
    if (h->tune_pin[kind] >= 0) {
        *variant = h->tune_pin[kind];
        return GD_OK;
    }
    auto it = h->cx_tune.find(tune_key(kind, n, (int)sub));
    if (it == h->cx_tune.end()) {
        *variant = -1;
        return GD_OK;
    }
    tune_resolve(it->second, it->second.nvar ? it->second.nvar : tune_nvar(kind));
    *variant = it->second.pick;
    return GD_OK;
}

}  // extern "C"

// ================================================================== micro-batch latency path
struct gd_microbatch {
    gd_handle* h = nullptr;
    uint32_t capacity = 0, n_act = 0;
    // One output block, same layout on both sides (capacity-sized, so host views never move):
    //   silo[cap] | act[cap] | perm[cap] | n_runs[1] | run_start[cap + 1] | run_act[cap] | status[cap] (u8)
    size_t out_bytes = 0;
    gd_key* h_keys = nullptr;
    uint8_t* h_out = nullptr;      // pinned
    gd_key* d_keys = nullptr;
    uint8_t* d_out = nullptr;
    // zero-copy (default; GD_MB_ZEROCOPY=0: staged copies): the route kernel reads the keys from the
    // pinned host block and writes silo / status into the pinned output block, the sort kernel writes
    // perm / runs / act there -- no H2D / D2H copy nodes; only act stays in HBM for the sort
    bool zero_copy = true;
    gd_key* h_keys_dev = nullptr;  // device view of h_keys
    uint8_t* h_out_dev = nullptr;  // device view of h_out
    uint32_t* d_act = nullptr;
    uint32_t split = 8;                 // k_mb_sort_runs workgroups (redundant sorts, split stores; GD_OPT_MB_SPLIT)
    uint32_t max_bits = MB_MAX_BITS;    // widest radix digit (11: two passes at n_act = 2^20)
    unsigned long long* ts = nullptr;   // GD_MB_TRACE: per-phase tick sums (device), printed at destroy
    uint64_t runs_done = 0;
    // GD_OPT_MB_POLL (zero-copy only): the sort's workgroups count themselves done into a pinned word; the
    // run returns when the count arrives instead of waiting for the dispatch's completion signal
    uint32_t* h_done = nullptr;         // pinned, coherent
    uint32_t* d_done = nullptr;         // its device view (null: no poll)
    uint32_t done_expect = 0;           // the count the last run waited for
    std::vector<std::pair<uint32_t, hipGraphExec_t>> graphs;
    uint64_t graphs_gen = 0;       // handle layout the cached graphs were captured against
    uint64_t graphs_cx = ~0ull;    // the probe index build they read (~0: the directory)

    uint32_t* out_u32(uint8_t* base, int k) const {
        const size_t c = capacity;
        const size_t at[6] = {0, c, 2 * c, 3 * c, 3 * c + 1, 4 * c + 2};   // silo act perm n_runs run_start run_act
        return (uint32_t*)base + at[k];
    }
    uint8_t* out_status(uint8_t* base) const { return base + (5 * (size_t)capacity + 2) * 4; }
};

namespace gdx {

// H2D keys -> route -> one-workgroup radix sort + runs -> one D2H of the whole output block; or, zero-copy,
// route (keys read from and silo / status written to pinned host memory) -> sort (perm / runs / act to host).
template <int IT>
int mb_launch_sort(gd_microbatch* mb, dim3 grid, uint32_t bits, const uint32_t* a, uint32_t n, uint32_t passes,
                   uint32_t* pm, uint32_t* ra, uint32_t* rs, uint32_t* nr, uint32_t* ac, uint32_t* done) {
    gd_handle* h = mb->h;
    const dim3 b(MB_THREADS);
    const uint32_t na = mb->n_act;
    unsigned long long* ts = mb->ts;
    const uint32_t bal = h->radix_rank_atomic ? 0u : 1u;
    switch (bits) {
        case 4: return launch(h, "k_mb_sort_runs", grid, b, 0, k_mb_sort_runs<4, IT>, a, n, passes, na, pm, ra, rs, nr, ac, ts, bal, done);
        case 5: return launch(h, "k_mb_sort_runs", grid, b, 0, k_mb_sort_runs<5, IT>, a, n, passes, na, pm, ra, rs, nr, ac, ts, bal, done);
        case 6: return launch(h, "k_mb_sort_runs", grid, b, 0, k_mb_sort_runs<6, IT>, a, n, passes, na, pm, ra, rs, nr, ac, ts, bal, done);
        case 7: return launch(h, "k_mb_sort_runs", grid, b, 0, k_mb_sort_runs<7, IT>, a, n, passes, na, pm, ra, rs, nr, ac, ts, bal, done);
        case 8: return launch(h, "k_mb_sort_runs", grid, b, 0, k_mb_sort_runs<8, IT>, a, n, passes, na, pm, ra, rs, nr, ac, ts, bal, done);
        case 9: return launch(h, "k_mb_sort_runs", grid, b, 0, k_mb_sort_runs<9, IT>, a, n, passes, na, pm, ra, rs, nr, ac, ts, bal, done);
        case 10: return launch(h, "k_mb_sort_runs", grid, b, 0, k_mb_sort_runs<10, IT>, a, n, passes, na, pm, ra, rs, nr, ac, ts, bal, done);
        default: return launch(h, "k_mb_sort_runs", grid, b, 0, k_mb_sort_runs<11, IT>, a, n, passes, na, pm, ra, rs, nr, ac, ts, bal, done);
    }
}

// The micro-batch route reads the 8-B index when it is built, current and not turned off (GD_OPT_PROBE
// 0) or pinned to the directory (gd_tune_set(GD_TUNE_PROBE_KEYS, 1)).
bool mb_use_index(const gd_handle* h) {
    return h->cx_mode != 0 && h->tune_pin[GD_TUNE_PROBE_KEYS] != 1 && h->cx8_ok && cx_current(h);
}

// k_mb_sort_runs's workgroups for n messages (each adds 1 to the done count)
uint32_t mb_sort_grid(const gd_microbatch* mb, uint32_t n) {
    return mb->zero_copy ? std::max<uint32_t>(1, std::min(mb->split, std::max<uint32_t>(1, n / 256))) : 1u;
}

// count_done: the sort counts itself done into mb->d_done (a captured graph's replays poll for it)
int mb_enqueue(gd_microbatch* mb, uint32_t n, bool count_done) {
    gd_handle* h = mb->h;
    const bool zc = mb->zero_copy;
    uint8_t* d = zc ? mb->h_out_dev : mb->d_out;
    uint32_t* act_dst = zc ? mb->d_act : mb->out_u32(d, 1);
    // keys min(act, n_act) need key_bits; passes of at most max_bits, as even as the digits allow
    uint32_t key_bits = 1;
    while (key_bits < 32 && (mb->n_act >> key_bits) != 0) ++key_bits;
    const uint32_t passes = (key_bits + mb->max_bits - 1) / mb->max_bits;
    const uint32_t bits = std::max<uint32_t>(4, (key_bits + passes - 1) / passes);
    if (n && zc && !h->cache_max) {
        h->routed += n;
        const dim3 g(blocks_for(n, MB_ROUTE_BLOCK)), b(MB_ROUTE_BLOCK);
        const gd_key* k = mb->h_keys_dev;
        uint32_t *so = mb->out_u32(d, 0);
        uint8_t* st = mb->out_status(d);
        // the 8-B index when it is current (gd_microbatch_run keys its graphs by that choice)
        if (mb_use_index(h)) {
            const Cx8Args c8 = cx8_args(h);
            switch (h->ring_mode) {
                case GD_RING_DIRECTORY:
                    GD_TRY(launch(h, "k_mb_route", g, b, ring_lds(h), k_mb_route<GD_RING_DIRECTORY, true>, k, n,
                                  ring_args(h), table_args(h), so, act_dst, st, mb->out_u32(d, 1), mb->ts, c8));
                    break;
                case GD_RING_CONSISTENT:
                    GD_TRY(launch(h, "k_mb_route", g, b, ring_lds(h), k_mb_route<GD_RING_CONSISTENT, true>, k, n,
                                  ring_args(h), table_args(h), so, act_dst, st, mb->out_u32(d, 1), mb->ts, c8));
                    break;
                default:
                    GD_TRY(launch(h, "k_mb_route", g, b, ring_lds(h), k_mb_route<GD_RING_VIRTUAL_BUCKETS, true>, k, n,
                                  ring_args(h), table_args(h), so, act_dst, st, mb->out_u32(d, 1), mb->ts, c8));
                    break;
            }
        } else {
            switch (h->ring_mode) {
                case GD_RING_DIRECTORY:
                    GD_TRY(launch(h, "k_mb_route", g, b, ring_lds(h), k_mb_route<GD_RING_DIRECTORY>, k, n,
                                  ring_args(h), table_args(h), so, act_dst, st, mb->out_u32(d, 1), mb->ts, Cx8Args{}));
                    break;
                case GD_RING_CONSISTENT:
                    GD_TRY(launch(h, "k_mb_route", g, b, ring_lds(h), k_mb_route<GD_RING_CONSISTENT>, k, n,
                                  ring_args(h), table_args(h), so, act_dst, st, mb->out_u32(d, 1), mb->ts, Cx8Args{}));
                    break;
                default:
                    GD_TRY(launch(h, "k_mb_route", g, b, ring_lds(h), k_mb_route<GD_RING_VIRTUAL_BUCKETS>, k, n,
                                  ring_args(h), table_args(h), so, act_dst, st, mb->out_u32(d, 1), mb->ts, Cx8Args{}));
                    break;
            }
        }
    } else if (n) {
        if (!zc)
            HIP_TRY(h, hipMemcpyAsync(mb->d_keys, mb->h_keys, (size_t)n * sizeof(gd_key), hipMemcpyHostToDevice,
                                      h->stream));
        GD_TRY(route_device(h, zc ? mb->h_keys_dev : mb->d_keys, n, mb->out_u32(d, 0), act_dst, mb->out_status(d)));
    }
    const uint32_t* a = act_dst;
    uint32_t *pm = mb->out_u32(d, 2), *ra = mb->out_u32(d, 5), *rs = mb->out_u32(d, 4), *nr = mb->out_u32(d, 3);
    // act to the host block: k_mb_route wrote it already; the LocalLookup route did not
    uint32_t* ac = zc && h->cache_max ? mb->out_u32(d, 1) : nullptr;
    const dim3 g1(mb_sort_grid(mb, n));
    uint32_t* done = count_done ? mb->d_done : nullptr;
    if (n <= MB_THREADS * 4) GD_TRY(mb_launch_sort<4>(mb, g1, bits, a, n, passes, pm, ra, rs, nr, ac, done));
    else GD_TRY(mb_launch_sort<8>(mb, g1, bits, a, n, passes, pm, ra, rs, nr, ac, done));
    if (!zc) HIP_TRY(h, hipMemcpyAsync(mb->h_out, d, mb->out_bytes, hipMemcpyDeviceToHost, h->stream));
    return GD_OK;
}

}  // namespace gdx

extern "C" {

void gd_microbatch_destroy(gd_microbatch* mb) {
    if (!mb) return;
    if (mb->h) (void)hipStreamSynchronize(mb->h->stream);
    if (mb->ts) {
        unsigned long long t[16] = {};
        if (hipMemcpy(t, mb->ts, sizeof(t), hipMemcpyDeviceToHost) == hipSuccess && mb->runs_done) {
            static const char* names[16] = {"", "route.ring", "route.core", "route.fence", "sort.p0.rank",
                                            "sort.pass0.gather", "sort.pass1", "sort.pass2", "sort.pass3",
                                            "sort.runs", "sort.stores", "sort.fence", "sort.clk", "sort.wall",
                                            "sort.p0.scan", "sort.p0.scatter"};
            std::fprintf(stderr, "[gd micro-batch trace] %llu runs, us per run:", (unsigned long long)mb->runs_done);
            for (int k = 0; k < 16; ++k)
                if (t[k]) std::fprintf(stderr, " %s=%.2f", names[k], t[k] * 0.01 / mb->runs_done);
            std::fprintf(stderr, "\n");
        }
        (void)hipFree(mb->ts);
    }
    for (auto& g : mb->graphs) (void)hipGraphExecDestroy(g.second);
    if (mb->h_done) (void)hipHostFree(mb->h_done);
    if (mb->h_keys) (void)hipHostFree(mb->h_keys);
    if (mb->h_out) (void)hipHostFree(mb->h_out);
    if (mb->d_keys) (void)hipFree(mb->d_keys);
    if (mb->d_out) (void)hipFree(mb->d_out);
    if (mb->d_act) (void)hipFree(mb->d_act);

    delete mb;
}

int gd_microbatch_create(gd_handle* h, uint32_t capacity, uint32_t n_act, gd_microbatch** out) {
    if (!h || !out || capacity == 0 || n_act == 0xFFFFFFFFu)
        return set_err(h, GD_EINVAL, "gd_microbatch_create: bad argument");
    if (capacity > MB_MAX) return set_err(h, GD_EINVAL, "micro-batch capacity %u above %u", capacity, MB_MAX);
    HIP_TRY(h, hipSetDevice(h->device));
    gd_microbatch* mb = new (std::nothrow) gd_microbatch();
    if (!mb) return set_err(h, GD_ENOMEM, "out of host memory");
    mb->h = h;
    mb->capacity = capacity;
    mb->n_act = n_act;
    mb->out_bytes = (5 * (size_t)capacity + 2) * 4 + capacity;
    const size_t kb = (size_t)capacity * sizeof(gd_key);
    mb->zero_copy = h->mb_zero_copy;
    mb->split = h->mb_split;
    if (h->mb_trace && hipMalloc((void**)&mb->ts, 16 * sizeof(unsigned long long)) == hipSuccess)
        (void)hipMemset(mb->ts, 0, 16 * sizeof(unsigned long long));
    // coherent (fine-grained) pinned memory: kernel stores reach the host without a cache flush
    const unsigned hf = mb->zero_copy ? hipHostMallocCoherent : hipHostMallocDefault;
    bool ok = hipHostMalloc((void**)&mb->h_keys, kb, hf) == hipSuccess &&
              hipHostMalloc((void**)&mb->h_out, mb->out_bytes, hf) == hipSuccess &&
              hipMalloc((void**)&mb->d_keys, kb) == hipSuccess && hipMalloc((void**)&mb->d_out, mb->out_bytes) == hipSuccess &&
              hipMalloc((void**)&mb->d_act, (size_t)capacity * 4 + 4) == hipSuccess;
    if (ok && mb->zero_copy)
        ok = hipHostGetDevicePointer((void**)&mb->h_keys_dev, mb->h_keys, 0) == hipSuccess &&
             hipHostGetDevicePointer((void**)&mb->h_out_dev, mb->h_out, 0) == hipSuccess;
    if (ok && mb->zero_copy && h->mb_poll) {
        ok = hipHostMalloc((void**)&mb->h_done, 64, hipHostMallocCoherent) == hipSuccess &&
             hipHostGetDevicePointer((void**)&mb->d_done, mb->h_done, 0) == hipSuccess;
        if (ok) *mb->h_done = 0;
    }
    if (!ok) {
        gd_microbatch_destroy(mb);
        return set_err(h, GD_ENOMEM, "gd_microbatch_create: allocation failed");
    }
    std::memset(mb->h_keys, 0, kb);
    std::memset(mb->h_out, 0, mb->out_bytes);
    *out = mb;
    return GD_OK;
}

gd_key* gd_microbatch_keys(gd_microbatch* mb) { return mb ? mb->h_keys : nullptr; }

int gd_microbatch_outputs(gd_microbatch* mb, uint32_t** silo, uint32_t** act, uint8_t** status, uint32_t** perm,
                          uint32_t** n_runs, uint32_t** run_start, uint32_t** run_act) {
    if (!mb) return set_err(nullptr, GD_EINVAL, "null micro-batch");
    if (silo) *silo = mb->out_u32(mb->h_out, 0);
    if (act) *act = mb->out_u32(mb->h_out, 1);
    if (perm) *perm = mb->out_u32(mb->h_out, 2);
    if (n_runs) *n_runs = mb->out_u32(mb->h_out, 3);
    if (run_start) *run_start = mb->out_u32(mb->h_out, 4);
    if (run_act) *run_act = mb->out_u32(mb->h_out, 5);
    if (status) *status = mb->out_status(mb->h_out);
    return GD_OK;
}

}  // extern "C"
namespace gdx {
// The end of a micro-batch graph replay: with the poll, until the sort's workgroups have counted the run done
// (their host stores fenced before), bounded -- a run not done within 2 s (a fault, a lost dispatch)
// falls back to the stream synchronisation, which reports it; else the stream synchronisation.
int mb_wait(gd_microbatch* mb, uint32_t n) {
    gd_handle* h = mb->h;
    if (!mb->d_done) return sync(h);
    mb->done_expect += mb_sort_grid(mb, n);
    const uint32_t want = mb->done_expect;
    volatile uint32_t* d = mb->h_done;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
        if ((int32_t)(*d - want) >= 0) return GD_OK;
        if ((spin & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
    }
    const int r = sync(h);
    if (r != GD_OK) return r;
    if ((int32_t)(*d - want) < 0) return set_err(h, GD_EHIP, "micro-batch: the sort's completion count did not arrive");
    return GD_OK;
}
}  // namespace gdx
extern "C" {

int gd_microbatch_run(gd_microbatch* mb, uint32_t n, int use_graph) {
    if (!mb) return set_err(nullptr, GD_EINVAL, "null micro-batch");
    gd_handle* h = mb->h;
    if (n > mb->capacity) return set_err(h, GD_EINVAL, "n %u above micro-batch capacity %u", n, mb->capacity);
    GD_TRY(check_ring(h));
    HIP_TRY(h, hipSetDevice(h->device));
    // LocalLookup (cache) mode routes through k_route_cached, whose scratch, cache table and silo
    // masks can be reallocated between runs (gd_cache_add rehashes, gd_cache_set_silos, larger
    // gd_route* calls); a captured graph would replay freed pointers.  That mode runs eagerly.
    ++mb->runs_done;
    if (!use_graph || h->cache_max) {
        // eager launches wait on the stream, without the count: polling after them, or the count's
        // system-scope fence and atomic at the sort's end, measured slower (p50 28.7 -> 33.7 / 40.8 us
        // at cfg 5, profiles/r06_mb_poll.json), while a graph replay gains by the poll (35.4 -> 33.5 us)
        GD_TRY(mb_enqueue(mb, n, false));
        return sync(h);
    }
    // ring or table moved, or the probe index was rebuilt (a new layout in the captured arguments) or
    // went stale (a directory change that did not re-project it): drop the captured graphs
    const uint64_t cx_key = mb_use_index(h) ? h->cx_builds : ~0ull;
    if (mb->graphs_gen != h->layout_gen || mb->graphs_cx != cx_key) {
        for (auto& g : mb->graphs) (void)hipGraphExecDestroy(g.second);
        mb->graphs.clear();
        mb->graphs_gen = h->layout_gen;
        mb->graphs_cx = cx_key;
    }
    hipGraphExec_t exec = nullptr;
    for (auto& g : mb->graphs)
        if (g.first == n) exec = g.second;
    if (!exec) {
        // no allocation happens inside mb_enqueue (route needs no scratch), so capture directly
        const int timing = h->timing;
        h->timing = 0;
        hipGraph_t graph = nullptr;
        const uint64_t routed = h->routed;       // counted per replay below, not at capture
        HIP_TRY(h, hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
        const int rc = mb_enqueue(mb, n, mb->d_done != nullptr);
        const hipError_t ec = hipStreamEndCapture(h->stream, &graph);
        h->timing = timing;
        h->routed = routed;
        if (rc != GD_OK) {
            if (graph) (void)hipGraphDestroy(graph);
            return rc;
        }
        if (ec != hipSuccess) return set_err(h, GD_EHIP, "hipStreamEndCapture: %s", hipGetErrorString(ec));
        const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        if (ei != hipSuccess) return set_err(h, GD_EHIP, "hipGraphInstantiate: %s", hipGetErrorString(ei));
        mb->graphs.emplace_back(n, exec);
    }
    HIP_TRY(h, hipGraphLaunch(exec, h->stream));
    h->routed += n;
    return mb_wait(mb, n);
}

}  // extern "C"

// ================================================================== membership change
namespace gdx {

// Mark + scan; returns the number of entries the split selects in *total.
int split_count(gd_handle* h, const uint8_t* keep, uint32_t n_keep, uint64_t* total) {
    GD_TRY(check_ring(h));
    const unsigned long long cap = h->capacity;
    if (cap > 0x7FFFFFFFull) return set_err(h, GD_EINVAL, "split: table of %llu slots too large", cap);
    GD_TRY(h2d(h, h->churn[0], keep, n_keep ? n_keep : 1));
    GD_TRY(ensure(h, h->churn[1], (size_t)cap * 4));
    GD_TRY(ensure(h, h->churn[2], (size_t)cap * 4));
    uint32_t* flag = (uint32_t*)h->churn[1].p;
    uint32_t* pos = (uint32_t*)h->churn[2].p;
    const dim3 g(blocks_for(cap, BLOCK)), b(BLOCK);
    const RingArgs r = ring_args(h);
    const uint8_t* dk = (const uint8_t*)h->churn[0].p;
    switch (h->ring_mode) {
        case GD_RING_DIRECTORY:
            GD_TRY(launch(h, "k_split_mark", g, b, ring_lds(h), k_split_mark<GD_RING_DIRECTORY>, (const Slot*)h->slots,
                          cap, r, dk, n_keep, flag));
            break;
        case GD_RING_CONSISTENT:
            GD_TRY(launch(h, "k_split_mark", g, b, ring_lds(h), k_split_mark<GD_RING_CONSISTENT>, (const Slot*)h->slots,
                          cap, r, dk, n_keep, flag));
            break;
        default:
            GD_TRY(launch(h, "k_split_mark", g, b, ring_lds(h), k_split_mark<GD_RING_VIRTUAL_BUCKETS>,
                          (const Slot*)h->slots, cap, r, dk, n_keep, flag));
    }
    HIP_TRY(h, hipMemcpyAsync(pos, flag, (size_t)cap * 4, hipMemcpyDeviceToDevice, h->stream));
    GD_TRY(scan_device<OpAdd>(h, pos, (uint32_t)cap, false, false, "split"));
    uint32_t last[2] = {0, 0};
    HIP_TRY(h, hipMemcpyAsync(&last[0], pos + cap - 1, 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipMemcpyAsync(&last[1], flag + cap - 1, 4, hipMemcpyDeviceToHost, h->stream));
    GD_TRY(sync(h));
    *total = (uint64_t)last[0] + last[1];
    return GD_OK;
}

int split_emit(gd_handle* h, int move, gd_key* d_keys, gd_val* d_vals) {
    const unsigned long long cap = h->capacity;
    return launch(h, "k_split_emit", dim3(blocks_for(cap, BLOCK)), dim3(BLOCK), 0, k_split_emit, h->slots, cap,
                  (const uint32_t*)h->churn[1].p, (const uint32_t*)h->churn[2].p, move, d_keys, d_vals, h->ctr);
}

}  // namespace gdx

extern "C" {

int gd_dir_split_device(gd_handle* h, const uint8_t* keep_silo, uint32_t n_keep, int move, gd_key* d_out_keys,
                        gd_val* d_out_vals, uint64_t out_capacity, uint64_t* out_n) {
    if (!h || !out_n || (n_keep && !keep_silo)) return set_err(h, GD_EINVAL, "null argument");
    if ((d_out_keys == nullptr) != (d_out_vals == nullptr)) return set_err(h, GD_EINVAL, "keys and vals go together");
    HIP_TRY(h, hipSetDevice(h->device));
    uint64_t total = 0;
    GD_TRY(split_count(h, keep_silo, n_keep, &total));
    *out_n = total;
    if (!d_out_keys || total == 0) return GD_OK;                  // size query
    if (total > out_capacity)
        return set_err(h, GD_EINVAL, "split selects %llu entries, output holds %llu", (unsigned long long)total,
                       (unsigned long long)out_capacity);
    GD_TRY(split_emit(h, move, d_out_keys, d_out_vals));
    return sync_checked(h);
}

int gd_dir_split(gd_handle* h, const uint8_t* keep_silo, uint32_t n_keep, int move, gd_key* out_keys,
                 gd_val* out_vals, uint64_t out_capacity, uint64_t* out_n) {
    if (!h || !out_n || (n_keep && !keep_silo)) return set_err(h, GD_EINVAL, "null argument");
    if ((out_keys == nullptr) != (out_vals == nullptr)) return set_err(h, GD_EINVAL, "keys and vals go together");
    HIP_TRY(h, hipSetDevice(h->device));
    uint64_t total = 0;
    GD_TRY(split_count(h, keep_silo, n_keep, &total));
    *out_n = total;
    if (!out_keys || total == 0) return GD_OK;
    if (total > out_capacity)
        return set_err(h, GD_EINVAL, "split selects %llu entries, output holds %llu", (unsigned long long)total,
                       (unsigned long long)out_capacity);
    GD_TRY(ensure(h, h->churn[3], (size_t)total * sizeof(gd_key)));
    GD_TRY(ensure(h, h->churn[4], (size_t)total * sizeof(gd_val)));
    GD_TRY(split_emit(h, move, (gd_key*)h->churn[3].p, (gd_val*)h->churn[4].p));
    HIP_TRY(h, hipMemcpyAsync(out_keys, h->churn[3].p, (size_t)total * sizeof(gd_key), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipMemcpyAsync(out_vals, h->churn[4].p, (size_t)total * sizeof(gd_val), hipMemcpyDeviceToHost, h->stream));
    return sync_checked(h);
}

}  // extern "C"
