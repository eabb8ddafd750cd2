// eng_frames.hip -- libgraindispatch: header decode and the receive path (ActivationDirectory + ReceiveMessage).
// Shared handle and helpers: gd_engine.h.
#include "gd_engine.h"

// ================================================================== header decode
namespace gdx {

FrameFields frame_fields(const gd_frame_fields* f) {
    return FrameFields{f->flags,
                       (uint64_t*)f->target_grain,
                       f->mask,
                       (uint64_t*)f->target_activation,
                       (uint64_t*)f->sending_activation,
                       (uint64_t*)f->sending_grain,
                       (uint32_t*)f->target_silo,
                       (uint32_t*)f->sending_silo,
                       f->correlation_id,
                       f->category,
                       f->direction,
                       nullptr,
                       nullptr};
}

int check_frames_args(gd_handle* h, const void* buf, const void* off, uint32_t n, const gd_frame_fields* out) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    if (n == 0) return GD_OK;
    if (!buf || !off || !out || !out->flags || !out->target_grain) return set_err(h, GD_EINVAL, "null argument");
    if (((uintptr_t)out->target_silo | (uintptr_t)out->sending_silo) & 3)
        return set_err(h, GD_EINVAL, "silo outputs must be 4-byte aligned");
    return GD_OK;
}

int decode_frames_device(gd_handle* h, const uint8_t* buf, uint64_t len, const uint64_t* off, uint32_t n,
                         const gd_frame_fields* out, bool ext) {
    FrameFields ff = frame_fields(out);
    if (ext) {                          // where each TargetGrain's KeyExt string lies in buf
        GD_TRY(ensure(h, h->fr_ext[0], (size_t)n * 8 + 8));
        GD_TRY(ensure(h, h->fr_ext[1], (size_t)n * 4 + 4));
        ff.tg_ext_off = (uint64_t*)h->fr_ext[0].p;
        ff.tg_ext_len = (int32_t*)h->fr_ext[1].p;
    }
    return launch(h, "k_decode_frames", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), 0, k_decode_frames, buf, len, off, n,
                  ff);
}

// ext: KeyExt targets (string-keyed grains) are routed too, their strings read from buf itself.

// ext: KeyExt targets (string-keyed grains) are routed too, their strings read from buf itself.  With an
// ActivationDirectory (gd_actdir_add), a frame whose address is complete (GD_ROUTE_ADDRESSED) gets the
// context of its TargetActivation as its act (k_frame_addressed_act), so it is bucketed with it.
int route_frames_device(gd_handle* h, const uint8_t* buf, uint64_t len, const uint64_t* off, uint32_t n,
                        uint32_t n_act, const gd_frame_fields* out, uint32_t* silo, uint32_t* act, uint8_t* status,
                        uint32_t* perm, uint32_t* offsets, bool ext) {
    if (n) {
        GD_TRY(check_ring(h));
        gd_frame_fields o2 = *out;
        if (h->ad_slots && !o2.target_activation) {
            GD_TRY(ensure(h, h->fr_recv[0], (size_t)n * sizeof(gd_key) + 8));
            o2.target_activation = (gd_key*)h->fr_recv[0].p;
        }
        GD_TRY(decode_frames_device(h, buf, len, off, n, &o2, ext));
        GD_TRY(route_device(h, o2.target_grain, n, silo, act, status, !ext));
        if (ext)
            GD_TRY(keyext_pass(h, o2.target_grain,
                               ExtArgs{buf, (const uint64_t*)h->fr_ext[0].p, (const int32_t*)h->fr_ext[1].p, len}, n,
                               silo, act, status));
        GD_TRY(launch(h, "k_frame_status", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), 0, k_frame_status,
                      (const uint32_t*)o2.flags, n, silo, act, status));
        if (h->ad_slots)
            GD_TRY(launch(h, "k_frame_addressed_act", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), 0, k_frame_addressed_act,
                          (const uint8_t*)status, (const gd_key*)o2.target_grain, (const gd_key*)o2.target_activation, n,
                          ad_args(h), act));
    }
    if (perm && offsets) GD_TRY(bucket_device(h, act, n, n_act, perm, offsets));
    return GD_OK;
}

// Host-pointer outputs -> device scratch fr[2..12] (fr[0] buffer, fr[1] offsets).
int frame_scratch(gd_handle* h, uint32_t n, const gd_frame_fields* want, gd_frame_fields* dev) {
    const size_t sz[11] = {4, 24, 4, 24, 24, 24, 24, 24, 8, 1, 1};
    void* const* w = (void* const*)want;
    void** d = (void**)dev;
    for (int k = 0; k < 11; ++k) {
        d[k] = nullptr;
        if (k < 2 || (w && w[k])) {
            GD_TRY(ensure(h, h->fr[2 + k], sz[k] * n + 8));
            d[k] = h->fr[2 + k].p;
        }
    }
    return GD_OK;
}

int frame_results(gd_handle* h, uint32_t n, const gd_frame_fields* want, const gd_frame_fields* dev) {
    if (!want) return GD_OK;
    const size_t sz[11] = {4, 24, 4, 24, 24, 24, 24, 24, 8, 1, 1};
    void* const* w = (void* const*)want;
    void* const* d = (void* const*)dev;
    for (int k = 0; k < 11; ++k)
        if (w[k] && d[k]) HIP_TRY(h, hipMemcpyAsync(w[k], d[k], sz[k] * n, hipMemcpyDeviceToHost, h->stream));
    return GD_OK;
}

}  // namespace gdx

extern "C" {

int gd_decode_frames_device(gd_handle* h, const uint8_t* d_buf, uint64_t buf_len, const uint64_t* d_frame_off,
                            uint32_t n, const gd_frame_fields* d_out) {
    GD_TRY(check_frames_args(h, d_buf, d_frame_off, n, d_out));
    return n ? decode_frames_device(h, d_buf, buf_len, d_frame_off, n, d_out) : GD_OK;
}

int gd_decode_frames(gd_handle* h, const uint8_t* buf, uint64_t buf_len, const uint64_t* frame_off, uint32_t n,
                     const gd_frame_fields* out) {
    GD_TRY(check_frames_args(h, buf, frame_off, n, out));
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(h2d(h, h->fr[0], buf, (size_t)buf_len));
    GD_TRY(h2d(h, h->fr[1], frame_off, n));
    gd_frame_fields dev{};
    GD_TRY(frame_scratch(h, n, out, &dev));
    GD_TRY(decode_frames_device(h, (const uint8_t*)h->fr[0].p, buf_len, (const uint64_t*)h->fr[1].p, n, &dev));
    GD_TRY(frame_results(h, n, out, &dev));
    return sync(h);
}

static int route_frames_device_abi(gd_handle* h, const uint8_t* d_buf, uint64_t buf_len, const uint64_t* d_frame_off,
                                   uint32_t n, uint32_t n_act, const gd_frame_fields* d_out, uint32_t* d_silo,
                                   uint32_t* d_act, uint8_t* d_status, uint32_t* d_perm, uint32_t* d_offsets,
                                   bool ext) {
    GD_TRY(check_frames_args(h, d_buf, d_frame_off, n, d_out));
    if (n && (!d_silo || !d_act || !d_status)) return set_err(h, GD_EINVAL, "null argument");
    if ((d_perm != nullptr) != (d_offsets != nullptr)) return set_err(h, GD_EINVAL, "perm and offsets go together");
    if (d_perm && n_act == 0xFFFFFFFFu) return set_err(h, GD_EINVAL, "n_act too large");
    return route_frames_device(h, d_buf, buf_len, d_frame_off, n, n_act, d_out, d_silo, d_act, d_status, d_perm,
                               d_offsets, ext);
}

int gd_route_frames_device(gd_handle* h, const uint8_t* d_buf, uint64_t buf_len, const uint64_t* d_frame_off,
                           uint32_t n, uint32_t n_act, const gd_frame_fields* d_out, uint32_t* d_silo,
                           uint32_t* d_act, uint8_t* d_status, uint32_t* d_perm, uint32_t* d_offsets) {
    return route_frames_device_abi(h, d_buf, buf_len, d_frame_off, n, n_act, d_out, d_silo, d_act, d_status, d_perm,
                                   d_offsets, false);
}

int gd_route_frames_ext_device(gd_handle* h, const uint8_t* d_buf, uint64_t buf_len, const uint64_t* d_frame_off,
                               uint32_t n, uint32_t n_act, const gd_frame_fields* d_out, uint32_t* d_silo,
                               uint32_t* d_act, uint8_t* d_status, uint32_t* d_perm, uint32_t* d_offsets) {
    return route_frames_device_abi(h, d_buf, buf_len, d_frame_off, n, n_act, d_out, d_silo, d_act, d_status, d_perm,
                                   d_offsets, true);
}

static int route_frames_host(gd_handle* h, const uint8_t* buf, uint64_t buf_len, const uint64_t* frame_off, uint32_t n,
                             uint32_t n_act, const gd_frame_fields* out, uint32_t* out_silo, uint32_t* out_act,
                             uint8_t* out_status, uint32_t* out_perm, uint32_t* out_offsets, bool ext) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    if (n && (!buf || !frame_off || !out_silo || !out_act || !out_status)) return set_err(h, GD_EINVAL, "null argument");
    if ((out_perm != nullptr) != (out_offsets != nullptr)) return set_err(h, GD_EINVAL, "perm and offsets go together");
    if (out_perm && n_act == 0xFFFFFFFFu) return set_err(h, GD_EINVAL, "n_act too large");
    if (out && (((uintptr_t)out->target_silo | (uintptr_t)out->sending_silo) & 3))
        return set_err(h, GD_EINVAL, "silo outputs must be 4-byte aligned");
    HIP_TRY(h, hipSetDevice(h->device));
    if (n) {
        GD_TRY(h2d(h, h->fr[0], buf, (size_t)buf_len));
        GD_TRY(h2d(h, h->fr[1], frame_off, n));
    }
    gd_frame_fields dev{};
    GD_TRY(frame_scratch(h, n, out, &dev));
    GD_TRY(ensure(h, h->fr[13], (size_t)n * 4 + 4));     // silo
    GD_TRY(ensure(h, h->fr[14], (size_t)n * 4 + 4));     // act
    GD_TRY(ensure(h, h->fr[15], (size_t)n + 8));         // status
    uint32_t* perm = nullptr;
    uint32_t* offs = nullptr;
    if (out_perm) {
        GD_TRY(ensure(h, h->u8_a, (size_t)n * 4 + 4));
        GD_TRY(ensure(h, h->offs, ((size_t)n_act + 2) * 4));
        perm = (uint32_t*)h->u8_a.p;
        offs = (uint32_t*)h->offs.p;
    }
    GD_TRY(route_frames_device(h, (const uint8_t*)h->fr[0].p, buf_len, (const uint64_t*)h->fr[1].p, n, n_act, &dev,
                               (uint32_t*)h->fr[13].p, (uint32_t*)h->fr[14].p, (uint8_t*)h->fr[15].p, perm, offs,
                               ext));
    GD_TRY(frame_results(h, n, out, &dev));
    if (n) {
        HIP_TRY(h, hipMemcpyAsync(out_silo, h->fr[13].p, (size_t)n * 4, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(h, hipMemcpyAsync(out_act, h->fr[14].p, (size_t)n * 4, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(h, hipMemcpyAsync(out_status, h->fr[15].p, (size_t)n, hipMemcpyDeviceToHost, h->stream));
    }
    if (out_perm) {
        if (n) HIP_TRY(h, hipMemcpyAsync(out_perm, perm, (size_t)n * 4, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(h, hipMemcpyAsync(out_offsets, offs, ((size_t)n_act + 2) * 4, hipMemcpyDeviceToHost, h->stream));
    }
    return sync_checked(h);
}

int gd_route_frames(gd_handle* h, const uint8_t* buf, uint64_t buf_len, const uint64_t* frame_off, uint32_t n,
                    uint32_t n_act, const gd_frame_fields* out, uint32_t* out_silo, uint32_t* out_act,
                    uint8_t* out_status, uint32_t* out_perm, uint32_t* out_offsets) {
    return route_frames_host(h, buf, buf_len, frame_off, n, n_act, out, out_silo, out_act, out_status, out_perm,
                             out_offsets, false);
}

int gd_route_frames_ext(gd_handle* h, const uint8_t* buf, uint64_t buf_len, const uint64_t* frame_off, uint32_t n,
                        uint32_t n_act, const gd_frame_fields* out, uint32_t* out_silo, uint32_t* out_act,
                        uint8_t* out_status, uint32_t* out_perm, uint32_t* out_offsets) {
    return route_frames_host(h, buf, buf_len, frame_off, n, n_act, out, out_silo, out_act, out_status, out_perm,
                             out_offsets, true);
}

}  // extern "C"

// ================================================================== receive path: ActivationDirectory +
// IncomingMessageAgent.ReceiveMessage (gd_actdir.h)
namespace gdx {

AdArgs ad_args(gd_handle* h) { return AdArgs{h->ad_slots, h->ad_cap ? h->ad_cap - 1 : 0ull, h->ad_ctr}; }


// Frames -> decode (TargetGrain, TargetActivation, Direction into the caller's arrays or scratch)
// -> ReceiveMessage -> bucketing.  Frames without a complete decoded address: RECV_UNDECODED.
int receive_frames_device(gd_handle* h, const uint8_t* buf, uint64_t len, const uint64_t* off, uint32_t n,
                          uint32_t n_ctx, const gd_recv_limits* lim, const gd_frame_fields* out, uint32_t* ctx,
                          uint8_t* st, uint32_t* perm, uint32_t* offsets) {
    gd_frame_fields o2 = *out;
    if (n) {
        if (!o2.target_activation) {
            GD_TRY(ensure(h, h->fr_recv[0], (size_t)n * sizeof(gd_key) + 8));
            o2.target_activation = (gd_key*)h->fr_recv[0].p;
        }
        if (!o2.direction) {
            GD_TRY(ensure(h, h->fr_recv[1], (size_t)n + 8));
            o2.direction = (uint8_t*)h->fr_recv[1].p;
        }
        GD_TRY(decode_frames_device(h, buf, len, off, n, &o2));
    }
    return receive_device(h, o2.target_grain, o2.target_activation, o2.direction, (const uint32_t*)o2.flags, n, n_ctx,
                          lim, ctx, st, perm, offsets);
}

int ad_pull(gd_handle* h) {
    GD_TRY(fold_counters(h, h->ad_ctr));
    HIP_TRY(h, hipMemcpyAsync(&h->ad_host, h->ad_ctr, sizeof(DevCounters), hipMemcpyDeviceToHost, h->stream));
    return sync(h);
}

// (Re)build the ActivationDirectory table with cap slots (tombstones dropped).
int ad_rehash(gd_handle* h, unsigned long long cap) {
    Slot* ns = nullptr;
    GD_TRY(alloc_table(h, cap, &ns));
    if (!h->ad_ctr) {
        hipError_t e = hipMalloc(&h->ad_ctr, CTR_BYTES);
        if (e != hipSuccess) {
            (void)hipFree(ns);
            return set_err(h, GD_ENOMEM, "activation directory counters: %s", hipGetErrorString(e));
        }
    }
    HIP_TRY(h, hipMemsetAsync(h->ad_ctr, 0, CTR_BYTES, h->stream));   // counters and their striped deltas
    if (h->ad_slots) {
        GD_TRY(launch(h, "k_rehash", dim3((uint32_t)((h->ad_cap + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, k_rehash,
                      (const Slot*)h->ad_slots, h->ad_cap, ns, cap - 1, h->ad_ctr, (const uint32_t*)nullptr,
                      (uint32_t*)nullptr));
        GD_TRY(sync(h));
        HIP_TRY(h, hipFree(h->ad_slots));
    }
    h->ad_slots = ns;
    h->ad_cap = cap;
    free_buf(h->ad_last);
    GD_TRY(ensure(h, h->ad_last, cap * 4));
    HIP_TRY(h, hipMemsetAsync(h->ad_last.p, 0, cap * 4, h->stream));
    h->layout_gen++;
    GD_TRY(ad_pull(h));
    if (h->ad_host.err) return set_err(h, GD_EFULL, "activation directory rehash failed (0x%x)", h->ad_host.err);
    return GD_OK;
}

int ad_reserve(gd_handle* h, uint64_t incoming) {
    if (!h->ad_slots) return ad_rehash(h, pow2_at_least(std::max<uint64_t>(2 * incoming, 1024)));
    GD_TRY(ad_pull(h));
    if ((h->ad_host.live + h->ad_host.tomb + incoming) * 4 <= h->ad_cap * 3) return GD_OK;
    unsigned long long cap = h->ad_cap;
    while ((h->ad_host.live + incoming) * 2 > cap) cap <<= 1;
    return ad_rehash(h, cap);
}

// ReceiveMessage for n messages already in HBM; ctx / status / perm / offsets device arrays.
int receive_device(gd_handle* h, const gd_key* tg, const gd_key* ta, const uint8_t* dir, const uint32_t* fflags,
                   uint32_t n, uint32_t n_ctx, const gd_recv_limits* lim, uint32_t* ctx, uint8_t* st, uint32_t* perm,
                   uint32_t* offsets) {
    if (n_ctx >= 0xFFFFFFFDu) return set_err(h, GD_EINVAL, "n_ctx too large");
    if (!h->ad_slots) GD_TRY(ad_rehash(h, 1024));
    const bool limits = lim && lim->request_count && (lim->hard_limit > 0 || lim->hard_limit_stateless_worker > 0);
    const dim3 g(blocks_for(n, BLOCK)), b(BLOCK);
    if (n) {
        if (limits)
            GD_TRY(launch(h, "k_receive", g, b, 0, k_receive<true>, tg, ta, dir, fflags, n, n_ctx, ad_args(h), ctx, st,
                          &h->ctr->err));
        else
            GD_TRY(launch(h, "k_receive", g, b, 0, k_receive<false>, tg, ta, dir, fflags, n, n_ctx, ad_args(h), ctx, st,
                          &h->ctr->err));
    }
    if (!perm && !(limits && n)) return GD_OK;
    const bool want_buckets = perm != nullptr;
    if (!want_buckets) {
        // CheckOverloaded needs each message's place in its activation's FIFO: bucket into scratch
        // (the caller asked for statuses only), then drop the buckets.
        GD_TRY(ensure(h, h->recv_scr[0], (size_t)n * 4 + 4));
        GD_TRY(ensure(h, h->recv_scr[1], ((size_t)n_ctx + 3) * 4));
        perm = (uint32_t*)h->recv_scr[0].p;
        offsets = (uint32_t*)h->recv_scr[1].p;
    }
    // buckets 0..n_ctx-1 contexts, n_ctx the null context, n_ctx + 1 not enqueued (ctx NONE32 clamps there)
    uint32_t* rank = nullptr;
    if (limits && n) {
        GD_TRY(ensure(h, h->fr_recv[2], (size_t)n * 4));
        rank = (uint32_t*)h->fr_recv[2].p;
    }
    GD_TRY(bucket_device(h, ctx, n, n_ctx + 1, perm, offsets, rank));
    if (limits && n) {
        GD_TRY(launch(h, "k_overload", g, b, 0, k_overload, (const uint32_t*)rank, (const uint32_t*)offsets, n, dir,
                      lim->request_count, lim->hard_limit, lim->hard_limit_stateless_worker, ctx, st));
        if (want_buckets) GD_TRY(bucket_device(h, ctx, n, n_ctx + 1, perm, offsets));
    }
    return GD_OK;
}

}  // namespace gdx

extern "C" {

int gd_actdir_add(gd_handle* h, const gd_key* act_ids, const uint32_t* ctx, const uint8_t* flags, uint32_t n,
                  uint8_t* out_added) {
    if (!h || (n && (!act_ids || !ctx || !flags))) return set_err(h, GD_EINVAL, "null argument");
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(ad_reserve(h, n));
    std::vector<gd_val> vals(n);
    for (uint32_t i = 0; i < n; ++i) vals[i] = gd_val{ctx[i], flags[i]};
    GD_TRY(h2d(h, h->ad_buf[0], act_ids, n));
    GD_TRY(h2d(h, h->ad_buf[1], vals.data(), n));
    GD_TRY(ensure(h, h->ad_buf[2], (size_t)n * 4));   // slot_of
    GD_TRY(ensure(h, h->ad_buf[3], (size_t)n * 4));   // win
    GD_TRY(ensure(h, h->ad_buf[4], (size_t)n));       // is_new
    GD_TRY(ensure(h, h->ad_buf[5], (size_t)n));       // added
    HIP_TRY(h, hipMemsetAsync(h->ad_buf[4].p, 0, n, h->stream));
    const dim3 g(blocks_for(n, BLOCK)), b(BLOCK);
    const gd_key* dk = (const gd_key*)h->ad_buf[0].p;
    uint32_t* slot_of = (uint32_t*)h->ad_buf[2].p;
    uint32_t* win = (uint32_t*)h->ad_buf[3].p;
    uint8_t* is_new = (uint8_t*)h->ad_buf[4].p;
    for (uint32_t pass = 0;; ++pass) {            // TryAdd: the registration's claim protocol, first add wins
        HIP_TRY(h, hipMemsetAsync(&h->ad_ctr->retry, 0, sizeof(uint32_t), h->stream));
        GD_TRY(launch(h, "k_reg_claim", g, b, 0, k_reg_claim, dk, n, h->ad_slots, h->ad_cap - 1, h->ad_ctr, slot_of,
                      is_new, pass, (const gd_val*)nullptr, TableArgs{}, (uint32_t*)nullptr));
        GD_TRY(ad_pull(h));
        if (h->ad_host.retry == 0 || h->ad_host.err) break;
        if (pass >= 64) return set_err(h, GD_ETIMEOUT, "gd_actdir_add: claims did not settle");
    }
    GD_TRY(launch(h, "k_reg_minwin", g, b, 0, k_reg_minwin, (const uint32_t*)slot_of, (const uint8_t*)is_new, n,
                  h->ad_slots));
    GD_TRY(launch(h, "k_reg_resolve", g, b, 0, k_reg_resolve, (const uint32_t*)slot_of, (const uint8_t*)is_new, n,
                  (const Slot*)h->ad_slots, win));
    GD_TRY(launch(h, "k_reg_commit", g, b, 0, k_reg_commit, (const uint32_t*)slot_of, (const uint32_t*)win,
                  (const gd_val*)h->ad_buf[1].p, n, h->ad_slots, h->ad_ctr, (uint32_t*)nullptr, 0u));
    GD_TRY(launch(h, "k_reg_report", g, b, 0, k_reg_report, (const uint32_t*)slot_of, (const uint32_t*)win, n,
                  (const Slot*)h->ad_slots, (gd_val*)nullptr, (uint8_t*)h->ad_buf[5].p));
    if (out_added) HIP_TRY(h, hipMemcpyAsync(out_added, h->ad_buf[5].p, n, hipMemcpyDeviceToHost, h->stream));
    GD_TRY(ad_pull(h));
    if (h->ad_host.err) return set_err(h, GD_EFULL, "gd_actdir_add: device error bits 0x%x", h->ad_host.err);
    return GD_OK;
}

int gd_actdir_remove(gd_handle* h, const gd_key* act_ids, uint32_t n, uint8_t* out_removed) {
    if (!h || (n && !act_ids)) return set_err(h, GD_EINVAL, "null argument");
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    if (!h->ad_slots) {
        if (out_removed) std::memset(out_removed, 0, n);
        return GD_OK;
    }
    GD_TRY(h2d(h, h->ad_buf[0], act_ids, n));
    GD_TRY(ensure(h, h->ad_buf[2], (size_t)n * 4));
    GD_TRY(ensure(h, h->ad_buf[5], (size_t)n));
    const dim3 g(blocks_for(n, BLOCK)), b(BLOCK);
    uint32_t* slot_of = (uint32_t*)h->ad_buf[2].p;
    // TryRemove: the first item of a key removes it (the unregistration election, gd_kernels.h)
    GD_TRY(launch(h, "k_ad_find", g, b, 0, k_ad_find, (const gd_key*)h->ad_buf[0].p, n, ad_args(h), slot_of));
    GD_TRY(launch(h, "k_unreg_poison", g, b, 0, k_unreg_poison, (const uint32_t*)slot_of, n, h->ad_slots));
    GD_TRY(launch(h, "k_unreg_min", g, b, 0, k_unreg_min, (const uint32_t*)slot_of, n, h->ad_slots));
    GD_TRY(launch(h, "k_unreg_commit", g, b, 0, k_unreg_commit, (const uint32_t*)slot_of, n, h->ad_slots, h->ad_ctr,
                  (uint8_t*)h->ad_buf[5].p));
    if (out_removed) HIP_TRY(h, hipMemcpyAsync(out_removed, h->ad_buf[5].p, n, hipMemcpyDeviceToHost, h->stream));
    return sync(h);
}

int gd_actdir_set_flags(gd_handle* h, const gd_key* act_ids, const uint8_t* flags, uint32_t n, uint8_t* out_found) {
    if (!h || (n && (!act_ids || !flags))) return set_err(h, GD_EINVAL, "null argument");
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    if (!h->ad_slots) GD_TRY(ad_rehash(h, 1024));
    GD_TRY(h2d(h, h->ad_buf[0], act_ids, n));
    GD_TRY(h2d(h, h->ad_buf[1], flags, n));
    GD_TRY(ensure(h, h->ad_buf[2], (size_t)n * 4));
    GD_TRY(ensure(h, h->ad_buf[5], (size_t)n));
    const dim3 g(blocks_for(n, BLOCK)), b(BLOCK);
    uint32_t* slot_of = (uint32_t*)h->ad_buf[2].p;
    uint32_t* last = (uint32_t*)h->ad_last.p;
    GD_TRY(launch(h, "k_ad_find", g, b, 0, k_ad_find, (const gd_key*)h->ad_buf[0].p, n, ad_args(h), slot_of));
    GD_TRY(launch(h, "k_up_last", g, b, 0, k_up_last, (const uint32_t*)slot_of, n, last));
    GD_TRY(launch(h, "k_ad_setflags", g, b, 0, k_ad_setflags, (const uint32_t*)slot_of, (const uint8_t*)h->ad_buf[1].p, n,
                  (const uint32_t*)last, h->ad_slots, (uint8_t*)h->ad_buf[5].p));
    GD_TRY(launch(h, "k_up_clear", g, b, 0, k_up_clear, (const uint32_t*)slot_of, n, last));
    if (out_found) HIP_TRY(h, hipMemcpyAsync(out_found, h->ad_buf[5].p, n, hipMemcpyDeviceToHost, h->stream));
    return sync(h);
}

int gd_actdir_lookup(gd_handle* h, const gd_key* act_ids, uint32_t n, uint32_t* out_ctx, uint8_t* out_flags,
                     uint8_t* out_found) {
    if (!h || (n && (!act_ids || !out_ctx || !out_flags || !out_found))) return set_err(h, GD_EINVAL, "null argument");
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    if (!h->ad_slots) GD_TRY(ad_rehash(h, 1024));
    GD_TRY(h2d(h, h->ad_buf[0], act_ids, n));
    GD_TRY(ensure(h, h->ad_buf[2], (size_t)n * 4));
    GD_TRY(ensure(h, h->ad_buf[4], (size_t)n));
    GD_TRY(ensure(h, h->ad_buf[5], (size_t)n));
    GD_TRY(launch(h, "k_ad_lookup", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), 0, k_ad_lookup,
                  (const gd_key*)h->ad_buf[0].p, n, ad_args(h), (uint32_t*)h->ad_buf[2].p, (uint8_t*)h->ad_buf[4].p,
                  (uint8_t*)h->ad_buf[5].p));
    HIP_TRY(h, hipMemcpyAsync(out_ctx, h->ad_buf[2].p, (size_t)n * 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipMemcpyAsync(out_flags, h->ad_buf[4].p, n, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipMemcpyAsync(out_found, h->ad_buf[5].p, n, hipMemcpyDeviceToHost, h->stream));
    return sync(h);
}

int gd_actdir_clear(gd_handle* h) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    HIP_TRY(h, hipSetDevice(h->device));
    if (!h->ad_slots) return GD_OK;
    HIP_TRY(h, hipMemsetAsync(h->ad_slots, 0, h->ad_cap * sizeof(Slot), h->stream));
    HIP_TRY(h, hipMemsetAsync(h->ad_ctr, 0, CTR_BYTES, h->stream));
    return sync(h);
}

int gd_actdir_count(gd_handle* h, uint64_t* out_live) {
    if (!h || !out_live) return set_err(h, GD_EINVAL, "null argument");
    HIP_TRY(h, hipSetDevice(h->device));
    *out_live = 0;
    if (!h->ad_slots) return GD_OK;
    GD_TRY(ad_pull(h));
    *out_live = h->ad_host.live;
    return GD_OK;
}

int gd_receive_device(gd_handle* h, const gd_key* d_target_grain, const gd_key* d_target_activation,
                      const uint8_t* d_direction, uint32_t n, uint32_t n_ctx, const gd_recv_limits* limits,
                      uint32_t* d_ctx, uint8_t* d_status, uint32_t* d_perm, uint32_t* d_offsets) {
    if (!h || (n && (!d_target_grain || !d_target_activation || !d_ctx || !d_status)))
        return set_err(h, GD_EINVAL, "null argument");
    if ((d_perm != nullptr) != (d_offsets != nullptr)) return set_err(h, GD_EINVAL, "perm and offsets go together");
    HIP_TRY(h, hipSetDevice(h->device));
    return receive_device(h, d_target_grain, d_target_activation, d_direction, nullptr, n, n_ctx, limits, d_ctx, d_status,
                          d_perm, d_offsets);
}

int gd_receive(gd_handle* h, const gd_key* target_grain, const gd_key* target_activation, const uint8_t* direction,
               uint32_t n, uint32_t n_ctx, const gd_recv_limits* limits, uint32_t* out_ctx, uint8_t* out_status,
               uint32_t* out_perm, uint32_t* out_offsets) {
    if (!h || (n && (!target_grain || !target_activation || !out_ctx || !out_status)))
        return set_err(h, GD_EINVAL, "null argument");
    if ((out_perm != nullptr) != (out_offsets != nullptr)) return set_err(h, GD_EINVAL, "perm and offsets go together");
    if (n_ctx >= 0xFFFFFFFDu) return set_err(h, GD_EINVAL, "n_ctx too large");
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(h2d(h, h->keys_in, target_grain, n));
    GD_TRY(h2d(h, h->ad_buf[6], target_activation, n));
    const uint8_t* ddir = nullptr;
    if (direction) {
        GD_TRY(h2d(h, h->ad_buf[7], direction, n));
        ddir = (const uint8_t*)h->ad_buf[7].p;
    }
    gd_recv_limits dl{};
    const gd_recv_limits* pl = nullptr;
    if (limits && limits->request_count) {
        GD_TRY(h2d(h, h->dirop_buf[0], limits->request_count, n_ctx));
        dl = *limits;
        dl.request_count = (const uint32_t*)h->dirop_buf[0].p;
        pl = &dl;
    }
    GD_TRY(ensure(h, h->out_a, (size_t)n * 4 + 4));
    GD_TRY(ensure(h, h->out_c, (size_t)n + 4));
    uint32_t* perm = nullptr;
    uint32_t* offs = nullptr;
    if (out_perm) {
        GD_TRY(ensure(h, h->u8_a, (size_t)n * 4 + 4));
        GD_TRY(ensure(h, h->offs, ((size_t)n_ctx + 3) * 4));
        perm = (uint32_t*)h->u8_a.p;
        offs = (uint32_t*)h->offs.p;
    }
    GD_TRY(receive_device(h, (const gd_key*)h->keys_in.p, (const gd_key*)h->ad_buf[6].p, ddir, nullptr, n, n_ctx, pl,
                          (uint32_t*)h->out_a.p, (uint8_t*)h->out_c.p, perm, offs));
    GD_TRY(d2h(h, out_ctx, h->out_a, n));
    if (n) HIP_TRY(h, hipMemcpyAsync(out_status, h->out_c.p, n, hipMemcpyDeviceToHost, h->stream));
    if (out_perm) {
        GD_TRY(d2h(h, out_perm, h->u8_a, n));
        HIP_TRY(h, hipMemcpyAsync(out_offsets, offs, ((size_t)n_ctx + 3) * 4, hipMemcpyDeviceToHost, h->stream));
    }
    return sync_checked(h);
}

}  // extern "C"

extern "C" {

int gd_receive_frames_device(gd_handle* h, const uint8_t* d_buf, uint64_t buf_len, const uint64_t* d_frame_off,
                             uint32_t n, uint32_t n_ctx, const gd_recv_limits* limits, const gd_frame_fields* d_out,
                             uint32_t* d_ctx, uint8_t* d_status, uint32_t* d_perm, uint32_t* d_offsets) {
    GD_TRY(check_frames_args(h, d_buf, d_frame_off, n, d_out));
    if (n && (!d_ctx || !d_status)) return set_err(h, GD_EINVAL, "null argument");
    if ((d_perm != nullptr) != (d_offsets != nullptr)) return set_err(h, GD_EINVAL, "perm and offsets go together");
    if (n_ctx >= 0xFFFFFFFDu) return set_err(h, GD_EINVAL, "n_ctx too large");
    HIP_TRY(h, hipSetDevice(h->device));
    gd_frame_fields none{};
    return receive_frames_device(h, d_buf, buf_len, d_frame_off, n, n_ctx, limits, d_out ? d_out : &none, d_ctx, d_status,
                                 d_perm, d_offsets);
}

int gd_receive_frames(gd_handle* h, const uint8_t* buf, uint64_t buf_len, const uint64_t* frame_off, uint32_t n,
                      uint32_t n_ctx, const gd_recv_limits* limits, const gd_frame_fields* out, uint32_t* out_ctx,
                      uint8_t* out_status, uint32_t* out_perm, uint32_t* out_offsets) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    if (n && (!buf || !frame_off || !out_ctx || !out_status)) return set_err(h, GD_EINVAL, "null argument");
    if ((out_perm != nullptr) != (out_offsets != nullptr)) return set_err(h, GD_EINVAL, "perm and offsets go together");
    if (n_ctx >= 0xFFFFFFFDu) return set_err(h, GD_EINVAL, "n_ctx too large");
    if (out && (((uintptr_t)out->target_silo | (uintptr_t)out->sending_silo) & 3))
        return set_err(h, GD_EINVAL, "silo outputs must be 4-byte aligned");
    HIP_TRY(h, hipSetDevice(h->device));
    if (n) {
        GD_TRY(h2d(h, h->fr[0], buf, (size_t)buf_len));
        GD_TRY(h2d(h, h->fr[1], frame_off, n));
    }
    gd_frame_fields dev{};
    GD_TRY(frame_scratch(h, n, out, &dev));
    gd_recv_limits dl{};
    const gd_recv_limits* pl = nullptr;
    if (limits && limits->request_count) {
        GD_TRY(h2d(h, h->dirop_buf[0], limits->request_count, n_ctx));
        dl = *limits;
        dl.request_count = (const uint32_t*)h->dirop_buf[0].p;
        pl = &dl;
    }
    GD_TRY(ensure(h, h->fr[13], (size_t)n * 4 + 4));     // ctx
    GD_TRY(ensure(h, h->fr[15], (size_t)n + 8));         // status
    uint32_t* perm = nullptr;
    uint32_t* offs = nullptr;
    if (out_perm) {
        GD_TRY(ensure(h, h->u8_a, (size_t)n * 4 + 4));
        GD_TRY(ensure(h, h->offs, ((size_t)n_ctx + 3) * 4));
        perm = (uint32_t*)h->u8_a.p;
        offs = (uint32_t*)h->offs.p;
    }
    GD_TRY(receive_frames_device(h, (const uint8_t*)h->fr[0].p, buf_len, (const uint64_t*)h->fr[1].p, n, n_ctx, pl, &dev,
                                 (uint32_t*)h->fr[13].p, (uint8_t*)h->fr[15].p, perm, offs));
    GD_TRY(frame_results(h, n, out, &dev));
    if (n) {
        HIP_TRY(h, hipMemcpyAsync(out_ctx, h->fr[13].p, (size_t)n * 4, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(h, hipMemcpyAsync(out_status, h->fr[15].p, (size_t)n, hipMemcpyDeviceToHost, h->stream));
    }
    if (out_perm) {
        if (n) HIP_TRY(h, hipMemcpyAsync(out_perm, perm, (size_t)n * 4, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(h, hipMemcpyAsync(out_offsets, offs, ((size_t)n_ctx + 3) * 4, hipMemcpyDeviceToHost, h->stream));
    }
    return sync_checked(h);
}

}  // extern "C"
