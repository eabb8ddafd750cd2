// eng_exchange.hip -- libgraindispatch: in-library exchange over RCCL (gd_route_multi*, gd_tune_agree) and the multi-rank directory handoff (SURVEY 8 e, f4).
// Shared handle and helpers: gd_engine.h.
#include "gd_engine.h"

// ================================================================== in-library exchange (RCCL)
namespace gdx {


// Launches inside the scope go to the exchange stream (launch() uses h->stream), with the
// exchange stream's own scratch for the helpers both streams run (scan partials, partition):
// the probe + bucketing of the previous batch may be using the handle's at the same time.
struct OnStream {
    gd_handle* h;
    hipStream_t saved;
    DevBuf* scratch;
    OnStream(gd_handle* hh, hipStream_t st, DevBuf* sc) : h(hh), saved(hh->stream), scratch(sc) {
        h->stream = st;
        swap_scratch();
    }
    ~OnStream() {
        swap_scratch();
        h->stream = saved;
    }
    void swap_scratch() {
        std::swap(h->partials, scratch[0]);
        std::swap(h->partials2, scratch[1]);
        std::swap(h->shard_dest, scratch[2]);
        std::swap(h->shard_hist, scratch[3]);
    }
};
struct OnXStream : OnStream {
    explicit OnXStream(gd_handle* hh) : OnStream(hh, hh->xstream, hh->x_scratch) {}
};
struct OnPStream : OnStream {
    explicit OnPStream(gd_handle* hh) : OnStream(hh, hh->pstream, hh->p_scratch) {}
};

void comm_release(gd_handle* h) {
    if (h->pstream) (void)hipStreamSynchronize(h->pstream);
    if (h->xstream) (void)hipStreamSynchronize(h->xstream);
    if (h->comm) (void)h->net->CommDestroy(h->comm);
    h->comm = nullptr;
    h->net = nullptr;
    for (hipEvent_t* e : {&h->x_in, &h->x_hdr[0], &h->x_hdr[1], &h->x_route[0], &h->x_route[1], &h->x_ret[0],
                          &h->x_ret[1], &h->x_done[0], &h->x_done[1], &h->p_packed, &h->x_sent[0], &h->x_sent[1], &h->x_fwd[0], &h->x_fwd[1],
                          &h->x_keys[0], &h->x_keys[1]})
        if (*e) {
            (void)hipEventDestroy(*e);
            *e = nullptr;
        }
    if (h->xstream) (void)hipStreamDestroy(h->xstream);
    h->xstream = nullptr;
    if (h->pstream) (void)hipStreamDestroy(h->pstream);
    h->pstream = nullptr;
    for (auto& par : h->mx_send)
        for (DevBuf& b : par) free_buf(b);
    for (DevBuf& b : h->p_scratch) free_buf(b);
    for (auto& slot : h->mx)
        for (DevBuf& b : slot) free_buf(b);
    for (auto& slot : h->mf)
        for (DevBuf& b : slot) free_buf(b);
    free_buf(h->mx_keys);
    for (DevBuf& b : h->mx_ext) free_buf(b);
    for (DevBuf& b : h->x_scratch) free_buf(b);
    for (auto& hop : h->fm_hop)
        for (DevBuf& b : hop) free_buf(b);
    h->fm_hop.clear();
    h->fm_res.clear();
    for (DevBuf& b : h->fm_scr) free_buf(b);
    for (DevBuf& b : h->fm_graph) free_buf(b);
    for (DevBuf& b : h->ho_send) free_buf(b);
    for (DevBuf& b : h->ho_recv) free_buf(b);
    h->ho_valid = false;
    if (h->h_xcnt) (void)hipHostFree(h->h_xcnt);
    h->h_xcnt = nullptr;
    h->x_done_rec[0] = h->x_done_rec[1] = false;
    h->x_sent_rec[0] = h->x_sent_rec[1] = false;
    h->mres[0] = h->mres[1] = gd_multi_result{};
    h->mcalls = 0;
    h->n_ranks = 0;
    h->rank = -1;
}

// Streams, events and the pinned count buffer of a communicator (any previous one released).
int comm_setup(gd_handle* h) {
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(sync(h));
    comm_release(h);
    HIP_TRY(h, hipHostMalloc((void**)&h->h_xcnt, 20 * 256 * sizeof(uint32_t)));
    HIP_TRY(h, hipStreamCreateWithFlags(&h->xstream, hipStreamNonBlocking));
    HIP_TRY(h, hipStreamCreateWithFlags(&h->pstream, hipStreamNonBlocking));
    for (hipEvent_t* e : {&h->x_in, &h->x_hdr[0], &h->x_hdr[1], &h->x_route[0], &h->x_route[1], &h->x_ret[0],
                          &h->x_ret[1], &h->x_done[0], &h->x_done[1], &h->p_packed, &h->x_sent[0], &h->x_sent[1],
                          &h->x_fwd[0], &h->x_fwd[1], &h->x_keys[0], &h->x_keys[1]})
        HIP_TRY(h, hipEventCreateWithFlags(e, hipEventDisableTiming));
    return GD_OK;
}

int need_comm(gd_handle* h) {
    if (!h->comm) return set_err(h, GD_ESTATE, "no communicator (gd_comm_init)");
    return GD_OK;
}

// Grow a buffer any of the streams may touch: drain them first.
int grow(gd_handle* h, DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes && b.p) return GD_OK;
    HIP_TRY(h, hipStreamSynchronize(h->pstream));
    HIP_TRY(h, hipStreamSynchronize(h->xstream));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    return ensure(h, b, bytes);
}

// One grouped send/recv round on h->stream: for every peer r, send sc[r] elements at soff[r] of
// each lane's send array and receive rc[r] elements at roff[r] of its recv array (both sides skip
// empty chunks, which they agree on: my count to r is r's count from me).  With per-kernel timing
// the round is bracketed by events under `name`.

int exchange_round(gd_handle* h, const char* name, const uint32_t* sc, const uint64_t* soff, const uint32_t* rc,
                   const uint64_t* roff, const Lane* lanes, int n_lanes) {
    const Rccl& R = *h->net;
    hipEvent_t a = nullptr, b = nullptr;
    if (h->timing == 1) {
        a = take_event(h);
        b = take_event(h);
        HIP_TRY(h, hipEventRecord(a, h->stream));
    }
    NCCL_TRY(h, R.GroupStart());
    for (int r = 0; r < h->n_ranks; ++r) {
        for (int l = 0; l < n_lanes; ++l) {
            const Lane& L = lanes[l];
            if (sc[r]) {
                if (L.sb) {                // byte ranges: an empty one is no send (the peer expects none)
                    if (L.sb[r + 1] > L.sb[r])
                        NCCL_TRY(h, R.Send((const uint8_t*)L.send + L.sb[r], (size_t)(L.sb[r + 1] - L.sb[r]),
                                           ncclUint8, r, h->comm, h->stream));
                } else
                    NCCL_TRY(h, R.Send((const uint8_t*)L.send + soff[r] * L.elem, (size_t)sc[r] * L.per, L.type, r,
                                       h->comm, h->stream));
            }
            if (rc[r]) {
                if (L.rb) {
                    const uint64_t nb = L.rsz ? L.rsz[r] : L.rb[r + 1] - L.rb[r];
                    if (nb) NCCL_TRY(h, R.Recv((uint8_t*)L.recv + L.rb[r], (size_t)nb, ncclUint8, r, h->comm, h->stream));
                } else
                    NCCL_TRY(h, R.Recv((uint8_t*)L.recv + roff[r] * L.elem, (size_t)rc[r] * L.per, L.type, r,
                                       h->comm, h->stream));
            }
        }
    }
    NCCL_TRY(h, R.GroupEnd());
    if (h->timing == 1) {
        HIP_TRY(h, hipEventRecord(b, h->stream));
        h->pending.push_back(TimedLaunch{name_id(h, name), a, b});
    }
    return GD_OK;
}

// GD_MULTI_FORWARD: the second hop, owner -> the rank hosting the activation (SURVEY 8 e caveat;
// the send to ActivationAddress.Silo after a remote lookup, LocalGrainDirectory.cs:920,
// OutboundMessageQueue.cs:125).  Directory hits go to silo % W with their route, origin index and
// origin rank; every other status stays here.  All messages of one grain pass through its one
// owner, so each activation's arrival order stays (sender rank, sender batch order).  r holds the
// owner's routes on entry (probe enqueued, x_route[s] recorded) and the forwarded result on exit.
// n1 (optional): the received keys as u32 N1s with one TypeCodeData tcd (a compact header round in
// mode 2): the forward round moves them as such (4 B instead of 24; descriptor in the counts round)
// and the final receiver rebuilds the 24-B keys (k_recv_expand).
int forward_multi(gd_handle* h, int s, uint32_t n_act, gd_multi_result& r, const uint32_t* n1 = nullptr,
                  uint64_t tcd = 0) {
    const int W = h->n_ranks;
    const Rccl& R = *h->net;
    const uint32_t m = r.n_recv;
    DevBuf* F = h->mf[s];
    const size_t m4 = (size_t)m * 4 + 4;
    const size_t want_s[8] = {(size_t)m * sizeof(gd_key) + 8, m4, m4, m4, m4, m4, (size_t)m + 4,
                              ((size_t)W * 6 + 4) * 4};
    for (int b = 0; b < 8; ++b) GD_TRY(grow(h, F[b], want_s[b]));
    uint32_t* fcnt = (uint32_t*)F[7].p;           // send [0,W), recv [W,2W), my descriptor, the peers'
    uint32_t* fdesc = fcnt + 2 * W;
    uint32_t* hc = h->h_xcnt + 10 * 256;
    uint32_t* mydesc = h->h_xcnt + 19 * 256;      // pinned; read by the copy before the sync below
    mydesc[0] = n1 ? 2u : 0u;
    mydesc[1] = 0u;
    mydesc[2] = (uint32_t)tcd;
    mydesc[3] = (uint32_t)(tcd >> 32);
    HIP_TRY(h, hipStreamWaitEvent(h->xstream, h->x_route[s], 0));
    {
        OnXStream on(h);
        HIP_TRY(h, hipMemcpyAsync(fdesc, mydesc, 16, hipMemcpyHostToDevice, h->stream));
        GD_TRY(fwd_pack(h, r.recv_keys, r.status, r.silo, m, (uint32_t)W, (uint32_t)h->rank, F[0].p,
                        (uint32_t*)F[1].p, fcnt, n1));
        if (m)
            GD_TRY(launch(h, "k_fwd_gather", dim3(blocks_for(m, BLOCK)), dim3(BLOCK), 0, k_fwd_gather,
                          (const uint32_t*)F[1].p, m, r.recv_idx, r.recv_src, r.silo, r.act, r.status,
                          (uint32_t*)F[2].p, (uint32_t*)F[3].p, (uint32_t*)F[4].p, (uint32_t*)F[5].p,
                          (uint8_t*)F[6].p));
        NCCL_TRY(h, R.GroupStart());
        for (int q = 0; q < W; ++q) {
            NCCL_TRY(h, R.Send(fcnt + q, 1, ncclUint32, q, h->comm, h->stream));
            NCCL_TRY(h, R.Recv(fcnt + W + q, 1, ncclUint32, q, h->comm, h->stream));
            NCCL_TRY(h, R.Send(fdesc, 4, ncclUint32, q, h->comm, h->stream));
            NCCL_TRY(h, R.Recv(fdesc + 4 + 4 * q, 4, ncclUint32, q, h->comm, h->stream));
        }
        NCCL_TRY(h, R.GroupEnd());
        HIP_TRY(h, hipMemcpyAsync(hc, fcnt, ((size_t)W * 6 + 4) * 4, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(h, hipStreamSynchronize(h->stream));
    }
    std::vector<uint32_t> sc(hc, hc + W), rc(hc + W, hc + 2 * W);
    std::vector<uint64_t> soff(W + 1, 0), roff(W + 1, 0);
    for (int q = 0; q < W; ++q) {
        soff[q + 1] = soff[q] + sc[q];
        roff[q + 1] = roff[q] + rc[q];
    }
    if (soff[W] != m)
        return set_err(h, GD_ERCCL, "forward counts sum to %llu, %u messages here", (unsigned long long)soff[W], m);
    if (roff[W] >= 0xFFFFFFFFull)
        return set_err(h, GD_EINVAL, "%llu forwarded messages: more than a batch can hold", (unsigned long long)roff[W]);
    const uint32_t m2 = (uint32_t)roff[W];
    // key bytes per peer: 4 (u32 N1s) or 24 by each side's descriptor; with any compact peer the
    // keys land in staging and k_recv_expand rebuilds them
    const uint32_t* hdsc = hc + 2 * W;             // mine, then the peers'
    std::vector<uint64_t> ksb(W + 1, 0), krb(W + 1, 0);
    bool any_c = false;
    for (int q = 0; q < W; ++q) {
        const uint32_t c = hdsc[4 + 4 * q];
        any_c |= c && rc[q];
        ksb[q + 1] = ksb[q] + (uint64_t)sc[q] * header_bytes(hdsc[0]);
        krb[q + 1] = krb[q] + (uint64_t)rc[q] * header_bytes(c);
    }
    const size_t q4 = (size_t)m2 * 4 + 4;
    const size_t want_r[9] = {(size_t)m2 * sizeof(gd_key) + 8, q4, q4, q4, q4, (size_t)m2 + 4, q4,
                              ((size_t)n_act + 2) * 4, any_c ? (size_t)krb[W] + 16 : 0};
    for (int b = 0; b < 9; ++b)
        if (want_r[b]) GD_TRY(grow(h, F[8 + b], want_r[b]));
    {
        OnXStream on(h);
        const Lane lanes[6] = {{F[0].p, any_c ? F[16].p : F[8].p, 1, ncclUint8, 1, ksb.data(), krb.data()},
                               {F[2].p, F[9].p, 4, ncclUint32, 1},
                               {F[3].p, F[10].p, 4, ncclUint32, 1},
                               {F[4].p, F[11].p, 4, ncclUint32, 1},
                               {F[5].p, F[12].p, 4, ncclUint32, 1},
                               {F[6].p, F[13].p, 1, ncclUint8, 1}};
        GD_TRY(exchange_round(h, "rccl_forward", sc.data(), soff.data(), rc.data(), roff.data(), lanes, 6));
        if (any_c && m2)
            GD_TRY(launch(h, "k_recv_expand", dim3(blocks_for(m2, BLOCK)), dim3(BLOCK), 0, k_recv_expand,
                          (const uint8_t*)F[16].p, (const uint32_t*)(fcnt + W), (const uint32_t*)(fdesc + 4),
                          (uint32_t)W, m2, (gd_key*)F[8].p, (uint32_t*)nullptr));
        HIP_TRY(h, hipEventRecord(h->x_fwd[s], h->xstream));
    }
    HIP_TRY(h, hipStreamWaitEvent(h->stream, h->x_fwd[s], 0));
    GD_TRY(bucket_device(h, (const uint32_t*)F[12].p, m2, n_act, (uint32_t*)F[14].p, (uint32_t*)F[15].p));
    r.n_recv = m2;
    r.recv_keys = (const gd_key*)F[8].p;
    r.recv_idx = (const uint32_t*)F[9].p;
    r.recv_src = (const uint32_t*)F[10].p;
    r.silo = (const uint32_t*)F[11].p;
    r.act = (const uint32_t*)F[12].p;
    r.status = (const uint8_t*)F[13].p;
    r.perm = (const uint32_t*)F[14].p;
    r.offsets = (const uint32_t*)F[15].p;
    return GD_OK;
}

// Sender batch d_keys[n] -> owner ranks (exchange) -> probe + bucket there (-> routes back).
//   xstream: [wait caller] partition, counts round, (host: sizes) header round, recv_src
//   stream:  [wait headers] probe, bucket
//   xstream: [wait probe] routes round, unpartition            (GD_MULTI_RETURN_ROUTES)
// Only the counts round blocks the host, and only on xstream, so batch i+1's partition and
// exchange run while batch i is probed and bucketed.
int route_multi(gd_handle* h, const gd_key* d_keys, uint32_t n, uint32_t n_act, int flags, gd_multi_result* out,
                const gd_key_ext* ext = nullptr) {
    GD_TRY(need_comm(h));
    GD_TRY(check_ring(h));
    if (n_act == 0xFFFFFFFFu) return set_err(h, GD_EINVAL, "n_act too large");
    const int W = h->n_ranks;
    const Rccl& R = *h->net;
    const int s = (int)(h->mcalls & 1);
    DevBuf* B = h->mx[s];
    const bool ret = (flags & GD_MULTI_RETURN_ROUTES) != 0;
    const bool fwd = (flags & GD_MULTI_FORWARD) != 0;
    const bool keep_keys = fwd || !(flags & GD_MULTI_NO_KEYS);   // the forward hop moves the keys on
    const bool has_ext = ext && n && !h->cache_max;      // KeyExt strings travel with their messages
    const ExtArgs x = has_ext ? ExtArgs{ext->bytes, ext->offset, ext->length, ext->bytes_len} : ExtArgs{};
    DevBuf* SB = h->mx_send[s];
    // 1. stable partition by owner rank (gd_shard.h) on the partition stream, into this parity's send
    //    buffers once batch i-2's rounds have read them; it runs beside batch i-1's header round
    GD_TRY(grow(h, SB[0], (size_t)n * sizeof(gd_key) + 8));
    GD_TRY(grow(h, SB[1], (size_t)n * 4 + 4));
    GD_TRY(grow(h, SB[2], ((size_t)W * 9 + 6) * 4));
    if (has_ext) {
        GD_TRY(grow(h, SB[3], (size_t)n * 4 + 4));
        GD_TRY(grow(h, SB[4], (size_t)n * 4 + 4));
    }
    // the partition waits for the handle's stream when the caller's keys are not known complete, and while
    // the previous batch's probe or bucketing was a timed launch of the measured choices (tune_choose): a
    // variant timed beside the next batch's partition measured slower than it is (the N1 probe's 8-B index
    // lost to the 16-B index's group reads there), so the first launches run unoverlapped
    if (!(flags & GD_MULTI_KEYS_READY) || h->measured_launch) {
        HIP_TRY(h, hipEventRecord(h->x_in, h->stream));
        HIP_TRY(h, hipStreamWaitEvent(h->pstream, h->x_in, 0));
    }
    h->measured_launch = false;
    if (h->x_sent_rec[s]) HIP_TRY(h, hipStreamWaitEvent(h->pstream, h->x_sent[s], 0));
    gd_key* send_keys = (gd_key*)SB[0].p;
    uint32_t* send_idx = (uint32_t*)SB[1].p;
    // send msgs [0,W), recv msgs [W,2W), send bytes, recv bytes, my key descriptor [4W,4W+4) (k_key_desc),
    // the peers' descriptors [4W+4, 8W+4), my 2-B index block count [8W+4], the peers' [8W+5, 9W+5)
    uint32_t* dcnt = (uint32_t*)SB[2].p;
    uint32_t* kdesc = dcnt + 4 * W;
    int32_t* send_len = (int32_t*)SB[3].p;
    uint32_t* send_boff = (uint32_t*)SB[4].p;
    uint32_t regions = 1;
    // region order needs the descriptor: its flag tells the owners (k_shard_counts)
    regions = h->region_probe && h->compact_headers && !h->cache_max && W * N_REGIONS <= 256 ? N_REGIONS : 1u;
    // 2-B origin indices (KD_IDX16): the senders' own 4-B copy is needed for returned routes and
    // KeyExt lengths; region order breaks the increasing order within a rank's chunk
    // (W > 1 only: at world 1 nothing crosses a link and the rebuild costs more HBM than it saves)
    const bool idx16 = h->idx16 && W > 1 && !ret && !has_ext && regions == 1 && n > 0;
    const uint32_t nblk = idx16 ? (uint32_t)(((uint64_t)n + 65535u) >> 16) : 0u;
    if (idx16) GD_TRY(grow(h, SB[6], (size_t)W * nblk * 4 + 16));
    uint32_t* nb_mine = dcnt + 8 * W + 4;
    {
        OnPStream on(h);
        h->pack_pay16 = idx16;
        const int prc = shard_pack<false>(h, d_keys, nullptr, n, 0, (uint32_t)W, send_keys, send_idx, dcnt, x,
                                          h->compact_headers ? kdesc : nullptr, regions);
        h->pack_pay16 = false;
        GD_TRY(prc);
        if (!h->compact_headers) HIP_TRY(h, hipMemsetAsync(kdesc, 0, 16, h->stream));
        if (idx16)                     // block starts per rank from the partition's scan; descriptor flag
            GD_TRY(launch(h, "k_block_prefix", dim3(blocks_for((uint64_t)W * nblk, BLOCK)), dim3(BLOCK), 0,
                          k_block_prefix, (const uint32_t*)h->shard_hist.p, blocks_for(n, SH_TILE), (uint32_t)W, nblk,
                          (uint32_t*)SB[6].p, kdesc, nb_mine));
        else
            HIP_TRY(h, hipMemsetAsync(nb_mine, 0, 4, h->stream));
        if (has_ext) {                 // KeyExt bytes per destination; lengths and byte offsets in send order
            HIP_TRY(h, hipMemsetAsync(dcnt + 2 * W, 0, (size_t)W * 4, h->stream));
            GD_TRY(launch(h, "k_dest_bytes", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), 0, k_dest_bytes,
                          (const uint8_t*)h->shard_dest.p, n, x, (uint32_t)W, dcnt + 2 * W, regions));
            GD_TRY(launch(h, "k_send_lengths", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), 0, k_send_lengths,
                          (const uint32_t*)send_idx, n, x, send_len, send_boff));
            GD_TRY(scan_device<OpAdd>(h, send_boff, n, false, false, "ext_offsets"));
        }
        HIP_TRY(h, hipEventRecord(h->p_packed, h->pstream));
    }
    // 2. counts round on the exchange stream (after batch i-1's rounds), then the host sizes
    HIP_TRY(h, hipStreamWaitEvent(h->xstream, h->p_packed, 0));
    {
        OnXStream on(h);
        NCCL_TRY(h, R.GroupStart());
        for (int r = 0; r < W; ++r) {
            NCCL_TRY(h, R.Send(dcnt + r, 1, ncclUint32, r, h->comm, h->stream));
            NCCL_TRY(h, R.Recv(dcnt + W + r, 1, ncclUint32, r, h->comm, h->stream));
            NCCL_TRY(h, R.Send(kdesc, 4, ncclUint32, r, h->comm, h->stream));
            NCCL_TRY(h, R.Recv(kdesc + 4 + 4 * r, 4, ncclUint32, r, h->comm, h->stream));
            NCCL_TRY(h, R.Send(nb_mine, 1, ncclUint32, r, h->comm, h->stream));
            NCCL_TRY(h, R.Recv(nb_mine + 1 + r, 1, ncclUint32, r, h->comm, h->stream));
            if (has_ext) {
                NCCL_TRY(h, R.Send(dcnt + 2 * W + r, 1, ncclUint32, r, h->comm, h->stream));
                NCCL_TRY(h, R.Recv(dcnt + 3 * W + r, 1, ncclUint32, r, h->comm, h->stream));
            }
        }
        NCCL_TRY(h, R.GroupEnd());
        HIP_TRY(h, hipMemcpyAsync(h->h_xcnt, dcnt, ((size_t)W * 9 + 6) * 4, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(h, hipStreamSynchronize(h->stream));
    }
    ncclResult_t async_err = ncclSuccess;
    NCCL_TRY(h, R.CommGetAsyncError(h->comm, &async_err));
    if (async_err != ncclSuccess) return set_err(h, GD_ERCCL, "RCCL async error: %s", R.GetErrorString(async_err));
    std::vector<uint32_t> sc(h->h_xcnt, h->h_xcnt + W), rc(h->h_xcnt + W, h->h_xcnt + 2 * W);
    std::vector<uint32_t> sbc(W, 0), rbc(W, 0);
    if (has_ext) {
        sbc.assign(h->h_xcnt + 2 * W, h->h_xcnt + 3 * W);
        rbc.assign(h->h_xcnt + 3 * W, h->h_xcnt + 4 * W);
    }
    std::vector<uint64_t> soff(W + 1, 0), roff(W + 1, 0), sboff(W + 1, 0), rboff(W + 1, 0);
    for (int r = 0; r < W; ++r) {
        soff[r + 1] = soff[r] + sc[r];
        roff[r + 1] = roff[r] + rc[r];
        sboff[r + 1] = sboff[r] + sbc[r];
        rboff[r + 1] = rboff[r] + rbc[r];
    }
    if (soff[W] != n)
        return set_err(h, GD_ERCCL, "partition counts sum to %llu, batch is %u", (unsigned long long)soff[W], n);
    if (roff[W] >= 0xFFFFFFFFull || rboff[W] >= 0xFFFFFFFFull || sboff[W] >= 0xFFFFFFFFull)
        return set_err(h, GD_EINVAL, "%llu messages / %llu KeyExt bytes received: more than a batch can hold",
                       (unsigned long long)roff[W], (unsigned long long)rboff[W]);
    const uint32_t m = (uint32_t)roff[W];
    // header bytes per peer: 8 or 4 (N1 only) when that side's batch is compact (k_key_desc), else 24
    const uint32_t* hd = h->h_xcnt + 4 * W;        // my descriptor, then the peers'
    const uint64_t my_esz = header_bytes(hd[0]);
    std::vector<uint64_t> hsb(W + 1, 0), hrb(W + 1, 0);
    bool any_compact = false;
    // every received chunk compact with one TypeCodeData: the probe reads the N1s as they arrive
    // (8 B a key instead of a 24-B rebuilt key); not with KeyExt strings or in cache mode
    bool n1_path = !has_ext && !h->cache_max && m > 0;
    uint64_t n1_tcd = 0;
    uint32_t n1_mode = 0;                          // every received chunk in one compact mode (u64 / u32)
    bool n1_first = true;
    // every non-empty chunk ordered by region (descriptor flag 4): the region-mapped probe
    bool by_region = !h->cache_max && m > 0;
    for (int r = 0; r < W; ++r) {
        const uint32_t c = hd[4 + 4 * r];
        if (rc[r] && !(hd[4 + 4 * r + 1] & KD_REGIONS)) by_region = false;
        any_compact |= c && rc[r];
        hsb[r + 1] = hsb[r] + sc[r] * my_esz;
        hrb[r + 1] = hrb[r] + rc[r] * header_bytes(c);
        if (rc[r]) {
            const uint64_t t = (uint64_t)hd[4 + 4 * r + 2] | ((uint64_t)hd[4 + 4 * r + 3] << 32);
            if (!c || (!n1_first && (t != n1_tcd || c != n1_mode))) n1_path = false;
            n1_tcd = t;
            n1_mode = c;
            n1_first = false;
        }
    }
    // origin indices: 2 B a message from KD_IDX16 senders (+ their block starts), else 4 B.  With any
    // 2-B peer every chunk lands in a staging buffer at 4-B aligned offsets and k_recv_idx16 rebuilds
    // them; otherwise the 4-B chunks land in recv_idx directly.
    bool any16 = false;
    std::vector<uint64_t> isb(W + 1, 0), irb(W + 1, 0), irs(W, 0), psb(W + 1, 0), prb(W + 1, 0), prs(W, 0);
    const uint32_t* rnb = h->h_xcnt + 8 * W + 5;
    for (int r = 0; r < W; ++r) {
        const bool w16 = rc[r] && (hd[4 + 4 * r + 1] & KD_IDX16);
        any16 |= w16;
        isb[r + 1] = isb[r] + (uint64_t)sc[r] * (idx16 ? 2 : 4);
        irs[r] = (uint64_t)rc[r] * (w16 ? 2 : 4);
        irb[r + 1] = irb[r] + ((irs[r] + 3) & ~3ull);
        psb[r + 1] = psb[r] + (idx16 && sc[r] ? (uint64_t)nblk * 4 : 0);
        prs[r] = w16 ? (uint64_t)rnb[r] * 4 : 0;
        prb[r + 1] = prb[r] + prs[r];
    }
    // the probe of compact N1s writes the sender ranks itself (no k_recv_src pass over the batch)
    const bool src_in_probe = n1_path && !any16 && !by_region;
    // 2. this parity's buffers: batch i-2 must be done with them (probe/bucket and routes round)
    const size_t m4 = (size_t)m * 4 + 4, n4 = (size_t)n * 4 + 4;
    const size_t want[22] = {(size_t)m * sizeof(gd_key) + 8, m4, m4, m4, m4, (size_t)m + 4, m4,
                             ((size_t)n_act + 2) * 4, n4, n4, (size_t)n + 4, n4, n4, (size_t)n + 4,
                             m4, (size_t)rboff[W] + 16, m4, (size_t)m * 8 + 8, (size_t)hrb[W] + 16,
                             (size_t)W * (N_REGIONS + 1) * 4, (size_t)irb[W] + 16, (size_t)prb[W] + 16};
    for (int b = 0; b < 22; ++b)
        if (want[b] && (b < 8 || (ret && b < 14) || (has_ext && b >= 14 && b < 18) || (any_compact && b == 18) ||
                        (by_region && b == 19) || (any16 && b >= 20)))
            GD_TRY(grow(h, B[b], want[b]));
    if (has_ext) GD_TRY(grow(h, SB[5], (size_t)sboff[W] + 16));
    // World 1 (the self-chunk skip): the one chunk is this rank's own, so the probe reads the send
    // buffers in place -- no header round, no copy of the headers and origin indices -- and those
    // buffers stay busy until this batch's probe and bucketing are done (x_sent below)
    const bool alias = W == 1 && !has_ext && !any16 && !by_region && !ret && !fwd;
    gd_key* recv_keys = alias && !any_compact ? send_keys : (gd_key*)B[0].p;
    uint32_t* recv_idx = alias ? send_idx : (uint32_t*)B[1].p;
    void* hdr = alias ? (void*)send_keys : (any_compact ? B[18].p : (void*)recv_keys);   // headers as received
    uint32_t* recv_src = (uint32_t*)B[2].p;
    uint32_t* silo = (uint32_t*)B[3].p;
    uint32_t* act = (uint32_t*)B[4].p;
    uint8_t* st = (uint8_t*)B[5].p;
    uint32_t* perm = (uint32_t*)B[6].p;
    uint32_t* offs = (uint32_t*)B[7].p;
    if (h->x_done_rec[s]) HIP_TRY(h, hipStreamWaitEvent(h->xstream, h->x_done[s], 0));
    {
        OnXStream on(h);
        if (has_ext)
            GD_TRY(launch(h, "k_gather_ext", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), 0, k_gather_ext,
                          (const uint32_t*)send_idx, n, x, (const uint32_t*)send_boff, (uint8_t*)SB[5].p));
        // keys: byte ranges per peer (compact chunks are 8 B a header); with any compact peer they
        // land in a staging buffer that k_recv_expand turns back into 24-B keys
        // keys, origin indices, KeyExt lengths, the block starts of 2-B origin indices
        Lane lanes[4];
        int nl = 0;
        lanes[nl++] = {send_keys, hdr, 1, ncclUint8, 1, hsb.data(), hrb.data()};
        lanes[nl++] = {send_idx, any16 ? B[20].p : (void*)recv_idx, 4, ncclUint32, 1, idx16 ? isb.data() : nullptr,
                       any16 ? irb.data() : nullptr, any16 ? irs.data() : nullptr};
        if (has_ext) lanes[nl++] = {send_len, B[14].p, 4, ncclInt32, 1};
        if (idx16 || any16) lanes[nl++] = {SB[6].p, B[21].p, 4, ncclUint32, 1, psb.data(), prb.data(), prs.data()};
        if (!alias) GD_TRY(exchange_round(h, "rccl_headers", sc.data(), soff.data(), rc.data(), roff.data(), lanes, nl));
        if (has_ext) {                 // the KeyExt strings, then their offsets in the receive blob
            const Lane bl[1] = {{SB[5].p, B[15].p, 1, ncclUint8, 1}};
            GD_TRY(exchange_round(h, "rccl_keyext", sbc.data(), sboff.data(), rbc.data(), rboff.data(), bl, 1));
            GD_TRY(launch(h, "k_len_bytes", dim3(blocks_for(m, BLOCK)), dim3(BLOCK), 0, k_len_bytes,
                          (const int32_t*)B[14].p, m, (uint32_t*)B[16].p));
            GD_TRY(scan_device<OpAdd>(h, (uint32_t*)B[16].p, m, false, false, "ext_offsets"));
            GD_TRY(launch(h, "k_u32_to_u64", dim3(blocks_for(m, BLOCK)), dim3(BLOCK), 0, k_u32_to_u64,
                          (const uint32_t*)B[16].p, m, (uint64_t*)B[17].p));
        }
        if (any_compact && !n1_path)
            GD_TRY(launch(h, "k_recv_expand", dim3(blocks_for(m, BLOCK)), dim3(BLOCK), 0, k_recv_expand,
                          (const uint8_t*)hdr, (const uint32_t*)(dcnt + W), (const uint32_t*)(kdesc + 4),
                          (uint32_t)W, m, recv_keys, recv_src));
        else if (!any16 && !src_in_probe)
            GD_TRY(launch(h, "k_recv_src", dim3(blocks_for(m, BLOCK)), dim3(BLOCK), 0, k_recv_src,
                          (const uint32_t*)(dcnt + W), (uint32_t)W, m, recv_src));
        if (any16)                     // 4-B origin indices and sender ranks from the 2-B form
            GD_TRY(launch(h, "k_recv_idx16", dim3(blocks_for(m, BLOCK)), dim3(BLOCK), 0, k_recv_idx16,
                          (const uint8_t*)B[20].p, (const uint32_t*)(dcnt + W), (const uint32_t*)(kdesc + 4),
                          (const uint32_t*)B[21].p, (const uint32_t*)(nb_mine + 1), (uint32_t)W, m, recv_idx,
                          recv_src));
        if (by_region) {               // where each sender's region runs start (binary search per chunk)
            const uint32_t nt = (uint32_t)W * (N_REGIONS + 1);
            const uint32_t* rcnt = dcnt + W;
            uint32_t* seg = (uint32_t*)B[19].p;
            const uint32_t w1 = n1_path ? header_bytes(n1_mode) : 0u;
            if (w1 == 4)
                GD_TRY(launch(h, "k_region_segments", dim3(blocks_for(nt, 64)), dim3(64), 0, k_region_segments<4>,
                              (const void*)B[18].p, rcnt, (uint32_t)W, n1_tcd, seg));
            else if (w1 == 8)
                GD_TRY(launch(h, "k_region_segments", dim3(blocks_for(nt, 64)), dim3(64), 0, k_region_segments<8>,
                              (const void*)B[18].p, rcnt, (uint32_t)W, n1_tcd, seg));
            else
                GD_TRY(launch(h, "k_region_segments", dim3(blocks_for(nt, 64)), dim3(64), 0, k_region_segments<0>,
                              (const void*)recv_keys, rcnt, (uint32_t)W, 0ull, seg));
        }
        HIP_TRY(h, hipEventRecord(h->x_hdr[s], h->xstream));
        if (n1_path && keep_keys) {    // the 24-B keys for the result, beside the probe
            GD_TRY(launch(h, "k_recv_expand", dim3(blocks_for(m, BLOCK)), dim3(BLOCK), 0, k_recv_expand,
                          (const uint8_t*)hdr, (const uint32_t*)(dcnt + W), (const uint32_t*)(kdesc + 4),
                          (uint32_t)W, m, recv_keys, src_in_probe ? nullptr : recv_src));
            HIP_TRY(h, hipEventRecord(h->x_keys[s], h->xstream));
        }
        if (!ret && !alias) {          // this parity's send buffers are free for batch i+2's partition
            HIP_TRY(h, hipEventRecord(h->x_sent[s], h->xstream));
            h->x_sent_rec[s] = true;
        }
    }
    // 3. probe + bucket on the owner (the handle's stream)
    HIP_TRY(h, hipStreamWaitEvent(h->stream, h->x_hdr[s], 0));
    if (by_region)
        GD_TRY(route_region_device(h, n1_path ? B[18].p : (const void*)recv_keys, n1_path ? header_bytes(n1_mode) : 0u,
                                   n1_tcd, m, (const uint32_t*)B[19].p, (uint32_t)W, silo, act, st));
    else if (n1_path)
        GD_TRY(route_n1_device(h, hdr, header_bytes(n1_mode), n1_tcd, m, silo, act, st,
                               src_in_probe ? (const uint32_t*)(dcnt + W) : nullptr, (uint32_t)W,
                               src_in_probe ? recv_src : nullptr));
    else if (m) GD_TRY(route_device(h, recv_keys, m, silo, act, st, !has_ext));
    if (m && has_ext)                  // the received strings: KeyExt grains are routed on their owner
        GD_TRY(keyext_pass(h, recv_keys,
                           ExtArgs{(const uint8_t*)B[15].p, (const uint64_t*)B[17].p, (const int32_t*)B[14].p,
                                   rboff[W]},
                           m, silo, act, st));
    HIP_TRY(h, hipEventRecord(h->x_route[s], h->stream));
    if (!fwd) GD_TRY(bucket_device(h, act, m, n_act, perm, offs));
    // 4. routes back to the senders, into their batch order (Dispatcher.AddressMessage)
    gd_multi_result r{};
    if (ret) {
        HIP_TRY(h, hipStreamWaitEvent(h->xstream, h->x_route[s], 0));
        {
            OnXStream on(h);
            const Lane lanes[3] = {{silo, B[8].p, 4, ncclUint32, 1},
                                   {act, B[9].p, 4, ncclUint32, 1},
                                   {st, B[10].p, 1, ncclUint8, 1}};
            GD_TRY(exchange_round(h, "rccl_routes", rc.data(), roff.data(), sc.data(), soff.data(), lanes, 3));
            GD_TRY(launch(h, "k_unpartition", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), 0, k_unpartition,
                          (const uint32_t*)send_idx, n, (const uint32_t*)B[8].p, (const uint32_t*)B[9].p,
                          (const uint8_t*)B[10].p, (uint32_t*)B[11].p, (uint32_t*)B[12].p, (uint8_t*)B[13].p));
            HIP_TRY(h, hipEventRecord(h->x_ret[s], h->xstream));
            HIP_TRY(h, hipEventRecord(h->x_sent[s], h->xstream));   // send_idx read: buffers free
            h->x_sent_rec[s] = true;
        }
        HIP_TRY(h, hipStreamWaitEvent(h->stream, h->x_ret[s], 0));   // the caller syncs one stream
        r.ret_silo = (const uint32_t*)B[11].p;
        r.ret_act = (const uint32_t*)B[12].p;
        r.ret_status = (const uint8_t*)B[13].p;
    }
    if (n1_path && keep_keys) HIP_TRY(h, hipStreamWaitEvent(h->stream, h->x_keys[s], 0));
    r.n_recv = m;
    r.n_act = n_act;
    r.recv_keys = keep_keys ? recv_keys : nullptr;
    r.recv_idx = recv_idx;
    r.recv_src = recv_src;
    r.silo = silo;
    r.act = act;
    r.status = st;
    r.perm = perm;
    r.offsets = offs;
    // compact forward keys: every received header a u32 N1 of one type (the probe's N1 path)
    if (fwd)
        GD_TRY(forward_multi(h, s, n_act, r, n1_path && n1_mode == 2 ? (const uint32_t*)B[18].p : nullptr, n1_tcd));
    HIP_TRY(h, hipEventRecord(h->x_done[s], h->stream));
    h->x_done_rec[s] = true;
    if (alias) {                       // the probe read the send buffers: free once it is done
        HIP_TRY(h, hipEventRecord(h->x_sent[s], h->stream));
        h->x_sent_rec[s] = true;
    }
    h->mres[s] = r;
    h->mres_n[s] = n;
    h->mcalls += 1;
    h->routed += m;
    if (out) *out = r;
    return GD_OK;
}

}  // namespace gdx

int gd_comm_unique_id(uint8_t out_id[GD_COMM_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == GD_COMM_ID_BYTES, "ncclUniqueId size");
    if (!out_id) return set_err(nullptr, GD_EINVAL, "null argument");
    const Rccl& R = rccl();
    if (!R.ok) return set_err(nullptr, GD_ERCCL, "%s", R.why);
    ncclUniqueId id;
    const ncclResult_t e = R.GetUniqueId(&id);
    if (e != ncclSuccess) return set_err(nullptr, GD_ERCCL, "ncclGetUniqueId: %s", R.GetErrorString(e));
    std::memcpy(out_id, &id, GD_COMM_ID_BYTES);
    return GD_OK;
}

int gd_comm_init(gd_handle* h, const uint8_t id[GD_COMM_ID_BYTES], int n_ranks, int rank) {
    if (!h || !id) return set_err(h, GD_EINVAL, "null argument");
    if (n_ranks < 1 || n_ranks > 256 || rank < 0 || rank >= n_ranks)
        return set_err(h, GD_EINVAL, "rank %d of %d: need 0 <= rank < n_ranks <= 256", rank, n_ranks);
    const Rccl& R = rccl();
    if (!R.ok) return set_err(h, GD_ERCCL, "%s", R.why);
    GD_TRY(comm_setup(h));
    ncclUniqueId uid;
    std::memcpy(&uid, id, GD_COMM_ID_BYTES);
    const ncclResult_t e = R.CommInitRank(&h->comm, n_ranks, uid, rank);
    if (e != ncclSuccess) {
        h->comm = nullptr;
        comm_release(h);
        return set_err(h, GD_ERCCL, "ncclCommInitRank(%d of %d): %s", rank, n_ranks, R.GetErrorString(e));
    }
    h->net = &R;
    h->n_ranks = n_ranks;
    h->rank = rank;
    return GD_OK;
}

int gd_comm_init_local(gd_handle* const* hs, int n_ranks) {
    if (!hs || n_ranks < 1 || n_ranks > 256) return set_err(nullptr, GD_EINVAL, "need 1 <= n_ranks <= 256 handles");
    for (int r = 0; r < n_ranks; ++r) {
        if (!hs[r]) return set_err(nullptr, GD_EINVAL, "null handle %d", r);
        for (int q = 0; q < r; ++q)
            if (hs[q] == hs[r]) return set_err(nullptr, GD_EINVAL, "handle %d given twice", r);
    }
    for (int r = 0; r < n_ranks; ++r) {
        HIP_TRY(hs[r], hipSetDevice(hs[r]->device));
        GD_TRY(comm_setup(hs[r]));
    }
    const std::vector<ncclComm_t> comms = local_comms(n_ranks);
    for (int r = 0; r < n_ranks; ++r) {
        hs[r]->comm = comms[r];
        hs[r]->net = &local_net();
        hs[r]->n_ranks = n_ranks;
        hs[r]->rank = r;
    }
    return GD_OK;
}

int gd_comm_destroy(gd_handle* h) {
    if (!h) return set_err(h, GD_EINVAL, "null argument");
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(sync(h));
    comm_release(h);
    return GD_OK;
}

int gd_comm_info(gd_handle* h, int* n_ranks, int* rank, int* transport) {
    if (!h || !n_ranks || !rank || !transport) return set_err(h, GD_EINVAL, "null argument");
    *n_ranks = 0;
    *rank = -1;
    *transport = GD_COMM_NONE;
    if (!h->comm) return GD_OK;
    const Rccl& R = rccl();
    if (h->net == &R) {
        *transport = GD_COMM_RCCL;
        int c = h->n_ranks, u = h->rank;
        if (R.CommCount) NCCL_TRY(h, R.CommCount(h->comm, &c));       // the count RCCL itself reports
        if (R.CommUserRank) NCCL_TRY(h, R.CommUserRank(h->comm, &u));
        *n_ranks = c;
        *rank = u;
        return GD_OK;
    }
    *transport = GD_COMM_LOCAL;
    *n_ranks = h->n_ranks;
    *rank = h->rank;
    return GD_OK;
}

// One all-gather of every rank's finished tune entries (key, best time a message per variant) in a
// grouped send/recv round, then the same reduction on every rank: per key, the summed times of the
// ranks that finished it (in rank order, so the floats agree bit for bit), argmin -> the pick.
int gd_tune_agree(gd_handle* h) {
    if (!h) return set_err(h, GD_EINVAL, "null argument");
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(need_comm(h));
    struct Rec {
        uint32_t key;
        float best[gd_handle::CXV];
    };
    static_assert(sizeof(Rec) == 4 + 4 * gd_handle::CXV, "packed records");
    constexpr uint32_t MAXE = 1023;                      // entries a rank contributes (+ a count record)
    const int W = h->n_ranks;
    std::vector<Rec> mine(MAXE + 1, Rec{0, {}});
    uint32_t ne = 0;
    for (auto& kt : h->cx_tune) {
        auto& t = kt.second;
        const int nvar = t.nvar ? t.nvar : tune_nvar(kt.first / (64 * 32));
        tune_resolve(t, nvar);
        bool done = true;
        for (int v = 0; v < nvar; ++v) done = done && t.best[v] < 1e29f;
        if (!done || ne == MAXE) continue;
        Rec& r = mine[1 + ne++];
        r.key = (uint32_t)kt.first;
        // a variant this rank does not have (the 8-B index not built here) can never win the sum
        for (int v = 0; v < gd_handle::CXV; ++v) r.best[v] = v < nvar ? t.best[v] : 1e30f;
    }
    mine[0].key = ne;
    const size_t bytes = (size_t)(MAXE + 1) * sizeof(Rec);
    DevBuf& buf = h->tune_buf;
    GD_TRY(sync(h));
    GD_TRY(ensure(h, buf, bytes * (W + 1)));
    uint8_t* d = (uint8_t*)buf.p;
    HIP_TRY(h, hipMemcpyAsync(d, mine.data(), bytes, hipMemcpyHostToDevice, h->stream));
    const Rccl& R = *h->net;
    NCCL_TRY(h, R.GroupStart());
    for (int r = 0; r < W; ++r) {
        NCCL_TRY(h, R.Send(d, bytes, ncclUint8, r, h->comm, h->stream));
        NCCL_TRY(h, R.Recv(d + bytes * (r + 1), bytes, ncclUint8, r, h->comm, h->stream));
    }
    NCCL_TRY(h, R.GroupEnd());
    std::vector<Rec> all((size_t)(MAXE + 1) * W);
    HIP_TRY(h, hipMemcpyAsync(all.data(), d + bytes, bytes * W, hipMemcpyDeviceToHost, h->stream));
    GD_TRY(sync(h));
    std::map<uint32_t, std::array<double, gd_handle::CXV>> sum;
    for (int r = 0; r < W; ++r) {
        const Rec* rr = all.data() + (size_t)(MAXE + 1) * r;
        const uint32_t cnt = std::min(rr[0].key, MAXE);
        for (uint32_t i = 0; i < cnt; ++i) {
            auto& s = sum.try_emplace(rr[1 + i].key, std::array<double, gd_handle::CXV>{}).first->second;
            for (int v = 0; v < gd_handle::CXV; ++v) s[v] += (double)rr[1 + i].best[v];
        }
    }
    for (const auto& ks : sum) {
        const int kind = (int)ks.first / (64 * 32), nvar = tune_nvar(kind);   // unavailable ones sum past 1e30
        int pick = 0;
        for (int v = 1; v < nvar; ++v)
            if (ks.second[v] < ks.second[pick]) pick = v;
        // only a variant this handle can launch: the entry's own variant count where it measured it,
        // else the count its launches have now (the 8-B index built or not); a later launch with
        // fewer variants measures again (tune_choose).  Results agree whatever each rank runs.
        auto it = h->cx_tune.find((int)ks.first);
        const int local = it != h->cx_tune.end() && it->second.nvar ? it->second.nvar : tune_nvar_now(h, kind);
        if (pick >= local) continue;
        auto& t = h->cx_tune[(int)ks.first];
        t.pick = pick;
        t.nvar = local;
        t.round = std::max(t.round, 2 * local);
    }
    return GD_OK;
}

int gd_route_multi_device(gd_handle* h, const gd_key* d_keys, uint32_t n, uint32_t n_act, int flags,
                          gd_multi_result* out) {
    if (!h || (n && !d_keys)) return set_err(h, GD_EINVAL, "null argument");
    if (flags & ~(GD_MULTI_RETURN_ROUTES | GD_MULTI_KEYS_READY | GD_MULTI_FORWARD | GD_MULTI_NO_KEYS)) return set_err(h, GD_EINVAL, "unknown flags 0x%x", flags);
    HIP_TRY(h, hipSetDevice(h->device));
    return route_multi(h, d_keys, n, n_act, flags, out);
}

int gd_route_multi(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t n_act, int flags, gd_multi_result* out) {
    if (!h || (n && !keys)) return set_err(h, GD_EINVAL, "null argument");
    if (flags & ~(GD_MULTI_RETURN_ROUTES | GD_MULTI_KEYS_READY | GD_MULTI_FORWARD | GD_MULTI_NO_KEYS)) return set_err(h, GD_EINVAL, "unknown flags 0x%x", flags);
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(need_comm(h));
    // the batch goes to the device on the exchange stream, so the partition needs no other wait
    GD_TRY(grow(h, h->mx_keys, (size_t)n * sizeof(gd_key) + 8));
    if (n) HIP_TRY(h, hipMemcpyAsync(h->mx_keys.p, keys, (size_t)n * sizeof(gd_key), hipMemcpyHostToDevice, h->pstream));
    GD_TRY(route_multi(h, (const gd_key*)h->mx_keys.p, n, n_act, flags | GD_MULTI_KEYS_READY, out));
    HIP_TRY(h, hipStreamSynchronize(h->xstream));
    return sync_checked(h);
}

int gd_route_multi_ext_device(gd_handle* h, const gd_key* d_keys, const gd_key_ext* d_ext, uint32_t n, uint32_t n_act,
                              int flags, gd_multi_result* out) {
    if (!h || (n && (!d_keys || !d_ext || !d_ext->offset || !d_ext->length))) return set_err(h, GD_EINVAL, "null argument");
    if (flags & ~(GD_MULTI_RETURN_ROUTES | GD_MULTI_KEYS_READY | GD_MULTI_FORWARD | GD_MULTI_NO_KEYS)) return set_err(h, GD_EINVAL, "unknown flags 0x%x", flags);
    HIP_TRY(h, hipSetDevice(h->device));
    return route_multi(h, d_keys, n, n_act, flags, out, d_ext);
}

int gd_route_multi_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, uint32_t n_act, int flags,
                       gd_multi_result* out) {
    if (!h || (n && (!keys || !ext || !ext->offset || !ext->length))) return set_err(h, GD_EINVAL, "null argument");
    if (flags & ~(GD_MULTI_RETURN_ROUTES | GD_MULTI_KEYS_READY | GD_MULTI_FORWARD | GD_MULTI_NO_KEYS)) return set_err(h, GD_EINVAL, "unknown flags 0x%x", flags);
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(need_comm(h));
    // the batch and its strings go to the device on the exchange stream
    GD_TRY(grow(h, h->mx_keys, (size_t)n * sizeof(gd_key) + 8));
    GD_TRY(grow(h, h->mx_ext[0], (size_t)ext->bytes_len + 16));
    GD_TRY(grow(h, h->mx_ext[1], (size_t)n * 8 + 8));
    GD_TRY(grow(h, h->mx_ext[2], (size_t)n * 4 + 4));
    if (n) {
        HIP_TRY(h, hipMemcpyAsync(h->mx_keys.p, keys, (size_t)n * sizeof(gd_key), hipMemcpyHostToDevice, h->pstream));
        if (ext->bytes_len)
            HIP_TRY(h, hipMemcpyAsync(h->mx_ext[0].p, ext->bytes, ext->bytes_len, hipMemcpyHostToDevice, h->pstream));
        HIP_TRY(h, hipMemcpyAsync(h->mx_ext[1].p, ext->offset, (size_t)n * 8, hipMemcpyHostToDevice, h->pstream));
        HIP_TRY(h, hipMemcpyAsync(h->mx_ext[2].p, ext->length, (size_t)n * 4, hipMemcpyHostToDevice, h->pstream));
    }
    const gd_key_ext dx{(const uint8_t*)h->mx_ext[0].p, (const uint64_t*)h->mx_ext[1].p,
                        (const int32_t*)h->mx_ext[2].p, ext->bytes_len};
    GD_TRY(route_multi(h, (const gd_key*)h->mx_keys.p, n, n_act, flags | GD_MULTI_KEYS_READY, out, &dx));
    HIP_TRY(h, hipStreamSynchronize(h->xstream));
    return sync_checked(h);
}

int gd_multi_fetch(gd_handle* h, gd_key* recv_keys, uint32_t* recv_idx, uint32_t* recv_src, uint32_t* silo,
                   uint32_t* act, uint8_t* status, uint32_t* perm, uint32_t* offsets, uint32_t* ret_silo,
                   uint32_t* ret_act, uint8_t* ret_status) {
    if (!h) return set_err(h, GD_EINVAL, "null argument");
    if (h->mcalls == 0) return set_err(h, GD_ESTATE, "no gd_route_multi result on this handle");
    const int s = (int)((h->mcalls - 1) & 1);
    const gd_multi_result& r = h->mres[s];
    if (!r.ret_silo && (ret_silo || ret_act || ret_status))
        return set_err(h, GD_EINVAL, "the last gd_route_multi ran without GD_MULTI_RETURN_ROUTES");
    HIP_TRY(h, hipSetDevice(h->device));
    const size_t m = r.n_recv, n = h->mres_n[s];
    auto cp = [&](void* dst, const void* src, size_t bytes) -> int {
        if (dst && bytes) HIP_TRY(h, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->stream));
        return GD_OK;
    };
    if (recv_keys && m && !r.recv_keys)
        return set_err(h, GD_EINVAL, "the last gd_route_multi ran with GD_MULTI_NO_KEYS");
    if (r.recv_keys) GD_TRY(cp(recv_keys, r.recv_keys, m * sizeof(gd_key)));
    GD_TRY(cp(recv_idx, r.recv_idx, m * 4));
    GD_TRY(cp(recv_src, r.recv_src, m * 4));
    GD_TRY(cp(silo, r.silo, m * 4));
    GD_TRY(cp(act, r.act, m * 4));
    GD_TRY(cp(status, r.status, m));
    GD_TRY(cp(perm, r.perm, m * 4));
    GD_TRY(cp(offsets, r.offsets, ((size_t)r.n_act + 2) * 4));
    if (r.ret_silo) {
        GD_TRY(cp(ret_silo, r.ret_silo, n * 4));
        GD_TRY(cp(ret_act, r.ret_act, n * 4));
        GD_TRY(cp(ret_status, r.ret_status, n));
    }
    return sync(h);
}

// ================================================================== multi-rank directory handoff (SURVEY 8 f4 over 8 e)
// A membership change moves directory entries between the ranks' partitions: every rank splits off
// the entries whose new owner (the installed ring) lives on another rank, they travel in one grouped
// round with their ActivationId and VersionTag, and the receiver applies them the way the reference
// distinguishes the two events (GrainDirectoryHandoffManager.cs):
//   GD_HANDOFF_ADD     ProcessSiloAddEvent (:195-245): RegisterMany(singleActivation: true) on the new
//                      owner -- AddSingleActivation, the first registration wins (:304-326)
//   GD_HANDOFF_REMOVE  ProcessSiloRemoveEvent (:125-158): GrainDirectoryPartition.Merge of the removed
//                      silo's partition (:497-522) -- GrainInfo.Merge keeps the lowest ActivationId
//                      (:139-179) and the loser goes to Catalog.DeleteActivations on its silo
namespace gdx {

int handoff_multi(gd_handle* h, const uint8_t* keep, uint32_t n_keep, int event, uint32_t act_base,
                  gd_handoff_result* out) {
    GD_TRY(need_comm(h));
    GD_TRY(check_ring(h));
    const int W = h->n_ranks;
    GD_TRY(sync(h));
    h->ho_valid = false;
    // 1. split: the entries this rank no longer owns, with ActivationId and tag, removed here
    uint64_t total = 0;
    GD_TRY(split_count(h, keep, n_keep, &total));
    if (total >= 0xFFFFFFFFull) return set_err(h, GD_EINVAL, "handoff of %llu entries", (unsigned long long)total);
    const uint32_t n = (uint32_t)total;
    DevBuf* S = h->ho_send;
    const size_t n4 = (size_t)n * 4 + 16, nk = (size_t)n * sizeof(gd_key) + 16;
    const size_t want_s[10] = {nk, nk, n4, n4, nk, n4, nk, (size_t)W * 8 + 16, n4, n4};
    for (int b = 0; b < 10; ++b) GD_TRY(ensure(h, S[b], want_s[b]));
    gd_key* keys = (gd_key*)S[0].p;             // split (slot) order
    gd_key* ids = (gd_key*)S[1].p;
    uint32_t* silo = (uint32_t*)S[2].p;
    uint32_t* tag = (uint32_t*)S[3].p;
    gd_key* send_keys = (gd_key*)S[4].p;        // partition order
    uint32_t* send_idx = (uint32_t*)S[5].p;
    gd_key* send_ids = (gd_key*)S[6].p;
    uint32_t* dcnt = (uint32_t*)S[7].p;
    uint32_t* send_silo = (uint32_t*)S[8].p;
    uint32_t* send_tag = (uint32_t*)S[9].p;
    if (n) {
        const unsigned long long cap = h->capacity;
        GD_TRY(launch(h, "k_split_emit_tagged", dim3(blocks_for(cap, BLOCK)), dim3(BLOCK), 0, k_split_emit_tagged,
                      h->slots, cap, (const uint32_t*)h->churn[1].p, (const uint32_t*)h->churn[2].p, 1,
                      (const uint32_t*)h->vtag, (const gd_key*)h->act_ids.p, (unsigned long long)h->n_act_ids, keys,
                      ids, silo, tag, h->ctr));
        GD_TRY(check_dir_err(h, "gd_dir_handoff_multi (split)"));
    }
    // 2. stable partition by the new owner's rank (slot order kept per destination), fields alongside
    GD_TRY(shard_pack<false>(h, keys, nullptr, n, 0, (uint32_t)W, send_keys, send_idx, dcnt));
    if (n)
        GD_TRY(launch(h, "k_gather_handoff", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), 0, k_gather_handoff,
                      (const uint32_t*)send_idx, n, (const gd_key*)ids, (const uint32_t*)silo, (const uint32_t*)tag,
                      send_ids, send_silo, send_tag));
    std::vector<uint32_t> sc, rc;
    // 3. counts, then one grouped round: key 24 B + ActivationId 24 B + silo 4 B + tag 4 B an entry
    GD_TRY(counts_round(h, dcnt, sc, rc));
    std::vector<uint64_t> soff(W + 1, 0), roff(W + 1, 0);
    for (int r = 0; r < W; ++r) {
        soff[r + 1] = soff[r] + sc[r];
        roff[r + 1] = roff[r] + rc[r];
    }
    if (soff[W] != n)
        return set_err(h, GD_ERCCL, "handoff partition counts sum to %llu, split %u", (unsigned long long)soff[W], n);
    if (roff[W] >= 0xFFFFFFFFull) return set_err(h, GD_EINVAL, "%llu entries received", (unsigned long long)roff[W]);
    const uint32_t m = (uint32_t)roff[W];
    if ((uint64_t)act_base + m >= GD_ACT_MULTI)
        return set_err(h, GD_EINVAL, "activation indices %u + %u run into the reserved range", act_base, m);
    DevBuf* R = h->ho_recv;
    const size_t m4 = (size_t)m * 4 + 16, mk = (size_t)m * sizeof(gd_key) + 16, mv = (size_t)m * sizeof(gd_val) + 16;
    const size_t want_r[11] = {mk, mk, m4, m4, m4, m4, (size_t)m + 16, mv, mv, mv, (size_t)m + 16};
    for (int b = 0; b < 11; ++b) GD_TRY(ensure(h, R[b], want_r[b]));
    gd_key* rkeys = (gd_key*)R[0].p;
    gd_key* rids = (gd_key*)R[1].p;
    uint32_t* rsilo = (uint32_t*)R[2].p;
    uint32_t* rtag = (uint32_t*)R[3].p;
    uint32_t* rsrc = (uint32_t*)R[4].p;
    uint32_t* racts = (uint32_t*)R[5].p;
    uint8_t* rst = (uint8_t*)R[6].p;
    gd_val* rdrop = (gd_val*)R[7].p;
    gd_val* vals = (gd_val*)R[8].p;
    gd_val* got = (gd_val*)R[9].p;
    uint8_t* ins = (uint8_t*)R[10].p;
    const Lane lanes[4] = {{send_keys, rkeys, sizeof(gd_key), ncclUint64, 3},
                           {send_ids, rids, sizeof(gd_key), ncclUint64, 3},
                           {send_silo, rsilo, 4, ncclUint32, 1},
                           {send_tag, rtag, 4, ncclUint32, 1}};
    GD_TRY(exchange_round(h, "rccl_handoff", sc.data(), soff.data(), rc.data(), roff.data(), lanes, 4));
    if (m)
        GD_TRY(launch(h, "k_recv_src", dim3(blocks_for(m, BLOCK)), dim3(BLOCK), 0, k_recv_src,
                      (const uint32_t*)(dcnt + W), (uint32_t)W, m, rsrc));
    // 4. apply on the receiver: activation indices act_base + j, then Register or Merge
    if (m) {
        GD_TRY(grow_act_ids(h, (uint64_t)act_base + m));
        GD_TRY(launch(h, "k_handoff_vals", dim3(blocks_for(m, BLOCK)), dim3(BLOCK), 0, k_handoff_vals,
                      (const gd_key*)rids, (const uint32_t*)rsilo, m, act_base, (gd_key*)h->act_ids.p, vals, racts));
        if (event == GD_HANDOFF_REMOVE) {
            GD_TRY(merge_core(h, rkeys, vals, (const int32_t*)rtag, m, rst, rdrop));
            GD_TRY(check_dir_err(h, "gd_dir_handoff_multi (merge)"));
        } else {
            GD_TRY(register_core(h, rkeys, vals, m, got, ins));
            GD_TRY(launch(h, "k_handoff_add_status", dim3(blocks_for(m, BLOCK)), dim3(BLOCK), 0, k_handoff_add_status,
                          (const gd_val*)vals, (const gd_val*)got, (const uint8_t*)ins, m, (const gd_key*)h->act_ids.p,
                          (unsigned long long)h->n_act_ids, rst, rdrop));
        }
    }
    GD_TRY(sync(h));
    gd_handoff_result& r = h->ho_res;
    r = gd_handoff_result{};
    r.n_sent = n;
    r.n_recv = m;
    r.recv_keys = rkeys;
    r.recv_ids = rids;
    r.recv_act = racts;
    r.recv_silo = rsilo;
    r.recv_src = rsrc;
    r.status = rst;
    r.dropped = rdrop;
    h->ho_valid = true;
    if (out) *out = r;
    return GD_OK;
}

}  // namespace gdx

extern "C" {

int gd_dir_handoff_multi(gd_handle* h, const uint8_t* keep_silo, uint32_t n_keep, int event, uint32_t act_base,
                         gd_handoff_result* out) {
    if (!h || (n_keep && !keep_silo)) return set_err(h, GD_EINVAL, "null argument");
    if (event != GD_HANDOFF_ADD && event != GD_HANDOFF_REMOVE) return set_err(h, GD_EINVAL, "unknown event %d", event);
    HIP_TRY(h, hipSetDevice(h->device));
    return handoff_multi(h, keep_silo, n_keep, event, act_base, out);
}

int gd_dir_handoff_fetch(gd_handle* h, gd_key* keys, gd_key* ids, uint32_t* acts, uint32_t* silos, uint32_t* src,
                         uint8_t* status, gd_val* dropped) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    if (!h->ho_valid) return set_err(h, GD_ESTATE, "no gd_dir_handoff_multi result on this handle");
    HIP_TRY(h, hipSetDevice(h->device));
    const gd_handoff_result& r = h->ho_res;
    const size_t m = r.n_recv;
    auto cp = [&](void* d, const void* sp, size_t bytes) -> int {
        if (d && bytes) HIP_TRY(h, hipMemcpyAsync(d, sp, bytes, hipMemcpyDeviceToHost, h->stream));
        return GD_OK;
    };
    GD_TRY(cp(keys, r.recv_keys, m * sizeof(gd_key)));
    GD_TRY(cp(ids, r.recv_ids, m * sizeof(gd_key)));
    GD_TRY(cp(acts, r.recv_act, m * 4));
    GD_TRY(cp(silos, r.recv_silo, m * 4));
    GD_TRY(cp(src, r.recv_src, m * 4));
    GD_TRY(cp(status, r.status, m));
    GD_TRY(cp(dropped, r.dropped, m * sizeof(gd_val)));
    GD_TRY(sync(h));
    if (silos)                                     // the multi-activation mark is internal
        for (size_t j = 0; j < m; ++j) silos[j] &= 0xFFFFu;
    return GD_OK;
}

}  // extern "C"
