// eng_fanout.hip -- libgraindispatch: follower fan-out on one GPU and the sharded fan-out cascade (SURVEY 8 f2, 8 e).
// Shared handle and helpers: gd_engine.h.
#include "gd_engine.h"

// ================================================================== follower fan-out
namespace gdx {

uint64_t grain_tcd(int32_t type_code) {
    // UniqueKey.NewKey(long, Category.Grain, typeData) (UniqueKey.cs:112-128): the int type code is
    // sign-extended, then masked to 56 bits.
    return ((uint64_t)CAT_GRAIN << 56) + ((uint64_t)(int64_t)type_code & 0x00FFFFFFFFFFFFFFull);
}

// Degrees + inclusive scan into fan[0] (ends); the total message count comes back to the host.
int fan_count(gd_handle* h, const uint32_t* row_off, uint32_t n_nodes, const uint32_t* frontier, uint32_t nf,
              uint64_t* total) {
    *total = 0;
    if (nf == 0) return GD_OK;
    GD_TRY(ensure(h, h->fan[0], (size_t)nf * 4));
    // frontiers up to 16M publishers: degrees with the scan's tile sums, the down-sweep, and the
    // partials back to the host (2 launches, one small pinned copy)
    const uint32_t nb4 = blocks_for(nf, SCAN_TILE), nb16 = blocks_for(nf, 4 * SCAN_TILE);
    if (nb4 <= 2048 || nb16 <= 4096) {
        const bool wide = nb4 > 2048;
        const uint32_t nb = wide ? nb16 : nb4;
        GD_TRY(ensure(h, h->fan[1], (size_t)nb * 4));
        GD_TRY(pinned_scratch(h, (size_t)nb * 4));
        uint32_t* ends = (uint32_t*)h->fan[0].p;
        uint32_t* part = (uint32_t*)h->fan[1].p;
        if (wide) {
            GD_TRY(launch(h, "k_fan_degree", dim3(nb), dim3(BLOCK), 0, k_fan_degree_tiles<16>, row_off, n_nodes, frontier,
                          nf, ends, part, (const uint32_t*)nullptr));
            GD_TRY(launch(h, "k_scan_down", dim3(nb), dim3(BLOCK), 0, k_scan_down<OpAdd, 16>, (const uint32_t*)ends, ends,
                          nf, false, true, (const uint32_t*)part, nb));
        } else {
            GD_TRY(launch(h, "k_fan_degree", dim3(nb), dim3(BLOCK), 0, k_fan_degree_tiles<4>, row_off, n_nodes, frontier,
                          nf, ends, part, (const uint32_t*)nullptr));
            GD_TRY(launch(h, "k_scan_down", dim3(nb), dim3(BLOCK), 0, k_scan_down<OpAdd, 4>, (const uint32_t*)ends, ends,
                          nf, false, true, (const uint32_t*)part, nb));
        }
        HIP_TRY(h, hipMemcpyAsync(h->h_pin, part, (size_t)nb * 4, hipMemcpyDeviceToHost, h->stream));
        GD_TRY(sync(h));
        uint64_t t = 0;
        for (uint32_t b = 0; b < nb; ++b) t += ((const uint32_t*)h->h_pin)[b];
        if (t > 0xFFFFFFFFull) return set_err(h, GD_EINVAL, "fan-out of %llu messages exceeds 2^32 - 1",
                                              (unsigned long long)t);
        *total = t;
        return GD_OK;
    }
    GD_TRY(ensure(h, h->fan[1], 8));
    unsigned long long* dtot = (unsigned long long*)h->fan[1].p;
    HIP_TRY(h, hipMemsetAsync(dtot, 0, 8, h->stream));
    uint32_t* ends = (uint32_t*)h->fan[0].p;
    GD_TRY(launch(h, "k_fan_degree", dim3(std::min<uint32_t>(blocks_for(nf, BLOCK), 1024)), dim3(BLOCK), 0, k_fan_degree, row_off, n_nodes,
                  frontier, nf, ends, dtot));
    GD_TRY(scan_device<OpAdd>(h, ends, nf, false, true, "fan"));
    unsigned long long t = 0;
    HIP_TRY(h, hipMemcpyAsync(&t, dtot, 8, hipMemcpyDeviceToHost, h->stream));
    GD_TRY(sync(h));
    if (t > 0xFFFFFFFFull) return set_err(h, GD_EINVAL, "fan-out of %llu messages exceeds 2^32 - 1", t);
    *total = t;
    return GD_OK;
}

int fan_args_ok(gd_handle* h, const uint32_t* row_off, const uint32_t* dst, uint32_t nf, const uint32_t* frontier,
                uint64_t* out_n) {
    if (!h || !out_n) return set_err(h, GD_EINVAL, "null argument");
    if (nf && (!row_off || !dst || !frontier)) return set_err(h, GD_EINVAL, "null graph / frontier");
    return GD_OK;
}

// Tiles of 512 outputs below 1,024 tiles of 2,048 (a small hop -- cfg 4's first, 0.64M messages -- would
// otherwise leave most CUs idle with 4 dependent probe rounds a thread).
constexpr uint32_t FAN_SMALL_TILES = 1024;

template <int MODE, bool CX, bool CX8, int IT>
int fan_route_launch_it(gd_handle* h, const uint32_t* row_off, const uint32_t* dst, const uint32_t* frontier,
                        uint32_t nf, uint32_t total, uint64_t tcd, uint32_t* target, uint32_t* sender, uint32_t* silo,
                        uint32_t* act, uint8_t* status, const uint32_t* d_nf, bool dev_total) {
    const dim3 g(blocks_for(total, BLOCK * IT)), b(BLOCK);
    const uint32_t* ends = (const uint32_t*)h->fan[0].p;
    const CxArgs cx = CX ? cx_args(h) : CxArgs{};
    const Cx8Args cx8 = CX8 ? cx8_args(h) : Cx8Args{};
    // GD_OPT_FAN_BOUND: the kernel's memory bound (k_fan_route<..., BOUND>) on this hop's own inputs, into
    // scratch outputs of the same layout; before the real launch on even launches, after it on odd ones, so
    // neither form always finds the other's lines in the caches
    const bool bound = CX8 && h->fan_bound && total;
    const bool after = bound && (h->fan_bound_n++ & 1u);
    auto launch_bound = [&]() -> int {
        const size_t cap = (size_t)total;
        GD_TRY(ensure(h, h->fan_bnd, cap * 17 + 64));
        uint32_t* o = (uint32_t*)h->fan_bnd.p;
        return launch(h, "k_fan_bound", g, b, ring_lds(h), k_fan_route<MODE, 2, false, (int)CX_GROUP, true, IT, true>,
                      row_off, dst, frontier, nf, ends, total, tcd, ring_args(h), table_args(h), target ? o : nullptr,
                      o + cap, o + 2 * cap, o + 3 * cap, (uint8_t*)(o + 4 * cap), CxArgs{}, cx8, d_nf,
                      (uint32_t)dev_total);
    };
    if (bound && !after) GD_TRY(launch_bound());
    // 2 outputs a thread in flight (1: 2.95 ms, 4: 3.03 ms against 2.87 ms a cfg 4 cascade,
    // profiles/r02_v1_fanout_cfg4_ilp_ab.jsonl)
    GD_TRY(launch(h, "k_fan_route", g, b, ring_lds(h), k_fan_route<MODE, 2, CX, (int)CX_GROUP, CX8, IT>, row_off, dst,
                  frontier, nf, ends, total, tcd, ring_args(h), table_args(h), target, sender, silo, act, status, cx, cx8,
                  d_nf, (uint32_t)dev_total));
    if (after) GD_TRY(launch_bound());
    return GD_OK;
}

template <int MODE, bool CX, bool CX8>
int fan_route_launch_cx(gd_handle* h, const uint32_t* row_off, const uint32_t* dst, const uint32_t* frontier,
                        uint32_t nf, uint32_t total, uint64_t tcd, uint32_t* target, uint32_t* sender, uint32_t* silo,
                        uint32_t* act, uint8_t* status, const uint32_t* d_nf, bool dev_total) {
    if (blocks_for(total, FAN_TILE) < FAN_SMALL_TILES)
        return fan_route_launch_it<MODE, CX, CX8, 2>(h, row_off, dst, frontier, nf, total, tcd, target, sender, silo,
                                                      act, status, d_nf, dev_total);
    return fan_route_launch_it<MODE, CX, CX8, FAN_IT>(h, row_off, dst, frontier, nf, total, tcd, target, sender, silo,
                                                       act, status, d_nf, dev_total);
}

template <int MODE>
int fan_route_launch(gd_handle* h, const uint32_t* row_off, const uint32_t* dst, const uint32_t* frontier, uint32_t nf,
                     uint32_t total, uint64_t tcd, uint32_t* target, uint32_t* sender, uint32_t* silo, uint32_t* act,
                     uint8_t* status, const uint32_t* d_nf, bool dev_total) {
    bool cx = false;
    GD_TRY(cx_ensure(h, &cx, total));
    int meas = -1;
    const int var = cx ? cx_choose(h, 2, total, &meas, h->cx8_ok ? 3 : 2) : 1;
    CxMeasure m(h, meas, total);
    if (var == 2)                      // the 8-B index
        return fan_route_launch_cx<MODE, false, true>(h, row_off, dst, frontier, nf, total, tcd, target, sender, silo,
                                                      act, status, d_nf, dev_total);
    if (var == 0)
        return fan_route_launch_cx<MODE, true, false>(h, row_off, dst, frontier, nf, total, tcd, target, sender, silo,
                                                      act, status, d_nf, dev_total);
    return fan_route_launch_cx<MODE, false, false>(h, row_off, dst, frontier, nf, total, tcd, target, sender, silo, act,
                                                   status, d_nf, dev_total);
}

// dev_total: `total` is the outputs' capacity and the hop's size is read on the device (k_fan_route); the
// caller counts the messages routed once it knows them.
int fan_route(gd_handle* h, const uint32_t* row_off, const uint32_t* dst, const uint32_t* frontier, uint32_t nf,
              uint32_t total, uint64_t tcd, uint32_t* target, uint32_t* sender, uint32_t* silo, uint32_t* act,
              uint8_t* status, const uint32_t* d_nf, bool dev_total) {
    if (!dev_total) h->routed += total;
    switch (h->ring_mode) {
        case GD_RING_DIRECTORY:
            return fan_route_launch<GD_RING_DIRECTORY>(h, row_off, dst, frontier, nf, total, tcd, target, sender, silo,
                                                       act, status, d_nf, dev_total);
        case GD_RING_CONSISTENT:
            return fan_route_launch<GD_RING_CONSISTENT>(h, row_off, dst, frontier, nf, total, tcd, target, sender, silo,
                                                        act, status, d_nf, dev_total);
        default:
            return fan_route_launch<GD_RING_VIRTUAL_BUCKETS>(h, row_off, dst, frontier, nf, total, tcd, target, sender,
                                                             silo, act, status, d_nf, dev_total);
    }
}

template <int MODE>
int route_nodes_mode(gd_handle* h, const uint32_t* nodes, uint32_t n, uint64_t tcd, uint32_t* silo, uint32_t* act,
                     uint8_t* status, bool cx, bool cx8 = false) {
    const dim3 g(blocks_for(n, BLOCK)), b(BLOCK);
    if (cx8)
        return launch(h, "k_route_nodes", g, b, ring_lds(h), k_route_nodes<MODE, false, (int)CX_GROUP, true>, nodes, n,
                      tcd, ring_args(h), table_args(h), silo, act, status, CxArgs{}, cx8_args(h));
    if (cx)
        return launch(h, "k_route_nodes", g, b, ring_lds(h), k_route_nodes<MODE, true>, nodes, n, tcd, ring_args(h),
                      table_args(h), silo, act, status, cx_args(h), Cx8Args{});
    return launch(h, "k_route_nodes", g, b, ring_lds(h), k_route_nodes<MODE, false>, nodes, n, tcd, ring_args(h),
                  table_args(h), silo, act, status, CxArgs{}, Cx8Args{});
}

int route_nodes(gd_handle* h, const uint32_t* nodes, uint32_t n, uint64_t tcd, uint32_t* silo, uint32_t* act,
                uint8_t* status) {
    GD_TRY(check_ring(h));
    h->routed += n;
    bool cx = false;
    GD_TRY(cx_ensure(h, &cx, n));
    int meas = -1;
    const int var = cx ? cx_choose(h, 3, n, &meas, h->cx8_ok ? 3 : 2) : 1;
    cx = var == 0;
    const bool cx8 = var == 2;
    CxMeasure m(h, meas, n);
    switch (h->ring_mode) {
        case GD_RING_DIRECTORY:
            return route_nodes_mode<GD_RING_DIRECTORY>(h, nodes, n, tcd, silo, act, status, cx, cx8);
        case GD_RING_CONSISTENT:
            return route_nodes_mode<GD_RING_CONSISTENT>(h, nodes, n, tcd, silo, act, status, cx, cx8);
        default: return route_nodes_mode<GD_RING_VIRTUAL_BUCKETS>(h, nodes, n, tcd, silo, act, status, cx, cx8);
    }
}

// count + compact over n_act (gd_fanout.h); returns the new frontier size.
int frontier_next(gd_handle* h, const uint32_t* offsets, uint32_t n_act, uint8_t* visited, uint32_t* out,
                  uint32_t* out_n) {
    *out_n = 0;
    if (n_act == 0) return GD_OK;
    const uint32_t nb = blocks_for(n_act, FR_TILE);
    GD_TRY(ensure(h, h->fan[2], (size_t)nb * BLOCK * sizeof(uint16_t)));
    GD_TRY(ensure(h, h->fan[3], ((size_t)nb + 1) * 4));
    uint16_t* flags = (uint16_t*)h->fan[2].p;
    uint32_t* counts = (uint32_t*)h->fan[3].p;
    uint32_t* total = counts + nb;
    GD_TRY(launch(h, "k_frontier_count", dim3(nb), dim3(BLOCK), 0, k_frontier_count, offsets, n_act, visited, flags,
                  counts));
    GD_TRY(launch(h, "k_frontier_compact", dim3(nb), dim3(BLOCK), 0, k_frontier_compact, (const uint16_t*)flags,
                  (const uint32_t*)counts, nb, out, total));
    GD_TRY(pinned_scratch(h, 4));
    HIP_TRY(h, hipMemcpyAsync(h->h_pin, total, 4, hipMemcpyDeviceToHost, h->stream));
    GD_TRY(sync(h));
    *out_n = *(const uint32_t*)h->h_pin;
    return GD_OK;
}

// frontier_next without the read-back: the new frontier's length stays on the device (*d_nf).
int frontier_next_dev(gd_handle* h, const uint32_t* offsets, uint32_t n_act, uint8_t* visited, uint32_t* out,
                      const uint32_t** d_nf) {
    const uint32_t nb = blocks_for(std::max<uint32_t>(n_act, 1), FR_TILE);
    GD_TRY(ensure(h, h->fan[2], (size_t)nb * BLOCK * sizeof(uint16_t)));
    GD_TRY(ensure(h, h->fan[3], ((size_t)nb + 1) * 4));
    uint16_t* flags = (uint16_t*)h->fan[2].p;
    uint32_t* counts = (uint32_t*)h->fan[3].p;
    uint32_t* total = counts + nb;
    *d_nf = total;
    if (n_act == 0) {
        HIP_TRY(h, hipMemsetAsync(total, 0, 4, h->stream));
        return GD_OK;
    }
    GD_TRY(launch(h, "k_frontier_count", dim3(nb), dim3(BLOCK), 0, k_frontier_count, offsets, n_act, visited, flags,
                  counts));
    return launch(h, "k_frontier_compact", dim3(nb), dim3(BLOCK), 0, k_frontier_compact, (const uint16_t*)flags,
                  (const uint32_t*)counts, nb, out, total);
}

// Degrees + inclusive scan of a frontier (nf_max rows; with d_nf, *d_nf <= nf_max rows on the device)
// into fan[0], then its tile sums and length copied to pinned memory behind h->fan_ev: fan_count_wait
// reads them.  The degree and scan grids are sized for nf_max.  *nb = 0: past 16M rows (one read-back
// cannot carry the tile sums), nothing enqueued -- fan_count_dev's slow path.
int fan_count_post(gd_handle* h, const uint32_t* row_off, uint32_t n_nodes, const uint32_t* frontier,
                   const uint32_t* d_nf, uint32_t nf_max, uint32_t* nb_out) {
    *nb_out = 0;
    const uint32_t nb4 = blocks_for(nf_max, SCAN_TILE), nb16 = blocks_for(nf_max, 4 * SCAN_TILE);
    if (nf_max == 0 || !(nb4 <= 2048 || nb16 <= 4096)) return GD_OK;
    const bool wide = nb4 > 2048;
    const uint32_t nb = wide ? nb16 : nb4;
    GD_TRY(ensure(h, h->fan[0], (size_t)nf_max * 4));
    GD_TRY(ensure(h, h->fan[1], (size_t)nb * 4));
    GD_TRY(pinned_scratch(h, ((size_t)nb + 1) * 4));
    if (!h->fan_ev) HIP_TRY(h, hipEventCreateWithFlags(&h->fan_ev, hipEventDisableTiming));
    uint32_t* ends = (uint32_t*)h->fan[0].p;
    uint32_t* part = (uint32_t*)h->fan[1].p;
    if (wide) {
        GD_TRY(launch(h, "k_fan_degree", dim3(nb), dim3(BLOCK), 0, k_fan_degree_tiles<16>, row_off, n_nodes, frontier,
                      nf_max, ends, part, d_nf));
        GD_TRY(launch(h, "k_scan_down", dim3(nb), dim3(BLOCK), 0, k_scan_down<OpAdd, 16>, (const uint32_t*)ends, ends,
                      nf_max, false, true, (const uint32_t*)part, nb));
    } else {
        GD_TRY(launch(h, "k_fan_degree", dim3(nb), dim3(BLOCK), 0, k_fan_degree_tiles<4>, row_off, n_nodes, frontier,
                      nf_max, ends, part, d_nf));
        GD_TRY(launch(h, "k_scan_down", dim3(nb), dim3(BLOCK), 0, k_scan_down<OpAdd, 4>, (const uint32_t*)ends, ends,
                      nf_max, false, true, (const uint32_t*)part, nb));
    }
    uint32_t* pin = (uint32_t*)h->h_pin;
    HIP_TRY(h, hipMemcpyAsync(pin, part, (size_t)nb * 4, hipMemcpyDeviceToHost, h->stream));
    if (d_nf) HIP_TRY(h, hipMemcpyAsync(pin + nb, d_nf, 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipEventRecord(h->fan_ev, h->stream));
    *nb_out = nb;
    return GD_OK;
}

// Waits for fan_count_post's read-back only (work enqueued after it keeps running): the frontier's
// length and the hop's u64 total.
int fan_count_wait(gd_handle* h, uint32_t nb, const uint32_t* d_nf, uint32_t nf_max, uint32_t* nf, uint64_t* total) {
    HIP_TRY(h, hipEventSynchronize(h->fan_ev));
    const uint32_t* pin = (const uint32_t*)h->h_pin;
    uint64_t t = 0;
    for (uint32_t b = 0; b < nb; ++b) t += pin[b];
    if (t > 0xFFFFFFFFull)
        return set_err(h, GD_EINVAL, "fan-out of %llu messages exceeds 2^32 - 1", (unsigned long long)t);
    *nf = d_nf ? pin[nb] : nf_max;
    *total = t;
    return GD_OK;
}

// fan_count of a frontier whose length is on the device (*d_nf <= nf_max): one read-back brings both
// the length and the total (instead of one for each).  Past 16M rows it reads the length first and
// takes fan_count.
int fan_count_dev(gd_handle* h, const uint32_t* row_off, uint32_t n_nodes, const uint32_t* frontier,
                  const uint32_t* d_nf, uint32_t nf_max, uint32_t* nf, uint64_t* total) {
    *nf = 0;
    *total = 0;
    if (nf_max == 0) return GD_OK;
    uint32_t nb = 0;
    GD_TRY(fan_count_post(h, row_off, n_nodes, frontier, d_nf, nf_max, &nb));
    if (nb) return fan_count_wait(h, nb, d_nf, nf_max, nf, total);
    GD_TRY(pinned_scratch(h, 4));
    HIP_TRY(h, hipMemcpyAsync(h->h_pin, d_nf, 4, hipMemcpyDeviceToHost, h->stream));
    GD_TRY(sync(h));
    *nf = *(const uint32_t*)h->h_pin;
    return fan_count(h, row_off, n_nodes, frontier, *nf, total);
}

// The whole single-GPU cascade in the library (gd_fanout_cascade_device): per hop the fused
// expand + route (k_fan_route), the bucketing and the next frontier, with one host read-back a hop
// (the next hop's size and its publishers' count together).  Results in the handle's hop buffers
// (fm_hop / fm_res, read by gd_fanout_multi_fetch).
int fanout_cascade(gd_handle* h, const uint32_t* row_off, const uint32_t* dst, uint32_t n_nodes, const uint32_t* seeds,
                   uint32_t n_seeds, int32_t type_code, uint32_t n_act, uint32_t hops, gd_fanout_hop* out) {
    GD_TRY(check_ring(h));
    if (n_act == 0xFFFFFFFFu) return set_err(h, GD_EINVAL, "n_act too large");
    const uint64_t tcd = grain_tcd(type_code);
    // no synchronisation with the previous cascade: its buffers are rewritten in stream order (ensure()
    // synchronises before it frees one), so this cascade's first launches queue behind its last ones
    if (h->fm_hop.size() < hops) h->fm_hop.resize(hops);
    h->fm_res.assign(hops, gd_fanout_hop{});
    h->fm_n_act = n_act;
    DevBuf* S = h->fm_scr;
    GD_TRY(ensure(h, S[5], (size_t)n_act + 16));
    uint8_t* visited = (uint8_t*)S[5].p;
    HIP_TRY(h, hipMemsetAsync(visited, 0, (size_t)n_act + 16, h->stream));
    {
        std::array<DevBuf, 10>& H0 = h->fm_hop[0];
        GD_TRY(ensure(h, H0[0], ((size_t)std::max(n_seeds, n_act) + 4) * 4));
        if (n_seeds) {
            HIP_TRY(h, hipMemcpyAsync(H0[0].p, seeds, (size_t)n_seeds * 4, hipMemcpyDeviceToDevice, h->stream));
            GD_TRY(launch(h, "k_mark_visited", dim3(blocks_for(n_seeds, BLOCK)), dim3(BLOCK), 0, k_mark_visited,
                          (const uint32_t*)H0[0].p, n_seeds, n_act, visited));
        }
    }
    // Per hop: the degrees and their scan, the read-back of the hop's size behind an event, then -- when
    // this hop's buffers (from an earlier cascade) can hold it -- k_fan_route at once, reading the size on
    // the device, while the host waits for the read-back and then queues the bucketing behind it.  The
    // first cascade of a shape, or a hop that outgrows its buffers, waits, sizes them and launches k_fan_route
    // with the host's count.
    const uint32_t* d_nf = nullptr;                    // the frontier's length on the device (hops > 0)
    uint32_t nf_max = n_seeds, nb = 0;
    GD_TRY(fan_count_post(h, row_off, n_nodes, (const uint32_t*)h->fm_hop[0][0].p, nullptr, nf_max, &nb));
    for (uint32_t hp = 0; hp < hops; ++hp) {
        std::array<DevBuf, 10>& H = h->fm_hop[hp];
        const uint32_t* frontier = (const uint32_t*)H[0].p;
        uint64_t cap = ~0ull;                          // messages the hop's buffers hold
        for (int b : {1, 2, 4, 5, 7}) cap = std::min<uint64_t>(cap, H[b].p && H[b].bytes >= 16 ? (H[b].bytes - 16) / 4 : 0);
        cap = std::min<uint64_t>(cap, H[6].p && H[6].bytes >= 16 ? H[6].bytes - 16 : 0);
        cap = std::min<uint64_t>(cap, 0xFFFFFFFFull);
        const bool early = nb && cap && nf_max;
        if (early)
            GD_TRY(fan_route(h, row_off, dst, frontier, nf_max, (uint32_t)cap, tcd, (uint32_t*)H[1].p, (uint32_t*)H[2].p,
                             (uint32_t*)H[4].p, (uint32_t*)H[5].p, (uint8_t*)H[6].p, d_nf, true));
        uint32_t nf = 0;
        uint64_t total = 0;
        if (nb) GD_TRY(fan_count_wait(h, nb, d_nf, nf_max, &nf, &total));
        else if (nf_max && d_nf) GD_TRY(fan_count_dev(h, row_off, n_nodes, frontier, d_nf, nf_max, &nf, &total));
        else if (nf_max) {
            nf = nf_max;
            GD_TRY(fan_count(h, row_off, n_nodes, frontier, nf, &total));
        }
        const uint32_t m = (uint32_t)total;
        const size_t m4 = (size_t)m * 4 + 16;
        const size_t want[10] = {0, m4, m4, 0, m4, m4, (size_t)m + 16, m4, ((size_t)n_act + 2) * 4, 0};
        for (int b = 1; b < 9; ++b)
            if (want[b]) GD_TRY(ensure(h, H[b], want[b]));   // synchronises first if it reallocates
        uint32_t* target = (uint32_t*)H[1].p;
        uint32_t* sender = (uint32_t*)H[2].p;
        uint32_t* silo = (uint32_t*)H[4].p;
        uint32_t* act = (uint32_t*)H[5].p;
        uint8_t* st = (uint8_t*)H[6].p;
        uint32_t* perm = (uint32_t*)H[7].p;
        uint32_t* offs = (uint32_t*)H[8].p;
        if (early && m <= cap) h->routed += m;
        else if (m) GD_TRY(fan_route(h, row_off, dst, frontier, nf, m, tcd, target, sender, silo, act, st));
        GD_TRY(bucket_device(h, act, m, n_act, perm, offs));
        gd_fanout_hop& res = h->fm_res[hp];
        res.n_frontier = nf;
        res.frontier = frontier;
        res.n_sent = total;
        res.n_recv = m;
        res.target = target;
        res.sender = sender;
        res.src = nullptr;
        res.silo = silo;
        res.act = act;
        res.status = st;
        res.perm = perm;
        res.offsets = offs;
        nb = 0;
        if (hp + 1 < hops) {
            std::array<DevBuf, 10>& N = h->fm_hop[hp + 1];
            GD_TRY(ensure(h, N[0], ((size_t)n_act + 4) * 4));
            GD_TRY(frontier_next_dev(h, offs, n_act, visited, (uint32_t*)N[0].p, &d_nf));
            // every new publisher received at least one of this hop's m messages: the scan's bound
            nf_max = std::min(n_act, m);
            GD_TRY(fan_count_post(h, row_off, n_nodes, (const uint32_t*)N[0].p, d_nf, nf_max, &nb));
        }
    }
    if (out) std::copy(h->fm_res.begin(), h->fm_res.end(), out);
    return GD_OK;
}

}  // namespace gdx

extern "C" {

int gd_fanout_cascade_device(gd_handle* h, const uint32_t* d_row_off, const uint32_t* d_dst, uint32_t n_nodes,
                             const uint32_t* d_seeds, uint32_t n_seeds, int32_t type_code, uint32_t n_act,
                             uint32_t hops, gd_fanout_hop* out) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    if (n_seeds && !d_seeds) return set_err(h, GD_EINVAL, "null seeds");
    if (!d_row_off || (!d_dst && n_nodes)) return set_err(h, GD_EINVAL, "null graph");
    if (hops == 0 || hops > 64) return set_err(h, GD_EINVAL, "hops %u not in [1, 64]", hops);
    HIP_TRY(h, hipSetDevice(h->device));
    return fanout_cascade(h, d_row_off, d_dst, n_nodes, d_seeds, n_seeds, type_code, n_act, hops, out);
}

int gd_fanout_expand_device(gd_handle* h, const uint32_t* d_row_off, const uint32_t* d_dst, uint32_t n_nodes,
                            const uint32_t* d_frontier, uint32_t n_frontier, uint32_t* d_target, uint32_t* d_sender,
                            uint64_t capacity, uint64_t* out_n) {
    GD_TRY(fan_args_ok(h, d_row_off, d_dst, n_frontier, d_frontier, out_n));
    if ((d_target == nullptr) != (d_sender == nullptr)) return set_err(h, GD_EINVAL, "target and sender go together");
    HIP_TRY(h, hipSetDevice(h->device));
    uint64_t total = 0;
    GD_TRY(fan_count(h, d_row_off, n_nodes, d_frontier, n_frontier, &total));
    *out_n = total;
    if (!d_target || total == 0) return GD_OK;                    // size query
    if (total > capacity)
        return set_err(h, GD_EINVAL, "fan-out emits %llu messages, output holds %llu", (unsigned long long)total,
                       (unsigned long long)capacity);
    return launch(h, "k_fan_expand", dim3(blocks_for(total, FAN_TILE)), dim3(BLOCK), 0, k_fan_expand, d_row_off, d_dst,
                  d_frontier, n_frontier, (const uint32_t*)h->fan[0].p, (uint32_t)total, d_target, d_sender,
                  (const uint32_t*)nullptr);
}

int gd_fanout_route_bucket_device(gd_handle* h, const uint32_t* d_row_off, const uint32_t* d_dst, uint32_t n_nodes,
                                  const uint32_t* d_frontier, uint32_t n_frontier, int32_t type_code, uint32_t n_act,
                                  uint32_t* d_target, uint32_t* d_sender, uint32_t* d_silo, uint32_t* d_act,
                                  uint8_t* d_status, uint32_t* d_perm, uint32_t* d_offsets, uint64_t capacity,
                                  uint64_t* out_n) {
    GD_TRY(fan_args_ok(h, d_row_off, d_dst, n_frontier, d_frontier, out_n));
    if (!d_sender || !d_silo || !d_act || !d_status) return set_err(h, GD_EINVAL, "null output");
    if ((d_perm == nullptr) != (d_offsets == nullptr)) return set_err(h, GD_EINVAL, "perm and offsets go together");
    if (d_perm && n_act == 0xFFFFFFFFu) return set_err(h, GD_EINVAL, "n_act too large");
    GD_TRY(check_ring(h));
    HIP_TRY(h, hipSetDevice(h->device));
    uint64_t total = 0;
    GD_TRY(fan_count(h, d_row_off, n_nodes, d_frontier, n_frontier, &total));
    *out_n = total;
    if (total > capacity)
        return set_err(h, GD_EINVAL, "fan-out emits %llu messages, output holds %llu", (unsigned long long)total,
                       (unsigned long long)capacity);
    if (total)
        GD_TRY(fan_route(h, d_row_off, d_dst, d_frontier, n_frontier, (uint32_t)total, grain_tcd(type_code), d_target,
                         d_sender, d_silo, d_act, d_status));
    if (d_perm) GD_TRY(bucket_device(h, d_act, (uint32_t)total, n_act, d_perm, d_offsets));
    return GD_OK;
}

int gd_fanout_route_bucket(gd_handle* h, const uint32_t* row_off, const uint32_t* dst, uint32_t n_nodes,
                           const uint32_t* frontier, uint32_t n_frontier, int32_t type_code, uint32_t n_act,
                           uint32_t* out_target, uint32_t* out_sender, uint32_t* out_silo, uint32_t* out_act,
                           uint8_t* out_status, uint32_t* out_perm, uint32_t* out_offsets, uint64_t capacity,
                           uint64_t* out_n) {
    GD_TRY(fan_args_ok(h, row_off, dst, n_frontier, frontier, out_n));
    if ((out_perm == nullptr) != (out_offsets == nullptr)) return set_err(h, GD_EINVAL, "perm and offsets go together");
    if (out_perm && n_act == 0xFFFFFFFFu) return set_err(h, GD_EINVAL, "n_act too large");
    GD_TRY(check_ring(h));
    HIP_TRY(h, hipSetDevice(h->device));
    *out_n = 0;
    if (n_frontier == 0 || n_nodes == 0) {
        if (out_perm) {
            GD_TRY(ensure(h, h->offs, ((size_t)n_act + 2) * 4));
            GD_TRY(bucket_device(h, nullptr, 0, n_act, nullptr, (uint32_t*)h->offs.p));
            GD_TRY(d2h(h, out_offsets, h->offs, (size_t)n_act + 2));
        }
        return sync_checked(h);
    }
    // graph + frontier in; the graph buffers are re-sent per call (the device form keeps them resident)
    uint64_t edges = 0;
    edges = row_off[n_nodes];
    GD_TRY(h2d(h, h->fan[4], row_off, (size_t)n_nodes + 1));
    GD_TRY(h2d(h, h->fan[5], dst, edges ? edges : 1));
    GD_TRY(h2d(h, h->fan[6], frontier, n_frontier));
    const uint32_t* d_row_off = (const uint32_t*)h->fan[4].p;
    const uint32_t* d_dst = (const uint32_t*)h->fan[5].p;
    const uint32_t* d_front = (const uint32_t*)h->fan[6].p;
    uint64_t total = 0;
    GD_TRY(fan_count(h, d_row_off, n_nodes, d_front, n_frontier, &total));
    *out_n = total;
    if (total > capacity)
        return set_err(h, GD_EINVAL, "fan-out emits %llu messages, output holds %llu", (unsigned long long)total,
                       (unsigned long long)capacity);
    const size_t n = (size_t)total;
    // message outputs: target, sender, silo, act (4 x u32), status (u8), perm (u32)
    GD_TRY(ensure(h, h->fan[7], n * 21 + 64));
    uint32_t* d_target = (uint32_t*)h->fan[7].p;
    uint32_t* d_sender = d_target + n;
    uint32_t* d_silo = d_sender + n;
    uint32_t* d_act = d_silo + n;
    uint32_t* d_perm = d_act + n;
    uint8_t* d_status = (uint8_t*)(d_perm + n);
    if (out_perm) GD_TRY(ensure(h, h->offs, ((size_t)n_act + 2) * 4));
    if (n)
        GD_TRY(fan_route(h, d_row_off, d_dst, d_front, n_frontier, (uint32_t)n, grain_tcd(type_code), d_target,
                         d_sender, d_silo, d_act, d_status));
    if (out_perm) GD_TRY(bucket_device(h, d_act, (uint32_t)n, n_act, d_perm, (uint32_t*)h->offs.p));
    auto get = [&](void* dstp, const void* src, size_t bytes) -> int {
        if (dstp && bytes) HIP_TRY(h, hipMemcpyAsync(dstp, src, bytes, hipMemcpyDeviceToHost, h->stream));
        return GD_OK;
    };
    GD_TRY(get(out_target, d_target, n * 4));
    GD_TRY(get(out_sender, d_sender, n * 4));
    GD_TRY(get(out_silo, d_silo, n * 4));
    GD_TRY(get(out_act, d_act, n * 4));
    GD_TRY(get(out_status, d_status, n));
    if (out_perm) {
        GD_TRY(get(out_perm, d_perm, n * 4));
        GD_TRY(d2h(h, out_offsets, h->offs, (size_t)n_act + 2));
    }
    return sync_checked(h);
}

int gd_route_nodes_device(gd_handle* h, const uint32_t* d_nodes, uint32_t n, int32_t type_code, uint32_t* d_silo,
                          uint32_t* d_act, uint8_t* d_status) {
    if (!h || (n && (!d_nodes || !d_silo || !d_act || !d_status))) return set_err(h, GD_EINVAL, "null argument");
    return n ? route_nodes(h, d_nodes, n, grain_tcd(type_code), d_silo, d_act, d_status) : GD_OK;
}

int gd_pack_nodes_by_shard_device(gd_handle* h, const uint32_t* d_nodes, const uint32_t* d_payload, uint32_t n,
                                  int32_t type_code, uint32_t n_shards, uint32_t* d_send_nodes,
                                  uint32_t* d_send_payload, uint32_t* d_counts) {
    if (!h || !d_counts || (n && (!d_nodes || !d_payload || !d_send_nodes || !d_send_payload)))
        return set_err(h, GD_EINVAL, "null argument");
    if (n_shards == 0 || n_shards > 256) return set_err(h, GD_EINVAL, "n_shards %u not in [1, 256]", n_shards);
    return shard_pack<true>(h, d_nodes, d_payload, n, grain_tcd(type_code), n_shards, d_send_nodes, d_send_payload,
                            d_counts);
}

int gd_frontier_next_device(gd_handle* h, const uint32_t* d_offsets, uint32_t n_act, uint8_t* d_visited,
                            uint32_t* d_out, uint32_t* out_n) {
    if (!h || !out_n || (n_act && (!d_offsets || !d_visited || !d_out))) return set_err(h, GD_EINVAL, "null argument");
    HIP_TRY(h, hipSetDevice(h->device));
    return frontier_next(h, d_offsets, n_act, d_visited, d_out, out_n);
}

}  // extern "C"

// ================================================================== sharded fan-out cascade (SURVEY 8 f2 + 8 e)
// BASELINE cfg 4 across GPUs: ChirperAccount.PublishMessage (ChirperAccount.cs:106-147) on every
// rank for the publishers it owns; each NewChirp goes to its follower's directory owner over the
// library's communicator (OutboundMessageQueue.cs:54-131 per target silo), is routed there and
// enqueued on the follower's activation in arrival order (sender rank, sender emission order).
namespace gdx {

// counts[W] (device, this rank's sends per peer) -> host send / receive counts; one grouped round.
int counts_round(gd_handle* h, uint32_t* dcnt, std::vector<uint32_t>& sc, std::vector<uint32_t>& rc) {
    const int W = h->n_ranks;
    const Rccl& R = *h->net;
    NCCL_TRY(h, R.GroupStart());
    for (int r = 0; r < W; ++r) {
        NCCL_TRY(h, R.Send(dcnt + r, 1, ncclUint32, r, h->comm, h->stream));
        NCCL_TRY(h, R.Recv(dcnt + W + r, 1, ncclUint32, r, h->comm, h->stream));
    }
    NCCL_TRY(h, R.GroupEnd());
    uint32_t* hc = h->h_xcnt + 11 * 256;
    HIP_TRY(h, hipMemcpyAsync(hc, dcnt, (size_t)W * 8, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    ncclResult_t async_err = ncclSuccess;
    NCCL_TRY(h, R.CommGetAsyncError(h->comm, &async_err));
    if (async_err != ncclSuccess) return set_err(h, GD_ERCCL, "RCCL async error: %s", R.GetErrorString(async_err));
    sc.assign(hc, hc + W);
    rc.assign(hc + W, hc + 2 * W);
    return GD_OK;
}

// node_of == nullptr: the replicated graph (rows = node ids = activation indices, n_nodes rows).
// node_of != nullptr: this rank's partition of the graph -- row i = local activation i, whose node
// is node_of[i] (n_nodes = n_act rows); publishers are rows, messages still carry node ids.
int fanout_multi(gd_handle* h, const uint32_t* row_off, const uint32_t* dst, uint32_t n_nodes, const uint32_t* seeds,
                 uint32_t n_seeds, int32_t type_code, uint32_t n_act, uint32_t hops, gd_fanout_hop* out,
                 const uint32_t* node_of = nullptr) {
    GD_TRY(need_comm(h));
    GD_TRY(check_ring(h));
    if (n_act == 0xFFFFFFFFu) return set_err(h, GD_EINVAL, "n_act too large");
    const int W = h->n_ranks;
    const uint64_t tcd = grain_tcd(type_code);
    GD_TRY(sync(h));                                   // the previous call's results may be in use
    if (h->fm_hop.size() < hops) h->fm_hop.resize(hops);
    h->fm_res.assign(hops, gd_fanout_hop{});
    h->fm_n_act = n_act;
    DevBuf* S = h->fm_scr;
    GD_TRY(ensure(h, S[4], (size_t)W * 8 + 16));
    GD_TRY(ensure(h, S[5], (size_t)n_act + 16));
    uint32_t* dcnt = (uint32_t*)S[4].p;
    uint8_t* visited = (uint8_t*)S[5].p;
    HIP_TRY(h, hipMemsetAsync(visited, 0, (size_t)n_act + 16, h->stream));
    // hop 0's publishers: the seeds this rank owns, in seed order (a stable partition of the seeds by
    // owner rank, then this rank's chunk)
    uint32_t nf = 0, seed_fail = 0;
    {
        std::array<DevBuf, 10>& H0 = h->fm_hop[0];
        GD_TRY(ensure(h, S[0], (size_t)n_seeds * 4 + 16));
        GD_TRY(ensure(h, S[1], (size_t)n_seeds * 4 + 16));
        GD_TRY(shard_pack<true>(h, seeds, seeds, n_seeds, tcd, (uint32_t)W, S[0].p, (uint32_t*)S[1].p, dcnt));
        uint32_t* hc = h->h_xcnt + 11 * 256;
        HIP_TRY(h, hipMemcpyAsync(hc, dcnt, (size_t)W * 4, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(h, hipStreamSynchronize(h->stream));
        uint64_t lo = 0;
        for (int r = 0; r < h->rank; ++r) lo += hc[r];
        nf = hc[h->rank];
        GD_TRY(ensure(h, H0[0], ((size_t)std::max(nf, n_act) + 4) * 4));
        if (nf && !node_of) {
            HIP_TRY(h, hipMemcpyAsync(H0[0].p, (const uint32_t*)S[0].p + lo, (size_t)nf * 4, hipMemcpyDeviceToDevice,
                                      h->stream));
            GD_TRY(launch(h, "k_mark_visited", dim3(blocks_for(nf, BLOCK)), dim3(BLOCK), 0, k_mark_visited,
                          (const uint32_t*)H0[0].p, nf, n_act, visited));
        } else if (nf) {
            // partitioned: the owned seeds' nodes (the hop's frontier as reported), their rows by the
            // directory probe (every seed must have a live activation on its owner)
            GD_TRY(ensure(h, H0[9], ((size_t)std::max(nf, n_act) + 4) * 4));
            GD_TRY(ensure(h, S[2], (size_t)nf * 4 + 16));
            GD_TRY(ensure(h, S[3], (size_t)nf * 5 + 16));
            uint32_t* nodes = (uint32_t*)H0[9].p;
            HIP_TRY(h, hipMemcpyAsync(nodes, (const uint32_t*)S[0].p + lo, (size_t)nf * 4, hipMemcpyDeviceToDevice,
                                      h->stream));
            uint32_t* acts = (uint32_t*)S[2].p;
            uint8_t* sts = (uint8_t*)S[3].p + (size_t)nf * 4;
            GD_TRY(route_nodes(h, nodes, nf, tcd, (uint32_t*)S[3].p, acts, sts));
            HIP_TRY(h, hipMemsetAsync(dcnt + 2 * W, 0, 4, h->stream));
            GD_TRY(launch(h, "k_seed_rows", dim3(blocks_for(nf, BLOCK)), dim3(BLOCK), 0, k_seed_rows, (const uint32_t*)acts,
                          (const uint8_t*)sts, nf, n_act, (uint32_t*)H0[0].p, dcnt + 2 * W));
            HIP_TRY(h, hipMemcpyAsync(hc, dcnt + 2 * W, 4, hipMemcpyDeviceToHost, h->stream));
            HIP_TRY(h, hipStreamSynchronize(h->stream));
            // a seed without a live activation fails the whole cascade on every rank: this rank goes on
            // with no publishers and flags its hop-0 counts (below), so no peer waits in a later round
            seed_fail = hc[0];
            if (seed_fail) nf = 0;
            else
                GD_TRY(launch(h, "k_mark_visited", dim3(blocks_for(nf, BLOCK)), dim3(BLOCK), 0, k_mark_visited,
                              (const uint32_t*)H0[0].p, nf, n_act, visited));
        }
    }
    uint64_t total = 0;
    for (uint32_t hp = 0; hp < hops; ++hp) {
        std::array<DevBuf, 10>& H = h->fm_hop[hp];
        const uint32_t* frontier = (const uint32_t*)H[0].p;
        gd_fanout_hop& res = h->fm_res[hp];
        res.n_frontier = nf;
        res.frontier = frontier;
        if (node_of) {                 // reported as nodes: hop 0's seeds are there already
            if (hp > 0) {
                GD_TRY(ensure(h, H[9], ((size_t)n_act + 4) * 4));
                if (nf)
                    GD_TRY(launch(h, "k_gather_u32", dim3(blocks_for(nf, BLOCK)), dim3(BLOCK), 0, k_gather_u32, frontier,
                                  nf, node_of, (uint32_t*)H[9].p));
            }
            res.frontier = (const uint32_t*)H[9].p;
        }
        // 1. expand this rank's publishers (follower lists in enumeration order); hop 0 counts here,
        //    later hops were counted with the previous hop's frontier (one read-back for both)
        if (hp == 0) GD_TRY(fan_count(h, row_off, n_nodes, frontier, nf, &total));
        const uint32_t n = (uint32_t)total;
        res.n_sent = total;
        GD_TRY(ensure(h, S[0], (size_t)n * 4 + 16));
        GD_TRY(ensure(h, S[1], (size_t)n * 4 + 16));
        GD_TRY(ensure(h, S[2], (size_t)n * 4 + 16));
        GD_TRY(ensure(h, S[3], (size_t)n * 4 + 16));
        if (n)
            GD_TRY(launch(h, "k_fan_expand", dim3(blocks_for(n, FAN_TILE)), dim3(BLOCK), 0, k_fan_expand, row_off,
                          dst, frontier, nf, (const uint32_t*)h->fan[0].p, n, (uint32_t*)S[0].p, (uint32_t*)S[1].p,
                          node_of));
        // 2. stable partition of (target, sender) by the target's owner rank
        GD_TRY(shard_pack<true>(h, S[0].p, (const uint32_t*)S[1].p, n, tcd, (uint32_t)W, S[2].p, (uint32_t*)S[3].p,
                                dcnt));
        // 3. counts, then one grouped round of 8 B a message.  Hop 0's counts carry a failed seed
        //    resolution to every peer (all ones: no real count, at most 2^32 - 2 messages a hop), and
        //    every rank returns the error after this same round
        if (hp == 0 && seed_fail) HIP_TRY(h, hipMemsetAsync(dcnt, 0xFF, (size_t)W * 4, h->stream));
        std::vector<uint32_t> sc, rc;
        GD_TRY(counts_round(h, dcnt, sc, rc));
        if (hp == 0) {
            for (int r = 0; r < W; ++r)
                if (rc[r] == 0xFFFFFFFFu)
                    return set_err(h, GD_EINVAL, "rank %d: %s seeds have no live activation on their owner (a "
                                   "partitioned graph's rows are activations)", r,
                                   r == h->rank ? std::to_string(seed_fail).c_str() : "some");
        }
        std::vector<uint64_t> soff(W + 1, 0), roff(W + 1, 0);
        for (int r = 0; r < W; ++r) {
            soff[r + 1] = soff[r] + sc[r];
            roff[r + 1] = roff[r] + rc[r];
        }
        if (soff[W] != n)
            return set_err(h, GD_ERCCL, "fan-out partition counts sum to %llu, hop emitted %u",
                           (unsigned long long)soff[W], n);
        if (roff[W] >= 0xFFFFFFFFull)
            return set_err(h, GD_EINVAL, "%llu messages received in one hop", (unsigned long long)roff[W]);
        const uint32_t m = (uint32_t)roff[W];
        const size_t m4 = (size_t)m * 4 + 16;
        const size_t want[10] = {0, m4, m4, m4, m4, m4, (size_t)m + 16, m4, ((size_t)n_act + 2) * 4, 0};
        for (int b = 1; b < 9; ++b) GD_TRY(ensure(h, H[b], want[b]));
        uint32_t* target = (uint32_t*)H[1].p;
        uint32_t* sender = (uint32_t*)H[2].p;
        uint32_t* src = (uint32_t*)H[3].p;
        uint32_t* silo = (uint32_t*)H[4].p;
        uint32_t* act = (uint32_t*)H[5].p;
        uint8_t* st = (uint8_t*)H[6].p;
        uint32_t* perm = (uint32_t*)H[7].p;
        uint32_t* offs = (uint32_t*)H[8].p;
        const Lane lanes[2] = {{S[2].p, target, 4, ncclUint32, 1}, {S[3].p, sender, 4, ncclUint32, 1}};
        GD_TRY(exchange_round(h, "rccl_fanout", sc.data(), soff.data(), rc.data(), roff.data(), lanes, 2));
        if (m)
            GD_TRY(launch(h, "k_recv_src", dim3(blocks_for(m, BLOCK)), dim3(BLOCK), 0, k_recv_src,
                          (const uint32_t*)(dcnt + W), (uint32_t)W, m, src));
        // 4. route + bucket on the owner
        if (m) GD_TRY(route_nodes(h, target, m, tcd, silo, act, st));
        GD_TRY(bucket_device(h, act, m, n_act, perm, offs));
        res.n_recv = m;
        res.target = target;
        res.sender = sender;
        res.src = src;
        res.silo = silo;
        res.act = act;
        res.status = st;
        res.perm = perm;
        res.offsets = offs;
        // 5. the next publishers: this rank's activations that got a chirp and have not published; their
        //    count stays on the device until the next hop's degree scan reads it back with its total
        if (hp + 1 < hops) {
            std::array<DevBuf, 10>& N = h->fm_hop[hp + 1];
            GD_TRY(ensure(h, N[0], ((size_t)n_act + 4) * 4));
            const uint32_t* d_nf = nullptr;
            GD_TRY(frontier_next_dev(h, offs, n_act, visited, (uint32_t*)N[0].p, &d_nf));
            // every new publisher received at least one of this hop's m messages: the scan's bound
            GD_TRY(fan_count_dev(h, row_off, n_nodes, (const uint32_t*)N[0].p, d_nf, std::min(n_act, m), &nf,
                                 &total));
        }
    }
    if (out) std::copy(h->fm_res.begin(), h->fm_res.end(), out);
    return GD_OK;
}

}  // namespace gdx

extern "C" {

int gd_fanout_multi_device(gd_handle* h, const uint32_t* d_row_off, const uint32_t* d_dst, uint32_t n_nodes,
                           const uint32_t* d_seeds, uint32_t n_seeds, int32_t type_code, uint32_t n_act, uint32_t hops,
                           gd_fanout_hop* out) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    if (n_seeds && !d_seeds) return set_err(h, GD_EINVAL, "null seeds");
    if (!d_row_off || (!d_dst && n_nodes)) return set_err(h, GD_EINVAL, "null graph");
    if (hops == 0 || hops > 64) return set_err(h, GD_EINVAL, "hops %u not in [1, 64]", hops);
    HIP_TRY(h, hipSetDevice(h->device));
    return fanout_multi(h, d_row_off, d_dst, n_nodes, d_seeds, n_seeds, type_code, n_act, hops, out);
}

int gd_fanout_multi_part_device(gd_handle* h, const uint32_t* d_row_off, const uint32_t* d_dst, uint32_t n_rows,
                                const uint32_t* d_node_of, const uint32_t* d_seeds, uint32_t n_seeds,
                                int32_t type_code, uint32_t hops, gd_fanout_hop* out) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    if (n_seeds && !d_seeds) return set_err(h, GD_EINVAL, "null seeds");
    if (!d_row_off || (n_rows && (!d_dst || !d_node_of))) return set_err(h, GD_EINVAL, "null graph");
    if (hops == 0 || hops > 64) return set_err(h, GD_EINVAL, "hops %u not in [1, 64]", hops);
    HIP_TRY(h, hipSetDevice(h->device));
    // an empty partition still needs a non-null node_of to select the partitioned form
    return fanout_multi(h, d_row_off, d_dst, n_rows, d_seeds, n_seeds, type_code, n_rows, hops, out,
                        d_node_of ? d_node_of : d_row_off);
}

int gd_fanout_multi(gd_handle* h, const uint32_t* row_off, const uint32_t* dst, uint32_t n_nodes,
                    const uint32_t* seeds, uint32_t n_seeds, int32_t type_code, uint32_t n_act, uint32_t hops,
                    gd_fanout_hop* out) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    if (!row_off || (n_seeds && !seeds)) return set_err(h, GD_EINVAL, "null argument");
    if (hops == 0 || hops > 64) return set_err(h, GD_EINVAL, "hops %u not in [1, 64]", hops);
    HIP_TRY(h, hipSetDevice(h->device));
    const uint64_t edges = row_off[n_nodes];
    if (edges && !dst) return set_err(h, GD_EINVAL, "null graph");
    GD_TRY(h2d(h, h->fm_graph[0], row_off, (size_t)n_nodes + 1));
    GD_TRY(h2d(h, h->fm_graph[1], dst ? dst : row_off, edges ? edges : 1));
    GD_TRY(h2d(h, h->fm_graph[2], seeds ? seeds : row_off, n_seeds ? n_seeds : 1));
    GD_TRY(fanout_multi(h, (const uint32_t*)h->fm_graph[0].p, (const uint32_t*)h->fm_graph[1].p, n_nodes,
                        (const uint32_t*)h->fm_graph[2].p, n_seeds, type_code, n_act, hops, out));
    return sync_checked(h);
}

int gd_fanout_multi_fetch(gd_handle* h, uint32_t hop, uint32_t* frontier, uint32_t* target, uint32_t* sender,
                          uint32_t* src, uint32_t* silo, uint32_t* act, uint8_t* status, uint32_t* perm,
                          uint32_t* offsets) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    if (hop >= h->fm_res.size()) return set_err(h, GD_ESTATE, "no hop %u in the last gd_fanout_multi* result", hop);
    HIP_TRY(h, hipSetDevice(h->device));
    const gd_fanout_hop& r = h->fm_res[hop];
    const size_t m = r.n_recv;
    auto cp = [&](void* d, const void* s, size_t bytes) -> int {
        if (d && bytes) HIP_TRY(h, hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToHost, h->stream));
        return GD_OK;
    };
    GD_TRY(cp(frontier, r.frontier, (size_t)r.n_frontier * 4));
    GD_TRY(cp(target, r.target, m * 4));
    GD_TRY(cp(sender, r.sender, m * 4));
    if (r.src) GD_TRY(cp(src, r.src, m * 4));
    else if (src) std::memset(src, 0, m * 4);           // the one-GPU cascade: every message is this rank's
    GD_TRY(cp(silo, r.silo, m * 4));
    GD_TRY(cp(act, r.act, m * 4));
    GD_TRY(cp(status, r.status, m));
    GD_TRY(cp(perm, r.perm, m * 4));
    GD_TRY(cp(offsets, r.offsets, ((size_t)h->fm_n_act + 2) * 4));
    return sync(h);
}

}  // extern "C"
