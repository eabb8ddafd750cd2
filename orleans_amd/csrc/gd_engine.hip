// gd_engine.hip -- handle, scratch management and the C ABI of libgraindispatch
// (declared in include/graindispatch.h).  Kernels live in gd_kernels.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <queue>
#include <map>
#include <unordered_map>
#include <string>
#include <vector>

#include "gd_common.h"
#include "gd_churn.h"
#include "gd_fanout.h"
#include "gd_cache.h"
#include "gd_cx.h"
#include "gd_msd.h"
#include "gd_msd2.h"
#include "gd_shard.h"
#include "gd_comm.h"
#include "gd_localcomm.h"
#include "gd_keyext.h"
#include "gd_frames.h"
#include "gd_dirops.h"
#include "gd_actdir.h"
#include "gd_bucket2.h"
#include "graindispatch.h"

using namespace gd;

namespace {

thread_local std::string g_tls_error = "";

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

struct TimedLaunch {
    int name;
    hipEvent_t a, b;
};

}  // namespace

struct gd_handle {
    gd_config cfg{};
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    // host-pointer entry points, large batches: copy-in / copy-out streams and their events
    hipStream_t cin = nullptr, cout = nullptr;
    std::vector<hipEvent_t> hp_ev;
    uint32_t host_chunk = 1u << 21;   // messages per pipelined chunk (GD_HOST_CHUNK; 0: no pipelining)
    std::string err;

    // ring snapshot
    int ring_mode = -1;
    uint32_t ring_n = 0, ring_top = 0;
    uint64_t layout_gen = 0;          // bumped whenever ring / table pointers or sizes change
                                      // (captured micro-batch graphs bake them in)
    DevBuf ring_pts, ring_own;

    // directory table
    Slot* slots = nullptr;
    unsigned long long capacity = 0;
    DevCounters* ctr = nullptr;       // device
    DevCounters ctr_host{};           // last copy

    // scratch
    DevBuf keys_in, u32_a, u32_b, u32_c, u32_d, u8_a, out_a, out_b, out_c, hist, partials, partials2, offs;
    DevBuf fr[16];                    // header-decode scratch (host-pointer entry points)
    DevBuf fr_ext[2];                 // TargetGrain KeyExt offsets / lengths (gd_route_frames_ext*)
    DevBuf churn[5];                  // split scratch: keep mask, flags, positions, out keys/vals
    DevBuf fan[8];                    // fan-out scratch: ends, total, flags, positions, host-form buffers

    // non-owner directory cache (LocalLookup mode when cache_max > 0)
    CacheSlot* cslots = nullptr;
    unsigned long long ccap = 0;
    CacheCounters* cctr = nullptr;   // device
    DevBuf cx_heap;                  // KeyExt strings of the cache's KeyExt entries (16-B aligned)
    uint64_t cx_used = 0;            // bytes of cx_heap handed out (compacted when it runs out)
    uint32_t cache_max = 0;
    uint32_t cache_nsilos = 0;
    DevBuf cache_local, cache_valid;
    DevBuf cbuf[8];                   // cache scratch
    DevBuf shard_dest, shard_hist;    // exchange partition scratch
    DevBuf shard_n1;                  // low N1 words of the batch (k_shard_hist -> k_shard_gather, compact u32)
    bool shard_n1_copy = true;        // GD_SHARD_N1=0: the gather reads N1 from the 24-B keys
    DevBuf up_last;                   // gd_dir_upsert: last batch item per table slot (zero between calls)

    // IsValidSilo (gd_dir_set_valid_silos): bitset over silo indices [0, n_valid); VersionTag and
    // GrainInfo.SingleInstance per slot (gd_dirops.h); dir_op numbers the mutating directory calls
    DevBuf dir_valid;
    uint32_t n_valid = 0;
    std::vector<uint8_t> valid_host;
    uint32_t* vtag = nullptr;
    uint32_t dir_op = 0;
    DevBuf act_ids;                   // ActivationId per host activation index (gd_activation_ids_set)
    uint64_t n_act_ids = 0;
    DevBuf dirop_buf[4];

    // ActivationDirectory of the receive path (gd_actdir.h): ActivationId -> context, flags
    Slot* ad_slots = nullptr;
    unsigned long long ad_cap = 0;
    DevCounters* ad_ctr = nullptr;
    DevCounters ad_host{};
    DevBuf ad_last;
    DevBuf ad_buf[8];
    DevBuf fr_recv[3];                // frames: TargetActivation / Direction scratch when the caller wants neither
    DevBuf recv_scr[2];               // receive with limits but no buckets wanted: perm / offsets scratch

    // KeyExt grains (gd_keyext.h): device table + heap, and the host index both are kept from
    KxSlot* kx_slots = nullptr;
    uint64_t kx_cap = 0;
    DevBuf kx_heap;
    uint64_t kx_heap_dev = 0;          // host heap bytes already on the device
    std::vector<KxSlot> kx_m;          // host index (same layout as the device table)
    std::vector<uint8_t> kx_hheap;
    uint64_t kx_live = 0, kx_tomb = 0;
    uint32_t kx_maxp = 0;
    DevBuf kx_buf[5];                  // apply / ext staging scratch

    // in-library exchange over RCCL (gd_comm.h): one communicator per handle.  The partition and
    // the RCCL rounds run on xstream; probe + bucketing on `stream`; batch i's exchange overlaps
    // batch i-1's probe + bucketing (receive/result buffers double-buffered by batch parity).
    ncclComm_t comm = nullptr;
    const Rccl* net = nullptr;        // the transport behind comm: RCCL, or the in-process one
    int n_ranks = 0, rank = -1;
    hipStream_t xstream = nullptr;
    hipStream_t pstream = nullptr;    // the partition (pack) of the next batch, beside this one's rounds
    hipEvent_t x_in = nullptr, x_hdr[2] = {}, x_route[2] = {}, x_ret[2] = {}, x_done[2] = {};
    hipEvent_t p_packed = nullptr, x_sent[2] = {}, x_fwd[2] = {}, x_keys[2] = {};
    bool x_done_rec[2] = {false, false}, x_sent_rec[2] = {false, false};
    DevBuf mx_send[2][7];             // per batch parity: send keys, send idx, counts (send/recv messages,
                                      // send/recv KeyExt bytes: 4 x [W]), KeyExt lengths, KeyExt byte
                                      // offsets, KeyExt blob, block starts of 2-B origin indices
    DevBuf mx[2][22];                 // per batch parity: receive / result buffers
    DevBuf mf[2][17];                 // per batch parity, GD_MULTI_FORWARD: forward send (keys, pos, idx,
                                      // src, silo, act, status, counts), forward receive (keys, idx, src,
                                      // silo, act, status), perm, offsets, compact key staging
    DevBuf mx_keys;                   // host-keys entry point: the batch, on xstream
    DevBuf mx_ext[3];                 // host-keys entry point: its KeyExt blob, offsets, lengths
    DevBuf x_scratch[4];              // xstream's own scan partials + partition scratch
    DevBuf p_scratch[4];              // pstream's
    uint32_t* h_xcnt = nullptr;       // pinned: send/recv message counts, send/recv KeyExt byte counts,
                                      // key descriptors (mine, every peer's), forward counts (12 x 256)
    gd_multi_result mres[2] = {};
    // sharded fan-out cascade (gd_fanout_multi_device): per hop the frontier and the owner-side
    // results, kept for the caller; shared expansion / partition scratch
    std::vector<std::array<DevBuf, 10>> fm_hop;
    std::vector<gd_fanout_hop> fm_res;
    uint32_t fm_n_act = 0;
    DevBuf fm_scr[6];                 // expand target / sender, partitioned target / sender, counts, visited
    DevBuf fm_graph[3];               // host-form entry point: row_off, dst, seeds
    // multi-rank directory handoff (gd_dir_handoff_multi): split / send scratch, received entries
    DevBuf ho_send[10];
    DevBuf ho_recv[11];
    gd_handoff_result ho_res{};
    bool ho_valid = false;
    uint32_t mres_n[2] = {0, 0};
    uint64_t mcalls = 0;
    uint64_t routed = 0;

    // kernel tuning (defaults measured on MI355X; GD_ROUTE_M / GD_ROUTE_NT override for A/B runs)
    bool route_xcd = true;      // route workgroups over XCD-contiguous message ranges (GD_ROUTE_XCD)
    // compact probe index (gd_cx.h): derived from the table, rebuilt after any change of it (GD_CX=0: off)
    int cx_mode = 1;            // 0 off, 1 measured (default), 2 index group reads, 3 index slot reads (GD_CX)
    bool mb_zero_copy = true;   // micro-batches: I/O from / to pinned host memory (GD_OPT_MB_ZEROCOPY)
    uint32_t mb_split = 8;      // micro-batches: redundant sorters splitting the host stores (GD_OPT_MB_SPLIT)
    bool mb_trace = false;      // micro-batches: per-phase timestamps (GD_OPT_MB_TRACE)
    int tune_pin[GD_TUNE_KINDS] = {-1, -1, -1, -1, -1};   // gd_tune_set: pinned variant per kind, -1 measured
    int msd_mode = 1;           // two-level bucketing (gd_msd.h, gd_msd2.h): 0 off, 1 measured (default), 2 always (GD_MSD)
    uint32_t l2_small = 1024;   // three-pass form: ranges of at most this many messages are sorted one wave a range
    uint32_t l2_mid = MSD_MID_CAP;  // three-pass form: staged ranges up to this many messages on the 512-thread sort
    uint32_t l2_staged = MSD_CAP;  // three-pass form: ranges up to this many messages one workgroup each, more: chunks
    uint32_t n_cu = 256;        // compute units (hipDeviceProp_t::multiProcessorCount): persistent grids
    DevBuf m3[15];              // three-pass form's scratch (msd3_bucket)
    DevBuf tune_buf;            // gd_tune_agree's send / receive records
    uint32_t cx_scale = 1;      // index slots = cx_scale x table capacity (GD_CX_SCALE, 1 or 2)
    // per launch kind and size class: the probe variant, timed on live launches.  Variants: 0 the index
    // in 64-B group reads, 1 the directory, 2 the index in 16-B slot reads, 3 the 8-B index (24-B keys)
    static constexpr int CXV = 4;
    struct CxTune {
        int pick = -1;          // -1 measuring, else the variant
        int round = 0;
        int nvar = 0;           // the variants this entry measures (the 8-B index only where it is built)
        float best[CXV] = {1e30f, 1e30f, 1e30f, 1e30f};
        hipEvent_t a[CXV] = {}, b[CXV] = {};
        bool pending[CXV] = {};
        uint64_t n[CXV] = {};
    };
    std::map<int, CxTune> cx_tune;   // key: (kind * 64 + size class (bit length of n)) * 32 + a second class
    uint64_t tab_gen = 0;       // bumped by every launch that takes the table as a writable Slot*
    bool cx_built = false, cx_ok = false;
    const Slot* cx_slots_at = nullptr;
    uint64_t cx_cap_at = 0, cx_gen_at = 0;
    uint32_t cx_rounds = 0;
    DevBuf cxi_tab, cxi_types, cxi_ctr;
    bool cx8_ok = false;        // the 8-B index (gd_cx.h k_cx8_build) is built and current with cx
    uint32_t cx8_rounds = 0, cx8_ab = 24;
    uint64_t cx8_tcd = 0;
    DevBuf cx8_tab;
    uint32_t xcd_tiles = 1;     // XCD-contiguous tile ranges in the radix scatter (GD_XCD_TILES)
    bool hist_xcd = true;       // multi-tile histograms in reverse XCD tile order (GD_HIST_XCD)
    bool compact_headers = true;    // 8-B exchange headers for uniform batches (GD_COMPACT_HEADERS=0: off)
    bool region_probe = false;      // gd_route_multi: chunks ordered by table region, region-mapped probe (GD_REGION_PROBE)
    bool idx16 = true;              // gd_route_multi: 2-B origin indices on the wire (KD_IDX16, GD_IDX16)
    bool pack_pay16 = false;        // set by route_multi around its partition: the scatter writes u16 payloads
    bool narrow_headers = true;     // compact headers as u32 N1s when every N1 < 2^32 (GD_NARROW_HEADERS=0: u64)
    bool shard_gather = true;   // exchange partition of keys: k_shard_gather (GD_SHARD_GATHER=0: k_shard_scatter, staged keys)
    const uint32_t* last_totals = nullptr;   // the last radix pass's digit totals (row scans), and their count
    uint32_t last_digits = 0;
    uint32_t radix_rank_atomic = 1;   // stable in-wave rank by ds_add_rtn (1, A/B: ab_bucket.py) or ballots (0)
    bool lane_order = true;           // gd_create's k_lane_order_check passed (else every rank by ballots)
    bool lane_order_forced_off = false;   // GD_CFG_NO_LANE_ORDER: behave as on a device without it (tests)

    // pinned host scratch for small device -> host read-backs (counts, totals)
    void* h_pin = nullptr;
    size_t h_pin_bytes = 0;

    // per-kernel timing
    bool timing = false;
    std::vector<std::string> tnames;
    std::vector<double> tms;
    std::vector<uint64_t> tcount;
    std::vector<TimedLaunch> pending;
    std::vector<hipEvent_t> event_pool;
};

namespace {

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

#define HIP_TRY(h, expr)                                                                    \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return set_err((h), GD_EHIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
    } while (0)

#define GD_TRY(expr)              \
    do {                          \
        int r_ = (expr);          \
        if (r_ != GD_OK) return r_; \
    } while (0)

int ensure(gd_handle* h, DevBuf& b, size_t bytes) {
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

// A launch argument that is the directory table as a writable Slot* (the kernel may change it).
template <typename T>
bool writes_table(const gd_handle*, const T&) { return false; }
bool writes_table(const gd_handle* h, Slot* p) { return p != nullptr && p == h->slots; }

// Launch a kernel on the handle's stream; with GD_CFG_KERNEL_TIMING bracket it by events.  A kernel
// handed the table as a writable Slot* invalidates the compact probe index (tab_gen).
template <typename K, typename... Args>
int launch(gd_handle* h, const char* name, dim3 grid, dim3 block, size_t lds, K kernel, Args... args) {
    if (grid.x == 0) return GD_OK;
    if ((writes_table(h, args) || ...)) h->tab_gen++;
    hipEvent_t a = nullptr, b = nullptr;
    if (h->timing) {
        a = take_event(h);
        b = take_event(h);
        HIP_TRY(h, hipEventRecord(a, h->stream));
    }
    hipLaunchKernelGGL(kernel, grid, block, lds, h->stream, args...);
    HIP_TRY(h, hipGetLastError());
    if (h->timing) {
        HIP_TRY(h, hipEventRecord(b, h->stream));
        h->pending.push_back(TimedLaunch{name_id(h, name), a, b});
    }
    return GD_OK;
}

int resolve_timing(gd_handle* h) {
    if (h->pending.empty()) return GD_OK;
    HIP_TRY(h, hipStreamSynchronize(h->stream));
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

inline uint32_t blocks_for(uint64_t n, uint32_t per) { return (uint32_t)((n + per - 1) / per); }

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

int pull_counters(gd_handle* h) {
    HIP_TRY(h, hipMemcpyAsync(&h->ctr_host, h->ctr, sizeof(DevCounters), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
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

// ---- compact probe index (gd_cx.h) ----------------------------------------------
// The index for the current table: rebuilt (two passes + one host sync) when the table changed since
// the last build; false when the table is not eligible (an N0 != 0 key, too many types) or GD_CX=0.
// n: the messages of the launch asking.  A stale index is rebuilt only for a launch of at least
// capacity / 16 messages: a small route after a directory write takes the directory probe instead of a
// full-table pass and a host sync; the next large launch rebuilds.
int cx_ensure(gd_handle* h, bool* ok, uint64_t n) {
    *ok = false;
    if (!h->cx_mode || !h->slots || h->capacity < CX_GROUP) return GD_OK;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;   // a captured graph keeps the directory probe
    HIP_TRY(h, hipStreamIsCapturing(h->stream, &cs));
    if (cs != hipStreamCaptureStatusNone) return GD_OK;
    if (h->cx_built && h->cx_slots_at == h->slots && h->cx_cap_at == h->capacity * h->cx_scale &&
        h->cx_gen_at == h->tab_gen) {
        *ok = h->cx_ok;
        return GD_OK;
    }
    if (h->cx_mode == 1 && n < h->capacity / 16) return GD_OK;
    const unsigned long long cap = h->capacity * h->cx_scale;
    GD_TRY(ensure(h, h->cxi_tab, cap * 16));
    GD_TRY(ensure(h, h->cxi_types, CX_TYPES * 8));
    GD_TRY(ensure(h, h->cxi_ctr, sizeof(CxCounters)));
    HIP_TRY(h, hipMemsetAsync(h->cxi_tab.p, 0, cap * 16, h->stream));
    HIP_TRY(h, hipMemsetAsync(h->cxi_types.p, 0xFF, CX_TYPES * 8, h->stream));
    HIP_TRY(h, hipMemsetAsync(h->cxi_ctr.p, 0, sizeof(CxCounters), h->stream));
    const dim3 g(blocks_for(h->capacity, BLOCK)), b(BLOCK);
    GD_TRY(launch(h, "k_cx_types", g, b, 0, k_cx_types, (const Slot*)h->slots, (unsigned long long)h->capacity,
                  (unsigned long long*)h->cxi_types.p, (CxCounters*)h->cxi_ctr.p));
    GD_TRY(launch(h, "k_cx_build", g, b, 0, k_cx_build, (const Slot*)h->slots, (unsigned long long)h->capacity,
                  (const unsigned long long*)h->cxi_types.p, (uint4*)h->cxi_tab.p, cap, (CxCounters*)h->cxi_ctr.p));
    CxCounters c{};
    unsigned long long types[CX_TYPES];
    HIP_TRY(h, hipMemcpyAsync(&c, h->cxi_ctr.p, sizeof c, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipMemcpyAsync(types, h->cxi_types.p, sizeof types, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    h->cx_built = true;
    h->cx_ok = c.flag == 0 && c.full == 0;
    // the 8-B index: one type, every N1 < 2^32, activation bits ab (all ones left for GD_ACT_MULTI) and
    // silo + 1 above them in a u32
    h->cx8_ok = false;
    uint32_t ntypes = 0;
    for (unsigned long long t : types)
        if (t != CX_NO_TYPE) {
            ++ntypes;
            h->cx8_tcd = t;
        }
    uint32_t ab = 1;
    while (ab < 32 && ((uint64_t)c.act_max + 1) >> ab) ++ab;          // act_max < 2^ab - 1
    const bool fits = ab < 32 && (((uint64_t)c.silo_max + 1) >> (32 - ab)) == 0;
    h->cx8_ab = ab;
    if (h->cx_ok && c.flag8 == 0 && ntypes == 1 && fits) {
        const unsigned long long cap8 = cap;           // as many 8-B slots as the 16-B index: half its bytes
        GD_TRY(ensure(h, h->cx8_tab, cap8 * 8));
        HIP_TRY(h, hipMemsetAsync(h->cx8_tab.p, 0, cap8 * 8, h->stream));
        GD_TRY(launch(h, "k_cx8_build", g, b, 0, k_cx8_build, (const Slot*)h->slots, (unsigned long long)h->capacity,
                      (unsigned long long*)h->cx8_tab.p, cap8, ab, (CxCounters*)h->cxi_ctr.p));
        HIP_TRY(h, hipMemcpyAsync(&c, h->cxi_ctr.p, sizeof c, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(h, hipStreamSynchronize(h->stream));
        h->cx8_ok = c.full8 == 0;
        h->cx8_rounds = c.max_rounds8;
    }
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
    h->cx_rounds = c.max_rounds;
    h->cx_slots_at = h->slots;
    h->cx_cap_at = cap;
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
int tune_choose(gd_handle* h, int kind, uint64_t n, int* meas, int nvar, int sub = 0) {
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
    }
    return v;
}

int cx_choose(gd_handle* h, int kind, uint64_t n, int* meas, int nvar = gd_handle::CXV) {
    *meas = -1;
    // variants: 0 index groups, 1 directory; kinds 0 / 1: 2 index slots, 3 the 8-B index; kinds 2 / 3:
    // 2 the 8-B index (when built: nvar says)
    if (h->cx_mode == 2) return 0;
    if (h->cx_mode == 3) return kind <= 1 && nvar > 2 ? 2 : 0;
    if (h->cx_mode == 4) return kind <= 1 ? (nvar > 3 ? 3 : 0) : ((kind == 2 || kind == 3) && nvar > 2 ? 2 : 0);
    return tune_choose(h, kind, n, meas, nvar);
}

// Brackets a launch chosen by cx_choose / tune_choose with the tune entry's events.
struct CxMeasure {
    gd_handle* h;
    int slot;
    uint64_t n;
    CxMeasure(gd_handle* hh, int sl, uint64_t nn) : h(hh), slot(sl), n(nn) {
        if (slot >= 0) (void)hipEventRecord(h->cx_tune[slot / gd_handle::CXV].a[slot % gd_handle::CXV], h->stream);
    }
    ~CxMeasure() {
        if (slot < 0) return;
        auto& t = h->cx_tune[slot / gd_handle::CXV];
        const int v = slot % gd_handle::CXV;
        (void)hipEventRecord(t.b[v], h->stream);
        t.n[v] = n;
        t.pending[v] = true;
    }
};

Cx8Args cx8_args(gd_handle* h) {
    return Cx8Args{(const uint4*)h->cx8_tab.p, h->capacity * h->cx_scale, h->cx8_tcd, h->cx8_rounds, h->cx8_ab};
}

CxArgs cx_args(gd_handle* h) {
    return CxArgs{(const uint4*)h->cxi_tab.p, h->capacity * h->cx_scale, (const unsigned long long*)h->cxi_types.p,
                  h->cx_rounds};
}

// ---- route -------------------------------------------------------------------
template <int MODE, int M, bool NT>
int route_launch(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t* silo, uint32_t* act, uint8_t* status) {
    bool cx = false;
    GD_TRY(cx_ensure(h, &cx, n));
    int meas = -1;
    const int var = cx ? cx_choose(h, 0, n, &meas, h->cx8_ok ? 4 : 3) : 1;
    CxMeasure m(h, meas, n);
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
                    uint32_t* act, uint8_t* status, const uint32_t* rcnt = nullptr, uint32_t world = 0,
                    uint32_t* src = nullptr) {
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

// One message a thread, plain (temporal) key reads: 2 a thread and non-temporal streams measured no
// faster (0.533 / 0.533-0.535 against 0.530-0.531 ms a cfg 2 step, profiles/r03_route_cx_ab.txt).
template <int MODE>
int route_mode(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t* silo, uint32_t* act, uint8_t* status) {
    return route_launch<MODE, 1, false>(h, keys, n, silo, act, status);
}

int route_cached(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t* silo, uint32_t* act, uint8_t* status,
                 bool touch);
int route_cached_keyext(gd_handle* h, const gd_key* keys, const ExtArgs& x, uint32_t n, uint32_t* silo, uint32_t* act,
                        uint8_t* st);

// touch = false (LocalLookup mode only): leave the batch's generation updates to the KeyExt pass
// that follows, so plain and KeyExt cache hits are numbered in one batch order.
int route_device(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t* silo, uint32_t* act, uint8_t* status,
                 bool touch = true) {
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
                uint32_t* out = nullptr) {
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
             uint32_t* v1, B2Pack pk = B2Pack{0, 0, 32}) {
    const uint32_t tiles = blocks_for(n, B2_TILE);
    const uint32_t hxr = h->hist_xcd && h->xcd_tiles ? 1u : 0u;
    GD_TRY(ensure(h, h->hist, ((size_t)R * tiles + R) * sizeof(uint32_t)));
    uint32_t* hist = (uint32_t*)h->hist.p;
    // 4 tiles a histogram workgroup from 1,024 tiles up (20.3 / 21.3 / 24.7 us at cfg 2 for 1 / 2 / 4,
    // profiles/r03_msd_htpb_ab.txt: 4 is the fastest; fewer tiles leave CUs idle)
    if (tiles >= 1024)
        GD_TRY(launch(h, "k_radix_hist", dim3(blocks_for(tiles, 4)), dim3(B2_NT), 0, k_b2_hist<B2_NT, B2_IT, 4, RMAX>,
                      acts, n, n_act, R, tiles, hist, shift, hxr));
    else
        GD_TRY(launch(h, "k_radix_hist", dim3(tiles), dim3(B2_NT), 0, k_b2_hist<B2_NT, B2_IT, 1, RMAX>, acts, n, n_act,
                      R, tiles, hist, shift, hxr));
    const uint32_t* tot = hist + (size_t)R * tiles;
    GD_TRY(launch(h, "k_radix_rowscan", dim3(R), dim3(BLOCK), 0, k_radix_rowscan, hist, tiles, hist + (size_t)R * tiles));
    GD_TRY(launch(h, "k_radix_scatter", dim3(tiles), dim3(B2_NT), 0, k_b2_scatter<B2_NT, B2_IT, RMAX, KOUT, BALLOT>, acts, n,
                  n_act, R, tiles, (const uint32_t*)hist, tot, k1, v1, shift, h->xcd_tiles, pk));
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
    const uint32_t R = (n_act >> MSD_SHIFT) + 1;
    if (R > MSD_MAX_RANGES) return set_err(h, GD_EINVAL, "two-level bucketing: n_act too large");
    GD_TRY(ensure(h, h->u32_a, (size_t)n * 4));
    GD_TRY(ensure(h, h->u32_c, (size_t)n * 4));
    uint32_t* k1 = (uint32_t*)h->u32_a.p;
    uint32_t* v1 = (uint32_t*)h->u32_c.p;
    GD_TRY((msd_pass<B2_RMAX2, B2_KEY16, BALLOT>(h, acts, n, n_act, R, MSD_SHIFT, k1, v1)));
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

int bucket_lsd(gd_handle* h, const uint32_t* acts, uint32_t n, uint32_t n_act, uint32_t* perm, uint32_t* offsets,
               uint32_t* rank_out);

// Stable partition of indices 0..n-1 by min(acts[i], n_act).  rank_out (optional): the inverse
// permutation, rank_out[perm[p]] = p.  Forms with identical output: LSD passes of <= 8 bits plus the
// bucket starts (bucket_lsd); for batches of at least 2^20 messages the two-level forms -- one MSD pass
// + the in-LDS range sort for n_act < 1056 x 1024 (msd_bucket), two MSD passes + the level-2 work lists
// up to n_act < 2^28 (msd3_bucket).  GD_MSD=1 (default) times the two-level form against the LSD
// passes on the first launches of each batch shape (tune_choose, kind 4) and keeps the faster, 2
// always takes the two-level form.
int bucket_device(gd_handle* h, const uint32_t* acts, uint32_t n, uint32_t n_act, uint32_t* perm, uint32_t* offsets,
                  uint32_t* rank_out = nullptr) {
    if (n_act == 0xFFFFFFFFu) return set_err(h, GD_EINVAL, "n_act too large");
    uint32_t a3 = 0, ra3 = 0;
    const bool one = (n_act >> MSD_SHIFT) + 1 <= MSD_MAX_RANGES;
    const bool three = !one && msd3_split(n_act, &a3, &ra3);
    if (h->msd_mode && n >= (1u << 20) && (one || three)) {
        int meas = -1;
        // keyed by the batch size and by the messages a range holds (which decide whether ranges are
        // staged in LDS): a handle bucketing 16M messages over 1M and over 10k activations keeps one
        // choice for each
        int per_range = 0;
        while (per_range < 31 && ((uint64_t)n / ((n_act >> MSD_SHIFT) + 1) >> per_range) > 1) ++per_range;
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

template <typename T>
int h2d(gd_handle* h, DevBuf& b, const T* src, size_t count) {
    GD_TRY(ensure(h, b, count * sizeof(T)));
    if (count) HIP_TRY(h, hipMemcpyAsync(b.p, src, count * sizeof(T), hipMemcpyHostToDevice, h->stream));
    return GD_OK;
}

template <typename T>
int d2h(gd_handle* h, T* dst, const DevBuf& b, size_t count) {
    if (count && dst) HIP_TRY(h, hipMemcpyAsync(dst, b.p, count * sizeof(T), hipMemcpyDeviceToHost, h->stream));
    return GD_OK;
}

int sync(gd_handle* h) {
    HIP_TRY(h, hipStreamSynchronize(h->stream));
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
        return set_err(h, GD_EFULL, "device error bits 0x%x", e);
    }
    return GD_OK;
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
               void* out_recs, uint32_t* out_pay, uint32_t* counts, const ExtArgs& ext = ExtArgs{},
               uint32_t* kdesc = nullptr, uint32_t regions = 1) {
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
             uint32_t my_rank, void* out_keys, uint32_t* out_pos, uint32_t* counts, const uint32_t* n1 = nullptr) {
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

}  // namespace

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
    h->timing = (cfg->flags & GD_CFG_KERNEL_TIMING) != 0;
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
        e = hipMalloc(&h->ctr, sizeof(DevCounters));
        if (e != hipSuccess) r = set_err(nullptr, GD_ENOMEM, "counters: %s", hipGetErrorString(e));
        else if ((e = hipMemsetAsync(h->ctr, 0, sizeof(DevCounters), h->stream)) != hipSuccess)
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

namespace {
void comm_release(gd_handle* h);
}

void gd_destroy(gd_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (DevBuf* b : {&h->ring_pts, &h->ring_own, &h->keys_in, &h->u32_a, &h->u32_b, &h->u32_c, &h->u32_d, &h->u8_a,
                      &h->out_a, &h->out_b, &h->out_c, &h->hist, &h->partials, &h->partials2, &h->offs})
        free_buf(*b);
    for (DevBuf& b : h->fr) free_buf(b);
    for (DevBuf& b : h->m3) free_buf(b);
    free_buf(h->tune_buf);
    for (DevBuf& b : h->fr_ext) free_buf(b);
    for (DevBuf& b : h->churn) free_buf(b);
    for (DevBuf& b : h->fan) free_buf(b);
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

namespace {
// AddSingleActivation for a batch of device-resident keys / values (first registration wins, batch
// order); out_vals / out_ins are device arrays (either may be null).  Synchronous.
int register_core(gd_handle* h, const gd_key* dk, const gd_val* dvals, uint32_t n, gd_val* out_vals,
                  uint8_t* out_ins) {
    GD_TRY(maybe_grow_table(h, n));
    const uint32_t op = ++h->dir_op;
    GD_TRY(ensure(h, h->u32_a, (size_t)n * 4));   // slot_of
    GD_TRY(ensure(h, h->u32_b, (size_t)n * 4));   // win
    GD_TRY(ensure(h, h->u8_a, (size_t)n));        // is_new
    HIP_TRY(h, hipMemsetAsync(h->u8_a.p, 0, n, h->stream));
    const dim3 g(blocks_for(n, BLOCK)), b(BLOCK);
    uint32_t* slot_of = (uint32_t*)h->u32_a.p;
    uint32_t* win = (uint32_t*)h->u32_b.p;
    uint8_t* is_new = (uint8_t*)h->u8_a.p;
    const unsigned long long mask = h->capacity - 1;
    // claim pass, then relaunches for the items that met an unpublished claim
    for (uint32_t pass = 0;; ++pass) {
        HIP_TRY(h, hipMemsetAsync(&h->ctr->retry, 0, sizeof(uint32_t), h->stream));
        GD_TRY(launch(h, "k_reg_claim", g, b, 0, k_reg_claim, dk, n, h->slots, mask, h->ctr, slot_of, is_new,
                      (uint32_t)(pass > 0), dvals, table_args(h)));
        GD_TRY(pull_counters(h));
        if (h->ctr_host.retry == 0 || h->ctr_host.err) break;
        if (pass >= 64) return set_err(h, GD_ETIMEOUT, "gd_dir_register: claims did not settle");
    }
    GD_TRY(launch(h, "k_reg_minwin", g, b, 0, k_reg_minwin, (const uint32_t*)slot_of, (const uint8_t*)is_new, n, h->slots));
    GD_TRY(launch(h, "k_reg_resolve", g, b, 0, k_reg_resolve, (const uint32_t*)slot_of, (const uint8_t*)is_new, n,
                  (const Slot*)h->slots, win));
    GD_TRY(launch(h, "k_reg_commit", g, b, 0, k_reg_commit, (const uint32_t*)slot_of, (const uint32_t*)win, dvals, n,
                  h->slots, h->ctr, h->vtag, op));
    if (out_vals || out_ins)
        GD_TRY(launch(h, "k_reg_report", g, b, 0, k_reg_report, (const uint32_t*)slot_of, (const uint32_t*)win, n,
                      (const Slot*)h->slots, out_vals, out_ins));
    GD_TRY(pull_counters(h));
    if (h->ctr_host.err) {
        const uint32_t e = h->ctr_host.err;
        HIP_TRY(h, hipMemsetAsync(&h->ctr->err, 0, sizeof(uint32_t), h->stream));
        GD_TRY(sync(h));
        return set_err(h, (e & 2) ? GD_EFULL : (e & 4) ? GD_EINVAL : GD_ETIMEOUT,
                       "gd_dir_register: device error bits 0x%x (2: table full, 4: silo index > 0xFFFE)", e);
    }
    return GD_OK;
}
}  // namespace

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
                         (uint8_t*)h->out_b.p));
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
    return register_core(h, d_keys, d_vals, n, d_out_vals, d_out_inserted);
}

int gd_dir_upsert(gd_handle* h, const gd_key* keys, const gd_val* vals, uint32_t n, uint8_t* out_inserted) {
    if (!h || (n && (!keys || !vals))) return set_err(h, GD_EINVAL, "null argument");
    for (uint32_t i = 0; i < n; ++i)
        if (vals[i].silo > 0xFFFEu) return set_err(h, GD_EINVAL, "silo index %u out of range at %u", vals[i].silo, i);
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(maybe_grow_table(h, n));
    const uint32_t op = ++h->dir_op;
    GD_TRY(h2d(h, h->keys_in, keys, n));
    GD_TRY(h2d(h, h->out_c, vals, n));            // gd_val staging
    GD_TRY(ensure(h, h->u32_a, (size_t)n * 4));   // slot_of
    GD_TRY(ensure(h, h->u8_a, (size_t)n));        // is_new
    GD_TRY(ensure(h, h->out_b, (size_t)n));
    if (h->up_last.bytes < h->capacity * 4) {     // one u32 per slot, kept zero between calls
        GD_TRY(ensure(h, h->up_last, h->capacity * 4));
        HIP_TRY(h, hipMemsetAsync(h->up_last.p, 0, h->up_last.bytes, h->stream));
    }
    HIP_TRY(h, hipMemsetAsync(h->u8_a.p, 0, n, h->stream));
    const dim3 g(blocks_for(n, BLOCK)), b(BLOCK);
    uint32_t* slot_of = (uint32_t*)h->u32_a.p;
    uint8_t* is_new = (uint8_t*)h->u8_a.p;
    uint32_t* last = (uint32_t*)h->up_last.p;
    const gd_key* dk = (const gd_key*)h->keys_in.p;
    const unsigned long long mask = h->capacity - 1;
    for (uint32_t pass = 0;; ++pass) {            // the registration's claim protocol (k_reg_claim)
        HIP_TRY(h, hipMemsetAsync(&h->ctr->retry, 0, sizeof(uint32_t), h->stream));
        GD_TRY(launch(h, "k_reg_claim", g, b, 0, k_reg_claim, dk, n, h->slots, mask, h->ctr, slot_of, is_new,
                      (uint32_t)(pass > 0), (const gd_val*)h->out_c.p, table_args(h)));
        GD_TRY(pull_counters(h));
        if (h->ctr_host.retry == 0 || h->ctr_host.err) break;
        if (pass >= 64) return set_err(h, GD_ETIMEOUT, "gd_dir_upsert: claims did not settle");
    }
    GD_TRY(launch(h, "k_up_last", g, b, 0, k_up_last, (const uint32_t*)slot_of, n, last));
    GD_TRY(launch(h, "k_up_apply", g, b, 0, k_up_apply, (const uint32_t*)slot_of, (const uint8_t*)is_new,
                  (const gd_val*)h->out_c.p, n, (const uint32_t*)last, h->slots, h->ctr, (uint8_t*)h->out_b.p,
                  h->vtag, op));
    GD_TRY(launch(h, "k_up_clear", g, b, 0, k_up_clear, (const uint32_t*)slot_of, n, last));
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
    GD_TRY(h2d(h, h->keys_in, keys, n));
    GD_TRY(h2d(h, h->u32_b, acts, n));
    GD_TRY(ensure(h, h->u32_a, (size_t)n * 4));
    GD_TRY(ensure(h, h->out_b, (size_t)n));
    const dim3 g(blocks_for(n, BLOCK)), b(BLOCK);
    uint32_t* slot_of = (uint32_t*)h->u32_a.p;
    const unsigned long long mask = h->capacity - 1;
    GD_TRY(launch(h, "k_unreg_find", g, b, 0, k_unreg_find, (const gd_key*)h->keys_in.p, (const uint32_t*)h->u32_b.p, n,
                  (const Slot*)h->slots, mask, (const DevCounters*)h->ctr, slot_of));
    GD_TRY(launch(h, "k_unreg_poison", g, b, 0, k_unreg_poison, (const uint32_t*)slot_of, n, h->slots));
    GD_TRY(launch(h, "k_unreg_min", g, b, 0, k_unreg_min, (const uint32_t*)slot_of, n, h->slots));
    GD_TRY(launch(h, "k_unreg_commit", g, b, 0, k_unreg_commit, (const uint32_t*)slot_of, n, h->slots, h->ctr,
                  (uint8_t*)h->out_b.p));
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
    HIP_TRY(h, hipMemsetAsync(h->ctr, 0, sizeof(DevCounters), h->stream));
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
    DevCounters fresh{};
    HIP_TRY(h, hipMemcpyAsync(h->ctr, &fresh, sizeof fresh, hipMemcpyHostToDevice, h->stream));
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
    return bucket_device(h, d_act, n, n_act, d_perm, d_offsets);
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
    GD_TRY(resolve_timing(h));
    h->timing = enable != 0;
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
    std::vector<std::pair<uint32_t, hipGraphExec_t>> graphs;
    uint64_t graphs_gen = 0;       // handle layout the cached graphs were captured against

    uint32_t* out_u32(uint8_t* base, int k) const {
        const size_t c = capacity;
        const size_t at[6] = {0, c, 2 * c, 3 * c, 3 * c + 1, 4 * c + 2};   // silo act perm n_runs run_start run_act
        return (uint32_t*)base + at[k];
    }
    uint8_t* out_status(uint8_t* base) const { return base + (5 * (size_t)capacity + 2) * 4; }
};

namespace {

// H2D keys -> route -> one-workgroup radix sort + runs -> one D2H of the whole output block; or, zero-copy,
// route (keys read from and silo / status written to pinned host memory) -> sort (perm / runs / act to host).
template <int IT>
int mb_launch_sort(gd_microbatch* mb, dim3 grid, uint32_t bits, const uint32_t* a, uint32_t n, uint32_t passes,
                   uint32_t* pm, uint32_t* ra, uint32_t* rs, uint32_t* nr, uint32_t* ac) {
    gd_handle* h = mb->h;
    const dim3 b(MB_THREADS);
    const uint32_t na = mb->n_act;
    unsigned long long* ts = mb->ts;
    const uint32_t bal = h->radix_rank_atomic ? 0u : 1u;
    switch (bits) {
        case 4: return launch(h, "k_mb_sort_runs", grid, b, 0, k_mb_sort_runs<4, IT>, a, n, passes, na, pm, ra, rs, nr, ac, ts, bal);
        case 5: return launch(h, "k_mb_sort_runs", grid, b, 0, k_mb_sort_runs<5, IT>, a, n, passes, na, pm, ra, rs, nr, ac, ts, bal);
        case 6: return launch(h, "k_mb_sort_runs", grid, b, 0, k_mb_sort_runs<6, IT>, a, n, passes, na, pm, ra, rs, nr, ac, ts, bal);
        case 7: return launch(h, "k_mb_sort_runs", grid, b, 0, k_mb_sort_runs<7, IT>, a, n, passes, na, pm, ra, rs, nr, ac, ts, bal);
        case 8: return launch(h, "k_mb_sort_runs", grid, b, 0, k_mb_sort_runs<8, IT>, a, n, passes, na, pm, ra, rs, nr, ac, ts, bal);
        case 9: return launch(h, "k_mb_sort_runs", grid, b, 0, k_mb_sort_runs<9, IT>, a, n, passes, na, pm, ra, rs, nr, ac, ts, bal);
        case 10: return launch(h, "k_mb_sort_runs", grid, b, 0, k_mb_sort_runs<10, IT>, a, n, passes, na, pm, ra, rs, nr, ac, ts, bal);
        default: return launch(h, "k_mb_sort_runs", grid, b, 0, k_mb_sort_runs<11, IT>, a, n, passes, na, pm, ra, rs, nr, ac, ts, bal);
    }
}

int mb_enqueue(gd_microbatch* mb, uint32_t n) {
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
        switch (h->ring_mode) {
            case GD_RING_DIRECTORY:
                GD_TRY(launch(h, "k_mb_route", g, b, ring_lds(h), k_mb_route<GD_RING_DIRECTORY>, k, n, ring_args(h),
                              table_args(h), so, act_dst, st, mb->out_u32(d, 1), mb->ts));
                break;
            case GD_RING_CONSISTENT:
                GD_TRY(launch(h, "k_mb_route", g, b, ring_lds(h), k_mb_route<GD_RING_CONSISTENT>, k, n, ring_args(h),
                              table_args(h), so, act_dst, st, mb->out_u32(d, 1), mb->ts));
                break;
            default:
                GD_TRY(launch(h, "k_mb_route", g, b, ring_lds(h), k_mb_route<GD_RING_VIRTUAL_BUCKETS>, k, n,
                              ring_args(h), table_args(h), so, act_dst, st, mb->out_u32(d, 1), mb->ts));
                break;
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
    const dim3 g1(zc ? std::max<uint32_t>(1, std::min(mb->split, std::max<uint32_t>(1, n / 256))) : 1);
    if (n <= MB_THREADS * 4) GD_TRY(mb_launch_sort<4>(mb, g1, bits, a, n, passes, pm, ra, rs, nr, ac));
    else GD_TRY(mb_launch_sort<8>(mb, g1, bits, a, n, passes, pm, ra, rs, nr, ac));
    if (!zc) HIP_TRY(h, hipMemcpyAsync(mb->h_out, d, mb->out_bytes, hipMemcpyDeviceToHost, h->stream));
    return GD_OK;
}

}  // namespace

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
        GD_TRY(mb_enqueue(mb, n));
        return sync(h);
    }
    if (mb->graphs_gen != h->layout_gen) {     // ring or table moved: drop stale graphs
        for (auto& g : mb->graphs) (void)hipGraphExecDestroy(g.second);
        mb->graphs.clear();
        mb->graphs_gen = h->layout_gen;
    }
    hipGraphExec_t exec = nullptr;
    for (auto& g : mb->graphs)
        if (g.first == n) exec = g.second;
    if (!exec) {
        // no allocation happens inside mb_enqueue (route needs no scratch), so capture directly
        const bool timing = h->timing;
        h->timing = false;
        hipGraph_t graph = nullptr;
        const uint64_t routed = h->routed;       // counted per replay below, not at capture
        HIP_TRY(h, hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
        const int rc = mb_enqueue(mb, n);
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
    return sync(h);
}

}  // extern "C"

// ================================================================== header decode
namespace {

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
                         const gd_frame_fields* out, bool ext = false) {
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
AdArgs ad_args(gd_handle* h);

// ext: KeyExt targets (string-keyed grains) are routed too, their strings read from buf itself.  With an
// ActivationDirectory (gd_actdir_add), a frame whose address is complete (GD_ROUTE_ADDRESSED) gets the
// context of its TargetActivation as its act (k_frame_addressed_act), so it is bucketed with it.
int route_frames_device(gd_handle* h, const uint8_t* buf, uint64_t len, const uint64_t* off, uint32_t n,
                        uint32_t n_act, const gd_frame_fields* out, uint32_t* silo, uint32_t* act, uint8_t* status,
                        uint32_t* perm, uint32_t* offsets, bool ext = false) {
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

}  // namespace

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

// ================================================================== membership change
namespace {

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

}  // namespace

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

// ================================================================== follower fan-out
namespace {

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

template <int MODE, bool CX>
int fan_route_launch_cx(gd_handle* h, const uint32_t* row_off, const uint32_t* dst, const uint32_t* frontier,
                        uint32_t nf, uint32_t total, uint64_t tcd, uint32_t* target, uint32_t* sender, uint32_t* silo,
                        uint32_t* act, uint8_t* status) {
    const dim3 g(blocks_for(total, FAN_TILE)), b(BLOCK);
    const uint32_t* ends = (const uint32_t*)h->fan[0].p;
    const CxArgs cx = CX ? cx_args(h) : CxArgs{};
    // 2 outputs a thread in flight (1: 2.95 ms, 4: 3.03 ms against 2.87 ms a cfg 4 cascade,
    // profiles/r02_v1_fanout_cfg4_ilp_ab.jsonl)
    return launch(h, "k_fan_route", g, b, ring_lds(h), k_fan_route<MODE, 2, CX>, row_off, dst, frontier, nf, ends,
                  total, tcd, ring_args(h), table_args(h), target, sender, silo, act, status, cx, Cx8Args{});
}

template <int MODE>
int fan_route_launch(gd_handle* h, const uint32_t* row_off, const uint32_t* dst, const uint32_t* frontier, uint32_t nf,
                     uint32_t total, uint64_t tcd, uint32_t* target, uint32_t* sender, uint32_t* silo, uint32_t* act,
                     uint8_t* status) {
    bool cx = false;
    GD_TRY(cx_ensure(h, &cx, total));
    int meas = -1;
    const int var = cx ? cx_choose(h, 2, total, &meas, h->cx8_ok ? 3 : 2) : 1;
    cx = var == 0;
    CxMeasure m(h, meas, total);
    if (var == 2) {                    // the 8-B index
        const dim3 g(blocks_for(total, FAN_TILE)), b(BLOCK);
        return launch(h, "k_fan_route", g, b, ring_lds(h), k_fan_route<MODE, 2, false, (int)CX_GROUP, true>, row_off,
                      dst, frontier, nf, (const uint32_t*)h->fan[0].p, total, tcd, ring_args(h), table_args(h), target,
                      sender, silo, act, status, CxArgs{}, cx8_args(h));
    }
    if (cx)
        return fan_route_launch_cx<MODE, true>(h, row_off, dst, frontier, nf, total, tcd, target, sender, silo, act,
                                               status);
    return fan_route_launch_cx<MODE, false>(h, row_off, dst, frontier, nf, total, tcd, target, sender, silo, act,
                                            status);
}

int fan_route(gd_handle* h, const uint32_t* row_off, const uint32_t* dst, const uint32_t* frontier, uint32_t nf,
              uint32_t total, uint64_t tcd, uint32_t* target, uint32_t* sender, uint32_t* silo, uint32_t* act,
              uint8_t* status) {
    h->routed += total;
    switch (h->ring_mode) {
        case GD_RING_DIRECTORY:
            return fan_route_launch<GD_RING_DIRECTORY>(h, row_off, dst, frontier, nf, total, tcd, target, sender, silo,
                                                       act, status);
        case GD_RING_CONSISTENT:
            return fan_route_launch<GD_RING_CONSISTENT>(h, row_off, dst, frontier, nf, total, tcd, target, sender, silo,
                                                        act, status);
        default:
            return fan_route_launch<GD_RING_VIRTUAL_BUCKETS>(h, row_off, dst, frontier, nf, total, tcd, target, sender,
                                                             silo, act, status);
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

// fan_count of a frontier whose length is on the device (*d_nf <= nf_max): the degree and scan grids
// are sized for nf_max, and one read-back brings both the length and the total (instead of one for
// each).  Past 16M rows it reads the length first and takes fan_count.
int fan_count_dev(gd_handle* h, const uint32_t* row_off, uint32_t n_nodes, const uint32_t* frontier,
                  const uint32_t* d_nf, uint32_t nf_max, uint32_t* nf, uint64_t* total) {
    *nf = 0;
    *total = 0;
    if (nf_max == 0) return GD_OK;
    const uint32_t nb4 = blocks_for(nf_max, SCAN_TILE), nb16 = blocks_for(nf_max, 4 * SCAN_TILE);
    if (!(nb4 <= 2048 || nb16 <= 4096)) {
        GD_TRY(pinned_scratch(h, 4));
        HIP_TRY(h, hipMemcpyAsync(h->h_pin, d_nf, 4, hipMemcpyDeviceToHost, h->stream));
        GD_TRY(sync(h));
        *nf = *(const uint32_t*)h->h_pin;
        return fan_count(h, row_off, n_nodes, frontier, *nf, total);
    }
    const bool wide = nb4 > 2048;
    const uint32_t nb = wide ? nb16 : nb4;
    GD_TRY(ensure(h, h->fan[0], (size_t)nf_max * 4));
    GD_TRY(ensure(h, h->fan[1], (size_t)nb * 4));
    GD_TRY(pinned_scratch(h, ((size_t)nb + 1) * 4));
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
    HIP_TRY(h, hipMemcpyAsync(pin + nb, d_nf, 4, hipMemcpyDeviceToHost, h->stream));
    GD_TRY(sync(h));
    uint64_t t = 0;
    for (uint32_t b = 0; b < nb; ++b) t += pin[b];
    if (t > 0xFFFFFFFFull)
        return set_err(h, GD_EINVAL, "fan-out of %llu messages exceeds 2^32 - 1", (unsigned long long)t);
    *nf = pin[nb];
    *total = t;
    return GD_OK;
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
    GD_TRY(sync(h));                                   // the previous call's results may be in use
    if (h->fm_hop.size() < hops) h->fm_hop.resize(hops);
    h->fm_res.assign(hops, gd_fanout_hop{});
    h->fm_n_act = n_act;
    DevBuf* S = h->fm_scr;
    GD_TRY(ensure(h, S[5], (size_t)n_act + 16));
    uint8_t* visited = (uint8_t*)S[5].p;
    HIP_TRY(h, hipMemsetAsync(visited, 0, (size_t)n_act + 16, h->stream));
    uint32_t nf = n_seeds;
    {
        std::array<DevBuf, 10>& H0 = h->fm_hop[0];
        GD_TRY(ensure(h, H0[0], ((size_t)std::max(nf, n_act) + 4) * 4));
        if (nf) {
            HIP_TRY(h, hipMemcpyAsync(H0[0].p, seeds, (size_t)nf * 4, hipMemcpyDeviceToDevice, h->stream));
            GD_TRY(launch(h, "k_mark_visited", dim3(blocks_for(nf, BLOCK)), dim3(BLOCK), 0, k_mark_visited,
                          (const uint32_t*)H0[0].p, nf, n_act, visited));
        }
    }
    uint64_t total = 0;
    GD_TRY(fan_count(h, row_off, n_nodes, (const uint32_t*)h->fm_hop[0][0].p, nf, &total));
    for (uint32_t hp = 0; hp < hops; ++hp) {
        std::array<DevBuf, 10>& H = h->fm_hop[hp];
        const uint32_t* frontier = (const uint32_t*)H[0].p;
        const uint32_t m = (uint32_t)total;
        gd_fanout_hop& res = h->fm_res[hp];
        res.n_frontier = nf;
        res.frontier = frontier;
        res.n_sent = total;
        const size_t m4 = (size_t)m * 4 + 16;
        const size_t want[10] = {0, m4, m4, 0, m4, m4, (size_t)m + 16, m4, ((size_t)n_act + 2) * 4, 0};
        for (int b = 1; b < 9; ++b)
            if (want[b]) GD_TRY(ensure(h, H[b], want[b]));
        uint32_t* target = (uint32_t*)H[1].p;
        uint32_t* sender = (uint32_t*)H[2].p;
        uint32_t* silo = (uint32_t*)H[4].p;
        uint32_t* act = (uint32_t*)H[5].p;
        uint8_t* st = (uint8_t*)H[6].p;
        uint32_t* perm = (uint32_t*)H[7].p;
        uint32_t* offs = (uint32_t*)H[8].p;
        if (m) GD_TRY(fan_route(h, row_off, dst, frontier, nf, m, tcd, target, sender, silo, act, st));
        GD_TRY(bucket_device(h, act, m, n_act, perm, offs));
        res.n_recv = m;
        res.target = target;
        res.sender = sender;
        res.src = nullptr;
        res.silo = silo;
        res.act = act;
        res.status = st;
        res.perm = perm;
        res.offsets = offs;
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

}  // namespace

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

// ================================================================== non-owner directory cache
namespace {

// KeyExt helpers (defined with the KeyExt section below).
bool is_keyext_cat(uint64_t tcd);
uint32_t kx_hash_host(const gd_key& k, const uint8_t* s, int32_t len);
int host_ext(gd_handle* h, const gd_key_ext* ext, uint32_t i, const uint8_t*& s, int32_t& len);
int stage_ext(gd_handle* h, const gd_key_ext* ext, uint32_t n, gd_key_ext* dx);
bool ext_ok(const gd_key_ext* ext, uint32_t n);
KxArgs kx_args(gd_handle* h);

CacheArgs cache_args(gd_handle* h) {
    return CacheArgs{h->cslots, h->ccap - 1, h->cctr, (const uint8_t*)h->cache_local.p,
                     (const uint8_t*)h->cache_valid.p, h->cache_nsilos, (const uint8_t*)h->cx_heap.p};
}

// Generations for the hits of a batch, in batch order (hit flags in `hit`, slots in `cslot`).
int cache_touch(gd_handle* h, uint32_t* hit, const uint32_t* cslot, uint32_t n) {
    GD_TRY(ensure(h, h->cbuf[2], (size_t)n * 4));
    uint32_t* pos = (uint32_t*)h->cbuf[2].p;
    GD_TRY(scan_device<OpAdd>(h, hit, n, false, true, "cache", pos));
    GD_TRY(launch(h, "k_cache_touch", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), 0, k_cache_touch, cslot,
                  (const uint32_t*)pos, n, h->cslots, (const CacheCounters*)h->cctr));
    return launch(h, "k_cache_advance", dim3(1), dim3(64), 0, k_cache_advance, (const uint32_t*)pos, n, h->cctr);
}

template <int MODE>
int route_cached_t(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t* silo, uint32_t* act, uint8_t* status,
                   uint32_t* hit, uint32_t* cslot) {
    return launch(h, "k_route_cached", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), ring_lds(h), k_route_cached<MODE>, keys,
                  n, ring_args(h), table_args(h), cache_args(h), silo, act, status, hit, cslot, h->cctr);
}

int route_cached(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t* silo, uint32_t* act, uint8_t* status,
                 bool touch) {
    if (n == 0) return GD_OK;
    GD_TRY(ensure(h, h->cbuf[0], (size_t)n * 4));
    GD_TRY(ensure(h, h->cbuf[1], (size_t)n * 4));
    uint32_t* hit = (uint32_t*)h->cbuf[0].p;
    uint32_t* cslot = (uint32_t*)h->cbuf[1].p;
    switch (h->ring_mode) {
        case GD_RING_DIRECTORY: GD_TRY(route_cached_t<GD_RING_DIRECTORY>(h, keys, n, silo, act, status, hit, cslot)); break;
        case GD_RING_CONSISTENT: GD_TRY(route_cached_t<GD_RING_CONSISTENT>(h, keys, n, silo, act, status, hit, cslot)); break;
        default: GD_TRY(route_cached_t<GD_RING_VIRTUAL_BUCKETS>(h, keys, n, silo, act, status, hit, cslot));
    }
    return touch ? cache_touch(h, hit, cslot, n) : GD_OK;
}

template <int MODE>
int route_cached_keyext_t(gd_handle* h, const gd_key* keys, const ExtArgs& x, uint32_t n, uint32_t* silo,
                          uint32_t* act, uint8_t* st, uint32_t* hit, uint32_t* cslot) {
    return launch(h, "k_route_cached_keyext", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), ring_lds(h),
                  k_route_cached_keyext<MODE>, keys, n, x, ring_args(h), kx_args(h), cache_args(h), silo, act, st, hit,
                  cslot, h->cctr);
}

// After route_cached(..., touch = false) over the same batch: the KeyExt LocalLookup over the
// messages it left at GD_ROUTE_KEYEXT (their hit flags join the batch's), then the generations.
int route_cached_keyext(gd_handle* h, const gd_key* keys, const ExtArgs& x, uint32_t n, uint32_t* silo, uint32_t* act,
                        uint8_t* st) {
    if (n == 0) return GD_OK;
    uint32_t* hit = (uint32_t*)h->cbuf[0].p;
    uint32_t* cslot = (uint32_t*)h->cbuf[1].p;
    if (h->cbuf[0].bytes < (size_t)n * 4 || h->cbuf[1].bytes < (size_t)n * 4)
        return set_err(h, GD_ESTATE, "KeyExt LocalLookup without the batch's route pass");
    switch (h->ring_mode) {
        case GD_RING_DIRECTORY: GD_TRY(route_cached_keyext_t<GD_RING_DIRECTORY>(h, keys, x, n, silo, act, st, hit, cslot)); break;
        case GD_RING_CONSISTENT: GD_TRY(route_cached_keyext_t<GD_RING_CONSISTENT>(h, keys, x, n, silo, act, st, hit, cslot)); break;
        default: GD_TRY(route_cached_keyext_t<GD_RING_VIRTUAL_BUCKETS>(h, keys, x, n, silo, act, st, hit, cslot));
    }
    return cache_touch(h, hit, cslot, n);
}

int cache_pull(gd_handle* h, CacheCounters* c) {
    HIP_TRY(h, hipMemcpyAsync(c, h->cctr, sizeof(CacheCounters), hipMemcpyDeviceToHost, h->stream));
    return sync(h);
}

int cache_check(gd_handle* h) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    if (!h->cache_max) return set_err(h, GD_ESTATE, "no directory cache configured (gd_cache_configure)");
    return GD_OK;
}

// (Re)build the table with `cap` slots, moving the live entries (tombstone compaction).
int cache_rehash(gd_handle* h, unsigned long long cap) {
    CacheSlot* ns = nullptr;
    hipError_t e = hipMalloc(&ns, cap * sizeof(CacheSlot));
    if (e != hipSuccess) return set_err(h, GD_ENOMEM, "cache hipMalloc(%llu slots): %s", cap, hipGetErrorString(e));
    HIP_TRY(h, hipMemsetAsync(ns, 0, cap * sizeof(CacheSlot), h->stream));
    CacheCounters c{};
    GD_TRY(cache_pull(h, &c));
    CacheCounters fresh = c;
    fresh.live = fresh.tomb = 0;
    fresh.max_probe = 0;
    fresh.err = 0;
    HIP_TRY(h, hipMemcpyAsync(h->cctr, &fresh, sizeof fresh, hipMemcpyHostToDevice, h->stream));
    if (h->cslots) {
        GD_TRY(launch(h, "k_cache_rehash", dim3(blocks_for(h->ccap, BLOCK)), dim3(BLOCK), 0, k_cache_rehash,
                      (const CacheSlot*)h->cslots, h->ccap, ns, cap - 1, h->cctr));
        GD_TRY(sync(h));
        HIP_TRY(h, hipFree(h->cslots));
    }
    h->cslots = ns;
    h->ccap = cap;
    return sync(h);
}

int cache_masks(gd_handle* h, const uint8_t* local, const uint8_t* valid, uint32_t n_silos) {
    std::vector<uint8_t> l(n_silos ? n_silos : 1, 0), v(n_silos ? n_silos : 1, 0);
    for (uint32_t i = 0; i < n_silos; ++i) {
        l[i] = local ? (local[i] != 0) : 0;
        v[i] = valid ? (valid[i] != 0) : 1;
    }
    GD_TRY(h2d(h, h->cache_local, l.data(), l.size()));
    GD_TRY(h2d(h, h->cache_valid, v.data(), v.size()));
    h->cache_nsilos = n_silos;
    return sync(h);
}

struct KeyHash {
    size_t operator()(const gd_key& k) const {
        return std::hash<uint64_t>()(k.n0 * 0x9E3779B97F4A7C15ull ^ k.n1 * 0xC2B2AE3D27D4EB4Full ^ k.type_code_data);
    }
};
struct KeyEq {
    bool operator()(const gd_key& a, const gd_key& b) const {
        return a.n0 == b.n0 && a.n1 == b.n1 && a.type_code_data == b.type_code_data;
    }
};

// The `v` lowest live generations as (gen, slot), ascending.
int cache_lowest(gd_handle* h, uint64_t v, uint64_t next_gen, std::vector<std::pair<uint64_t, uint32_t>>* out) {
    out->clear();
    if (v == 0) return GD_OK;
    GD_TRY(ensure(h, h->cbuf[6], 16));
    unsigned long long* dcount = (unsigned long long*)h->cbuf[6].p;
    const uint32_t grid = std::min<uint32_t>(blocks_for(h->ccap, BLOCK), 2048);
    // smallest t with |{live: gen <= t}| >= v (generations are distinct, so the count is exactly v)
    uint64_t lo = 1, hi = next_gen;
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        HIP_TRY(h, hipMemsetAsync(dcount, 0, 8, h->stream));
        GD_TRY(launch(h, "k_cache_count_le", dim3(grid), dim3(BLOCK), 0, k_cache_count_le, (const CacheSlot*)h->cslots,
                      h->ccap, (unsigned long long)mid, dcount));
        unsigned long long c = 0;
        HIP_TRY(h, hipMemcpyAsync(&c, dcount, 8, hipMemcpyDeviceToHost, h->stream));
        GD_TRY(sync(h));
        if (c >= v) hi = mid;
        else lo = mid + 1;
    }
    GD_TRY(ensure(h, h->cbuf[7], (size_t)v * 12 + 16));
    unsigned long long* dgen = (unsigned long long*)h->cbuf[7].p;
    uint32_t* dslot = (uint32_t*)(dgen + v);
    uint32_t* cursor = (uint32_t*)h->cbuf[6].p;
    HIP_TRY(h, hipMemsetAsync(cursor, 0, 4, h->stream));
    GD_TRY(launch(h, "k_cache_collect_le", dim3(blocks_for(h->ccap, BLOCK)), dim3(BLOCK), 0, k_cache_collect_le,
                  (const CacheSlot*)h->cslots, h->ccap, (unsigned long long)lo, cursor, dgen, dslot, (uint32_t)v));
    uint32_t got = 0;
    std::vector<unsigned long long> g(v);
    std::vector<uint32_t> sl(v);
    HIP_TRY(h, hipMemcpyAsync(&got, cursor, 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipMemcpyAsync(g.data(), dgen, v * 8, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipMemcpyAsync(sl.data(), dslot, v * 4, hipMemcpyDeviceToHost, h->stream));
    GD_TRY(sync(h));
    if (got != v) return set_err(h, GD_ESTATE, "cache: %u entries at or below generation %llu, expected %llu", got,
                                 (unsigned long long)lo, (unsigned long long)v);
    out->resize(v);
    for (uint64_t i = 0; i < v; ++i) (*out)[i] = {g[i], sl[i]};
    std::sort(out->begin(), out->end());
    return GD_OK;
}

}  // namespace

extern "C" {

int gd_cache_configure(gd_handle* h, uint32_t max_size, const uint8_t* local_silo, const uint8_t* valid_silo,
                       uint32_t n_silos) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    if (n_silos && !local_silo) return set_err(h, GD_EINVAL, "null local_silo");
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(sync(h));
    h->layout_gen++;
    if (max_size == 0) {                       // back to whole-node mode
        h->cache_max = 0;
        return GD_OK;
    }
    if (!h->cctr) {
        hipError_t e = hipMalloc(&h->cctr, sizeof(CacheCounters));
        if (e != hipSuccess) return set_err(h, GD_ENOMEM, "cache counters: %s", hipGetErrorString(e));
    }
    CacheCounters z{};
    HIP_TRY(h, hipMemcpyAsync(h->cctr, &z, sizeof z, hipMemcpyHostToDevice, h->stream));
    if (h->cslots) {
        HIP_TRY(h, hipFree(h->cslots));
        h->cslots = nullptr;
    }
    const unsigned long long cap = pow2_at_least(2ull * max_size);
    h->cache_max = max_size;
    h->cx_used = 0;
    GD_TRY(cache_rehash(h, cap));
    return cache_masks(h, local_silo, valid_silo, n_silos);
}

int gd_cache_set_silos(gd_handle* h, const uint8_t* local_silo, const uint8_t* valid_silo, uint32_t n_silos) {
    GD_TRY(cache_check(h));
    if (n_silos && !local_silo) return set_err(h, GD_EINVAL, "null local_silo");
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(sync(h));
    return cache_masks(h, local_silo, valid_silo, n_silos);
}

}  // extern "C"

namespace {

// A batch's KeyExt view on the host: per item the string (len >= 0) or GD_KEYEXT_NULL, and the
// KeyExt uniform hash.  Only KeyExt-category keys read `ext` (the others have no KeyExt,
// UniqueKey.HasKeyExt); GD_KEYEXT_HOST or a bad range is GD_EINVAL here.
struct HostExt {
    std::vector<const uint8_t*> s;
    std::vector<int32_t> len;
    std::vector<uint32_t> uh;
};

int host_ext_batch(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, HostExt* x) {
    x->s.assign(n, nullptr);
    x->len.assign(n, GD_KEYEXT_NULL);
    x->uh.assign(n, 0);
    if (!ext) return GD_OK;
    for (uint32_t i = 0; i < n; ++i) {
        if (!is_keyext_cat(keys[i].type_code_data)) continue;
        GD_TRY(host_ext(h, ext, i, x->s[i], x->len[i]));
        if (x->len[i] >= 0) x->uh[i] = kx_hash_host(keys[i], x->s[i], x->len[i]);
    }
    return GD_OK;
}

// The LRU's key: the three words, plus the KeyExt string for a KeyExt entry.
std::string cache_key(const gd_key& k, const uint8_t* s, int32_t len) {
    std::string r(reinterpret_cast<const char*>(&k), sizeof(gd_key));
    if (len >= 0) {
        r.push_back('\1');
        r.append(reinterpret_cast<const char*>(s), (size_t)len);
    }
    return r;
}

// Slot of each item's entry (NONE32 when absent) into h->cbuf[4]; keys staged in h->cbuf[3].
int cache_find_batch(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, std::vector<uint32_t>* slot_of) {
    GD_TRY(h2d(h, h->cbuf[3], keys, n));
    GD_TRY(ensure(h, h->cbuf[4], (size_t)n * 4));
    GD_TRY(ensure(h, h->cbuf[5], (size_t)n * 8));
    ExtArgs x{};
    gd_key_ext dx{};
    if (ext) {
        GD_TRY(stage_ext(h, ext, n, &dx));
        x = ExtArgs{dx.bytes, dx.offset, dx.length, dx.bytes_len};
    }
    GD_TRY(launch(h, "k_cache_find", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), 0, k_cache_find,
                  (const gd_key*)h->cbuf[3].p, n, x, cache_args(h), (uint32_t*)h->cbuf[4].p,
                  (unsigned long long*)h->cbuf[5].p));
    slot_of->resize(n);
    HIP_TRY(h, hipMemcpyAsync(slot_of->data(), h->cbuf[4].p, (size_t)n * 4, hipMemcpyDeviceToHost, h->stream));
    return sync(h);
}

// Room for `need` more bytes of KeyExt strings in the cache heap: compact it to the live entries'
// strings (k_cx_sizes, scan, k_cx_move into a new buffer of twice what is then needed) when it is full.
int cx_reserve(gd_handle* h, uint64_t need) {
    if (h->cx_heap.p && h->cx_used + need <= h->cx_heap.bytes) return GD_OK;
    uint64_t live = 0;
    DevBuf nb;
    if (h->cx_used) {
        if (h->ccap > 0x7FFFFFFFull) return set_err(h, GD_EINVAL, "cache table too large to compact");
        const uint32_t cap = (uint32_t)h->ccap;
        GD_TRY(ensure(h, h->cbuf[0], (size_t)cap * 4));
        GD_TRY(ensure(h, h->cbuf[2], (size_t)cap * 4));
        uint32_t* size = (uint32_t*)h->cbuf[0].p;
        uint32_t* pos = (uint32_t*)h->cbuf[2].p;
        GD_TRY(launch(h, "k_cx_sizes", dim3(blocks_for(cap, BLOCK)), dim3(BLOCK), 0, k_cx_sizes,
                      (const CacheSlot*)h->cslots, cap, size));
        GD_TRY(scan_device<OpAdd>(h, size, cap, false, true, "cache", pos));
        uint32_t total = 0;
        HIP_TRY(h, hipMemcpyAsync(&total, pos + cap - 1, 4, hipMemcpyDeviceToHost, h->stream));
        GD_TRY(sync(h));
        live = total;
        GD_TRY(ensure(h, nb, std::max<uint64_t>(2 * (live + need), 1 << 16)));
        GD_TRY(launch(h, "k_cx_move", dim3(blocks_for(cap, BLOCK)), dim3(BLOCK), 0, k_cx_move, h->cslots, cap,
                      (const uint32_t*)size, (const uint32_t*)pos, (const uint8_t*)h->cx_heap.p, (uint8_t*)nb.p));
        GD_TRY(sync(h));
    } else {
        GD_TRY(ensure(h, nb, std::max<uint64_t>(2 * need, 1 << 16)));
    }
    if (nb.bytes > 0xFFFFFFF0ull) {
        free_buf(nb);
        return set_err(h, GD_ENOMEM, "cache KeyExt heap past 4 GiB");
    }
    free_buf(h->cx_heap);
    h->cx_heap = nb;
    h->cx_used = live;
    return GD_OK;
}

// AddOrUpdate of a batch (LRU.Add, LRU.cs:71-76,165-182), KeyExt entries keyed by their string.
int cache_add_impl(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, const gd_val* vals,
                   const int32_t* versions, uint32_t n) {
    GD_TRY(cache_check(h));
    if (n && (!keys || !vals || !versions)) return set_err(h, GD_EINVAL, "null argument");
    for (uint32_t i = 0; i < n; ++i)
        if (vals[i].silo > 0xFFFEu) return set_err(h, GD_EINVAL, "silo index %u out of range at %u", vals[i].silo, i);
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    HostExt hx;
    GD_TRY(host_ext_batch(h, keys, ext, n, &hx));
    CacheCounters c{};
    GD_TRY(cache_pull(h, &c));
    if ((c.live + c.tomb + n) * 4 > h->ccap * 3) {      // compact tombstones (and grow if a batch needs it)
        unsigned long long cap = pow2_at_least(2ull * h->cache_max);
        while ((c.live + n) * 2 > cap) cap <<= 1;
        GD_TRY(cache_rehash(h, cap));
        GD_TRY(cache_pull(h, &c));
    }
    // 1. where each key lives now
    std::vector<uint32_t> slot_of;
    GD_TRY(cache_find_batch(h, keys, ext, n, &slot_of));
    // 2. eviction candidates: each add evicts at most one entry and renews at most one, so the
    //    2n lowest generations cover every pre-existing entry this batch can evict
    const uint64_t M = h->cache_max;
    std::vector<std::pair<uint64_t, uint32_t>> victims;
    if (c.live + n >= M) GD_TRY(cache_lowest(h, std::min<uint64_t>(c.live, 2ull * n), c.next_gen, &victims));
    // 3. AdjustSize + Add (LRU.cs:71-76,165-182) in batch order
    struct Ent {
        uint32_t item;        // batch item that created the entry (its key and KeyExt)
        uint32_t act, silo;
        int32_t ver;
        uint64_t gen;
        uint32_t from_slot;   // pre-existing slot this entry renews, or NONE32
        bool alive;
    };
    std::vector<Ent> ents;
    ents.reserve(n);
    std::unordered_map<std::string, uint32_t> ent_of;
    std::unordered_map<uint32_t, uint8_t> pre;          // pre-existing slot -> 1 evicted, 2 renewed
    typedef std::pair<uint64_t, uint32_t> GI;
    std::priority_queue<GI, std::vector<GI>, std::greater<GI>> heap;   // (gen, ent) of batch entries
    size_t vp = 0;
    uint64_t count = c.live, ng = c.next_gen;
    for (uint32_t i = 0; i < n; ++i) {
        while (count >= M) {
            while (vp < victims.size() && pre.count(victims[vp].second)) ++vp;
            if (vp < victims.size()) {
                pre[victims[vp].second] = 1;
                ++vp;
                --count;
                continue;
            }
            bool evicted = false;
            while (!heap.empty()) {
                const GI top = heap.top();
                heap.pop();
                Ent& e = ents[top.second];
                if (!e.alive || e.gen != top.first) continue;
                e.alive = false;
                --count;
                evicted = true;
                break;
            }
            if (!evicted) return set_err(h, GD_ESTATE, "cache: nothing to evict at add %u (count %llu)", i,
                                         (unsigned long long)count);
        }
        const std::string key = cache_key(keys[i], hx.s[i], hx.len[i]);
        auto it = ent_of.find(key);
        if (it != ent_of.end() && ents[it->second].alive) {
            Ent& e = ents[it->second];
            e.act = vals[i].act;
            e.silo = vals[i].silo;
            e.ver = versions[i];
            e.gen = ++ng;
            heap.push({e.gen, it->second});
        } else if (it == ent_of.end() && slot_of[i] != NONE32 && !pre.count(slot_of[i])) {
            pre[slot_of[i]] = 2;
            ents.push_back(Ent{i, vals[i].act, vals[i].silo, versions[i], ++ng, slot_of[i], true});
            ent_of[key] = (uint32_t)ents.size() - 1;
            heap.push({ng, (uint32_t)ents.size() - 1});
        } else {
            ents.push_back(Ent{i, vals[i].act, vals[i].silo, versions[i], ++ng, NONE32, true});
            ent_of[key] = (uint32_t)ents.size() - 1;
            heap.push({ng, (uint32_t)ents.size() - 1});
            ++count;
        }
    }
    // 4. apply: tombstones and in-place updates, then the new entries (KeyExt strings into the heap)
    std::vector<CacheOp> ops;
    std::vector<gd_key> ins_keys;
    std::vector<CacheOp> ins;
    std::vector<uint32_t> ins_x;                         // {uh, len + 1, heap offset} per new entry
    std::vector<uint32_t> ins_item;
    bool any_x = false;
    uint64_t xbytes = 0;
    for (const auto& p : pre)
        if (p.second == 1) ops.push_back(CacheOp{p.first, 0, 0, 0, 0, 0, 0});
    for (const Ent& e : ents) {
        if (e.from_slot != NONE32)
            ops.push_back(e.alive ? CacheOp{e.from_slot, 1, e.act, e.silo, e.gen, e.ver, 0}
                                  : CacheOp{e.from_slot, 0, 0, 0, 0, 0, 0});
        else if (e.alive) {
            ins_keys.push_back(keys[e.item]);
            ins.push_back(CacheOp{NONE32, 1, e.act, e.silo, e.gen, e.ver, 0});
            ins_item.push_back(e.item);
            const int32_t len = hx.len[e.item];
            ins_x.push_back(len >= 0 ? hx.uh[e.item] : 0u);
            ins_x.push_back(len >= 0 ? (uint32_t)len + 1u : 0u);
            ins_x.push_back(0u);
            if (len >= 0) any_x = true;
            if (len > 0) xbytes += ((uint64_t)len + 15) & ~15ull;
        }
    }
    if (!ops.empty()) {
        GD_TRY(h2d(h, h->cbuf[4], ops.data(), ops.size()));
        GD_TRY(launch(h, "k_cache_apply", dim3(blocks_for(ops.size(), BLOCK)), dim3(BLOCK), 0, k_cache_apply,
                      (const CacheOp*)h->cbuf[4].p, (uint32_t)ops.size(), h->cslots, h->cctr));
    }
    if (xbytes) {                                        // after the evictions: their strings are dropped
        GD_TRY(cx_reserve(h, xbytes));
        std::vector<uint8_t> blob(xbytes, 0);
        uint64_t at = 0;
        for (size_t j = 0; j < ins.size(); ++j) {
            const uint32_t len1 = ins_x[3 * j + 1];
            if (len1 <= 1) continue;
            std::memcpy(blob.data() + at, hx.s[ins_item[j]], len1 - 1);
            ins_x[3 * j + 2] = (uint32_t)(h->cx_used + at);
            at += ((uint64_t)(len1 - 1) + 15) & ~15ull;
        }
        HIP_TRY(h, hipMemcpyAsync((uint8_t*)h->cx_heap.p + h->cx_used, blob.data(), xbytes, hipMemcpyHostToDevice,
                                  h->stream));
        GD_TRY(sync(h));                                 // blob is a host temporary
        h->cx_used += xbytes;
    }
    if (!ins.empty()) {
        GD_TRY(h2d(h, h->cbuf[3], ins_keys.data(), ins_keys.size()));
        GD_TRY(h2d(h, h->cbuf[5], ins.data(), ins.size()));
        if (any_x) GD_TRY(h2d(h, h->cbuf[6], ins_x.data(), ins_x.size()));
        GD_TRY(launch(h, "k_cache_insert", dim3(blocks_for(ins.size(), BLOCK)), dim3(BLOCK), 0, k_cache_insert,
                      (const gd_key*)h->cbuf[3].p, (const CacheOp*)h->cbuf[5].p,
                      any_x ? (const uint32_t*)h->cbuf[6].p : (const uint32_t*)nullptr, (uint32_t)ins.size(),
                      h->cslots, h->ccap - 1, h->cctr));
    }
    GD_TRY(sync(h));
    CacheCounters after{};
    GD_TRY(cache_pull(h, &after));
    after.next_gen = ng;
    HIP_TRY(h, hipMemcpyAsync(&h->cctr->next_gen, &after.next_gen, 8, hipMemcpyHostToDevice, h->stream));
    GD_TRY(sync(h));
    if (after.err) return set_err(h, GD_EFULL, "cache: device error bits 0x%x", after.err);
    if (after.live != count)
        return set_err(h, GD_ESTATE, "cache: %llu live entries after the batch, expected %llu",
                       (unsigned long long)after.live, (unsigned long long)count);
    return GD_OK;
}

// Remove (AdaptiveGrainDirectoryCache.cs:79-83 -> LRU.RemoveKey, LRU.cs:84-92).
int cache_remove_impl(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, uint8_t* out_removed) {
    GD_TRY(cache_check(h));
    if (n && !keys) return set_err(h, GD_EINVAL, "null argument");
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    HostExt hx;
    GD_TRY(host_ext_batch(h, keys, ext, n, &hx));
    std::vector<uint32_t> slot_of;
    GD_TRY(cache_find_batch(h, keys, ext, n, &slot_of));
    std::vector<CacheOp> ops;
    std::unordered_map<uint32_t, bool> seen;
    for (uint32_t i = 0; i < n; ++i) {
        const bool first = slot_of[i] != NONE32 && seen.emplace(slot_of[i], true).second;
        if (first) ops.push_back(CacheOp{slot_of[i], 0, 0, 0, 0, 0, 0});
        if (out_removed) out_removed[i] = first ? 1 : 0;
    }
    if (!ops.empty()) {
        GD_TRY(h2d(h, h->cbuf[6], ops.data(), ops.size()));
        GD_TRY(launch(h, "k_cache_apply", dim3(blocks_for(ops.size(), BLOCK)), dim3(BLOCK), 0, k_cache_apply,
                      (const CacheOp*)h->cbuf[6].p, (uint32_t)ops.size(), h->cslots, h->cctr));
    }
    return sync(h);
}

// LookUp in batch order (AdaptiveGrainDirectoryCache.cs:90-109).
int cache_lookup_impl(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, gd_val* out_vals,
                      int32_t* out_versions, uint8_t* out_found) {
    GD_TRY(cache_check(h));
    if (n && (!keys || !out_vals || !out_versions || !out_found)) return set_err(h, GD_EINVAL, "null argument");
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    HostExt hx;
    GD_TRY(host_ext_batch(h, keys, ext, n, &hx));       // validates the KeyExt items
    GD_TRY(h2d(h, h->cbuf[3], keys, n));
    ExtArgs x{};
    gd_key_ext dx{};
    if (ext) {
        GD_TRY(stage_ext(h, ext, n, &dx));
        x = ExtArgs{dx.bytes, dx.offset, dx.length, dx.bytes_len};
    }
    GD_TRY(ensure(h, h->cbuf[0], (size_t)n * 4));
    GD_TRY(ensure(h, h->cbuf[1], (size_t)n * 4));
    GD_TRY(ensure(h, h->cbuf[4], (size_t)n * sizeof(gd_val)));
    GD_TRY(ensure(h, h->cbuf[5], (size_t)n * 4));
    uint32_t* hit = (uint32_t*)h->cbuf[0].p;
    GD_TRY(launch(h, "k_cache_lookup", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), 0, k_cache_lookup,
                  (const gd_key*)h->cbuf[3].p, n, x, cache_args(h), (gd_val*)h->cbuf[4].p, (int32_t*)h->cbuf[5].p,
                  hit, (uint32_t*)h->cbuf[1].p));
    std::vector<uint32_t> found(n);
    HIP_TRY(h, hipMemcpyAsync(found.data(), hit, (size_t)n * 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipMemcpyAsync(out_vals, h->cbuf[4].p, (size_t)n * sizeof(gd_val), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipMemcpyAsync(out_versions, h->cbuf[5].p, (size_t)n * 4, hipMemcpyDeviceToHost, h->stream));
    GD_TRY(launch(h, "k_cache_count_access", dim3(1), dim3(64), 0, k_cache_count_access, n, h->cctr));
    GD_TRY(cache_touch(h, hit, (const uint32_t*)h->cbuf[1].p, n));
    GD_TRY(sync(h));
    for (uint32_t i = 0; i < n; ++i) out_found[i] = found[i] ? 1 : 0;
    return GD_OK;
}

}  // namespace

extern "C" {

int gd_cache_add(gd_handle* h, const gd_key* keys, const gd_val* vals, const int32_t* versions, uint32_t n) {
    return cache_add_impl(h, keys, nullptr, vals, versions, n);
}

int gd_cache_add_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, const gd_val* vals,
                     const int32_t* versions, uint32_t n) {
    if (!h || (n && !ext_ok(ext, n))) return set_err(h, GD_EINVAL, "null argument");
    return cache_add_impl(h, keys, ext, vals, versions, n);
}

int gd_cache_remove(gd_handle* h, const gd_key* keys, uint32_t n, uint8_t* out_removed) {
    return cache_remove_impl(h, keys, nullptr, n, out_removed);
}

int gd_cache_remove_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, uint8_t* out_removed) {
    if (!h || (n && !ext_ok(ext, n))) return set_err(h, GD_EINVAL, "null argument");
    return cache_remove_impl(h, keys, ext, n, out_removed);
}

int gd_cache_lookup(gd_handle* h, const gd_key* keys, uint32_t n, gd_val* out_vals, int32_t* out_versions,
                    uint8_t* out_found) {
    return cache_lookup_impl(h, keys, nullptr, n, out_vals, out_versions, out_found);
}

int gd_cache_lookup_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, gd_val* out_vals,
                        int32_t* out_versions, uint8_t* out_found) {
    if (!h || (n && !ext_ok(ext, n))) return set_err(h, GD_EINVAL, "null argument");
    return cache_lookup_impl(h, keys, ext, n, out_vals, out_versions, out_found);
}

int gd_cache_clear(gd_handle* h) {
    GD_TRY(cache_check(h));
    HIP_TRY(h, hipSetDevice(h->device));
    // LRU.Clear (:94-106) empties the dictionary; nextGeneration and the statistics stay
    HIP_TRY(h, hipMemsetAsync(h->cslots, 0, h->ccap * sizeof(CacheSlot), h->stream));
    h->cx_used = 0;
    CacheCounters c{};
    GD_TRY(cache_pull(h, &c));
    c.live = c.tomb = 0;
    c.max_probe = 0;
    HIP_TRY(h, hipMemcpyAsync(h->cctr, &c, sizeof c, hipMemcpyHostToDevice, h->stream));
    return sync(h);
}

int gd_cache_stats_get(gd_handle* h, gd_cache_stats* out) {
    GD_TRY(cache_check(h));
    if (!out) return set_err(h, GD_EINVAL, "null argument");
    HIP_TRY(h, hipSetDevice(h->device));
    CacheCounters c{};
    GD_TRY(cache_pull(h, &c));
    *out = gd_cache_stats{c.live, c.accesses, c.hits, c.next_gen, h->cache_max, h->ccap};
    return GD_OK;
}

}  // extern "C"

namespace {

// KeyValues (AdaptiveGrainDirectoryCache.cs:111-127) in slot order.  With ext_len: each entry's
// KeyExt length (GD_KEYEXT_NULL for a three-word key) and its string at ext_off[] in ext_bytes;
// *out_bytes = the bytes those strings need.  keys NULL = size query.
int cache_entries_impl(gd_handle* h, gd_key* keys, gd_val* vals, int32_t* versions, uint64_t* generations,
                       uint64_t capacity, uint64_t* out_n, int32_t* ext_len, uint64_t* ext_off, uint8_t* ext_bytes,
                       uint64_t bytes_capacity, uint64_t* out_bytes) {
    GD_TRY(cache_check(h));
    if (!out_n) return set_err(h, GD_EINVAL, "null argument");
    if (keys && (!vals || !versions || !generations)) return set_err(h, GD_EINVAL, "null output");
    const bool want_x = out_bytes != nullptr;
    if (want_x && keys && (!ext_len || !ext_off)) return set_err(h, GD_EINVAL, "null KeyExt output");
    HIP_TRY(h, hipSetDevice(h->device));
    if (h->ccap > 0x7FFFFFFFull) return set_err(h, GD_EINVAL, "cache table too large to dump");
    const uint32_t cap = (uint32_t)h->ccap;
    GD_TRY(ensure(h, h->cbuf[0], (size_t)cap * 4));
    GD_TRY(ensure(h, h->cbuf[2], (size_t)cap * 4));
    uint32_t* flag = (uint32_t*)h->cbuf[0].p;
    uint32_t* pos = (uint32_t*)h->cbuf[2].p;
    GD_TRY(launch(h, "k_cache_live_flag", dim3(blocks_for(cap, BLOCK)), dim3(BLOCK), 0, k_cache_live_flag,
                  (const CacheSlot*)h->cslots, cap, flag));
    GD_TRY(scan_device<OpAdd>(h, flag, cap, false, true, "cache", pos));
    uint32_t total = 0;
    HIP_TRY(h, hipMemcpyAsync(&total, pos + cap - 1, 4, hipMemcpyDeviceToHost, h->stream));
    GD_TRY(sync(h));
    *out_n = total;
    if (want_x) *out_bytes = 0;
    if ((!keys && !want_x) || total == 0) return GD_OK;
    if (keys && total > capacity)
        return set_err(h, GD_EINVAL, "cache holds %u entries, output holds %llu", total, (unsigned long long)capacity);
    GD_TRY(ensure(h, h->cbuf[7], (size_t)total * (sizeof(gd_key) + sizeof(gd_val) + 4 + 8 + 8) + 64));
    uint8_t* base = (uint8_t*)h->cbuf[7].p;
    gd_key* dk = (gd_key*)base;
    unsigned long long* dg = (unsigned long long*)(base + (size_t)total * sizeof(gd_key));
    gd_val* dv = (gd_val*)(dg + total);
    int32_t* dver = (int32_t*)(dv + total);
    uint32_t* dxl = (uint32_t*)(dver + total);
    uint32_t* dxo = dxl + total;
    GD_TRY(launch(h, "k_cache_dump", dim3(blocks_for(cap, BLOCK)), dim3(BLOCK), 0, k_cache_dump,
                  (const CacheSlot*)h->cslots, cap, (const uint32_t*)flag, (const uint32_t*)pos, dk, dv, dver, dg,
                  want_x ? dxl : (uint32_t*)nullptr, want_x ? dxo : (uint32_t*)nullptr));
    std::vector<uint32_t> xl, xo;
    if (want_x) {
        xl.resize(total);
        xo.resize(total);
        HIP_TRY(h, hipMemcpyAsync(xl.data(), dxl, (size_t)total * 4, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(h, hipMemcpyAsync(xo.data(), dxo, (size_t)total * 4, hipMemcpyDeviceToHost, h->stream));
    }
    if (keys) {
        HIP_TRY(h, hipMemcpyAsync(keys, dk, (size_t)total * sizeof(gd_key), hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(h, hipMemcpyAsync(vals, dv, (size_t)total * sizeof(gd_val), hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(h, hipMemcpyAsync(versions, dver, (size_t)total * 4, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(h, hipMemcpyAsync(generations, dg, (size_t)total * 8, hipMemcpyDeviceToHost, h->stream));
    }
    GD_TRY(sync(h));
    if (!want_x) return GD_OK;
    uint64_t need = 0;
    for (uint32_t k = 0; k < total; ++k) need += xl[k] > 1 ? xl[k] - 1 : 0;
    *out_bytes = need;
    if (!keys) return GD_OK;
    if (need > bytes_capacity || (need && !ext_bytes))
        return set_err(h, GD_EINVAL, "cache KeyExt strings need %llu bytes, output holds %llu",
                       (unsigned long long)need, (unsigned long long)bytes_capacity);
    std::vector<uint8_t> heap(h->cx_used);
    if (h->cx_used) {
        HIP_TRY(h, hipMemcpyAsync(heap.data(), h->cx_heap.p, h->cx_used, hipMemcpyDeviceToHost, h->stream));
        GD_TRY(sync(h));
    }
    uint64_t at = 0;
    for (uint32_t k = 0; k < total; ++k) {
        ext_len[k] = xl[k] ? (int32_t)(xl[k] - 1) : GD_KEYEXT_NULL;
        ext_off[k] = at;
        if (xl[k] > 1) {
            if ((uint64_t)xo[k] + xl[k] - 1 > heap.size()) return set_err(h, GD_ESTATE, "cache KeyExt heap offset");
            std::memcpy(ext_bytes + at, heap.data() + xo[k], xl[k] - 1);
            at += xl[k] - 1;
        }
    }
    return GD_OK;
}

}  // namespace

extern "C" {

int gd_cache_entries(gd_handle* h, gd_key* keys, gd_val* vals, int32_t* versions, uint64_t* generations,
                     uint64_t capacity, uint64_t* out_n) {
    return cache_entries_impl(h, keys, vals, versions, generations, capacity, out_n, nullptr, nullptr, nullptr, 0,
                              nullptr);
}

int gd_cache_entries_ext(gd_handle* h, gd_key* keys, gd_val* vals, int32_t* versions, uint64_t* generations,
                         int32_t* ext_len, uint64_t* ext_off, uint8_t* ext_bytes, uint64_t capacity,
                         uint64_t bytes_capacity, uint64_t* out_n, uint64_t* out_bytes) {
    if (!out_bytes) return set_err(h, GD_EINVAL, "null argument");
    return cache_entries_impl(h, keys, vals, versions, generations, capacity, out_n, ext_len, ext_off, ext_bytes,
                              bytes_capacity, out_bytes);
}

// ================================================================== in-library exchange (RCCL)
namespace {

#define NCCL_TRY(h, expr)                                                                          \
    do {                                                                                           \
        ncclResult_t r_ = (expr);                                                                  \
        if (r_ != ncclSuccess)                                                                     \
            return set_err((h), GD_ERCCL, "%s: %s", #expr, (h)->net->GetErrorString(r_));          \
    } while (0)

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
struct Lane {
    const void* send;
    void* recv;
    size_t elem;            // bytes per element
    ncclDataType_t type;
    size_t per;             // elements of `type` per element
    const uint64_t* sb = nullptr;   // set: per-peer byte ranges [sb[r], sb[r+1]) sent to r and
    const uint64_t* rb = nullptr;   // [rb[r], rb[r+1]) received from r (compact headers)
    const uint64_t* rsz = nullptr;  // set (with rb): bytes received from r at rb[r] (padded layouts)
};

int exchange_round(gd_handle* h, const char* name, const uint32_t* sc, const uint64_t* soff, const uint32_t* rc,
                   const uint64_t* roff, const Lane* lanes, int n_lanes) {
    const Rccl& R = *h->net;
    hipEvent_t a = nullptr, b = nullptr;
    if (h->timing) {
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
    if (h->timing) {
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
    if (!(flags & GD_MULTI_KEYS_READY)) {
        HIP_TRY(h, hipEventRecord(h->x_in, h->stream));
        HIP_TRY(h, hipStreamWaitEvent(h->pstream, h->x_in, 0));
    }
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

}  // namespace

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

// ================================================================== sharded fan-out cascade (SURVEY 8 f2 + 8 e)
// BASELINE cfg 4 across GPUs: ChirperAccount.PublishMessage (ChirperAccount.cs:106-147) on every
// rank for the publishers it owns; each NewChirp goes to its follower's directory owner over the
// library's communicator (OutboundMessageQueue.cs:54-131 per target silo), is routed there and
// enqueued on the follower's activation in arrival order (sender rank, sender emission order).
namespace {

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

}  // namespace

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

// ================================================================== KeyExt grains (gd_keyext.h)
namespace {

bool is_keyext_cat(uint64_t tcd) {
    const uint32_t c = (uint32_t)(tcd >> 56);
    return c == CAT_KEYEXT_GRAIN || c == CAT_GEO_CLIENT;
}

// UniqueKey.GetUniformHashCode of a KeyExt-category key (UniqueKey.cs:272-336).
uint32_t kx_hash_host(const gd_key& k, const uint8_t* s, int32_t len) {
    if (len < 0) return jenkins_u64x3(k.type_code_data, k.n0, k.n1);
    std::vector<uint8_t> b(28 + (size_t)len);
    std::memcpy(b.data(), &k.n0, 8);
    std::memcpy(b.data() + 8, &k.n1, 8);
    std::memcpy(b.data() + 16, &k.type_code_data, 8);
    std::memcpy(b.data() + 24, &len, 4);
    if (len) std::memcpy(b.data() + 28, s, (size_t)len);
    return jenkins_bytes(b.data(), b.size());
}

// Host view of message i's KeyExt (validated: GD_EINVAL for GD_KEYEXT_HOST or a bad range).
int host_ext(gd_handle* h, const gd_key_ext* ext, uint32_t i, const uint8_t*& s, int32_t& len) {
    len = ext->length[i];
    s = nullptr;
    if (len == GD_KEYEXT_NULL) return GD_OK;
    if (len < 0) return set_err(h, GD_EINVAL, "item %u: KeyExt length %d (GD_KEYEXT_HOST is for routing only)", i, len);
    const uint64_t off = ext->offset[i];
    if (off > ext->bytes_len || (uint64_t)len > ext->bytes_len - off)
        return set_err(h, GD_EINVAL, "item %u: KeyExt [%llu, +%d) outside the %llu-byte buffer", i,
                       (unsigned long long)off, len, (unsigned long long)ext->bytes_len);
    s = ext->bytes + off;
    return GD_OK;
}

// Probe the host index: the live equal entry, else the first reusable slot on the way.
bool kx_find_host(gd_handle* h, const gd_key& k, const uint8_t* s, int32_t len, uint32_t uh, uint64_t* at,
                  uint64_t* free_at, uint32_t* dist) {
    const uint64_t mask = h->kx_cap - 1;
    uint64_t i = fmix32(uh) & mask;
    *free_at = UINT64_MAX;
    for (uint64_t p = 0; p < h->kx_cap; ++p, i = (i + 1) & mask) {
        const KxSlot& q = h->kx_m[i];
        const uint32_t st = slot_state(q.meta);
        if (st == SLOT_EMPTY) {
            if (*free_at == UINT64_MAX) {
                *free_at = i;
                *dist = (uint32_t)p;
            }
            return false;
        }
        if (st == SLOT_TOMB) {
            if (*free_at == UINT64_MAX) {
                *free_at = i;
                *dist = (uint32_t)p;
            }
            continue;
        }
        if (q.uhash == uh && q.len == len && q.n0 == k.n0 && q.n1 == k.n1 && q.tcd == k.type_code_data &&
            (len <= 0 || (len <= KX_INLINE ? kx_inline_eq(q, s, len)
                                           : std::memcmp(h->kx_hheap.data() + q.off, s, (size_t)len) == 0))) {
            *at = i;
            return true;
        }
    }
    return false;
}

int kx_upload_all(gd_handle* h) {
    if (h->kx_slots) {
        HIP_TRY(h, hipStreamSynchronize(h->stream));
        HIP_TRY(h, hipFree(h->kx_slots));
        h->kx_slots = nullptr;
    }
    hipError_t e = hipMalloc((void**)&h->kx_slots, h->kx_cap * sizeof(KxSlot));
    if (e != hipSuccess) return set_err(h, GD_ENOMEM, "KeyExt table (%llu slots): %s",
                                        (unsigned long long)h->kx_cap, hipGetErrorString(e));
    HIP_TRY(h, hipMemcpyAsync(h->kx_slots, h->kx_m.data(), h->kx_cap * sizeof(KxSlot), hipMemcpyHostToDevice,
                              h->stream));
    GD_TRY(ensure(h, h->kx_heap, std::max<size_t>(2 * h->kx_hheap.size(), 1 << 16)));   // room to append
    if (!h->kx_hheap.empty())
        HIP_TRY(h, hipMemcpyAsync(h->kx_heap.p, h->kx_hheap.data(), h->kx_hheap.size(), hipMemcpyHostToDevice,
                                  h->stream));
    h->kx_heap_dev = h->kx_hheap.size();
    h->layout_gen++;
    return sync(h);
}

// Rebuild the host index at cap slots (tombstones dropped, heap compacted), then upload it whole.
int kx_rehash(gd_handle* h, uint64_t cap) {
    std::vector<KxSlot> old;
    old.swap(h->kx_m);
    std::vector<uint8_t> old_heap;
    old_heap.swap(h->kx_hheap);
    h->kx_cap = cap;
    h->kx_m.assign(cap, KxSlot{});
    h->kx_live = h->kx_tomb = 0;
    h->kx_maxp = 0;
    const uint64_t mask = cap - 1;
    for (const KxSlot& q : old) {
        if (slot_state(q.meta) != SLOT_LIVE) continue;
        KxSlot v = q;
        if (q.len > KX_INLINE) {
            h->kx_hheap.resize((h->kx_hheap.size() + 15) & ~(size_t)15, 0);
            v.off = h->kx_hheap.size();
            h->kx_hheap.insert(h->kx_hheap.end(), old_heap.begin() + q.off, old_heap.begin() + q.off + q.len);
        }
        uint64_t i = fmix32(q.uhash) & mask;
        uint32_t p = 0;
        while (slot_state(h->kx_m[i].meta) != SLOT_EMPTY) {
            i = (i + 1) & mask;
            ++p;
        }
        h->kx_m[i] = v;
        h->kx_maxp = std::max(h->kx_maxp, p);
        h->kx_live++;
    }
    return kx_upload_all(h);
}

// Push the host index changes: new heap bytes, then the changed slots.
int kx_commit(gd_handle* h, std::vector<uint64_t>& dirty) {
    if (h->kx_hheap.size() > h->kx_heap.bytes) {
        std::sort(dirty.begin(), dirty.end());
        return kx_upload_all(h);   // the device heap grows: upload table + heap whole
    }
    if (h->kx_hheap.size() > h->kx_heap_dev) {
        HIP_TRY(h, hipMemcpyAsync((uint8_t*)h->kx_heap.p + h->kx_heap_dev, h->kx_hheap.data() + h->kx_heap_dev,
                                  h->kx_hheap.size() - h->kx_heap_dev, hipMemcpyHostToDevice, h->stream));
        h->kx_heap_dev = h->kx_hheap.size();
    }
    std::sort(dirty.begin(), dirty.end());
    dirty.erase(std::unique(dirty.begin(), dirty.end()), dirty.end());
    const uint32_t m = (uint32_t)dirty.size();
    if (m == 0) return sync(h);
    if ((uint64_t)m * 4 > h->kx_cap) {
        HIP_TRY(h, hipMemcpyAsync(h->kx_slots, h->kx_m.data(), h->kx_cap * sizeof(KxSlot), hipMemcpyHostToDevice,
                                  h->stream));
        return sync(h);
    }
    std::vector<KxSlot> vals(m);
    for (uint32_t j = 0; j < m; ++j) vals[j] = h->kx_m[dirty[j]];
    GD_TRY(h2d(h, h->kx_buf[0], dirty.data(), m));
    GD_TRY(h2d(h, h->kx_buf[1], vals.data(), m));
    GD_TRY(launch(h, "k_kx_apply", dim3(blocks_for(m, BLOCK)), dim3(BLOCK), 0, k_kx_apply,
                  (const uint64_t*)h->kx_buf[0].p, (const KxSlot*)h->kx_buf[1].p, m, h->kx_slots));
    return sync(h);
}

// Route (24-B keys) then the KeyExt pass over what it left at GD_ROUTE_KEYEXT.
int route_ext_device(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, uint32_t* silo,
                     uint32_t* act, uint8_t* st) {
    GD_TRY(route_device(h, keys, n, silo, act, st, !ext));
    if (!ext || n == 0) return GD_OK;
    return keyext_pass(h, keys, ExtArgs{ext->bytes, ext->offset, ext->length, ext->bytes_len}, n, silo, act, st);
}

// Host ext -> device copies in kx_buf[2..4]; *dx gets the device form.
int stage_ext(gd_handle* h, const gd_key_ext* ext, uint32_t n, gd_key_ext* dx) {
    GD_TRY(h2d(h, h->kx_buf[2], ext->bytes, (size_t)ext->bytes_len));
    GD_TRY(h2d(h, h->kx_buf[3], ext->offset, n));
    GD_TRY(h2d(h, h->kx_buf[4], ext->length, n));
    *dx = gd_key_ext{(const uint8_t*)h->kx_buf[2].p, (const uint64_t*)h->kx_buf[3].p,
                     (const int32_t*)h->kx_buf[4].p, ext->bytes_len};
    return GD_OK;
}

bool ext_ok(const gd_key_ext* ext, uint32_t n) {
    return !ext || n == 0 || (ext->offset && ext->length && (ext->bytes || ext->bytes_len == 0));
}

}  // namespace

int gd_dir_register_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, const gd_val* vals, uint32_t n,
                        gd_val* out_vals, uint8_t* out_inserted) {
    if (!h || (n && (!keys || !ext || !vals || !ext_ok(ext, n)))) return set_err(h, GD_EINVAL, "null argument");
    HIP_TRY(h, hipSetDevice(h->device));
    std::vector<uint32_t> uh(n);
    for (uint32_t i = 0; i < n; ++i) {
        if (!is_keyext_cat(keys[i].type_code_data))
            return set_err(h, GD_EINVAL, "item %u: category %u has no KeyExt (use gd_dir_register)", i,
                           (unsigned)(keys[i].type_code_data >> 56));
        const uint8_t* s;
        int32_t len;
        GD_TRY(host_ext(h, ext, i, s, len));
        uh[i] = kx_hash_host(keys[i], s, len);
    }
    if (h->kx_cap == 0 || (h->kx_live + h->kx_tomb + n) * 2 > h->kx_cap) {
        uint64_t cap = std::max<uint64_t>(h->kx_cap, 1024);
        while ((h->kx_live + n) * 2 > cap) cap *= 2;
        GD_TRY(kx_rehash(h, cap));
    }
    std::vector<uint64_t> dirty;
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t* s;
        int32_t len;
        GD_TRY(host_ext(h, ext, i, s, len));
        uint64_t at = 0, free_at = 0;
        uint32_t dist = 0;
        if (!host_silo_valid(h, vals[i].silo)) {    // AddSingleActivation's IsValidSilo check (:310-311)
            if (out_vals) out_vals[i] = gd_val{NONE32, NONE32};
            if (out_inserted) out_inserted[i] = 0;
            continue;
        }
        if (kx_find_host(h, keys[i], s, len, uh[i], &at, &free_at, &dist)) {     // first registration wins
            if (out_vals) out_vals[i] = gd_val{h->kx_m[at].act, slot_silo(h->kx_m[at].meta)};
            if (out_inserted) out_inserted[i] = 0;
            continue;
        }
        if (free_at == UINT64_MAX) return set_err(h, GD_EFULL, "KeyExt table full");
        KxSlot& q = h->kx_m[free_at];
        if (slot_state(q.meta) == SLOT_TOMB) h->kx_tomb--;
        q = KxSlot{};
        q.n0 = keys[i].n0;
        q.n1 = keys[i].n1;
        q.tcd = keys[i].type_code_data;
        q.len = len;
        q.uhash = uh[i];
        q.act = vals[i].act;
        q.meta = make_meta(SLOT_LIVE, vals[i].silo);
        if (len > 0 && len <= KX_INLINE) {
            kx_inline_put(q, s, len);
        } else if (len > 0) {          // 16-B aligned entries: the device compares them word by word
            h->kx_hheap.resize((h->kx_hheap.size() + 15) & ~(size_t)15, 0);
            q.off = h->kx_hheap.size();
            h->kx_hheap.insert(h->kx_hheap.end(), s, s + len);
        }
        h->kx_live++;
        h->kx_maxp = std::max(h->kx_maxp, dist);
        dirty.push_back(free_at);
        if (out_vals) out_vals[i] = vals[i];
        if (out_inserted) out_inserted[i] = 1;
    }
    return kx_commit(h, dirty);
}

int gd_dir_unregister_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, const uint32_t* acts, uint32_t n,
                          uint8_t* out_removed) {
    if (!h || (n && (!keys || !ext || !acts || !ext_ok(ext, n)))) return set_err(h, GD_EINVAL, "null argument");
    HIP_TRY(h, hipSetDevice(h->device));
    std::vector<uint64_t> dirty;
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t* s;
        int32_t len;
        GD_TRY(host_ext(h, ext, i, s, len));
        uint64_t at = 0, free_at = 0;
        uint32_t dist = 0;
        bool removed = false;
        if (h->kx_cap && kx_find_host(h, keys[i], s, len, kx_hash_host(keys[i], s, len), &at, &free_at, &dist) &&
            h->kx_m[at].act == acts[i]) {          // RemoveActivation: only the matching activation
            h->kx_m[at].meta = make_meta(SLOT_TOMB, slot_silo(h->kx_m[at].meta));
            h->kx_live--;
            h->kx_tomb++;
            dirty.push_back(at);
            removed = true;
        }
        if (out_removed) out_removed[i] = removed ? 1 : 0;
    }
    return kx_commit(h, dirty);
}

int gd_dir_lookup_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, gd_val* out_vals,
                      uint8_t* out_found) {
    if (!h || (n && (!keys || !ext || !out_vals || !out_found || !ext_ok(ext, n))))
        return set_err(h, GD_EINVAL, "null argument");
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t* s;
        int32_t len;
        GD_TRY(host_ext(h, ext, i, s, len));
    }
    gd_key_ext dx;
    GD_TRY(h2d(h, h->keys_in, keys, n));
    GD_TRY(stage_ext(h, ext, n, &dx));
    GD_TRY(ensure(h, h->out_a, (size_t)n * sizeof(gd_val)));
    GD_TRY(ensure(h, h->out_c, (size_t)n));
    const ExtArgs x{dx.bytes, dx.offset, dx.length, dx.bytes_len};
    GD_TRY(launch(h, "k_kx_lookup", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), 0, k_kx_lookup,
                  (const gd_key*)h->keys_in.p, n, x, kx_args(h), (gd_val*)h->out_a.p, (uint8_t*)h->out_c.p));
    GD_TRY(d2h(h, out_vals, h->out_a, n));
    GD_TRY(d2h(h, out_found, h->out_c, n));
    return sync(h);
}

int gd_dir_ext_stats(gd_handle* h, uint64_t* live, uint64_t* capacity, uint64_t* heap_bytes) {
    if (!h) return set_err(nullptr, GD_EINVAL, "null handle");
    if (live) *live = h->kx_live;
    if (capacity) *capacity = h->kx_cap;
    if (heap_bytes) *heap_bytes = h->kx_hheap.size();
    return GD_OK;
}

int gd_route_ext_device(gd_handle* h, const gd_key* d_keys, const gd_key_ext* d_ext, uint32_t n, uint32_t* d_silo,
                        uint32_t* d_act, uint8_t* d_status) {
    if (!h || (n && (!d_keys || !d_silo || !d_act || !d_status || !ext_ok(d_ext, n))))
        return set_err(h, GD_EINVAL, "null argument");
    return n ? route_ext_device(h, d_keys, d_ext, n, d_silo, d_act, d_status) : GD_OK;
}

int gd_route_bucket_ext_device(gd_handle* h, const gd_key* d_keys, const gd_key_ext* d_ext, uint32_t n,
                               uint32_t n_act, uint32_t* d_silo, uint32_t* d_act, uint8_t* d_status,
                               uint32_t* d_perm, uint32_t* d_offsets) {
    if (!h || !d_offsets || (n && (!d_keys || !d_silo || !d_act || !d_status || !d_perm || !ext_ok(d_ext, n))))
        return set_err(h, GD_EINVAL, "null argument");
    if (n) GD_TRY(route_ext_device(h, d_keys, d_ext, n, d_silo, d_act, d_status));
    return bucket_device(h, d_act, n, n_act, d_perm, d_offsets);
}

int gd_route_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, uint32_t* out_silo,
                 uint32_t* out_act, uint8_t* out_status) {
    if (!h || (n && (!keys || !out_silo || !out_act || !out_status || !ext_ok(ext, n))))
        return set_err(h, GD_EINVAL, "null argument");
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    gd_key_ext dx{};
    GD_TRY(h2d(h, h->keys_in, keys, n));
    if (ext) GD_TRY(stage_ext(h, ext, n, &dx));
    GD_TRY(ensure(h, h->out_a, (size_t)n * 4));
    GD_TRY(ensure(h, h->out_b, (size_t)n * 4));
    GD_TRY(ensure(h, h->out_c, (size_t)n));
    GD_TRY(route_ext_device(h, (const gd_key*)h->keys_in.p, ext ? &dx : nullptr, n, (uint32_t*)h->out_a.p,
                            (uint32_t*)h->out_b.p, (uint8_t*)h->out_c.p));
    GD_TRY(d2h(h, out_silo, h->out_a, n));
    GD_TRY(d2h(h, out_act, h->out_b, n));
    GD_TRY(d2h(h, out_status, h->out_c, n));
    return sync(h);
}

int gd_route_bucket_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, uint32_t n_act,
                        uint32_t* out_silo, uint32_t* out_act, uint8_t* out_status, uint32_t* out_perm,
                        uint32_t* out_offsets) {
    if (!h || !out_offsets || (n && (!keys || !out_silo || !out_act || !out_status || !out_perm || !ext_ok(ext, n))))
        return set_err(h, GD_EINVAL, "null argument");
    if (n_act == 0xFFFFFFFFu) return set_err(h, GD_EINVAL, "n_act too large");
    HIP_TRY(h, hipSetDevice(h->device));
    gd_key_ext dx{};
    GD_TRY(h2d(h, h->keys_in, keys, n));
    if (ext && n) GD_TRY(stage_ext(h, ext, n, &dx));
    GD_TRY(ensure(h, h->out_a, (size_t)n * 4 + 4));
    GD_TRY(ensure(h, h->out_b, (size_t)n * 4 + 4));
    GD_TRY(ensure(h, h->out_c, (size_t)n + 4));
    GD_TRY(ensure(h, h->u8_a, (size_t)n * 4 + 4));   // perm
    GD_TRY(ensure(h, h->offs, ((size_t)n_act + 2) * 4));
    if (n)
        GD_TRY(route_ext_device(h, (const gd_key*)h->keys_in.p, ext ? &dx : nullptr, n, (uint32_t*)h->out_a.p,
                                (uint32_t*)h->out_b.p, (uint8_t*)h->out_c.p));
    GD_TRY(bucket_device(h, (const uint32_t*)h->out_b.p, n, n_act, (uint32_t*)h->u8_a.p, (uint32_t*)h->offs.p));
    GD_TRY(d2h(h, out_silo, h->out_a, n));
    GD_TRY(d2h(h, out_act, h->out_b, n));
    GD_TRY(d2h(h, out_status, h->out_c, n));
    GD_TRY(d2h(h, out_perm, h->u8_a, n));
    GD_TRY(d2h(h, out_offsets, h->offs, (size_t)n_act + 2));
    return sync_checked(h);
}

int gd_uniform_hashes_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, uint32_t* out) {
    if (!h || (n && (!keys || !ext || !out || !ext_ok(ext, n)))) return set_err(h, GD_EINVAL, "null argument");
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    gd_key_ext dx;
    GD_TRY(h2d(h, h->keys_in, keys, n));
    GD_TRY(stage_ext(h, ext, n, &dx));
    GD_TRY(ensure(h, h->out_a, (size_t)n * 4));
    const ExtArgs x{dx.bytes, dx.offset, dx.length, dx.bytes_len};
    GD_TRY(launch(h, "k_kx_hash", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), 0, k_kx_hash, (const gd_key*)h->keys_in.p,
                  n, x, (uint32_t*)h->out_a.p));
    GD_TRY(d2h(h, out, h->out_a, n));
    return sync(h);
}

int gd_ring_owner_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, uint32_t* out_silo) {
    if (!h || (n && (!keys || !ext || !out_silo || !ext->offset || !ext->length)))
        return set_err(h, GD_EINVAL, "null argument");
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(check_ring(h));
    gd_key_ext dx;
    GD_TRY(h2d(h, h->keys_in, keys, n));
    GD_TRY(stage_ext(h, ext, n, &dx));
    GD_TRY(ensure(h, h->out_a, (size_t)n * 4));
    const ExtArgs x{dx.bytes, dx.offset, dx.length, dx.bytes_len};
    const gd_key* k = (const gd_key*)h->keys_in.p;
    uint32_t* o = (uint32_t*)h->out_a.p;
    const dim3 g(blocks_for(n, BLOCK)), b(BLOCK);
    if (h->ring_mode == GD_RING_DIRECTORY)
        GD_TRY(launch(h, "k_owner_ext", g, b, ring_lds(h), k_owner_ext<GD_RING_DIRECTORY>, k, n, ring_args(h), x, o));
    else if (h->ring_mode == GD_RING_CONSISTENT)
        GD_TRY(launch(h, "k_owner_ext", g, b, ring_lds(h), k_owner_ext<GD_RING_CONSISTENT>, k, n, ring_args(h), x, o));
    else
        GD_TRY(launch(h, "k_owner_ext", g, b, ring_lds(h), k_owner_ext<GD_RING_VIRTUAL_BUCKETS>, k, n, ring_args(h), x,
                      o));
    GD_TRY(d2h(h, out_silo, h->out_a, n));
    return sync(h);
}


int gd_dir_split_ext(gd_handle* h, const uint8_t* keep_silo, uint32_t n_keep, int move, gd_key* out_keys,
                     gd_val* out_vals, uint64_t* out_offset, int32_t* out_length, uint8_t* out_bytes,
                     uint64_t capacity, uint64_t bytes_capacity, uint64_t* out_n, uint64_t* out_nbytes) {
    if (!h || !out_n || !out_nbytes || (n_keep && !keep_silo)) return set_err(h, GD_EINVAL, "null argument");
    if (out_keys && (!out_vals || !out_offset || !out_length || !out_bytes))
        return set_err(h, GD_EINVAL, "keys, vals, offsets, lengths and bytes go together");
    *out_n = *out_nbytes = 0;
    if (h->kx_live == 0) return GD_OK;
    // owners of the live entries' stored uniform hashes under the installed ring (slot order)
    std::vector<uint64_t> live;
    std::vector<uint32_t> hashes;
    for (uint64_t i = 0; i < h->kx_cap; ++i)
        if (slot_state(h->kx_m[i].meta) == SLOT_LIVE) {
            live.push_back(i);
            hashes.push_back(h->kx_m[i].uhash);
        }
    std::vector<uint32_t> owner(live.size());
    GD_TRY(gd_ring_lookup_hashes(h, hashes.data(), (uint32_t)live.size(), owner.data()));
    std::vector<uint64_t> sel;
    uint64_t nbytes = 0;
    for (size_t j = 0; j < live.size(); ++j) {
        const bool kept = owner[j] < n_keep && keep_silo[owner[j]];
        if (kept) continue;
        sel.push_back(live[j]);
        nbytes += (uint64_t)std::max(0, h->kx_m[live[j]].len);
    }
    *out_n = sel.size();
    *out_nbytes = nbytes;
    if (!out_keys || sel.empty()) return GD_OK;
    if (sel.size() > capacity || nbytes > bytes_capacity)
        return set_err(h, GD_EINVAL, "split selects %llu entries / %llu bytes, output holds %llu / %llu",
                       (unsigned long long)sel.size(), (unsigned long long)nbytes, (unsigned long long)capacity,
                       (unsigned long long)bytes_capacity);
    uint64_t pos = 0;
    std::vector<uint64_t> dirty;
    for (size_t j = 0; j < sel.size(); ++j) {
        KxSlot& q = h->kx_m[sel[j]];
        out_keys[j] = gd_key{q.n0, q.n1, q.tcd};
        out_vals[j] = gd_val{q.act, slot_silo(q.meta)};
        out_length[j] = q.len;
        out_offset[j] = pos;
        if (q.len > 0) {
            if (q.len <= KX_INLINE) {
                uint8_t b[KX_INLINE];
                std::memcpy(b, &q.off, 8);
                std::memcpy(b + 8, q.tail, 16);
                std::memcpy(out_bytes + pos, b, (size_t)q.len);
            } else {
                std::memcpy(out_bytes + pos, h->kx_hheap.data() + q.off, (size_t)q.len);
            }
            pos += (uint64_t)q.len;
        }
        if (move) {                    // the RemoveGrain after RegisterMany (GrainDirectoryHandoffManager.cs:228-232)
            q.meta = make_meta(SLOT_TOMB, slot_silo(q.meta));
            h->kx_live--;
            h->kx_tomb++;
            dirty.push_back(sel[j]);
        }
    }
    return move ? kx_commit(h, dirty) : GD_OK;
}
}  // extern "C"

// ================================================================== membership churn: IsValidSilo, VersionTag,
// silo removal, handoff merge (gd_dirops.h)
namespace {

int set_bitset(gd_handle* h, DevBuf& b, const std::vector<uint32_t>& bits) {
    GD_TRY(h2d(h, b, bits.data(), bits.size()));
    return GD_OK;
}

// Room for activation indices [0, need) in the index -> ActivationId map, keeping the ids set.
int grow_act_ids(gd_handle* h, uint64_t need) {
    if (need <= h->n_act_ids) return GD_OK;
    DevBuf nb;
    size_t cap = std::max<size_t>(need, 2 * h->n_act_ids) * sizeof(gd_key);
    GD_TRY(ensure(h, nb, cap));
    HIP_TRY(h, hipMemsetAsync(nb.p, 0, cap, h->stream));
    if (h->n_act_ids)
        HIP_TRY(h, hipMemcpyAsync(nb.p, h->act_ids.p, h->n_act_ids * sizeof(gd_key), hipMemcpyDeviceToDevice,
                                  h->stream));
    GD_TRY(sync(h));
    free_buf(h->act_ids);
    h->act_ids = nb;
    h->n_act_ids = cap / sizeof(gd_key);
    return GD_OK;
}

int check_dir_err(gd_handle* h, const char* what) {
    GD_TRY(pull_counters(h));
    if (h->ctr_host.err) {
        const uint32_t e = h->ctr_host.err;
        HIP_TRY(h, hipMemsetAsync(&h->ctr->err, 0, sizeof(uint32_t), h->stream));
        GD_TRY(sync(h));
        if (e & 2) return set_err(h, GD_EFULL, "%s: table full (0x%x)", what, e);
        if (e & 8) return set_err(h, GD_EINVAL, "%s: a grain appears twice in one merge batch (0x%x)", what, e);
        if (e & 16) return set_err(h, GD_EINVAL, "%s: an activation index has no ActivationId (gd_activation_ids_set) (0x%x)", what, e);
        return set_err(h, GD_EINVAL, "%s: device error bits 0x%x", what, e);
    }
    return GD_OK;
}

// GrainDirectoryPartition.Merge over device arrays (one item per grain): claims, the duplicate
// check, then k_merge_apply.  Synchronous up to the apply (which stays enqueued); errors through
// check_dir_err.
int merge_core(gd_handle* h, const gd_key* dk, const gd_val* dvals, const int32_t* dtags, uint32_t n,
               uint8_t* d_status, gd_val* d_dropped) {
    GD_TRY(maybe_grow_table(h, n));
    const uint32_t op = ++h->dir_op;
    GD_TRY(ensure(h, h->u32_a, (size_t)n * 4));   // slot_of
    GD_TRY(ensure(h, h->u8_a, (size_t)n));        // is_new
    if (h->up_last.bytes < h->capacity * 4) {
        GD_TRY(ensure(h, h->up_last, h->capacity * 4));
        HIP_TRY(h, hipMemsetAsync(h->up_last.p, 0, h->up_last.bytes, h->stream));
    }
    HIP_TRY(h, hipMemsetAsync(h->u8_a.p, 0, n, h->stream));
    const dim3 g(blocks_for(n, BLOCK)), b(BLOCK);
    uint32_t* slot_of = (uint32_t*)h->u32_a.p;
    uint8_t* is_new = (uint8_t*)h->u8_a.p;
    for (uint32_t pass = 0;; ++pass) {            // the registration's claim protocol; no IsValidSilo check in Merge
        HIP_TRY(h, hipMemsetAsync(&h->ctr->retry, 0, sizeof(uint32_t), h->stream));
        GD_TRY(launch(h, "k_reg_claim", g, b, 0, k_reg_claim, dk, n, h->slots, h->capacity - 1, h->ctr, slot_of,
                      is_new, (uint32_t)(pass > 0), (const gd_val*)nullptr, table_args(h)));
        GD_TRY(pull_counters(h));
        if (h->ctr_host.retry == 0 || h->ctr_host.err) break;
        if (pass >= 64) return set_err(h, GD_ETIMEOUT, "gd_dir_merge: claims did not settle");
    }
    uint32_t* last = (uint32_t*)h->up_last.p;
    GD_TRY(launch(h, "k_dup_mark", g, b, 0, k_dup_mark, (const uint32_t*)slot_of, n, last, h->ctr));
    GD_TRY(launch(h, "k_up_clear", g, b, 0, k_up_clear, (const uint32_t*)slot_of, n, last));
    GD_TRY(pull_counters(h));
    if (h->ctr_host.err) {
        // a duplicated grain: the pending claims of this batch must not stay half-made
        GD_TRY(launch(h, "k_reg_abort", g, b, 0, k_reg_abort, (const uint32_t*)slot_of, (const uint8_t*)is_new, n,
                      h->slots, h->ctr));
        return check_dir_err(h, "gd_dir_merge");
    }
    return launch(h, "k_merge_apply", g, b, 0, k_merge_apply, dk, dvals, dtags, n, (const uint32_t*)slot_of,
                  (const uint8_t*)is_new, h->slots, h->vtag, h->ctr, (const gd_key*)h->act_ids.p,
                  (unsigned long long)h->n_act_ids, op, d_status, d_dropped);
}

}  // namespace

extern "C" {

int gd_dir_set_valid_silos(gd_handle* h, const uint8_t* valid, uint32_t n_silos) {
    if (!h || (n_silos && !valid)) return set_err(h, GD_EINVAL, "null argument");
    if (n_silos > 0x10000u) return set_err(h, GD_EINVAL, "n_silos %u above 65536", n_silos);
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(sync(h));
    std::vector<uint32_t> bits((n_silos + 31) / 32 + 1, 0);
    h->valid_host.assign(valid, valid + n_silos);
    for (uint32_t s = 0; s < n_silos; ++s)
        if (valid[s]) bits[s >> 5] |= 1u << (s & 31);
    GD_TRY(set_bitset(h, h->dir_valid, bits));
    GD_TRY(sync(h));
    h->n_valid = n_silos;
    h->layout_gen++;                  // captured micro-batch graphs bake TableArgs in
    return GD_OK;
}

int gd_dir_lookup_tagged(gd_handle* h, const gd_key* keys, uint32_t n, gd_val* out_vals, int32_t* out_tags,
                         uint8_t* out_found) {
    if (!h || (n && (!keys || !out_vals || !out_tags || !out_found))) return set_err(h, GD_EINVAL, "null argument");
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(h2d(h, h->keys_in, keys, n));
    GD_TRY(ensure(h, h->dirop_buf[0], (size_t)n * sizeof(gd_val)));
    GD_TRY(ensure(h, h->dirop_buf[1], (size_t)n * 4));
    GD_TRY(ensure(h, h->dirop_buf[2], (size_t)n));
    GD_TRY(launch(h, "k_dir_lookup_tagged", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), 0, k_dir_lookup_tagged,
                  (const gd_key*)h->keys_in.p, n, table_args(h), (const uint32_t*)h->vtag, (gd_val*)h->dirop_buf[0].p,
                  (int32_t*)h->dirop_buf[1].p, (uint8_t*)h->dirop_buf[2].p));
    HIP_TRY(h, hipMemcpyAsync(out_vals, h->dirop_buf[0].p, (size_t)n * sizeof(gd_val), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipMemcpyAsync(out_tags, h->dirop_buf[1].p, (size_t)n * 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipMemcpyAsync(out_found, h->dirop_buf[2].p, n, hipMemcpyDeviceToHost, h->stream));
    return sync(h);
}

int gd_dir_remove_silos(gd_handle* h, const uint32_t* silos, uint32_t n_silos, uint64_t* out_removed,
                        uint64_t* out_multi, uint64_t* out_cache_removed) {
    if (!h || (n_silos && !silos)) return set_err(h, GD_EINVAL, "null argument");
    HIP_TRY(h, hipSetDevice(h->device));
    std::vector<uint32_t> bits(0x10000 / 32, 0);
    for (uint32_t i = 0; i < n_silos; ++i) {
        if (silos[i] > 0xFFFEu) return set_err(h, GD_EINVAL, "silo index %u out of range", silos[i]);
        bits[silos[i] >> 5] |= 1u << (silos[i] & 31);
    }
    GD_TRY(set_bitset(h, h->dirop_buf[3], bits));
    GD_TRY(ensure(h, h->dirop_buf[2], 32));
    unsigned long long* cnt = (unsigned long long*)h->dirop_buf[2].p;
    HIP_TRY(h, hipMemsetAsync(cnt, 0, 32, h->stream));
    const uint32_t* set = (const uint32_t*)h->dirop_buf[3].p;
    GD_TRY(launch(h, "k_dir_remove_silos", dim3((uint32_t)((h->capacity + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0,
                  k_dir_remove_silos, h->slots, h->capacity, set, h->ctr, cnt));
    if (h->cache_max) {               // AdjustLocalCache under the installed (post-removal) ring
        GD_TRY(check_ring(h));
        const dim3 g((uint32_t)((h->ccap + BLOCK - 1) / BLOCK)), b(BLOCK);
        const RingArgs r = ring_args(h);
        const uint8_t* loc = (const uint8_t*)h->cache_local.p;
        switch (h->ring_mode) {
            case GD_RING_DIRECTORY:
                GD_TRY(launch(h, "k_cache_adjust", g, b, ring_lds(h), k_cache_adjust<GD_RING_DIRECTORY>, h->cslots,
                              h->ccap, r, loc, h->cache_nsilos, set, h->cctr, cnt));
                break;
            case GD_RING_CONSISTENT:
                GD_TRY(launch(h, "k_cache_adjust", g, b, ring_lds(h), k_cache_adjust<GD_RING_CONSISTENT>, h->cslots,
                              h->ccap, r, loc, h->cache_nsilos, set, h->cctr, cnt));
                break;
            default:
                GD_TRY(launch(h, "k_cache_adjust", g, b, ring_lds(h), k_cache_adjust<GD_RING_VIRTUAL_BUCKETS>, h->cslots,
                              h->ccap, r, loc, h->cache_nsilos, set, h->cctr, cnt));
        }
    }
    unsigned long long c[4] = {0, 0, 0, 0};
    HIP_TRY(h, hipMemcpyAsync(c, cnt, 32, hipMemcpyDeviceToHost, h->stream));
    GD_TRY(sync(h));
    // KeyExt entries live in the host index: the same rule there
    std::vector<uint64_t> dirty;
    for (uint64_t j = 0; j < h->kx_cap; ++j) {
        KxSlot& q = h->kx_m[j];
        if (slot_state(q.meta) != SLOT_LIVE || !((bits[slot_silo(q.meta) >> 5] >> (slot_silo(q.meta) & 31)) & 1))
            continue;
        if (q.act == GD_ACT_MULTI) {
            c[1]++;
            continue;
        }
        q.meta = make_meta(SLOT_TOMB, slot_silo(q.meta));
        h->kx_live--;
        h->kx_tomb++;
        c[0]++;
        dirty.push_back(j);
    }
    if (!dirty.empty()) GD_TRY(kx_commit(h, dirty));
    if (out_removed) *out_removed = c[0];
    if (out_multi) *out_multi = c[1];
    if (out_cache_removed) *out_cache_removed = c[2];
    return GD_OK;
}

int gd_activation_ids_set(gd_handle* h, const uint32_t* acts, const gd_key* ids, uint32_t n) {
    if (!h || (n && (!acts || !ids))) return set_err(h, GD_EINVAL, "null argument");
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    uint64_t need = h->n_act_ids;
    for (uint32_t i = 0; i < n; ++i) {
        if (acts[i] >= GD_ACT_MULTI) return set_err(h, GD_EINVAL, "activation index %u reserved", acts[i]);
        need = std::max<uint64_t>(need, (uint64_t)acts[i] + 1);
    }
    GD_TRY(grow_act_ids(h, need));
    // scatter on the host side of a staging copy (small batches: registration is off the hot path)
    GD_TRY(h2d(h, h->dirop_buf[0], acts, n));
    GD_TRY(h2d(h, h->dirop_buf[1], ids, n));
    GD_TRY(launch(h, "k_scatter_ids", dim3(blocks_for(n, BLOCK)), dim3(BLOCK), 0, k_scatter_ids,
                  (const uint32_t*)h->dirop_buf[0].p, (const gd_key*)h->dirop_buf[1].p, n, (gd_key*)h->act_ids.p));
    return sync(h);
}

int gd_dir_merge(gd_handle* h, const gd_key* keys, const gd_val* vals, const int32_t* tags, uint32_t n,
                 uint8_t* out_status, gd_val* out_dropped) {
    if (!h || (n && (!keys || !vals || !out_status))) return set_err(h, GD_EINVAL, "null argument");
    for (uint32_t i = 0; i < n; ++i)
        if (vals[i].silo > 0xFFFEu) return set_err(h, GD_EINVAL, "silo index %u out of range at %u", vals[i].silo, i);
    if (n == 0) return GD_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    GD_TRY(h2d(h, h->keys_in, keys, n));
    GD_TRY(h2d(h, h->out_c, vals, n));
    if (tags) GD_TRY(h2d(h, h->dirop_buf[1], tags, n));
    GD_TRY(ensure(h, h->out_b, (size_t)n));
    GD_TRY(ensure(h, h->out_a, (size_t)n * sizeof(gd_val)));
    GD_TRY(merge_core(h, (const gd_key*)h->keys_in.p, (const gd_val*)h->out_c.p,
                      tags ? (const int32_t*)h->dirop_buf[1].p : nullptr, n, (uint8_t*)h->out_b.p,
                      (gd_val*)h->out_a.p));
    HIP_TRY(h, hipMemcpyAsync(out_status, h->out_b.p, n, hipMemcpyDeviceToHost, h->stream));
    if (out_dropped)
        HIP_TRY(h, hipMemcpyAsync(out_dropped, h->out_a.p, (size_t)n * sizeof(gd_val), hipMemcpyDeviceToHost, h->stream));
    return check_dir_err(h, "gd_dir_merge");
}

}  // extern "C"

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
namespace {

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

}  // namespace

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

// ================================================================== receive path: ActivationDirectory +
// IncomingMessageAgent.ReceiveMessage (gd_actdir.h)
namespace {

AdArgs ad_args(gd_handle* h) { return AdArgs{h->ad_slots, h->ad_cap ? h->ad_cap - 1 : 0ull, h->ad_ctr}; }

int receive_device(gd_handle* h, const gd_key* tg, const gd_key* ta, const uint8_t* dir, const uint32_t* fflags,
                   uint32_t n, uint32_t n_ctx, const gd_recv_limits* lim, uint32_t* ctx, uint8_t* st, uint32_t* perm,
                   uint32_t* offsets);

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
    HIP_TRY(h, hipMemcpyAsync(&h->ad_host, h->ad_ctr, sizeof(DevCounters), hipMemcpyDeviceToHost, h->stream));
    return sync(h);
}

// (Re)build the ActivationDirectory table with cap slots (tombstones dropped).
int ad_rehash(gd_handle* h, unsigned long long cap) {
    Slot* ns = nullptr;
    GD_TRY(alloc_table(h, cap, &ns));
    if (!h->ad_ctr) {
        hipError_t e = hipMalloc(&h->ad_ctr, sizeof(DevCounters));
        if (e != hipSuccess) {
            (void)hipFree(ns);
            return set_err(h, GD_ENOMEM, "activation directory counters: %s", hipGetErrorString(e));
        }
    }
    DevCounters fresh{};
    HIP_TRY(h, hipMemcpyAsync(h->ad_ctr, &fresh, sizeof fresh, hipMemcpyHostToDevice, h->stream));
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

}  // namespace

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
                      is_new, (uint32_t)(pass > 0), (const gd_val*)nullptr, TableArgs{}));
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
    HIP_TRY(h, hipMemsetAsync(h->ad_ctr, 0, sizeof(DevCounters), h->stream));
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
