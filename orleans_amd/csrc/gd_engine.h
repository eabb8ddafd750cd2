// gd_engine.h -- libgraindispatch's engine-internal header: the handle, the launch / scratch helpers and
// the functions the engine's translation units share (eng_*.hip).  Not part of the ABI (include/
// graindispatch.h is).  Every kernel header is included here; their non-template kernels are static, so
// each translation unit keeps its own copies.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
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

namespace gdx {

extern thread_local std::string g_tls_error;

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

struct TimedLaunch {
    int name;
    hipEvent_t a, b;
};

}  // namespace gdx

using namespace gdx;

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
    bool ctr_stale = true;            // an untracked table write since the last copy (maybe_grow_async pulls)
    uint64_t pending_in = 0;          // entries asynchronous registrations may have added since the last copy
    DevBuf reg_retry;                 // asynchronous registrations: deferred-claim counts of the gated passes
    DevBuf dir_scr[3];                // directory batches' scratch (slot_of, win, is_new): never the bucketing's

    // scratch
    DevBuf keys_in, u32_a, u32_b, u32_c, u32_d, u8_a, out_a, out_b, out_c, hist, partials, partials2, offs;
    DevBuf fr[16];                    // header-decode scratch (host-pointer entry points)
    DevBuf fr_ext[2];                 // TargetGrain KeyExt offsets / lengths (gd_route_frames_ext*)
    DevBuf churn[5];                  // split scratch: keep mask, flags, positions, out keys/vals
    DevBuf fan_bnd;                   // k_fan_bound's scratch outputs
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
    // gd_set_bucket_stream: gd_route_bucket_device's bucketing on this stream after the route (event
    // b_ev on the handle's stream), so the next batch's route overlaps this batch's bucketing
    hipStream_t bstream = nullptr;
    hipEvent_t b_ev = nullptr;
    hipEvent_t b_fence_ev = nullptr;  // bfence: the handle's stream waits for a bucketing on bstream
    bool b_pending = false;           // a bucketing was enqueued on bstream since the last bfence
    hipEvent_t fan_ev = nullptr;   // the cascade's per-hop size read-back (fan_count_post / fan_count_wait)
    hipStream_t pstream = nullptr;    // the partition (pack) of the next batch, beside this one's rounds
    hipEvent_t x_in = nullptr, x_hdr[2] = {}, x_route[2] = {}, x_ret[2] = {}, x_done[2] = {};
    // a launch timed for tune_choose was enqueued since the last exchange call: the next call's partition
    // waits for it (route_multi), so the timings are not taken beside the pipeline's overlapped work
    bool measured_launch = false;
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
    bool fan_bound = false;     // a k_fan_bound launch beside each 8-B-index k_fan_route (GD_OPT_FAN_BOUND)
    uint32_t fan_bound_n = 0;   // ... before it on even launches, after it on odd ones
    bool mb_poll = true;        // micro-batches: completion by the sort's pinned count (GD_OPT_MB_POLL)
    int tune_pin[GD_TUNE_KINDS] = {-1, -1, -1, -1, -1};   // gd_tune_set: pinned variant per kind, -1 measured
    int msd_mode = 1;           // two-level bucketing (gd_msd.h, gd_msd2.h): 0 off, 1 measured (default), 2 always (GD_MSD)
    uint32_t l2_small = 1024;   // three-pass form: ranges of at most this many messages are sorted one wave a range
    uint32_t l2_mid = MSD_MID_CAP;  // three-pass form: staged ranges up to this many messages on the 512-thread sort
    uint32_t b2_persist = 2;       // one-pass MSD scatter: persistent workgroups a CU (0: one a tile; GD_OPT_B2_PERSIST)
    uint32_t b2_order = 0;         // its tile order: 0 strided, 1 consecutive runs a workgroup (GD_OPT_B2_ORDER)
    uint32_t l2_staged = MSD_CAP;  // three-pass form: ranges up to this many messages one workgroup each, more: chunks
    uint32_t n_cu = 256;        // compute units (hipDeviceProp_t::multiProcessorCount): persistent grids
    DevBuf m3[15];              // three-pass form's scratch (msd3_bucket)
    DevBuf tune_buf;            // gd_tune_agree's send / receive records
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
    uint64_t tab_gen = 0;       // bumped by every launch that takes the table as a writable Slot* (untracked)
    uint32_t tab_track = 0;     // > 0: inside a directory batch that re-projects its slots (TabTrack, k_cx_sync)
    bool cx_built = false, cx_ok = false;
    const Slot* cx_slots_at = nullptr;
    uint64_t cx_cap_at = 0, cx_gen_at = 0;
    DevBuf cxi_tab, cxi_types, cxi_ctr;   // 16-B index; its type set (+ a count per slot); CxCounters
    bool cx8_ok = false;        // the 8-B index is built and current with cx
    // ... and pure: one grain class, every live entry held and none redirected (CxCounters::out8 = 0), as of
    // a counter read-back with no directory batch enqueued since -- k_route_m's PURE form, whose walks
    // need no directory fallback
    bool cx8_pure = false;
    Cx8Args cx8_layout{};       // its layout (types, bits), fixed at the build
    DevBuf cx8_tab;
    CxCounters cx_ctr_host{};   // the last read-back of the index counters
    uint32_t cx_out8_at = 0, cx_held8_at = 0;   // at the build: live entries the 8-B index left out / held
    uint64_t cx_builds = 0, cx_synced = 0;      // full builds; slots re-projected by k_cx_sync (gd_stats)
    double cx_build_ms = 0.0;                   // host wall time of the last full build
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
    int timing = 0;             // gd_set_kernel_timing: 0 off, 1 every launch, 2 the stages (StageTime) only
    std::vector<std::string> tnames;
    std::vector<double> tms;
    std::vector<uint64_t> tcount;
    std::vector<TimedLaunch> pending;
    std::vector<hipEvent_t> event_pool;
};

namespace gdx {

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

#define NCCL_TRY(h, expr)                                                                          \
    do {                                                                                           \
        ncclResult_t r_ = (expr);                                                                  \
        if (r_ != ncclSuccess)                                                                     \
            return set_err((h), GD_ERCCL, "%s: %s", #expr, (h)->net->GetErrorString(r_));          \
    } while (0)

inline uint32_t blocks_for(uint64_t n, uint32_t per) { return (uint32_t)((n + per - 1) / per); }

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

// ---- shared across the engine's translation units (definitions in eng_*.hip)
int set_err(gd_handle* h, int code, const char* fmt, ...);
int ensure(gd_handle* h, DevBuf& b, size_t bytes);
int ensure_own(gd_handle* h, DevBuf& b, size_t bytes);
void free_buf(DevBuf& b);
int name_id(gd_handle* h, const char* name);
hipEvent_t take_event(gd_handle* h);
int resolve_timing(gd_handle* h);
int check_ring(gd_handle* h);
RingArgs ring_args(gd_handle* h);
TableArgs table_args(gd_handle* h);
bool host_silo_valid(const gd_handle* h, uint32_t silo);
size_t ring_lds(gd_handle* h);
int pull_counters(gd_handle* h);
int fold_counters(gd_handle* h, DevCounters* c);
int alloc_table(gd_handle* h, unsigned long long cap, Slot** out);
int alloc_vtag(gd_handle* h, unsigned long long cap, uint32_t** out);
unsigned long long pow2_at_least(unsigned long long x);
int cx_ensure(gd_handle* h, bool* ok, uint64_t n);
bool cx_current(const gd_handle* h);
struct TabTrack;
int cx_sync(gd_handle* h, TabTrack& tt, const uint32_t* slot_of, uint32_t n);
bool cx_inline(gd_handle* h, TabTrack& tt, uint32_t n);
CxBuild cx_build_args(gd_handle* h);
int tune_key(int kind, uint64_t n, int sub);
int tune_nvar(int kind);
int tune_nvar_now(const gd_handle* h, int kind);
void tune_resolve(gd_handle::CxTune& t, int nvar);
int tune_choose(gd_handle* h, int kind, uint64_t n, int* meas, int nvar, int sub = 0);
int cx_choose(gd_handle* h, int kind, uint64_t n, int* meas, int nvar = gd_handle::CXV);
Cx8Args cx8_args(gd_handle* h);
CxArgs cx_args(gd_handle* h);
int route_n1_device(gd_handle* h, const void* n1s, uint32_t n1w, uint64_t tcd, uint32_t n, uint32_t* silo,
                    uint32_t* act, uint8_t* status, const uint32_t* rcnt = nullptr, uint32_t world = 0,
                    uint32_t* src = nullptr);
int route_region_device(gd_handle* h, const void* k, uint32_t n1w, uint64_t tcd, uint32_t m, const uint32_t* seg,
                        uint32_t world, uint32_t* silo, uint32_t* act, uint8_t* status);
int route_cached(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t* silo, uint32_t* act, uint8_t* status,
                 bool touch);
int route_cached_keyext(gd_handle* h, const gd_key* keys, const ExtArgs& x, uint32_t n, uint32_t* silo, uint32_t* act,
                        uint8_t* st);
int route_device(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t* silo, uint32_t* act, uint8_t* status,
                 bool touch = true);
int route_bound_device(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t* silo, uint32_t* act,
                       uint8_t* status);
KxArgs kx_args(gd_handle* h);
int keyext_pass(gd_handle* h, const gd_key* keys, const ExtArgs& x, uint32_t n, uint32_t* silo, uint32_t* act,
                uint8_t* st);
int ring_owner_device(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t* silo);
int bucket_device(gd_handle* h, const uint32_t* acts, uint32_t n, uint32_t n_act, uint32_t* perm, uint32_t* offsets,
                  uint32_t* rank_out = nullptr);
int sync(gd_handle* h);
int pinned_scratch(gd_handle* h, size_t bytes);
int sync_checked(gd_handle* h);
int maybe_grow_table(gd_handle* h, uint64_t incoming);
int fwd_pack(gd_handle* h, const gd_key* keys, const uint8_t* st, const uint32_t* silo, uint32_t n, uint32_t n_shards,
             uint32_t my_rank, void* out_keys, uint32_t* out_pos, uint32_t* counts, const uint32_t* n1 = nullptr);
bool host_pinned(const void* p);
int route_bucket_host_pipelined(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t n_act, uint32_t* out_silo,
                                uint32_t* out_act, uint8_t* out_status, uint32_t* out_perm, uint32_t* out_offsets);
int register_core(gd_handle* h, const gd_key* dk, const gd_val* dvals, uint32_t n, gd_val* out_vals,
                  uint8_t* out_ins, bool async = false);
int unregister_core(gd_handle* h, const gd_key* dk, const uint32_t* dacts, uint32_t n, uint8_t* out_removed);
int maybe_grow_async(gd_handle* h, uint64_t incoming);
int bfence(gd_handle* h);
int slot_words(gd_handle* h);
int split_count(gd_handle* h, const uint8_t* keep, uint32_t n_keep, uint64_t* total);
uint64_t grain_tcd(int32_t type_code);
int fan_count(gd_handle* h, const uint32_t* row_off, uint32_t n_nodes, const uint32_t* frontier, uint32_t nf,
              uint64_t* total);
int route_nodes(gd_handle* h, const uint32_t* nodes, uint32_t n, uint64_t tcd, uint32_t* silo, uint32_t* act,
                uint8_t* status);
int frontier_next_dev(gd_handle* h, const uint32_t* offsets, uint32_t n_act, uint8_t* visited, uint32_t* out,
                      const uint32_t** d_nf);
int fan_count_dev(gd_handle* h, const uint32_t* row_off, uint32_t n_nodes, const uint32_t* frontier,
                  const uint32_t* d_nf, uint32_t nf_max, uint32_t* nf, uint64_t* total);
void comm_release(gd_handle* h);
int need_comm(gd_handle* h);
int exchange_round(gd_handle* h, const char* name, const uint32_t* sc, const uint64_t* soff, const uint32_t* rc,
                   const uint64_t* roff, const Lane* lanes, int n_lanes);
int counts_round(gd_handle* h, uint32_t* dcnt, std::vector<uint32_t>& sc, std::vector<uint32_t>& rc);
bool is_keyext_cat(uint64_t tcd);
uint32_t kx_hash_host(const gd_key& k, const uint8_t* s, int32_t len);
int host_ext(gd_handle* h, const gd_key_ext* ext, uint32_t i, const uint8_t*& s, int32_t& len);
int kx_commit(gd_handle* h, std::vector<uint64_t>& dirty);
int stage_ext(gd_handle* h, const gd_key_ext* ext, uint32_t n, gd_key_ext* dx);
bool ext_ok(const gd_key_ext* ext, uint32_t n);
int grow_act_ids(gd_handle* h, uint64_t need);
int check_dir_err(gd_handle* h, const char* what);
int merge_core(gd_handle* h, const gd_key* dk, const gd_val* dvals, const int32_t* dtags, uint32_t n,
               uint8_t* d_status, gd_val* d_dropped);
AdArgs ad_args(gd_handle* h);
int check_frames_args(gd_handle* h, const void* buf, const void* off, uint32_t n, const gd_frame_fields* out);
int decode_frames_device(gd_handle* h, const uint8_t* buf, uint64_t len, const uint64_t* off, uint32_t n,
                         const gd_frame_fields* out, bool ext = false);
int frame_scratch(gd_handle* h, uint32_t n, const gd_frame_fields* want, gd_frame_fields* dev);
int frame_results(gd_handle* h, uint32_t n, const gd_frame_fields* want, const gd_frame_fields* dev);
int bucket_lsd(gd_handle* h, const uint32_t* acts, uint32_t n, uint32_t n_act, uint32_t* perm, uint32_t* offsets,
               uint32_t* rank_out);
bool msd3_split(uint32_t n_act, uint32_t* a_out, uint32_t* ra_out);
int frontier_next(gd_handle* h, const uint32_t* offsets, uint32_t n_act, uint8_t* visited, uint32_t* out,
                  uint32_t* out_n);
int route_frames_device(gd_handle* h, const uint8_t* buf, uint64_t len, const uint64_t* off, uint32_t n,
                        uint32_t n_act, const gd_frame_fields* out, uint32_t* silo, uint32_t* act, uint8_t* status,
                        uint32_t* perm, uint32_t* offsets, bool ext = false);
int receive_device(gd_handle* h, const gd_key* tg, const gd_key* ta, const uint8_t* dir, const uint32_t* fflags,
                   uint32_t n, uint32_t n_ctx, const gd_recv_limits* lim, uint32_t* ctx, uint8_t* st, uint32_t* perm,
                   uint32_t* offsets);
int receive_frames_device(gd_handle* h, const uint8_t* buf, uint64_t len, const uint64_t* off, uint32_t n,
                          uint32_t n_ctx, const gd_recv_limits* lim, const gd_frame_fields* out, uint32_t* ctx,
                          uint8_t* st, uint32_t* perm, uint32_t* offsets);
int grow(gd_handle* h, DevBuf& b, size_t bytes);
int comm_setup(gd_handle* h);
int kx_rehash(gd_handle* h, uint64_t cap);
int kx_upload_all(gd_handle* h);
int cache_check(gd_handle* h);
int cache_rehash(gd_handle* h, unsigned long long cap);
int cx_reserve(gd_handle* h, uint64_t need);
int ad_reserve(gd_handle* h, uint64_t incoming);
int ad_pull(gd_handle* h);
int ad_rehash(gd_handle* h, unsigned long long cap);
int fan_args_ok(gd_handle* h, const uint32_t* row_off, const uint32_t* dst, uint32_t nf, const uint32_t* frontier,
                uint64_t* out_n);
int fan_route(gd_handle* h, const uint32_t* row_off, const uint32_t* dst, const uint32_t* frontier, uint32_t nf,
              uint32_t total, uint64_t tcd, uint32_t* target, uint32_t* sender, uint32_t* silo, uint32_t* act,
              uint8_t* status, const uint32_t* d_nf = nullptr, bool dev_total = false);
int cache_pull(gd_handle* h, CacheCounters* c);
int cache_touch(gd_handle* h, uint32_t* hit, const uint32_t* cslot, uint32_t n);
int split_emit(gd_handle* h, int move, gd_key* d_keys, gd_val* d_vals);
int set_bitset(gd_handle* h, DevBuf& b, const std::vector<uint32_t>& bits);
int mb_enqueue(gd_microbatch* mb, uint32_t n, bool count_done);
template <class Op>
int scan_device(gd_handle* h, uint32_t* data, uint32_t n, bool reverse, bool inclusive, const char* tag,
                uint32_t* out = nullptr);
template <bool NODES>
int shard_pack(gd_handle* h, const void* recs, const uint32_t* payload, uint32_t n, uint64_t tcd, uint32_t n_shards,
               void* out_recs, uint32_t* out_pay, uint32_t* counts, const ExtArgs& ext = ExtArgs{},
               uint32_t* kdesc = nullptr, uint32_t regions = 1);

// A launch argument that is the directory table as a writable Slot* (the kernel may change it).
template <typename T>
bool writes_table(const gd_handle*, const T&) { return false; }
inline bool writes_table(const gd_handle* h, Slot* p) { return p != nullptr && p == h->slots; }

// Launch a kernel on the handle's stream; with GD_CFG_KERNEL_TIMING bracket it by events.  A kernel
// handed the table as a writable Slot* invalidates the compact probe index (tab_gen), unless it runs
// inside a TabTrack scope, whose batch re-projects the slots it touched (cx_sync).
template <typename K, typename... Args>
int launch(gd_handle* h, const char* name, dim3 grid, dim3 block, size_t lds, K kernel, Args... args) {
    if (grid.x == 0) return GD_OK;
    if (!h->tab_track && (writes_table(h, args) || ...)) {
        h->tab_gen++;
        h->ctr_stale = true;
    }
    hipEvent_t a = nullptr, b = nullptr;
    if (h->timing == 1) {
        a = take_event(h);
        b = take_event(h);
        HIP_TRY(h, hipEventRecord(a, h->stream));
    }
    hipLaunchKernelGGL(kernel, grid, block, lds, h->stream, args...);
    HIP_TRY(h, hipGetLastError());
    if (h->timing == 1) {
        HIP_TRY(h, hipEventRecord(b, h->stream));
        h->pending.push_back(TimedLaunch{name_id(h, name), a, b});
    }
    return GD_OK;
}

// Stage timing (gd_set_kernel_timing 2): one event pair around a whole stage -- e.g. every launch of a
// bucketing -- recorded under `name`, with no events between its kernels (per-launch events add ~5 us a
// kernel and so inflate a many-kernel stage).
struct StageTime {
    gd_handle* h;
    int name = -1;
    hipEvent_t a = nullptr, b = nullptr;
    StageTime(gd_handle* hh, const char* nm) : h(hh) {
        if (h->timing != 2) return;
        name = name_id(h, nm);
        a = take_event(h);
        b = take_event(h);
        (void)hipEventRecord(a, h->stream);
    }
    ~StageTime() {
        if (name < 0) return;
        (void)hipEventRecord(b, h->stream);
        h->pending.push_back(TimedLaunch{name, a, b});
    }
};

// A directory batch whose table writes keep the probe indexes current: the slots it touched are
// re-projected by cx_sync (which calls done()); a batch that ends early (an error) leaves the indexes
// stale instead, and the next large route rebuilds them.
struct TabTrack {
    gd_handle* h;
    bool was_current;
    bool synced = false;
    explicit TabTrack(gd_handle* hh);
    ~TabTrack() {
        --h->tab_track;
        if (!synced) h->tab_gen++;
    }
};

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

}  // namespace gdx
