/*
 * graindispatch.h -- C ABI of libgraindispatch.so, the MI355X (gfx950) batched
 * message-routing engine for the Orleans virtual-actor dispatch path.
 *
 * The Orleans host (C#) keeps its Dispatcher / MessageCenter / IGrainFactory
 * surface.  A batching stage hands message headers to this library through
 * P/Invoke (see INTEGRATION.md for the [DllImport] stubs).  Plain pointers and
 * sizes only; no exceptions cross this boundary; every entry point returns
 * GD_OK (0) or a negative GD_E* code, with a message in gd_last_error().
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * rikbosch/orleans root):
 *   ring       LocalGrainDirectory.CalculateTargetSilo      src/Orleans.Runtime/GrainDirectory/LocalGrainDirectory.cs:477-545
 *              IConsistentRingProvider.GetPrimaryTargetSilo src/Orleans.Runtime/ConsistentRing/IConsistentRingProvider.cs:34
 *              (ConsistentRingProvider.cs:322-372, VirtualBucketsRingProvider.cs:244-293)
 *              ring rebuild: LocalGrainDirectory.AddServer  LocalGrainDirectory.cs:284-309,
 *              VirtualBucketsRingProvider.AddServer         VirtualBucketsRingProvider.cs:122-149
 *   directory  GrainDirectoryPartition.AddSingleActivation  src/Orleans.Runtime/GrainDirectory/GrainDirectoryPartition.cs:304-326
 *              GrainDirectoryPartition.RemoveActivation     GrainDirectoryPartition.cs:335-363
 *              GrainDirectoryPartition.LookUpActivations    GrainDirectoryPartition.cs:385-441
 *              ILocalGrainDirectory.LocalLookup             src/Orleans.Runtime/GrainDirectory/ILocalGrainDirectory.cs:22
 *   address    Dispatcher.AddressMessage                    src/Orleans.Runtime/Core/Dispatcher.cs:715-767
 *   enqueue    IncomingMessageAgent.ReceiveMessage          src/Orleans.Runtime/Messaging/IncomingMessageAgent.cs:92-190
 *              + ActivationData.EnqueueMessage (FIFO)       src/Orleans.Runtime/Catalog/ActivationData.cs:566-606
 *   identity   JenkinsHash.ComputeHash                      src/Orleans.Core.Abstractions/IDs/JenkinsHash.cs:25-105
 *              UniqueKey.GetUniformHashCode                 src/Orleans.Core.Abstractions/IDs/UniqueKey.cs:272-293
 *              SiloAddress.GetConsistentHashCode / GetUniformHashCodes  SiloAddress.cs:164-248
 *              Utils.CalculateIdHash                        src/Orleans.Core/Utils/Utils.cs:184-203
 *
 * Threading: one handle = one HIP stream.  Calls on a handle are serialised
 * by the caller (the reference serialises the same state under
 * lock(membershipCache) / lock(lockable), LocalGrainDirectory.cs:512,
 * GrainDirectoryPartition.cs:282,393).  gd_ring_set installs a new immutable
 * ring snapshot that the next route call uses (the mirror of the lock-free
 * snapshot swap at VirtualBucketsRingProvider.cs:143-144).
 *
 * Ownership: host arrays are caller-owned and never retained past return.
 * *_device entry points take device pointers (hipMalloc'd / torch tensors)
 * and only enqueue on the handle's stream; call gd_synchronize() before
 * reading results.  The library owns the table, ring snapshot and scratch.
 */
#ifndef GRAINDISPATCH_H
#define GRAINDISPATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GD_ABI_VERSION 1

/* ---- return codes ------------------------------------------------------ */
#define GD_OK        0
#define GD_EINVAL   -1   /* bad argument / unsorted ring / n too large       */
#define GD_ENOMEM   -2   /* device or host allocation failed                 */
#define GD_EHIP     -3   /* HIP runtime error                                */
#define GD_ERCCL    -4   /* collective error (multi-GPU path)                */
#define GD_EFULL    -5   /* directory table cannot take more entries         */
#define GD_ESTATE   -6   /* no ring installed / handle not ready             */
#define GD_ETIMEOUT -7   /* a bounded device spin gave up (never expected)   */

/* ---- ring modes ----------------------------------------- */
#define GD_RING_DIRECTORY        0 /* D: LocalGrainDirectory, signed predecessor, wrap to last */
#define GD_RING_CONSISTENT       1 /* R: ConsistentRingProvider, (long)int >= (long)uint, wrap to first */
#define GD_RING_VIRTUAL_BUCKETS  2 /* V: VirtualBucketsRingProvider, uint successor, wrap to first */

/* ---- per-message routing status (out_status) ------------------------------ */
#define GD_ROUTE_OK             0 /* directory hit: (silo, act) = the single activation     */
#define GD_ROUTE_MISS           1 /* not registered: C# slow path (Dispatcher.cs:742);
                                     out_silo = directory owner silo                         */
#define GD_ROUTE_SYSTEM_TARGET  2 /* UniqueKey category SystemTarget: out_silo = my silo
                                     (LocalGrainDirectory.cs:480-485)                         */
#define GD_ROUTE_MEMBERSHIP     3 /* Constants.SystemMembershipTableId: out_silo = seed silo
                                     (LocalGrainDirectory.cs:487-503)                         */
#define GD_ROUTE_KEYEXT         4 /* KeyExtGrain / GeoClient: the uniform hash needs the
                                     KeyExt string (UniqueKey.cs:279-281); C# handles it     */

#define GD_ROUTE_MULTI_ACT      7 /* the grain has several activations (GrainInfo.Instances.Count >= 2,
                                     e.g. StatelessWorker): RandomPlacementDirector picks one in C#
                                     (RandomPlacementDirector.cs:33-53); out_silo = directory owner */

#define GD_NO_ACTIVATION 0xFFFFFFFFu
#define GD_ACT_MULTI     0xFFFFFFFEu   /* gd_val.act of a multi-activation grain (gd_dir_upsert)   */
#define GD_NO_SILO       0xFFFFFFFFu

/* UniqueKey fields (UniqueKey.cs:28-31) of a GrainId.  24 bytes, AoS. */
typedef struct gd_key {
    uint64_t n0;
    uint64_t n1;
    uint64_t type_code_data;
} gd_key;

/* Directory value: the compact form of ActivationAddress (ActivationAddress.cs:6-34).
 * act  = host-side activation index (the C# side maps it to its ActivationData),
 * silo = index into the host's silo table. */
typedef struct gd_val {
    uint32_t act;
    uint32_t silo;
} gd_val;

/* SiloAddress (SiloAddress.cs:33-35): IPv4 in ip[12..15] with is_v4 = 1
 * (BinaryTokenStreamWriter.cs:485-500 layout), or 16-byte IPv6. */
typedef struct gd_silo_addr {
    uint8_t ip[16];
    int32_t port;
    int32_t generation;
    int32_t is_v4;
} gd_silo_addr;

typedef struct gd_config {
    uint32_t struct_size;     /* sizeof(gd_config)                                   */
    int32_t  device;          /* HIP device ordinal                                  */
    uint64_t table_capacity;  /* directory slots (rounded up to a power of two);
                                 0 = 1<<20.  Keep load <= 0.5 for short probes.      */
    uint32_t my_silo;         /* silo index this handle acts for (system targets)    */
    uint32_t seed_silo;       /* owner of the membership-table grain; GD_NO_SILO = none */
    uint32_t max_batch;       /* messages per call the scratch is sized for (0 = 1<<24);
                                 larger calls grow the scratch (outside graph capture) */
    uint32_t flags;           /* GD_CFG_* bits                                       */
} gd_config;

#define GD_CFG_KERNEL_TIMING 1u  /* record per-kernel HIP events (gd_kernel_times) */
#define GD_CFG_NO_LANE_ORDER 2u  /* behave as on a device whose LDS atomics are not served in lane order:
                                    every stable rank by ballots (GD_OPT_STABLE_RANK 0, 1 refused); the
                                    library's own choice when gd_create's check fails (tests force it) */

typedef struct gd_stats {
    uint64_t routed;          /* messages through gd_route*                          */
    uint64_t table_live;      /* live directory entries                              */
    uint64_t table_tombstones;
    uint64_t table_capacity;
    uint64_t ring_points;
    uint64_t ring_mode;
} gd_stats;

typedef struct gd_handle gd_handle;

/* ---- lifecycle -------------------------------------------------------------- */
int         gd_create(const gd_config* cfg, gd_handle** out);
void        gd_destroy(gd_handle* h);
const char* gd_last_error(const gd_handle* h);   /* never NULL; h may be NULL     */
int         gd_abi_version(void);
int         gd_set_stream(gd_handle* h, void* hip_stream); /* NULL = library stream */
void*       gd_get_stream(gd_handle* h);
/* Pinned (page-locked) host memory for batch buffers.  The host-pointer entry points overlap
 * their PCIe copies with the kernels for large batches (gd_route_bucket: keys up, routes down
 * while later chunks are probed); the copies are asynchronous only from pinned memory.  A C# host
 * allocates its batch arrays here once and reuses them (Span<T> over the pointer). */
int         gd_host_alloc(size_t bytes, void** out);
int         gd_host_free(void* p);
int         gd_synchronize(gd_handle* h);
int         gd_stats_get(gd_handle* h, gd_stats* out);

/* ---- identity (host; L0) ------------------------------------------------------ */
uint32_t gd_jenkins_hash_bytes(const uint8_t* data, size_t len);                 /* JenkinsHash.cs:25-74  */
uint32_t gd_jenkins_hash_u64x3(uint64_t u1, uint64_t u2, uint64_t u3);          /* JenkinsHash.cs:85-105 */
uint32_t gd_uniform_hash(const gd_key* key);                                     /* UniqueKey.cs:272-293 (no KeyExt) */
int32_t  gd_calculate_id_hash(const char* utf8_text);                            /* Utils.cs:184-203      */
int32_t  gd_silo_consistent_hash(const gd_silo_addr* silo);                      /* SiloAddress.cs:164-173 */
int      gd_silo_uniform_hashes(const gd_silo_addr* silo, uint32_t n, uint32_t* out); /* SiloAddress.cs:197-248 */
int      gd_silo_compare(const gd_silo_addr* a, const gd_silo_addr* b);          /* SiloAddress.cs:280-329 */

/* ---- ring ------------------------------------------------------------------- */
/* Build a ring from silos added in the given order (membership-change order):
 * mode D/R -> AddServer sorted insert by signed consistent hash (ties: newcomer
 * before equals); mode V -> buckets_per_silo uniform points per silo, uint
 * sorted, collision -> lesser SiloAddress.  out_points / out_owner must hold
 * n_silos (D/R) or n_silos*buckets_per_silo (V) entries; *out_n = ring size. */
int gd_ring_build(int mode, const gd_silo_addr* silos, uint32_t n_silos, uint32_t buckets_per_silo,
                  uint32_t* out_points, uint32_t* out_owner, uint32_t* out_n);
/* Install a ring snapshot: points are 32-bit patterns in ring order (int32 sorted
 * ascending for D/R, uint32 ascending for V); owner[i] = silo index of point i. */
int gd_ring_set(gd_handle* h, int mode, const uint32_t* points, const uint32_t* owner, uint32_t n);

/* CalculateTargetSilo(GrainId) for a batch: directory-owner silo per key
 * (special categories follow the same rules as gd_route).  Host pointers. */
int gd_ring_owner(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t* out_silo);
/* GetPrimaryTargetSilo(uint key) for a batch of raw ring keys.  Host pointers. */
int gd_ring_lookup_hashes(gd_handle* h, const uint32_t* hashes, uint32_t n, uint32_t* out_silo);

/* ---- directory (one table per handle = the silo partitions this GPU owns) ---- */
/* AddSingleActivation for a batch, applied in batch order: the first registration
 * of a grain wins; out_vals receives the winning (act, silo) for every item and
 * out_inserted 1 for the item that created the entry.  Host pointers. */
int gd_dir_register(gd_handle* h, const gd_key* keys, const gd_val* vals, uint32_t n,
                    gd_val* out_vals, uint8_t* out_inserted);
/* gd_dir_register with device arrays (keys, values and the optional outputs, which may be NULL):
 * bulk population of a partition whose grains are already in HBM (activation tables built on
 * the GPU, a handoff received over RCCL).  Waits for work enqueued on the handle's stream, runs
 * synchronously.  A value with silo > 0xFFFE fails the call with GD_EINVAL. */
int gd_dir_register_device(gd_handle* h, const gd_key* d_keys, const gd_val* d_vals, uint32_t n,
                           gd_val* d_out_vals, uint8_t* d_out_inserted);
/* Overwrite for a batch, applied in batch order (the last item of a grain wins): how the host
 * mirrors GrainDirectoryPartition.AddActivation (GrainDirectoryPartition.cs:274-302; GrainInfo
 * .AddActivation :89-108) for multi-instance grains: one instance -> {act, silo}, two or more ->
 * {GD_ACT_MULTI, any silo} (routes then return GD_ROUTE_MULTI_ACT).  out_inserted[i] = 1 for the
 * item that created a grain's entry (may be NULL).  Host pointers. */
int gd_dir_upsert(gd_handle* h, const gd_key* keys, const gd_val* vals, uint32_t n, uint8_t* out_inserted);
/* RemoveActivation(grain, act) for a batch; out_removed may be NULL. */
int gd_dir_unregister(gd_handle* h, const gd_key* keys, const uint32_t* acts, uint32_t n,
                      uint8_t* out_removed);
/* The continuous-registration forms (round 6): activations register and deactivate all the time
 * (Catalog.cs:540-552,1270-1277 -> GrainDirectoryPartition.AddSingleActivation / RemoveActivation,
 * GrainDirectoryPartition.cs:304-363), between route batches.  Both only enqueue on the handle's
 * stream (device arrays, outputs optional): no host round trip, so a host interleaves them with
 * gd_route_bucket_device batches and the stream runs them back to back; the probe indexes are
 * re-projected for the touched slots, not rebuilt.  Same semantics as gd_dir_register_device /
 * gd_dir_unregister; a device-side failure (table full, claims not settled after the gated passes)
 * is returned by the next synchronising call on the handle (gd_synchronize, gd_stats_get, ...).
 * gd_dir_unregister_device with d_out_removed NULL is one launch (which of a key's matching items
 * removes it is then unobservable: the CAS on the entry's LIVE meta picks it); with a report, the
 * first matching item of the batch is elected in a second launch. */
int gd_dir_register_device_async(gd_handle* h, const gd_key* d_keys, const gd_val* d_vals, uint32_t n,
                                 gd_val* d_out_vals, uint8_t* d_out_inserted);
int gd_dir_unregister_device(gd_handle* h, const gd_key* d_keys, const uint32_t* d_acts, uint32_t n,
                             uint8_t* d_out_removed);
/* LookUpActivations for a batch; out_found[i] = 0 -> out_vals[i] = {GD_NO_ACTIVATION, GD_NO_SILO}. */
int gd_dir_lookup(gd_handle* h, const gd_key* keys, uint32_t n, gd_val* out_vals, uint8_t* out_found);
int gd_dir_clear(gd_handle* h);
/* Rebuild into a table of new_capacity slots (drops tombstones). */
int gd_dir_rehash(gd_handle* h, uint64_t new_capacity);

/* ---- KeyExt grains (string keys, compound keys, geo clients) ---------
 * UniqueKey.HasKeyExt categories (KeyExtGrain 6, GeoClient 7; UniqueKey.cs:60-66) hash
 * JenkinsHash.ComputeHash(ToByteArray()) = N0|N1|TCD|int32 len|UTF-8 when KeyExt != null
 * (UniqueKey.cs:272-336) and compare the KeyExt string (UniqueKey.cs:245-251).  They live in a
 * second table (64-B slots + a KeyExt byte heap).  A batch's KeyExt strings travel beside the
 * 24-B keys: message i's UTF-8 bytes are bytes[offset[i] .. offset[i] + length[i]).  Messages
 * of other categories ignore their entry.  Equality is on UTF-8 bytes, which is C#'s ordinal
 * equality except for strings with unpaired surrogates (Encoding.UTF8 maps them to U+FFFD):
 * send those as GD_KEYEXT_HOST and they keep status GD_ROUTE_KEYEXT. */
#define GD_KEYEXT_NULL (-1)   /* KeyExt == null: three-word hash; equal only to a null KeyExt */
#define GD_KEYEXT_HOST (-2)   /* leave the message to the C# path (status GD_ROUTE_KEYEXT)    */
typedef struct gd_key_ext {
    const uint8_t*  bytes;      /* UTF-8 KeyExt strings of the batch, concatenated      */
    const uint64_t* offset;     /* [n] start of message i's string in bytes              */
    const int32_t*  length;     /* [n] UTF-8 byte length, GD_KEYEXT_NULL or GD_KEYEXT_HOST */
    uint64_t        bytes_len;  /* size of bytes (offset + length beyond it -> KEYEXT)  */
} gd_key_ext;

/* AddSingleActivation / RemoveActivation / LookUpActivations for KeyExt grains, batch order,
 * first registration wins (as gd_dir_register).  Keys must have a KeyExt category (GD_EINVAL
 * otherwise).  Registrations are applied to a host-side index of the table and the changed
 * slots uploaded (registration is off the per-message path); lookups run on the GPU.
 * Host pointers (ext included). */
int gd_dir_register_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, const gd_val* vals, uint32_t n,
                        gd_val* out_vals, uint8_t* out_inserted);
int gd_dir_unregister_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, const uint32_t* acts,
                          uint32_t n, uint8_t* out_removed);
int gd_dir_lookup_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, gd_val* out_vals,
                      uint8_t* out_found);
/* UniqueKey.GetUniformHashCode of KeyExt keys computed on the device (the hash k_route_keyext
 * uses; 0 for GD_KEYEXT_HOST items).  Host pointers. */
int gd_uniform_hashes_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, uint32_t* out);
/* KeyExt entries, capacity, heap bytes in use. */
int gd_dir_ext_stats(gd_handle* h, uint64_t* live, uint64_t* capacity, uint64_t* heap_bytes);

/* gd_route / gd_route_bucket with KeyExt grains routed on the GPU too (their status is then
 * OK or MISS like any grain; GD_KEYEXT_HOST items stay GD_ROUTE_KEYEXT).  ext == NULL behaves
 * as gd_route.  Host pointers. */
int gd_route_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n,
                 uint32_t* out_silo, uint32_t* out_act, uint8_t* out_status);
int gd_route_bucket_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, uint32_t n_act,
                        uint32_t* out_silo, uint32_t* out_act, uint8_t* out_status,
                        uint32_t* out_perm, uint32_t* out_offsets);
/* Device forms: d_keys and the arrays inside *d_ext are device pointers (d_ext itself is a host
 * struct).  Enqueue only. */
int gd_route_ext_device(gd_handle* h, const gd_key* d_keys, const gd_key_ext* d_ext, uint32_t n,
                        uint32_t* d_silo, uint32_t* d_act, uint8_t* d_status);
int gd_route_bucket_ext_device(gd_handle* h, const gd_key* d_keys, const gd_key_ext* d_ext, uint32_t n,
                               uint32_t n_act, uint32_t* d_silo, uint32_t* d_act, uint8_t* d_status,
                               uint32_t* d_perm, uint32_t* d_offsets);

/* ---- the hot path -------------------------------------------------------------- */
/* Address a batch: ring lookup + directory probe.  Host pointers. */
int gd_route(gd_handle* h, const gd_key* keys, uint32_t n,
             uint32_t* out_silo, uint32_t* out_act, uint8_t* out_status);
/* Per-activation bucketing: stable partition of message indices by activation.
 * acts >= n_act (e.g. GD_NO_ACTIVATION) go to the trailing bucket n_act.
 * out_perm[n]; out_offsets[n_act + 2] (bucket a = [off[a], off[a+1])).  Host pointers. */
int gd_bucket(gd_handle* h, const uint32_t* acts, uint32_t n, uint32_t n_act,
              uint32_t* out_perm, uint32_t* out_offsets);
/* Fused route + bucket.  Host pointers. */
int gd_route_bucket(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t n_act,
                    uint32_t* out_silo, uint32_t* out_act, uint8_t* out_status,
                    uint32_t* out_perm, uint32_t* out_offsets);

/* Device-pointer forms (enqueue only).  Same semantics as above.  One exception to "enqueue only": the
 * first large route after a directory change the probe indexes do not track (rehash, clear, silo
 * removal, merge, split, handoff; gd_index_stats below) rebuilds them (two streaming passes over the
 * table) and synchronises the handle's stream once to read the build's counters;
 * registration / upsert / unregister batches keep the indexes current and routes after them enqueue
 * only.  gd_option_set(GD_OPT_PROBE, 0) turns the indexes off. */
int gd_route_device(gd_handle* h, const gd_key* d_keys, uint32_t n,
                    uint32_t* d_silo, uint32_t* d_act, uint8_t* d_status);
int gd_bucket_device(gd_handle* h, const uint32_t* d_acts, uint32_t n, uint32_t n_act,
                     uint32_t* d_perm, uint32_t* d_offsets);
int gd_route_bucket_device(gd_handle* h, const gd_key* d_keys, uint32_t n, uint32_t n_act,
                           uint32_t* d_silo, uint32_t* d_act, uint8_t* d_status,
                           uint32_t* d_perm, uint32_t* d_offsets);
/* Pipelining of batches (no reference counterpart): with a bucket stream set (non-NULL, not the handle's
 * stream), gd_route_bucket_device enqueues the route on the handle's stream and the bucketing on the
 * bucket stream after it (an event), without making the handle's stream wait: the next batch's route
 * overlaps this batch's bucketing.  The caller must not reuse a batch's act / perm / offsets before the
 * bucket stream has passed them (an event on it, or gd_synchronize, which waits for both streams).
 * NULL restores the default (everything on the handle's stream).  Synchronizes the handle.
 * Measured on MI355X (profiles/r05_pipeline_ab.txt): route and bucketing contend for HBM and L2, and the
 * overlap is slower than the serial order (BASELINE cfg 2 -4 %, cfg 3 -30 %); off by default. */
int gd_set_bucket_stream(gd_handle* h, void* hip_stream);
int gd_ring_owner_device(gd_handle* h, const gd_key* d_keys, uint32_t n, uint32_t* d_silo);

/* ---- multi-GPU helpers (directory sharded by ring owner, SURVEY 8 e) ------------ */
/* Stable partition of a batch by destination shard = owner_silo % n_shards
 * (owner from the installed ring).  Writes the keys in shard order to
 * d_send_keys, the original message index to d_send_idx, and per-shard
 * message counts to d_counts[n_shards].  Device pointers; n_shards <= 256. */
int gd_pack_by_shard_device(gd_handle* h, const gd_key* d_keys, uint32_t n, uint32_t n_shards,
                            gd_key* d_send_keys, uint32_t* d_send_idx, uint32_t* d_counts);
/* The second hop when the directory owner is not the activation's silo (ActivationAddress.Silo,
 * the send after a remote lookup, LocalGrainDirectory.cs:920 -> OutboundMessageQueue.cs:125):
 * stable partition of routed messages by the rank hosting their activation -- status
 * GD_ROUTE_OK: d_silo[i] % n_shards; any other status: my_rank (the message stays on the owner).
 * Writes the keys in rank order to d_send_keys, each message's input position to d_send_pos and
 * per-rank counts to d_counts[n_shards].  Device pointers; n_shards <= 256. */
int gd_pack_routes_by_rank_device(gd_handle* h, const gd_key* d_keys, const uint8_t* d_status,
                                  const uint32_t* d_silo, uint32_t n, uint32_t n_shards, uint32_t my_rank,
                                  gd_key* d_send_keys, uint32_t* d_send_pos, uint32_t* d_counts);

/* ---- in-library exchange over RCCL (SURVEY 8 b gd_route_multi, 8 e) ------------------
 * One process (one handle) per GPU.  Rank r hosts the directory partitions of silos
 * s with s % n_ranks == r (GrainDirectoryPartition per silo, LocalGrainDirectory.cs:477-545).
 * gd_route_multi sends each message of a rank's batch to the rank owning its grain
 * (the per-target-silo outbound queues of OutboundMessageQueue.SendMessage,
 * OutboundMessageQueue.cs:54-131, as one grouped RCCL send/recv over xGMI), probes the
 * directory and buckets per activation there (IncomingMessageAgent.cs:92-190), and with
 * return_routes sends (silo, act, status) back so the sender holds each of its messages'
 * target address in batch order (Dispatcher.AddressMessage, Dispatcher.cs:715-767).
 * RCCL is loaded at run time (librccl.so.1); without it these return GD_ERCCL.
 * The unique id (128 B) is created by one rank and handed to the others by the host
 * (any out-of-band channel); gd_comm_init is collective over all ranks. */
#define GD_COMM_ID_BYTES 128
int gd_comm_unique_id(uint8_t out_id[GD_COMM_ID_BYTES]);
int gd_comm_init(gd_handle* h, const uint8_t id[GD_COMM_ID_BYTES], int n_ranks, int rank);
/* Rehearsal transport: hs[0..n_ranks) (handles of this process, any devices, one host thread
 * driving each) become ranks 0..n_ranks-1 of an in-process communicator whose send/recv are
 * device-to-device copies with RCCL's matching and stream-ordering rules (gd_localcomm.h).  It
 * runs the W > 1 exchange on one GPU, which RCCL refuses (one rank per device).  Each handle
 * leaves it with gd_comm_destroy / gd_destroy. */
int gd_comm_init_local(gd_handle* const* hs, int n_ranks);
int gd_comm_destroy(gd_handle* h);

/* Results of the last gd_route_multi* call on a handle: device pointers into library-owned
 * buffers, valid until the next gd_route_multi* / gd_comm_destroy / gd_destroy.  The received
 * messages are in arrival order = (sender rank, table region, sender batch order): each sender
 * groups its chunk for an owner by the eighth of the owner's directory table the grain's home slot
 * lies in (region 0 for system targets, the membership grain and KeyExt grains), so the owner's
 * probe maps one region to one XCD.  Without header compaction (GD_COMPACT_HEADERS=0) or with
 * GD_REGION_PROBE=0 on the sender, or more than 32 ranks, the order is (sender rank, sender batch
 * order).  One grain has one region, so every activation's messages are in (sender rank, sender
 * batch order) either way; perm / offsets are the stable per-activation bucketing of the arrival
 * order (offsets: n_act + 2 entries). */
typedef struct gd_multi_result {
    uint32_t        n_recv;       /* messages this rank owns in this batch            */
    uint32_t        n_act;
    const gd_key*   recv_keys;    /* [n_recv]                                         */
    const uint32_t* recv_idx;     /* [n_recv] index in the sender's batch             */
    const uint32_t* recv_src;     /* [n_recv] sender rank                             */
    const uint32_t* silo;         /* [n_recv] route results on the owner              */
    const uint32_t* act;
    const uint8_t*  status;
    const uint32_t* perm;         /* [n_recv]                                         */
    const uint32_t* offsets;      /* [n_act + 2]                                      */
    const uint32_t* ret_silo;     /* [n] in this rank's batch order (return_routes)   */
    const uint32_t* ret_act;
    const uint8_t*  ret_status;
} gd_multi_result;

/* flags: GD_MULTI_RETURN_ROUTES -- also send (silo, act, status) back to the senders (ret_*).
 *        GD_MULTI_KEYS_READY    -- d_keys are complete already (their producer was synchronised);
 *        without it the exchange waits for all work enqueued on the handle's stream, which includes
 *        the previous batch's probe + bucketing.  With it, batch i+1's partition and RCCL rounds
 *        (on the library's exchange stream) run while batch i is probed and bucketed (on the
 *        handle's stream).  Results are complete when the handle's stream reaches them
 *        (gd_synchronize, or stream order for later work); they stay valid through the next
 *        call and are overwritten by the one after (two batches in flight).
 * Blocks the host once per call, on the per-rank counts round (it sizes the receive). */
#define GD_MULTI_RETURN_ROUTES 1
#define GD_MULTI_KEYS_READY    2
/* GD_MULTI_FORWARD -- the directory owner is not the activation's silo in general (Orleans
 *        co-locates neither; ActivationAddress.Silo): after the probe on the owner, directory hits
 *        travel on to the rank hosting their activation (silo % n_ranks, a second grouped round,
 *        gd_pack_routes_by_rank_device) and are bucketed there; every other status stays on the
 *        owner.  The result then describes the messages delivered to this rank: recv_idx / recv_src
 *        still name the original sender, silo / act / status are the owner's routes, and each
 *        activation's messages keep (sender rank, sender batch order).  A second host sync (the
 *        forward counts) per call.  Combines with GD_MULTI_RETURN_ROUTES (routes go back from the
 *        owner). */
#define GD_MULTI_FORWARD       4
/* GD_MULTI_NO_KEYS -- the result's recv_keys stay unset (NULL): the receiver identifies each
 *        message by (recv_src, recv_idx).  When every received header was compact in one form
 *        (N1 alone, 4 B when all of a sender's N1s are below 2^32, else 8 B; one TypeCodeData: the
 *        batches of every sender held long-keyed grains of one type) the probe reads the N1s
 *        directly and the 24-B keys are never rebuilt.  Ignored with
 *        GD_MULTI_FORWARD (the keys move on). */
#define GD_MULTI_NO_KEYS       8
int gd_route_multi_device(gd_handle* h, const gd_key* d_keys, uint32_t n, uint32_t n_act, int flags,
                          gd_multi_result* out);
/* Host keys in (C# pinned array), copied on the exchange stream; returns with the batch done
 * (results stay on the device -> gd_multi_fetch). */
int gd_route_multi(gd_handle* h, const gd_key* keys, uint32_t n, uint32_t n_act, int flags,
                   gd_multi_result* out);
/* CalculateTargetSilo (LocalGrainDirectory.cs:477-545) with KeyExt strings: the owner silo the
 * exchange partition uses (system targets / KeyExt without a string -> my silo, the membership
 * grain -> the seed).  Host pointers. */
int gd_ring_owner_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, uint32_t* out_silo);
/* With the batch's KeyExt strings (gd_key_ext, as gd_route_ext): KeyExt grains go to the rank
 * owning their KeyExt hash, their strings travel in a byte round after the header round, and they
 * are routed there like any grain (without ext they stay on the sender, status GD_ROUTE_KEYEXT).
 * The _device form takes device arrays inside *d_ext. */
int gd_route_multi_ext_device(gd_handle* h, const gd_key* d_keys, const gd_key_ext* d_ext, uint32_t n,
                              uint32_t n_act, int flags, gd_multi_result* out);
int gd_route_multi_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, uint32_t n_act,
                       int flags, gd_multi_result* out);
/* Copy the last result to host arrays sized from gd_multi_result (any pointer may be NULL). */
int gd_multi_fetch(gd_handle* h, gd_key* recv_keys, uint32_t* recv_idx, uint32_t* recv_src, uint32_t* silo,
                   uint32_t* act, uint8_t* status, uint32_t* perm, uint32_t* offsets, uint32_t* ret_silo,
                   uint32_t* ret_act, uint8_t* ret_status);

/* ---- micro-batch latency path (BASELINE config 5) ----------------------
 * Small batches (e.g. 4k messages: Presence / GPSTracker traffic,
 * Samples/GPSTracker/GPSTracker.GrainImplementation/DeviceGrain.cs:18-37) pay launch
 * and copy overheads, not bandwidth.  A micro-batch owns pinned host buffers and
 * device buffers; the whole step (H2D keys -> route -> one-workgroup stable sort by
 * activation -> one D2H of every result) is captured once per batch size as a hipGraph
 * and replayed.  Instead of gd_bucket's n_act+2 offsets it returns the runs of the
 * activations present: run r = activation run_act[r] (n_act for acts >= n_act), its
 * messages perm[run_start[r] .. run_start[r+1]) in arrival order; run_start[n_runs] = n.
 * The caller writes gd_microbatch_keys(), calls gd_microbatch_run(), reads the outputs. */
#define GD_MICROBATCH_MAX 8192u
typedef struct gd_microbatch gd_microbatch;
int      gd_microbatch_create(gd_handle* h, uint32_t capacity, uint32_t n_act, gd_microbatch** out);
void     gd_microbatch_destroy(gd_microbatch* mb);
gd_key*  gd_microbatch_keys(gd_microbatch* mb);                     /* pinned, capacity entries */
/* Pinned host results, valid after gd_microbatch_run: silo/act/status/perm[capacity],
 * n_runs[1], run_start[capacity + 1], run_act[capacity]. */
int      gd_microbatch_outputs(gd_microbatch* mb, uint32_t** silo, uint32_t** act, uint8_t** status,
                               uint32_t** perm, uint32_t** n_runs, uint32_t** run_start, uint32_t** run_act);
/* Route + bucket the first n keys (n <= capacity <= GD_MICROBATCH_MAX); synchronous.
 * use_graph = 0 runs the same launches eagerly; the graph for a given n is captured on first use. */
int      gd_microbatch_run(gd_microbatch* mb, uint32_t n, int use_graph);

/* ---- batched header decode -------------------------------------------
 * Replaces, for the fields the dispatch path reads, the per-message
 * HeadersContainer.Deserializer (src/Orleans.Core/Messaging/Message.cs:1247-1356) run by
 * IncomingMessageBuffer (src/Orleans.Core/Messaging/IncomingMessageBuffer.cs) over each frame
 * [int32 headerLength][int32 bodyLength][header][body] (Message.cs:481-516).  The caller hands
 * over the receive buffer as is plus the byte offset of every frame (the receive loop already
 * knows them from the two length prefixes). */
#define GD_FRAME_HAS_TARGET     0x01u /* TargetGrain decoded                                       */
#define GD_FRAME_COMPLETE       0x02u /* TargetGrain + TargetActivation + TargetSilo bits set:
                                         TargetAddress.IsComplete -> AddressMessage skips it        */
#define GD_FRAME_FALLBACK       0x04u /* an object-serialized field precedes a field read here:
                                         CacheInvalidationHeader / RequestContext -> nothing decoded;
                                         TargetObserver -> all but TargetSilo decoded. C# decodes it */
#define GD_FRAME_MALFORMED      0x08u /* lengths run past the header or the buffer: nothing decoded  */
#define GD_FRAME_TARGET_KEYEXT  0x10u /* TargetGrain carries a KeyExt string (not returned)          */

#define GD_ROUTE_ADDRESSED      5 /* frame address already complete: not looked up (Dispatcher.cs:718) */
#define GD_ROUTE_UNDECODED      6 /* no TargetGrain decoded (absent / fallback / malformed): C# path    */

/* Output arrays, n entries each.  flags and target_grain are required; any other pointer may
 * be NULL (field not extracted).  Absent fields read 0 (direction: 0xFF = null).  Silo
 * addresses are the 24-byte wire form (16-byte IP, int32 port, int32 generation,
 * BinaryTokenStreamWriter.cs:485-513), 4-byte aligned. */
typedef struct gd_frame_fields {
    uint32_t* flags;               /* GD_FRAME_* */
    gd_key*   target_grain;
    uint32_t* mask;                /* HeadersContainer.Headers bits (Message.cs:728-765) */
    gd_key*   target_activation;
    gd_key*   sending_activation;
    gd_key*   sending_grain;
    uint8_t*  target_silo;         /* 24 B per frame */
    uint8_t*  sending_silo;        /* 24 B per frame */
    int64_t*  correlation_id;
    uint8_t*  category;            /* Message.Categories */
    uint8_t*  direction;           /* Message.Directions, 0xFF = null */
} gd_frame_fields;

/* Device pointers; enqueue only.  frame_off[i] = byte offset of frame i in buf. */
int gd_decode_frames_device(gd_handle* h, const uint8_t* d_buf, uint64_t buf_len, const uint64_t* d_frame_off,
                            uint32_t n, const gd_frame_fields* d_out);
/* Host pointers (buffer, offsets and outputs); synchronous. */
int gd_decode_frames(gd_handle* h, const uint8_t* buf, uint64_t buf_len, const uint64_t* frame_off, uint32_t n,
                     const gd_frame_fields* out);
/* Decode -> route -> (optional) bucket, device pointers, enqueue only.  d_out receives the
 * decoded fields (flags + target_grain required).  Statuses are gd_route's plus
 * GD_ROUTE_ADDRESSED / GD_ROUTE_UNDECODED (silo = act = GD_NO_*, trailing bucket).  With an
 * ActivationDirectory (gd_actdir_add), an ADDRESSED frame whose TargetActivation FindTarget finds
 * Valid gets that context as its act and is bucketed with it (IncomingMessageAgent.cs:131-152).
 * d_perm / d_offsets NULL = no bucketing. */
int gd_route_frames_device(gd_handle* h, const uint8_t* d_buf, uint64_t buf_len, const uint64_t* d_frame_off,
                           uint32_t n, uint32_t n_act, const gd_frame_fields* d_out, uint32_t* d_silo,
                           uint32_t* d_act, uint8_t* d_status, uint32_t* d_perm, uint32_t* d_offsets);
/* Host-pointer form of gd_route_frames_device (flags + target keys are returned through out
 * when it is non-NULL; perm/offsets NULL = no bucketing); synchronous. */
int gd_route_frames(gd_handle* h, const uint8_t* buf, uint64_t buf_len, const uint64_t* frame_off, uint32_t n,
                    uint32_t n_act, const gd_frame_fields* out, uint32_t* out_silo, uint32_t* out_act,
                    uint8_t* out_status, uint32_t* out_perm, uint32_t* out_offsets);
/* The same with KeyExt targets (string-keyed grains) routed on the GPU as gd_route_ext does:
 * each TargetGrain's KeyExt string is read from the frame buffer where the decoder found it. */
int gd_route_frames_ext_device(gd_handle* h, const uint8_t* d_buf, uint64_t buf_len, const uint64_t* d_frame_off,
                               uint32_t n, uint32_t n_act, const gd_frame_fields* d_out, uint32_t* d_silo,
                               uint32_t* d_act, uint8_t* d_status, uint32_t* d_perm, uint32_t* d_offsets);
int gd_route_frames_ext(gd_handle* h, const uint8_t* buf, uint64_t buf_len, const uint64_t* frame_off, uint32_t n,
                        uint32_t n_act, const gd_frame_fields* out, uint32_t* out_silo, uint32_t* out_act,
                        uint8_t* out_status, uint32_t* out_perm, uint32_t* out_offsets);

/* ---- membership change ------------------------------------------------
 * GrainDirectoryPartition.Split(predicate, modifyOrigin) (GrainDirectoryPartition.cs:532-570)
 * with the handoff predicate "CalculateTargetSilo(grain) is not me"
 * (GrainDirectoryHandoffManager.cs:212-218), evaluated on the GPU under the installed ring
 * (install the new ring with gd_ring_set first).  "me" = the silos whose partitions this
 * handle holds: keep_silo[s] != 0 (silo indices >= n_keep count as not kept).  Selected live
 * entries are written in slot order; move != 0 also removes them (the RemoveGrain after
 * RegisterMany, :228-232).  KeyExt grains are never selected (their owner needs the C# hash).
 * out_keys == NULL: size query only (*out_n = entries selected, nothing moved).  The merge on
 * the receiving handle is gd_dir_register (GrainDirectoryPartition.Merge, :497-520: entries
 * already present keep their activation and are reported; the host applies the reference's
 * smallest-ActivationId rule to those). */
int gd_dir_split(gd_handle* h, const uint8_t* keep_silo, uint32_t n_keep, int move, gd_key* out_keys,
                 gd_val* out_vals, uint64_t out_capacity, uint64_t* out_n);
/* The same split over the KeyExt table (string-keyed grains): the owner of each entry's stored
 * uniform hash under the installed ring.  Entries in slot order with their KeyExt strings:
 * out_length[i] (GD_KEYEXT_NULL for a null KeyExt), out_offset[i] into out_bytes.  out_keys == NULL:
 * size query (*out_n entries, *out_nbytes string bytes).  Host pointers; the merge on the receiving
 * handle is gd_dir_register_ext. */
int gd_dir_split_ext(gd_handle* h, const uint8_t* keep_silo, uint32_t n_keep, int move, gd_key* out_keys,
                     gd_val* out_vals, uint64_t* out_offset, int32_t* out_length, uint8_t* out_bytes,
                     uint64_t capacity, uint64_t bytes_capacity, uint64_t* out_n, uint64_t* out_nbytes);
/* Same, device output arrays (keep_silo stays a host array); synchronous. */
int gd_dir_split_device(gd_handle* h, const uint8_t* keep_silo, uint32_t n_keep, int move, gd_key* d_out_keys,
                        gd_val* d_out_vals, uint64_t out_capacity, uint64_t* out_n);

/* ---- follower fan-out (BASELINE cfg 4) -----------------------------------
 * ChirperAccount.PublishMessage (Samples/Chirper/ChirperGrains/ChirperAccount.cs:106-147): each
 * publisher sends IChirperSubscriber.NewChirp to every follower, in State.Followers enumeration
 * order (:131-134).  The follower graph is CSR over node ids, where node u is the grain
 * GrainId(type_code, (long)u) (GrainId.cs:72-77): row_off[n_nodes + 1] (u32, row_off[n_nodes] =
 * edges < 2^32), dst[edges] = the followers of u in row_off[u]..row_off[u+1], in enumeration
 * order.  One hop over a frontier of publishers emits, in this order,
 *     for i in 0..n_frontier:  for each follower f of frontier[i]:  (target f, sender frontier[i])
 * Publishers >= n_nodes have no followers.  *out_n = messages emitted (the hop's size; computed
 * on the device and read back, so these calls synchronise).  capacity = room in the outputs;
 * more messages than that is GD_EINVAL with *out_n set (a size query).  All ids are u32. */
/* Expansion only (the multi-GPU path ships (target, sender) to the owner).  d_target == NULL:
 * size query. */
int gd_fanout_expand_device(gd_handle* h, const uint32_t* d_row_off, const uint32_t* d_dst, uint32_t n_nodes,
                            const uint32_t* d_frontier, uint32_t n_frontier, uint32_t* d_target, uint32_t* d_sender,
                            uint64_t capacity, uint64_t* out_n);
/* Fused expansion + route (GrainId formed in registers, K0+K1+K2 as gd_route) + optional
 * bucketing by activation (d_perm / d_offsets NULL = none; as gd_bucket over d_act).
 * d_target may be NULL. */
int gd_fanout_route_bucket_device(gd_handle* h, const uint32_t* d_row_off, const uint32_t* d_dst, uint32_t n_nodes,
                                  const uint32_t* d_frontier, uint32_t n_frontier, int32_t type_code, uint32_t n_act,
                                  uint32_t* d_target, uint32_t* d_sender, uint32_t* d_silo, uint32_t* d_act,
                                  uint8_t* d_status, uint32_t* d_perm, uint32_t* d_offsets, uint64_t capacity,
                                  uint64_t* out_n);
/* Host-pointer form (graph, frontier and outputs in host memory; any output may be NULL
 * except that perm and offsets go together). */
int gd_fanout_route_bucket(gd_handle* h, const uint32_t* row_off, const uint32_t* dst, uint32_t n_nodes,
                           const uint32_t* frontier, uint32_t n_frontier, int32_t type_code, uint32_t n_act,
                           uint32_t* out_target, uint32_t* out_sender, uint32_t* out_silo, uint32_t* out_act,
                           uint8_t* out_status, uint32_t* out_perm, uint32_t* out_offsets, uint64_t capacity,
                           uint64_t* out_n);
/* gd_route_device for GrainId(type_code, (long)node) given node ids (4 B per message instead of
 * a 24-B key): the owner side of the sharded fan-out. */
int gd_route_nodes_device(gd_handle* h, const uint32_t* d_nodes, uint32_t n, int32_t type_code, uint32_t* d_silo,
                          uint32_t* d_act, uint8_t* d_status);
/* gd_pack_by_shard_device for (node, payload) pairs: stable partition by owner silo % n_shards
 * under the installed ring (OutboundMessageQueue.cs:54-131 per target silo). */
int gd_pack_nodes_by_shard_device(gd_handle* h, const uint32_t* d_nodes, const uint32_t* d_payload, uint32_t n,
                                  int32_t type_code, uint32_t n_shards, uint32_t* d_send_nodes,
                                  uint32_t* d_send_payload, uint32_t* d_counts);
/* Next cascade frontier from a hop's bucketing: activations a < n_act with
 * d_offsets[a+1] > d_offsets[a] and d_visited[a] == 0, ascending; marks them visited.
 * d_out holds n_act entries; *out_n = frontier size (synchronises). */
int gd_frontier_next_device(gd_handle* h, const uint32_t* d_offsets, uint32_t n_act, uint8_t* d_visited,
                            uint32_t* d_out, uint32_t* out_n);

/* ---- the sharded fan-out cascade (BASELINE cfg 4 across GPUs: SURVEY 8 f2 over 8 e) ---------
 * Over the library's communicator (gd_comm_init / gd_comm_init_local): rank r owns the directory
 * partitions of silos s % n_ranks == r, as in gd_route_multi; the follower graph is replicated.
 * From `seeds` (the same array on every rank) each rank takes the seeds whose grain it owns, in seed
 * order, and marks them published.  Then per hop, on every rank:
 *   expand its publishers (ChirperAccount.cs:131-134, as gd_fanout_expand_device) -> stable
 *   partition of the (target, sender) pairs by the target's owner rank (the per-silo outbound
 *   queues, OutboundMessageQueue.cs:54-131) -> one grouped send/recv round, 8 B a message ->
 *   route the targets and bucket per activation on the owner, in arrival order = (sender rank,
 *   sender emission order) -> the next publishers: this rank's activations that received a chirp
 *   and have not published yet, ascending (gd_frontier_next_device).
 * Collective: every rank calls it with the same seeds, hops and n_act.  out[hops] (may be NULL):
 * device pointers into library-owned buffers, valid until the next call on the handle,
 * gd_comm_destroy or gd_destroy.  Blocks the host twice per hop (the hop's size, the counts round). */
typedef struct gd_fanout_hop {
    uint32_t        n_frontier;   /* this rank's publishers of the hop                        */
    const uint32_t* frontier;
    uint64_t        n_sent;       /* messages they emitted                                    */
    uint32_t        n_recv;       /* messages delivered here (this rank owns their grain)     */
    const uint32_t* target;       /* [n_recv] follower node, arrival order                    */
    const uint32_t* sender;       /* [n_recv] publisher node                                  */
    const uint32_t* src;          /* [n_recv] sending rank                                    */
    const uint32_t* silo;         /* [n_recv] route results (as gd_route_nodes_device)        */
    const uint32_t* act;
    const uint8_t*  status;
    const uint32_t* perm;         /* [n_recv] stable per-activation order                     */
    const uint32_t* offsets;      /* [n_act + 2]                                              */
} gd_fanout_hop;
int gd_fanout_multi_device(gd_handle* h, const uint32_t* d_row_off, const uint32_t* d_dst, uint32_t n_nodes,
                           const uint32_t* d_seeds, uint32_t n_seeds, int32_t type_code, uint32_t n_act,
                           uint32_t hops, gd_fanout_hop* out);
/* The same cascade over a partitioned follower graph: each rank holds only the
 * follower lists of the grains it owns -- the publishers a rank expands are always its own activations
 * (a chirp is enqueued on its follower's activation, on the follower's directory owner, which then
 * publishes; ChirperAccount.cs:131-134) -- so per-rank graph memory is ~1/n_ranks.  Row i of this
 * rank's CSR (d_row_off[n_rows + 1], d_dst = follower node ids) is local activation i, whose node is
 * d_node_of[i]; the directory must map each owned node to its row (act = i), with rows in ascending
 * node order so that publishers run in the replicated form's order (the hops are then bit-identical
 * to gd_fanout_multi_device's).  Every seed needs a live activation on its owner (else GD_EINVAL).
 * n_act = n_rows: buckets and offsets are over local rows; frontier, target and sender are node ids. */
int gd_fanout_multi_part_device(gd_handle* h, const uint32_t* d_row_off, const uint32_t* d_dst, uint32_t n_rows,
                                const uint32_t* d_node_of, const uint32_t* d_seeds, uint32_t n_seeds,
                                int32_t type_code, uint32_t hops, gd_fanout_hop* out);
/* Host graph and seeds (uploaded per call); returns with the cascade done. */
int gd_fanout_multi(gd_handle* h, const uint32_t* row_off, const uint32_t* dst, uint32_t n_nodes,
                    const uint32_t* seeds, uint32_t n_seeds, int32_t type_code, uint32_t n_act, uint32_t hops,
                    gd_fanout_hop* out);
/* The single-GPU cascade inside the library (BASELINE cfg 4 on one GPU; what gd_fanout_route_bucket
 * + gd_frontier_next do hop by hop from the host): `seeds` publish in seed order, then per hop the
 * fused expand + route (ChirperAccount.cs:131-134), the bucketing per activation and the next
 * publishers (this handle's activations that received a chirp and have not published, ascending).
 * Node u = activation u (n_act >= the nodes that have activations).  One host read-back a hop (the
 * next hop's message and publisher counts together, the frontier's size staying on the device until
 * then).  out[hops] (may be NULL): device pointers into library buffers as gd_fanout_multi_device's
 * (src = NULL); gd_fanout_multi_fetch copies a hop out (src as zeros). */
int gd_fanout_cascade_device(gd_handle* h, const uint32_t* d_row_off, const uint32_t* d_dst, uint32_t n_nodes,
                             const uint32_t* d_seeds, uint32_t n_seeds, int32_t type_code, uint32_t n_act,
                             uint32_t hops, gd_fanout_hop* out);
/* Copy hop `hop` of the last cascade to host arrays sized from its gd_fanout_hop (any may be NULL). */
int gd_fanout_multi_fetch(gd_handle* h, uint32_t hop, uint32_t* frontier, uint32_t* target, uint32_t* sender,
                          uint32_t* src, uint32_t* silo, uint32_t* act, uint8_t* status, uint32_t* perm,
                          uint32_t* offsets);

/* ---- non-owner directory cache -------------------------------------------
 * AdaptiveGrainDirectoryCache over LRU<GrainId, entry> (src/Orleans.Runtime/GrainDirectory/
 * AdaptiveGrainDirectoryCache.cs:7-140, src/Orleans.Core/Utils/LRU.cs) on the LocalLookup path
 * (LocalGrainDirectory.cs:797-850).  Configured (max_size > 0), gd_route / gd_route_device /
 * gd_route_bucket[_device] run LocalLookup per message: a grain whose ring owner is a local
 * silo (local_silo[owner] != 0) is probed in this handle's directory partition; any other grain
 * in the cache.  A cache hit whose silo is not valid (valid_silo[silo] == 0, IsValidSilo) is
 * GD_ROUTE_MISS, as is a cache miss (silo = ring owner, act = GD_NO_ACTIVATION).  The LRU is the
 * reference's exactly: every hit and every add takes the next generation (hits in batch order),
 * AdjustSize evicts the lowest generation while count >= max_size.  max_size 0 = no cache
 * (whole-node mode: every grain is probed in this handle's table).  The frame and micro-batch
 * paths run LocalLookup too (the micro-batch eagerly in this mode); the fan-out paths do not
 * consult the cache. */
typedef struct gd_cache_stats {
    uint64_t count;             /* live entries (LRU.Count)                       */
    uint64_t accesses;          /* NumAccesses                                     */
    uint64_t hits;              /* NumHits                                         */
    uint64_t next_generation;   /* LRU.nextGeneration                              */
    uint64_t max_size;
    uint64_t capacity;          /* table slots                                     */
} gd_cache_stats;
int gd_cache_configure(gd_handle* h, uint32_t max_size, const uint8_t* local_silo, const uint8_t* valid_silo,
                       uint32_t n_silos);
/* Membership change: new local / valid silo masks; entries stay (the maintainer refreshes them). */
int gd_cache_set_silos(gd_handle* h, const uint8_t* local_silo, const uint8_t* valid_silo, uint32_t n_silos);
/* AddOrUpdate(key, value, version) for each entry in order (after a remote lookup, :920). */
int gd_cache_add(gd_handle* h, const gd_key* keys, const gd_val* vals, const int32_t* versions, uint32_t n);
/* Remove (:79-83); out_removed may be NULL. */
int gd_cache_remove(gd_handle* h, const gd_key* keys, uint32_t n, uint8_t* out_removed);
/* LookUp (:90-109) in order: value + version (ETag) of hits. */
int gd_cache_lookup(gd_handle* h, const gd_key* keys, uint32_t n, gd_val* out_vals, int32_t* out_versions,
                    uint8_t* out_found);
int gd_cache_clear(gd_handle* h);
int gd_cache_stats_get(gd_handle* h, gd_cache_stats* out);
/* KeyValues (:111-127) with each entry's generation, in slot order; keys NULL = size query. */
int gd_cache_entries(gd_handle* h, gd_key* keys, gd_val* vals, int32_t* versions, uint64_t* generations,
                     uint64_t capacity, uint64_t* out_n);
/* KeyExt grains (string, compound keys, geo clients: UniqueKey.HasKeyExt) in the cache, keyed by their
 * KeyExt as UniqueKey.Equals is (UniqueKey.cs:245-251) and homed by the KeyExt uniform hash
 * (UniqueKey.cs:272-336).  gd_route_ext / gd_route_bucket_ext[_device] / gd_route_frames_ext* in
 * LocalLookup mode route KeyExt grains the same way as the three-word ones: the owner by the KeyExt
 * hash, a local owner's grains in this handle's KeyExt partition (gd_dir_register_ext), the others
 * in the cache (AdaptiveGrainDirectoryCache.cs:93-110), every hit of the batch numbered in batch
 * order.  One LRU holds both kinds (one generation sequence, one max_size).  `ext` is read for
 * KeyExt-category keys only; GD_KEYEXT_NULL there is the three-word entry, GD_KEYEXT_HOST is
 * GD_EINVAL.  The plain forms above treat a KeyExt-category key as KeyExt null. */
int gd_cache_add_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, const gd_val* vals,
                     const int32_t* versions, uint32_t n);
int gd_cache_remove_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, uint8_t* out_removed);
int gd_cache_lookup_ext(gd_handle* h, const gd_key* keys, const gd_key_ext* ext, uint32_t n, gd_val* out_vals,
                        int32_t* out_versions, uint8_t* out_found);
/* gd_cache_entries with each entry's KeyExt: ext_len[k] (GD_KEYEXT_NULL for a three-word key), its
 * UTF-8 bytes at ext_bytes + ext_off[k]; *out_bytes = the bytes all strings need.  keys NULL = size
 * query (*out_n, *out_bytes). */
int gd_cache_entries_ext(gd_handle* h, gd_key* keys, gd_val* vals, int32_t* versions, uint64_t* generations,
                         int32_t* ext_len, uint64_t* ext_off, uint8_t* ext_bytes, uint64_t capacity,
                         uint64_t bytes_capacity, uint64_t* out_n, uint64_t* out_bytes);

/* ---- membership change: IsValidSilo, VersionTag, silo removal, handoff merge ----
 * GrainDirectoryPartition.IsValidSilo (GrainDirectoryPartition.cs:242-245, the membership oracle's
 * IsFunctionalDirectory): valid[s] != 0 for every silo index s < n_silos that is a functional
 * directory member; silo indices >= n_silos count as valid; n_silos = 0 = every silo valid (the
 * default).  With the mask set:
 *   - gd_dir_register / gd_dir_register_device / gd_dir_register_ext (AddSingleActivation, :304-326)
 *     and gd_dir_upsert (AddActivation, :274-302) skip an item whose silo is not valid (no entry, out
 *     value {GD_NO_ACTIVATION, GD_NO_SILO}, not inserted);
 *   - LookUpActivations (:385-441) filters an entry on an invalid silo: routes give GD_ROUTE_MISS (an
 *     empty address list fails FastLookup, Catalog.cs:1321-1330), gd_dir_lookup_tagged reports it. */
int gd_dir_set_valid_silos(gd_handle* h, const uint8_t* valid, uint32_t n_silos);
/* LookUpActivations with its VersionTag: out_found[i] = 0 no entry (tag 0, the AddressesAndTag
 * default), 1 an entry with a valid address (out_vals), 2 an entry whose activation's silo is not
 * valid (empty address list; tag still given).  VersionTags are non-negative int32.  The reference
 * draws a fresh rand.Next() whenever a grain's entry changes (GrainInfo :106,120,135,154); this
 * library gives a deterministic 31-bit function of (the mutating call's sequence number, the grain's
 * uniform hash), changed exactly where the reference draws one.  Host pointers. */
int gd_dir_lookup_tagged(gd_handle* h, const gd_key* keys, uint32_t n, gd_val* out_vals, int32_t* out_tags,
                         uint8_t* out_found);
/* RemoveServer's AdjustLocalDirectory (LocalGrainDirectory.cs:340-361): every entry whose activation
 * lives on one of the removed silos is dropped (RemoveActivation, Force; single-activation grains lose
 * their grain).  Multi-activation entries (GD_ACT_MULTI) are counted in *out_multi and left to the host
 * (their instance silos live in C#).  In LocalLookup mode (gd_cache_configure) also AdjustLocalCache
 * (:371-385) under the installed ring -- install the ring without the removed silos first: cache
 * entries pointing at a removed silo or whose grain a local silo now owns are removed
 * (*out_cache_removed).  KeyExt entries follow the same rule.  Any out pointer may be NULL. */
int gd_dir_remove_silos(gd_handle* h, const uint32_t* silos, uint32_t n_silos, uint64_t* out_removed,
                        uint64_t* out_multi, uint64_t* out_cache_removed);
/* The ActivationId (ActivationId.cs; a UniqueKey, NewId = Guid with Category None) of host activation
 * indices: ids[i] for acts[i].  gd_dir_merge orders activations by it (UniqueKey.CompareTo,
 * UniqueKey.cs:255-265: TypeCodeData, N0, N1).  Host pointers. */
int gd_activation_ids_set(gd_handle* h, const uint32_t* acts, const gd_key* ids, uint32_t n);
/* GrainDirectoryPartition.Merge (GrainDirectoryPartition.cs:497-522) of a received partition (the copy
 * merged by GrainDirectoryHandoffManager.ProcessSiloRemoveEvent, :125-158): one item per grain (a
 * duplicated grain fails with GD_EINVAL and changes nothing).  Per item:
 *   GD_MERGE_INSERTED  the grain was absent: the incoming entry is added with its VersionTag
 *                      (tags[i]; tags NULL = a new tag)
 *   GD_MERGE_SAME      the same activation is registered: nothing changes (GrainInfo.Merge :146)
 *   GD_MERGE_KEPT      single-activation grain, the incoming ActivationId is the lower: it replaces the
 *                      existing entry (GrainInfo.Merge :159-176); out_dropped[i] = the displaced one
 *   GD_MERGE_DROPPED   the existing ActivationId is the lower: out_dropped[i] = the incoming activation
 *   GD_MERGE_UNION     a multi-instance grain holding one instance here meets another: both kept (below)
 *   GD_MERGE_HOST      a grain with several instances on either side (its lists are unioned by C#)
 * out_dropped lists what Catalog.DeleteActivations gets per silo (:514-518); {GD_NO_*} otherwise.  Both
 * activations of a conflict need an ActivationId (gd_activation_ids_set), else GD_EINVAL.  No
 * IsValidSilo check (Merge has none).  Host pointers; out_dropped may be NULL. */
#define GD_MERGE_INSERTED 0
#define GD_MERGE_KEPT     1
#define GD_MERGE_SAME     2
#define GD_MERGE_DROPPED  3
#define GD_MERGE_HOST     4
/* GD_MERGE_UNION     the grain here is a multi-instance one (AddActivation, SingleInstance false) holding
 *                    one instance, and the incoming instance is another: GrainInfo.Merge unions the lists
 *                    (:141-152) and keeps both; the entry becomes GD_ACT_MULTI with a new VersionTag and
 *                    the host adds the incoming instance to its list */
#define GD_MERGE_UNION    5
/* tags[i] | GD_MERGE_TAG_MULTI_INSTANCE: the incoming GrainInfo is not SingleInstance (an AddActivation
 * grain holding one instance); partitionData.Add keeps it so (tags NULL: single unless GD_ACT_MULTI). */
#define GD_MERGE_TAG_MULTI_INSTANCE 0x80000000u
int gd_dir_merge(gd_handle* h, const gd_key* keys, const gd_val* vals, const int32_t* tags, uint32_t n,
                 uint8_t* out_status, gd_val* out_dropped);

/* ---- multi-rank directory handoff (SURVEY 8 f4 over 8 e) ------------------------------------------
 * After a membership change (the new ring installed on every rank with gd_ring_set), each rank splits
 * off the entries whose new owner silo it does not host (keep_silo as gd_dir_split, removed here), they
 * travel to the owner's rank (silo % n_ranks) in one grouped round over the library's communicator with
 * their ActivationId (gd_activation_ids_set) and VersionTag, and the receiver applies them as the
 * reference distinguishes the two events (GrainDirectoryHandoffManager.cs):
 *   GD_HANDOFF_ADD     ProcessSiloAddEvent (:195-245): RegisterMany(singleActivation: true) --
 *                      AddSingleActivation, the first registration wins (GrainDirectoryPartition.cs:304-326)
 *   GD_HANDOFF_REMOVE  ProcessSiloRemoveEvent (:125-158): GrainDirectoryPartition.Merge (:497-522) --
 *                      GrainInfo.Merge keeps the lowest ActivationId (:139-179), the incoming VersionTag
 *                      and SingleInstance flag travel with the entry
 * Received entries take this handle's activation indices act_base + j (j = arrival position; their
 * ActivationIds are set at those indices as by gd_activation_ids_set); multi-activation entries stay
 * GD_ACT_MULTI (their instance lists are the host's).  Per received entry, status:
 *   GD_MERGE_INSERTED  the grain was absent here: the entry is added
 *   GD_MERGE_SAME      the same ActivationId already holds the grain
 *   GD_MERGE_KEPT      (REMOVE) the incoming ActivationId is the lower: it replaces the holder;
 *                      dropped = the displaced {act, silo} (Catalog.DeleteActivations on that silo)
 *   GD_MERGE_DROPPED   REMOVE: the holder's ActivationId is the lower, dropped = the incoming entry;
 *                      ADD: another activation holds the grain (first registration wins) or the silo is
 *                      not valid, dropped = the holder (none when refused)
 *   GD_MERGE_HOST      a multi-activation entry on either side: C# unions the instance lists
 * Collective over the communicator; synchronous.  The result's device arrays (arrival order = sender
 * rank, sender slot order) stay valid until the next call, gd_comm_destroy or gd_destroy. */
#define GD_HANDOFF_ADD    0
#define GD_HANDOFF_REMOVE 1
typedef struct gd_handoff_result {
    uint64_t        n_sent;       /* entries this rank split off and sent              */
    uint32_t        n_recv;       /* entries received                                  */
    const gd_key*   recv_keys;    /* [n_recv] GrainIds                                 */
    const gd_key*   recv_ids;     /* [n_recv] ActivationIds (zero for multi-activation) */
    const uint32_t* recv_act;     /* [n_recv] activation index here (GD_ACT_MULTI kept) */
    const uint32_t* recv_silo;    /* [n_recv] silo index (bit 31: a multi-activation entry) */
    const uint32_t* recv_src;     /* [n_recv] sending rank                             */
    const uint8_t*  status;       /* [n_recv] GD_MERGE_*                               */
    const gd_val*   dropped;      /* [n_recv] see above; {GD_NO_*} otherwise           */
} gd_handoff_result;
int gd_dir_handoff_multi(gd_handle* h, const uint8_t* keep_silo, uint32_t n_keep, int event, uint32_t act_base,
                         gd_handoff_result* out);
/* Host copies of the last handoff's received entries (any pointer may be NULL; silos without the
 * multi-activation mark). */
int gd_dir_handoff_fetch(gd_handle* h, gd_key* keys, gd_key* ids, uint32_t* acts, uint32_t* silos, uint32_t* src,
                         uint8_t* status, gd_val* dropped);

/* ---- receive path: ActivationDirectory + IncomingMessageAgent -----------------
 * ActivationDirectory (src/Orleans.Runtime/Catalog/ActivationDirectory.cs): ActivationId -> the
 * host's scheduling-context index + flags, in an HBM table.  Activations (RecordNewTarget :86-93) and
 * system targets (RecordNewSystemTarget :95-98, flag GD_ACTDIR_SYSTEM_TARGET) share one table and
 * one context index space; FindTarget (:41-45) sees only activations, FindSystemTarget (:47-51) only
 * system targets.  Use the grain directory's activation index as the context index of a local
 * activation, so gd_route_frames' addressed frames and gd_bucket agree. */
#define GD_ACTDIR_VALID            1u  /* ActivationData.State == Valid                          */
#define GD_ACTDIR_SYSTEM_TARGET    2u  /* an entry of systemTargets                               */
#define GD_ACTDIR_STATELESS_WORKER 4u  /* IsStatelessWorker: the *_StatelessWorker limits apply    */
/* TryAdd (first add of an ActivationId wins); out_added may be NULL. */
int gd_actdir_add(gd_handle* h, const gd_key* act_ids, const uint32_t* ctx, const uint8_t* flags, uint32_t n,
                  uint8_t* out_added);
/* TryRemove (RemoveTarget :116-131); out_removed may be NULL. */
int gd_actdir_remove(gd_handle* h, const gd_key* act_ids, uint32_t n, uint8_t* out_removed);
/* State changes (ActivationData.SetState): new flags, batch order (last wins); out_found may be NULL. */
int gd_actdir_set_flags(gd_handle* h, const gd_key* act_ids, const uint8_t* flags, uint32_t n, uint8_t* out_found);
int gd_actdir_lookup(gd_handle* h, const gd_key* act_ids, uint32_t n, uint32_t* out_ctx, uint8_t* out_flags,
                     uint8_t* out_found);
int gd_actdir_clear(gd_handle* h);
int gd_actdir_count(gd_handle* h, uint64_t* out_live);

/* IncomingMessageAgent.ReceiveMessage (IncomingMessageAgent.cs:92-170) for a batch in arrival order.
 * Per message, from TargetGrain (its category), TargetActivation and Direction (NULL array = every
 * message a Request; 0xFF = header absent = Request, Message.cs:113-116):
 *   GD_RECV_ACTIVATION      FindTarget found a Valid activation: enqueued on its context
 *   GD_RECV_SYSTEM_TARGET   FindSystemTarget found it, Request or Response: enqueued on its context
 *   GD_RECV_NULL_CONTEXT    no activation, or not Valid: EnqueueReceiveMessage(msg, null, null)
 *   GD_RECV_REJECT_UNKNOWN  system target not active here: rejection response (Unrecoverable)
 *   GD_RECV_REJECT_OVERLOADED  CheckOverloaded's hard limit (ActivationData.cs:616-649), see limits
 *   GD_RECV_DROPPED         system target message neither Request nor Response (logged, dropped)
 *   GD_RECV_UNDECODED       (frames) no complete decoded address: C# deserializes it
 * out_ctx[i] = the bucket it is enqueued in: the context index (< n_ctx), n_ctx for the null context,
 * GD_NO_ACTIVATION when not enqueued.  perm / offsets (both or neither): the stable bucketing of the
 * batch over n_ctx + 2 buckets -- contexts, the null context, then the messages not enqueued -- each
 * in arrival order (WorkItemGroup FIFO, WorkItemGroup.cs:174-201); offsets has n_ctx + 3 entries.
 * limits (NULL = none, the default options): request_count[c] = GetRequestCount() of context c when
 * the batch starts (n_ctx entries), hard limits as SiloMessagingOptions' MaxEnqueuedRequestsHardLimit
 * (_StatelessWorker); <= 0 = no limit.  Every enqueued message of an activation counts
 * (IncrementEnqueuedOnDispatcherCount), as when the agent thread enqueues the batch before a worker
 * runs any of it.  The limits apply whether or not perm / offsets are asked for.
 * Every context index gd_actdir_add stored for an entry the batch finds must be < n_ctx: a larger one
 * fails the call with GD_EINVAL (the *_device forms: the next gd_synchronize), the message left
 * un-enqueued with GD_RECV_UNDECODED. */
#define GD_RECV_ACTIVATION        0
#define GD_RECV_SYSTEM_TARGET     1
#define GD_RECV_NULL_CONTEXT      2
#define GD_RECV_REJECT_UNKNOWN    3
#define GD_RECV_REJECT_OVERLOADED 4
#define GD_RECV_DROPPED           5
#define GD_RECV_UNDECODED         6
typedef struct gd_recv_limits {
    const uint32_t* request_count;   /* [n_ctx]; device memory for the *_device entry points */
    int32_t hard_limit;
    int32_t hard_limit_stateless_worker;
} gd_recv_limits;
int gd_receive(gd_handle* h, const gd_key* target_grain, const gd_key* target_activation, const uint8_t* direction,
               uint32_t n, uint32_t n_ctx, const gd_recv_limits* limits, uint32_t* out_ctx, uint8_t* out_status,
               uint32_t* out_perm, uint32_t* out_offsets);
int gd_receive_device(gd_handle* h, const gd_key* d_target_grain, const gd_key* d_target_activation,
                      const uint8_t* d_direction, uint32_t n, uint32_t n_ctx, const gd_recv_limits* limits,
                      uint32_t* d_ctx, uint8_t* d_status, uint32_t* d_perm, uint32_t* d_offsets);
/* The same straight from the receive buffer (frames as gd_route_frames): decode -> ReceiveMessage ->
 * bucketing.  d_out may be NULL or name the decoded fields wanted. */
int gd_receive_frames_device(gd_handle* h, const uint8_t* d_buf, uint64_t buf_len, const uint64_t* d_frame_off,
                             uint32_t n, uint32_t n_ctx, const gd_recv_limits* limits, const gd_frame_fields* d_out,
                             uint32_t* d_ctx, uint8_t* d_status, uint32_t* d_perm, uint32_t* d_offsets);
int gd_receive_frames(gd_handle* h, const uint8_t* buf, uint64_t buf_len, const uint64_t* frame_off, uint32_t n,
                      uint32_t n_ctx, const gd_recv_limits* limits, const gd_frame_fields* out, uint32_t* out_ctx,
                      uint8_t* out_status, uint32_t* out_perm, uint32_t* out_offsets);

/* ---- per-kernel timing (cfg.flags & GD_CFG_KERNEL_TIMING) ----------------------- */
/* Up to max entries of {name, launches, total_ms} accumulated since the last reset. */
typedef struct gd_kernel_time {
    char     name[48];
    uint64_t launches;
    double   total_ms;
} gd_kernel_time;
int gd_kernel_times(gd_handle* h, gd_kernel_time* out, uint32_t max, uint32_t* out_n);
int gd_kernel_times_reset(gd_handle* h);
int gd_set_kernel_timing(gd_handle* h, int enable);   /* 0 off, 1 every launch, 2 stages only
                                                         ("stage:bucket": one event pair around each
                                                         bucketing, none between its kernels) */

/* ---- handle options (no reference counterpart: the reference has no device kernels) ------------
 * Round 4 replaces the library's GD_* environment switches: a host's behaviour no longer depends on
 * its environment, only on these calls.  Every option changes speed only, never results (the parity
 * tests run both sides of each one that changes a data layout); the defaults are the measured
 * winners.  Exchange options are per sender and may differ between ranks. */
#define GD_OPT_PROBE        1   /* route probe: 0 directory, 1 measured per launch kind (default),
                                   2 compact index in 64-B group reads, 3 compact index in 16-B slot reads,
                                   4 the 8-B index where the directory allows it (one type, N1 < 2^32,
                                   activation and silo numbers fitting a u32 together; else as 2) */
#define GD_OPT_BUCKET       2   /* bucketing: 0 LSD passes, 1 measured (default), 2 the two-level form
                                   wherever it applies (batches >= 2^20 messages, n_act < 2^28) */
#define GD_OPT_L2_SMALL     3   /* two-level three-pass form: ranges of at most this many messages are
                                   sorted one wave a range (default 1024) */
#define GD_OPT_STABLE_RANK  4   /* every bucketing form's in-wave rank: 1 ds_add_rtn, whose same-address
                                   lanes the hardware serves in lane order (default; gd_create checks that
                                   order on the device), 0 ballots -- stable by construction; a device
                                   failing the check gets 0 and refuses 1 */
#define GD_OPT_WIRE_HEADERS 5   /* exchange headers of one-type long-key batches: 0 24-B keys, 1 u64
                                   N1s, 2 u32 N1s when every N1 < 2^32 (default) */
#define GD_OPT_REGION_PROBE 6   /* exchange: (rank, region) partition + region-mapped owner probe: 0 (default) / 1 */
#define GD_OPT_IDX16        7   /* exchange at W > 1: 2-B origin indices on the wire: 1 (default) / 0 */
#define GD_OPT_HOST_CHUNK   8   /* host-pointer gd_route / gd_route_bucket: messages a pipelined chunk
                                   (default 2,097,152; 0 = one chunk, the serial copies) */
#define GD_OPT_MB_ZEROCOPY  9   /* micro-batches created after: I/O from / to pinned host memory: 1 (default)
                                   / 0 staged copies */
#define GD_OPT_MB_SPLIT     10  /* micro-batches created after: redundant sorters splitting the host stores (8) */
#define GD_OPT_MB_TRACE     11  /* micro-batches created after: per-phase timestamps printed at destroy (0) */
#define GD_OPT_L2_STAGED    12  /* two-level three-pass form: ranges of at most this many messages (and more
                                   than GD_OPT_L2_SMALL) sorted one workgroup a range, larger ones in 8K
                                   chunks over several workgroups (default 24,576, the staging capacity) */
#define GD_OPT_L2_MID       13  /* two-level three-pass form: ranges of at most this many messages (and more
                                   than GD_OPT_L2_SMALL) sorted by 512-thread workgroups, three a CU, the rest
                                   of the staged class by 1,024-thread ones (default 8,192, the 512-thread
                                   capacity; 0 = every staged range on the 1,024-thread sort) */
#define GD_OPT_B2_PERSIST   14  /* one-pass two-level form's MSD scatter: k = 1..8 persistent workgroups a
                                   CU, each loading its next tile under the current tile's write-out
                                   (default 2); 0 one workgroup a tile */
#define GD_OPT_B2_ORDER     15  /* that persistent scatter's tile order within its XCD's tile range: 0 strided
                                   (workgroup k takes tiles k, k + per, ...), 1 chunked (workgroup k takes a
                                   run of consecutive tiles, so one digit's runs of neighbouring tiles -- one
                                   128-B line between them -- leave one workgroup back to back; measured
                                   slower, profiles/r06_b2_order_ab.txt) */
#define GD_OPT_MB_POLL      16  /* micro-batches created after, zero-copy: a graph replay (gd_microbatch_run
                                   with use_graph) returns when the sort's workgroups have counted
                                   themselves done in pinned host memory (their stores fenced first)
                                   instead of waiting for the dispatch's completion signal; eager runs
                                   still synchronise the stream (measured faster): 1 (default) / 0 */
#define GD_OPT_FAN_BOUND    17  /* measurement: each fan-out route over the 8-B index is preceded by a launch
                                   of its memory traffic alone (k_fan_bound: the same expansion reads, one
                                   64-B index group read a message and the same result writes into scratch,
                                   no ring search, no walk), timed under its own name: 0 (default) / 1 */
int gd_option_set(gd_handle* h, int option, int64_t value);
int gd_option_get(const gd_handle* h, int option, int64_t* value);

/* ---- measured choices -------------------------------------------------------------------------
 * With GD_OPT_PROBE / GD_OPT_BUCKET at 1 the library times its interchangeable variants on the first
 * launches of each launch kind and size class (HIP events, read without a stream sync) and keeps the
 * fastest per message.  These calls let a host see, pin and share those choices, so that performance
 * is deterministic: pinned choices run from the first launch; gd_tune_agree makes every rank of the
 * communicator run the same variant. */
#define GD_TUNE_PROBE_KEYS   0  /* k_route over 24-B keys: 0 index groups, 1 directory, 2 index slots,
                                   3 the 8-B index (when the directory allows it) */
#define GD_TUNE_PROBE_N1     1  /* the exchange owner's probe over received N1s: same variants (0..3) */
#define GD_TUNE_PROBE_FANOUT 2  /* k_fan_route: 0 index groups, 1 directory, 2 the 8-B index */
#define GD_TUNE_PROBE_NODES  3  /* the sharded fan-out owner's probe: 0 index groups, 1 directory, 2 the 8-B index */
#define GD_TUNE_BUCKET       4  /* bucketing: 0 LSD passes, 1 the two-level form */
#define GD_TUNE_KINDS        5
int gd_tune_reset(gd_handle* h);                         /* forget every measured choice */
/* Pin kind's choice for every size (variant >= 0), or return it to measuring (-1). */
int gd_tune_set(gd_handle* h, int kind, int variant);
/* The choice a launch of kind over n messages (sub: the bucketing's messages-a-range class, else 0)
 * would take: the pinned or measured variant, or -1 while still measuring. */
int gd_tune_get(gd_handle* h, int kind, uint64_t n, uint32_t sub, int* variant);
/* Collective over the handle's communicator (gd_comm_init*): every rank contributes its finished
 * measurements (best time per message of each variant of each kind and size class) and every rank
 * keeps, per entry any rank finished, the variant with the least summed time -- the same pick on every
 * rank.  Entries no rank finished keep measuring. */
int gd_tune_agree(gd_handle* h);

/* The handle's communicator: its rank count and this handle's rank as the transport reports them
 * (RCCL: ncclCommCount / ncclCommUserRank), and the transport. */
#define GD_COMM_NONE  0
#define GD_COMM_RCCL  1   /* gd_comm_init */
#define GD_COMM_LOCAL 2   /* gd_comm_init_local (in-process device copies) */
int gd_comm_info(gd_handle* h, int* n_ranks, int* rank, int* transport);

/* ---- probe indexes (round 6) -------------------------------------------------------------------
 * The compact probe indexes mirror the directory table slot for slot.  AddSingleActivation /
 * AddActivation / RemoveActivation batches (gd_dir_register*, gd_dir_upsert, gd_dir_unregister) keep
 * them current by re-projecting the slots they touched -- the reference's O(1) dictionary updates
 * (GrainDirectoryPartition.cs:304-363) stay O(batch); other directory changes (rehash, clear, silo
 * removal, merge, split, handoff) leave them to a full rebuild (two streaming passes) at the next large
 * route.  Keys an index does not hold (N0 != 0, a grain class or N1 it does not cover) are probed in
 * the directory per message.  Read-only statistics: */
typedef struct gd_index_stats {
    uint64_t builds;          /* full builds since gd_create                                      */
    uint64_t synced_slots;    /* table slots re-projected by directory batches                    */
    double   last_build_ms;   /* host wall time of the last build (both passes, one read-back)    */
    uint32_t current;         /* 1: the indexes match the table now                               */
    uint32_t types8;          /* grain classes (TypeCodeData) the 8-B index holds                 */
    uint32_t act_bits8;       /* its activation and silo field widths                             */
    uint32_t silo_bits8;
    uint32_t n0_live;         /* at the last build: live entries with N0 != 0 (directory probe)    */
    uint32_t out8;            /* live entries projected since the build that the 8-B index does not
                                 hold or redirects to the directory (incl. the build's own)         */
} gd_index_stats;
int gd_index_stats_get(gd_handle* h, gd_index_stats* out);
/* Diagnostic (no reference counterpart; bench.py's roofline.route_bound): gd_route_device's memory
 * bound over the current 8-B index -- the route kernel's launch shape, key reads, one 64-B index group
 * read per message at the key's home and its silo / act / status writes, without the ring search,
 * the walk past the home group or the directory fallback.  The outputs are NOT route results.
 * GD_EINVAL when the directory has no 8-B index. */
int gd_route_bound_device(gd_handle* h, const gd_key* d_keys, uint32_t n, uint32_t* d_silo, uint32_t* d_act,
                          uint8_t* d_status);

#ifdef __cplusplus
}
#endif
#endif /* GRAINDISPATCH_H */
