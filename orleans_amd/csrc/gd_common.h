// gd_common.h -- definitions shared by the host identity code and the gfx950
// kernels of libgraindispatch.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>

#include "graindispatch.h"

#if defined(__HIPCC__)
#define GD_HD __host__ __device__ __forceinline__
#else
#define GD_HD inline
#endif

namespace gd {

// ---- L0 identity (host), gd_identity.cpp --------------------------------------------
uint32_t jenkins_bytes(const uint8_t* data, size_t len);
uint32_t jenkins_u64x3(uint64_t u1, uint64_t u2, uint64_t u3);
void sha256(const uint8_t* data, size_t len, uint8_t out[32]);
int32_t calculate_id_hash(const char* utf8);
std::string endpoint_string(const gd_silo_addr& s);
int32_t silo_consistent_hash(const gd_silo_addr& s);
void silo_uniform_hashes(const gd_silo_addr& s, uint32_t n, uint32_t* out);
int silo_compare(const gd_silo_addr& a, const gd_silo_addr& b);

// ---- UniqueKey categories (UniqueKey.cs:17-26) ---------------------------------------
constexpr uint32_t CAT_SYSTEM_TARGET = 1;
constexpr uint32_t CAT_SYSTEM_GRAIN = 2;
constexpr uint32_t CAT_GRAIN = 3;
constexpr uint32_t CAT_KEYEXT_GRAIN = 6;
constexpr uint32_t CAT_GEO_CLIENT = 7;
// Categories whose keys carry a KeyExt (UniqueKey.HasKeyExt, Orleans.Core.Abstractions/IDs/UniqueKey.cs:61-68).
GD_HD bool is_keyext_tcd(uint64_t tcd) {
    const uint32_t c = (uint32_t)(tcd >> 56);
    return c == CAT_KEYEXT_GRAIN || c == CAT_GEO_CLIENT;
}

// Constants.SystemMembershipTableId (src/Orleans.Core/Runtime/Constants.cs:52):
// SystemGrain key of Guid 01145FEC-C21E-11E0-9105-D0FB4724019B in Guid.ToByteArray
// order (bytes EC 5F 14 01 1E C2 E0 11 | 91 05 D0 FB 47 24 01 9B, little-endian
// u64 words).  Cross-checked against the oracle in the GPU parity tests.
constexpr uint64_t MEMBERSHIP_N0 = 0x11E0C21E01145FECull;
constexpr uint64_t MEMBERSHIP_N1 = 0x9B012447FBD00591ull;
constexpr uint64_t MEMBERSHIP_TCD = (uint64_t)CAT_SYSTEM_GRAIN << 56;

// ---- directory slot layout in HBM ---------------------------------------------------
// 32 B slot, 4 per 128-B line: the 24-B GrainId key, the activation index and a
// meta word {silo:16 | state:16}.  The state lives in the word the CAS claims.
enum SlotState : uint32_t {
    SLOT_EMPTY = 0,
    SLOT_LIVE = 1,
    SLOT_TOMB = 2,
    SLOT_CLAIMED = 3,   // transient inside the register kernel
    SLOT_PENDING = 4,   // created by the current register batch, winner not yet chosen
};

struct alignas(32) Slot {
    uint64_t n0;
    uint64_t n1;
    uint64_t tcd;
    uint32_t act;
    uint32_t meta;  // (state << 16) | silo
};
static_assert(sizeof(Slot) == 32, "slot must be 32 bytes");

// KeyExt grain slot (gd_keyext.h): one 64-B DRAM atom -- the three words, the KeyExt string
// (inline when it has at most KX_INLINE bytes: bytes 0..7 in `off`, 8..23 in `tail`; else its
// place in the KeyExt heap), its uniform hash (compared before the bytes) and the value.
constexpr int32_t KX_INLINE = 24;
struct alignas(64) KxSlot {
    uint64_t n0;
    uint64_t n1;
    uint64_t tcd;
    uint64_t off;       // heap offset of the UTF-8 KeyExt, or its first 8 bytes (inline)
    int32_t len;        // UTF-8 length, GD_KEYEXT_NULL = null KeyExt
    uint32_t uhash;     // UniqueKey.GetUniformHashCode
    uint32_t act;
    uint32_t meta;      // (state << 16) | silo
    uint64_t tail[2];   // inline string bytes 8..23
};
inline void kx_inline_put(KxSlot& q, const uint8_t* s, int32_t len) {
    uint8_t b[KX_INLINE] = {0};
    for (int32_t i = 0; i < len; ++i) b[i] = s[i];
    __builtin_memcpy(&q.off, b, 8);
    __builtin_memcpy(q.tail, b + 8, 16);
}
inline bool kx_inline_eq(const KxSlot& q, const uint8_t* s, int32_t len) {
    uint8_t b[KX_INLINE];
    __builtin_memcpy(b, &q.off, 8);
    __builtin_memcpy(b + 8, q.tail, 16);
    for (int32_t i = 0; i < len; ++i)
        if (b[i] != s[i]) return false;
    return true;
}
static_assert(sizeof(KxSlot) == 64, "KeyExt slot must be 64 bytes");

GD_HD uint32_t slot_state(uint32_t meta) { return meta >> 16; }
GD_HD uint32_t slot_silo(uint32_t meta) { return meta & 0xFFFFu; }
GD_HD uint32_t make_meta(uint32_t state, uint32_t silo) { return (state << 16) | (silo & 0xFFFFu); }

// Home slot: murmur3 fmix32 of the uniform hash, so that a shard holding one
// contiguous ring range still spreads over the whole table.
GD_HD uint32_t fmix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu;
    h ^= h >> 13; h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

// Home slot of a grain in a directory table of mask + 1 slots (a power of two, at most 2^32): the
// TOP bits of fmix32(uniform hash) (multiply-shift), so that the table's eighths hold the grains of
// region fmix32(h) >> 29 whatever its size -- the region the exchange groups messages by, and the
// owner's probe workgroups are mapped by (one region per XCD, its L2 serving one eighth of the table).
// The home slot is the first of an aligned group of SLOT_GROUP slots (2 x 32 B = one 64-B DRAM
// atom): linear probing from the group start, so the lookup (route_m_core) reads a whole group per
// round trip.  At load 0.5 a 64-lane wave waits on the longest chain of its lanes: ~7.7 dependent
// rounds with one slot a round, ~4.1 with two (tools/sim_probe_rounds.py).  Measured on cfg 2:
// k_route 0.385 (1 slot) / 0.366 (2) / 0.382 (4) / 0.675 ms (8).  But on cfg 3 (Zipf(1.1)
// over 100M grains) the 64-B reads double the hot set's cache traffic: k_route 1.24 (1 slot) vs
// 2.25 ms (2) (profiles/r03_cfg3_group_ab.txt).  Uniform batches take the compact probe index
// (gd_cx.h) instead, so the directory keeps one slot a round.
#ifndef GD_SLOT_GROUP
#define GD_SLOT_GROUP 1
#endif
constexpr uint32_t SLOT_GROUP = GD_SLOT_GROUP;
static_assert((SLOT_GROUP & (SLOT_GROUP - 1)) == 0 && SLOT_GROUP <= 1024, "slot group: a power of two <= 1024");
// Homes are aligned to HOME_ALIGN slots (round 6): the compact probe indexes mirror the table slot for
// slot (gd_cx.h), and an 8-B index reads 8 slots (one 64-B atom) a round, so a home at the start of its
// atom lets the first read cover the 8 slots a grain can first sit in -- the layout the round-4/5 index
// had when it was placed by CAS (exact homes in the mirror: cfg 2 k_route 0.285 -> 0.397 ms, most waves
// waiting for a second read).  The directory's own probe still reads SLOT_GROUP slots a round.
constexpr uint32_t HOME_ALIGN = SLOT_GROUP > 8 ? SLOT_GROUP : 8;
GD_HD unsigned long long home_slot(uint32_t h, unsigned long long mask) {
    return (((unsigned long long)fmix32(h) * (mask + 1ull)) >> 32) & ~(unsigned long long)(HOME_ALIGN - 1);
}
constexpr uint32_t N_REGIONS = 8;
GD_HD uint32_t grain_region(uint32_t h) { return fmix32(h) >> 29; }

}  // namespace gd
