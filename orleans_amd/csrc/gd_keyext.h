// gd_keyext.h -- gfx950 device code for KeyExt grains (string keys, compound keys, geo clients;
// SURVEY 8 a1/a2).
//
// UniqueKey.GetUniformHashCode of a HasKeyExt key with KeyExt != null is
// JenkinsHash.ComputeHash(byte[]) over ToByteArray() = N0 | N1 | TCD | int32 UTF-8 length |
// UTF-8 (UniqueKey.cs:272-336, JenkinsHash.cs:25-74).  jenkins_keyext walks that byte stream as
// little-endian words without building it: words 0..6 come from the key and the length, words
// 7.. from the string, zero past its end -- which is also exactly the byte variant's tail rule
// (the tail bytes go to a, b and c << 8, the rest is zero).
//
// KeyExt grains live in their own open-addressing table of 64-B KxSlots (one DRAM atom per
// probe) plus a byte heap holding the KeyExt strings.  Equality = the three words, the length,
// the uniform hash (a cheap filter) and the bytes (UniqueKey.Equals, UniqueKey.cs:245-251).
//
// k_route_keyext runs after the route kernel over the messages it left at GD_ROUTE_KEYEXT, so
// the 24-B-key hot path is untouched by the variable-length work.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gd_common.h"
#include "gd_kernels.h"

namespace gd {

struct KxArgs {
    const KxSlot* slots;
    unsigned long long mask;
    uint32_t max_probe;
    const uint8_t* heap;
    const uint32_t* valid;     // IsValidSilo bitset (TableArgs::valid), n_valid 0 = all valid
    uint32_t n_valid;
};

struct ExtArgs {
    const uint8_t* bytes;
    const uint64_t* off;
    const int32_t* len;
    uint64_t bytes_len;
};

// Little-endian word q of the string (bytes 4q .. 4q+3), zero past `len`.
__device__ __forceinline__ uint32_t str_word(const uint8_t* s, int32_t len, uint32_t q) {
    uint32_t w = 0;
#pragma unroll
    for (uint32_t b = 0; b < 4; ++b) {
        const uint32_t i = 4 * q + b;
        if ((int32_t)i < len) w |= (uint32_t)s[i] << (8 * b);
    }
    return w;
}

__device__ __forceinline__ uint32_t keyext_word(uint64_t n0, uint64_t n1, uint64_t tcd, const uint8_t* s,
                                                int32_t len, uint32_t k) {
    switch (k) {
        case 0: return (uint32_t)n0;
        case 1: return (uint32_t)(n0 >> 32);
        case 2: return (uint32_t)n1;
        case 3: return (uint32_t)(n1 >> 32);
        case 4: return (uint32_t)tcd;
        case 5: return (uint32_t)(tcd >> 32);
        case 6: return (uint32_t)len;
        default: return str_word(s, len, k - 7);
    }
}

// JenkinsHash.ComputeHash(ToByteArray()) for len >= 0 (JenkinsHash.cs:25-74).
__device__ __forceinline__ uint32_t jenkins_keyext(uint64_t n0, uint64_t n1, uint64_t tcd, const uint8_t* s,
                                                   int32_t len) {
    const uint32_t L = 28u + (uint32_t)len;
    uint32_t a = 0x9e3779b9u, b = a, c = 0;
    const uint32_t nb = L / 12u;
    for (uint32_t j = 0; j < nb; ++j) {
        a += keyext_word(n0, n1, tcd, s, len, 3 * j);
        b += keyext_word(n0, n1, tcd, s, len, 3 * j + 1);
        c += keyext_word(n0, n1, tcd, s, len, 3 * j + 2);
        jmix(a, b, c);
    }
    c += L;
    a += keyext_word(n0, n1, tcd, s, len, 3 * nb);
    b += keyext_word(n0, n1, tcd, s, len, 3 * nb + 1);
    c += keyext_word(n0, n1, tcd, s, len, 3 * nb + 2) << 8;
    jmix(a, b, c);
    return c;
}

__device__ __forceinline__ bool bytes_equal(const uint8_t* x, const uint8_t* y, int32_t len) {
    for (int32_t i = 0; i < len; ++i)
        if (x[i] != y[i]) return false;
    return true;
}

// ---- register fast path: KeyExt strings up to KX_FAST_BYTES ---------------------------------
// The string is fetched as the aligned dwords covering it (clamped indices: every load is issued,
// none past the string's last dword) and shifted into place with v_alignbyte; bytes past `len` are
// zero.  The Jenkins blocks then run fully unrolled over registers (at most 92 stream bytes = 8
// blocks incl. the tail), and the heap copy (16-B aligned by the host) is compared word by word.
constexpr int KX_FAST_WORDS = 16;
constexpr int KX_FAST_BYTES = 4 * KX_FAST_WORDS;

__device__ __forceinline__ void load_str_fast(const uint8_t* s, int32_t len, uint32_t (&w)[KX_FAST_WORDS]) {
    if (len <= 0) {                                      // nothing to read (s may be one past the end)
#pragma unroll
        for (int q = 0; q < KX_FAST_WORDS; ++q) w[q] = 0;
        return;
    }
    const uintptr_t a = reinterpret_cast<uintptr_t>(s);
    const uint32_t* base = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const int32_t nd = (int32_t)((sh + (uint32_t)len + 3) >> 2);   // dwords holding the string
    uint32_t d[KX_FAST_WORDS + 1];
#pragma unroll
    for (int j = 0; j <= KX_FAST_WORDS; ++j) d[j] = base[min(j, nd - 1)];
#pragma unroll
    for (int q = 0; q < KX_FAST_WORDS; ++q) {
        const uint32_t v = __builtin_amdgcn_alignbyte(d[q + 1], d[q], sh);
        const int32_t left = len - 4 * q;                 // valid bytes in word q
        w[q] = left >= 4 ? v : (left <= 0 ? 0u : (v & ((1u << (8 * left)) - 1u)));
    }
}

__device__ __forceinline__ uint32_t jenkins_keyext_fast(uint64_t n0, uint64_t n1, uint64_t tcd, int32_t len,
                                                        const uint32_t (&w)[KX_FAST_WORDS]) {
    uint32_t W[24];
    W[0] = (uint32_t)n0;
    W[1] = (uint32_t)(n0 >> 32);
    W[2] = (uint32_t)n1;
    W[3] = (uint32_t)(n1 >> 32);
    W[4] = (uint32_t)tcd;
    W[5] = (uint32_t)(tcd >> 32);
    W[6] = (uint32_t)len;
#pragma unroll
    for (int q = 0; q < KX_FAST_WORDS; ++q) W[7 + q] = w[q];
    W[23] = 0;
    const uint32_t L = 28u + (uint32_t)len;
    const uint32_t nb = L / 12u;
    uint32_t a = 0x9e3779b9u, b = a, c = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        if (j < nb) {
            a += W[3 * j];
            b += W[3 * j + 1];
            c += W[3 * j + 2];
            jmix(a, b, c);
        } else if (j == nb) {                               // the byte variant's tail (JenkinsHash.cs:51-73)
            c += L;
            a += W[3 * j];
            b += W[3 * j + 1];
            c += W[3 * j + 2] << 8;
            jmix(a, b, c);
        }
    }
    return c;
}

__device__ __forceinline__ bool heap_equal_fast(const uint8_t* heap, uint64_t off, int32_t len,
                                                const uint32_t (&w)[KX_FAST_WORDS]) {
    const uint32_t* hp = reinterpret_cast<const uint32_t*>(heap + off);   // 16-B aligned by the host
    const int32_t nw = (len + 3) >> 2;
    bool eq = true;
#pragma unroll
    for (int q = 0; q < KX_FAST_WORDS; ++q) {
        if (q < nw) {
            const int32_t left = len - 4 * q;
            const uint32_t m = left >= 4 ? 0xFFFFFFFFu : ((1u << (8 * left)) - 1u);
            eq = eq && ((hp[q] & m) == w[q]);
        }
    }
    return eq;
}

// Live KeyExt entry equal to (n0, n1, tcd, s[0..len)) -- len = GD_KEYEXT_NULL for a null KeyExt.
// FAST: the string is in w[] (len <= KX_FAST_BYTES).  The slot is read as four 16-B loads (one
// 64-B atom); strings of at most KX_INLINE bytes are compared in the slot, longer ones in the heap.
template <bool FAST>
__device__ __forceinline__ bool kx_find(const KxArgs& t, uint64_t n0, uint64_t n1, uint64_t tcd, const uint8_t* s,
                                        int32_t len, uint32_t uh, const uint32_t (&w)[KX_FAST_WORDS], uint32_t& act,
                                        uint32_t& meta) {
    unsigned long long i = fmix32(uh) & t.mask;
    for (uint32_t p = 0; p <= t.max_probe; ++p) {
        const uint4* qp = reinterpret_cast<const uint4*>(t.slots + i);
        const uint4 q0 = qp[0], q1 = qp[1], q2 = qp[2], q3 = qp[3];
        const uint32_t m = q2.w;
        const uint32_t st = slot_state(m);
        if (st == SLOT_EMPTY) return false;
        const uint64_t k0 = (uint64_t)q0.x | ((uint64_t)q0.y << 32);
        const uint64_t k1 = (uint64_t)q0.z | ((uint64_t)q0.w << 32);
        const uint64_t k2 = (uint64_t)q1.x | ((uint64_t)q1.y << 32);
        const uint64_t off = (uint64_t)q1.z | ((uint64_t)q1.w << 32);
        if (st == SLOT_LIVE && q2.y == uh && (int32_t)q2.x == len && k0 == n0 && k1 == n1 && k2 == tcd) {
            bool eq = true;
            if (len > 0 && len <= KX_INLINE) {              // inline: compare against the slot itself
                if constexpr (FAST) {
                    const uint32_t iw[6] = {q1.z, q1.w, q3.x, q3.y, q3.z, q3.w};
#pragma unroll
                    for (int k = 0; k < 6; ++k) eq = eq && (iw[k] == w[k]);   // zero past len on both sides
                } else {
                    const uint32_t iw[6] = {q1.z, q1.w, q3.x, q3.y, q3.z, q3.w};
                    for (int32_t k = 0; k < len; ++k)
                        eq = eq && (((iw[k >> 2] >> (8 * (k & 3))) & 0xFFu) == s[k]);
                }
            } else if (len > 0) {
                if constexpr (FAST) eq = heap_equal_fast(t.heap, off, len, w);
                else eq = bytes_equal(t.heap + off, s, len);
            }
            if (eq) {
                act = q2.z;
                meta = m;
                return true;
            }
        }
        i = (i + 1) & t.mask;
    }
    return false;
}

// Uniform hash + lookup of one KeyExt message; FAST path for strings that fit the registers.
__device__ __forceinline__ uint32_t kx_hash_and_find(const KxArgs& t, uint64_t n0, uint64_t n1, uint64_t tcd,
                                                     const uint8_t* s, int32_t len, bool& found, uint32_t& act,
                                                     uint32_t& meta) {
    uint32_t w[KX_FAST_WORDS];
    uint32_t uh;
    found = false;
    if (len <= KX_FAST_BYTES) {
        if (len >= 0) {
            load_str_fast(s, len, w);
            uh = jenkins_keyext_fast(n0, n1, tcd, len, w);
        } else {
#pragma unroll
            for (int q = 0; q < KX_FAST_WORDS; ++q) w[q] = 0;
            uh = uniform_hash(n0, n1, tcd);
        }
        if (t.slots) found = kx_find<true>(t, n0, n1, tcd, s, len, uh, w, act, meta);
    } else {
        uh = jenkins_keyext(n0, n1, tcd, s, len);
        if (t.slots) found = kx_find<false>(t, n0, n1, tcd, s, len, uh, w, act, meta);
    }
    return uh;
}

// Message i's KeyExt: false when the host keeps it (GD_KEYEXT_HOST, or a range outside bytes).
__device__ __forceinline__ bool ext_of(const ExtArgs& e, uint32_t i, const uint8_t*& s, int32_t& len) {
    len = e.len[i];
    if (len == GD_KEYEXT_NULL) {
        s = nullptr;
        return true;
    }
    if (len < 0) return false;
    const uint64_t off = e.off[i];
    if (off > e.bytes_len || (uint64_t)len > e.bytes_len - off) return false;
    s = e.bytes + off;
    return true;
}

// The messages k_route left at GD_ROUTE_KEYEXT: owner by the KeyExt hash
// (CalculateTargetSilo, LocalGrainDirectory.cs:477-545), then the KeyExt table.
template <int MODE>
static __global__ void __launch_bounds__(BLOCK) k_route_keyext(const gd_key* __restrict__ keys, uint32_t n, ExtArgs ext,
                                                        RingArgs ring, KxArgs tab, uint32_t* __restrict__ out_silo,
                                                        uint32_t* __restrict__ out_act,
                                                        uint8_t* __restrict__ out_status) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_ring[];
    uint32_t* s_pts = s_ring;
    uint32_t* s_own = s_ring + ring.n;
    stage_ring(ring, s_pts, s_own);
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n || out_status[i] != GD_ROUTE_KEYEXT) return;
    const uint8_t* s;
    int32_t len;
    if (!ext_of(ext, i, s, len)) return;
    const uint64_t* kp = reinterpret_cast<const uint64_t*>(keys + i);
    const uint64_t n0 = kp[0], n1 = kp[1], tcd = kp[2];
    uint32_t act = NONE32, meta = 0;
    bool found;
    const uint32_t uh = kx_hash_and_find(tab, n0, n1, tcd, s, len, found, act, meta);
    const uint32_t owner = s_own[ring_position<MODE>(s_pts, ring.n, ring.top, uh)];
    if (found && valid_silo(tab.valid, tab.n_valid, slot_silo(meta))) {   // IsValidSilo filter (:431)
        out_silo[i] = slot_silo(meta);                 // ActivationAddress.Silo (Message.cs:629-639)
        out_act[i] = act;
        out_status[i] = GD_ROUTE_OK;
    } else {
        out_silo[i] = owner;
        out_act[i] = NONE32;
        out_status[i] = GD_ROUTE_MISS;                 // Dispatcher.cs:742 slow path
    }
}

// LookUpActivations for KeyExt keys (no ring needed).  found: 1 hit, 0 miss, 2 not a KeyExt
// lookup the device can answer (GD_KEYEXT_HOST / bad range).
static __global__ void __launch_bounds__(BLOCK) k_kx_lookup(const gd_key* __restrict__ keys, uint32_t n, ExtArgs ext,
                                                     KxArgs tab, gd_val* __restrict__ out_vals,
                                                     uint8_t* __restrict__ out_found) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint8_t* s;
    int32_t len;
    gd_val v{NONE32, NONE32};
    uint8_t f = 2;
    if (ext_of(ext, i, s, len)) {
        const uint64_t* kp = reinterpret_cast<const uint64_t*>(keys + i);
        const uint64_t n0 = kp[0], n1 = kp[1], tcd = kp[2];
        uint32_t act = NONE32, meta = 0;
        bool found;
        (void)kx_hash_and_find(tab, n0, n1, tcd, s, len, found, act, meta);
        f = 0;
        if (found) {
            v.act = act;
            v.silo = slot_silo(meta);
            f = 1;
        }
    }
    out_vals[i] = v;
    out_found[i] = f;
}

// Uniform hashes of KeyExt keys on the device (the host index checks its own against these in
// the parity tests): GD_KEYEXT_NULL -> three-word hash.
static __global__ void __launch_bounds__(BLOCK) k_kx_hash(const gd_key* __restrict__ keys, uint32_t n, ExtArgs ext,
                                                   uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint8_t* s;
    int32_t len;
    const uint64_t* kp = reinterpret_cast<const uint64_t*>(keys + i);
    if (!ext_of(ext, i, s, len)) {
        out[i] = 0;
        return;
    }
    if (len < 0) {
        out[i] = uniform_hash(kp[0], kp[1], kp[2]);
    } else if (len <= KX_FAST_BYTES) {               // the path k_route_keyext takes
        uint32_t w[KX_FAST_WORDS];
        load_str_fast(s, len, w);
        out[i] = jenkins_keyext_fast(kp[0], kp[1], kp[2], len, w);
    } else {
        out[i] = jenkins_keyext(kp[0], kp[1], kp[2], s, len);
    }
}

// Apply host-index changes: slots[idx[j]] = val[j].
static __global__ void __launch_bounds__(BLOCK) k_kx_apply(const uint64_t* __restrict__ idx, const KxSlot* __restrict__ val,
                                                    uint32_t m, KxSlot* __restrict__ slots) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j < m) slots[idx[j]] = val[j];
}

}  // namespace gd
