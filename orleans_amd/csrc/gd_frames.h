// gd_frames.h -- gfx950 device code for SURVEY 8 f1: batched decode of Orleans message
// frames straight from the receive buffer.
//
// Frame  = [int32 headerLength][int32 bodyLength][header][body]   (Message.cs:481-516)
// Header = int32 mask (HeadersContainer.Headers, Message.cs:728-765) followed by the present
//          fields in HeadersContainer.Serializer order (Message.cs:1126-1245); encodings from
//          BinaryTokenStreamWriter.cs:22-57 (CorrelationId, UniqueKey), :280-293 (string),
//          :485-513 (SiloAddress).  Oracle: oracle/headers.py decode_frame.
//
// One lane per frame.  Each wave first stages a FRAME_WIN-byte window of each of its 64 frames
// into LDS (12 independent 16-B loads per lane cover the wave's 64 windows), then
// every lane walks its own frame's mask-driven layout out of LDS.  Reads past the window (long
// strings) fall back to byte loads from global memory for that lane only.  HBM-bound byte
// work: no MFMA.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gd_common.h"
#include "gd_kernels.h"

namespace gd {

constexpr int FRAME_WIN = 192;                    // staged bytes per frame (typical headers < 140 B)
constexpr int FRAME_WIN_DW = FRAME_WIN / 4;
constexpr int FRAME_ROW = FRAME_WIN_DW + 1;       // +1 dword: alignbyte reads row[w + 1]

// HeadersContainer.Headers bits read here (Message.cs:728-765)
enum : uint32_t {
    H_ALWAYS_INTERLEAVE = 1u << 0, H_CACHE_INVALIDATION = 1u << 1, H_CATEGORY = 1u << 2,
    H_CORRELATION_ID = 1u << 3, H_DEBUG_CONTEXT = 1u << 4, H_DIRECTION = 1u << 5, H_TIME_TO_LIVE = 1u << 6,
    H_FORWARD_COUNT = 1u << 7, H_NEW_GRAIN_TYPE = 1u << 8, H_GENERIC_GRAIN_TYPE = 1u << 9, H_RESULT = 1u << 10,
    H_REJECTION_INFO = 1u << 11, H_REJECTION_TYPE = 1u << 12, H_READ_ONLY = 1u << 13, H_RESEND_COUNT = 1u << 14,
    H_SENDING_ACTIVATION = 1u << 15, H_SENDING_GRAIN = 1u << 16, H_SENDING_SILO = 1u << 17,
    H_IS_NEW_PLACEMENT = 1u << 18, H_TARGET_ACTIVATION = 1u << 19, H_TARGET_GRAIN = 1u << 20,
    H_TARGET_SILO = 1u << 21, H_TARGET_OBSERVER = 1u << 22, H_IS_UNORDERED = 1u << 23, H_REQUEST_CONTEXT = 1u << 24,
};

// frame flags (GD_FRAME_* in include/graindispatch.h)
enum : uint32_t { FR_HAS_TARGET = 1u, FR_COMPLETE = 2u, FR_FALLBACK = 4u, FR_MALFORMED = 8u, FR_TARGET_KEYEXT = 16u };

// route statuses added for frames (GD_ROUTE_ADDRESSED / GD_ROUTE_UNDECODED)
constexpr uint8_t ROUTE_ADDRESSED = 5, ROUTE_UNDECODED = 6;

struct FrameFields {   // device pointers; nullptr = field not wanted (flags and target_grain required)
    uint32_t* flags;
    uint64_t* target_grain;        // 3 x u64 per frame (gd_key)
    uint32_t* mask;
    uint64_t* target_activation;
    uint64_t* sending_activation;
    uint64_t* sending_grain;
    uint32_t* target_silo;         // 6 x u32 per frame (24-B wire SiloAddress)
    uint32_t* sending_silo;
    int64_t* correlation_id;
    uint8_t* category;
    uint8_t* direction;
    uint64_t* tg_ext_off;          // TargetGrain's KeyExt: absolute offset in buf (KeyExt routing)
    int32_t* tg_ext_len;           //   and UTF-8 length (-1 null, GD_KEYEXT_HOST: no target decoded)
};

// Byte cursor over one frame: LDS window first, global memory past it.
struct FrameCursor {
    const uint32_t* row;   // LDS row of this frame (dword aligned at frame_start & ~3)
    const uint8_t* g;      // frame start in global memory
    uint32_t sh;           // frame_start & 3
    uint32_t lim;          // bytes from frame start readable from the window

    __device__ __forceinline__ uint32_t u8(uint32_t pos) const {
        if (pos < lim) {
            const uint32_t p = pos + sh;
            return (row[p >> 2] >> ((p & 3) * 8)) & 0xFFu;
        }
        return g[pos];
    }
    __device__ __forceinline__ uint32_t u32(uint32_t pos) const {
        if (pos + 4 <= lim) {
            const uint32_t p = pos + sh;
            return __builtin_amdgcn_alignbyte(row[(p >> 2) + 1], row[p >> 2], p & 3);
        }
        return (uint32_t)g[pos] | ((uint32_t)g[pos + 1] << 8) | ((uint32_t)g[pos + 2] << 16) |
               ((uint32_t)g[pos + 3] << 24);
    }
    __device__ __forceinline__ uint64_t u64(uint32_t pos) const {
        return (uint64_t)u32(pos) | ((uint64_t)u32(pos + 4) << 32);
    }
};

struct Key3 {
    uint64_t n0, n1, tcd;
};

// Walker state: p = next byte (relative to frame start), end = header end.  Any read past end
// sets bad; later reads are then don't-care (the caller discards the frame).
struct HeaderWalk {
    FrameCursor c;
    uint32_t p, end;
    bool bad;

    __device__ __forceinline__ bool take(uint32_t k) {
        if ((uint64_t)p + k > end) {
            bad = true;
            return false;
        }
        p += k;
        return true;
    }
    // BinaryTokenStreamReader.ReadString: int32 UTF-8 length (-1 = null) + bytes.  Returns length.
    __device__ __forceinline__ int32_t skip_string() {
        if (bad || !take(4)) return -1;
        const int32_t ln = (int32_t)c.u32(p - 4);
        if (ln < -1) {
            bad = true;
            return -1;
        }
        if (ln > 0) take((uint32_t)ln);
        return ln;
    }
    // ReadUniqueKey (BinaryTokenStreamReader.cs:36-43): N0, N1, TypeCodeData, KeyExt.
    __device__ __forceinline__ Key3 key(int32_t* ext_len) {
        Key3 k{0, 0, 0};
        if (bad || !take(24)) return k;
        k.n0 = c.u64(p - 24);
        k.n1 = c.u64(p - 16);
        k.tcd = c.u64(p - 8);
        const int32_t e = skip_string();
        if (ext_len) *ext_len = e;
        return k;
    }
};

__device__ __forceinline__ void store_key(uint64_t* out, uint32_t i, const Key3& k) {
    if (!out) return;
    out[3ull * i] = k.n0;
    out[3ull * i + 1] = k.n1;
    out[3ull * i + 2] = k.tcd;
}

__device__ __forceinline__ void store_silo(uint32_t* out, uint32_t i, const uint32_t (&s)[6]) {
    if (!out) return;
#pragma unroll
    for (int j = 0; j < 6; ++j) out[6ull * i + j] = s[j];
}

static __global__ __launch_bounds__(BLOCK) void k_decode_frames(const uint8_t* __restrict__ buf, uint64_t buf_len,
                                                         const uint64_t* __restrict__ frame_off, uint32_t n,
                                                         FrameFields o) {
    __shared__ uint32_t s_win[BLOCK / WAVE][WAVE][FRAME_ROW];
    const uint32_t lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
    const uint32_t base = blockIdx.x * BLOCK + w * WAVE;
    const uint32_t i = base + lane;
    const bool valid = i < n;
    const uint64_t start = frame_off[valid ? i : (n - 1)];   // clamped, branch-free load

    // ---- stage: frame f's window = dwords [start_f & ~3, +FRAME_WIN) clamped into the buffer
    const uint64_t dw_end = buf_len & ~3ull;                  // [0, dw_end) readable as dwords
    // The wave's 64 windows are 64 x 12 chunks of 16 B: chunk q = it * 64 + lane belongs to frame
    // q / 12.  Every lane issues its 12 loads back to back (one memory round trip per wave);
    // a chunk that would cross dw_end is clamped to the last whole 16 B below it (its bytes are
    // then wrong, but lim keeps the walk from using bytes at or past dw_end).
    constexpr int CHUNKS = FRAME_WIN / 16;
    __shared__ unsigned long long s_start[BLOCK / WAVE][WAVE];
    s_start[w][lane] = start;
    __syncthreads();
    if (dw_end >= 16) {
        uint4 v[CHUNKS];
#pragma unroll
        for (int it = 0; it < CHUNKS; ++it) {
            const uint32_t q = it * WAVE + lane, f = q / CHUNKS, c = q % CHUNKS;
            const uint64_t a = (s_start[w][f] & ~3ull) + 16ull * c;
            v[it] = *(const uint4*)(buf + (a <= dw_end - 16 ? a : ((dw_end - 16) & ~3ull)));
        }
#pragma unroll
        for (int it = 0; it < CHUNKS; ++it) {
            const uint32_t q = it * WAVE + lane, f = q / CHUNKS, c = q % CHUNKS;
            uint32_t* r = &s_win[w][f][4 * c];
            r[0] = v[it].x;
            r[1] = v[it].y;
            r[2] = v[it].z;
            r[3] = v[it].w;
        }
    }
    __syncthreads();
    if (!valid) return;

    // ---- walk (HeadersContainer.Deserializer order, Message.cs:1247-1356)
    uint32_t flags = 0, mask = 0, cat = 0, dir = 0xFFu;
    int64_t corr = 0;
    Key3 tg{0, 0, 0}, ta{0, 0, 0}, sa{0, 0, 0}, sg{0, 0, 0};
    int32_t tg_ext = GD_KEYEXT_HOST;
    uint64_t tg_ext_off = 0;
    uint32_t ts[6] = {0, 0, 0, 0, 0, 0}, ss[6] = {0, 0, 0, 0, 0, 0};

    const uint64_t a0 = start & ~3ull;
    // staged bytes = the whole 16-B chunks of the window that lie below dw_end
    uint64_t win_end = a0;
    if (dw_end >= 16 && dw_end > a0) {
        const uint64_t full = (dw_end - a0) / 16;
        win_end = a0 + 16 * (full < (uint64_t)CHUNKS ? full : (uint64_t)CHUNKS);
    }
    HeaderWalk hw;
    hw.c.row = s_win[w][lane];
    hw.c.g = buf + start;
    hw.c.sh = (uint32_t)(start & 3);
    hw.c.lim = (start < win_end) ? (uint32_t)(win_end - start) : 0u;
    hw.bad = false;

    bool malformed = start > buf_len || buf_len - start < 8;
    int32_t hl = 0, bl = 0;
    if (!malformed) {
        hl = (int32_t)hw.c.u32(0);
        bl = (int32_t)hw.c.u32(4);
        malformed = hl < 4 || bl < 0 || (uint64_t)hl + (uint64_t)bl > buf_len - start - 8;
    }
    if (!malformed) {
        hw.p = 12;
        hw.end = 8u + (uint32_t)hl;
        mask = hw.c.u32(8);
        const uint32_t m = mask;
        const uint32_t full = H_TARGET_ACTIVATION | H_TARGET_SILO | H_TARGET_GRAIN;
        if ((m & full) == full) flags |= FR_COMPLETE;
        if (m & (H_CACHE_INVALIDATION | H_REQUEST_CONTEXT)) {
            flags |= FR_FALLBACK;          // object-serialized field before TargetGrain: nothing decoded
        } else {
            if ((m & H_CATEGORY) && hw.take(1)) cat = hw.c.u8(hw.p - 1);
            if (m & H_DEBUG_CONTEXT) hw.skip_string();
            if ((m & H_DIRECTION) && !hw.bad && hw.take(1)) dir = hw.c.u8(hw.p - 1);
            if (m & H_TIME_TO_LIVE) hw.take(8);
            if (m & H_FORWARD_COUNT) hw.take(4);
            if (m & H_GENERIC_GRAIN_TYPE) hw.skip_string();
            if ((m & H_CORRELATION_ID) && !hw.bad && hw.take(8)) corr = (int64_t)hw.c.u64(hw.p - 8);
            // bool tokens: 1 byte each
            const uint32_t nb = __popc(m & (H_ALWAYS_INTERLEAVE | H_IS_NEW_PLACEMENT | H_READ_ONLY | H_IS_UNORDERED));
            if (nb) hw.take(nb);
            if (m & H_NEW_GRAIN_TYPE) hw.skip_string();
            if (m & H_REJECTION_INFO) hw.skip_string();
            if (m & H_REJECTION_TYPE) hw.take(1);
            if (m & H_RESEND_COUNT) hw.take(4);
            if (m & H_RESULT) hw.take(1);
            if (m & H_SENDING_ACTIVATION) sa = hw.key(nullptr);
            if (m & H_SENDING_GRAIN) sg = hw.key(nullptr);
            if ((m & H_SENDING_SILO) && !hw.bad && hw.take(24)) {
#pragma unroll
                for (int j = 0; j < 6; ++j) ss[j] = hw.c.u32(hw.p - 24 + 4 * j);
            }
            if (m & H_TARGET_ACTIVATION) ta = hw.key(nullptr);
            if (m & H_TARGET_GRAIN) {
                int32_t ext = -1;
                tg = hw.key(&ext);
                flags |= FR_HAS_TARGET | (ext >= 0 ? FR_TARGET_KEYEXT : 0u);
                tg_ext = ext;                              // the string is the last ext bytes read
                tg_ext_off = start + hw.p - (uint32_t)(ext > 0 ? ext : 0);
            }
            if (m & H_TARGET_SILO) {
                if (m & H_TARGET_OBSERVER) {
                    flags |= FR_FALLBACK;  // TargetObserver (object-serialized) precedes TargetSilo
                } else if (!hw.bad && hw.take(24)) {
#pragma unroll
                    for (int j = 0; j < 6; ++j) ts[j] = hw.c.u32(hw.p - 24 + 4 * j);
                }
            }
            malformed = hw.bad;
        }
    }
    if (malformed) {
        flags = FR_MALFORMED;
        mask = 0;
        cat = 0;
        dir = 0xFFu;
        corr = 0;
        tg = ta = sa = sg = Key3{0, 0, 0};
        tg_ext = GD_KEYEXT_HOST;
#pragma unroll
        for (int j = 0; j < 6; ++j) ts[j] = ss[j] = 0;
    }
    o.flags[i] = flags;
    store_key(o.target_grain, i, tg);
    if (o.mask) o.mask[i] = mask;
    store_key(o.target_activation, i, ta);
    store_key(o.sending_activation, i, sa);
    store_key(o.sending_grain, i, sg);
    store_silo(o.target_silo, i, ts);
    store_silo(o.sending_silo, i, ss);
    if (o.correlation_id) o.correlation_id[i] = corr;
    if (o.category) o.category[i] = (uint8_t)cat;
    if (o.direction) o.direction[i] = (uint8_t)dir;
    if (o.tg_ext_len) {
        o.tg_ext_len[i] = (flags & FR_FALLBACK) ? GD_KEYEXT_HOST : tg_ext;
        o.tg_ext_off[i] = tg_ext_off;
    }
}

// Dispatcher.AddressMessage skips complete addresses (Dispatcher.cs:718); frames without a decoded
// TargetGrain go back to the C# deserializer.  Neither carries a silo / activation.
static __global__ __launch_bounds__(BLOCK) void k_frame_status(const uint32_t* __restrict__ flags, uint32_t n,
                                                        uint32_t* __restrict__ silo, uint32_t* __restrict__ act,
                                                        uint8_t* __restrict__ status) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t f = flags[i];
    const bool undecoded = !(f & FR_HAS_TARGET) || (f & (FR_FALLBACK | FR_MALFORMED));
    const bool addressed = !undecoded && (f & FR_COMPLETE);
    if (undecoded || addressed) {
        status[i] = undecoded ? ROUTE_UNDECODED : ROUTE_ADDRESSED;
        silo[i] = 0xFFFFFFFFu;
        act[i] = 0xFFFFFFFFu;
    }
}

}  // namespace gd
