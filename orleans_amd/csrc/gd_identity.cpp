// gd_identity.cpp -- host-side identity primitives of libgraindispatch (L0 of
// the Orleans dispatch path) and the ring builders (membership-change time,
// not per message).
//
//   JenkinsHash        src/Orleans.Core.Abstractions/IDs/JenkinsHash.cs:11-105
//   UniqueKey hash     src/Orleans.Core.Abstractions/IDs/UniqueKey.cs:272-293
//   CalculateIdHash    src/Orleans.Core/Utils/Utils.cs:184-203 (SHA-256, UTF-16LE,
//                      XOR of 8 big-endian int32)
//   SiloAddress        src/Orleans.Core.Abstractions/IDs/SiloAddress.cs:164-329
//   ring D / R build   LocalGrainDirectory.cs:284-309, ConsistentRingProvider.cs:92-133
//   ring V build       VirtualBucketsRingProvider.cs:122-149
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "graindispatch.h"
#include "gd_common.h"

namespace gd {

// ---------------------------------------------------------------- Jenkins
static inline void jmix(uint32_t& a, uint32_t& b, uint32_t& c) {
    a -= b; a -= c; a ^= (c >> 13);
    b -= c; b -= a; b ^= (a << 8);
    c -= a; c -= b; c ^= (b >> 13);
    a -= b; a -= c; a ^= (c >> 12);
    b -= c; b -= a; b ^= (a << 16);
    c -= a; c -= b; c ^= (b >> 5);
    a -= b; a -= c; a ^= (c >> 3);
    b -= c; b -= a; b ^= (a << 10);
    c -= a; c -= b; c ^= (b >> 15);
}

static inline uint32_t le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

uint32_t jenkins_bytes(const uint8_t* data, size_t len) {
    uint32_t a = 0x9e3779b9u, b = a, c = 0;
    size_t i = 0;
    for (; i + 12 <= len; i += 12) {
        a += le32(data + i);
        b += le32(data + i + 4);
        c += le32(data + i + 8);
        jmix(a, b, c);
    }
    c += (uint32_t)len;
    // The tail fills a (bytes 0-3), b (4-7), then c from bit 8 (JenkinsHash.cs:50-71).
    const size_t rem = len - i;
    for (size_t k = 0; k < rem; ++k) {
        const uint32_t v = data[i + k];
        if (k < 4) a += v << (8 * k);
        else if (k < 8) b += v << (8 * (k - 4));
        else c += v << (8 * (k - 8) + 8);
    }
    jmix(a, b, c);
    return c;
}

uint32_t jenkins_u64x3(uint64_t u1, uint64_t u2, uint64_t u3) {
    uint32_t a = 0x9e3779b9u, b = a, c = 0;
    a += (uint32_t)u1;
    b += (uint32_t)(u1 >> 32);
    c += (uint32_t)u2;
    jmix(a, b, c);
    a += (uint32_t)(u2 >> 32);
    b += (uint32_t)u3;
    c += (uint32_t)(u3 >> 32);
    jmix(a, b, c);
    c += 24;
    jmix(a, b, c);
    return c;
}

// ---------------------------------------------------------------- SHA-256 (FIPS 180-4)
namespace {
const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

void sha256_block(uint32_t st[8], const uint8_t* blk) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
        w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) |
               ((uint32_t)blk[4 * i + 2] << 8) | (uint32_t)blk[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
        const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
        const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; ++i) {
        const uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
        const uint32_t ch = (e & f) ^ (~e & g);
        const uint32_t t1 = h + S1 + ch + K256[i] + w[i];
        const uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
        const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        const uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}
}  // namespace

void sha256(const uint8_t* data, size_t len, uint8_t out[32]) {
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                      0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    size_t i = 0;
    for (; i + 64 <= len; i += 64) sha256_block(st, data + i);
    uint8_t tail[128];
    const size_t rem = len - i;
    std::memcpy(tail, data + i, rem);
    tail[rem] = 0x80;
    const size_t tl = (rem + 1 + 8 <= 64) ? 64 : 128;
    std::memset(tail + rem + 1, 0, tl - rem - 1);
    const uint64_t bits = (uint64_t)len * 8;
    for (int k = 0; k < 8; ++k) tail[tl - 1 - k] = (uint8_t)(bits >> (8 * k));
    sha256_block(st, tail);
    if (tl == 128) sha256_block(st, tail + 64);
    for (int k = 0; k < 8; ++k) {
        out[4 * k] = (uint8_t)(st[k] >> 24);
        out[4 * k + 1] = (uint8_t)(st[k] >> 16);
        out[4 * k + 2] = (uint8_t)(st[k] >> 8);
        out[4 * k + 3] = (uint8_t)st[k];
    }
}

// UTF-8 -> UTF-16LE (Encoding.Unicode); invalid sequences map to U+FFFD as .NET does.
static std::vector<uint8_t> utf16le(const char* s) {
    std::vector<uint8_t> out;
    const uint8_t* p = (const uint8_t*)s;
    auto put = [&](uint32_t u) { out.push_back((uint8_t)u); out.push_back((uint8_t)(u >> 8)); };
    while (*p) {
        uint32_t cp;
        int extra;
        if (*p < 0x80) { cp = *p; extra = 0; }
        else if ((*p & 0xE0) == 0xC0) { cp = *p & 0x1F; extra = 1; }
        else if ((*p & 0xF0) == 0xE0) { cp = *p & 0x0F; extra = 2; }
        else if ((*p & 0xF8) == 0xF0) { cp = *p & 0x07; extra = 3; }
        else { put(0xFFFD); ++p; continue; }
        ++p;
        bool ok = true;
        for (int k = 0; k < extra; ++k) {
            if ((*p & 0xC0) != 0x80) { ok = false; break; }
            cp = (cp << 6) | (*p & 0x3F);
            ++p;
        }
        if (!ok) { put(0xFFFD); continue; }
        if (cp >= 0x10000) {
            cp -= 0x10000;
            put(0xD800 + (cp >> 10));
            put(0xDC00 + (cp & 0x3FF));
        } else {
            put(cp);
        }
    }
    return out;
}

int32_t calculate_id_hash(const char* utf8) {
    const std::vector<uint8_t> u = utf16le(utf8);
    uint8_t d[32];
    sha256(u.data(), u.size(), d);
    uint32_t h = 0;
    for (int i = 0; i < 32; i += 4)
        h ^= ((uint32_t)d[i] << 24) | ((uint32_t)d[i + 1] << 16) | ((uint32_t)d[i + 2] << 8) | d[i + 3];
    return (int32_t)h;
}

// IPEndPoint.ToString(): "a.b.c.d:port" or "[v6]:port" (RFC 5952 compressed,
// lower-case; IPv4-mapped as ::ffff:a.b.c.d).
std::string endpoint_string(const gd_silo_addr& s) {
    char buf[96];
    if (s.is_v4) {
        std::snprintf(buf, sizeof buf, "%u.%u.%u.%u:%d", s.ip[12], s.ip[13], s.ip[14], s.ip[15], s.port);
        return buf;
    }
    uint16_t w[8];
    for (int i = 0; i < 8; ++i) w[i] = (uint16_t)((s.ip[2 * i] << 8) | s.ip[2 * i + 1]);
    std::string a;
    bool mapped = true;
    for (int i = 0; i < 5; ++i) mapped &= (w[i] == 0);
    mapped &= (w[5] == 0xFFFF);
    if (mapped) {
        std::snprintf(buf, sizeof buf, "::ffff:%u.%u.%u.%u", s.ip[12], s.ip[13], s.ip[14], s.ip[15]);
        a = buf;
    } else {
        int best = -1, bestlen = 1;
        for (int i = 0; i < 8;) {
            if (w[i] != 0) { ++i; continue; }
            int j = i;
            while (j < 8 && w[j] == 0) ++j;
            if (j - i > bestlen) { best = i; bestlen = j - i; }
            i = j;
        }
        for (int i = 0; i < 8; ++i) {
            if (i == best) { a += (i == 0) ? "::" : ":"; i += bestlen - 1; continue; }
            std::snprintf(buf, sizeof buf, "%x", w[i]);
            a += buf;
            if (i != 7) a += ":";
        }
    }
    std::snprintf(buf, sizeof buf, "]:%d", s.port);
    return "[" + a + buf;
}

int32_t silo_consistent_hash(const gd_silo_addr& s) {
    const std::string text = endpoint_string(s) + std::to_string(s.generation);
    return calculate_id_hash(text.c_str());
}

void silo_uniform_hashes(const gd_silo_addr& s, uint32_t n, uint32_t* out) {
    uint8_t bytes[28];
    std::memcpy(bytes, s.ip, 16);
    if (s.is_v4) std::memset(bytes, 0, 12);
    std::memcpy(bytes + 16, &s.port, 4);        // little-endian int32 (Buffer.BlockCopy)
    std::memcpy(bytes + 20, &s.generation, 4);
    for (uint32_t e = 0; e < n; ++e) {
        const int32_t extra = (int32_t)e;
        std::memcpy(bytes + 24, &extra, 4);
        out[e] = jenkins_bytes(bytes, sizeof bytes);
    }
}

int silo_compare(const gd_silo_addr& a, const gd_silo_addr& b) {
    if (a.generation != b.generation) return a.generation < b.generation ? -1 : 1;
    if (a.port != b.port) return a.port < b.port ? -1 : 1;
    // AddressFamily InterNetwork(2) < InterNetworkV6(23)
    if (a.is_v4 != b.is_v4) return a.is_v4 ? -1 : 1;
    const int off = a.is_v4 ? 12 : 0;
    for (int i = off; i < 16; ++i)
        if (a.ip[i] != b.ip[i]) return a.ip[i] < b.ip[i] ? -1 : 1;
    return 0;
}

}  // namespace gd

// ---------------------------------------------------------------- C ABI
extern "C" {

uint32_t gd_jenkins_hash_bytes(const uint8_t* data, size_t len) {
    return gd::jenkins_bytes(data, len);
}
uint32_t gd_jenkins_hash_u64x3(uint64_t u1, uint64_t u2, uint64_t u3) {
    return gd::jenkins_u64x3(u1, u2, u3);
}
uint32_t gd_uniform_hash(const gd_key* k) {
    return k ? gd::jenkins_u64x3(k->type_code_data, k->n0, k->n1) : 0;
}
int32_t gd_calculate_id_hash(const char* utf8_text) {
    return utf8_text ? gd::calculate_id_hash(utf8_text) : 0;
}
int32_t gd_silo_consistent_hash(const gd_silo_addr* silo) {
    return silo ? gd::silo_consistent_hash(*silo) : 0;
}
int gd_silo_uniform_hashes(const gd_silo_addr* silo, uint32_t n, uint32_t* out) {
    if (!silo || (n && !out)) return GD_EINVAL;
    gd::silo_uniform_hashes(*silo, n, out);
    return GD_OK;
}
int gd_silo_compare(const gd_silo_addr* a, const gd_silo_addr* b) {
    return gd::silo_compare(*a, *b);
}

int gd_ring_build(int mode, const gd_silo_addr* silos, uint32_t n_silos, uint32_t buckets_per_silo,
                  uint32_t* out_points, uint32_t* out_owner, uint32_t* out_n) {
    if (!silos || !out_points || !out_owner || !out_n || n_silos == 0) return GD_EINVAL;
    if (mode == GD_RING_DIRECTORY || mode == GD_RING_CONSISTENT) {
        // AddServer: insert at FindLastIndex(h < hash) + 1, silos in membership order
        // (LocalGrainDirectory.cs:296-303; ConsistentRingProvider.cs:105-110).
        std::vector<int32_t> h(n_silos);
        for (uint32_t i = 0; i < n_silos; ++i) h[i] = gd::silo_consistent_hash(silos[i]);
        std::vector<uint32_t> ring;
        for (uint32_t i = 0; i < n_silos; ++i) {
            int last = -1;
            for (size_t j = 0; j < ring.size(); ++j)
                if (h[ring[j]] < h[i]) last = (int)j;
            ring.insert(ring.begin() + (last + 1), i);
        }
        for (uint32_t j = 0; j < n_silos; ++j) {
            out_points[j] = (uint32_t)h[ring[j]];
            out_owner[j] = ring[j];
        }
        *out_n = n_silos;
        return GD_OK;
    }
    if (mode == GD_RING_VIRTUAL_BUCKETS) {
        if (buckets_per_silo == 0) return GD_EINVAL;
        // SortedDictionary<uint, SiloAddress>; a collision keeps the lesser silo
        // (VirtualBucketsRingProvider.cs:127-136).
        std::map<uint32_t, uint32_t> bmap;
        std::vector<uint32_t> pts(buckets_per_silo);
        for (uint32_t i = 0; i < n_silos; ++i) {
            gd::silo_uniform_hashes(silos[i], buckets_per_silo, pts.data());
            for (uint32_t p : pts) {
                auto it = bmap.find(p);
                if (it != bmap.end() && gd::silo_compare(silos[i], silos[it->second]) > 0) continue;
                bmap[p] = i;
            }
        }
        uint32_t j = 0;
        for (const auto& kv : bmap) {
            out_points[j] = kv.first;
            out_owner[j] = kv.second;
            ++j;
        }
        *out_n = j;
        return GD_OK;
    }
    return GD_EINVAL;
}

int gd_abi_version(void) { return GD_ABI_VERSION; }

}  // extern "C"
