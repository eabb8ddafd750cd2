// eng_cache.hip -- libgraindispatch: non-owner directory cache (LocalLookup).
// Shared handle and helpers: gd_engine.h.
#include "gd_engine.h"

// ================================================================== non-owner directory cache
namespace gdx {

// KeyExt helpers (defined with the KeyExt section below).

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

}  // namespace gdx

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

namespace gdx {

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

}  // namespace gdx

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

namespace gdx {

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

}  // namespace gdx

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

}  // extern "C"