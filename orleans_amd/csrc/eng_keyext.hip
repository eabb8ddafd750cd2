// eng_keyext.hip -- libgraindispatch: KeyExt grains (string keys) and membership churn (IsValidSilo, VersionTag, Merge).
// Shared handle and helpers: gd_engine.h.
#include "gd_engine.h"

// ================================================================== KeyExt grains (gd_keyext.h)
namespace gdx {

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

}  // namespace gdx

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

// ================================================================== membership churn: IsValidSilo, VersionTag,
// silo removal, handoff merge (gd_dirops.h)
namespace gdx {

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
                      is_new, pass, (const gd_val*)nullptr, table_args(h), (uint32_t*)nullptr));
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

}  // namespace gdx

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
