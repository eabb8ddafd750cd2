// orleans_dispatch.hpp -- C++ host layer above the libgraindispatch C ABI that
// mirrors the reference's interfaces on the dispatch path (same names, argument
// meaning and error behaviour), so host code and parity tests read like the
// reference's own.  The reference is C# (rikbosch/orleans); .NET is absent from
// this image, so this C++ layer stands where the C# batching stage would
// (INTEGRATION.md shows the C# P/Invoke form of the same calls).
//
//   UniqueKey / GrainId / SiloAddress   src/Orleans.Core.Abstractions/IDs/{UniqueKey,GrainId,SiloAddress}.cs
//   ActivationAddress                   src/Orleans.Core.Abstractions/IDs/ActivationAddress.cs:6-34
//   AddressAndTag / AddressesAndTag     src/Orleans.Core/GrainDirectory/IGrainDirectory.cs:75-87
//   GrainDirectoryPartition             src/Orleans.Runtime/GrainDirectory/GrainDirectoryPartition.cs:207-441
//   LocalGrainDirectory                 src/Orleans.Runtime/GrainDirectory/LocalGrainDirectory.cs:284-850
//   ConsistentRingProvider              src/Orleans.Runtime/ConsistentRing/ConsistentRingProvider.cs:54-372
//   VirtualBucketsRingProvider          src/Orleans.Runtime/ConsistentRing/VirtualBucketsRingProvider.cs:122-293
//   Dispatcher.AddressMessage           src/Orleans.Runtime/Core/Dispatcher.cs:715-767
//   IncomingMessageAgent.ReceiveMessage src/Orleans.Runtime/Messaging/IncomingMessageAgent.cs:92-190
//   ActivationDirectory                 src/Orleans.Runtime/Catalog/ActivationDirectory.cs:41-131
//   AdaptiveGrainDirectoryCache         src/Orleans.Runtime/GrainDirectory/AdaptiveGrainDirectoryCache.cs:7-140
//                                       (over LRU, src/Orleans.Core/Utils/LRU.cs)
//
// Every per-message decision runs on the GPU through the C ABI; single-grain
// calls are batches of one.  Errors from the ABI throw OrleansException (the C#
// side's exception type on this path).
#pragma once

#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
#include <map>
#include <optional>
#include <stdexcept>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "graindispatch.h"

namespace orleans {

class OrleansException : public std::runtime_error {
public:
    OrleansException(int code, const std::string& msg) : std::runtime_error(msg), code(code) {}
    int code;
};

inline void Check(gd_handle* h, int rc) {
    if (rc != GD_OK) throw OrleansException(rc, gd_last_error(h));
}

// ------------------------------------------------------------------ identity
struct UniqueKey {
    enum class Category : uint8_t { None = 0, SystemTarget = 1, SystemGrain = 2, Grain = 3, Client = 4,
                                    KeyExtGrain = 6, GeoClient = 7 };   // UniqueKey.cs:17-26
    uint64_t N0 = 0, N1 = 0, TypeCodeData = 0;
    std::optional<std::string> KeyExt;

    Category IdCategory() const { return static_cast<Category>((TypeCodeData >> 56) & 0xFF); }
    bool HasKeyExt() const { return IdCategory() == Category::KeyExtGrain || IdCategory() == Category::GeoClient; }
    bool IsLongKey() const { return N0 == 0; }

    // UniqueKey.NewKey(long, category, typeData) (UniqueKey.cs:112-128): typeData is a long,
    // sign-extended from the int grain type code before the 56-bit mask.
    static UniqueKey NewKey(int64_t longKey, Category category, int64_t typeData) {
        UniqueKey k;
        k.N1 = static_cast<uint64_t>(longKey);
        k.TypeCodeData = (static_cast<uint64_t>(category) << 56) + (static_cast<uint64_t>(typeData) & 0x00FFFFFFFFFFFFFFull);
        return k;
    }

    // UniqueKey.ToByteArray (UniqueKey.cs:295-336)
    std::vector<uint8_t> ToByteArray() const {
        const int32_t len = KeyExt ? static_cast<int32_t>(KeyExt->size()) : -1;
        std::vector<uint8_t> b(28 + (KeyExt ? KeyExt->size() : 0));
        std::memcpy(b.data(), &N0, 8);
        std::memcpy(b.data() + 8, &N1, 8);
        std::memcpy(b.data() + 16, &TypeCodeData, 8);
        std::memcpy(b.data() + 24, &len, 4);
        if (KeyExt && !KeyExt->empty()) std::memcpy(b.data() + 28, KeyExt->data(), KeyExt->size());
        return b;
    }

    // UniqueKey.GetUniformHashCode (UniqueKey.cs:272-293)
    uint32_t GetUniformHashCode() const {
        if (HasKeyExt() && KeyExt) {
            const auto b = ToByteArray();
            return gd_jenkins_hash_bytes(b.data(), b.size());
        }
        const gd_key k{N0, N1, TypeCodeData};
        return gd_uniform_hash(&k);
    }

    bool operator==(const UniqueKey& o) const {   // UniqueKey.Equals (:245-251)
        return N0 == o.N0 && N1 == o.N1 && TypeCodeData == o.TypeCodeData && (!HasKeyExt() || KeyExt == o.KeyExt);
    }
    bool operator<(const UniqueKey& o) const {    // UniqueKey.CompareTo order (:255-265)
        if (TypeCodeData != o.TypeCodeData) return TypeCodeData < o.TypeCodeData;
        if (N0 != o.N0) return N0 < o.N0;
        if (N1 != o.N1) return N1 < o.N1;
        return HasKeyExt() && KeyExt < o.KeyExt;
    }
    gd_key ToNative() const { return gd_key{N0, N1, TypeCodeData}; }
};

struct GrainId {
    UniqueKey Key;
    // GrainId.GetGrainId(long typeCode, long primaryKey, string keyExt = null) (GrainId.cs:72-77):
    // a key extension makes it a KeyExtGrain (compound key).
    static GrainId GetGrainId(int64_t typeCode, int64_t primaryKey,
                              const std::optional<std::string>& keyExt = std::nullopt) {
        GrainId g{UniqueKey::NewKey(primaryKey, keyExt ? UniqueKey::Category::KeyExtGrain : UniqueKey::Category::Grain,
                                    typeCode)};
        g.Key.KeyExt = keyExt;
        return g;
    }
    // GrainId.GetGrainId(long typeCode, string primaryKey) (GrainId.cs:86-91): string-keyed grains
    // (IGrainWithStringKey), N0 = N1 = 0, the string is the KeyExt (UTF-8 here).
    static GrainId GetGrainId(int64_t typeCode, const std::string& primaryKey) {
        GrainId g{UniqueKey::NewKey(0, UniqueKey::Category::KeyExtGrain, typeCode)};
        g.Key.KeyExt = primaryKey;
        return g;
    }
    bool IsSystemTarget() const { return Key.IdCategory() == UniqueKey::Category::SystemTarget; }
    uint32_t GetUniformHashCode() const { return Key.GetUniformHashCode(); }
    bool operator==(const GrainId& o) const { return Key == o.Key; }
    bool operator<(const GrainId& o) const { return Key < o.Key; }
};

using ActivationId = UniqueKey;   // ActivationId.cs: a UniqueKey of Category None

struct SiloAddress {
    std::array<uint8_t, 16> Ip{};   // IPv4 in [12..15]
    bool IsV4 = true;
    int32_t Port = 0;
    int32_t Generation = 0;

    static SiloAddress New(uint8_t a, uint8_t b, uint8_t c, uint8_t d, int32_t port, int32_t gen) {
        SiloAddress s;
        s.Ip[12] = a; s.Ip[13] = b; s.Ip[14] = c; s.Ip[15] = d;
        s.Port = port;
        s.Generation = gen;
        return s;
    }
    gd_silo_addr ToNative() const {
        gd_silo_addr n{};
        std::memcpy(n.ip, Ip.data(), 16);
        n.port = Port;
        n.generation = Generation;
        n.is_v4 = IsV4 ? 1 : 0;
        return n;
    }
    int32_t GetConsistentHashCode() const { const auto n = ToNative(); return gd_silo_consistent_hash(&n); }
    std::vector<uint32_t> GetUniformHashCodes(int numHashes) const {
        std::vector<uint32_t> out(numHashes);
        const auto n = ToNative();
        if (gd_silo_uniform_hashes(&n, numHashes, out.data()) != GD_OK) throw OrleansException(GD_EINVAL, "hashes");
        return out;
    }
    int CompareTo(const SiloAddress& o) const { const auto a = ToNative(), b = o.ToNative(); return gd_silo_compare(&a, &b); }
    bool operator==(const SiloAddress& o) const {
        return Ip == o.Ip && IsV4 == o.IsV4 && Port == o.Port && Generation == o.Generation;
    }
    std::string ToString() const {
        return std::to_string(Ip[12]) + "." + std::to_string(Ip[13]) + "." + std::to_string(Ip[14]) + "." +
               std::to_string(Ip[15]) + ":" + std::to_string(Port) + "@" + std::to_string(Generation);
    }
};

struct SiloLess {            // SiloAddress.CompareTo order, for maps keyed by silo
    bool operator()(const SiloAddress& a, const SiloAddress& b) const { return a.CompareTo(b) < 0; }
};

struct ActivationAddress {   // ActivationAddress.cs:6-34
    SiloAddress Silo;
    GrainId Grain;
    ActivationId Activation;
};

struct AddressAndTag { std::optional<ActivationAddress> Address; int VersionTag = 0; };
struct AddressesAndTag { std::optional<std::vector<ActivationAddress>> Addresses; int VersionTag = 0; };

// The KeyExt strings of a batch of keys in the gd_key_ext layout (one UTF-8 blob, offset + length
// per key; GD_KEYEXT_NULL for a null KeyExt or a category without one).
class KeyExtBatch {
public:
    explicit KeyExtBatch(const std::vector<const UniqueKey*>& keys) {
        off_.resize(keys.size());
        len_.resize(keys.size());
        for (size_t i = 0; i < keys.size(); ++i) {
            const UniqueKey& k = *keys[i];
            if (k.HasKeyExt() && k.KeyExt) {
                off_[i] = bytes_.size();
                len_[i] = (int32_t)k.KeyExt->size();
                bytes_.insert(bytes_.end(), k.KeyExt->begin(), k.KeyExt->end());
            } else {
                off_[i] = 0;
                len_[i] = GD_KEYEXT_NULL;
            }
        }
        bytes_.push_back(0);   // a valid pointer even when empty
    }
    const gd_key_ext* get() {
        ext_ = gd_key_ext{bytes_.data(), off_.data(), len_.data(), (uint64_t)(bytes_.size() - 1)};
        return &ext_;
    }

private:
    std::vector<uint8_t> bytes_;
    std::vector<uint64_t> off_;
    std::vector<int32_t> len_;
    gd_key_ext ext_{};
};

// ------------------------------------------------------------------ native handle
class DispatchHandle {
public:
    explicit DispatchHandle(int device = 0, uint64_t tableCapacity = 1u << 20, uint32_t mySilo = 0,
                            uint32_t seedSilo = GD_NO_SILO) {
        gd_config cfg{};
        cfg.struct_size = sizeof(gd_config);
        cfg.device = device;
        cfg.table_capacity = tableCapacity;
        cfg.my_silo = mySilo;
        cfg.seed_silo = seedSilo;
        Check(nullptr, gd_create(&cfg, &h_));
    }
    ~DispatchHandle() { gd_destroy(h_); }
    DispatchHandle(const DispatchHandle&) = delete;
    DispatchHandle& operator=(const DispatchHandle&) = delete;
    gd_handle* get() const { return h_; }

private:
    gd_handle* h_ = nullptr;
};

// Index tables shared by the host-side objects: the GPU stores compact indices.
class SiloTable {
public:
    uint32_t IndexOf(const SiloAddress& s) {
        for (uint32_t i = 0; i < silos_.size(); ++i)
            if (silos_[i] == s) return i;
        silos_.push_back(s);
        return static_cast<uint32_t>(silos_.size() - 1);
    }
    const SiloAddress& At(uint32_t i) const { return silos_.at(i); }
    size_t Size() const { return silos_.size(); }

private:
    std::vector<SiloAddress> silos_;
};

// ------------------------------------------------------------------ rings
// A ring snapshot built by the reference's AddServer rules and installed on the GPU.
class RingSnapshot {
public:
    RingSnapshot(gd_handle* h, int mode, uint32_t bucketsPerSilo) : h_(h), mode_(mode), buckets_(bucketsPerSilo) {}

    void Rebuild(const std::vector<SiloAddress>& membershipInAddOrder) {
        members_ = membershipInAddOrder;
        if (members_.empty()) { n_ = 0; return; }
        std::vector<gd_silo_addr> nat;
        for (const auto& s : members_) nat.push_back(s.ToNative());
        const size_t cap = members_.size() * (mode_ == GD_RING_VIRTUAL_BUCKETS ? buckets_ : 1);
        points_.assign(cap, 0);
        owner_.assign(cap, 0);
        uint32_t n = 0;
        Check(h_, gd_ring_build(mode_, nat.data(), (uint32_t)nat.size(), buckets_, points_.data(), owner_.data(), &n));
        points_.resize(n);
        owner_.resize(n);
        n_ = n;
        Check(h_, gd_ring_set(h_, mode_, points_.data(), owner_.data(), n));
    }
    const std::vector<SiloAddress>& Members() const { return members_; }
    const std::vector<uint32_t>& Points() const { return points_; }
    const std::vector<uint32_t>& Owners() const { return owner_; }
    uint32_t Size() const { return n_; }

    // batch GetPrimaryTargetSilo(uint key)
    std::vector<uint32_t> LookupHashes(const std::vector<uint32_t>& keys) const {
        std::vector<uint32_t> out(keys.size());
        if (!keys.empty()) Check(h_, gd_ring_lookup_hashes(h_, keys.data(), (uint32_t)keys.size(), out.data()));
        return out;
    }

private:
    gd_handle* h_;
    int mode_;
    uint32_t buckets_;
    std::vector<SiloAddress> members_;
    std::vector<uint32_t> points_, owner_;
    uint32_t n_ = 0;
};

// IConsistentRingProvider, ConsistentRingProvider flavour (mode R, clockwise, one point per silo)
class ConsistentRingProvider {
public:
    ConsistentRingProvider(gd_handle* h, SiloAddress me) : ring_(h, GD_RING_CONSISTENT, 1), me_(std::move(me)) {
        AddServer(me_);
    }
    void AddServer(const SiloAddress& s) {
        auto m = ring_.Members();
        if (std::find(m.begin(), m.end(), s) != m.end()) return;
        m.push_back(s);
        ring_.Rebuild(m);
    }
    void RemoveServer(const SiloAddress& s) {
        auto m = ring_.Members();
        m.erase(std::remove(m.begin(), m.end(), s), m.end());
        ring_.Rebuild(m);
    }
    SiloAddress GetPrimaryTargetSilo(uint32_t key) const { return ring_.Members().at(ring_.LookupHashes({key})[0]); }
    std::vector<uint32_t> GetPrimaryTargetSilos(const std::vector<uint32_t>& keys) const { return ring_.LookupHashes(keys); }
    // MyRange (ConsistentRingProvider.cs:112-124): (predecessor hash, my hash] as uint; full ring if alone
    std::pair<uint32_t, uint32_t> GetMyRange() const {
        const auto& pts = ring_.Points();
        const auto& own = ring_.Owners();
        const auto& mem = ring_.Members();
        if (pts.size() <= 1) return {0u, 0u};
        for (size_t i = 0; i < pts.size(); ++i)
            if (mem[own[i]] == me_) return {pts[(i + pts.size() - 1) % pts.size()], pts[i]};
        throw OrleansException(GD_ESTATE, "not in the ring");
    }
    const RingSnapshot& Ring() const { return ring_; }

private:
    RingSnapshot ring_;
    SiloAddress me_;
};

// IConsistentRingProvider default: VirtualBucketsRingProvider (mode V, 30 buckets per silo)
class VirtualBucketsRingProvider {
public:
    VirtualBucketsRingProvider(gd_handle* h, SiloAddress me, uint32_t numBucketsPerSilo = 30)
        : ring_(h, GD_RING_VIRTUAL_BUCKETS, numBucketsPerSilo), me_(std::move(me)) {
        AddServer(me_);
    }
    void AddServer(const SiloAddress& s) {
        auto m = ring_.Members();
        if (std::find(m.begin(), m.end(), s) != m.end()) return;
        m.push_back(s);
        ring_.Rebuild(m);
    }
    void RemoveServer(const SiloAddress& s) {
        auto m = ring_.Members();
        m.erase(std::remove(m.begin(), m.end(), s), m.end());
        ring_.Rebuild(m);
    }
    SiloAddress GetPrimaryTargetSilo(uint32_t key) const { return ring_.Members().at(ring_.LookupHashes({key})[0]); }
    // CalculateRange (VirtualBucketsRingProvider.cs:176-200): (prev point, point] for each of my buckets
    std::vector<std::pair<uint32_t, uint32_t>> GetMyRanges() const {
        std::vector<std::pair<uint32_t, uint32_t>> r;
        const auto& pts = ring_.Points();
        const auto& own = ring_.Owners();
        const auto& mem = ring_.Members();
        for (size_t i = 0; i < pts.size(); ++i)
            if (mem[own[i]] == me_) r.emplace_back(pts[(i + pts.size() - 1) % pts.size()], pts[i]);
        return r;
    }
    const RingSnapshot& Ring() const { return ring_; }

private:
    RingSnapshot ring_;
    SiloAddress me_;
};

// ------------------------------------------------------------------ directory
// GrainDirectoryPartition: single-activation entries in the GPU table.
class GrainDirectoryPartition {
public:
    GrainDirectoryPartition(gd_handle* h, SiloTable& silos) : h_(h), silos_(silos) {}

    // AddSingleActivation (GrainDirectoryPartition.cs:304-326): first registration wins; an
    // activation on a silo that is not valid (IsValidSilo, :310-311) is refused (no Address).
    // VersionTag: the library's deterministic stand-in for GrainInfo's rand.Next() (:121).
    AddressAndTag AddSingleActivation(const GrainId& grain, const ActivationId& act, const SiloAddress& silo) {
        return AddSingleActivations({grain}, {act}, {silo}).at(0);
    }
    std::vector<AddressAndTag> AddSingleActivations(const std::vector<GrainId>& grains,
                                                    const std::vector<ActivationId>& acts,
                                                    const std::vector<SiloAddress>& silos) {
        const size_t n = grains.size();
        std::vector<gd_val> out(n);
        // KeyExt grains (string / compound keys) go to the KeyExt table, the rest to the main one;
        // each keeps its batch order (first registration wins within each).
        for (int ext = 0; ext < 2; ++ext) {
            std::vector<size_t> idx;
            for (size_t i = 0; i < n; ++i)
                if (grains[i].Key.HasKeyExt() == (ext == 1)) idx.push_back(i);
            if (idx.empty()) continue;
            std::vector<gd_key> keys;
            std::vector<gd_val> vals, o(idx.size());
            std::vector<const UniqueKey*> uk;
            std::vector<uint8_t> ins(idx.size());
            for (size_t i : idx) {
                keys.push_back(grains[i].Key.ToNative());
                vals.push_back(gd_val{ActIndex(acts[i]), silos_.IndexOf(silos[i])});
                uk.push_back(&grains[i].Key);
            }
            if (ext) {
                KeyExtBatch kx(uk);
                Check(h_, gd_dir_register_ext(h_, keys.data(), kx.get(), vals.data(), (uint32_t)idx.size(), o.data(),
                                              ins.data()));
            } else {
                Check(h_, gd_dir_register(h_, keys.data(), vals.data(), (uint32_t)idx.size(), o.data(), ins.data()));
            }
            for (size_t j = 0; j < idx.size(); ++j) out[idx[j]] = o[j];
        }
        std::vector<AddressAndTag> r(n);
        std::vector<gd_key> tk;
        std::vector<size_t> ti;
        for (size_t i = 0; i < n; ++i) {
            if (out[i].act == GD_NO_ACTIVATION) continue;          // refused: IsValidSilo
            r[i].Address = ActivationAddress{silos_.At(out[i].silo), grains[i], acts_.at(out[i].act)};
            if (!grains[i].Key.HasKeyExt()) {
                tk.push_back(grains[i].Key.ToNative());
                ti.push_back(i);
            }
        }
        if (!tk.empty()) {
            std::vector<gd_val> v(tk.size());
            std::vector<int32_t> tags(tk.size());
            std::vector<uint8_t> f(tk.size());
            Check(h_, gd_dir_lookup_tagged(h_, tk.data(), (uint32_t)tk.size(), v.data(), tags.data(), f.data()));
            for (size_t j = 0; j < ti.size(); ++j) r[ti[j]].VersionTag = tags[j];
        }
        return r;
    }

    // GrainDirectoryPartition.Merge (GrainDirectoryPartition.cs:497-522) of a handed-off partition
    // (distinct grains).  Conflicting single-activation grains keep the lowest ActivationId
    // (GrainInfo.Merge :139-179); the activations to delete come back grouped per silo -- what the
    // reference hands to Catalog.DeleteActivations on each silo (:514-518).  Multi-instance grains
    // (AddActivation) are unioned here on the host.
    std::map<SiloAddress, std::vector<ActivationAddress>, SiloLess> Merge(const std::vector<GrainId>& grains,
                                                                          const std::vector<ActivationId>& acts,
                                                                          const std::vector<SiloAddress>& silos) {
        const size_t n = grains.size();
        std::map<SiloAddress, std::vector<ActivationAddress>, SiloLess> del;
        // KeyExt grains (string / compound keys) live in the KeyExt table, which gd_dir_merge does not
        // probe: they are merged here, by the same rule, as AddSingleActivations splits them.
        std::vector<size_t> main, ext;
        for (size_t i = 0; i < n; ++i) (grains[i].Key.HasKeyExt() ? ext : main).push_back(i);
        std::vector<gd_key> keys(main.size());
        std::vector<gd_val> vals(main.size()), dropped(main.size());
        std::vector<uint8_t> st(main.size());
        for (size_t j = 0; j < main.size(); ++j) {
            keys[j] = grains[main[j]].Key.ToNative();
            vals[j] = gd_val{ActIndex(acts[main[j]]), silos_.IndexOf(silos[main[j]])};
        }
        FlushIds();
        if (!main.empty())
            Check(h_, gd_dir_merge(h_, keys.data(), vals.data(), nullptr, (uint32_t)main.size(), st.data(),
                                   dropped.data()));
        for (size_t j = 0; j < main.size(); ++j) {
            const size_t i = main[j];
            if (st[j] == GD_MERGE_KEPT || st[j] == GD_MERGE_DROPPED)
                del[silos_.At(dropped[j].silo)].push_back(
                    ActivationAddress{silos_.At(dropped[j].silo), grains[i], acts_.at(dropped[j].act)});
            else if (st[j] == GD_MERGE_UNION)            // the device entry is GD_ACT_MULTI already
                multi_[grains[i]][acts[i]] = silos[i];
            else if (st[j] == GD_MERGE_HOST && multi_.count(grains[i]))
                AddActivation(grains[i], acts[i], silos[i]);
        }
        for (size_t i : ext) {
            const gd_key k = grains[i].Key.ToNative();
            KeyExtBatch kx({&grains[i].Key});
            gd_val cur{};
            uint8_t found = 0;
            Check(h_, gd_dir_lookup_ext(h_, &k, kx.get(), 1, &cur, &found));
            const gd_val in{ActIndex(acts[i]), silos_.IndexOf(silos[i])};
            if (!found) {                                  // partitionData.Add (:517-520)
                gd_val o{};
                uint8_t ins = 0;
                Check(h_, gd_dir_register_ext(h_, &k, kx.get(), &in, 1, &o, &ins));
                continue;
            }
            if (cur.act == in.act) continue;               // the same activation: nothing to drop
            const ActivationId& have = acts_.at(cur.act);
            if (acts[i] < have) {                          // OrderBy(ActivationId).First() stays (:160-163)
                uint8_t removed = 0;
                Check(h_, gd_dir_unregister_ext(h_, &k, kx.get(), &cur.act, 1, &removed));
                gd_val o{};
                uint8_t ins = 0;
                Check(h_, gd_dir_register_ext(h_, &k, kx.get(), &in, 1, &o, &ins));
                del[silos_.At(cur.silo)].push_back(ActivationAddress{silos_.At(cur.silo), grains[i], have});
            } else {
                del[silos[i]].push_back(ActivationAddress{silos[i], grains[i], acts[i]});
            }
        }
        return del;
    }

    // LocalGrainDirectory.AdjustLocalDirectory (LocalGrainDirectory.cs:351-361): drop every
    // instance located on the removed silo.  Returns the entries removed.
    uint64_t RemoveActivationsOn(const SiloAddress& removed) {
        const uint32_t s = silos_.IndexOf(removed);
        uint64_t n = 0, multi = 0;
        Check(h_, gd_dir_remove_silos(h_, &s, 1, &n, &multi, nullptr));
        std::vector<GrainId> touched;
        for (auto& kv : multi_)                        // multi-instance grains: their instances live here
            for (auto it = kv.second.begin(); it != kv.second.end();)
                if (it->second == removed) {
                    it = kv.second.erase(it);
                    touched.push_back(kv.first);
                } else {
                    ++it;
                }
        for (const auto& g : touched) {
            auto& inst = multi_[g];
            if (inst.empty()) {
                // the GPU entry is GD_ACT_MULTI unless one instance was left, and that one lived on
                // the removed silo: gd_dir_remove_silos already dropped and counted it
                const gd_key k = g.Key.ToNative();
                const uint32_t a = GD_ACT_MULTI;
                uint8_t removed = 0;
                Check(h_, gd_dir_unregister(h_, &k, &a, 1, &removed));
                multi_.erase(g);
                if (removed) ++n;
            } else {
                Publish(g, inst);
            }
        }
        return n;
    }

    // AddActivation (GrainDirectoryPartition.cs:274-302; GrainInfo.AddActivation :89-108): multi-
    // instance grains (StatelessWorker).  The instances live here; the GPU table holds the lookup
    // result -- the single instance, or GD_ACT_MULTI once there are two or more (routes then answer
    // GD_ROUTE_MULTI_ACT and the random choice of RandomPlacementDirector.cs:33-53 stays on the host).
    // Returns false when the activation was already registered on that silo (a refresh).
    bool AddActivation(const GrainId& grain, const ActivationId& act, const SiloAddress& silo) {
        auto& inst = multi_[grain];
        const auto it = inst.find(act);
        if (it != inst.end() && it->second == silo) return false;
        inst[act] = silo;
        ActIndex(act);
        Publish(grain, inst);
        return true;
    }

    // RemoveActivation (GrainDirectoryPartition.cs:335-363, UnregistrationCause.Force)
    bool RemoveActivation(const GrainId& grain, const ActivationId& act) {
        const auto mit = multi_.find(grain);
        if (mit != multi_.end()) {                     // a multi-instance grain: update its GPU entry
            if (!mit->second.erase(act)) return false;
            if (mit->second.empty()) {
                const gd_key k = grain.Key.ToNative();
                const uint32_t a = GD_ACT_MULTI;
                uint8_t removed = 0;
                Check(h_, gd_dir_unregister(h_, &k, &a, 1, &removed));
                if (!removed) {                        // the entry held the last single instance
                    const uint32_t a1 = ActIndex(act);
                    Check(h_, gd_dir_unregister(h_, &k, &a1, 1, &removed));
                }
                multi_.erase(mit);
            } else {
                Publish(grain, mit->second);
            }
            return true;
        }
        const auto it = act_index_.find(act);
        if (it == act_index_.end()) return false;
        const gd_key k = grain.Key.ToNative();
        const uint32_t a = it->second;
        uint8_t removed = 0;
        if (grain.Key.HasKeyExt()) {
            KeyExtBatch kx({&grain.Key});
            Check(h_, gd_dir_unregister_ext(h_, &k, kx.get(), &a, 1, &removed));
        } else {
            Check(h_, gd_dir_unregister(h_, &k, &a, 1, &removed));
        }
        return removed != 0;
    }

    // LookUpActivations (GrainDirectoryPartition.cs:385-441): null Addresses when absent; the
    // addresses on silos that are not valid are filtered out (:431), the VersionTag stays.
    AddressesAndTag LookUpActivations(const GrainId& grain) const {
        const gd_key k = grain.Key.ToNative();
        gd_val v{};
        uint8_t found = 0;
        int32_t tag = 0;
        if (grain.Key.HasKeyExt()) {
            KeyExtBatch kx({&grain.Key});
            Check(h_, gd_dir_lookup_ext(h_, &k, kx.get(), 1, &v, &found));
        } else {
            Check(h_, gd_dir_lookup_tagged(h_, &k, 1, &v, &tag, &found));
        }
        AddressesAndTag r;
        r.VersionTag = tag;
        if (found == 2) {                              // only an invalid silo: an empty list
            r.Addresses = std::vector<ActivationAddress>{};
            return r;
        }
        if (found && v.act == GD_ACT_MULTI) {          // every instance, from the host's list
            std::vector<ActivationAddress> all;
            for (const auto& kv : multi_.at(grain)) all.push_back(ActivationAddress{kv.second, grain, kv.first});
            r.Addresses = std::move(all);
        } else if (found) {
            r.Addresses = std::vector<ActivationAddress>{{silos_.At(v.silo), grain, acts_.at(v.act)}};
        }
        return r;
    }

    int Count() const {
        gd_stats s{};
        Check(h_, gd_stats_get(h_, &s));
        uint64_t ext = 0;
        Check(h_, gd_dir_ext_stats(h_, &ext, nullptr, nullptr));
        return (int)(s.table_live + ext);
    }
    const ActivationId& ActivationAt(uint32_t idx) const { return acts_.at(idx); }
    uint32_t ActIndex(const ActivationId& a) {
        const auto it = act_index_.find(a);
        if (it != act_index_.end()) return it->second;
        acts_.push_back(a);
        act_index_.emplace(a, (uint32_t)acts_.size() - 1);
        pending_ids_.push_back((uint32_t)acts_.size() - 1);
        return (uint32_t)acts_.size() - 1;
    }
    // The ActivationIds of new indices to the library (Merge orders by them).
    void FlushIds() {
        if (pending_ids_.empty()) return;
        std::vector<gd_key> ids;
        for (uint32_t i : pending_ids_) ids.push_back(acts_[i].ToNative());
        Check(h_, gd_activation_ids_set(h_, pending_ids_.data(), ids.data(), (uint32_t)ids.size()));
        pending_ids_.clear();
    }
    size_t ActivationCount() const { return acts_.size(); }

private:
    void Publish(const GrainId& grain, const std::map<ActivationId, SiloAddress>& inst) {
        const gd_key k = grain.Key.ToNative();
        const auto& first = *inst.begin();
        const gd_val v{inst.size() == 1 ? ActIndex(first.first) : GD_ACT_MULTI, silos_.IndexOf(first.second)};
        Check(h_, gd_dir_upsert(h_, &k, &v, 1, nullptr));
    }

    gd_handle* h_;
    SiloTable& silos_;
    std::vector<ActivationId> acts_;
    std::map<ActivationId, uint32_t> act_index_;
    std::vector<uint32_t> pending_ids_;
    std::map<GrainId, std::map<ActivationId, SiloAddress>> multi_;   // AddActivation grains
};

// AdaptiveGrainDirectoryCache<IReadOnlyList<Tuple<SiloAddress, ActivationId>>> for
// single-activation grains (AdaptiveGrainDirectoryCache.cs:7-140 over LRU.cs): the handle's GPU
// cache, exact LRU generations, string-keyed grains keyed by their KeyExt (gd_cache_*_ext).
// Owned by a LocalGrainDirectory in per-silo mode.
class AdaptiveGrainDirectoryCache {
public:
    using Value = std::pair<SiloAddress, ActivationId>;
    AdaptiveGrainDirectoryCache(gd_handle* h, SiloTable& silos, GrainDirectoryPartition& acts)
        : h_(h), silos_(silos), acts_(acts) {}

    // AddOrUpdate (:71-77); a batch is applied in order.
    void AddOrUpdate(const GrainId& key, const Value& value, int version) {
        AddOrUpdate(std::vector<GrainId>{key}, std::vector<Value>{value}, std::vector<int>{version});
    }
    void AddOrUpdate(const std::vector<GrainId>& keys, const std::vector<Value>& values,
                     const std::vector<int>& versions) {
        const size_t n = keys.size();
        std::vector<gd_key> k(n);
        std::vector<gd_val> v(n);
        std::vector<int32_t> ver(versions.begin(), versions.end());
        std::vector<const UniqueKey*> uk(n);
        for (size_t i = 0; i < n; ++i) {
            k[i] = keys[i].Key.ToNative();
            uk[i] = &keys[i].Key;
            v[i] = gd_val{acts_.ActIndex(values[i].second), silos_.IndexOf(values[i].first)};
        }
        KeyExtBatch kx(uk);
        if (n) Check(h_, gd_cache_add_ext(h_, k.data(), kx.get(), v.data(), ver.data(), (uint32_t)n));
    }
    bool Remove(const GrainId& key) {                   // :79-83
        const gd_key k = key.Key.ToNative();
        KeyExtBatch kx({&key.Key});
        uint8_t removed = 0;
        Check(h_, gd_cache_remove_ext(h_, &k, kx.get(), 1, &removed));
        return removed != 0;
    }
    void Clear() { Check(h_, gd_cache_clear(h_)); }     // :85-88
    bool LookUp(const GrainId& key, Value& result, int& version) {   // :90-109
        const gd_key k = key.Key.ToNative();
        KeyExtBatch kx({&key.Key});
        gd_val v{};
        int32_t ver = 0;
        uint8_t found = 0;
        Check(h_, gd_cache_lookup_ext(h_, &k, kx.get(), 1, &v, &ver, &found));
        if (!found) return false;
        result = Value{silos_.At(v.silo), acts_.ActivationAt(v.act)};
        version = ver;
        return true;
    }
    // KeyValues (:111-127)
    std::vector<std::tuple<GrainId, Value, int>> KeyValues() const {
        uint64_t n = 0, nb = 0;
        Check(h_, gd_cache_entries_ext(h_, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, &n,
                                       &nb));
        std::vector<gd_key> k(n);
        std::vector<gd_val> v(n);
        std::vector<int32_t> ver(n), xl(n);
        std::vector<uint64_t> gen(n), xo(n);
        std::vector<uint8_t> bytes(nb + 1);
        if (n)
            Check(h_, gd_cache_entries_ext(h_, k.data(), v.data(), ver.data(), gen.data(), xl.data(), xo.data(),
                                           bytes.data(), n, nb, &n, &nb));
        std::vector<std::tuple<GrainId, Value, int>> r;
        for (uint64_t i = 0; i < n; ++i) {
            GrainId g;
            g.Key.N0 = k[i].n0;
            g.Key.N1 = k[i].n1;
            g.Key.TypeCodeData = k[i].type_code_data;
            if (xl[i] >= 0) g.Key.KeyExt = std::string(reinterpret_cast<const char*>(bytes.data() + xo[i]), (size_t)xl[i]);
            r.emplace_back(g, Value{silos_.At(v[i].silo), acts_.ActivationAt(v[i].act)}, ver[i]);
        }
        return r;
    }
    int Count() const { return (int)Stats().count; }
    long NumAccesses() const { return (long)Stats().accesses; }
    long NumHits() const { return (long)Stats().hits; }

private:
    gd_cache_stats Stats() const {
        gd_cache_stats s{};
        Check(h_, gd_cache_stats_get(h_, &s));
        return s;
    }
    gd_handle* h_;
    SiloTable& silos_;
    GrainDirectoryPartition& acts_;
};

// LocalGrainDirectory: directory ring (mode D) + this GPU's partition.  Whole-node model by
// default (the owner partition is always consulted); EnableCache switches to the reference's
// per-silo model: only MyAddress's partition is local, other grains go through the cache.
class LocalGrainDirectory {
public:
    // One ring snapshot per handle: give every ring provider its own DispatchHandle.
    LocalGrainDirectory(gd_handle* h, SiloAddress me)
        : MyAddress(std::move(me)), h_(h), ring_(h, GD_RING_DIRECTORY, 1), partition_(h, silos_),
          cache_(h, silos_, partition_) {
        silos_.IndexOf(MyAddress);
        AddServer(MyAddress);
    }

    // AddServer / RemoveServer (LocalGrainDirectory.cs:284-345): membership in add order.
    void AddServer(const SiloAddress& s) {
        auto m = ring_.Members();
        if (std::find(m.begin(), m.end(), s) != m.end()) return;
        silos_.IndexOf(s);
        m.push_back(s);
        Install(m);
    }
    // RemoveServer (:311-345): the ring without the silo (membershipRingList.Remove), the valid silos
    // without it, then AdjustLocalDirectory (:351-361) and, per-silo, AdjustLocalCache (:371-385).
    void RemoveServer(const SiloAddress& s) {
        auto m = ring_.Members();
        if (std::find(m.begin(), m.end(), s) == m.end()) return;     // already removed
        m.erase(std::remove(m.begin(), m.end(), s), m.end());
        Install(m);
        partition_.RemoveActivationsOn(s);
    }

    // CalculateTargetSilo (LocalGrainDirectory.cs:477-545) for a batch; excludeThisSiloIfStopping is
    // false (what LocalLookup passes, :801) -- a running silo.
    std::vector<SiloAddress> CalculateTargetSilos(const std::vector<GrainId>& grains) const {
        std::vector<gd_key> keys;
        for (const auto& g : grains) keys.push_back(g.Key.ToNative());
        std::vector<uint32_t> idx(keys.size());
        if (!keys.empty()) Check(h_, gd_ring_owner(h_, keys.data(), (uint32_t)keys.size(), idx.data()));
        // KeyExt grains: the owner of their uniform hash over ToByteArray (UniqueKey.cs:272-293)
        std::vector<uint32_t> at, hashes;
        for (size_t i = 0; i < grains.size(); ++i)
            if (grains[i].Key.HasKeyExt()) {
                at.push_back((uint32_t)i);
                hashes.push_back(grains[i].GetUniformHashCode());
            }
        if (!at.empty()) {
            std::vector<uint32_t> own(at.size());
            Check(h_, gd_ring_lookup_hashes(h_, hashes.data(), (uint32_t)at.size(), own.data()));
            for (size_t j = 0; j < at.size(); ++j) idx[at[j]] = own[j];
        }
        std::vector<SiloAddress> r;
        for (uint32_t i : idx) r.push_back(RingSilo(i));
        return r;
    }
    SiloAddress CalculateTargetSilo(const GrainId& grain) const { return CalculateTargetSilos({grain})[0]; }
    SiloAddress GetPrimaryForGrain(const GrainId& grain) const { return CalculateTargetSilo(grain); }

    // Per-silo model with a DirectoryCache of maxCacheSize entries (GrainDirectoryOptions'
    // CacheSize, default 1,000,000).  The valid silos are the ring's members (IsValidSilo).
    void EnableCache(uint32_t maxCacheSize) {
        cacheOn_ = true;
        const auto m = Masks();
        Check(h_, gd_cache_configure(h_, maxCacheSize, m.first.data(), m.second.data(), (uint32_t)m.first.size()));
    }
    AdaptiveGrainDirectoryCache& DirectoryCache() { return cache_; }

    // LocalLookup (LocalGrainDirectory.cs:797-837).  Whole-node model: the owning partition is
    // always consulted.  Per-silo model: the partition when this silo owns the
    // grain, else the cache (a hit on an invalid silo, an empty list in the reference, is a
    // false return here: either way the dispatcher takes the full lookup).
    bool LocalLookup(const GrainId& grain, AddressesAndTag& result) const {
        if (!cacheOn_) {
            result = partition_.LookUpActivations(grain);
            return result.Addresses.has_value();
        }
        const gd_key k = grain.Key.ToNative();
        uint32_t silo = 0, act = 0;
        uint8_t st = 0;
        KeyExtBatch kx({&grain.Key});                 // string-keyed grains: KeyExt owner, partition or cache
        Check(h_, gd_route_ext(h_, &k, kx.get(), 1, &silo, &act, &st));
        result = AddressesAndTag{};
        if (st != GD_ROUTE_OK) return false;
        result.Addresses = std::vector<ActivationAddress>{{silos_.At(silo), grain, partition_.ActivationAt(act)}};
        return true;
    }
    AddressesAndTag GetLocalDirectoryData(const GrainId& grain) const { return partition_.LookUpActivations(grain); }

    GrainDirectoryPartition& DirectoryPartition() { return partition_; }
    SiloTable& Silos() { return silos_; }
    gd_handle* Handle() const { return h_; }
    const RingSnapshot& Ring() const { return ring_; }

    const SiloAddress MyAddress;

private:
    // the ring stores member positions; translate to the shared silo table
    void Install(const std::vector<SiloAddress>& m) {
        ring_.Rebuild(m);
        // re-install with owners expressed as silo-table indices
        std::vector<uint32_t> own;
        for (uint32_t o : ring_.Owners()) own.push_back(silos_.IndexOf(m[o]));
        std::vector<uint32_t> pts = ring_.Points();
        Check(h_, gd_ring_set(h_, GD_RING_DIRECTORY, pts.data(), own.data(), (uint32_t)pts.size()));
        const auto mk = Masks();           // membership changed: new IsValidSilo set (the members)
        Check(h_, gd_dir_set_valid_silos(h_, mk.second.data(), (uint32_t)mk.second.size()));
        if (cacheOn_) Check(h_, gd_cache_set_silos(h_, mk.first.data(), mk.second.data(), (uint32_t)mk.first.size()));
    }
    std::pair<std::vector<uint8_t>, std::vector<uint8_t>> Masks() {
        const uint32_t me = silos_.IndexOf(MyAddress);
        std::vector<uint8_t> local(silos_.Size(), 0), valid(silos_.Size(), 0);
        local[me] = 1;
        for (const auto& s : ring_.Members()) valid[silos_.IndexOf(s)] = 1;
        local.resize(silos_.Size(), 0);
        valid.resize(silos_.Size(), 0);
        return {local, valid};
    }
    SiloAddress RingSilo(uint32_t siloIndex) const {
        if (siloIndex == GD_NO_SILO) throw OrleansException(GD_ESTATE, "no owner");
        return silos_.At(siloIndex);
    }

    gd_handle* h_;
    SiloTable silos_;
    RingSnapshot ring_;
    GrainDirectoryPartition partition_;
    AdaptiveGrainDirectoryCache cache_;
    bool cacheOn_ = false;
};

// ------------------------------------------------------------------ dispatch stages
struct Message {                       // the header fields the path reads/writes (Message.cs:105-330)
    GrainId TargetGrain;
    std::optional<SiloAddress> TargetSilo;
    std::optional<ActivationId> TargetActivation;
    uint8_t RouteStatus = 0xFF;        // GD_ROUTE_* after AddressMessages
};

// Batched Dispatcher.AddressMessage (Dispatcher.cs:715-767): messages whose TargetAddress is
// complete are skipped (:718); the rest get SetTargetPlacement (Message.cs:629-639) on a hit.
// Returns the indices that stay on the C# slow path (MISS, system target, membership grain, and
// multi-activation grains, whose random choice is RandomPlacementDirector's).
class Dispatcher {
public:
    explicit Dispatcher(LocalGrainDirectory& dir) : dir_(dir) {}
    std::vector<size_t> AddressMessages(std::vector<Message>& msgs) {
        std::vector<size_t> todo;
        std::vector<gd_key> keys;
        std::vector<const UniqueKey*> uk;
        for (size_t i = 0; i < msgs.size(); ++i)
            if (!(msgs[i].TargetSilo && msgs[i].TargetActivation)) {
                todo.push_back(i);
                keys.push_back(msgs[i].TargetGrain.Key.ToNative());
                uk.push_back(&msgs[i].TargetGrain.Key);
            }
        std::vector<uint32_t> silo(keys.size()), act(keys.size());
        std::vector<uint8_t> st(keys.size());
        if (!keys.empty()) {        // string-keyed targets are routed on the GPU too (gd_route_ext)
            KeyExtBatch kx(uk);
            Check(dir_.Handle(), gd_route_ext(dir_.Handle(), keys.data(), kx.get(), (uint32_t)keys.size(), silo.data(),
                                              act.data(), st.data()));
        }
        std::vector<size_t> slow;
        for (size_t j = 0; j < todo.size(); ++j) {
            Message& m = msgs[todo[j]];
            m.RouteStatus = st[j];
            if (st[j] == GD_ROUTE_OK) {
                m.TargetSilo = dir_.Silos().At(silo[j]);
                m.TargetActivation = dir_.DirectoryPartition().ActivationAt(act[j]);
            } else {
                slow.push_back(todo[j]);
            }
        }
        return slow;
    }

private:
    LocalGrainDirectory& dir_;
};

// ActivationDirectory (src/Orleans.Runtime/Catalog/ActivationDirectory.cs): ActivationId -> the
// scheduling context (index) of an activation or system target, with its state, in the GPU table.
class ActivationDirectory {
public:
    explicit ActivationDirectory(gd_handle* h) : h_(h) {}
    // RecordNewTarget (:86-93) / RecordNewSystemTarget (:95-98): TryAdd.
    bool RecordNewTarget(const ActivationId& act, uint32_t context, bool valid, bool statelessWorker = false) {
        return Add(act, context, (valid ? GD_ACTDIR_VALID : 0u) | (statelessWorker ? GD_ACTDIR_STATELESS_WORKER : 0u));
    }
    bool RecordNewSystemTarget(const ActivationId& act, uint32_t context) {
        return Add(act, context, GD_ACTDIR_SYSTEM_TARGET | GD_ACTDIR_VALID);
    }
    bool RemoveTarget(const ActivationId& act) {       // :116-131, TryRemove
        const gd_key k = act.ToNative();
        uint8_t r = 0;
        Check(h_, gd_actdir_remove(h_, &k, 1, &r));
        return r != 0;
    }
    void SetValid(const ActivationId& act, bool valid) {   // ActivationData.SetState as the agent sees it
        const gd_key k = act.ToNative();
        uint32_t ctx = 0;
        uint8_t fl = 0, found = 0;
        Check(h_, gd_actdir_lookup(h_, &k, 1, &ctx, &fl, &found));
        if (!found) return;
        fl = (uint8_t)(valid ? (fl | GD_ACTDIR_VALID) : (fl & ~GD_ACTDIR_VALID));
        Check(h_, gd_actdir_set_flags(h_, &k, &fl, 1, nullptr));
    }
    // FindTarget (:41-45): the context of a Valid-or-not activation, nullopt when absent.
    std::optional<uint32_t> FindTarget(const ActivationId& act) const {
        const gd_key k = act.ToNative();
        uint32_t ctx = 0;
        uint8_t fl = 0, found = 0;
        Check(h_, gd_actdir_lookup(h_, &k, 1, &ctx, &fl, &found));
        if (!found || (fl & GD_ACTDIR_SYSTEM_TARGET)) return std::nullopt;
        return ctx;
    }
    int Count() const {
        uint64_t n = 0;
        Check(h_, gd_actdir_count(h_, &n));
        return (int)n;
    }

private:
    bool Add(const ActivationId& act, uint32_t context, uint32_t flags) {
        const gd_key k = act.ToNative();
        const uint8_t f = (uint8_t)flags;
        uint8_t added = 0;
        Check(h_, gd_actdir_add(h_, &k, &context, &f, 1, &added));
        return added != 0;
    }
    gd_handle* h_;
};

// What IncomingMessageAgent.ReceiveMessage did with each message of a batch, and the per-context
// FIFOs (WorkItemGroup.EnqueueTask, WorkItemGroup.cs:174-201).
struct ReceiveResult {
    std::vector<uint8_t> Status;                        // GD_RECV_*
    std::vector<std::vector<uint32_t>> PerContext;      // batch positions per context, arrival order
    std::vector<uint32_t> NullContext;                  // EnqueueReceiveMessage(msg, null, null)
    std::vector<uint32_t> NotEnqueued;                  // rejections and drops
};

// Batched IncomingMessageAgent.ReceiveMessage (IncomingMessageAgent.cs:92-190) up to the
// per-activation FIFO (ActivationData.EnqueueMessage, ActivationData.cs:566-606).
class IncomingMessageAgent {
public:
    explicit IncomingMessageAgent(gd_handle* h) : h_(h) {}

    // Messages by (TargetGrain, TargetActivation, Direction) against the ActivationDirectory.
    ReceiveResult ReceiveMessages(const std::vector<GrainId>& targetGrain, const std::vector<ActivationId>& targetActivation,
                                  const std::vector<uint8_t>& direction, uint32_t numContexts) {
        const uint32_t n = (uint32_t)targetGrain.size();
        std::vector<gd_key> tg(n), ta(n);
        for (uint32_t i = 0; i < n; ++i) {
            tg[i] = targetGrain[i].Key.ToNative();
            ta[i] = targetActivation[i].ToNative();
        }
        std::vector<uint32_t> ctx(n), perm(n), off((size_t)numContexts + 3);
        ReceiveResult r;
        r.Status.resize(n);
        Check(h_, gd_receive(h_, tg.data(), ta.data(), direction.empty() ? nullptr : direction.data(), n, numContexts,
                             nullptr, ctx.data(), r.Status.data(), perm.data(), off.data()));
        r.PerContext.resize(numContexts);
        for (uint32_t c = 0; c < numContexts; ++c) r.PerContext[c].assign(perm.begin() + off[c], perm.begin() + off[c + 1]);
        r.NullContext.assign(perm.begin() + off[numContexts], perm.begin() + off[numContexts + 1]);
        r.NotEnqueued.assign(perm.begin() + off[numContexts + 1], perm.begin() + off[numContexts + 2]);
        return r;
    }

    // Activation indices already resolved (the whole-node path): the stable bucketing alone.
    std::vector<std::vector<uint32_t>> ReceiveMessages(const std::vector<uint32_t>& targetActivation,
                                                       uint32_t numActivations) {
        const uint32_t n = (uint32_t)targetActivation.size();
        std::vector<uint32_t> perm(n), off(numActivations + 2);
        Check(h_, gd_bucket(h_, targetActivation.data(), n, numActivations, perm.data(), off.data()));
        std::vector<std::vector<uint32_t>> q(numActivations + 1);
        for (uint32_t a = 0; a <= numActivations; ++a) q[a].assign(perm.begin() + off[a], perm.begin() + off[a + 1]);
        return q;
    }

private:
    gd_handle* h_;
};

// ------------------------------------------------------------------ whole-node exchange
// One silo per GPU (SURVEY 8 e).  Exchange() takes the messages this silo's batcher addressed,
// moves each to the silo owning its grain's directory partition (the per-target-silo outbound
// queues of OutboundMessageQueue.SendMessage, OutboundMessageQueue.cs:54-131), looks it up there
// (GrainDirectoryPartition.cs:385-441) and queues it per activation (ActivationData.cs:566-606).
// With forward = true a hit travels on to the silo hosting its activation (the send to
// ActivationAddress.Silo after a remote lookup, LocalGrainDirectory.cs:920,
// OutboundMessageQueue.cs:125).  Every silo calls Exchange for every batch (collective).
struct Delivery {                        // the messages this silo received, in arrival order
    std::vector<uint32_t> SenderSilo;    // silo index of the sender
    std::vector<uint32_t> SenderIndex;   // position in the sender's batch
    std::vector<uint8_t> Status;         // GD_ROUTE_* from the owner's lookup
    std::vector<uint32_t> Activation;    // activation index (GD_NO_ACTIVATION unless OK)
    std::vector<std::vector<uint32_t>> PerActivation;   // arrival positions per activation, FIFO
    std::vector<uint32_t> Unrouted;      // arrival positions with no activation here
};

class SiloMessageCenter {
public:
    // RCCL communicator: silo 0 creates the id (gd_comm_unique_id) and publishes it to the others.
    SiloMessageCenter(gd_handle* h, const uint8_t id[GD_COMM_ID_BYTES], int nSilos, int myIndex) : h_(h) {
        Check(h, gd_comm_init(h, id, nSilos, myIndex));
    }
    // Handles already joined (gd_comm_init_local: every silo of the group in this process).
    explicit SiloMessageCenter(gd_handle* h) : h_(h) {}
    static void JoinInProcess(const std::vector<gd_handle*>& silos) {
        Check(nullptr, gd_comm_init_local(silos.data(), (int)silos.size()));
    }
    ~SiloMessageCenter() { gd_comm_destroy(h_); }
    SiloMessageCenter(const SiloMessageCenter&) = delete;
    SiloMessageCenter& operator=(const SiloMessageCenter&) = delete;

    Delivery Exchange(const std::vector<GrainId>& targets, uint32_t numActivations, bool forward = false) {
        std::vector<gd_key> keys(targets.size());
        for (size_t i = 0; i < targets.size(); ++i) keys[i] = targets[i].Key.ToNative();
        gd_multi_result r{};
        Check(h_, gd_route_multi(h_, keys.data(), (uint32_t)keys.size(), numActivations,
                                 forward ? GD_MULTI_FORWARD : 0, &r));
        const uint32_t m = r.n_recv;
        Delivery d;
        d.SenderSilo.resize(m);
        d.SenderIndex.resize(m);
        d.Status.resize(m);
        d.Activation.resize(m);
        std::vector<uint32_t> perm(m), off((size_t)numActivations + 2);
        Check(h_, gd_multi_fetch(h_, nullptr, d.SenderIndex.data(), d.SenderSilo.data(), nullptr, d.Activation.data(),
                                 d.Status.data(), perm.data(), off.data(), nullptr, nullptr, nullptr));
        d.PerActivation.resize(numActivations);
        for (uint32_t a = 0; a < numActivations; ++a)
            d.PerActivation[a].assign(perm.begin() + off[a], perm.begin() + off[a + 1]);
        d.Unrouted.assign(perm.begin() + off[numActivations], perm.begin() + off[numActivations + 1]);
        return d;
    }

private:
    gd_handle* h_;
};

}  // namespace orleans
