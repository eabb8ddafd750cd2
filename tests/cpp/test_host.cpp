// test_host.cpp -- the reference's own tests on this path, restated in C++ against
// the host layer (orleans_amd/host/orleans_dispatch.hpp) over the C ABI.
//
//   ./test_host cpu            identity tests only (no GPU needed)
//   ./test_host all DUMPFILE   + GPU tests; writes a routing dump that
//                              tests/test_host_cpp.py compares with the oracle
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <memory>
#include <algorithm>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "orleans_dispatch.hpp"

using namespace orleans;

static int g_failures = 0;
#define EXPECT(cond)                                                               \
    do {                                                                           \
        if (!(cond)) {                                                             \
            std::fprintf(stderr, "  FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            ++g_failures;                                                          \
        }                                                                          \
    } while (0)

static void Run(const char* name, const std::function<void()>& f) {
    const int before = g_failures;
    std::fprintf(stderr, "RUN %s\n", name);
    try {
        f();
    } catch (const std::exception& e) {
        std::fprintf(stderr, "  EXCEPTION in %s: %s\n", name, e.what());
        ++g_failures;
    }
    std::printf("%s %s\n", g_failures == before ? "PASS" : "FAIL", name);
    std::fflush(stdout);
}

static SiloAddress Loopback(int gen) { return SiloAddress::New(127, 0, 0, 1, 0, gen); }  // SiloAddressUtils.NewLocalSiloAddress

// ---------------------------------------------------------------- Identifiertests.cs
static void ID_HashCorrectness() {        // Identifiertests.cs:278-293
    std::mt19937_64 r(278);
    for (int i = 0; i < 1000; ++i) {
        uint8_t b[24];
        for (auto& x : b) x = (uint8_t)r();
        uint64_t u1, u2, u3;
        std::memcpy(&u1, b, 8);
        std::memcpy(&u2, b + 8, 8);
        std::memcpy(&u3, b + 16, 8);
        EXPECT(gd_jenkins_hash_bytes(b, 24) == gd_jenkins_hash_u64x3(u1, u2, u3));
    }
}

static void SiloAddressGetUniformHashCodes() {   // Identifiertests.cs:51-68
    const SiloAddress s = SiloAddress::New(127, 0, 0, 1, 8080, 26);
    const auto result = s.GetUniformHashCodes(3);
    for (int i = 0; i < 3; ++i) {
        // BinaryTokenStreamWriter: Write(SiloAddress) then Write(int)
        uint8_t w[28] = {0};
        w[12] = 127; w[15] = 1;
        const int32_t port = 8080, gen = 26, extra = i;
        std::memcpy(w + 16, &port, 4);
        std::memcpy(w + 20, &gen, 4);
        std::memcpy(w + 24, &extra, 4);
        EXPECT(result[i] == gd_jenkins_hash_bytes(w, 28));
    }
}

static void UniqueKeyToByteArray() {              // Identifiertests.cs:32-48
    UniqueKey k;
    k.N0 = 0x1122334455667788ull;
    k.N1 = 0x99AABBCCDDEEFF00ull;
    k.TypeCodeData = (uint64_t)UniqueKey::Category::KeyExtGrain << 56;
    k.KeyExt = "hello world";
    const auto b = k.ToByteArray();
    EXPECT(b.size() == 24 + 4 + 11);
    int32_t len;
    std::memcpy(&len, b.data() + 24, 4);
    EXPECT(len == 11);
    EXPECT(std::string(b.begin() + 28, b.end()) == "hello world");
    EXPECT(k.GetUniformHashCode() == gd_jenkins_hash_bytes(b.data(), b.size()));
    UniqueKey plain = UniqueKey::NewKey(42, UniqueKey::Category::Grain, -7);
    EXPECT(plain.TypeCodeData == ((3ull << 56) | (0x00FFFFFFFFFFFFFFull & (uint64_t)(int64_t)-7)));
    EXPECT(plain.GetUniformHashCode() == gd_jenkins_hash_u64x3(plain.TypeCodeData, plain.N0, plain.N1));
}

static void CalculateIdHashKnownSilos() {
    // 127.0.0.1:0 generations 1..5 (RingTests_Standalone silos)
    const int32_t want[5] = {-2064684674, -1337777665, -605710880, -2359351, -1047635457};
    for (int g = 1; g <= 5; ++g) EXPECT(Loopback(g).GetConsistentHashCode() == want[g - 1]);
    EXPECT(gd_calculate_id_hash("BenchmarkGrains.Ping.PingGrain") == 1596181187);
}

// ---------------------------------------------------------------- RingTests_Standalone.cs
// RangeBreakable (RingTests_Standalone.cs:212-261): every point of the ring is owned exactly once.
static bool InRange(uint32_t b, uint32_t e, uint32_t n) {   // RingRange.cs:72-81
    if (b == e) return true;   // full range
    if (b < e) return n > b && n <= e;
    return n > b || n <= e;
}
static void VerifyRing(const std::vector<std::vector<std::pair<uint32_t, uint32_t>>>& ranges) {
    std::set<uint32_t> pts = {0u, 1u, 0xFFFFFFFFu, 0x7FFFFFFFu, 0x80000000u};
    for (const auto& rs : ranges)
        for (const auto& r : rs)
            for (int d = -1; d <= 1; ++d) {
                pts.insert(r.first + d);
                pts.insert(r.second + d);
            }
    std::mt19937 rng(5);
    for (int i = 0; i < 4000; ++i) pts.insert(rng());
    for (uint32_t p : pts) {
        int owners = 0;
        for (const auto& rs : ranges)
            for (const auto& r : rs) owners += InRange(r.first, r.second, p);
        EXPECT(owners == 1);
        if (owners != 1) return;
    }
}

static void RingStandalone(const std::vector<int>& failIdx, const std::vector<int>& joinIdx) {
    // CreateServers(5) -> Combine -> fail -> join -> VerifyRing (RingTests_Standalone.cs:73-97)
    std::vector<SiloAddress> all;
    for (int g = 1; g <= 5; ++g) all.push_back(Loopback(g));
    std::vector<SiloAddress> byHash = all;
    std::sort(byHash.begin(), byHash.end(),
              [](const SiloAddress& a, const SiloAddress& b) { return a.GetConsistentHashCode() < b.GetConsistentHashCode(); });
    std::vector<SiloAddress> live, joiners;
    for (int i = 0; i < 5; ++i) {
        if (std::find(failIdx.begin(), failIdx.end(), i) != failIdx.end()) continue;
        if (std::find(joinIdx.begin(), joinIdx.end(), i) != joinIdx.end()) joiners.push_back(byHash[i]);
        else live.push_back(byHash[i]);
    }
    std::vector<std::unique_ptr<DispatchHandle>> handles;
    std::vector<std::unique_ptr<ConsistentRingProvider>> rings;
    for (const auto& s : live) {
        handles.emplace_back(new DispatchHandle(0, 1024));
        rings.emplace_back(new ConsistentRingProvider(handles.back()->get(), s));
    }
    for (auto& r : rings)
        for (const auto& s : all) r->AddServer(s);               // Combine(rings, rings) incl. to-be-failed
    for (auto& r : rings)
        for (int i : failIdx) r->RemoveServer(byHash[i]);
    for (const auto& s : joiners) {
        handles.emplace_back(new DispatchHandle(0, 1024));
        rings.emplace_back(new ConsistentRingProvider(handles.back()->get(), s));
    }
    for (auto& r : rings)
        for (const auto& s : live) r->AddServer(s);
    for (auto& r : rings)
        for (const auto& s : joiners) r->AddServer(s);
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> ranges;
    for (auto& r : rings) ranges.push_back({r->GetMyRange()});
    VerifyRing(ranges);
    // ConsistentRingProviderTests_Silo.VerifyKey (:254-275): every silo agrees on the owner
    std::mt19937 rng(254);
    std::vector<uint32_t> keys;
    for (int i = 0; i < 2000; ++i) keys.push_back(rng());
    const auto first = rings[0]->GetPrimaryTargetSilos(keys);
    for (auto& r : rings) {
        const auto got = r->GetPrimaryTargetSilos(keys);
        for (size_t i = 0; i < keys.size(); ++i)
            EXPECT(r->Ring().Members()[got[i]] == rings[0]->Ring().Members()[first[i]]);
    }
}

static void VirtualBucketsRanges() {
    std::vector<SiloAddress> silos;
    for (int i = 1; i <= 6; ++i) silos.push_back(SiloAddress::New(10, 0, 0, (uint8_t)i, 11111, 1));
    std::vector<std::unique_ptr<DispatchHandle>> handles;
    std::vector<std::unique_ptr<VirtualBucketsRingProvider>> rings;
    for (const auto& s : silos) {
        handles.emplace_back(new DispatchHandle(0, 1024));
        rings.emplace_back(new VirtualBucketsRingProvider(handles.back()->get(), s, 30));
    }
    for (auto& r : rings)
        for (const auto& s : silos) r->AddServer(s);
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> ranges;
    for (auto& r : rings) ranges.push_back(r->GetMyRanges());
    VerifyRing(ranges);
    // the lookup lands in the owner's ranges
    std::mt19937 rng(9);
    for (int i = 0; i < 500; ++i) {
        const uint32_t k = rng();
        const SiloAddress o = rings[0]->GetPrimaryTargetSilo(k);
        size_t oi = std::find(silos.begin(), silos.end(), o) - silos.begin();
        bool in = false;
        for (const auto& r : ranges[oi]) in |= InRange(r.first, r.second, k);
        EXPECT(in);
    }
}

// ---------------------------------------------------------------- directory partition
static ActivationId NewActivationId(uint64_t seed) {  // ActivationId.NewId: Category None guid key
    ActivationId a;
    a.N0 = seed * 0x9E3779B97F4A7C15ull + 1;
    a.N1 = ~seed;
    a.TypeCodeData = 0;
    return a;
}

static void DirectorySemantics() {
    DispatchHandle h(0, 4096, 0);
    const SiloAddress me = SiloAddress::New(10, 0, 0, 1, 11111, 1);
    LocalGrainDirectory dir(h.get(), me);
    for (int i = 2; i <= 8; ++i) dir.AddServer(SiloAddress::New(10, 0, 0, (uint8_t)i, 11111, 1));
    auto& part = dir.DirectoryPartition();
    const int tc = gd_calculate_id_hash("BenchmarkGrains.Ping.PingGrain");
    const GrainId g1 = GrainId::GetGrainId(tc, 1), g2 = GrainId::GetGrainId(tc, 2);
    const ActivationId a1 = NewActivationId(1), a2 = NewActivationId(2);
    const SiloAddress s3 = SiloAddress::New(10, 0, 0, 3, 11111, 1);
    // AddSingleActivation: first registration wins, the second gets the first's address back
    auto r1 = part.AddSingleActivation(g1, a1, s3);
    EXPECT(r1.Address && r1.Address->Activation == a1 && r1.Address->Silo == s3);
    auto r2 = part.AddSingleActivation(g1, a2, me);
    EXPECT(r2.Address && r2.Address->Activation == a1 && r2.Address->Silo == s3);
    // LookUpActivations / LocalLookup
    AddressesAndTag res;
    EXPECT(dir.LocalLookup(g1, res) && res.Addresses->size() == 1 && (*res.Addresses)[0].Activation == a1);
    EXPECT(!dir.LocalLookup(g2, res) && !res.Addresses);
    // RemoveActivation: wrong activation is a no-op, right one removes the grain
    EXPECT(!part.RemoveActivation(g1, a2));
    EXPECT(part.RemoveActivation(g1, a1));
    EXPECT(!dir.GetLocalDirectoryData(g1).Addresses);
    auto r3 = part.AddSingleActivation(g1, a2, me);
    EXPECT(r3.Address && r3.Address->Activation == a2);
    EXPECT(part.Count() == 1);
    // CalculateTargetSilo equals the silo the ring's owner table gives
    EXPECT(dir.GetPrimaryForGrain(g1) == dir.CalculateTargetSilo(g1));
}

static void DispatcherAndAgent() {
    DispatchHandle h(0, 1 << 14, 0, /*seed*/ 0);
    const SiloAddress me = SiloAddress::New(10, 0, 0, 1, 11111, 1);
    LocalGrainDirectory dir(h.get(), me);
    for (int i = 2; i <= 8; ++i) dir.AddServer(SiloAddress::New(10, 0, 0, (uint8_t)i, 11111, 1));
    auto& part = dir.DirectoryPartition();
    const int tc = gd_calculate_id_hash("BenchmarkGrains.Ping.PingGrain");
    std::vector<GrainId> grains;
    std::vector<ActivationId> acts;
    std::vector<SiloAddress> where;
    for (int k = 0; k < 1000; ++k) {
        grains.push_back(GrainId::GetGrainId(tc, k));
        acts.push_back(NewActivationId(1000 + k));
    }
    const auto owners = dir.CalculateTargetSilos(grains);
    part.AddSingleActivations(grains, acts, owners);          // co-located with the directory owner
    std::vector<Message> msgs;
    std::mt19937 rng(7);
    for (int i = 0; i < 5000; ++i) msgs.push_back(Message{GrainId::GetGrainId(tc, rng() % 1100), {}, {}, 0xFF});
    Message st;                                                 // a system target: stays in C#
    st.TargetGrain.Key = UniqueKey::NewKey(3, UniqueKey::Category::Grain, 0);
    st.TargetGrain.Key.TypeCodeData = 1ull << 56;
    msgs.push_back(st);
    Message done = msgs[0];                                     // complete address: skipped (Dispatcher.cs:718)
    done.TargetSilo = me;
    done.TargetActivation = acts[0];
    msgs.push_back(done);
    Dispatcher disp(dir);
    const auto slow = disp.AddressMessages(msgs);
    size_t expect_slow = 0;
    for (size_t i = 0; i + 2 < msgs.size(); ++i) {
        const int64_t k = (int64_t)msgs[i].TargetGrain.Key.N1;
        if (k < 1000) {
            EXPECT(msgs[i].RouteStatus == GD_ROUTE_OK);
            EXPECT(msgs[i].TargetActivation && *msgs[i].TargetActivation == acts[k]);
            EXPECT(msgs[i].TargetSilo && *msgs[i].TargetSilo == owners[k]);
        } else {
            EXPECT(msgs[i].RouteStatus == GD_ROUTE_MISS && !msgs[i].TargetActivation);
            ++expect_slow;
        }
    }
    EXPECT(msgs[msgs.size() - 2].RouteStatus == GD_ROUTE_SYSTEM_TARGET);
    EXPECT(msgs.back().RouteStatus == 0xFF);
    EXPECT(slow.size() == expect_slow + 1);
    // IncomingMessageAgent: per-activation FIFO of the routed messages
    std::vector<uint32_t> target;
    for (size_t i = 0; i + 2 < msgs.size(); ++i)
        target.push_back(msgs[i].RouteStatus == GD_ROUTE_OK ? part.ActIndex(*msgs[i].TargetActivation) : GD_NO_ACTIVATION);
    IncomingMessageAgent agent(h.get());
    const uint32_t nAct = (uint32_t)part.ActivationCount();
    const auto q = agent.ReceiveMessages(target, nAct);
    size_t total = 0;
    for (uint32_t a = 0; a <= nAct; ++a) {
        total += q[a].size();
        for (size_t j = 0; j < q[a].size(); ++j) {
            EXPECT((a < nAct ? target[q[a][j]] == a : target[q[a][j]] >= nAct));
            if (j) EXPECT(q[a][j - 1] < q[a][j]);                      // arrival order kept
        }
    }
    EXPECT(total == target.size());
}

// String-keyed grains (GrainId.GetGrainId(long, string), GrainId.cs:86-91) and compound keys
// (:72-77) through the same partition / directory / dispatcher objects.
static SiloAddress RingOwnerD(const LocalGrainDirectory& dir, uint32_t hash) {   // LocalGrainDirectory.cs:506-541
    const auto& pts = dir.Ring().Points();
    const auto& own = dir.Ring().Owners();
    size_t pick = pts.size() - 1;
    for (size_t i = pts.size(); i-- > 0;)
        if ((int32_t)pts[i] <= (int32_t)hash) { pick = i; break; }
    return dir.Ring().Members()[own[pick]];
}

static void StringKeyGrains() {
    DispatchHandle h(0, 4096, 0);
    const SiloAddress me = SiloAddress::New(10, 0, 0, 1, 11111, 1);
    LocalGrainDirectory dir(h.get(), me);
    for (int i = 2; i <= 8; ++i) dir.AddServer(SiloAddress::New(10, 0, 0, (uint8_t)i, 11111, 1));
    auto& part = dir.DirectoryPartition();
    const int tc = gd_calculate_id_hash("UnitTests.GrainInterfaces.IStringKeyGrain");
    std::vector<GrainId> grains;
    std::vector<ActivationId> acts;
    for (int k = 0; k < 600; ++k) {
        std::string name = "user/" + std::to_string(k) + (k % 3 ? "" : "\xC3\xA9") + std::string(k % 40, 'x');
        grains.push_back(k % 5 ? GrainId::GetGrainId(tc, name) : GrainId::GetGrainId(tc, (int64_t)k, name));
        acts.push_back(NewActivationId(9000 + k));
    }
    const auto owners = dir.CalculateTargetSilos(grains);
    for (size_t i = 0; i < grains.size(); ++i) EXPECT(owners[i] == RingOwnerD(dir, grains[i].GetUniformHashCode()));
    std::vector<GrainId> reg(grains.begin(), grains.begin() + 400);
    std::vector<ActivationId> regActs(acts.begin(), acts.begin() + 400);
    std::vector<SiloAddress> regSilos(owners.begin(), owners.begin() + 400);
    const GrainId plain = GrainId::GetGrainId(tc, (int64_t)77);          // same type, no KeyExt
    reg.push_back(plain);
    regActs.push_back(NewActivationId(1));
    regSilos.push_back(me);
    reg.push_back(grains[0]);                                             // duplicate: first wins
    regActs.push_back(NewActivationId(2));
    regSilos.push_back(me);
    const auto r = part.AddSingleActivations(reg, regActs, regSilos);
    EXPECT(r.back().Address && r.back().Address->Activation == acts[0]);
    EXPECT(part.Count() == 401);
    AddressesAndTag res;
    EXPECT(dir.LocalLookup(grains[7], res) && (*res.Addresses)[0].Activation == acts[7]);
    EXPECT(!dir.LocalLookup(grains[500], res));
    EXPECT(dir.LocalLookup(plain, res) && (*res.Addresses)[0].Activation == regActs[400]);
    // a string grain and a long grain with the same words but another (or no) KeyExt differ
    GrainId other = grains[5];
    other.Key.KeyExt = *other.Key.KeyExt + "!";
    EXPECT(!dir.LocalLookup(other, res));
    // Dispatcher: string targets are addressed on the GPU
    std::vector<Message> msgs;
    std::mt19937 rng(11);
    std::vector<int> pick;
    for (int i = 0; i < 3000; ++i) {
        const int k = (int)(rng() % 600);
        pick.push_back(k);
        msgs.push_back(Message{grains[k], {}, {}, 0xFF});
    }
    Dispatcher disp(dir);
    const auto slow = disp.AddressMessages(msgs);
    size_t misses = 0;
    for (size_t i = 0; i < msgs.size(); ++i) {
        const int k = pick[i];
        if (k < 400) {
            EXPECT(msgs[i].RouteStatus == GD_ROUTE_OK && *msgs[i].TargetActivation == acts[k] &&
                   *msgs[i].TargetSilo == owners[k]);
        } else {
            EXPECT(msgs[i].RouteStatus == GD_ROUTE_MISS);
            ++misses;
        }
    }
    EXPECT(slow.size() == misses);
    // RemoveActivation on a string grain
    EXPECT(!part.RemoveActivation(grains[3], acts[4]));
    EXPECT(part.RemoveActivation(grains[3], acts[3]));
    EXPECT(!dir.LocalLookup(grains[3], res));
    EXPECT(part.Count() == 400);
}

// Multi-instance grains (GrainDirectoryPartition.AddActivation, GrainInfo.AddActivation :89-108).
static void MultiActivationGrains() {
    DispatchHandle h(0, 4096, 0);
    const SiloAddress me = SiloAddress::New(10, 0, 0, 1, 11111, 1);
    LocalGrainDirectory dir(h.get(), me);
    for (int i = 2; i <= 4; ++i) dir.AddServer(SiloAddress::New(10, 0, 0, (uint8_t)i, 11111, 1));
    auto& part = dir.DirectoryPartition();
    const int tc = gd_calculate_id_hash("UnitTests.Grains.StatelessWorkerGrain");
    const GrainId g = GrainId::GetGrainId(tc, 5);
    const SiloAddress s2 = SiloAddress::New(10, 0, 0, 2, 11111, 1), s3 = SiloAddress::New(10, 0, 0, 3, 11111, 1);
    const ActivationId a1 = NewActivationId(71), a2 = NewActivationId(72);
    EXPECT(part.AddActivation(g, a1, s2));
    EXPECT(!part.AddActivation(g, a1, s2));                         // refresh: same silo
    std::vector<Message> m{Message{g, {}, {}, 0xFF}};
    Dispatcher disp(dir);
    EXPECT(disp.AddressMessages(m).empty() && m[0].RouteStatus == GD_ROUTE_OK && *m[0].TargetActivation == a1);
    EXPECT(part.AddActivation(g, a2, s3));                          // a second instance
    m = {Message{g, {}, {}, 0xFF}};
    const auto slow = disp.AddressMessages(m);
    EXPECT(slow.size() == 1 && m[0].RouteStatus == GD_ROUTE_MULTI_ACT && !m[0].TargetActivation);
    EXPECT(!m[0].TargetSilo);                                       // the host picks the instance
    AddressesAndTag res;
    EXPECT(dir.LocalLookup(g, res) && res.Addresses->size() == 2);
    EXPECT(part.RemoveActivation(g, a1));                          // back to one instance
    m = {Message{g, {}, {}, 0xFF}};
    EXPECT(disp.AddressMessages(m).empty() && *m[0].TargetActivation == a2 && *m[0].TargetSilo == s3);
    EXPECT(part.RemoveActivation(g, a2));
    EXPECT(!dir.LocalLookup(g, res));
}

// ---------------------------------------------------------------- LruTest.cs (test/NonSilo.Tests/General)
// The reference's LRU tests, restated against the GPU directory cache (AdaptiveGrainDirectoryCache
// over LRU); keys "1".."n" become grains 1..n of one type.
struct CacheFixture {
    DispatchHandle h{0, 4096, 0};
    LocalGrainDirectory dir{h.get(), SiloAddress::New(10, 0, 0, 1, 11111, 1)};
    int tc = gd_calculate_id_hash("UnitTests.LruTestGrain");
    explicit CacheFixture(uint32_t maxSize) {
        for (int i = 2; i <= 4; ++i) dir.AddServer(SiloAddress::New(10, 0, 0, (uint8_t)i, 11111, 1));
        dir.EnableCache(maxSize);
    }
    GrainId Key(int i) const { return GrainId::GetGrainId(tc, i); }
    AdaptiveGrainDirectoryCache::Value Val(int i) const {
        return {SiloAddress::New(10, 0, 0, 2, 11111, 1), NewActivationId(500 + i)};
    }
    bool Contains(int i) const {
        for (const auto& kv : const_cast<CacheFixture*>(this)->dir.DirectoryCache().KeyValues())
            if (std::get<0>(kv) == Key(i)) return true;
        return false;
    }
};

static void LruCountTest() {                 // LruTest.cs:14-29
    CacheFixture f(10);
    auto& c = f.dir.DirectoryCache();
    EXPECT(c.Count() == 0);
    c.AddOrUpdate(f.Key(1), f.Val(1), 0);
    EXPECT(c.Count() == 1);
    c.AddOrUpdate(f.Key(2), f.Val(2), 0);
    EXPECT(c.Count() == 2);
}

static void LruMaximumSizeTest() {           // LruTest.cs:31-52
    const int maxSize = 10;
    CacheFixture f(maxSize);
    auto& c = f.dir.DirectoryCache();
    for (int i = 1; i <= maxSize + 5; ++i) c.AddOrUpdate(f.Key(i), f.Val(i), i);
    EXPECT(c.Count() == maxSize);
    for (int i = 1; i <= 5; ++i) EXPECT(!f.Contains(i));      // 'Older' entries are gone
}

static void LruUsageTest() {                 // LruTest.cs:54-88
    const int maxSize = 10;
    CacheFixture f(maxSize);
    auto& c = f.dir.DirectoryCache();
    for (int i = 1; i <= maxSize; ++i) c.AddOrUpdate(f.Key(i), f.Val(i), i);
    AdaptiveGrainDirectoryCache::Value v;
    int ver = 0;
    for (int i = maxSize; i >= 1; --i) EXPECT(c.LookUp(f.Key(i), v, ver) && ver == i && v == f.Val(i));
    c.AddOrUpdate(f.Key(maxSize + 1), f.Val(maxSize + 1), 0);
    EXPECT(c.Count() == maxSize);
    EXPECT(!f.Contains(maxSize));                              // the least recently used went
    for (int i = 1; i < maxSize; ++i) EXPECT(f.Contains(i));
    EXPECT(c.NumAccesses() == maxSize && c.NumHits() == maxSize);
}

static void PerSiloLocalLookup() {           // LocalGrainDirectory.LocalLookup, :797-837
    CacheFixture f(100);
    auto& part = f.dir.DirectoryPartition();
    auto& c = f.dir.DirectoryCache();
    int mine = -1, theirs = -1;
    for (int k = 0; k < 200 && (mine < 0 || theirs < 0); ++k) {
        const bool own = f.dir.CalculateTargetSilo(f.Key(k)) == f.dir.MyAddress;
        if (own && mine < 0) mine = k;
        if (!own && theirs < 0) theirs = k;
    }
    EXPECT(mine >= 0 && theirs >= 0);
    part.AddSingleActivation(f.Key(mine), NewActivationId(1), f.dir.MyAddress);
    AddressesAndTag r;
    EXPECT(f.dir.LocalLookup(f.Key(mine), r) && (*r.Addresses)[0].Activation == NewActivationId(1));
    EXPECT(!f.dir.LocalLookup(f.Key(theirs), r));              // not owned, not cached
    EXPECT(c.NumAccesses() == 1 && c.NumHits() == 0);
    const SiloAddress s3 = SiloAddress::New(10, 0, 0, 3, 11111, 1);
    c.AddOrUpdate(f.Key(theirs), {s3, NewActivationId(2)}, 7);  // after a remote lookup (:920)
    EXPECT(f.dir.LocalLookup(f.Key(theirs), r) && (*r.Addresses)[0].Silo == s3);
    // a cached address on a silo that is not a member: the hit counts, IsValidSilo (:848) filters the
    // address out; the reference returns true with an empty list, which its consumer, Catalog's
    // FastLookup (Catalog.cs:1323), takes as a miss -- the status the batched path gives
    const SiloAddress s9 = SiloAddress::New(10, 0, 0, 9, 11111, 1);
    c.AddOrUpdate(f.Key(theirs), {s9, NewActivationId(3)}, 8);
    EXPECT(!f.dir.LocalLookup(f.Key(theirs), r));
    EXPECT(c.NumAccesses() == 3 && c.NumHits() == 2 && c.Count() == 1);
    // the cached silo leaves the membership: AdjustLocalCache (:371-385) drops the entries pointing
    // at it (and those this silo now owns), so the lookup is a plain miss
    c.AddOrUpdate(f.Key(theirs), {s3, NewActivationId(2)}, 9);
    f.dir.RemoveServer(s3);
    EXPECT(!f.dir.LocalLookup(f.Key(theirs), r));
    EXPECT(c.Count() == 0 && !c.Remove(f.Key(theirs)));
}

// LocalLookup of string-keyed grains in the per-silo model: the owner by the KeyExt uniform hash,
// this silo's KeyExt partition for its own grains, the cache for the others -- keyed by the string
// (UniqueKey.Equals, UniqueKey.cs:245-251): "alice" and "alice!" of one type are different entries.
static void PerSiloLocalLookupStringKeys() {
    CacheFixture f(100);
    auto& part = f.dir.DirectoryPartition();
    auto& c = f.dir.DirectoryCache();
    const int stc = gd_calculate_id_hash("UnitTests.StringKeyGrain");
    std::vector<GrainId> mine, theirs;
    for (int k = 0; k < 400 && (mine.size() < 2 || theirs.size() < 2); ++k) {
        const GrainId g = GrainId::GetGrainId(stc, std::string("user/") + std::to_string(k));
        (f.dir.CalculateTargetSilo(g) == f.dir.MyAddress ? mine : theirs).push_back(g);
    }
    EXPECT(mine.size() >= 2 && theirs.size() >= 2);
    part.AddSingleActivation(mine[0], NewActivationId(11), f.dir.MyAddress);
    AddressesAndTag r;
    EXPECT(f.dir.LocalLookup(mine[0], r) && (*r.Addresses)[0].Activation == NewActivationId(11));
    EXPECT(!f.dir.LocalLookup(mine[1], r));                    // owned, not registered
    EXPECT(!f.dir.LocalLookup(theirs[0], r));                  // not owned, not cached
    const SiloAddress s3 = SiloAddress::New(10, 0, 0, 3, 11111, 1);
    c.AddOrUpdate(theirs[0], {s3, NewActivationId(12)}, 5);
    EXPECT(f.dir.LocalLookup(theirs[0], r) && (*r.Addresses)[0].Silo == s3 &&
           (*r.Addresses)[0].Activation == NewActivationId(12));
    GrainId other = theirs[0];
    other.Key.KeyExt = *other.Key.KeyExt + "!";                // same words, another KeyExt
    AdaptiveGrainDirectoryCache::Value v;
    int ver = 0;
    EXPECT(!c.LookUp(other, v, ver));
    EXPECT(c.LookUp(theirs[0], v, ver) && ver == 5 && v.second == NewActivationId(12));
    bool dumped = false;                                        // KeyValues returns the string key
    for (const auto& kv : c.KeyValues()) dumped = dumped || std::get<0>(kv) == theirs[0];
    EXPECT(dumped && c.Count() == 1);
    EXPECT(c.NumAccesses() == 4 && c.NumHits() == 2);
    EXPECT(c.Remove(theirs[0]) && !c.Remove(theirs[0]) && c.Count() == 0);
    EXPECT(!f.dir.LocalLookup(theirs[0], r));
}

static void RoutingDump(const char* path) {
    // bench silos, ring D, 20000 grains of the Ping type: owner silo index per grain (oracle-checked)
    DispatchHandle h(0, 1 << 15, 0);
    LocalGrainDirectory dir(h.get(), SiloAddress::New(10, 0, 0, 1, 11111, 1));
    for (int i = 2; i <= 8; ++i) dir.AddServer(SiloAddress::New(10, 0, 0, (uint8_t)i, 11111, 1));
    const int tc = gd_calculate_id_hash("BenchmarkGrains.Ping.PingGrain");
    std::vector<GrainId> grains;
    for (int k = -10000; k < 10000; ++k) grains.push_back(GrainId::GetGrainId(tc, k));
    const auto owners = dir.CalculateTargetSilos(grains);
    std::ofstream f(path);
    for (size_t i = 0; i < grains.size(); ++i)
        f << (int64_t)grains[i].Key.N1 << " " << (int)owners[i].Ip[15] << "\n";
}

// Whole-node exchange (SURVEY 8 e) with three silos in this process (gd_comm_init_local), one
// thread each: every message is delivered exactly once, to the silo owning its grain (or, with
// forward, to the silo hosting its activation), and each activation's queue keeps (sender silo,
// sender order) -- the order one IncomingMessageAgent thread per silo produces.
static void WholeNodeExchange() {
    const int W = 3, G = 3000, N = 20000;
    const int tc = gd_calculate_id_hash("BenchmarkGrains.Ping.PingGrain");
    std::vector<SiloAddress> silos;
    for (int i = 1; i <= W; ++i) silos.push_back(SiloAddress::New(10, 0, 0, (uint8_t)i, 11111, 1));
    std::vector<gd_silo_addr> addrs;
    for (const auto& s : silos) addrs.push_back(s.ToNative());
    std::vector<uint32_t> pts(64), own(64);
    uint32_t npts = 0;
    Check(nullptr, gd_ring_build(GD_RING_DIRECTORY, addrs.data(), W, 0, pts.data(), own.data(), &npts));
    std::vector<std::unique_ptr<DispatchHandle>> hs;
    std::vector<gd_handle*> raw;
    for (int r = 0; r < W; ++r) {
        hs.push_back(std::make_unique<DispatchHandle>(0, 1 << 13, (uint32_t)r));
        raw.push_back(hs.back()->get());
        Check(raw[r], gd_ring_set(raw[r], GD_RING_DIRECTORY, pts.data(), own.data(), npts));
    }
    // grain k: directory owner from the ring; activation on silo (k * 7 + 1) % W, numbered per silo
    const int K = G + 200;                  // grains G.. are never registered: MISS on their owner
    std::vector<gd_key> gk(K);
    for (int k = 0; k < K; ++k) gk[k] = GrainId::GetGrainId(tc, k).Key.ToNative();
    std::vector<uint32_t> owner(K), actSilo(G), actIdx(G), perSilo(W, 0);
    Check(raw[0], gd_ring_owner(raw[0], gk.data(), K, owner.data()));
    for (int k = 0; k < G; ++k) {
        actSilo[k] = (uint32_t)((k * 7 + 1) % W);
        actIdx[k] = perSilo[actSilo[k]]++;
    }
    for (int r = 0; r < W; ++r) {
        std::vector<gd_key> mk;
        std::vector<gd_val> mv;
        for (int k = 0; k < G; ++k)
            if ((int)owner[k] == r) {
                mk.push_back(gk[k]);
                mv.push_back(gd_val{actIdx[k], actSilo[k]});
            }
        std::vector<gd_val> win(mk.size());
        std::vector<uint8_t> ins(mk.size());
        Check(raw[r], gd_dir_register(raw[r], mk.data(), mv.data(), (uint32_t)mk.size(), win.data(), ins.data()));
    }
    SiloMessageCenter::JoinInProcess(raw);
    std::vector<std::vector<GrainId>> batch(W);
    std::vector<std::vector<int>> batchK(W);
    std::mt19937 rng(11);
    for (int r = 0; r < W; ++r)
        for (int i = 0; i < N + r * 100; ++i) {
            const int k = (int)(rng() % K);
            batch[r].push_back(GrainId::GetGrainId(tc, k));
            batchK[r].push_back(k);
        }
    std::vector<std::unique_ptr<SiloMessageCenter>> mc;      // destroying one leaves the group
    for (int r = 0; r < W; ++r) mc.push_back(std::make_unique<SiloMessageCenter>(raw[r]));
    for (bool forward : {false, true}) {
        std::vector<Delivery> got(W);
        std::vector<std::string> err(W);
        std::vector<std::thread> th;
        for (int r = 0; r < W; ++r)
            th.emplace_back([&, r] {
                try {
                    got[r] = mc[r]->Exchange(batch[r], perSilo[r], forward);
                } catch (const std::exception& e) {
                    err[r] = e.what();
                }
            });
        for (auto& t : th) t.join();
        bool ok = true;
        for (int r = 0; r < W; ++r)
            if (!err[r].empty()) {
                std::fprintf(stderr, "  silo %d: %s\n", r, err[r].c_str());
                ok = false;
            }
        EXPECT(ok);
        if (!ok) return;
        std::set<std::pair<uint32_t, uint32_t>> seen;
        size_t total = 0;
        for (int r = 0; r < W; ++r) {
            const Delivery& d = got[r];
            total += d.SenderSilo.size();
            for (size_t j = 0; j < d.SenderSilo.size(); ++j) {
                EXPECT(seen.insert({d.SenderSilo[j], d.SenderIndex[j]}).second);
                const int k = batchK[d.SenderSilo[j]][d.SenderIndex[j]];
                if (k < G) {
                    EXPECT(d.Status[j] == GD_ROUTE_OK && d.Activation[j] == actIdx[k]);
                    EXPECT((forward ? actSilo[k] : owner[k]) == (uint32_t)r);
                } else {
                    EXPECT(d.Status[j] == GD_ROUTE_MISS && owner[k] == (uint32_t)r);
                }
            }
            if (!forward) continue;
            for (uint32_t a = 0; a < perSilo[r]; ++a)
                for (size_t q = 1; q < d.PerActivation[a].size(); ++q) {
                    const uint32_t x = d.PerActivation[a][q - 1], y = d.PerActivation[a][q];
                    EXPECT(d.Activation[y] == a);
                    EXPECT(std::make_pair(d.SenderSilo[x], d.SenderIndex[x]) <
                           std::make_pair(d.SenderSilo[y], d.SenderIndex[y]));
                }
        }
        size_t sent = 0;
        for (int r = 0; r < W; ++r) sent += batch[r].size();
        EXPECT(total == sent);
    }
}

// LocalGrainDirectory.RemoveServer (LocalGrainDirectory.cs:311-361): the ring loses the silo, it is
// no longer a valid silo, and AdjustLocalDirectory drops the activations located on it; a second
// removal is a no-op (membershipCache.Contains check, :318-322).
static void SiloRemovalAdjustsDirectory() {
    DispatchHandle h(0, 4096, 0);
    const SiloAddress me = SiloAddress::New(10, 0, 0, 1, 11111, 1);
    LocalGrainDirectory dir(h.get(), me);
    std::vector<SiloAddress> silos{me};
    for (int i = 2; i <= 6; ++i) {
        silos.push_back(SiloAddress::New(10, 0, 0, (uint8_t)i, 11111, 1));
        dir.AddServer(silos.back());
    }
    auto& part = dir.DirectoryPartition();
    const int tc = gd_calculate_id_hash("BenchmarkGrains.Ping.PingGrain");
    std::vector<GrainId> g;
    for (int i = 0; i < 60; ++i) {
        g.push_back(GrainId::GetGrainId(tc, i));
        part.AddSingleActivation(g.back(), NewActivationId(100 + i), silos[i % 6]);
    }
    EXPECT(part.Count() == 60);
    dir.RemoveServer(silos[3]);
    EXPECT(part.Count() == 50);
    for (int i = 0; i < 60; ++i) {
        const auto r = dir.GetLocalDirectoryData(g[i]);
        EXPECT((i % 6 == 3) ? !r.Addresses.has_value() : (r.Addresses && r.Addresses->size() == 1));
        EXPECT(!(dir.CalculateTargetSilo(g[i]) == silos[3]));
    }
    // an activation on the removed silo is refused now (IsValidSilo, GrainDirectoryPartition.cs:310-311)
    const auto refused = part.AddSingleActivation(GrainId::GetGrainId(tc, 999), NewActivationId(999), silos[3]);
    EXPECT(!refused.Address.has_value());
    dir.RemoveServer(silos[3]);
    EXPECT(part.Count() == 50);
}

// GrainDirectoryPartition.Merge (:497-522): absent grains are added; for a grain held by both sides
// the lowest ActivationId stays and the other goes to DeleteActivations on its silo.
static void MergeKeepsLowestActivationId() {
    DispatchHandle h(0, 4096, 0);
    const SiloAddress me = SiloAddress::New(10, 0, 0, 1, 11111, 1), s2 = SiloAddress::New(10, 0, 0, 2, 11111, 1);
    LocalGrainDirectory dir(h.get(), me);
    dir.AddServer(s2);
    auto& part = dir.DirectoryPartition();
    const int tc = gd_calculate_id_hash("BenchmarkGrains.Ping.PingGrain");
    const GrainId g1 = GrainId::GetGrainId(tc, 1), g2 = GrainId::GetGrainId(tc, 2), g3 = GrainId::GetGrainId(tc, 3);
    ActivationId lo = NewActivationId(5), hi = NewActivationId(6);
    lo.N0 = 1;
    hi.N0 = 2;
    part.AddSingleActivation(g1, hi, me);
    part.AddSingleActivation(g2, lo, me);
    const auto tag1 = part.LookUpActivations(g1).VersionTag;
    const auto del = part.Merge({g1, g2, g3}, {lo, hi, NewActivationId(7)}, {s2, s2, s2});
    const auto a1 = part.LookUpActivations(g1), a2 = part.LookUpActivations(g2), a3 = part.LookUpActivations(g3);
    EXPECT(a1.Addresses && (*a1.Addresses)[0].Activation == lo && (*a1.Addresses)[0].Silo == s2);
    EXPECT(a1.VersionTag != tag1);
    EXPECT(a2.Addresses && (*a2.Addresses)[0].Activation == lo && (*a2.Addresses)[0].Silo == me);
    EXPECT(a3.Addresses && (*a3.Addresses)[0].Silo == s2);
    // hi on me (displaced from g1) and hi on s2 (the incoming one for g2) are deleted
    EXPECT(del.size() == 2 && del.at(me).size() == 1 && del.at(s2).size() == 1);
    EXPECT(del.at(me)[0].Activation == hi && del.at(me)[0].Grain == g1);
    EXPECT(del.at(s2)[0].Activation == hi && del.at(s2)[0].Grain == g2);
}

// Merge with string-keyed grains: they live in the KeyExt table and merge by the same rule
// (they used to land in the main table, where LookUpActivations never looks).
static void MergeStringKeyGrains() {
    DispatchHandle h(0, 4096, 0);
    const SiloAddress me = SiloAddress::New(10, 0, 0, 1, 11111, 1), s2 = SiloAddress::New(10, 0, 0, 2, 11111, 1);
    LocalGrainDirectory dir(h.get(), me);
    dir.AddServer(s2);
    auto& part = dir.DirectoryPartition();
    const int tc = gd_calculate_id_hash("UnitTests.GrainInterfaces.IStringKeyGrain");
    const GrainId g1 = GrainId::GetGrainId(tc, std::string("alice")), g2 = GrainId::GetGrainId(tc, std::string("bob"));
    const GrainId g3 = GrainId::GetGrainId(tc, std::string("carol-with-a-name-longer-than-24-bytes"));
    ActivationId lo = NewActivationId(5), hi = NewActivationId(6);
    lo.N0 = 1;
    hi.N0 = 2;
    part.AddSingleActivation(g1, hi, me);
    part.AddSingleActivation(g2, lo, me);
    const int before = part.Count();
    const auto del = part.Merge({g1, g2, g3}, {lo, hi, NewActivationId(7)}, {s2, s2, s2});
    const auto a1 = part.LookUpActivations(g1), a2 = part.LookUpActivations(g2), a3 = part.LookUpActivations(g3);
    EXPECT(a1.Addresses && (*a1.Addresses)[0].Activation == lo && (*a1.Addresses)[0].Silo == s2);
    EXPECT(a2.Addresses && (*a2.Addresses)[0].Activation == lo && (*a2.Addresses)[0].Silo == me);
    EXPECT(a3.Addresses && (*a3.Addresses)[0].Silo == s2);
    EXPECT(part.Count() == before + 1);
    EXPECT(del.size() == 2 && del.at(me).size() == 1 && del.at(s2).size() == 1);
    EXPECT(del.at(me)[0].Activation == hi && del.at(me)[0].Grain == g1);
    EXPECT(del.at(s2)[0].Activation == hi && del.at(s2)[0].Grain == g2);
    // a plain long-keyed grain with the same type is a different grain: untouched by the KeyExt merge
    const GrainId plain = GrainId::GetGrainId(tc, (int64_t)0);
    EXPECT(!part.LookUpActivations(plain).Addresses);
}

// AdjustLocalDirectory counts each removed grain once, also a multi-instance grain whose last
// instance lived on the removed silo (it was counted twice).
static void RemoveLastInstanceCountsOnce() {
    DispatchHandle h(0, 4096, 0);
    const SiloAddress me = SiloAddress::New(10, 0, 0, 1, 11111, 1);
    const SiloAddress s2 = SiloAddress::New(10, 0, 0, 2, 11111, 1), s3 = SiloAddress::New(10, 0, 0, 3, 11111, 1);
    LocalGrainDirectory dir(h.get(), me);
    dir.AddServer(s2);
    dir.AddServer(s3);
    auto& part = dir.DirectoryPartition();
    const int tc = gd_calculate_id_hash("UnitTests.Grains.StatelessWorkerGrain");
    const GrainId one = GrainId::GetGrainId(tc, 1), two = GrainId::GetGrainId(tc, 2);
    EXPECT(part.AddActivation(one, NewActivationId(71), s2));          // one instance, on s2
    EXPECT(part.AddActivation(two, NewActivationId(72), s2));          // two instances, one on s2
    EXPECT(part.AddActivation(two, NewActivationId(73), s3));
    EXPECT(part.RemoveActivationsOn(s2) == 1);
    EXPECT(!part.LookUpActivations(one).Addresses);
    const auto r = part.LookUpActivations(two);
    EXPECT(r.Addresses && r.Addresses->size() == 1 && (*r.Addresses)[0].Silo == s3);
}

// ActivationDirectory + IncomingMessageAgent.ReceiveMessage (IncomingMessageAgent.cs:92-170).
static void ActivationDirectoryReceive() {
    DispatchHandle h(0, 4096, 0);
    ActivationDirectory ad(h.get());
    IncomingMessageAgent agent(h.get());
    const int tc = gd_calculate_id_hash("BenchmarkGrains.Ping.PingGrain");
    const ActivationId a0 = NewActivationId(10), a1 = NewActivationId(11), a2 = NewActivationId(12);
    EXPECT(ad.RecordNewTarget(a0, 0, true));
    EXPECT(ad.RecordNewTarget(a1, 1, false));                  // not Valid yet
    EXPECT(!ad.RecordNewTarget(a0, 7, true));                  // TryAdd: first wins
    GrainId st;
    st.Key = UniqueKey::NewKey(77, UniqueKey::Category::SystemTarget, 3);
    EXPECT(ad.RecordNewSystemTarget(st.Key, 2));
    EXPECT(ad.FindTarget(a0) == std::optional<uint32_t>(0) && !ad.FindTarget(st.Key) && !ad.FindTarget(a2));
    const GrainId app = GrainId::GetGrainId(tc, 1);
    std::vector<GrainId> tg{app, app, app, st, st, app, st};
    std::vector<ActivationId> ta{a0, a1, a2, st.Key, st.Key, a0, a0};
    std::vector<uint8_t> dir{0, 0, 0, 1, 2, 1, 0};
    auto r = agent.ReceiveMessages(tg, ta, dir, 3);
    EXPECT((r.Status == std::vector<uint8_t>{GD_RECV_ACTIVATION, GD_RECV_NULL_CONTEXT, GD_RECV_NULL_CONTEXT,
                                             GD_RECV_SYSTEM_TARGET, GD_RECV_DROPPED, GD_RECV_ACTIVATION,
                                             GD_RECV_REJECT_UNKNOWN}));
    EXPECT((r.PerContext[0] == std::vector<uint32_t>{0, 5}) && r.PerContext[1].empty() &&
           (r.PerContext[2] == std::vector<uint32_t>{3}));
    EXPECT((r.NullContext == std::vector<uint32_t>{1, 2}) && (r.NotEnqueued == std::vector<uint32_t>{4, 6}));
    ad.SetValid(a1, true);
    EXPECT(ad.RemoveTarget(a0) && !ad.RemoveTarget(a0) && ad.Count() == 2);
    r = agent.ReceiveMessages({app, app}, {a0, a1}, {}, 3);
    EXPECT((r.Status == std::vector<uint8_t>{GD_RECV_NULL_CONTEXT, GD_RECV_ACTIVATION}));
    EXPECT((r.PerContext[1] == std::vector<uint32_t>{1}));
}

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "all";
    Run("ID_HashCorrectness", ID_HashCorrectness);
    Run("SiloAddressGetUniformHashCodes", SiloAddressGetUniformHashCodes);
    Run("UniqueKeyToByteArray", UniqueKeyToByteArray);
    Run("CalculateIdHashKnownSilos", CalculateIdHashKnownSilos);
    if (mode == "all") {
        Run("RingStandalone_Basic", [] { RingStandalone({}, {}); });
        Run("RingStandalone_Failures", [] {
            for (auto f : std::vector<std::vector<int>>{{0}, {0, 1}, {4}, {4, 3}, {2}, {2, 3}, {1, 3}, {0, 4}})
                RingStandalone(f, {});
        });
        Run("RingStandalone_Joins", [] {
            for (auto j : std::vector<std::vector<int>>{{0}, {0, 1}, {4}, {4, 3}, {2}, {2, 3}, {1, 3}, {0, 4}})
                RingStandalone({}, j);
        });
        Run("RingStandalone_Mixed", [] {
            RingStandalone({0}, {1});
            RingStandalone({1}, {0});
            RingStandalone({3}, {4});
            RingStandalone({4}, {3});
        });
        Run("VirtualBucketsRanges", VirtualBucketsRanges);
        Run("DirectorySemantics", DirectorySemantics);
        Run("DispatcherAndAgent", DispatcherAndAgent);
        Run("StringKeyGrains", StringKeyGrains);
        Run("MultiActivationGrains", MultiActivationGrains);
        Run("LruCountTest", LruCountTest);
        Run("LruMaximumSizeTest", LruMaximumSizeTest);
        Run("LruUsageTest", LruUsageTest);
        Run("PerSiloLocalLookup", PerSiloLocalLookup);
        Run("PerSiloLocalLookupStringKeys", PerSiloLocalLookupStringKeys);
        Run("WholeNodeExchange", WholeNodeExchange);
        Run("SiloRemovalAdjustsDirectory", SiloRemovalAdjustsDirectory);
        Run("MergeKeepsLowestActivationId", MergeKeepsLowestActivationId);
        Run("MergeStringKeyGrains", MergeStringKeyGrains);
        Run("RemoveLastInstanceCountsOnce", RemoveLastInstanceCountsOnce);
        Run("ActivationDirectoryReceive", ActivationDirectoryReceive);
        if (argc > 2) Run("RoutingDump", [&] { RoutingDump(argv[2]); });
    }
    std::printf("%s (%d failure%s)\n", g_failures ? "FAILED" : "OK", g_failures, g_failures == 1 ? "" : "s");
    return g_failures ? 1 : 0;
}
