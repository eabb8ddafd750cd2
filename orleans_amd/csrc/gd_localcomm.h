// gd_localcomm.h -- an in-process transport with RCCL's point-to-point interface, for rehearsing the
// multi-rank exchange (gd_route_multi*) on one GPU: W library handles in one process, one host
// thread driving each, exchange through device-to-device copies.  RCCL itself refuses two ranks on
// one device, so without this the W > 1 paths of the exchange would first run on an 8-GPU node.
// gd_comm_init_local installs it; the exchange code is the same code that drives RCCL.
//
// Semantics of ncclSend / ncclRecv inside ncclGroupStart / ncclGroupEnd: per (src, dst) pair the
// sends and receives match in posting order; a receive's copy is ordered after the sender's stream
// reached the send (an event), and the sender's stream continues only after that copy is done.
// Every GroupEnd blocks its host thread until its receives are matched and its sends consumed,
// which RCCL does not do; the exchange code never relies on the difference (all ranks post every
// round in the same order).  A peer that never posts fails the call after 60 s instead of hanging.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <vector>

#include "gd_comm.h"

namespace gd {

struct LocalShared {
    struct Msg {
        const void* buf;
        size_t bytes;
        hipEvent_t ready;
    };
    int world = 0;
    int refs = 0;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<std::deque<Msg>> box;          // [src * world + dst]: posted sends
    std::vector<std::deque<hipEvent_t>> ack;   // [src * world + dst]: the receiver's copy is done
};

struct LocalRank {
    LocalShared* sh;
    int rank;
};

struct LocalOp {
    bool send;
    void* buf;
    size_t bytes;
    int peer;
    LocalRank* comm;
    hipStream_t stream;
};

inline thread_local int t_local_depth = 0;
inline thread_local std::vector<LocalOp> t_local_ops;

inline size_t nccl_type_bytes(ncclDataType_t t) {
    switch (t) {
        case ncclInt8:
        case ncclUint8: return 1;
        case ncclFloat16:
        case ncclBfloat16: return 2;
        case ncclInt32:
        case ncclUint32:
        case ncclFloat32: return 4;
        default: return 8;
    }
}

inline LocalRank* local_rank(ncclComm_t c) { return reinterpret_cast<LocalRank*>(c); }

inline ncclResult_t local_group_start() {
    ++t_local_depth;
    return ncclSuccess;
}

inline ncclResult_t local_post(bool send, const void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm,
                               hipStream_t stream) {
    LocalRank* r = local_rank(comm);
    if (!r || peer < 0 || peer >= r->sh->world) return ncclInvalidArgument;
    t_local_ops.push_back(LocalOp{send, const_cast<void*>(buf), count * nccl_type_bytes(type), peer, r, stream});
    return t_local_depth ? ncclSuccess : ncclInvalidUsage;   // the exchange always groups
}

inline ncclResult_t local_send(const void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm,
                               hipStream_t stream) {
    return local_post(true, buf, count, type, peer, comm, stream);
}

inline ncclResult_t local_recv(void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm,
                               hipStream_t stream) {
    return local_post(false, buf, count, type, peer, comm, stream);
}

inline ncclResult_t local_group_end() {
    if (t_local_depth == 0) return ncclInvalidUsage;
    if (--t_local_depth > 0) return ncclSuccess;
    std::vector<LocalOp> ops;
    ops.swap(t_local_ops);
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(60);
    ncclResult_t res = ncclSuccess;
    // 1. post the sends: buffer, size, and an event at the send's place in the sender's stream
    for (LocalOp& op : ops) {
        if (!op.send) continue;
        LocalShared* sh = op.comm->sh;
        hipEvent_t ev = nullptr;
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess || hipEventRecord(ev, op.stream) != hipSuccess)
            return ncclUnhandledCudaError;
        {
            std::lock_guard<std::mutex> lk(sh->mu);
            sh->box[op.comm->rank * sh->world + op.peer].push_back({op.buf, op.bytes, ev});
        }
        sh->cv.notify_all();
    }
    // 2. the receives: wait for the matching send, copy after it on the receiver's stream, ack
    for (LocalOp& op : ops) {
        if (op.send) continue;
        LocalShared* sh = op.comm->sh;
        LocalShared::Msg m{};
        {
            std::unique_lock<std::mutex> lk(sh->mu);
            auto& q = sh->box[op.peer * sh->world + op.comm->rank];
            if (!sh->cv.wait_until(lk, deadline, [&] { return !q.empty(); })) return ncclSystemError;
            m = q.front();
            q.pop_front();
        }
        if (m.bytes != op.bytes) res = ncclInvalidUsage;
        if (hipStreamWaitEvent(op.stream, m.ready, 0) != hipSuccess) return ncclUnhandledCudaError;
        const size_t b = m.bytes < op.bytes ? m.bytes : op.bytes;
        if (b && hipMemcpyAsync(op.buf, m.buf, b, hipMemcpyDeviceToDevice, op.stream) != hipSuccess)
            return ncclUnhandledCudaError;
        (void)hipEventDestroy(m.ready);
        hipEvent_t done = nullptr;
        if (hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess ||
            hipEventRecord(done, op.stream) != hipSuccess)
            return ncclUnhandledCudaError;
        {
            std::lock_guard<std::mutex> lk(sh->mu);
            sh->ack[op.peer * sh->world + op.comm->rank].push_back(done);
        }
        sh->cv.notify_all();
    }
    // 3. a send completes (for its stream) when the receiver's copy has
    for (LocalOp& op : ops) {
        if (!op.send) continue;
        LocalShared* sh = op.comm->sh;
        hipEvent_t done = nullptr;
        {
            std::unique_lock<std::mutex> lk(sh->mu);
            auto& q = sh->ack[op.comm->rank * sh->world + op.peer];
            if (!sh->cv.wait_until(lk, deadline, [&] { return !q.empty(); })) return ncclSystemError;
            done = q.front();
            q.pop_front();
        }
        if (hipStreamWaitEvent(op.stream, done, 0) != hipSuccess) return ncclUnhandledCudaError;
        (void)hipEventDestroy(done);
    }
    return res;
}

inline ncclResult_t local_comm_destroy(ncclComm_t comm) {
    LocalRank* r = local_rank(comm);
    if (!r) return ncclSuccess;
    LocalShared* sh = r->sh;
    bool last;
    {
        std::lock_guard<std::mutex> lk(sh->mu);
        last = --sh->refs == 0;
    }
    delete r;
    if (last) {
        for (auto& q : sh->box)
            for (auto& m : q) (void)hipEventDestroy(m.ready);
        for (auto& q : sh->ack)
            for (hipEvent_t e : q) (void)hipEventDestroy(e);
        delete sh;
    }
    return ncclSuccess;
}

inline ncclResult_t local_async_error(ncclComm_t, ncclResult_t* e) {
    *e = ncclSuccess;
    return ncclSuccess;
}

inline const char* local_error_string(ncclResult_t e) {
    switch (e) {
        case ncclSuccess: return "no error";
        case ncclInvalidUsage: return "local transport: send/recv sizes differ or call outside a group";
        case ncclInvalidArgument: return "local transport: invalid argument";
        case ncclSystemError: return "local transport: a peer did not post its send/recv within 60 s";
        default: return "local transport: HIP call failed";
    }
}

inline const Rccl& local_net() {
    static Rccl r = [] {
        Rccl t;
        t.ok = true;
        t.CommDestroy = local_comm_destroy;
        t.GroupStart = local_group_start;
        t.GroupEnd = local_group_end;
        t.Send = local_send;
        t.Recv = local_recv;
        t.GetErrorString = local_error_string;
        t.CommGetAsyncError = local_async_error;
        return t;
    }();
    return r;
}

// Rank comms of a new in-process communicator of `world` ranks.
inline std::vector<ncclComm_t> local_comms(int world) {
    LocalShared* sh = new LocalShared();
    sh->world = world;
    sh->refs = world;
    sh->box.resize((size_t)world * world);
    sh->ack.resize((size_t)world * world);
    std::vector<ncclComm_t> out;
    for (int r = 0; r < world; ++r) out.push_back(reinterpret_cast<ncclComm_t>(new LocalRank{sh, r}));
    return out;
}

}  // namespace gd
