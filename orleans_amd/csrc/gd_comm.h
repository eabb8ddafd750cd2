// gd_comm.h -- RCCL, loaded at run time, for the in-library exchange (SURVEY 8 b gd_route_multi, 8 e).
//
// The library does not link librccl: the single-GPU entry points must load where RCCL is absent,
// and a host that already holds an RCCL (PyTorch's bundled copy, soname librccl.so.1) must not get
// a second one.  dlopen("librccl.so.1") returns the copy already in the process, else the ROCm one.
// Types come from rccl.h; only the entry points are resolved through dlsym.
#pragma once
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <mutex>

namespace gd {

struct Rccl {
    bool ok = false;
    char why[256] = {0};
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclCommAbort) CommAbort = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
    decltype(&ncclCommGetAsyncError) CommGetAsyncError = nullptr;
    decltype(&ncclCommCount) CommCount = nullptr;          // optional (gd_comm_info)
    decltype(&ncclCommUserRank) CommUserRank = nullptr;    // optional (gd_comm_info)
};

inline const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* lib = nullptr;
        for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
            lib = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
            if (lib) break;
        }
        if (!lib) {
            const char* e = dlerror();
            snprintf(r.why, sizeof r.why, "librccl.so.1 not loadable: %s", e ? e : "?");
            return;
        }
        bool all = true;
        auto sym = [&](auto& fp, const char* name) {
            fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(lib, name));
            if (!fp) {
                all = false;
                snprintf(r.why, sizeof r.why, "librccl.so.1 lacks %s", name);
            }
        };
        sym(r.GetUniqueId, "ncclGetUniqueId");
        sym(r.CommInitRank, "ncclCommInitRank");
        sym(r.CommDestroy, "ncclCommDestroy");
        sym(r.CommAbort, "ncclCommAbort");
        sym(r.GroupStart, "ncclGroupStart");
        sym(r.GroupEnd, "ncclGroupEnd");
        sym(r.Send, "ncclSend");
        sym(r.Recv, "ncclRecv");
        sym(r.GetErrorString, "ncclGetErrorString");
        sym(r.CommGetAsyncError, "ncclCommGetAsyncError");
        r.ok = all;
        r.CommCount = reinterpret_cast<decltype(&ncclCommCount)>(dlsym(lib, "ncclCommCount"));
        r.CommUserRank = reinterpret_cast<decltype(&ncclCommUserRank)>(dlsym(lib, "ncclCommUserRank"));
    });
    return r;
}

}  // namespace gd
