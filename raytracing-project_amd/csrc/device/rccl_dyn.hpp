// rccl_dyn.hpp — RCCL, loaded on first use.
//
// librccl.so is ~570 MB of host and device code; linked into librtamd it is
// mapped and initialised by every process that loads the library, including
// the one-GPU `ray` CLI, which never makes a collective (~4 ms of its process
// start).  rt_dist.hip includes this header after <rccl/rccl.h>: each RCCL
// entry point it calls is redirected (by the macros below) to a wrapper that
// dlopens librccl.so.1 the first time a collective path needs it and calls
// through the resolved pointer.  Without the library every wrapper returns
// ncclSystemError and ncclGetErrorString names the load failure.
#pragma once

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <mutex>

namespace rccl_dyn {

struct Api {
    decltype(&::ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&::ncclCommInitRank) CommInitRank = nullptr;
    decltype(&::ncclCommInitAll) CommInitAll = nullptr;
    decltype(&::ncclCommDestroy) CommDestroy = nullptr;
    decltype(&::ncclCommAbort) CommAbort = nullptr;
    decltype(&::ncclCommCount) CommCount = nullptr;
    decltype(&::ncclCommGetAsyncError) CommGetAsyncError = nullptr;
    decltype(&::ncclAllReduce) AllReduce = nullptr;
    decltype(&::ncclGather) Gather = nullptr;
    decltype(&::ncclGetErrorString) GetErrorString = nullptr;
    bool ok = false;
};

inline const Api& api() {
    static Api a;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        bool ok = true;
        auto sym = [&](auto& fp, const char* name) {
            fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
            ok = ok && fp != nullptr;
        };
        sym(a.GetUniqueId, "ncclGetUniqueId");
        sym(a.CommInitRank, "ncclCommInitRank");
        sym(a.CommInitAll, "ncclCommInitAll");
        sym(a.CommDestroy, "ncclCommDestroy");
        sym(a.CommAbort, "ncclCommAbort");
        sym(a.CommCount, "ncclCommCount");
        sym(a.CommGetAsyncError, "ncclCommGetAsyncError");
        sym(a.AllReduce, "ncclAllReduce");
        sym(a.Gather, "ncclGather");
        sym(a.GetErrorString, "ncclGetErrorString");
        a.ok = ok;
    });
    return a;
}

inline ncclResult_t GetUniqueId(ncclUniqueId* id) { return api().ok ? api().GetUniqueId(id) : ncclSystemError; }
inline ncclResult_t CommInitRank(ncclComm_t* c, int n, ncclUniqueId id, int r) {
    return api().ok ? api().CommInitRank(c, n, id, r) : ncclSystemError;
}
inline ncclResult_t CommInitAll(ncclComm_t* c, int n, const int* devs) {
    return api().ok ? api().CommInitAll(c, n, devs) : ncclSystemError;
}
inline ncclResult_t CommDestroy(ncclComm_t c) { return api().ok ? api().CommDestroy(c) : ncclSystemError; }
inline ncclResult_t CommAbort(ncclComm_t c) { return api().ok ? api().CommAbort(c) : ncclSystemError; }
inline ncclResult_t CommCount(const ncclComm_t c, int* n) { return api().ok ? api().CommCount(c, n) : ncclSystemError; }
inline ncclResult_t CommGetAsyncError(ncclComm_t c, ncclResult_t* e) {
    return api().ok ? api().CommGetAsyncError(c, e) : ncclSystemError;
}
inline ncclResult_t AllReduce(const void* s, void* r, size_t n, ncclDataType_t t, ncclRedOp_t op, ncclComm_t c,
                              hipStream_t st) {
    return api().ok ? api().AllReduce(s, r, n, t, op, c, st) : ncclSystemError;
}
inline ncclResult_t Gather(const void* s, void* r, size_t n, ncclDataType_t t, int root, ncclComm_t c,
                           hipStream_t st) {
    return api().ok ? api().Gather(s, r, n, t, root, c, st) : ncclSystemError;
}
inline const char* GetErrorString(ncclResult_t e) {
    return api().ok ? api().GetErrorString(e) : "librccl.so.1 could not be loaded (dlopen)";
}

}  // namespace rccl_dyn

#define ncclGetUniqueId rccl_dyn::GetUniqueId
#define ncclCommInitRank rccl_dyn::CommInitRank
#define ncclCommInitAll rccl_dyn::CommInitAll
#define ncclCommDestroy rccl_dyn::CommDestroy
#define ncclCommAbort rccl_dyn::CommAbort
#define ncclCommCount rccl_dyn::CommCount
#define ncclCommGetAsyncError rccl_dyn::CommGetAsyncError
#define ncclAllReduce rccl_dyn::AllReduce
#define ncclGather rccl_dyn::Gather
#define ncclGetErrorString rccl_dyn::GetErrorString
