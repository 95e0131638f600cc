// RCCL (ncclAllReduce over xGMI) for the end-of-scan counter exchange. Replaces the host future.get()
// reductions of per-thread vectors at /root/reference/src/fm_scanner.cpp:224-233 (and :497-505, :740-748,
// :1006-1022, :1550-1560). The message is G+2 u64 (<= 1.6 KB at G = 200): latency-bound, one call per scan.
//
// librccl (~570 MB with its device code) is loaded on first use with dlopen, not linked: a single-GPU `speq scan`
// or Python process never maps it (linking it cost every process start the load and registration of its code).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>

#include "capi_internal.hpp"
#include "em.hpp"
#include "scan_internal.hpp"

namespace {
struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

const Rccl& rccl() {
    static Rccl r;
    static std::string failure;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = ::dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = ::dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char* e = ::dlerror();
            failure = std::string("cannot load librccl.so.1: ") + (e ? e : "unknown error");
            return;
        }
        auto sym = [&](const char* name) {
            void* f = ::dlsym(h, name);
            if (!f && failure.empty()) failure = std::string("librccl.so.1 lacks ") + name;
            return f;
        };
        r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
        r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(sym("ncclCommInitRank"));
        r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(sym("ncclCommDestroy"));
        r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(sym("ncclAllReduce"));
        r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
    });
    if (!failure.empty()) throw speq::DeviceError(failure);
    return r;
}

void nccl_ok(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw speq::DeviceError(std::string(what) + ": " + rccl().error_string(r));
}
}  // namespace

extern "C" {

int speq_comm_unique_id(void* id_out) {
    return speq::guarded([&] {
        if (!id_out) throw std::invalid_argument("speq_comm_unique_id: null argument");
        static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
        ncclUniqueId id;
        nccl_ok(rccl().get_unique_id(&id), "ncclGetUniqueId");
        std::memcpy(id_out, &id, sizeof(id));
    });
}

int speq_comm_init(int nranks, int rank, const void* id, void** comm_out) {
    return speq::guarded([&] {
        if (!id || !comm_out || nranks < 1 || rank < 0 || rank >= nranks)
            throw std::invalid_argument("speq_comm_init: bad argument");
        ncclUniqueId uid;
        std::memcpy(&uid, id, sizeof(uid));
        ncclComm_t comm = nullptr;
        nccl_ok(rccl().comm_init_rank(&comm, nranks, uid, rank), "ncclCommInitRank");
        *comm_out = comm;
    });
}

int speq_comm_destroy(void* comm) {
    return speq::guarded([&] {
        if (comm) nccl_ok(rccl().comm_destroy(static_cast<ncclComm_t>(comm)), "ncclCommDestroy");
    });
}

int speq_allreduce_u64(void* comm, uint64_t* d_buf, uint64_t count, void* stream) {
    return speq::guarded([&] {
        if (!comm || !d_buf) throw std::invalid_argument("speq_allreduce_u64: null argument");
        nccl_ok(rccl().all_reduce(d_buf, d_buf, count, ncclUint64, ncclSum, static_cast<ncclComm_t>(comm),
                              static_cast<hipStream_t>(stream)),
                "ncclAllReduce");
    });
}

int speq_allreduce_host(void* comm, int device, void* buf, uint64_t count, int is_f64) {
    return speq::guarded([&] {
        if (!comm || (!buf && count)) throw std::invalid_argument("speq_allreduce_host: null argument");
        if (count == 0) return;
        int prev = 0;
        if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess)
            throw speq::DeviceError("speq_allreduce_host: cannot select GPU " + std::to_string(device));
        void* d = nullptr;
        struct Release {
            int dev;
            void*& p;
            ~Release() {
                if (p) (void)hipFree(p);
                (void)hipSetDevice(dev);
            }
        } release{prev, d};
        const size_t bytes = (size_t)count * 8;
        if (hipMalloc(&d, bytes) != hipSuccess) throw speq::DeviceError("speq_allreduce_host: hipMalloc failed");
        if (hipMemcpy(d, buf, bytes, hipMemcpyHostToDevice) != hipSuccess)
            throw speq::DeviceError("speq_allreduce_host: copy to the device failed");
        nccl_ok(rccl().all_reduce(d, d, count, is_f64 ? ncclFloat64 : ncclUint64, ncclSum,
                                  static_cast<ncclComm_t>(comm), nullptr),
                "ncclAllReduce");
        if (hipMemcpy(buf, d, bytes, hipMemcpyDeviceToHost) != hipSuccess)
            throw speq::DeviceError("speq_allreduce_host: copy to the host failed");
    });
}

int speq_em_allreduce(speq_em* em, void* comm, void* stream) {
    return speq::guarded([&] {
        if (!em || !comm) throw std::invalid_argument("speq_em_allreduce: null argument");
        if (em->finalized || !em->d_mult) throw std::invalid_argument("speq_em_allreduce: histogram already finalized");
        int prev = 0;
        if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(speq::device_ordinal(em->dev)) != hipSuccess)
            throw speq::DeviceError("speq_em_allreduce: cannot select the histogram's GPU");
        struct Restore {
            int dev;
            ~Restore() { (void)hipSetDevice(dev); }
        } restore{prev};
        hipStream_t st = static_cast<hipStream_t>(stream);
        ncclComm_t c = static_cast<ncclComm_t>(comm);
        nccl_ok(rccl().all_reduce(em->d_mult, em->d_mult, em->n, ncclUint32, ncclSum, c, st), "ncclAllReduce");
        nccl_ok(rccl().all_reduce(em->d_hi, em->d_hi, em->n, ncclUint32, ncclMax, c, st), "ncclAllReduce");
        if (hipStreamSynchronize(st) != hipSuccess) throw speq::DeviceError("speq_em_allreduce: stream failed");
    });
}

int speq_allreduce_f64(void* comm, double* d_buf, uint64_t count, void* stream) {
    return speq::guarded([&] {
        if (!comm || !d_buf) throw std::invalid_argument("speq_allreduce_f64: null argument");
        nccl_ok(rccl().all_reduce(d_buf, d_buf, count, ncclFloat64, ncclSum, static_cast<ncclComm_t>(comm),
                              static_cast<hipStream_t>(stream)),
                "ncclAllReduce");
    });
}

}  // extern "C"
