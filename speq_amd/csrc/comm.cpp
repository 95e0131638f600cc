// RCCL (ncclAllReduce over xGMI) for the end-of-scan counter exchange. Replaces the host future.get()
// reductions of per-thread vectors at /root/reference/src/fm_scanner.cpp:224-233 (and :497-505, :740-748,
// :1006-1022, :1550-1560). The message is G+2 u64 (<= 1.6 KB at G = 200): latency-bound, one call per scan.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "capi_internal.hpp"

namespace {
void nccl_ok(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw speq::DeviceError(std::string(what) + ": " + ncclGetErrorString(r));
}
}  // namespace

extern "C" {

int speq_comm_unique_id(void* id_out) {
    return speq::guarded([&] {
        if (!id_out) throw std::invalid_argument("speq_comm_unique_id: null argument");
        static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
        ncclUniqueId id;
        nccl_ok(ncclGetUniqueId(&id), "ncclGetUniqueId");
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
        nccl_ok(ncclCommInitRank(&comm, nranks, uid, rank), "ncclCommInitRank");
        *comm_out = comm;
    });
}

int speq_comm_destroy(void* comm) {
    return speq::guarded([&] {
        if (comm) nccl_ok(ncclCommDestroy(static_cast<ncclComm_t>(comm)), "ncclCommDestroy");
    });
}

int speq_allreduce_u64(void* comm, uint64_t* d_buf, uint64_t count, void* stream) {
    return speq::guarded([&] {
        if (!comm || !d_buf) throw std::invalid_argument("speq_allreduce_u64: null argument");
        nccl_ok(ncclAllReduce(d_buf, d_buf, count, ncclUint64, ncclSum, static_cast<ncclComm_t>(comm),
                              static_cast<hipStream_t>(stream)),
                "ncclAllReduce");
    });
}

int speq_allreduce_f64(void* comm, double* d_buf, uint64_t count, void* stream) {
    return speq::guarded([&] {
        if (!comm || !d_buf) throw std::invalid_argument("speq_allreduce_f64: null argument");
        nccl_ok(ncclAllReduce(d_buf, d_buf, count, ncclFloat64, ncclSum, static_cast<ncclComm_t>(comm),
                              static_cast<hipStream_t>(stream)),
                "ncclAllReduce");
    });
}

}  // extern "C"
