// comm.cpp -- RCCL communicator for the exchange step of parallel tempering
// (one replica per GPU, an allgather of every replica's phi per
// swap round over xGMI).  The reference has no counterpart: its chains are
// independent pmap workers (main_inversion.jl:15).  td_rounds_exchange
// (chain.cpp) issues the allgathers on comm->stream, each waiting on a
// counter the resident chain kernel raises -- no host in the loop.
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "comm.h"
#include "ctx.h"

using namespace tdstar;

namespace {
int nccl_err(ncclResult_t r, const char *what) {
    return set_err(nullptr, TD_ERR_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}
}  // namespace

namespace tdstar {
hipError_t dedicated_stream(hipStream_t *s, int device) {
    hipError_t e = hipSetDevice(device);
    int least = 0, greatest = 0;
    if (e == hipSuccess) e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (e != hipSuccess) return e;
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest);
}

hipError_t rounds_stream(hipStream_t *s, int device) {
    static std::mutex mu;
    static hipStream_t per_device[64] = {};
    if (device < 0 || device >= 64) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> g(mu);
    if (!per_device[device]) {
        const hipError_t e = dedicated_stream(&per_device[device], device);
        if (e != hipSuccess) return e;
    }
    *s = per_device[device];
    return hipSuccess;
}
}  // namespace tdstar

extern "C" {

int td_comm_unique_id(uint8_t *id) {
    if (!id) return set_err(nullptr, TD_ERR_ARG, "td_comm_unique_id: NULL");
    static_assert(sizeof(ncclUniqueId) == TD_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return nccl_err(r, "ncclGetUniqueId");
    std::memcpy(id, &u, sizeof u);
    return TD_OK;
}

int td_comm_create(td_comm **out, int device, int nranks, int rank, const uint8_t *id) {
    if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks)
        return set_err(nullptr, TD_ERR_ARG, "td_comm_create: bad arguments");
    *out = nullptr;
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return hip_err(nullptr, e, "td_comm_create: hipSetDevice");
    td_comm *c = new (std::nothrow) td_comm();
    if (!c) return set_err(nullptr, TD_ERR_NOMEM, "td_comm_create");
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);  // (blocks until every rank joined)
    if (r != ncclSuccess) {
        delete c;
        return nccl_err(r, "ncclCommInitRank");
    }
    e = dedicated_stream(&c->stream, device);
    if (e != hipSuccess) {
        (void)td_comm_destroy(c);
        return hip_err(nullptr, e, "td_comm_create: exchange stream");
    }
    *out = c;
    return TD_OK;
}

int td_comm_allgather(td_comm *c, const double *in, int64_t count, double *out) {
    if (!c || count < 0 || (count > 0 && (!in || !out))) return set_err(nullptr, TD_ERR_ARG, "td_comm_allgather");
    if (count == 0) return TD_OK;
    TD_HIP(nullptr, hipSetDevice(c->device));
    const int64_t need = count * (1 + c->nranks);
    if (need > c->stage_count) {
        if (c->stage) (void)hipFree(c->stage);
        c->stage = nullptr;
        c->stage_count = 0;
        TD_HIP(nullptr, hipMalloc(&c->stage, sizeof(double) * (size_t)need));
        c->stage_count = need;
    }
    double *din = c->stage, *dout = c->stage + count;
    TD_HIP(nullptr, hipMemcpyAsync(din, in, sizeof(double) * (size_t)count, hipMemcpyHostToDevice, c->stream));
    const ncclResult_t r = ncclAllGather(din, dout, (size_t)count, ncclFloat64, c->comm, c->stream);
    if (r != ncclSuccess) return nccl_err(r, "ncclAllGather");
    TD_HIP(nullptr, hipMemcpyAsync(out, dout, sizeof(double) * (size_t)(count * c->nranks), hipMemcpyDeviceToHost,
                                   c->stream));
    TD_HIP(nullptr, hipStreamSynchronize(c->stream));
    return TD_OK;
}

int td_comm_destroy(td_comm *c) {
    if (!c) return TD_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    int rc = TD_OK;
    if (c->comm) {
        const ncclResult_t r = ncclCommDestroy(c->comm);
        if (r != ncclSuccess) rc = nccl_err(r, "ncclCommDestroy");
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->stage) (void)hipFree(c->stage);
    delete c;
    return rc;
}

}  // extern "C"
