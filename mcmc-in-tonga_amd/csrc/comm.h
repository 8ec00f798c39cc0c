// comm.h -- the RCCL communicator of the exchange rounds (td_comm_*, comm.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

struct td_comm {
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0, device = 0;
    hipStream_t stream = nullptr;  // the exchange stream: a hardware queue of its own (dedicated_stream)
    double *stage = nullptr;       // td_comm_allgather: device in | out
    int64_t stage_count = 0;
};

namespace tdstar {
// A stream on a hardware queue of its own.  HIP deals the streams of one
// priority onto GPU_MAX_HW_QUEUES (4) shared queues, where a resident kernel
// would hold back every other stream of its queue: this one is of the highest
// priority (a pool no one else here uses -- torch's and RCCL's streams are of
// normal priority) and non-blocking (work on the legacy null stream, torch's
// default, does not wait for it).  (A CU-masked stream has a queue of its own
// too, but it is a blocking stream: torch's null-stream copies waited behind
// the resident launch until its watchdog.)
hipError_t dedicated_stream(hipStream_t *s, int device);
// The stream every resident tempering launch of this process runs on, one per
// device, made on first use and kept (one resident launch at a time: the few
// high-priority queues are not spent on every td_rounds).
hipError_t rounds_stream(hipStream_t *s, int device);
}  // namespace tdstar
