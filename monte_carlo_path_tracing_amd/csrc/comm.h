// Library-internal RCCL helpers (comm.cpp): the communicators behind mcpt_render_opts.devices
// (ncclCommInitAll, one process) and mcpt_comm (ncclCommInitRank, one process per device).
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <vector>

#include "mcpt.h"

namespace mcpt {
int comm_all_init(const std::vector<int>& devices, std::vector<void*>& comms);
void comm_all_destroy(std::vector<void*>& comms);
// in-place ncclReduce(sum, root 0 = devices[0]) of bufs[i] on devices[i]; enqueued on streams[i]
int comm_all_reduce_sum(const std::vector<void*>& comms, const std::vector<int>& devices, const std::vector<double*>& bufs,
                        const std::vector<hipStream_t>& streams, size_t n);
// in-place ncclReduce(sum, root rank 0) of this rank's buffer
int comm_rank_reduce_sum(mcpt_comm* c, double* buf, size_t n, hipStream_t st);
// ncclCommAbort after a failed enqueue (the handle stays; further reduces fail with MCPT_E_DEVICE)
void comm_rank_abort(mcpt_comm* c);
int comm_rank_info(const mcpt_comm* c, int* nranks, int* rank, int* device);
}  // namespace mcpt
