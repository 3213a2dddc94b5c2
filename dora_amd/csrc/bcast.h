// RCCL broadcast groups for 1 -> N fan-out outputs ("1 -> N: ncclBroadcast rooted at
// the producer, one communicator per fan-out output").
//
// A producer started with DORA_GPU_FANOUT=rccl asks the daemon, once per output, for a group
// of that output's receivers (REQ_BCAST_GROUP).  The daemon admits a group only when every
// receiver runs on its own GPU, none on the producer's (one RCCL rank per device); it tells each
// receiver its rank (EV_BCAST_JOIN) and the producer the group size (DROP_BCAST_GROUP).  All
// ranks then build one communicator.  Per message the producer packs into its slot and
// broadcasts the slot on its node stream; each receiver posts the matching receive into its
// local receive pool the moment it drains the descriptor (every rank issues the broadcasts of
// one output in the daemon's routing order, so ranks never disagree on the sequence), and the
// input is handed out once the receive has completed.  RCCL is loaded on first use (dlopen):
// nodes that never fan out do not load it.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>
#include <string>

namespace dora {

constexpr size_t kBcastIdBytes = 128;  // ncclUniqueId

struct BcastComm;  // opaque: one RCCL communicator

// True once librccl could be loaded (first call loads it); `why` explains a failure.
bool bcast_available(std::string* why);
// A fresh ncclUniqueId of the root (rank 0).
int bcast_unique_id(uint8_t id[kBcastIdBytes]);
// Join (and wait for) the communicator of `nranks` ranks; bounded by `timeout_ms`.  On timeout
// or error the partial communicator is aborted and an error returned.
int bcast_join(const uint8_t id[kBcastIdBytes], int nranks, int rank, int64_t timeout_ms,
               BcastComm** out);
// Enqueue one broadcast of `bytes` from rank 0's `buf` into every other rank's `buf` on `st`.
int bcast_enqueue(BcastComm* c, void* buf, uint64_t bytes, hipStream_t st);
// Wait (bounded) for `st`, then release the communicator: a clean destroy when the stream
// drained, an abort (which ends kernels still waiting on a peer) when it did not.
void bcast_close(BcastComm* c, hipStream_t st, int64_t timeout_ms);
int bcast_rank(const BcastComm* c);
int bcast_nranks(const BcastComm* c);

}  // namespace dora
