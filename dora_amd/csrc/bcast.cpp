// RCCL broadcast groups of fan-out outputs (bcast.h).  librccl is loaded with dlopen on first
// use and driven through a handful of entry points; communicators are created non-blocking so a
// rank that never joins cannot hang a node: every wait here is bounded.
#include "bcast.h"

#include <dlfcn.h>
#include <rccl/rccl.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>
#include <mutex>

#include "common.h"
#include "shm.h"

namespace dora {

struct BcastComm {
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 0;
};

namespace {

struct Rccl {
  bool loaded = false;
  std::string why;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*init_rank_config)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*) = nullptr;
  ncclResult_t (*get_async_error)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*abort)(ncclComm_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    // every rank of a dataflow is on this host: bootstrap over loopback unless told otherwise
    setenv("NCCL_SOCKET_IFNAME", "lo", 0);
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      r.why = std::string("dlopen librccl: ") + (e ? e : "not found");
      return;
    }
    auto sym = [&](const char* name) {
      void* p = dlsym(h, name);
      if (!p && r.why.empty()) r.why = std::string("librccl lacks ") + name;
      return p;
    };
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
    r.init_rank_config = reinterpret_cast<decltype(r.init_rank_config)>(sym("ncclCommInitRankConfig"));
    r.get_async_error = reinterpret_cast<decltype(r.get_async_error)>(sym("ncclCommGetAsyncError"));
    r.broadcast = reinterpret_cast<decltype(r.broadcast)>(sym("ncclBroadcast"));
    r.abort = reinterpret_cast<decltype(r.abort)>(sym("ncclCommAbort"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
    r.loaded = r.why.empty();
  });
  return r;
}

const char* err(ncclResult_t e) {
  Rccl& r = rccl();
  return r.error_string ? r.error_string(e) : "rccl error";
}

// Poll a non-blocking communicator until its last call has finished (bounded).
ncclResult_t settle(ncclComm_t c, int64_t timeout_ms) {
  Rccl& r = rccl();
  const uint64_t t0 = mono_ns();
  ncclResult_t st = ncclInProgress;
  for (;;) {
    if (r.get_async_error(c, &st) != ncclSuccess) return ncclSystemError;
    if (st != ncclInProgress) return st;
    if (timeout_ms >= 0 && int64_t(mono_ns() - t0) / 1000000 > timeout_ms) return ncclInProgress;
    usleep(200);
  }
}

}  // namespace

bool bcast_available(std::string* why) {
  Rccl& r = rccl();
  if (!r.loaded && why) *why = r.why;
  return r.loaded;
}

int bcast_unique_id(uint8_t id[kBcastIdBytes]) {
  Rccl& r = rccl();
  if (!r.loaded) return fail(DORA_ERR_UNSUPPORTED, "%s", r.why.c_str());
  ncclUniqueId u;
  ncclResult_t e = r.get_unique_id(&u);
  if (e != ncclSuccess) return fail(DORA_ERR_HIP, "ncclGetUniqueId: %s", err(e));
  static_assert(sizeof(u) == kBcastIdBytes, "ncclUniqueId size");
  std::memcpy(id, &u, kBcastIdBytes);
  return DORA_OK;
}

int bcast_join(const uint8_t id[kBcastIdBytes], int nranks, int rank, int64_t timeout_ms,
               BcastComm** out) {
  *out = nullptr;
  Rccl& r = rccl();
  if (!r.loaded) return fail(DORA_ERR_UNSUPPORTED, "%s", r.why.c_str());
  if (nranks < 1 || rank < 0 || rank >= nranks)
    return fail(DORA_ERR_INVALID, "broadcast group rank %d of %d", rank, nranks);
  ncclUniqueId u;
  std::memcpy(&u, id, kBcastIdBytes);
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclComm_t c = nullptr;
  ncclResult_t e = r.init_rank_config(&c, nranks, u, rank, &cfg);
  if (e != ncclSuccess && e != ncclInProgress) {
    if (c) (void)r.abort(c);
    return fail(DORA_ERR_HIP, "ncclCommInitRankConfig (rank %d of %d): %s", rank, nranks, err(e));
  }
  e = settle(c, timeout_ms);
  if (e != ncclSuccess) {
    (void)r.abort(c);
    if (e == ncclInProgress)
      return fail(DORA_ERR_TIMEOUT, "broadcast group (rank %d of %d) not formed within %lld ms",
                  rank, nranks, (long long)timeout_ms);
    return fail(DORA_ERR_HIP, "broadcast group (rank %d of %d): %s", rank, nranks, err(e));
  }
  auto* b = new BcastComm();
  b->comm = c;
  b->rank = rank;
  b->nranks = nranks;
  *out = b;
  return DORA_OK;
}

int bcast_enqueue(BcastComm* c, void* buf, uint64_t bytes, hipStream_t st) {
  Rccl& r = rccl();
  ncclResult_t e = r.broadcast(buf, buf, bytes, ncclUint8, 0, c->comm, st);
  if (e == ncclInProgress) e = settle(c->comm, 30000);
  if (e != ncclSuccess) return fail(DORA_ERR_HIP, "ncclBroadcast of %llu bytes: %s",
                                    (unsigned long long)bytes, err(e));
  return DORA_OK;
}

void bcast_close(BcastComm* c, hipStream_t st, int64_t timeout_ms) {
  if (!c) return;
  Rccl& r = rccl();
  const uint64_t t0 = mono_ns();
  while (st && hipStreamQuery(st) == hipErrorNotReady &&
         int64_t(mono_ns() - t0) / 1000000 <= timeout_ms)
    usleep(100);
  (void)hipGetLastError();
  // Abort frees the communicator without a collective handshake; a broadcast still waiting for
  // a rank that left (stream not drained by now) would otherwise spin forever — abort ends it.
  (void)r.abort(c->comm);
  delete c;
}

int bcast_rank(const BcastComm* c) { return c ? c->rank : -1; }
int bcast_nranks(const BcastComm* c) { return c ? c->nranks : 0; }

}  // namespace dora
