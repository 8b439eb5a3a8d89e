// RCCL communicator for the chain/star fabrics.
//
// One process per MI355X; the communicator is created from a unique id that the Python launcher
// broadcasts over the torch.distributed control plane (gloo/TCPStore), so the hot path never goes
// through torch's ProcessGroup. Every op is enqueued on the caller's HIP stream, which makes the
// chain exchange capturable into the engine's hipGraph together with the compute kernels.
//
// GADMM needs only grouped neighbour send/recv (<= 2 peers per phase for a static chain over
// contiguous segments; arbitrary peers after a D-GADMM re-chain). The star comparators use
// reduce/broadcast, GD uses all-reduce, and the multi-rank stopping monitor all-reduces a small ring
// of per-iteration partial objectives (monitoring only; the algorithm itself uses no collective).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>
#include <atomic>
#include <chrono>
#include <thread>

#include "gadmm_common.h"
#include "gadmm_chain.h"


// Watchdog (RCCL has no deadline of its own): the communicator is created NON-BLOCKING, so neither its
// set-up nor a grouped enqueue can block the host forever -- both are polled with
// ncclCommGetAsyncError against `timeout_s`; host waits on a stream that carries RCCL work go through
// gadmm_rccl_wait (event polling against the deadline, async errors checked). A deadline that passes
// aborts the communicator (ncclCommAbort: the RCCL kernels in flight observe the abort flag and exit),
// marks it dead, and returns an error: the caller falls back, together with every other rank, to the
// IPC transport (engine/multigpu.py, parallel/dataplane.py). A dead communicator refuses every call.
struct RcclComm {
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 0, device = 0;
  double timeout_s = 60.0;
  bool aborted = false;
  hipEvent_t ev = nullptr;
  std::atomic<long long> bytes_sent{0}, bytes_recv{0}, msgs_sent{0}, coll_bytes{0};
};

namespace {

double since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

void abort_comm(RcclComm* c) {
  if (c->comm && !c->aborted) ncclCommAbort(c->comm);  // frees the communicator
  c->comm = nullptr;
  c->aborted = true;
}

// Drive a non-blocking call to completion: ncclInProgress is polled until the communicator reports
// success or an error, or the deadline passes (then the communicator is aborted).
ncclResult_t settle(RcclComm* c, ncclResult_t r) {
  if (r != ncclInProgress) return r;
  const auto t0 = std::chrono::steady_clock::now();
  for (int k = 0;; ++k) {
    ncclResult_t a = ncclSuccess;
    ncclResult_t q = ncclCommGetAsyncError(c->comm, &a);
    if (q != ncclSuccess) return q;
    if (a != ncclInProgress) return a;
    if (since(t0) > c->timeout_s) {
      abort_comm(c);
      return ncclSystemError;
    }
    if (k > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

}  // namespace

// Every entry point takes the handle from Python / the engine: a null one is an error, not a crash.
#define RCCL_HANDLE(h)                                                                  \
  RcclComm* c = (RcclComm*)(h);                                                         \
  do {                                                                                  \
    if (!c) {                                                                           \
      gadmm_set_error("%s: null RCCL communicator", __func__);                          \
      return -1;                                                                        \
    }                                                                                   \
    if (c->aborted) {                                                                   \
      gadmm_set_error("%s: RCCL communicator aborted by its watchdog", __func__);       \
      return GADMM_RCCL_DEAD;                                                           \
    }                                                                                   \
  } while (0)

// Every RCCL call of this file: ncclInProgress (non-blocking communicator) is settled against the
// watchdog deadline; a communicator aborted meanwhile reports GADMM_RCCL_DEAD.
#define NCCL_CHECK(expr)                                                                  \
  do {                                                                                    \
    ncclResult_t _r = settle(c, (expr));                                                  \
    if (_r != ncclSuccess) {                                                              \
      gadmm_set_error("%s:%d %s -> %s%s", __FILE__, __LINE__, #expr, ncclGetErrorString(_r), \
                      c->aborted ? " (watchdog: communicator aborted)" : "");            \
      return c->aborted ? GADMM_RCCL_DEAD : -(int)_r - 1000;                              \
    }                                                                                     \
  } while (0)

extern "C" {

int gadmm_rccl_unique_id(char* out128) {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) {
    gadmm_set_error("ncclGetUniqueId: %s", ncclGetErrorString(r));
    return -(int)r - 1000;
  }
  static_assert(sizeof(ncclUniqueId) == 128, "unexpected ncclUniqueId size");
  memcpy(out128, &id, 128);
  return 0;
}

int gadmm_rccl_version(void) {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}

// Non-blocking communicator set-up with a deadline (timeout_s <= 0: 60 s). nullptr on failure or timeout
// (gadmm_last_error says which); a timed-out set-up is aborted, never left half-initialised.
void* gadmm_rccl_init_timeout(const char* id128, int nranks, int rank, int device, double timeout_s) {
  hipError_t he = hipSetDevice(device);
  if (he != hipSuccess) {
    gadmm_set_error("hipSetDevice(%d): %s", device, hipGetErrorString(he));
    return nullptr;
  }
  ncclUniqueId id;
  memcpy(&id, id128, 128);
  RcclComm* c = new RcclComm();
  c->rank = rank;
  c->nranks = nranks;
  c->device = device;
  c->timeout_s = timeout_s > 0 ? timeout_s : 60.0;
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclResult_t r = ncclCommInitRankConfig(&c->comm, nranks, id, rank, &cfg);
  if (r == ncclInProgress || r == ncclSuccess) r = settle(c, ncclInProgress);
  if (r != ncclSuccess) {
    gadmm_set_error("ncclCommInitRankConfig: %s%s", ncclGetErrorString(r),
                    c->aborted ? " (set-up deadline passed: aborted)" : "");
    if (!c->aborted && c->comm) ncclCommAbort(c->comm);
    delete c;
    return nullptr;
  }
  if (hipEventCreateWithFlags(&c->ev, hipEventDisableTiming) != hipSuccess) {
    gadmm_set_error("rccl_init: hipEventCreate failed");
    ncclCommDestroy(c->comm);
    delete c;
    return nullptr;
  }
  return c;
}

void* gadmm_rccl_init(const char* id128, int nranks, int rank, int device) {
  return gadmm_rccl_init_timeout(id128, nranks, rank, device, 60.0);
}

int gadmm_rccl_set_timeout(void* h, double timeout_s) {
  RCCL_HANDLE(h);
  c->timeout_s = timeout_s > 0 ? timeout_s : 60.0;
  return 0;
}

// 1 = usable, 0 = aborted by the watchdog (or a null handle).
int gadmm_rccl_alive(void* h) {
  RcclComm* c = (RcclComm*)h;
  return (c && !c->aborted && c->comm) ? 1 : 0;
}

// Abort the communicator now (a peer is known to be gone). Idempotent.
int gadmm_rccl_abort(void* h) {
  RcclComm* c = (RcclComm*)h;
  if (!c) return 0;
  abort_comm(c);
  return 0;
}

// Host wait for the work queued on `st` so far (RCCL included), bounded by the watchdog deadline
// (timeout_s <= 0: the communicator's). 0 = done; GADMM_RCCL_DEAD = the deadline passed or RCCL
// reported an asynchronous error: the communicator was aborted (its kernels exit), the stream is
// drained for up to 10 s more, and the caller must fall back.
int gadmm_rccl_wait(void* h, hipStream_t st, double timeout_s) {
  RCCL_HANDLE(h);
  const double lim = timeout_s > 0 ? timeout_s : c->timeout_s;
  GADMM_CHECK(hipEventRecord(c->ev, st));
  const auto t0 = std::chrono::steady_clock::now();
  for (int k = 0;; ++k) {
    hipError_t q = hipEventQuery(c->ev);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) GADMM_CHECK(q);
    ncclResult_t a = ncclSuccess;
    ncclCommGetAsyncError(c->comm, &a);
    const bool bad = a != ncclSuccess && a != ncclInProgress;
    if (bad || since(t0) > lim) {
      abort_comm(c);
      const auto t1 = std::chrono::steady_clock::now();
      while (hipEventQuery(c->ev) == hipErrorNotReady && since(t1) < 10.0)
        std::this_thread::sleep_for(std::chrono::microseconds(200));
      if (hipEventQuery(c->ev) == hipErrorNotReady) {
        // the stream did not drain after the abort: nothing further may run on this device
        gadmm_set_error("rccl_wait: %s after %.3f s; communicator aborted but the stream did not drain in 10 s",
                        bad ? ncclGetErrorString(a) : "deadline passed", since(t0));
        return GADMM_RCCL_WEDGED;
      }
      gadmm_set_error("rccl_wait: %s after %.3f s: communicator aborted", bad ? ncclGetErrorString(a) : "deadline passed",
                      since(t0));
      return GADMM_RCCL_DEAD;
    }
    if (k > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

int gadmm_rccl_destroy(void* h) {
  RcclComm* c = (RcclComm*)h;
  if (!c) return 0;
  if (c->comm && !c->aborted) ncclCommDestroy(c->comm);
  if (c->ev) hipEventDestroy(c->ev);
  delete c;
  return 0;
}

// Grouped point-to-point exchange of rows of a row-major (rows x d) f64 table.
int gadmm_rccl_exchange_rows(void* h, const XchgOp* ops, int nops, double* table, int d, hipStream_t st) {
  RCCL_HANDLE(h);
  if (nops == 0) return 0;
  NCCL_CHECK(ncclGroupStart());
  long long s = 0, r = 0, ns = 0;
  for (int i = 0; i < nops; ++i) {
    const XchgOp& o = ops[i];
    const size_t cnt = o.count > 0 ? (size_t)o.count : (size_t)d;
    double* p = table + (long)o.row * d;
    if (o.is_send) {
      NCCL_CHECK(ncclSend(p, cnt, ncclDouble, o.peer, c->comm, st));
      s += (long long)cnt * 8;
      ns += 1;
    } else {
      NCCL_CHECK(ncclRecv(p, cnt, ncclDouble, o.peer, c->comm, st));
      r += (long long)cnt * 8;
    }
  }
  NCCL_CHECK(ncclGroupEnd());
  c->bytes_sent += s;
  c->bytes_recv += r;
  c->msgs_sent += ns;
  return 0;
}

// Raw-buffer send/recv pairs (LAG uploads, star ADMM) — pointers are device addresses.
int gadmm_rccl_sendrecv_raw(void* h, int nops, const int* peers, const int* is_send, double* const* bufs,
                            const long* counts, hipStream_t st) {
  RCCL_HANDLE(h);
  if (nops == 0) return 0;
  NCCL_CHECK(ncclGroupStart());
  for (int i = 0; i < nops; ++i) {
    if (is_send[i]) {
      NCCL_CHECK(ncclSend(bufs[i], (size_t)counts[i], ncclDouble, peers[i], c->comm, st));
      c->bytes_sent += counts[i] * 8;
      c->msgs_sent += 1;
    } else {
      NCCL_CHECK(ncclRecv(bufs[i], (size_t)counts[i], ncclDouble, peers[i], c->comm, st));
      c->bytes_recv += counts[i] * 8;
    }
  }
  NCCL_CHECK(ncclGroupEnd());
  return 0;
}

int gadmm_rccl_allreduce_sum_f64(void* h, const double* send, double* recv, long count, hipStream_t st) {
  RCCL_HANDLE(h);
  NCCL_CHECK(ncclAllReduce(send, recv, (size_t)count, ncclDouble, ncclSum, c->comm, st));
  c->coll_bytes += count * 8;
  return 0;
}

int gadmm_rccl_reduce_sum_f64(void* h, const double* send, double* recv, long count, int root, hipStream_t st) {
  RCCL_HANDLE(h);
  NCCL_CHECK(ncclReduce(send, recv, (size_t)count, ncclDouble, ncclSum, root, c->comm, st));
  c->coll_bytes += count * 8;
  return 0;
}

int gadmm_rccl_bcast_f64(void* h, double* buf, long count, int root, hipStream_t st) {
  RCCL_HANDLE(h);
  NCCL_CHECK(ncclBroadcast(buf, buf, (size_t)count, ncclDouble, root, c->comm, st));
  c->coll_bytes += count * 8;
  return 0;
}

int gadmm_rccl_counters(void* h, long long* out4) {
  RCCL_HANDLE(h);
  out4[0] = c->bytes_sent.load();
  out4[1] = c->bytes_recv.load();
  out4[2] = c->msgs_sent.load();
  out4[3] = c->coll_bytes.load();
  return 0;
}

int gadmm_rccl_reset_counters(void* h) {
  RCCL_HANDLE(h);
  c->bytes_sent = 0;
  c->bytes_recv = 0;
  c->msgs_sent = 0;
  c->coll_bytes = 0;
  return 0;
}

}  // extern "C"
