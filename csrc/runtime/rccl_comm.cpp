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

#include "gadmm_common.h"
#include "gadmm_chain.h"


struct RcclComm {
  ncclComm_t comm;
  int rank, nranks, device;
  std::atomic<long long> bytes_sent{0}, bytes_recv{0}, msgs_sent{0}, coll_bytes{0};
};

// Every entry point takes the handle from Python / the engine: a null one is an error, not a crash.
#define RCCL_HANDLE(h)                                         \
  RcclComm* c = (RcclComm*)(h);                                \
  do {                                                         \
    if (!c) {                                                  \
      gadmm_set_error("%s: null RCCL communicator", __func__); \
      return -1;                                               \
    }                                                          \
  } while (0)

#define NCCL_CHECK(expr)                                                                  \
  do {                                                                                    \
    ncclResult_t _r = (expr);                                                             \
    if (_r != ncclSuccess) {                                                              \
      gadmm_set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr, ncclGetErrorString(_r)); \
      return -(int)_r - 1000;                                                             \
    }                                                                                     \
  } while (0)

extern "C" {

int gadmm_rccl_unique_id(char* out128) {
  ncclUniqueId id;
  NCCL_CHECK(ncclGetUniqueId(&id));
  static_assert(sizeof(ncclUniqueId) == 128, "unexpected ncclUniqueId size");
  memcpy(out128, &id, 128);
  return 0;
}

int gadmm_rccl_version(void) {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}

void* gadmm_rccl_init(const char* id128, int nranks, int rank, int device) {
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
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
  if (r != ncclSuccess) {
    gadmm_set_error("ncclCommInitRank: %s", ncclGetErrorString(r));
    delete c;
    return nullptr;
  }
  return c;
}

int gadmm_rccl_destroy(void* h) {
  RcclComm* c = (RcclComm*)h;
  if (!c) return 0;
  ncclCommDestroy(c->comm);
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
